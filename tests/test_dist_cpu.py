"""Data-parallel plumbing on CPU with the gloo backend, world_size 2 (the GPU path uses the
same code over RCCL): gradient mean incl. the in-backward word-table hook, the reference's
strided train sharding and contiguous eval partitions."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from newsrec_amd import dist as D
from newsrec_amd import functions as F


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.table = torch.nn.Parameter(torch.randn(10, 4))
        self.users = torch.nn.Parameter(torch.randn(50, 4))
        self.lin = torch.nn.Linear(4, 3)
        self.lin2 = torch.nn.Linear(3, 2)


def _grads(model, x, use_hook):
    """loss = sum(lin(table[x])**2); the table grad goes through TABLE_GRAD_HOOK when asked."""
    class Gather(torch.autograd.Function):
        @staticmethod
        def forward(ctx, table, idx):
            ctx.save_for_backward(idx)
            ctx.table_ref = table
            return table[idx]

        @staticmethod
        def backward(ctx, g):
            (idx,) = ctx.saved_tensors
            dt = torch.zeros_like(ctx.table_ref).index_add_(0, idx, g)
            if use_hook and F.TABLE_GRAD_HOOK(ctx.table_ref, dt):
                dt = None
            return dt, None
    class UserRows(torch.autograd.Function):   # LSTUR's h0 = userEmbedding[u] (RNNUserFn)
        @staticmethod
        def forward(ctx, table, idx):
            ctx.save_for_backward(idx)
            ctx.table_ref = table
            return table[idx]

        @staticmethod
        def backward(ctx, g):
            (idx,) = ctx.saved_tensors
            if use_hook and F.SPARSE_GRAD_HOOK(ctx.table_ref, idx, g):
                return None, None
            return torch.zeros_like(ctx.table_ref).index_add_(0, idx, g), None
    model.zero_grad(set_to_none=True)
    u = torch.tensor([int(x[0]) * 7 % 50, 3, 3])    # a repeated user row, a rank-dependent one
    out = model.lin2(model.lin(Gather.apply(model.table, x) + UserRows.apply(model.users, u)))
    (out ** 2).sum().backward()


def _rows_add_cpu(dout, idx, dtable):
    """nr_rows_add_ordered restated for CPU tensors (this host-only test cannot launch it): each id's
    rows summed in ascending position, the sum added once."""
    seen = set()
    for i, t in enumerate(idx.tolist()):
        if t in seen:
            continue
        seen.add(t)
        rows = [j for j in range(i, idx.numel()) if int(idx[j]) == t]
        s = dout[rows[0]].clone()
        for j in rows[1:]:
            s += dout[j]
        dtable[t] += s


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.setup(rank, world, backend="gloo", master_port=str(port))
    model = Tiny()
    x = torch.tensor([rank, rank + 3, 7])
    sync = D.GradSync(model, bucket_mb=1e-4, rows_add=_rows_add_cpu)   # tiny buckets: several collectives
    _grads(model, x, use_hook=True)
    scale = sync()
    sync.close()
    # numpy copies travel by value: a tensor would be shared through a file descriptor that the
    # parent can only fetch while this process is still alive
    q.put((rank, scale, {n: (p.grad * scale).numpy().copy() for n, p in model.named_parameters()}))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_sync_mean_gloo_world2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: per-rank grads computed serially, averaged
    want = {}
    for r in range(world):
        m = Tiny()
        _grads(m, torch.tensor([r, r + 3, 7]), use_hook=False)
        for n, p in m.named_parameters():
            want[n] = want.get(n, 0) + p.grad / world
    for rank, scale, g in res:
        assert scale == 0.5
        for n in want:
            torch.testing.assert_close(torch.from_numpy(g[n]), want[n], rtol=1e-6, atol=1e-6)


def test_shard_train_matches_distributed_sampler():
    from torch.utils.data.distributed import DistributedSampler
    ds = list(range(11))
    for world in (1, 2, 3, 4):
        for shuffle in (False, True):
            for r in range(world):
                s = DistributedSampler(ds, num_replicas=world, rank=r, shuffle=shuffle, seed=5)
                s.set_epoch(2)
                assert D.shard_train(len(ds), world, r, shuffle=shuffle, seed=5, epoch=2) == list(iter(s))


def test_partition_sampler_contiguous():
    ds = list(range(10))
    parts = [list(D.Partition_Sampler(ds, 3, r)) for r in range(3)]
    assert parts == [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]]


_CHILD = r"""
import os, sys, torch.distributed as dist
dist.init_process_group("gloo")
assert dist.get_world_size() == int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == os.environ["RANK"]
import torch
t = torch.tensor([dist.get_rank() + 1.0])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print("SUM", float(t), flush=True)
rank = dist.get_rank()
dist.barrier()
dist.destroy_process_group()
sys.exit(3 if int(os.environ.get("FAIL_RANK", "-1")) == rank else 0)
"""


def test_spawn_ranks_world3(tmp_path, capfd):
    """bench.py --gpus N without WORLD_SIZE: dist.spawn_ranks launches N fresh ranks with
    torch.distributed.run's environment (twotower.py:62-73 mp.spawn) and joins them."""
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    assert D.spawn_ranks(3, [str(script)], env=env, timeout=120) == 0
    assert "SUM 6.0" in capfd.readouterr().out


def test_spawn_ranks_failure_propagates(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["FAIL_RANK"] = "1"
    assert D.spawn_ranks(2, [str(script)], env=env, timeout=120) == 3


def _deferred_worker(rank, world, port, q):
    """GradSync in deferred (graphed-step) mode: the weight gradient of ``lin`` comes from a
    closure the backward hands to WGRAD_DEFER_HOOK; in-place buckets written by a deferred GEMM
    must be reduced after it (pack() 'late'), the others may start early."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.setup(rank, world, backend="gloo", master_port=str(port))
    try:
        model = Tiny()
        x = torch.tensor([rank, rank + 3, 7])

        class LinDeferred(torch.autograd.Function):
            @staticmethod
            def forward(ctx, h, w, b):
                ctx.save_for_backward(h, w)
                return h @ w.t() + b

            @staticmethod
            def backward(ctx, g):
                h, w = ctx.saved_tensors
                dw = torch.zeros_like(w)

                def run(max_cus=0):
                    dw.add_(g.t() @ h)
                if not F.WGRAD_DEFER_HOOK(run, dw):
                    run()
                # a fresh view (as MHANewsFn's joined weights hand back): autograd installs it as
                # .grad without a copy, so the deferred GEMM's writes land in the gradient
                return g @ w, dw[:], g.sum(0)

        sync = D.GradSync(model, bucket_mb=1e-4, inplace_mb=1e-5, deferred=True)
        model.zero_grad(set_to_none=True)
        h = model.table[x]
        out = model.lin2(LinDeferred.apply(h, model.lin.weight, model.lin.bias))
        (out ** 2).sum().backward()
        assert len(sync._runs) == 1 and float(model.lin.weight.grad.abs().sum()) == 0.0   # deferred
        rec = sync.take_sparse()
        outs = sync.run_deferred()
        early, packed = sync.pack(rec, outs)
        late_ids = {id(b[0]) for b, _, inplace in packed if inplace}
        assert id(model.lin.weight) in late_ids, "the deferred gradient's bucket must run after the GEMM"
        assert all(id(b[0]) != id(model.lin.weight) for b, _, _ in early)
        works = sync.issue(early)
        sync.exchange(packed, rec, works)
        sync.unpack(packed)
        sync.close()
        q.put((rank, None, {n: (p.grad * sync.scale).numpy().copy() for n, p in model.named_parameters()
                            if p.grad is not None}))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_sync_deferred_wgrad_gloo_world2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_deferred_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    want = {}
    for r in range(world):
        m = Tiny()
        m.zero_grad(set_to_none=True)
        out = m.lin2(m.lin(m.table[torch.tensor([r, r + 3, 7])]))
        (out ** 2).sum().backward()
        for n, p in m.named_parameters():
            if p.grad is not None:
                want[n] = want.get(n, 0) + p.grad / world
    for rank, err, g in res:
        assert err is None, err
        assert set(g) == set(want), (set(g), set(want))
        for n in want:
            torch.testing.assert_close(torch.from_numpy(g[n]), want[n], rtol=1e-6, atol=1e-6)


def _dense_rows_worker(rank, world, port, q):
    """GradSync(sparse_tables=False): the row-sparse user-table gradient goes through the dense
    all-reduce, so functions.LOCAL_ROW_GRAD (the single-process row buffer + Adam row flags) must
    stand aside -- its flags would miss the rows other ranks touched."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.setup(rank, world, backend="gloo", master_port=str(port))
    try:
        model = Tiny()
        x = torch.tensor([rank, rank + 3, 7])
        sync = D.GradSync(model, bucket_mb=1e-4, sparse_tables=False)

        class UserRows(torch.autograd.Function):   # RNNUserFn's table gradient order of hooks
            @staticmethod
            def forward(ctx, table, idx):
                ctx.save_for_backward(idx)
                ctx.table_ref = table
                return table[idx]

            @staticmethod
            def backward(ctx, g):
                (idx,) = ctx.saved_tensors
                if F.SPARSE_GRAD_HOOK(ctx.table_ref, idx, g) or F.LOCAL_ROW_GRAD(ctx.table_ref, idx, g):
                    return None, None
                return torch.zeros_like(ctx.table_ref).index_add_(0, idx, g), None
        model.zero_grad(set_to_none=True)
        u = torch.tensor([int(x[0]) * 7 % 50, 3, 3])
        out = model.lin2(model.lin(model.table[x] + UserRows.apply(model.users, u)))
        (out ** 2).sum().backward()
        assert getattr(model.users, "_nr_row_touched", None) is None
        scale = sync()
        sync.close()
        q.put((rank, None, {n: (p.grad * scale).numpy().copy() for n, p in model.named_parameters()}))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))
    dist.barrier()
    dist.destroy_process_group()


def test_local_row_grad_stands_aside_under_dense_sync_gloo_world2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dense_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    want = {}
    for r in range(world):
        m = Tiny()
        _grads(m, torch.tensor([r, r + 3, 7]), use_hook=False)
        for n, p in m.named_parameters():
            want[n] = want.get(n, 0) + p.grad / world
    for rank, err, g in res:
        assert err is None, err
        for n in want:
            torch.testing.assert_close(torch.from_numpy(g[n]), want[n], rtol=1e-6, atol=1e-6)


def _dp_check_worker(rank, world, port, q, diverge):
    """bench.dp_check: float64 checksums of parameters and Adam moments compared across ranks."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.setup(rank, world, backend="gloo", master_port=str(port))
    try:
        model = Tiny()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        for p in model.parameters():
            p.grad = torch.ones_like(p)
        opt.step()
        if diverge and rank == 1:
            with torch.no_grad():
                model.lin.bias[0] += 1e-3
        q.put((rank, None, bench.dp_check(model, opt, world, torch.device("cpu"))))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("diverge", [False, True])
def test_bench_dp_check_gloo_world2(diverge):
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_check_worker, args=(r, world, port, q, diverge)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, err, out in res:
        assert err is None, err
        assert out["dp_world_size"] == 2
        assert out["dp_in_sync"] is (not diverge)
        assert out["dp_bitwise_equal"] is (not diverge)


class TinyWords(torch.nn.Module):
    """A word table (named like BERT_Embedding's, so GradSync(shard_tables=True) shards it) of 11 rows:
    world 2 -> slabs of 6 (one pad row), world 3 -> slabs of 4 (the last rank owns 3 rows)."""
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.bert_word_embedding = torch.nn.Embedding(11, 4)
        self.lin = torch.nn.Linear(4, 3)


def _words_loss(model, x, hook=True):
    """hook: the news tower's table gradient handling (MHANewsFn hands it to TABLE_GRAD_HOOK); without,
    the BERT tower's (BertFn returns it to autograd)."""
    class Gather(torch.autograd.Function):
        @staticmethod
        def forward(ctx, table, idx):
            ctx.save_for_backward(idx)
            ctx.table_ref = table
            return table[idx]

        @staticmethod
        def backward(ctx, g):
            (idx,) = ctx.saved_tensors
            t = ctx.table_ref
            dt = F.table_grad_buffer(t, t.shape[0], t.shape[1], t.device, zero=True)
            dt.index_add_(0, idx, g)
            if hook and F.TABLE_GRAD_HOOK(t, dt):
                dt = None
            return dt, None
    out = model.lin(Gather.apply(model.bert_word_embedding.weight, x))
    return (out ** 2).sum()


def _adam_cpu(entries, beta1, beta2, eps, weight_decay, grad_scale=1.0, advance_steps=False):
    """K.adam_multi's arithmetic on CPU tensors (torch.optim.Adam's, elementwise) for this host test."""
    for p, g, m, v, lr, step in (e[:6] for e in entries):
        gg = g * grad_scale
        m.mul_(beta1).add_(gg, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
        c1, c2 = 1 - beta1 ** step, 1 - beta2 ** step
        p.sub_(lr * (m / c1) / ((v / c2).sqrt() + eps))


def _shard_worker(rank, world, port, q, deferred, hook=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.setup(rank, world, backend="gloo", master_port=str(port))
    try:
        from newsrec_amd import optim as O
        O.K.adam_multi = _adam_cpu
        res = {}
        for shard in (False, True):
            model = TinyWords()
            sync = D.GradSync(model, bucket_mb=1e-4, inplace_mb=1e-5, shard_tables=shard, deferred=deferred)
            opt = O.FusedAdam(model.parameters(), lr=1e-2)
            w = model.bert_word_embedding.weight
            if shard:
                S = -(-11 // world)
                assert w._nr_grad_rows == world * S and w._nr_shard == (rank * S, max(0, min(S, 11 - rank * S)))
            for step in range(3):
                opt.zero_grad(set_to_none=True)
                x = torch.tensor([rank, (rank + 5 * step) % 11, 10, 7])
                _words_loss(model, x, hook).backward()
                opt.step(grad_scale=sync())
                sync.after_step()
            if shard:   # moments for the rank's own rows only
                assert opt.state[w]["exp_avg"].shape[0] == w._nr_shard[1]
            sync.close()
            res[shard] = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
        q.put((rank, None, res))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("hook", [True, False])
@pytest.mark.parametrize("world,deferred", [(2, False), (3, False), (2, True), (3, True)])
def test_grad_sync_shard_tables_bitwise_gloo(world, deferred, hook):
    """GradSync(shard_tables=True): the word table's gradient reduce-scattered in place into row slabs,
    Adam on each rank's slab only (moments for those rows), the slabs all-gathered in place after the
    step -- three steps, eager (the reduce-scatter issued from inside the backward) and deferred (the
    graphed step's issue / exchange), world 2 and 3 (a pad row; a short last slab), the table's
    gradient handed to TABLE_GRAD_HOOK (the news towers) or returned to autograd (the BERT tower: the
    eager exchange reduce-scatters it then -- it once skipped it): every parameter BITWISE equal to the
    dense all-reduce path on every rank."""
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q, deferred, hook)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, err, r in res:
        assert err is None, err
        for n in r[False]:
            assert (r[False][n] == r[True][n]).all(), (rank, n)
    first = res[0][2][True]
    for rank, _, r in res[1:]:
        for n in first:
            assert (r[True][n] == first[n]).all(), (rank, n)   # replicas identical
