"""Data parallelism of the REAL models on the GPU (utils/Manager.py:167,211-213; twotower.py:49-50):
two ranks, spawned as fresh processes on the one leased GPU, each train on half of a batch through
GradSync and must reproduce one process training on the whole batch (DDP's gradient mean).

This exercises the production hook sites: the word-table gradient handed over inside the news
tower backward (functions.py MHANewsFn / CNNNewsRowsFn, TABLE_GRAD_HOOK), LSTUR's row-sparse
user-table exchange (RNNUserFn, SPARSE_GRAD_HOOK), the bucketed dense all-reduce, and the
two-graph data-parallel step (bench.GraphedStep: forward/backward graph, collectives, optimizer
graph).  The collectives run over gloo on device tensors (RCCL cannot put two ranks on one GPU);
GradSync's code path is the same for both backends."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

CASES = {"nrms": ("mha", "mha", 384), "lstur": ("cnn", "lstur", 150), "xformer": ("bert", "xformer", 768)}
V, USERS, BT, C, NH, L = 2000, 40, 8, 5, 10, 30


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(case, dev):
    from newsrec_amd.manager import build_model
    encN, encU, H = CASES[case]
    torch.manual_seed(11)
    if case == "xformer":
        # configs[4] (xformer.py:17-20): BERT-base width, 2 layers, the word table trained at bert_lr
        from newsrec_amd.bert import BertConfig
        from newsrec_amd.manager import ManagerConfig
        from newsrec_amd.xformer import XFormer
        bc = BertConfig(vocab_size=V, num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        m = XFormer(ManagerConfig("bert", "xformer", H, bert_dim=H), bert_config=bc).to(dev)
        with torch.no_grad():   # spread the scores (BERT's 0.02 init gives near-equal logits)
            for n, p in m.named_parameters():
                if p.dim() == 2 and "embeddings" not in n:
                    p.normal_(0, 1.5 / p.shape[1] ** 0.5)
        return m
    m = build_model(encN, encU, H, vocab=V, device=dev, user_num=USERS, dropout_p=0.0)
    with torch.no_grad():
        m.embedding.bert_word_embedding.weight.normal_(0, 0.5)
    return m


def _batch(seed, dev):
    g = torch.Generator().manual_seed(seed)

    def titles(n):
        tok = torch.randint(1000, V, (n, L), generator=g)
        lens = torch.randint(5, L + 1, (n,), generator=g)
        mask = (torch.arange(L)[None] < lens[:, None]).long()
        return tok * mask, mask
    ct, cm = titles(BT * C)
    ht, hm = titles(BT * NH)
    his = (torch.arange(NH)[None] < torch.randint(1, NH + 1, (BT, 1), generator=g)).double().unsqueeze(-1)
    x = {"cdd_encoded_index": ct.view(BT, C, L), "cdd_attn_mask": cm.view(BT, C, L),
         "his_encoded_index": ht.view(BT, NH, L), "his_attn_mask": hm.view(BT, NH, L), "his_mask": his,
         "user_id": torch.randint(1, USERS, (BT,), generator=g), "label": torch.zeros(BT, dtype=torch.long)}
    x["user_id"][0] = x["user_id"][BT // 2]    # one user row on both ranks: the sparse sum adds
    return {k: v.to(dev) for k, v in x.items()}


def _half(x, rank, world):
    n = BT // world
    return {k: v[rank * n:(rank + 1) * n].contiguous() for k, v in x.items()}


def _set_keep(model, case, keep):
    if case == "lstur":
        model.encoderU.keep_override = keep


def _worker(rank, world, port, case, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        import bench
        from newsrec_amd.dist import GradSync
        from newsrec_amd.manager import get_optim
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        steps = 4
        batches = [_batch(100 + i, dev) for i in range(steps)]
        keep = torch.ones(BT, dtype=torch.long, device=dev)   # device-resident: read inside the captured graph
        keep[1] = 0
        # reference: one process, whole batches, eager
        ref = _model(case, dev)
        _set_keep(ref, case, keep)
        o_ref = get_optim(ref)
        ref.train()
        for x in batches:
            bench.train_step(ref, o_ref, x, None)
        # this rank: half of every batch, gradients averaged over the two ranks
        m = _model(case, dev)
        _set_keep(m, case, keep[rank * BT // world:(rank + 1) * BT // world])
        m.train()
        sync = GradSync(m, bucket_mb=0.5)   # several dense buckets
        halves = [_half(x, rank, world) for x in batches]
        if mode == "eager":
            opt = get_optim(m)
            for x in halves:
                bench.train_step(m, opt, x, sync)
        else:   # two-graph step: 2 eager warm-up steps, capture, 2 replays
            opt = get_optim(m, capturable=True)
            g = bench.GraphedStep(m, opt, bench.ResidentFeed(halves), sync, 2)
            for i in range(2, steps):
                g(i)
        torch.cuda.synchronize()
        sync.close()
        diffs = {}
        for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
            d = (b.detach() - a.detach()).abs()
            diffs[n] = (d.max().item(), int((d > 1e-7).sum().item()), d.numel())
        q.put((rank, None, diffs))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # report instead of hanging the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))


@pytest.mark.parametrize("mode", ["eager", "graphs"])
@pytest.mark.parametrize("case", list(CASES))
def test_data_parallel_real_model_world2(case, mode):
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, case, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, err, diffs in res:
        assert err is None, err
        for n, (dmax, n_off, n_all) in diffs.items():
            if n.endswith("attention.self.key.bias"):
                # BERT's key bias adds q . b_k to every score of a query: softmax cancels it, so its
                # gradient is zero in exact arithmetic and rounding noise here -- Adam's lr * g / |g|
                # turns that noise into +-lr moves on both sides; only the common bound applies
                assert dmax <= 4 * 2 * 6e-6 + 1e-7, (rank, n, dmax)
                continue
            # 4 Adam steps from identical state.  Adam moves each element by ~lr * g / |g|, so an
            # element whose gradient sits at the rounding level (the two ranks' half-batch means vs
            # one whole-batch mean) may differ by up to 2 lr per step; every other element agrees to
            # 1e-3 lr.  A missing or wrong exchange moves most elements off.
            assert dmax <= 4 * 2 * 1e-4 + 1e-6, (rank, n, dmax)
            assert n_off <= max(4, 1e-3 * n_all), (rank, n, n_off, n_all)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shard", [False, True])
def test_bench_gpus2_spawns_two_ranks(shard):
    """`bench.py --gpus 2` (no WORLD_SIZE) must launch two ranks itself (twotower.py:62-73) and
    report the live world size, with the 8-GPU configurations of BASELINE.json measured on those
    ranks too: configs[3] LSTUR (the row-sparse user-table exchange) and configs[4] XFormer, each
    with its replicas bitwise identical after the timed steps; gloo on the one leased GPU stands in
    for RCCL here."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["NR_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--eval-impr", "0", "--legs", "cnn_lstur", "--xformer-steps", "2", "--no-cpu-baseline"] + \
        (["--shard-table"] if shard else [])
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 64
    assert out["value"] > 0
    assert out["dp_bitwise_equal"] is True and out["dp_world_size"] == 2
    assert out["dp_shard_tables"] is shard
    for leg in (out["other_configs"]["cnn_lstur"], out["xformer"]):
        assert leg["n_gpus"] == 2 and leg["impressions_per_s"] > 0, leg
        assert leg["dp_world_size"] == 2 and leg["dp_in_sync"] is True, leg
        assert leg["dp_bitwise_equal"] is True, leg


def _shard_worker(rank, world, port, case, mode, q):
    """Dense all-reduce vs GradSync(shard_tables=True) on the same half batches: the sharded run's
    replicas bitwise identical across the ranks, and its parameters within Adam's rounding-level
    spread of the dense run's.  (Not bitwise against the dense run: a rank's local gradients are not
    bitwise reproducible from run to run -- the attention backward's parameter-gradient copies and the
    LayerNorm dgamma / dbeta take atomic adds in arrival order -- and Adam turns a gradient at the
    rounding level into a move of up to 2 lr; on the CPU, where the local gradients are deterministic,
    tests/test_dist_cpu.py asserts the sharded parameters BITWISE equal to the dense path's.)"""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        import bench
        from newsrec_amd.dist import GradSync
        from newsrec_amd.manager import get_optim
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        steps = 4
        halves = [_half(_batch(100 + i, dev), rank, world) for i in range(steps)]
        out = {}
        # dense twice (the run-to-run spread of this build's gradients, which Adam amplifies into moves
        # of up to 2 lr), then sharded
        for shard in ("dense", "dense2", True):
            m = _model(case, dev)
            m.train()
            sync = GradSync(m, bucket_mb=0.5, shard_tables=shard is True)
            if mode == "eager":
                opt = get_optim(m)
                for x in halves:
                    bench.train_step(m, opt, x, sync)
            else:
                opt = get_optim(m, capturable=True)
                g = bench.GraphedStep(m, opt, bench.ResidentFeed(halves), sync, 2)
                for i in range(2, steps):
                    g(i)
            torch.cuda.synchronize()
            if shard is True:
                sh = [p for p in m.parameters() if getattr(p, "_nr_shard", None) is not None]
                assert len(sh) == 1 and opt.state[sh[0]]["exp_avg"].shape[0] == sh[0]._nr_shard[1]
                chk = bench.dp_check(m, opt, world, dev)
                assert chk["dp_bitwise_equal"] and chk["dp_shard_tables"], chk
            sync.close()
            out[shard] = {n: p.detach().clone() for n, p in m.named_parameters()}
        diffs = {}
        for n in out["dense"]:
            d = (out[True][n] - out["dense"][n]).abs()
            noise = int(((out["dense2"][n] - out["dense"][n]).abs() > 1e-7).sum().item())
            diffs[n] = (d.max().item(), int((d > 1e-7).sum().item()), d.numel(), noise)
        q.put((rank, None, diffs))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))


@pytest.mark.parametrize("mode", ["eager", "graphs"])
@pytest.mark.parametrize("case", ["nrms", "xformer"])
def test_data_parallel_shard_tables_world2(case, mode):
    """GradSync(shard_tables=True) on the real models at world 2 (gloo on device tensors): the word
    table's gradient reduce-scattered in place, FusedAdam on the rank's row slab, the slabs all-gathered
    -- replicas bitwise identical (bench.dp_check), every parameter within the dense path's spread: the
    largest difference within Adam's 2 lr per step, and no more elements off than a second dense run
    differs from the first (plus a small slack) -- a slab Adam skipped or an all-gather that missed rows
    would move every row of it."""
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, case, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, err, diffs in res:
        assert err is None, err
        for n, (dmax, n_off, n_all, noise) in diffs.items():
            # the bounds of test_data_parallel_real_model_world2 (4 Adam steps, rounding-level gradients)
            lr = 6e-6 if "bert" in n else 1e-4
            assert dmax <= 4 * 2 * lr + 1e-6, (rank, n, dmax)
            assert n_off <= 2 * noise + max(4, 1e-3 * n_all), (rank, n, n_off, noise, n_all)
