"""Data-parallel plumbing of the train/eval loop (utils/Manager.py:154-180, 211-213;
utils/utils.py:267-283; twotower.py:49-50, 62-73), MI355X-first:

* one process per GPU, ``torch.distributed`` over RCCL (the "nccl" backend) on xGMI;
* ``GradSync``: the DDP all-reduce-mean of every gradient.  The 94 MB word-table gradient is
  produced last in the backward, so it is handed to RCCL from INSIDE the news-tower backward
  (right after the dgrad/scatter GEMM) and reduces while the weight-gradient GEMM runs; the
  mean's 1/world is folded into the Adam kernel (``grad_scale``) instead of a scaling pass;
* ``shard_train`` / ``Partition_Sampler``: the reference's DistributedSampler (strided, padded)
  and contiguous eval partitions.
"""
import os
from datetime import timedelta

import torch
import torch.distributed as dist

from . import functions
from . import kernels as K


def setup(rank, world_size, backend="nccl", master_port="12355"):
    """Manager.setup (Manager.py:154-180) with the rendezvous on 127.0.0.1 (the reference's
    'localhost' may not resolve in containers) and a finite timeout."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", master_port)
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(rank)
        kw["device_id"] = torch.device("cuda", rank)
    dist.init_process_group(backend, rank=rank, world_size=world_size, timeout=timedelta(minutes=30), **kw)


def free_port(host="127.0.0.1"):
    """An unused TCP port on ``host`` for the rendezvous (the reference hard-codes 12355,
    Manager.py:160, which collides when two jobs share a node)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def spawn_ranks(world_size, argv, env=None, timeout=None):
    """twotower.py:62-73 (``mp.spawn(main, nprocs=world_size, join=True)``) for a script: start
    ``world_size`` fresh interpreters running ``argv`` with RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (torch.distributed.run's environment), wait
    for all of them and return the first non-zero exit code (0 when every rank succeeded).

    The caller must not have touched the GPU: each rank initialises its own device.  Like
    ``mp.spawn(join=True)``, one failing rank ends the job: the others are terminated by PID."""
    import subprocess
    import sys
    import time
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(free_port(base["MASTER_ADDR"]))
    procs = []
    for r in range(world_size):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world_size),
                 LOCAL_WORLD_SIZE=str(world_size), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    t0 = time.monotonic()
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
        if rc != 0 or (timeout is not None and time.monotonic() - t0 > timeout):
            rc = rc or 124
            for p in procs:
                p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.05)
    return rc


def shard_train(n, world_size, rank, shuffle=False, seed=0, epoch=0):
    """torch.utils.data.DistributedSampler index order (Manager.py:212): optional seeded
    shuffle, pad to a multiple of world_size by repeating from the front, take rank::world."""
    if shuffle:
        g = torch.Generator().manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    total = -(-n // world_size) * world_size
    pad = total - n
    if pad > 0:
        idx += (idx * (pad // len(idx) + 1))[:pad]
    return idx[rank:total:world_size]


class Partition_Sampler:
    """utils/utils.py:267-283: contiguous eval shards; the last rank takes the remainder."""

    def __init__(self, dataset, num_replicas, rank):
        per, extra = divmod(len(dataset), num_replicas)
        self.start = per * rank
        self.end = self.start + per + extra * (rank + 1 == num_replicas)

    def __iter__(self):
        return iter(range(self.start, self.end))

    def __len__(self):
        return self.end - self.start


class GradSync:
    """The DDP all-reduce-mean of every gradient; ``__call__`` (after backward) returns the 1/world
    factor for ``FusedAdam.step(grad_scale=...)``.

    * word table (dense [30522, 768] gradient, produced last in the backward): its all-reduce is
      started from INSIDE the news-tower backward (TABLE_GRAD_HOOK) and overlaps the remaining
      weight-gradient GEMMs;
    * row-sparse tables (LSTUR's 876,957-row user table, SPARSE_GRAD_HOOK): an exact row-sparse
      exchange -- all-gather of the step's (row id, gradient row) pairs, then every rank adds all
      ranks' rows in rank order into a dense gradient buffer that persists across steps (only the
      previous step's rows are re-zeroed) -- the same sum DDP's dense all-reduce forms, at B rows
      per rank instead of 526 MB;
    * every other gradient: flattened into buckets of <= ``bucket_mb`` MB, one all-reduce per
      bucket (a few large collectives over xGMI instead of one per parameter); a gradient of
      >= ``inplace_mb`` MB is all-reduced in place, never copied into a bucket.

    ``shard_tables`` (N > 1): the word tables' optimizer step is sharded by rows instead of
    replicated (ZeRO-1 for the two [V, 768] tables, BERT.py:16-21 / XFormer.py:44-48's
    word_embeddings): each rank owns a slab of ceil(V / world) rows, its gradient is
    reduce-scattered in place (every rank receives the complete sum of its own slab), FusedAdam
    updates that slab with moments for those rows only, and ``after_step`` all-gathers the updated
    slabs in place.  The wire bytes equal the all-reduce's (a ring all-reduce IS a reduce-scatter +
    an all-gather), while the table's Adam stream (28 B per element: 657 MB for the NRMS word table)
    and its moments (188 MB) drop world-fold per rank; every rank ends with the same bytes of every
    row, so replicas stay bitwise identical.  The parameter is re-homed into a buffer padded to
    world x slab rows (``p.data`` a view of it) and its gradient comes padded as well
    (functions.table_grad_buffer), so neither collective copies.  Dense all-reduce stays the default.

    ``deferred`` (a train step replayed as HIP graphs, bench.GraphedStep at N > 1): no collective
    is ever captured; they run between graphs.  The news tower's projection weight-gradient GEMM
    (WGRAD_DEFER_HOOK) is taken out of the backward, so the step is three graphs:
      1. forward + backward up to the word-table gradient, then ``take_sparse()`` (the sparse
         tables' persistent gradient buffers);
      -- ``issue(early)``: the word-table all-reduce (and any other in-place bucket complete after
         graph 1) starts on RCCL's stream;
      2. ``run_deferred()`` (the weight-gradient GEMMs, on ``gemm_cus`` CUs so RCCL keeps some)
         + ``pack()`` of the remaining dense buckets -- this graph runs BESIDE the all-reduce;
      -- ``exchange(packed, records, works)``: the bucket all-reduces and the sparse exchange, then
         every collective is waited for;
      3. ``unpack(packed)`` + the optimizer.
    The gradient tensors keep the graph pool's static addresses.
    """

    def __init__(self, model, group=None, overlap_tables=True, sparse_tables=True, bucket_mb=128, inplace_mb=16,
                 deferred=False, collective_cus=16, rows_add=None, shard_tables=False):
        self.model = model
        # the ordered row-sparse sum (nr_rows_add_ordered); host-only tests of this plumbing on CPU
        # tensors inject their own
        self.rows_add = rows_add if rows_add is not None else K.rows_add_ordered
        self.group = group
        self.world = dist.get_world_size(group)
        self.pending = []
        self.sparse = []
        self._dense, self._touched, self._gather_bufs = {}, {}, {}
        self.bucket_elems = int(bucket_mb * (1 << 20) // 4)
        self.inplace_elems = int(inplace_mb * (1 << 20) // 4)
        self.overlap = overlap_tables and self.world > 1
        self.use_sparse = sparse_tables and self.world > 1
        self.collective_cus = int(collective_cus)
        self._rec = []
        self._runs = []
        self._deferred = False
        self.shards = {}   # id(param) -> (param, padded storage, first row, slab rows)
        if shard_tables and self.world > 1:
            for name, p in model.named_parameters():
                if "word_embedding" in name and p.dim() == 2 and p.is_contiguous():
                    self._shard_param(p)
        if self.overlap:
            functions.TABLE_GRAD_HOOK.set(self._table_hook)
        if self.use_sparse:
            functions.SPARSE_GRAD_HOOK.set(self._sparse_hook)
        self.deferred = deferred

    def _shard_param(self, p):
        """Re-home p's rows into a buffer of world x slab rows (p.data a view of it) and mark the slab
        this rank's optimizer updates (optim.FusedAdam reads p._nr_shard = (first row, rows))."""
        V, E = p.shape
        S = -(-V // self.world)
        r = dist.get_rank(self.group)
        with torch.no_grad():
            padded = torch.zeros(self.world * S, E, device=p.device, dtype=p.dtype)
            padded[:V].copy_(p.data)
            p.data = padded[:V]
        row0 = r * S
        p._nr_shard = (row0, max(0, min(S, V - row0)))
        p._nr_grad_rows = self.world * S
        self.shards[id(p)] = (p, padded, row0, S)

    def _padded_grad(self, p, g):
        """g ([V, E], p's gradient) as the [world x slab, E] tensor it is the head of: the buffer
        functions.table_grad_buffer allocated padded (the reduce-scatter runs on it in place)."""
        _, padded, _, S = self.shards[id(p)]
        rows, E = padded.shape
        if (g.stride() != (E, 1) or
                g.untyped_storage().nbytes() < (g.storage_offset() + rows * E) * g.element_size()):
            raise RuntimeError("GradSync(shard_tables): the table gradient is not padded to %d rows "
                               "(functions.table_grad_buffer)" % rows)
        return g.as_strided((rows, E), (E, 1))

    def _reduce_scatter(self, p, g):
        full = self._padded_grad(p, g)
        _, _, row0, S = self.shards[id(p)]
        return dist.reduce_scatter_tensor(full[row0:row0 + S], full, group=self.group, async_op=True)

    def after_step(self):
        """After the optimizer step: all-gather every sharded table's updated slabs in place (each
        rank's slab of its padded storage), so every rank holds every row again."""
        for p, padded, row0, S in self.shards.values():
            dist.all_gather_into_tensor(padded, padded[row0:row0 + S], group=self.group)

    @property
    def deferred(self):
        return self._deferred

    @deferred.setter
    def deferred(self, on):
        self._deferred = bool(on)
        if self.overlap:
            functions.WGRAD_DEFER_HOOK.set(self._defer_hook if self._deferred else None, self.gemm_cus)

    @property
    def gemm_cus(self):
        """CUs a weight-gradient GEMM running beside a collective may use (the rest stay free for
        RCCL's kernels; 0 = no limit, e.g. without a GPU)."""
        if not torch.cuda.is_available():
            return 0
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        return max(1, cus - self.collective_cus) if self.collective_cus > 0 else 0

    @property
    def scale(self):
        return 1.0 / self.world

    def _defer_hook(self, run, out):
        self._runs.append((run, out))
        return True

    def run_deferred(self):
        """Launch the weight-gradient GEMMs the backward deferred (graph 2 of the graphed step);
        -> their output tensors.  ``self.kept`` holds the closures (and so their operands) alive
        for a graph that captured them."""
        runs, self._runs = self._runs, []
        cus = self.gemm_cus
        for run, _ in runs:
            run(cus)
        self.kept = runs
        return [out for _, out in runs]

    def _table_hook(self, table, dtable):
        if self.deferred:          # an ordinary gradient: all-reduced in exchange()
            return False
        if id(table) in self.shards:
            if table.grad is not None:
                raise RuntimeError("GradSync(shard_tables): accumulating into a sharded table's .grad is "
                                   "not supported; call optimizer.zero_grad(set_to_none=True) before backward")
            self.pending.append((table, dtable, self._reduce_scatter(table, dtable)))
            return True
        work = dist.all_reduce(dtable, group=self.group, async_op=True)
        self.pending.append((table, dtable, work))
        return True

    def _sparse_hook(self, table, rows, grads):
        rows = rows.reshape(-1).contiguous()
        grads = grads.reshape(rows.numel(), -1).contiguous()
        if self.deferred:          # recorded; exchanged between the graphs
            self._rec.append((table, rows, grads))
            return True
        ids, gs, w1, w2 = self._gather(table, rows, grads)
        self.sparse.append((table, ids, gs, w1, w2))
        return True

    def _gather(self, table, rows, grads):
        """Async all-gather of one sparse table's (row ids, gradient rows) into persistent
        [world, n] / [world, n, E] buffers (no per-step allocation); -> (ids, grads, work, work)."""
        key = id(table)
        bufs = self._gather_bufs.get(key)
        n = rows.numel()
        if bufs is None or bufs[0].shape != (self.world, n) or bufs[1].shape[1:] != grads.shape:
            bufs = (torch.empty(self.world, n, dtype=rows.dtype, device=rows.device),
                    torch.empty((self.world,) + tuple(grads.shape), dtype=grads.dtype, device=grads.device))
            self._gather_bufs[key] = bufs
        w1 = dist.all_gather_into_tensor(bufs[0].view(-1), rows, group=self.group, async_op=True)
        w2 = dist.all_gather_into_tensor(bufs[1].view(-1, *grads.shape[1:]), grads, group=self.group, async_op=True)
        return bufs[0], bufs[1], w1, w2

    def _sparse_buffer(self, table):
        """The dense gradient of a row-sparse table, allocated and zeroed ONCE: each step only
        re-zeroes the rows the previous step wrote (B * world rows instead of a 526 MB fill)."""
        buf = self._dense.get(id(table))
        if buf is None:
            buf = torch.zeros_like(table)
            self._dense[id(table)] = buf
        else:
            prev = self._touched.get(id(table))
            if prev is not None:
                buf.index_fill_(0, prev, 0.0)
        return buf

    def _sparse_reduce(self, table, ids, gs):
        buf = self._dense.get(id(table))
        if buf is not None and table.grad is not None and table.grad.data_ptr() == buf.data_ptr() \
                and not self.deferred:
            # eager mode: the buffer still installed as .grad from the previous step (grads not set
            # to None) could hold a dense gradient accumulated this step, which the row re-zeroing
            # would partly erase and the exchange would never reduce
            raise RuntimeError("GradSync: %s.grad is still the row-sparse exchange buffer; call "
                               "optimizer.zero_grad(set_to_none=True) before backward" % type(table).__name__)
        g = self._sparse_buffer(table)
        # every rank adds the same [world * n] rows in the same fixed order (rank-major, each id's rows
        # summed in ascending position by one wave, no atomics): the replicas stay bitwise identical
        # although LSTUR's dropped ids put about half of every rank's rows on row 0 (RNN.py:100-101)
        self.rows_add(gs.view(-1, gs.shape[-1]), ids.view(-1), g)
        self._touched[id(table)] = ids.reshape(-1).clone()   # the gather buffer is reused next step
        return g

    def close(self):
        if self.overlap:
            functions.TABLE_GRAD_HOOK.set(None)
            functions.WGRAD_DEFER_HOOK.set(None)
        if self.use_sparse:
            functions.SPARSE_GRAD_HOOK.set(None)
        for p, _, _, _ in self.shards.values():   # p keeps its padded storage (a view, same values)
            del p._nr_shard, p._nr_grad_rows
        self.shards.clear()
        self._dense.clear()       # the row-sparse buffers (526 MB for the LSTUR user table)
        self._touched.clear()
        self._gather_bufs.clear()

    def _buckets(self, params):
        """-> [(params, inplace)]: big gradients alone and in place, the rest in flat buckets."""
        out, cur, n = [], [], 0
        for p in params:
            if p.grad.numel() >= self.inplace_elems and p.grad.is_contiguous():
                out.append(([p], True))
                continue
            if cur and n + p.grad.numel() > self.bucket_elems:
                out.append((cur, False))
                cur, n = [], 0
            cur.append(p)
            n += p.grad.numel()
        if cur:
            out.append((cur, len(cur) == 1 and cur[0].grad.is_contiguous()))
        return out

    def _dense_params(self, skip):
        return [p for p in self.model.parameters()
                if p.grad is not None and id(p) not in skip and id(p) not in self.shards]

    # ---- deferred (graph) mode
    def take_sparse(self):
        """End of the forward/backward (graph 1): takes the step's sparse records and gives each
        sparse table its persistent gradient buffer as .grad (the optimizer reads it)."""
        rec, self._rec = self._rec, []
        for table, _, _ in rec:
            table.grad = self._sparse_buffer_noreset(table)
        return rec

    def pack(self, rec, deferred_outs=()):
        """-> (early, packed): in-place buckets complete after graph 1 (all-reduced while the
        deferred GEMMs run), and the rest (in-place buckets a deferred GEMM writes, and flat copies
        of the small gradients) for exchange() / unpack()."""
        skip = {id(t) for t, _, _ in rec}
        spans = [(o.data_ptr(), o.data_ptr() + o.numel() * o.element_size()) for o in deferred_outs]
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        for s, e in spans:
            # the deferred GEMM writes into the tensor the backward returned: autograd must have
            # installed it (or views of it) as the parameters' .grad, not a copy
            if not any(g.data_ptr() < e and s < g.data_ptr() + g.numel() * g.element_size() for g in grads):
                raise RuntimeError("GradSync: a deferred weight gradient is not any parameter's .grad "
                                   "(autograd copied it); its GEMM would write a detached buffer")
        early, packed = [], []
        for p, _, _, _ in self.shards.values():
            if p.grad is not None:   # the sharded tables: reduce-scattered in place by issue()
                g = p.grad
                a, b = g.data_ptr(), g.data_ptr() + g.numel() * g.element_size()
                if any(a < e and s < b for s, e in spans):
                    raise RuntimeError("GradSync(shard_tables): a deferred GEMM writes a sharded table's gradient")
                early.append(([p], g, "shard"))
        for bucket, inplace in self._buckets(self._dense_params(skip)):
            if inplace:
                g = bucket[0].grad
                a, b = g.data_ptr(), g.data_ptr() + g.numel() * g.element_size()
                late = any(a < e and s < b for s, e in spans)
                (packed if late else early).append((bucket, g.view(-1), True))
            else:
                packed.append((bucket, torch.cat([p.grad.reshape(-1) for p in bucket]), False))
        return early, packed

    def prepare(self):
        """The whole deferred preparation in one go (eager steps of a graphed run):
        -> (buckets, records) for exchange() / unpack()."""
        rec = self.take_sparse()
        outs = self.run_deferred()
        early, packed = self.pack(rec, outs)
        return early + packed, rec

    def issue(self, early):
        """Start the all-reduce of the buckets complete after graph 1 (async, RCCL's stream); the
        sharded tables' gradients are reduce-scattered in place instead."""
        return [self._reduce_scatter(b[0], flat) if kind == "shard" else
                dist.all_reduce(flat, group=self.group, async_op=True) for b, flat, kind in early]

    def _sparse_buffer_noreset(self, table):
        buf = self._dense.get(id(table))
        if buf is None:
            buf = torch.zeros_like(table)
            self._dense[id(table)] = buf
        return buf

    def exchange(self, packed, rec, works=()):
        """Eager, between the graphs: the remaining collectives of the step, then wait for all of
        them (``works``: those ``issue`` started)."""
        works = list(works) + self.issue(packed)
        gathers = [(table,) + self._gather(table, rows, grads) for table, rows, grads in rec]
        for table, ids, gs, w1, w2 in gathers:
            w1.wait()
            w2.wait()
            self._sparse_reduce(table, ids, gs)
        for w in works:
            w.wait()

    @staticmethod
    def unpack(packed):
        """Head of the optimizer (graph): copy the reduced buckets back into the gradients."""
        for bucket, flat, inplace in packed:
            if inplace:
                continue
            off = 0
            for p in bucket:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n

    def __call__(self):
        if self.world == 1:
            return 1.0
        if self.deferred:
            packed, rec = self.prepare()
            self.exchange(packed, rec)
            self.unpack(packed)
            return self.scale
        hooked = {id(t) for t, _, _ in self.pending} | {id(t) for t, *_ in self.sparse}
        flights = []
        # a sharded table whose backward did not hand its gradient to TABLE_GRAD_HOOK (the BERT tower's
        # word embeddings: BertFn returns it to autograd): reduce-scattered in place here
        for p, _, _, _ in self.shards.values():
            if id(p) not in hooked and p.grad is not None:
                flights.append(([p], p.grad, True, self._reduce_scatter(p, p.grad)))
        for bucket, inplace in self._buckets(self._dense_params(hooked)):
            flat = bucket[0].grad.view(-1) if inplace else torch.cat([p.grad.reshape(-1) for p in bucket])
            flights.append((bucket, flat, inplace, dist.all_reduce(flat, group=self.group, async_op=True)))
        for table, ids, gs, w1, w2 in self.sparse:
            w1.wait()
            w2.wait()
            g = self._sparse_reduce(table, ids, gs)
            if table.grad is None:
                table.grad = g
            elif table.grad.data_ptr() != g.data_ptr():
                table.grad.add_(g)
        self.sparse = []
        for bucket, flat, inplace, w in flights:
            w.wait()
            if not inplace:
                off = 0
                for p in bucket:
                    n = p.grad.numel()
                    p.grad.copy_(flat[off:off + n].view_as(p.grad))
                    off += n
        for table, dtable, w in self.pending:
            w.wait()
            if table.grad is None:
                table.grad = dtable
            else:
                table.grad.add_(dtable)
        self.pending = []
        return self.scale
