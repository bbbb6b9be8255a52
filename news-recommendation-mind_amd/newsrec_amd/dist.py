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
    """All-reduce-SUM of every gradient over the group; ``__call__`` (after backward) returns the
    1/world factor for ``FusedAdam.step(grad_scale=...)``.

    overlap_tables: install the word-table gradient hook so the table's all-reduce starts inside
    the backward (the Function then hands the table its gradient directly)."""

    def __init__(self, model, group=None, overlap_tables=True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.pending = []
        self.overlap = overlap_tables and self.world > 1
        if self.overlap:
            functions.TABLE_GRAD_HOOK.set(self._table_hook)

    def _table_hook(self, table, dtable):
        work = dist.all_reduce(dtable, group=self.group, async_op=True)
        self.pending.append((table, dtable, work))
        return True

    def close(self):
        if self.overlap:
            functions.TABLE_GRAD_HOOK.set(None)

    def __call__(self):
        if self.world == 1:
            return 1.0
        hooked = {id(t) for t, _, _ in self.pending}
        works = [dist.all_reduce(p.grad, group=self.group, async_op=True)
                 for p in self.model.parameters() if p.grad is not None and id(p) not in hooked]
        for w in works:
            w.wait()
        for table, dtable, w in self.pending:
            w.wait()
            if table.grad is None:
                table.grad = dtable
            else:
                table.grad.add_(dtable)
        self.pending = []
        return 1.0 / self.world
