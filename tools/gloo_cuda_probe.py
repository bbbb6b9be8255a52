"""Probe the collectives GradSync(shard_tables=True) uses, on device tensors over gloo (the only
multi-rank transport on a one-GPU box): in-place reduce_scatter_tensor vs the all-reduce's slice,
out-of-place reduce_scatter_tensor, in-place / out-of-place all_gather_into_tensor, each right after a
kernel that writes its input (stream order).  python tools/gloo_cuda_probe.py  -> one JSON line."""
import json
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(rank + 1)
    S, E = 1000, 64
    res = {}
    base = torch.randn(world * S, E, device=dev, generator=g)
    ref = base * 2
    dist.all_reduce(ref)
    torch.cuda.synchronize()
    # in-place reduce-scatter after a kernel writes the input
    x = base.clone()
    x.mul_(2)
    w = dist.reduce_scatter_tensor(x[rank * S:(rank + 1) * S], x, async_op=True)
    w.wait()
    res["rs_inplace"] = bool(torch.equal(x[rank * S:(rank + 1) * S], ref[rank * S:(rank + 1) * S]))
    # out of place
    x = base.clone()
    x.mul_(2)
    out = torch.empty(S, E, device=dev)
    dist.reduce_scatter_tensor(out, x)
    res["rs_outofplace"] = bool(torch.equal(out, ref[rank * S:(rank + 1) * S]))
    # all-gather in place after a kernel writes the slab
    y = torch.zeros(world * S, E, device=dev)
    y[rank * S:(rank + 1) * S].fill_(rank + 1.0)
    dist.all_gather_into_tensor(y, y[rank * S:(rank + 1) * S])
    res["ag_inplace"] = all(bool((y[r * S:(r + 1) * S] == r + 1.0).all()) for r in range(world))
    y2 = torch.empty(world * S, E, device=dev)
    sl = torch.full((S, E), rank + 1.0, device=dev)
    dist.all_gather_into_tensor(y2, sl)
    res["ag_outofplace"] = all(bool((y2[r * S:(r + 1) * S] == r + 1.0).all()) for r in range(world))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    print(json.dumps(out))
