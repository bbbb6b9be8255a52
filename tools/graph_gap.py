"""How much of the graphed NRMS step is outside its kernels: per replay, GPU time between events
around the replay vs wall time per step over back-to-back replays; and the same step captured twice
into one graph (two train steps per replay).  One process, variants interleaved."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))

import torch

import bench


def main():
    dev = torch.device("cuda", 0)
    feed = bench.DeviceFeed(dev, 1, 0)
    model = bench.build(dev)
    model.train()
    opt = bench.make_optim(model, capturable=True)
    one = bench.GraphedStep(model, opt, feed, None, 3)
    two = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(two):
        bench.train_step(model, opt, feed.form(), None)
        bench.train_step(model, opt, feed.form(), None)
    torch.cuda.synchronize()
    res = {"one_wall_ms": [], "one_gpu_ms": [], "two_wall_ms_per_step": []}
    n = 20
    for r in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            one(i)
        torch.cuda.synchronize()
        res["one_wall_ms"].append((time.perf_counter() - t0) / n * 1e3)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            ev[i][0].record()
            one.graph.replay()
            ev[i][1].record()
        torch.cuda.synchronize()
        res["one_gpu_ms"].append(sum(a.elapsed_time(b) for a, b in ev) / n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n // 2):
            two.replay()
        torch.cuda.synchronize()
        res["two_wall_ms_per_step"].append((time.perf_counter() - t0) / n * 1e3)
    print(json.dumps({k: [round(x, 4) for x in v] for k, v in res.items()}))


if __name__ == "__main__":
    main()
