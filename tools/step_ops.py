"""Attributes the NRMS train step's GPU kernels to the Python lines that launch them (torch.profiler
with stacks over eager steps), to find the small torch-side kernels (fills, copies, cats) between
the library's own.  python tools/step_ops.py [--steps 2] [--filter Fill,Cat,copy,fill]"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda", 0)
    model = bench.build(dev)
    model.train()
    opt = bench.make_optim(model, capturable=True)
    feed = bench.DeviceFeed(dev, 1, 0)
    for i in range(2):
        feed.feed(i)
        bench.train_step(model, opt, feed.form(), None)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(a.steps):
            feed.feed(i)
            bench.train_step(model, opt, feed.form(), None)
        torch.cuda.synchronize()
    keys = [k for k in a.filter.split(",") if k]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        kern = [k for k in ev.kernels] if hasattr(ev, "kernels") else []
        for k in kern:
            name = k.name
            if keys and not any(x in name for x in keys):
                continue
            stack = [f for f in (ev.stack or []) if "newsrec_amd" in f or "bench.py" in f or "torch/nn" in f]
            site = " < ".join(stack[:3]) if stack else "(no python frame) " + ev.name
            agg[(name[:60], ev.name, site)][0] += 1
            agg[(name[:60], ev.name, site)][1] += k.duration / 1e3 if hasattr(k, "duration") else 0.0
    for (kn, op, site), (n, us) in sorted(agg.items(), key=lambda t: -t[1][1]):
        print("%5.1f calls/step %8.1f us/step  %-40s %-28s %s" % (n / a.steps, us / a.steps, kn, op[:28], site))


if __name__ == "__main__":
    main()
