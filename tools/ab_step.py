"""A/B of the NRMS train step (bench.py's headline, graphed, device-formed batches) under module-level
switches (newsrec_amd.functions NAME, or encoders.NAME / bench.NAME), interleaved in ONE process (rounds x variants), so box-to-box and
clock drift cancel.  python tools/ab_step.py DEDUP_ROWS=1 DEDUP_ROWS=0 [--rounds 3 --steps 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))

import torch

import bench
from newsrec_amd import functions as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    feed = bench.DeviceFeed(dev, 1, 0)
    steps = {}
    from newsrec_amd import encoders as EN
    mods = {"functions": F, "encoders": EN, "bench": bench}
    for v in a.variants:
        for kv in v.split(","):
            k, val = kv.split("=")
            mod = F
            if "." in k:   # module.NAME (functions, encoders, bench); bare NAME = functions.NAME
                m, k = k.split(".", 1)
                mod = mods[m]
            cur = getattr(mod, k)
            setattr(mod, k, bool(int(val)) if isinstance(cur, bool) else float(val) if isinstance(cur, float) else int(val))
        model = bench.build(dev)
        model.train()
        opt = bench.make_optim(model, capturable=True)
        steps[v] = bench.GraphedStep(model, opt, feed, None, 3)
    res = {v: [] for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            st = steps[v]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                st(i)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    print(json.dumps({v: {"ms_per_step": [round(x, 4) for x in ms], "min": round(min(ms), 4)} for v, ms in res.items()}))


if __name__ == "__main__":
    main()
