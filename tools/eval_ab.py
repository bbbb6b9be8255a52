"""A/B of the fast-eval leg (bench.fast_eval_leg: MIND-large-shaped dev split, news-table encode,
predict, metrics) under module switches of newsrec_amd.encoders (NAME=v) or bench (bench.NAME=v),
interleaved in one process.  python tools/eval_ab.py USER_POOL_FUSED=0 USER_POOL_FUSED=1 [--rounds 2]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))

import torch

import bench
from newsrec_amd import encoders as E


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = bench.build(dev)
    res = {v: [] for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            for kv in v.split(","):
                k, val = kv.split("=")
                mod, name = (bench, k.split(".", 1)[1]) if k.startswith("bench.") else (E, k)
                cur = getattr(mod, name)
                setattr(mod, name, bool(int(val)) if isinstance(cur, bool) else type(cur)(val))
            out = bench.fast_eval_leg(model, dev, 1, 0, bench.DEV_IMPR_LARGE)
            res[v].append({k: out[k] for k in ("predict_ms", "end_to_end_ms", "end_to_end_candidates_per_s",
                                               "metrics_random_model")})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
