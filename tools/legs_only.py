"""Run bench.config_legs alone (profiling helper): python tools/legs_only.py [leg ...] [--steps K];
``xformer`` alone runs bench.xformer_leg."""
import argparse
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("legs", nargs="*")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--set", action="append", default=[], help="NAME=INT: a newsrec_amd.functions switch (A/B)")
a = ap.parse_args()
from newsrec_amd import functions as F  # noqa: E402
for kv in a.set:
    k, v = kv.split("=")
    mod = F
    if "." in k:   # module.NAME (e.g. bert.ATTN_KEEP_BITS)
        import importlib
        m, k = k.rsplit(".", 1)
        mod = importlib.import_module("newsrec_amd." + m)
    setattr(mod, k, bool(int(v)) if isinstance(getattr(mod, k), bool) else int(v))
dev = torch.device("cuda", 0)
if a.legs == ["xformer"]:
    print(json.dumps(bench.xformer_leg(dev, steps=a.steps)))
else:
    feed = bench.DeviceFeed(dev, 1, 0)
    print(json.dumps(bench.config_legs(dev, feed, steps=a.steps, only=a.legs or None)))
