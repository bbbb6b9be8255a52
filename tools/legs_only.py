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
a = ap.parse_args()
dev = torch.device("cuda", 0)
if a.legs == ["xformer"]:
    print(json.dumps(bench.xformer_leg(dev, steps=a.steps)))
else:
    feed = bench.DeviceFeed(dev, 1, 0)
    print(json.dumps(bench.config_legs(dev, feed, steps=a.steps, only=a.legs or None)))
