"""Summarise a tools/passes/r6t.sh output directory: test tails, XFormer ms/step per variant and
round, the attention-backward kernels' average durations per variant."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "tests_*.log"))):
    print(os.path.basename(f), open(f).read().strip().splitlines()[-1])
runs = {}
for f in sorted(glob.glob(os.path.join(d, "xf_*_*.json"))):
    v = os.path.basename(f)[3:-5].rsplit("_", 1)[0]
    runs.setdefault(v, []).append(json.load(open(f))["ms_per_step"])
for v, ms in runs.items():
    print(f"{v:6s} ms/step {ms}  mean {sum(ms) / len(ms):.2f}")
for k in sorted(glob.glob(os.path.join(d, "kt*", "run_kernel_stats.csv"))):
    for r in csv.DictReader(open(k)):
        if "attn_bwd" in r["Name"] and ("true, true" in r["Name"] or "_ds_" in r["Name"]):
            print(os.path.basename(os.path.dirname(k)), r["Name"][:62], r["Calls"], f"{float(r['AverageNs']) / 1e3:.1f} us")
