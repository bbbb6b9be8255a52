"""Kernel time of one train step from a rocprofv3 kernel trace whose step ends in SEVERAL optimizer
launches (XFormer: ~200 parameters, 32 per nr_adam_multi launch), grouped by kernel name.
python tools/step_groups.py TRACE_DIR [BACK]: the BACK-th last complete step (a step = the kernels
after one run of consecutive Adam launches up to and including the next run)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
is_adam = ["adam_multi" in r["Kernel_Name"] for r in rows]
ends = [i for i in range(len(rows)) if is_adam[i] and (i + 1 == len(rows) or not is_adam[i + 1])]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
seg = rows[ends[-1 - back] + 1:ends[-back] + 1]
agg = collections.OrderedDict()
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"][:90]
    n, t = agg.get(k, (0, 0.0))
    agg[k] = (n + 1, t + d)
tot = sum(t for _, t in agg.values())
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%9.1f us %4d  %s" % (t, n, k))
print("%9.1f us total over %d kernels; wall %.1f us" % (tot, len(seg), (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3))
