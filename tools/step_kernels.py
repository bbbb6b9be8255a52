"""Kernels of one train step in a rocprofv3 kernel trace (between two consecutive Adam launches), with
durations.  python tools/step_kernels.py TRACE_DIR [BACK]: BACK = 1 (default) takes the last segment;
bench.py's trace ends with its eager probe step, so BACK = 2 is its last graphed step."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adam_multi" in r["Kernel_Name"]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
seg = rows[ad[-1 - back] + 1:ad[-back] + 1]
tot = 0.0
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print("%7.1f  %s" % (d, r["Kernel_Name"][:100]))
print("%7.1f  total over %d kernels" % (tot, len(seg)))
