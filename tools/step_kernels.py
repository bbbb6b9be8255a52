"""Kernels of the last graphed train step in a rocprofv3 kernel trace (between the last two Adam
launches), with durations.  python tools/step_kernels.py TRACE_DIR"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adam_multi" in r["Kernel_Name"]]
seg = rows[ad[-2] + 1:ad[-1] + 1]
tot = 0.0
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print("%7.1f  %s" % (d, r["Kernel_Name"][:100]))
print("%7.1f  total over %d kernels" % (tot, len(seg)))
