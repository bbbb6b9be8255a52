"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) per kernel: calls, average and
total duration, share of GPU time.  Full template names are kept so instantiations of one
kernel template (e.g. the projection GEMM vs the wgrad GEMM) get separate lines.

usage: python tools/kernel_summary.py gpurun_out/bprof/b_results.db [--csv out.csv] [--short]
"""
import argparse
import re
import sqlite3


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"\(.*$", "", name)          # drop argument lists
    name = name.replace("void ", "")
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--short", action="store_true", help="merge template instantiations")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, duration from kernels").fetchall()
    agg = {}
    for name, d in rows:
        k = short(name)
        if a.short:
            k = re.sub(r"<.*$", "", k)
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, t + d)
    total = sum(t for _, t in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ["kernel,calls,avg_us,total_us,total_pct"]
    for k, (c, t) in out[: a.top]:
        lines.append('"%s",%d,%.1f,%.1f,%.2f' % (k, c, t / c / 1e3, t / 1e3, 100 * t / total))
    print("\n".join(lines))
    print("# total kernel time %.1f us over %d dispatches" % (total / 1e3, len(rows)))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
