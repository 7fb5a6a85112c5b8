"""Per-kernel summary of a rocprofv3 kernel trace (the rocpd SQLite output
rocprofv3 7.x writes by default, or its --output-format csv kernel_trace.csv):
kernel name + grid, calls, average
and total duration, share of the total.  Optional --per NAME divides the
totals by the call count of that kernel (e.g. a once-per-step kernel) to give
microseconds per step.

usage: python tools/rocpd_stats.py <results.db | kernel_trace.csv> [--top N] [--per KERNEL] [--grep S]
"""
import argparse
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"^[A-Za-z_]+::", "", name)
    return name


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--per", default=None)
    ap.add_argument("--grep", default=None)
    ap.add_argument("--by-name", action="store_true", help="merge grids of one kernel")
    a = ap.parse_args(argv)
    if a.db.endswith(".csv"):  # rocprofv3 --output-format csv kernel trace
        import csv
        rows = [(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]),
                 int(r["Grid_Size_Z"]), int(r["Workgroup_Size_X"]),
                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in csv.DictReader(open(a.db))]
    else:
        c = sqlite3.connect(a.db)
        rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration "
                         "from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    calls_by_name = defaultdict(int)
    for name, gx, gy, gz, wx, dur in rows:
        n = short(name)
        calls_by_name[n] += 1
        if a.by_name:
            key = (n, "", wx)
        else:
            wg = max(wx, 1)
            blocks = "%d" % (gx // wg) if gy == 1 else "%dx%d" % (gx // wg, gy)
            if gz > 1:
                blocks += "x%d" % gz
            key = (n, blocks, wx)
        agg[key][0] += 1
        agg[key][1] += dur
    tot = sum(v[1] for v in agg.values())
    per = None
    if a.per:
        hits = [k for k in calls_by_name if a.per in k]
        if not hits:
            sys.exit("no kernel matches --per %s" % a.per)
        per = calls_by_name[hits[0]]
    print("%-64s %10s %5s %6s %10s %10s %6s" % ("kernel", "blocks", "wg", "calls", "avg_us",
                                             "us/step" if per else "total_us", "pct"))
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.grep:
        items = [kv for kv in items if a.grep in kv[0][0]]
    for (n, blocks, wx), (cnt, dur) in items[:a.top]:
        t = dur / 1e3 / per if per else dur / 1e3
        print("%-64s %10s %5d %6d %10.1f %10.1f %5.2f%%" % (n[:64], blocks, wx, cnt, dur / cnt / 1e3,
                                                          t, 100 * dur / tot))
    print("total %.1f ms%s over %d dispatches" % (tot / 1e6 / (per or 1),
                                                  " per step" if per else "", len(rows)))


if __name__ == "__main__":
    main()
