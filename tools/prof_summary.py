"""Summarise a rocprofv3 kernel trace: per-kernel (name, grid) groups, so the
dominant kernel can be read separately from the other convs of the same
template (batched launches show as "<blocks>x<grid_y>").

usage: python tools/prof_summary.py <kernel_trace.csv | results.db> [top] [--stats out.csv]
Accepts rocprofv3's CSV kernel trace or its SQLite output (`kernels` view);
--stats also writes the per-kernel-name table (calls, total, average, percent)
that `rocprofv3 --stats` prints.
"""
import collections
import csv
import sqlite3
import sys


def load(path):
    """-> list of (name, blocks, wg, duration_ns)"""
    out = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, gx, gy, wx, dur in c.execute(
                "select name, grid_x, grid_y, workgroup_x, duration from kernels"):
            b = int(gx) // max(1, int(wx))
            out.append((name, b if int(gy) <= 1 else "%dx%d" % (b, int(gy)), int(wx), int(dur)))
        return out
    for r in csv.DictReader(open(path)):
        b = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        gy = int(r.get("Grid_Size_Y", 1) or 1) // max(1, int(r.get("Workgroup_Size_Y", 1) or 1))
        out.append((r["Kernel_Name"], b if gy <= 1 else "%dx%d" % (b, gy),
                    int(r["Workgroup_Size_X"]),
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def clean(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0]
    top = int(args[1]) if len(args) > 1 else 25
    rows = load(path)
    g = collections.defaultdict(list)
    for name, blocks, wg, dur in rows:
        g[(clean(name)[:70], blocks, wg)].append(dur)
    tot = sum(sum(v) for v in g.values())
    print("%-72s %8s %5s %6s %12s %7s" % ("kernel", "blocks", "wg", "calls", "avg_us", "pct"))
    for (name, blocks, wg), v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print("%-72s %8s %5d %6d %12.1f %6.2f%%" % (name, blocks, wg, len(v), sum(v) / len(v) / 1e3,
                                                  100.0 * sum(v) / tot))
    if "--stats" in sys.argv:
        out = sys.argv[sys.argv.index("--stats") + 1]
        byname = collections.defaultdict(list)
        for name, _, _, dur in rows:
            byname[clean(name)].append(dur)
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, v in sorted(byname.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot])


if __name__ == "__main__":
    main()
