"""Summarise a rocprofv3 kernel trace: per-kernel (name, grid) groups, so the
dominant kernel (head.conv2: conv_mfma_kernel<128,128> with 19200*8/8 blocks
at B=8) can be read separately from the other 128x128 convs."""
import collections
import csv
import sys


def main(path, top=25):
    rows = list(csv.DictReader(open(path)))
    g = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        key = (name[:70], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
               int(r["Workgroup_Size_X"]))
        g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in g.values())
    print("%-72s %8s %5s %6s %12s %7s" % ("kernel", "blocks", "wg", "calls", "avg_us", "pct"))
    for (name, blocks, wg), v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print("%-72s %8d %5d %6d %12.1f %6.2f%%" % (name, blocks, wg, len(v), sum(v) / len(v) / 1e3,
                                                  100.0 * sum(v) / tot))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
