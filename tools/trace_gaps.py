"""Device idle gaps and long HIP runtime calls in a rocprofv3 CSV trace
(--kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv):
the device busy fraction per time bin, every gap between kernels longer than
--gap µs with the kernels either side and the runtime calls that overlap it,
and the HIP calls longer than --long µs.  Times relative to the first kernel.

usage: python tools/trace_gaps.py <prof dir> [--gap 200] [--long 500] [--bin 50]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:60]


def load(d, suffix):
    fs = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap", type=float, default=200.0)
    ap.add_argument("--long", type=float, default=500.0)
    ap.add_argument("--bin", type=float, default=50.0, help="ms per busy bin")
    a = ap.parse_args()
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
          for r in load(a.dir, "kernel_trace.csv")]
    ks.sort()
    cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy"))
          for r in load(a.dir, "memory_copy_trace.csv")]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
           for r in load(a.dir, "hip_api_trace.csv")]
    api.sort()
    t0 = ks[0][0]
    print("kernels %d, copies %d, runtime calls %d, span %.1f ms" % (
        len(ks), len(cp), len(api), (ks[-1][1] - t0) / 1e6))
    # busy per bin (kernels merged as intervals: streams overlap)
    binw = a.bin * 1e6
    busy = defaultdict(float)
    cur_s, cur_e = ks[0][0], ks[0][1]
    merged = []
    for s, e, _ in ks[1:]:
        if s <= cur_e:
            cur_e = max(cur_e, e)
        else:
            merged.append((cur_s, cur_e))
            cur_s, cur_e = s, e
    merged.append((cur_s, cur_e))
    for s, e in merged:
        while s < e:
            b = int((s - t0) // binw)
            be = t0 + (b + 1) * binw
            busy[b] += min(e, be) - s
            s = min(e, be)
    print("device busy per %.0f ms bin:" % a.bin)
    line = []
    for b in range(int((ks[-1][1] - t0) // binw) + 1):
        line.append("%d:%.2f" % (b, busy[b] / binw))
    for i in range(0, len(line), 12):
        print("  " + " ".join(line[i:i + 12]))
    # gaps
    print("gaps > %.0f us (t ms, gap us, before -> after, overlapping runtime calls > 20 us):" % a.gap)
    ai = 0
    ngap, tgap = 0, 0.0
    for (s0, e0), (s1, e1) in zip(merged, merged[1:]):
        g = (s1 - e0) / 1e3
        if g < a.gap:
            continue
        ngap += 1
        tgap += g
        before = [k for k in ks if k[1] == e0]
        after = [k for k in ks if k[0] == s1]
        while ai < len(api) and api[ai][1] < e0:
            ai += 1
        calls = defaultdict(lambda: [0, 0.0])
        j = ai
        while j < len(api) and api[j][0] < s1:
            d = (api[j][1] - api[j][0]) / 1e3
            if d > 20:
                calls[api[j][2]][0] += 1
                calls[api[j][2]][1] += d
            j += 1
        cs = ", ".join("%s x%d %.0fus" % (k, v[0], v[1]) for k, v in
                       sorted(calls.items(), key=lambda kv: -kv[1][1])[:4])
        print("  %9.2f %8.0f  %s -> %s  [%s]" % ((e0 - t0) / 1e6, g,
                                                  before[0][2] if before else "?",
                                                  after[0][2] if after else "?", cs))
    print("gaps > %.0f us: %d, %.1f ms total" % (a.gap, ngap, tgap / 1e3))
    print("runtime calls > %.0f us:" % a.long)
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, f in api:
        d = (e - s) / 1e3
        if d > a.long:
            agg[f][0] += 1
            agg[f][1] += d
            if agg[f][0] <= 5:
                print("  %9.2f %8.0f us %s" % ((s - t0) / 1e6, d, f))
    for f, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("  total %s: %d calls, %.1f ms" % (f, n, t / 1e3))


if __name__ == "__main__":
    main()
