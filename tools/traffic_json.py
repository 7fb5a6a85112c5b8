"""HBM traffic of one kernel from rocprofv3 PMC passes (tools/pmc_conv2.sh):
bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB units; gfx950 FETCH_SIZE counts half
the bytes of wide streaming reads, MI355X_MICROARCH.md "FETCH_SIZE").
Averaged over the dispatches of the kernel whose name contains <kernel>
(B images per launch); writes {"bytes_per_launch_per_image": ...} for bench.py.

usage: python tools/traffic_json.py <pmc_dir> <out.json> [batch] [kernel] [algorithmic_bytes]
       [column=value ...]   (extra dispatch filters, e.g. Grid_Size=11059200)
"""
import collections
import csv
import json
import os
import sys


FILTERS = {}


def per_dispatch(path, counter, kernel):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if any(r.get(k) != v for k, v in FILTERS.items()):
            continue
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    for a in sys.argv[6:]:
        k, v = a.split("=", 1)
        FILTERS[k] = v
    d, out = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    kernel = sys.argv[4] if len(sys.argv) > 4 else "conv_up4_kernel"
    fetch = per_dispatch(os.path.join(d, "fetch", "pmc_counter_collection.csv"), "FETCH_SIZE", kernel)
    write = per_dispatch(os.path.join(d, "write", "pmc_counter_collection.csv"), "WRITE_SIZE", kernel)
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    total = (2.0 * f_kb + w_kb) * 1024.0
    # conv_up4_kernel: L (120x160x192) + y residual read + y write + its
    # phase weights (16 x 128 x 1728)
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else (
        batch * (120 * 160 * 192 + 2 * 480 * 640 * 128) * 4 + 16 * 128 * 1728 * 4)
    labels = [l for l in os.environ.get("LABELS", "").split(",") if l]
    rec = {"kernel": kernel, "filters": FILTERS, "labels": labels,
           "probe": os.environ.get("PROBE", "tools/up4_probe.py") + " (B=%d, 480x640)" % batch,
           "batch": batch, "fetch_kb_raw": f_kb, "write_kb": w_kb,
           "bytes_per_launch": total, "bytes_per_launch_per_image": total / batch,
           "algorithmic_bytes_per_launch": alg, "ratio_to_algorithmic": total / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (KB)"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
