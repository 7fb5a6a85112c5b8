"""HBM traffic of the head.conv2 launch from rocprofv3 PMC passes
(tools/pmc_conv2.sh): bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB units; gfx950
FETCH_SIZE counts half the bytes of wide streaming reads, MI355X_MICROARCH.md
"FETCH_SIZE").  Averaged over the conv dispatches of the probe (B images per
launch); writes {"bytes_per_launch_per_image": ...} for bench.py.

usage: python tools/traffic_json.py <pmc_dir> <out.json> [batch]
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "conv_" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    d, out = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    fetch = per_dispatch(os.path.join(d, "fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    total = (2.0 * f_kb + w_kb) * 1024.0
    alg = batch * 480 * 640 * (256 + 128) * 4 + 128 * 2304 * 4
    rec = {"kernel": "head.conv2 3x3 256->128 @480x640 (tools/conv2_probe.py)",
           "batch": batch, "fetch_kb_raw": f_kb, "write_kb": w_kb,
           "bytes_per_launch": total, "bytes_per_launch_per_image": total / batch,
           "algorithmic_bytes_per_launch": alg, "ratio_to_algorithmic": total / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (KB)"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
