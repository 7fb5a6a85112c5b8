"""PMC view of one kernel's dispatches from the separate rocprofv3 --pmc passes
of tools/gpu_round.sh (<dir>/{fetch,write,sq}/pmc_counter_collection.csv).

  traffic   = 2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950's FETCH_SIZE counts half
              the bytes of wide streaming reads, MI355X_MICROARCH.md)
  clock     = GRBM_GUI_ACTIVE / 8 (sum over the 8 XCDs) / dispatch wall time
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
              the fraction of SIMD-cycles the matrix pipe was busy (the
              counter counts 32 cycles per v_mfma_f32_32x32x16_bf16)

usage: python tools/pmc_dominant.py <pmc_dir> <kernel substring> <Grid_Size> <out.json>
       [labels] [algorithmic_bytes]
"""
import collections
import csv
import json
import os
import sys


def dispatches(path, kernel, grid):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Grid_Size"] == grid:
            e = d[r["Dispatch_Id"]]
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            e["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return list(d.values())


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    pdir, kernel, grid, out = sys.argv[1:5]
    labels = sys.argv[5].split(",") if len(sys.argv) > 5 else []
    alg = float(sys.argv[6]) if len(sys.argv) > 6 else None
    f = dispatches(os.path.join(pdir, "fetch", "pmc_counter_collection.csv"), kernel, grid)
    w = dispatches(os.path.join(pdir, "write", "pmc_counter_collection.csv"), kernel, grid)
    s = dispatches(os.path.join(pdir, "sq", "pmc_counter_collection.csv"), kernel, grid)
    fetch_kb = mean([e["FETCH_SIZE"] for e in f])
    write_kb = mean([e["WRITE_SIZE"] for e in w])
    total = (2.0 * fetch_kb + write_kb) * 1024.0
    rec = {"kernel": kernel, "grid_size": int(grid), "labels": labels,
           "dispatches": {"fetch": len(f), "write": len(w), "sq": len(s)},
           "fetch_kb_raw": fetch_kb, "write_kb": write_kb, "bytes_per_launch": total,
           "method": "rocprofv3 --pmc, one pass per counter group (FETCH_SIZE | WRITE_SIZE | "
                     "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES); "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (KB)"}
    if alg:
        rec["algorithmic_bytes_per_launch"] = alg
        rec["ratio_to_algorithmic"] = total / alg
    if s:
        gui = mean([e["GRBM_GUI_ACTIVE"] for e in s]) / 8.0
        ns = mean([e["_ns"] for e in s])
        busy = mean([e["SQ_VALU_MFMA_BUSY_CYCLES"] for e in s])
        rec.update({"grbm_gui_active_per_xcd": gui, "dispatch_ns_profiled": ns,
                    "effective_clock_ghz": gui / ns,
                    "sq_valu_mfma_busy_cycles": busy,
                    "sq_busy_cycles": mean([e["SQ_BUSY_CYCLES"] for e in s]),
                    "sq_waves": mean([e["SQ_WAVES"] for e in s]),
                    "mfma_util": busy / (1024.0 * gui),
                    "mfma_busy_over_sq_busy": busy / mean([e["SQ_BUSY_CYCLES"] for e in s])})
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
