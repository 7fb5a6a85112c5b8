"""Per-kernel summary of rocprofv3 --pmc CSVs (tools/_r3o.sh): counter sums
per kernel name, shown relative to SQ_WAVE_CYCLES / per wave where useful."""
import collections
import csv
import sys


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return agg, disp


if __name__ == "__main__":
    a1, d1 = load(sys.argv[1])
    a2, _ = load(sys.argv[2]) if len(sys.argv) > 2 else ({}, {})
    top = sorted(a1, key=lambda k: -a1[k].get("SQ_BUSY_CYCLES", 0))[:12]
    for k in top:
        c = dict(a1[k])
        c.update(a2.get(k, {}))
        wc = c.get("SQ_WAVE_CYCLES", 1)
        waves = c.get("SQ_WAVES", 1)
        print("%-70s n=%d" % (k, len(d1[k])))
        print("   wave-cycle shares: wait_any %.2f wait_inst %.2f active %.2f valu %.2f lds %.2f"
              % tuple(c.get(x, 0) / wc for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                  "SQ_ACTIVE_INST_LDS")))
        print("   mfma_busy/busy %.3f  per wave: valu %.0f mfma %.0f lds %.0f vmem %.0f  "
              "lds_conflict/lds %.3f wait_inst_lds/wc %.3f"
              % (c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(c.get("SQ_BUSY_CYCLES", 1), 1),
                 c.get("SQ_INSTS_VALU", 0) / waves, c.get("SQ_INSTS_MFMA", 0) / waves,
                 c.get("SQ_INSTS_LDS", 0) / waves, c.get("SQ_INSTS_VMEM", 0) / waves,
                 c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 1), 1),
                 c.get("SQ_WAIT_INST_LDS", 0) / wc))
