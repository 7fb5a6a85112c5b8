"""Memory-path counters per kernel (rocprofv3 --pmc CSV passes of a short
bench.py run, tools/gpu/r14z.sh): TA / TD busy as a fraction of the GPU's
active cycles (TA_BUSY_avr per instance; TD_TD_BUSY_sum over the 256 CUs),
the TA address stalls on the L1 (TCP) and the L1 pending stalls per CU-cycle,
the L1 -> L2 read latency in cycles, the L2 (TCC) hit rate.  Kernels keyed by
name + grid (grid in threads).  A "busy" counter counts cycles with work in
flight, not bandwidth used.
usage: python tools/pmc_mem.py <csv> [<csv> ...]"""
import collections
import csv
import re
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = re.sub(r"\(.*$", "", r["Kernel_Name"].replace("void ", "").replace(
                "(anonymous namespace)::", ""))[:48]
            key = "%s [%s]" % (name, r.get("Grid_Size", r.get("Grid_Size_X", "")))
            agg[key][r["Counter_Name"] + "@" + path[-40:]] += float(r["Counter_Value"])
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[key].add((path, r["Dispatch_Id"]))

    def g(c, k):
        return c.get(k, 0.0)
    rows = sorted(agg.items(), key=lambda kv: -g(kv[1], "GRBM_GUI_ACTIVE"))[:14]
    print("%-62s %6s %6s %7s %8s %6s %7s" % ("kernel [grid]", "TAbusy", "TDbusy", "TAstlTC",
                                            "L1->L2", "L2hit", "pend"))
    for k, c in rows:
        # GRBM_GUI_ACTIVE summed over the passes that held it: per-pass average
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md's
        # MFMA-utilisation recipe divides it by 8), and over the passes that held it
        npass = sum(1 for kk in c if kk.startswith("GRBM_GUI_ACTIVE@"))
        act = g(c, "GRBM_GUI_ACTIVE") / max(npass, 1) / 8
        ta = g(c, "TA_BUSY_avr") / act if act else 0
        td = g(c, "TD_TD_BUSY_sum") / (act * 256) if act else 0
        tas = g(c, "TA_ADDR_STALLED_BY_TC_CYCLES_sum") / (act * 256) if act else 0
        lat = g(c, "TCP_TCC_READ_REQ_LATENCY_sum") / max(g(c, "TCP_TCC_READ_REQ_sum"), 1)
        hit = g(c, "TCC_HIT_sum") / max(g(c, "TCC_HIT_sum") + g(c, "TCC_MISS_sum"), 1)
        pend = g(c, "TCP_PENDING_STALL_CYCLES_sum") / (act * 256) if act else 0
        print("%-62s %6.2f %6.2f %7.2f %8.0f %6.2f %7.2f" % (k[:62], ta, td, tas, lat, hit, pend))


if __name__ == "__main__":
    main()
