"""Static instruction mix of kernels in the built libposfeat_hip.so (CPU only).

For every kernel whose symbol contains the given substring: the number of VALU
(v_* without v_mfma), MFMA, LDS (ds_*), vector-memory (global_/buffer_), SALU
and branch instructions in its disassembly.  For straight-line (fully
unrolled) kernels the static count is the per-wave dynamic count, which is how
the VALU:MFMA ratios in DESIGN.md were first estimated before PMC confirmed
them (SQ_INSTS_VALU / SQ_INSTS_MFMA per wave).

usage: python tools/isa_stats.py KERNEL_SUBSTRING [--lib PATH]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402


def mix(body):
    c = collections.Counter()
    for ln in body:
        op = ln.split("//")[0].split()
        if not op:
            continue
        op = op[0]
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("v_pk_"):
            c["valu"] += 1
            c["valu_pk"] += 1
        elif op.startswith("v_") and ("f64" in op):
            c["valu"] += 1
            c["valu_f64"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_load_lds", "buffer_load_lds")):
            c["dma"] += 1
        elif op.startswith(("global_load", "buffer_load")):
            c["vload"] += 1
        elif op.startswith(("global_store", "buffer_store")):
            c["vstore"] += 1
        elif op.startswith("s_cbranch") or op == "s_branch":
            c["branch"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--lib", default=isa_check.LIB)
    a = ap.parse_args()
    funcs = isa_check.functions(isa_check.disassemble(isa_check.code_objects(a.lib)))
    keys = ["valu", "valu_pk", "valu_f64", "mfma", "lds", "dma", "vload", "vstore", "salu",
            "waitcnt", "branch"]
    for k, v in funcs.items():
        if a.kernel in k:
            c = mix(v)
            r = c["valu"] / c["mfma"] if c["mfma"] else float("nan")
            print("%s\n  %s  valu/mfma %.1f" % (k[:110], " ".join("%s %d" % (x, c[x]) for x in keys), r))


if __name__ == "__main__":
    main()
