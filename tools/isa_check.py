"""ISA checks on the built libposfeat_hip.so (CPU only, no GPU needed).

Extracts the gfx950 code objects from the library's clang offload bundles,
disassembles them with llvm-objdump and checks properties the kernels' counted
waits rely on but the source cannot pin by itself:

* conv_bf6d_kernel: inside the K loop every wave-instruction batch of B-plane
  LDS-DMA (global_load_lds_dwordx4) is issued BEFORE the A register loads
  (global_load_dwordx4) of the same step, and no `s_waitcnt vmcnt(0)` sits
  between them (the counted vmcnt(4) / vmcnt(4 D) waits assume exactly four
  younger A loads per chunk).
* every kernel: no MFMA reads a VGPR written by v_cvt_pk_bf16_f32 within the
  two preceding instructions without an s_nop between (the VALU-write ->
  MFMA-SrcA/B wait states).  The conversion once came from inline asm, whose
  VGPR write the compiler's hazard recognizer does not see: it padded
  nothing and the MFMAs read stale operands (nondeterministic results,
  DESIGN.md 4.1n).
* every kernel: no v_pk_fma_f32 whose LOW result reads the HIGH dword of a
  source pair that is also its destination (`v_pk_fma_f32 v[120:121], v[236:237],
  v[120:121], v[174:175] op_sel:[0,1,0]`).  Round 4's packed y interpolation in
  up4tap_gcombine_kernel (commit b97528c, POSFEAT_GC_ABL=16) compiled to nine
  of these and gave run-to-run different low results in lanes 48-63 (the last
  16-lane pass of the wave) -- 23 of 29 repeats on an MI355X, 29 of 29 with an
  extra s_waitcnt lgkmcnt(0) before its barriers, 0 of 19 for the scalar form
  (profiles/round5/gcombine_pk_probe_r13a.txt).  The compiler
  pads nothing for it, so no shipped kernel may contain it.  The same in-place
  low<-high read on v_pk_add_f32 / v_pk_mul_f32 / v_pk_mov_b32 (ocml's
  log1pf, 64-bit pair copies), and every other in-place cross-half read
  (op_sel_hi selecting the low dword for the high result), fail too (round
  6): the kernels that held them are built without packed-fp32 ops
  (PF_NO_PK_FP32 in common.h).
* every kernel: no s_barrier crossed with an LDS load or store of the wave
  still outstanding (straight-line scan; the state resets at an
  unconditional branch).  The bf6d / bf6s K loops held ten, whose safety
  rested on timing (the DMA refilling the stage after the barrier lands a
  global-memory latency after the wave's last fragment reads); they wait
  lgkmcnt(0) with their counted vmcnt now.
* every kernel: no device-function call (s_swappc): a kernel built without
  packed-fp32 ops does not inline a callee built with them.

usage: python tools/isa_check.py [--dump KERNEL_SUBSTRING] [--lib PATH]
Exit status 1 on a violated property.  tests/test_weights_abi.py runs it.
"""
import argparse
import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "posfeat_amd", "libposfeat_hip.so")
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path=LIB):
    """The gfx950 ELF code objects of every offload bundle in the library."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return out


def disassemble(blobs):
    text = []
    with tempfile.TemporaryDirectory() as td:
        for i, b in enumerate(blobs):
            f = os.path.join(td, "co%d.o" % i)
            open(f, "wb").write(b)
            r = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f], capture_output=True,
                               text=True, check=True)
            text.append(r.stdout)
    return "\n".join(text)


def functions(asm):
    """{symbol: [instruction lines]} from llvm-objdump output."""
    funcs, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur and line.strip() and not line.startswith("Disassembly"):
            funcs[cur].append(line.strip())
    return funcs


def check_bf6d(name, body):
    """Per K-loop step: [B DMA batch] then [A loads], no vmcnt(0) in between."""
    errs = []
    ops = []
    for ln in body:
        op = ln.split()[0]
        if op.startswith("global_load_lds"):
            ops.append("B")
        elif op.startswith("global_load_dwordx4"):
            ops.append("A")
        elif op == "s_waitcnt" and "vmcnt(0)" in ln:
            ops.append("W0")
        elif op.startswith("v_mfma"):
            ops.append("M")
        elif op == "s_barrier":
            ops.append("S")
        elif op.startswith("ds_"):
            ops.append("L")
        elif op.startswith(("global_store", "buffer_store", "s_endpgm")):
            ops.append("G")
        elif op.startswith("s_cbranch") or op == "s_branch":
            ops.append("J")
    # collapse runs; inspect every B-batch that has A loads after it before the
    # next MFMA: between the B batch and its A loads no W0 may occur, and no A
    # load may precede the B batch within that step
    seq = []
    for o in ops:
        if seq and seq[-1][0] == o:
            seq[-1][1] += 1
        else:
            seq.append([o, 1])
    nsteps = 0
    for i, (o, n) in enumerate(seq):
        if o != "B":
            continue
        # the step: from this B batch to the next MFMA run
        j = i + 1
        step = []
        while j < len(seq) and seq[j][0] not in ("M", "B", "S", "L", "G"):
            step.append(seq[j][0])
            j += 1
        if "A" in step:
            nsteps += 1
            if "W0" in step[:max(k for k, s in enumerate(step) if s == "A") + 1]:
                errs.append("%s: s_waitcnt vmcnt(0) between a B-DMA batch and its A loads" % name)
        # the A loads of a step must all come after its B batch: an A run
        # between the step's barrier and this B batch is a reordering
        # (straight-line only: barrier, A loads, this B batch with nothing else
        # between -- the prologue's A(0..D-2) -> B(0) -> A(D-1) order is intended)
        if i >= 2 and seq[i - 1][0] == "A" and seq[i - 2][0] == "S":
            errs.append("%s: A loads issued before the B-DMA batch of their step" % name)
    if nsteps == 0:
        errs.append("%s: no B-DMA -> A-load step found (pattern changed?)" % name)
    return errs, nsteps


def _regs(s):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]|v(\d+)\b", s):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check_cvt_mfma_hazard(name, body):
    ins = [ln.split("//")[0].strip() for ln in body if ln.split("//")[0].strip()]
    errs = []
    for i, ln in enumerate(ins):
        if not ln.startswith("v_mfma"):
            continue
        ops = ln.split(None, 1)[1].split(",")
        if len(ops) < 3:
            continue
        src = _regs(ops[1]) | _regs(ops[2])
        for d in (1, 2):
            if i - d < 0:
                break
            p = ins[i - d]
            if p.startswith("s_nop"):
                break
            if p.startswith("v_cvt_pk_bf16_f32") and _regs(p.split(None, 1)[1].split(",")[0]) & src:
                errs.append("%s: MFMA %d instruction(s) after the v_cvt_pk_bf16_f32 that wrote its "
                            "operand, no wait state: %s" % (name, d, ln[:60]))
    return errs


def check_pk_inplace_swap(name, body):
    """v_pk_*_f32 / v_pk_mov_b32 whose destination pair is also a source pair
    read CROSS-HALF (op_sel selecting the high dword for the low result, or
    op_sel_hi selecting the low dword for the high result).  Measured on gfx950
    (DESIGN.md 4.1q): `v_pk_fma_f32 v[68:69], v[68:69], s[22:23], v[84:85]
    op_sel:[1,0,0]` gave run-to-run different low results in lanes 48-63 --
    the high result's write reached the register before the last quarter-wave
    read it.  The compiler inserts nothing for this, so no kernel may contain
    the pattern."""
    errs = []
    for ln in body:
        ins = ln.split("//")[0].strip()
        if not ins.startswith(("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_mov_b32")):
            continue
        op, rest = ins.split(None, 1)
        mods = {}
        for key in ("op_sel_hi", "op_sel"):
            m = re.search(key + r":\[([01,]+)\]", rest)
            if m:
                mods[key] = [int(x) for x in m.group(1).split(",")]
                rest = rest.replace(m.group(0), "")
        ops = [o.strip() for o in rest.split(",")]
        dst = _regs(ops[0])
        if not dst:
            continue
        sel = mods.get("op_sel", [0, 0, 0])
        selhi = mods.get("op_sel_hi", [1, 1, 1])
        for k, src in enumerate(ops[1:4]):
            if k >= len(sel) or not (_regs(src) & dst):
                continue
            if sel[k] == 1 or selhi[k] == 0:
                errs.append("%s: in-place cross-half packed op: %s" % (name, ins[:90]))
    return errs


def _pk_parse(ins):
    op, rest = ins.split(None, 1)
    mods = {}
    for key in ("op_sel_hi", "op_sel"):
        m = re.search(key + r":\[([01,]+)\]", rest)
        if m:
            mods[key] = [int(x) for x in m.group(1).split(",")]
            rest = rest.replace(m.group(0), "")
    rest = re.sub(r"\b(neg_lo|neg_hi):\[[01,]+\]", "", rest)
    return op, [o.strip() for o in rest.split(",")], mods


def pk_inplace_lo_from_hi(body, ops=("v_pk_fma_f32",)):
    """Packed ops whose low result reads the high dword of a source pair that
    is also the destination pair (op_sel[k] = 1 on an in-place source k)."""
    out = []
    for ln in body:
        ins = ln.split("//")[0].strip()
        if not ins.startswith(ops):
            continue
        op, args, mods = _pk_parse(ins)
        dst = _regs(args[0])
        sel = mods.get("op_sel", [0, 0, 0])
        for k, src in enumerate(args[1:4]):
            r = _regs(src)
            if k < len(sel) and sel[k] == 1 and len(r) == 2 and max(r) in dst:
                out.append(ins)
    return out


def check_lds_barrier(name, body):
    """s_barrier with an LDS load/store of this wave still outstanding."""
    errs, pending = [], []
    for ln in body:
        ins = ln.split("//")[0].strip()
        if not ins:
            continue
        op = ins.split()[0]
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", ins)
            if m:
                n = int(m.group(1))
                pending = pending[len(pending) - n:] if 0 < n < len(pending) else ([] if n == 0 else pending)
        elif op.startswith("ds_") or op.startswith(("s_load", "s_buffer_load")):
            pending.append(op)
        elif op == "s_branch":
            pending = []
        elif op == "s_barrier":
            lds = [o for o in pending if o.startswith("ds_") and "permute" not in o and "swizzle" not in o]
            if lds:
                errs.append("%s: s_barrier with %d LDS access(es) outstanding (%s)" % (name, len(lds), lds[-1]))
    return errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", default=None)
    ap.add_argument("--lib", default=LIB, help="library or object to check (default: the shipped one)")
    args = ap.parse_args()
    funcs = functions(disassemble(code_objects(args.lib)))
    if args.dump:
        for k, v in funcs.items():
            if args.dump in k:
                print("<%s>" % k)
                print("\n".join(v))
        return 0
    errs = []
    found = 0
    for k, v in funcs.items():
        if "conv_bf6d_kernel" in k or "conv_bf6s_kernel" in k:
            found += 1
            e, n = check_bf6d(k, v)
            # a vmcnt(0) drain is conservative (never wrong) but defeats the
            # prefetch: an error for the default depth D = 2, a warning for
            # the A/B depths 3 and 4
            default = "ELi2ELi" in k
            drains = [x for x in e if "vmcnt(0)" in x]
            if not default:
                e = [x for x in e if x not in drains]
            errs += e
            print("%-90s steps checked %d%s%s" % (k[:90], n, "  FAIL" if e else "",
                                                  "  (warning: vmcnt(0) drain)" if drains and not e
                                                  else ""))
    if not found and args.lib == LIB:
        errs.append("no conv_bf6d_kernel instance in %s" % LIB)
    nh = 0
    for k, v in funcs.items():
        e = check_cvt_mfma_hazard(k, v)
        nh += len(e)
        errs += e
    print("cvt_pk_bf16 -> MFMA operand hazards: %d" % nh)
    # every in-place cross-half packed op FAILS: the low<-high
    # v_pk_fma_f32 form gave run-to-run different results,
    # and the other forms (v_pk_add/mul/mov, and op_sel_hi reading the low
    # dword for the high result) are the same in-place cross-half read; the
    # kernels the compiler emitted them in are built without packed-fp32 ops
    # (PF_NO_PK_FP32, common.h)
    npk = collections.Counter()
    for k, v in funcs.items():
        e = check_pk_inplace_swap(k, v)
        npk[k] = len(e)
        errs += e
    print("in-place cross-half packed-fp32 ops: %d in %d kernels" % (
        sum(npk.values()), sum(1 for v in npk.values() if v)))
    nfma, nother = 0, collections.Counter()
    for k, v in funcs.items():
        bad = pk_inplace_lo_from_hi(v)
        nfma += len(bad)
        errs += ["%s: v_pk_fma_f32 low result reads the high dword of its own destination: %s"
                 % (k, b[:90]) for b in bad]
        for b in pk_inplace_lo_from_hi(v, ("v_pk_add_f32", "v_pk_mul_f32", "v_pk_mov_b32")):
            nother[k] += 1
            errs.append("%s: packed op low result reads the high dword of its own destination: %s"
                        % (k, b[:90]))
    print("in-place low<-high v_pk_fma_f32: %d" % nfma)
    print("in-place low<-high v_pk_add/mul/mov: %d in %s" % (
        sum(nother.values()), sorted(set(re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", k).split("E")[0]
                                         for k in nother))))
    # an s_barrier crossed with the wave's own LDS accesses outstanding FAILS:
    # the ordering must not rest on the LDS answering before another wave's
    # DMA lands (the bf6d / bf6s K loops wait lgkmcnt(0) with their vmcnt)
    nb = collections.Counter()
    for k, v in funcs.items():
        e = check_lds_barrier(k, v)
        nb[k] = len(e)
        errs += e
    print("s_barrier with LDS accesses outstanding: %d in %s" % (
        sum(nb.values()), sorted(set(re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", k).split("I")[0]
                                     for k in nb if nb[k]))))
    # no kernel calls a device function: a kernel built without packed-fp32
    # ops cannot inline a callee built with them, and the call would carry
    # the callee's own packed code (and a call's cost) into the kernel
    ncall = 0
    for k, v in funcs.items():
        calls = [ln for ln in v if ln.split("//")[0].strip().startswith("s_swappc")]
        if calls:
            ncall += len(calls)
            errs.append("%s: %d device-function call(s) (s_swappc)" % (k, len(calls)))
    print("device-function calls (s_swappc): %d" % ncall)
    for e in errs:
        print("ISA CHECK FAILED:", e)
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
