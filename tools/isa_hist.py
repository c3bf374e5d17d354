"""Static opcode histogram of the loops of one kernel in a --save-temps .s.

  make -C raytraceheattransfer.jl_amd/csrc asm
  python tools/isa_hist.py raytraceheattransfer.jl_amd/csrc/_build/rthx_kernels-hip-amdgcn-amd-amdhsa-gfx950.s \
      "trace_exchange_kernel<true, 1, false, true, false, false, true, 1>" [--top 60]

A loop is the run of basic blocks from a label to the last branch back to it
(natural loops of the straight-line layout the compiler emits).  For every
loop the tool prints its line range and its instruction classes; for the
loops with the most fp64 FMAs (the ray loops) it prints the whole opcode
histogram.  Classes: fp64 (v_*_f64 except conversions / compares /
transcendentals), fp64 transcendental (v_rcp/rsq/sqrt_f64, v_div_*, v_frexp,
v_ldexp), VALU int32 (v_*_u32/_i32/_b32 arithmetic and bit ops), VALU other
(compares, conversions, selects, moves, 64-bit integer), SALU, VMEM, LDS,
branch / wait / misc.  Static counts: each instruction once, not weighted by
how often it runs.
"""
import argparse
import re
import subprocess
import sys
from collections import Counter, OrderedDict


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return out[:len(names)]


def kernel_lines(path, want):
    lines = open(path).read().split("\n")
    starts = [(i, ln[:-1]) for i, ln in enumerate(lines) if re.match(r"^_Z[A-Za-z0-9_]*:", ln)]
    starts = [(i, n.split(":")[0]) for i, n in starts]
    dem = demangle([n for _, n in starts])
    for (i, n), d in zip(starts, dem):
        if want in d:
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                j += 1
            return lines[i:j], d
    sys.exit(f"kernel {want!r} not found")


def classify(op):
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_barrier", "s_sleep", "s_setprio", "s_endpgm"):
        return "wait/misc"
    if op.startswith("s_cbranch") or op in ("s_branch", "s_setpc_b64", "s_swappc_b64"):
        return "branch"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("v_"):
        if re.search(r"_f64", op):
            if re.match(r"v_(rcp|rsq|sqrt|div_|frexp|ldexp|fract|trig|exp|log)", op):
                return "VALU fp64 transcendental"
            if op.startswith(("v_cmp", "v_cvt", "v_cndmask")):
                return "VALU other"
            return "VALU fp64"
        if re.search(r"_(u32|i32|b32|u16|i16|b16)(_e32|_e64|_dpp|_sdwa)?$", op) and not op.startswith(
                ("v_cmp", "v_cvt", "v_cndmask", "v_mov", "v_readfirstlane", "v_readlane", "v_writelane")):
            return "VALU int32"
        return "VALU other"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=80)
    ap.add_argument("--loops", type=int, default=2, help="full histograms of this many fp64-heaviest loops")
    ap.add_argument("--dump", default="", help="print instructions FIRST-LAST (the numbering of the loop list)")
    a = ap.parse_args()
    body, name = kernel_lines(a.asm, a.kernel)
    print(f"kernel: {name}")
    labels, insts = {}, []  # label -> index of its first instruction; (op, text, line)
    for k, ln in enumerate(body):
        s = ln.strip()
        m = re.match(r"^(\.LBB[0-9_]+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not s or s.startswith((";", ".", "_Z")) or s.endswith(":"):
            continue
        op = s.split()[0]
        insts.append((op, s, k))
    # loops: branch at i back to a label at j <= i
    loops = {}
    for i, (op, s, _k) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                j = labels[tgt]
                loops[j] = max(loops.get(j, i), i)
    spans = sorted(loops.items())
    if a.dump:
        first, last = (int(x) for x in a.dump.split("-"))
        at = {v: k for k, v in labels.items()}
        for t in range(first, last + 1):
            if t in at:
                print(f"{at[t]}:")
            print(f"  {t:5d}  {insts[t][1]}")
        return
    print(f"{len(insts)} instructions, {len(spans)} loops")
    rows = []
    for j, i in spans:
        ops = [insts[t][0] for t in range(j, i + 1)]
        cls = Counter(classify(o) for o in ops)
        rows.append((j, i, ops, cls))
        print(f"  loop insts {j}-{i} ({i - j + 1}): " + ", ".join(f"{c} {n}" for c, n in sorted(cls.items())))
    heavy = sorted(rows, key=lambda r: -sum(1 for o in r[2] if classify(o) == "VALU fp64"))[:a.loops]
    for j, i, ops, cls in heavy:
        print(f"\n== loop insts {j}-{i}: {i - j + 1} instructions")
        order = ["VALU fp64", "VALU fp64 transcendental", "VALU int32", "VALU other", "SALU", "LDS", "VMEM",
                 "branch", "wait/misc", "other"]
        for c in order:
            if cls.get(c):
                print(f"  {c:26s} {cls[c]:5d}")
        print("  opcodes:")
        for op, n in Counter(ops).most_common(a.top):
            print(f"    {n:5d}  {op:28s} {classify(op)}")


if __name__ == "__main__":
    main()
