#!/usr/bin/env python3
"""Instruction-class histogram of one loop iteration of a device kernel, from
hipcc -S output (the non-product issue of one compressed
squaring).  The loop body is the innermost block range closed by a backward
branch whose header line carries --loop; each out-of-line callee's body is
counted once per call as given by --call NAME=COUNT.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o capi.s drand_amd/csrc/capi.hip
    python tools/isa_hist.py capi.s KERNEL --loop .LBB137_17 --call fp_mul_r=12 --call fp_reduce_r=8
"""
import argparse
import collections
import re


def body(asm, name):
    a = asm.index("\n" + name + ":")
    return asm[a:asm.index(".Lfunc_end", a)].split("\n")


def cls(ins):
    op = ins.split()[0]
    if op == "v_mad_u64_u32":
        return "v_mad_u64_u32"
    if op.startswith(("v_add", "v_sub", "v_addc", "v_subb")):
        return "valu_add_sub"
    if op.startswith(("v_lshr", "v_lshl", "v_ashr", "v_alignbit", "v_bfe", "v_and", "v_or", "v_xor", "v_bfi",
                      "v_perm")):
        return "valu_shift_logic"
    if op.startswith(("v_mov", "v_cndmask", "v_readlane", "v_writelane", "v_readfirstlane", "v_accvgpr")):
        return "valu_move_select"
    if op.startswith("v_cmp"):
        return "valu_compare"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "global_mem"
    if op.startswith("ds_"):
        return "lds"
    if op in ("s_swappc_b64", "s_setpc_b64"):
        return "call_return"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_nop", "s_sleep")):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def hist(lines):
    h = collections.Counter()
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        h[cls(t)] += 1
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--loop", required=True, help="label of the loop block (e.g. .LBB137_17)")
    ap.add_argument("--call", action="append", default=[], help="callee-substring=calls per iteration")
    a = ap.parse_args()
    asm = open(a.asm).read()
    k = body(asm, a.kernel)
    start = next(i for i, l in enumerate(k) if l.startswith(a.loop + ":"))
    end = next(i for i in range(start + 1, len(k)) if re.search(r"s_cbranch_\w+\s+" + re.escape(a.loop) + r"\b", k[i])
               or re.search(r"s_branch\s+" + re.escape(a.loop) + r"\b", k[i]))
    tot = hist(k[start:end + 1])
    rows = [("loop body", dict(tot))]
    names = re.findall(r"^(_Z\w+):", asm, re.M)
    for c in a.call:
        sub, n = c.split("=")
        fn = next(x for x in names if sub in x)
        h = hist(body(asm, fn))
        rows.append((f"{fn} x{n}", dict(h)))
        for kk, v in h.items():
            tot[kk] += int(n) * v
    allk = sorted(tot, key=lambda x: -tot[x])
    s = sum(tot.values())
    for name, h in rows:
        print(f"{name}: {sum(h.values())} instructions")
    print(f"per iteration: {s} instructions")
    for kk in allk:
        print(f"  {kk:18s} {tot[kk]:6d}  {100 * tot[kk] / s:5.1f}%")


if __name__ == "__main__":
    main()
