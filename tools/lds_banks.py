#!/usr/bin/env python3
"""LDS bank-conflict model of the pairing engine's operand loads.

Every operand (and post) slot read of a sub-op is 7 ds_read_b64 per lane
(engine.cuh eng_ld).  For ds_read_b64 a wave64 access is served in two
32-lane halves, bank = (byte address / 4) mod 64, each lane touching an even
bank pair; within a half, each extra distinct address on a bank costs one
LDS cycle (MI355X_MICROARCH.md, LDS).  Lane L of the wave is lane k = L % 12
of group g = L // 12 (lanes 60..63 repeat group 4's lanes 0..3); group g's
slot s sits at word (NCONST + g * S + s) * 14, constant slot c >= 64 at word
(c - 64) * 14.  This script counts, for each kernel program, the LDS cycles
of its operand loads for a group stride S (slots per group), so the stride
can be padded where that removes conflicts without costing occupancy.

    python3 tools/lds_banks.py            # table for every kernel, S range
"""
import os
import sys
from collections import Counter, defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_engine as ge  # noqa: E402

SW = ge.SLOT_WORDS


def lane_map():
    out = []
    for L in range(64):
        out.append((L // 12, L % 12) if L < 60 else (4, L - 60))
    return out


LANES = lane_map()


def word(g, s, S):
    """S: the group stride (group g at NCONST + g S), or a list of the five
    group bases (slots from the start of LDS)."""
    if s >= 64:
        return (s - 64) * SW
    base = S[g] if isinstance(S, (list, tuple)) else ge.N_CONST + g * S
    return (base + s) * SW


def cycles_b64(slot_of_k, S):
    """LDS cycles of the 7 ds_read_b64 that load, on every lane k with
    slot_of_k[k] not None, the slot slot_of_k[k] of its group."""
    tot = 0
    for i in range(SW // 2):
        for half in (range(0, 32), range(32, 64)):
            banks = defaultdict(set)
            for L in half:
                g, k = LANES[L]
                s = slot_of_k[k] if k < len(slot_of_k) else None
                if s is None:
                    continue
                a = word(g, s, S) + 2 * i
                banks[(a // 2) % 32].add(a)
            tot += max([len(v) for v in banks.values()] + [1])
    return tot


def sub_loads(sub):
    """Per-lane slot lists in load order: per term t (a then b), then posts."""
    lanes = [sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2)) for r in sub] + [[]] * (ge.LANES - len(sub))
    posts = [list(r.post) for r in sub] + [[]] * (ge.LANES - len(sub))
    nt = max(len(t) for t in lanes)
    npst = max(len(p) for p in posts)
    loads = []
    for t in range(nt):
        for which in (0, 1):
            loads.append([ts[t][which] if t < len(ts) else None for ts in lanes])
    for u in range(npst):
        loads.append([p[u][0] if u < len(p) else None for p in posts])
    return loads


def op_cycles(op, S, cache={}):
    key = (op.name, tuple(S) if isinstance(S, list) else S)
    if key not in cache:
        c = 0
        for sub in op.subs:
            for ld in sub_loads(sub):
                c += cycles_b64(ld, S)
        cache[key] = c
    return cache[key]


def min_cycles(op):
    """Conflict-free cost: 2 cycles per ds_read_b64."""
    return sum(len(sub_loads(sub)) * (SW // 2) * 2 for sub in op.subs)


def program_ops(prog):
    return Counter(ins[1] for ins in prog if ins[0] == "run")


def search_bases(ops, cnt, used, max_slots, rounds=3):
    """Group bases NCONST + g used + c_g with 0 = c_0 <= c_1 <= ... <= c_4 and
    the wave's LDS within max_slots, by coordinate descent on the gaps
    (conflicts depend on the bases mod 32 only, so gaps < 32)."""
    spare = max_slots - ge.N_CONST - 5 * used

    def cost(gaps):
        cs = [0]
        for x in gaps:
            cs.append(cs[-1] + x)
        bases = [ge.N_CONST + g * used + cs[g] for g in range(5)]
        return sum(n * op_cycles(ops[o], bases) for o, n in cnt.items()), bases

    gaps = [0, 0, 0, 0]
    best = cost(gaps)
    for _ in range(rounds):
        for j in range(4):
            for x in range(min(31, spare) + 1):
                trial = gaps[:j] + [x] + gaps[j + 1:]
                if sum(trial) > spare:
                    break
                c = cost(trial)
                if c[0] < best[0]:
                    best, gaps = c, trial
    return best


def main():
    ops = {o.name: o for o in ge.build_ops()}
    progs = {"lines": (ge.prog_lines(), ge.LINE_PAIR_SLOTS * 2 + 2),
             "miller": (ge.prog_miller(), None), "fe": (ge.prog_fe(), None)}
    tabs = {}
    for name, (prog, _) in progs.items():
        cnt = program_ops(prog)
        used = max(max([s for sub in ops[o].subs for r in sub
                        for s in [r.dst] + [t[0] for t in r.terms] + [t[1] for t in r.terms] + [p[0] for p in r.post]
                        if s is not None and s < 64] + [0]) + 1 for o in cnt)
        rows = []
        for S in range(used, used + 12):
            c = sum(n * op_cycles(ops[o], S) for o, n in cnt.items())
            rows.append((S, c))
        ideal = sum(n * min_cycles(ops[o]) for o, n in cnt.items())
        tabs[name] = (used, ideal, rows)
        print(f"{name}: slots used {used}, conflict-free {ideal} cycles/wave")
        for S, c in rows:
            lds = (ge.N_CONST + 5 * S) * SW * 4
            print(f"   S={S:3d}  cycles {c:9d}  x{c / ideal:5.3f}  LDS/wave {lds} B  waves/CU {163840 // lds}")
    return tabs


if __name__ == "__main__":
    main()
