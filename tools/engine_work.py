#!/usr/bin/env python3
"""Exact arithmetic work of the pairing engine's kernel programs, per item
(one two-pair pairing check), from the generated tables (tools/gen_engine.py):

  product terms  -- one 14 x 14-limb column product each (196 v_mad_u64_u32)
  reductions     -- one Montgomery reduction per output with a product part (196)

summed over the 12 lanes of a group (idle lanes and SIMT padding are not
counted: this is the algorithm's work, not the schedule's).  Writes
profiles/engine_work.json, which bench.py uses for roofline.achieved.

    python tools/engine_work.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_engine as G  # noqa: E402

MADS_PER_PRODUCT = 14 * 14


def program_work(ops, prog):
    by = {op.name: op for op in ops}
    terms = redc = outputs = sub_ops = simt_terms = 0
    for ins in prog:
        if ins[0] != "run":
            continue
        for sub in by[ins[1]].subs:
            sub_ops += 1
            nt = max([len(r.terms) for r in sub] + [0])
            simt_terms += nt + (1 if nt else 0)
            for r in sub:
                terms += len(r.terms)
                outputs += 1
                redc += 1 if r.terms else 0
    return {"product_terms": terms, "reductions": redc, "outputs": outputs, "sub_ops": sub_ops,
            "mads": (terms + redc) * MADS_PER_PRODUCT,
            "simt_lane_mads": 12 * simt_terms * MADS_PER_PRODUCT}


INV_MADS = 32 * 140 + 392  # one field inversion by divsteps (round 4; a^(p-2) was 82 mul + 380 sqr)


def main():
    ops = G.build_ops()
    kern = {
        "k_eng_lines": program_work(ops, G.prog_lines()),
        "k_eng_miller": program_work(ops, G.prog_miller()),
        "k_eng_fe": program_work(ops, G.prog_fe()),
        # Montgomery's trick: 3 Fp multiplications per item (392 mads each), one
        # inversion per 64 items amortized (fp.cuh fp_inv: 32 divstep batches of
        # 140 signed 32x32->64 mads, 4,480, plus one multiplication by R^3)
        "k_eng_inv": {"mads": 3 * 392 + INV_MADS // 64},
    }
    # Karabina FE: the 12-lane program segments, the 8-lane
    # compressed chains (63 squarings of the E_CYC records for f1, f2, f4, f5,
    # five exponentiations), and the per-thread decompression side: norms of
    # the six stored values (k_eng_kb_norm: 2 sqr each, 5 mul), their product's
    # inversion (k_eng_inv: 3 mul + an inversion, INV_MADS, per
    # KB_INV_CHAIN items), the per-value inverses and eng_kb_decompress
    # (k_eng_kb_dec: 12 sqr + 5 mul forward, 2 mul + 2 sqr per value after the
    # first backward, 17 mul per decompression)
    segs = G.prog_fe_kb()
    seg_work = program_work(ops, [ins for sg in segs for ins in sg])
    cyc = {o.name: o for o in ops}["E_CYC"].subs[1]
    comp = {G.E_R + c for c in G.KB_COMP}
    sq_terms = sum(len(r.terms) for r in cyc if r.dst in comp)
    sq_redc = sum(1 for r in cyc if r.dst in comp and r.terms)
    n_exp, n_sq = 5, 63
    chain = {"squarings": n_exp * n_sq, "product_terms": n_exp * n_sq * sq_terms,
             "reductions": n_exp * n_sq * sq_redc, "mads": n_exp * n_sq * (sq_terms + sq_redc) * MADS_PER_PRODUCT}
    MUL, SQR = 392, 301
    KB_INV_CHAIN = 16
    ns = len(G.KB_SNAP)
    norm = 2 * ns * SQR + (ns - 1) * MUL
    inv = 3 * MUL + INV_MADS // KB_INV_CHAIN
    dec = 2 * ns * SQR + (ns - 1) * MUL + (ns - 1) * (2 * MUL + 2 * SQR) + ns * 17 * MUL
    kern["k_eng_fe_seg"] = seg_work
    kern["k_eng_kb_chain"] = chain
    kern["k_eng_kb_inv"] = {"mads": n_exp * (norm + inv + dec), "per_exponentiation": {
        "k_eng_kb_norm": norm, "k_eng_inv": inv, "k_eng_kb_dec": dec}}
    kern["k_eng_fe_karabina"] = {"mads": seg_work["mads"] + chain["mads"] + kern["k_eng_kb_inv"]["mads"]}
    # on-G1 schemes: the Miller program with every line formed at its LDLINE
    # from the key's fixed table, 8 of the 12 exports scaled by one Fp
    # multiplication (a P coordinate): 68 line steps x 8 x 392 mads more
    n_ld = sum(1 for ins in G.prog_miller() if ins[0] == "ldline")
    fixed = dict(kern["k_eng_miller"])
    fixed["line_scalings"] = n_ld * 8
    fixed["mads"] = kern["k_eng_miller"]["mads"] + n_ld * 8 * 392
    kern["k_eng_miller_fixed"] = fixed
    out = {
        "unit": "per item (one two-pair pairing check); mads = 32x32->64 v_mad_u64_u32 products the algorithm performs",
        "kernels": kern,
        "pairing_total_mads": sum(kern[k]["mads"] for k in ("k_eng_lines", "k_eng_miller", "k_eng_inv",
                                                             "k_eng_fe_karabina")),
        "pairing_total_mads_granger_scott_fe": sum(kern[k]["mads"] for k in ("k_eng_lines", "k_eng_miller",
                                                                              "k_eng_inv", "k_eng_fe")),
    }
    path = os.path.join(os.path.dirname(HERE), "profiles", "engine_work.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
