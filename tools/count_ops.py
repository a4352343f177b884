"""Count the Fp multiplications/squarings of one per-round verification as
executed by the kernels' code (host build with -DDG_COUNT_OPS) and write
profiles/op_counts.json -- the work figure behind bench.py's roofline.

    python tools/count_ops.py
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
FP_LIMBS = 14
MADS_MUL = 2 * FP_LIMBS * FP_LIMBS
MADS_SQR = FP_LIMBS * (FP_LIMBS + 1) // 2 + FP_LIMBS * FP_LIMBS


def main():
    so = os.path.join(ROOT, "tests", "hostsim", "libdrand_hostsim_count.so")
    subprocess.check_call(["hipcc", "-O1", "-std=c++17", "--cuda-host-only", "-DDG_COUNT_OPS", "-fPIC", "-shared",
                           "-o", so, os.path.join(ROOT, "tests", "hostsim", "hostsim.hip")])
    L = ctypes.CDLL(so)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "chain_chained_s1.json")))
    r = g["rounds"][1]
    prev = bytes.fromhex(r["prev"])
    out = (ctypes.c_ulonglong * 8)()
    rc = L.hs_count_stages(bytes.fromhex(g["pk"]), prev, len(prev), ctypes.c_uint64(r["round"]),
                           bytes.fromhex(r["sig"]), out)
    assert rc == 0, rc
    stages = {}
    for i, name in enumerate(["hash_to_g2", "decode_g2", "miller_loop", "final_exp"]):
        stages[name] = {"fp_mul": out[2 * i], "fp_sqr": out[2 * i + 1]}
    tot_mul = sum(v["fp_mul"] for v in stages.values())
    tot_sqr = sum(v["fp_sqr"] for v in stages.values())
    # the per-round pipeline's own kernels (hash split in three, decode with
    # membership left to the engine); v_mad_u64_u32 per call of fp.cuh's
    # FIPS forms: mul 14*14 product + 14*14 reduction, sqr 14*15/2 + 14*14
    kout = (ctypes.c_ulonglong * 8)()
    rc = L.hs_count_kernels(prev, len(prev), ctypes.c_uint64(r["round"]), bytes.fromhex(r["sig"]), kout)
    assert rc == 0, rc
    kernels = {}
    for i, name in enumerate(["k_h2c_field", "k_h2c_sswu", "k_h2c_finish", "k_decode_g2_sigs"]):
        mul, sqr = kout[2 * i], kout[2 * i + 1]
        kernels[name] = {"fp_mul": mul, "fp_sqr": sqr, "mads": MADS_MUL * mul + MADS_SQR * sqr}
    lo = (ctypes.c_ulonglong * 2)()
    assert L.hs_count_lines_thr(bytes.fromhex(r["sig"]), lo) == 0
    kernels["k_lines_thr"] = {"fp_mul": lo[0], "fp_sqr": lo[1], "mads": MADS_MUL * lo[0] + MADS_SQR * lo[1]}
    # the FE's five per-thread compressed chains (bench stage eng_fe_chain)
    assert L.hs_count_kb_chain_thr(lo) == 0
    kernels["k_kb_chain_thr"] = {"fp_mul": 5 * lo[0], "fp_sqr": 5 * lo[1],
                                 "mads": 5 * (MADS_MUL * lo[0] + MADS_SQR * lo[1])}
    h = [kernels[k] for k in ("k_h2c_field", "k_h2c_sswu", "k_h2c_finish")]
    # bench.py's stage "hash_to_g2" = the three hash kernels' launches summed
    kernels["hash_to_g2"] = {k: sum(x[k] for x in h) for k in ("fp_mul", "fp_sqr", "mads")}
    # RLC mode (configs[2]) and the on-G1 schemes (configs[3]): per-round work
    # of their stages (bench.py stage names), same host build of the device code
    import hashlib
    g1 = json.load(open(os.path.join(ROOT, "tests", "golden", "chain_on_g1_s1.json")))
    msg = hashlib.sha256(bytes.fromhex(r["prev"]) + r["round"].to_bytes(8, "big")).digest()
    xo = (ctypes.c_ulonglong * 22)()
    rc = L.hs_count_extra(msg, bytes.fromhex(r["sig"]), bytes.fromhex(g1["rounds"][0]["sig"]),
                          ctypes.c_uint64(0x9E3779B97F4A7C15), xo)
    assert rc == 0, rc
    part = {name: (xo[2 * i], xo[2 * i + 1]) for i, name in enumerate(
        ["rlc_hash", "decode_sub", "leaf", "node", "g2_affine", "hash_g1", "decode_g1", "g1_affine",
         "rlc_hash_g1", "leaf_g1", "node_g1"])}

    def ent(*terms):
        mul = sum(c * part[p][0] for c, p in terms)
        sqr = sum(c * part[p][1] for c, p in terms)
        return {"fp_mul": mul, "fp_sqr": sqr, "mads": MADS_MUL * mul + MADS_SQR * sqr}
    # per round: the raw hash (no cofactor); decode with membership; two
    # leaves (P and S trees) + the affine conversion of R + two tree nodes
    kernels["rlc_hash_to_g2_raw"] = ent((1, "rlc_hash"))
    kernels["k_decode_g2_sigs+subgroup"] = ent((1, "decode_sub"))
    kernels["rlc_leaves_tree"] = ent((2, "leaf"), (1, "g2_affine"), (2, "node"))
    kernels["k_hash_to_g1_beacons"] = ent((1, "hash_g1"))
    kernels["k_g1_batch_affine"] = ent((1, "g1_affine"))
    kernels["k_g2_batch_affine"] = ent((1, "g2_affine"))
    kernels["k_decode_g1_sigs"] = ent((1, "decode_g1"))
    # RLC for the G1-signature schemes: raw hash (no h_eff), two G1 leaves
    # (phi split) + the affine conversion of R + two tree nodes
    kernels["rlc_hash_to_g1_raw"] = ent((1, "rlc_hash_g1"))
    kernels["rlc_leaves_tree_g1"] = ent((2, "leaf_g1"), (1, "g1_affine"), (2, "node_g1"))
    # the localization tree of plain sums (rlc_resolve_locked): leaves are the
    # points themselves, about two node additions per round
    kernels["rlc_plain_tree"] = ent((2, "node"))
    kernels["rlc_plain_tree_g1"] = ent((2, "node_g1"))
    # group-law ops: the recovery MSM's work figure is composed from these
    go = (ctypes.c_ulonglong * 14)()
    assert L.hs_count_group_ops(msg, go) == 0
    res_ops = {}
    for i, name in enumerate(["g2_dbl", "g2_add", "g2_add_affine", "g1_dbl", "g1_add_affine", "g2_psi",
                              "g2_to_affine"]):
        mul, sqr = go[2 * i], go[2 * i + 1]
        res_ops[name] = {"fp_mul": mul, "fp_sqr": sqr, "mads": MADS_MUL * mul + MADS_SQR * sqr}
    # the bucket-MSM root: one mixed addition per point and (MSM, window) --
    # 8 per round (4 MSMs x 2 windows; bucket reduction and window sums are
    # per bucket, < 0.2 additions per round at 10M rounds)
    kernels["rlc_root_msm"] = {k: 8 * res_ops["g2_add_affine"][k] for k in ("fp_mul", "fp_sqr", "mads")}
    kernels["rlc_root_msm_g1"] = {k: 8 * res_ops["g1_add_affine"][k] for k in ("fp_mul", "fp_sqr", "mads")}
    res = {"per_round_verify": {"fp_mul": tot_mul, "fp_sqr": tot_sqr, "stages": stages},
           "kernels": kernels, "group_ops": res_ops,
           "unit": "per round; mads = v_mad_u64_u32 issued by the Fp multiplications (%d per mul, %d per sqr)"
                   % (MADS_MUL, MADS_SQR),
           "note": "executed algorithm of drand_amd/csrc, counted on one chained round by the host build of the "
                   "device code; per_round_verify = the per-thread reference composition (hash with its own "
                   "affine inversion, decode with the membership test), kernels = the per-round pipeline's "
                   "kernels (membership left to k_eng_lines, affine conversion batched in k_g2_batch_affine)"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "op_counts.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
