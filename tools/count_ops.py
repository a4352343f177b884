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
    h = [kernels[k] for k in ("k_h2c_field", "k_h2c_sswu", "k_h2c_finish")]
    # bench.py's stage "hash_to_g2" = the three hash kernels' launches summed
    kernels["hash_to_g2"] = {k: sum(x[k] for x in h) for k in ("fp_mul", "fp_sqr", "mads")}
    res = {"per_round_verify": {"fp_mul": tot_mul, "fp_sqr": tot_sqr, "stages": stages},
           "kernels": kernels,
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
