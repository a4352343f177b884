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
    res = {"per_round_verify": {"fp_mul": tot_mul, "fp_sqr": tot_sqr, "stages": stages},
           "note": "executed algorithm of drand_amd/csrc (per-round mode), counted on one chained round"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "op_counts.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
