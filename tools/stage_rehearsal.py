#!/usr/bin/env python3
"""Rehearse the 8-GPU host side of dgpu_verify_multi on one GPU (VERDICT r05
item 4): eight contexts of device 0 (DGPU_MULTI_ALLOW_SAME_DEVICE=1), each
staging its 1.25M-round shard of a 10M-round chained chain through its own
pinned ring, all at once from one process -- the host memcpy into the rings
contends exactly as on an 8-GPU node.  The A/B build's DGPU_TEST_STAGE_ONLY=1
stops each shard after its staging, so the timing holds nothing else.  Per
device: the staging thread's host wall time and the copy-stream span (on one
GPU the eight copy streams also share one PCIe link, which 8 GPUs do not).

    DRAND_GPU_LIB=$PWD/drand_amd/libdrand_gpu_ab.so DGPU_MULTI_ALLOW_SAME_DEVICE=1 \\
        DGPU_TEST_STAGE_ONLY=1 python tools/stage_rehearsal.py [--rounds N] [--devices 8]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(mctx, k):
    from drand_amd import _lib
    h = ctypes.c_void_p()
    _lib.check(mctx.lib.dgpu_multi_context(mctx.handle, k, ctypes.byref(h)), mctx.lib)
    ms, hms, nb = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
    _lib.check(mctx.lib.dgpu_staging_stats(h, ctypes.byref(ms), ctypes.byref(hms), ctypes.byref(nb)), mctx.lib)
    return {"device_ms": round(ms.value, 2), "host_ms": round(hms.value, 2), "bytes": nb.value}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10_000_000)
    ap.add_argument("--devices", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    assert os.environ.get("DGPU_TEST_STAGE_ONLY") == "1" and os.environ.get("DGPU_MULTI_ALLOW_SAME_DEVICE") == "1"
    from drand_amd import _lib
    from drand_amd.multi import MultiVerifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.synth import make_chain
    chain = make_chain(2, args.rounds, _lib.SCHEME_CHAINED, seg_len=64)
    out = {}
    for ndev in (1, args.devices):
        mctx = _lib.MultiContext([0] * ndev)
        mv = MultiVerifier(get_scheme_by_id_with_default("pedersen-bls-chained"), mctx=mctx)
        n = args.rounds // args.devices * ndev  # 1.25M rounds per shard in both cases
        reps = []
        for _ in range(args.reps + 1):  # the first call grows the buffers
            t0 = time.perf_counter()
            mv.verify_records(chain.pk, chain.rounds[:n], chain.sigs[:n], chain.sig_len[:n], chain.prev[:n],
                              chain.prev_len[:n], _lib.MODE_PER_ROUND, 0)
            wall = time.perf_counter() - t0
            reps.append({"call_wall_ms": round(wall * 1e3, 2), "per_device": [stats(mctx, k) for k in range(ndev)]})
        mctx.close()
        last = reps[1:]
        out[f"{ndev}_contexts"] = {
            "rounds_per_shard": n // ndev, "bytes_per_shard": last[-1]["per_device"][0]["bytes"],
            "max_host_ms": max(max(d["host_ms"] for d in r["per_device"]) for r in last),
            "max_device_ms": max(max(d["device_ms"] for d in r["per_device"]) for r in last),
            "reps": last}
    out["note"] = ("host_ms: each shard's staging thread, first memcpy into its pinned ring to its last DMA enqueued "
                   "(the host-side cost 8 GPUs share); device_ms: its copy-stream span (one GPU: the 8 copy streams "
                   "share one PCIe link, unlike 8 GPUs)")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
