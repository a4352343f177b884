#!/usr/bin/env python3
"""Benchmark: verified drand beacon rounds/s on MI355X (BASELINE.json metric).

One step = one pass of the verify hot path (DigestMessage -> hash-to-G2 ->
signature decode + subgroup check -> pairing check -> verdict bitmap) over this
rank's whole shard of a synthetic chained BLS12-381 chain, with every input
already resident in HBM.  Shards are contiguous round ranges (weak scaling:
each rank verifies --rounds rounds); after the timed loop rank 0 gathers the
per-rank verdict bitmaps over RCCL and checks them against construction.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rounds R]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# measured on MI355X: profiles/r01_microbench_intmul.txt (v_mad_u64_u32, 32x32->64 products/s)
PEAK_MAD_U64_PER_S = 33.48e12
# W = (Fp mul + Fp sqr) count x 288 (12x12 limb products x 2)
PRODUCTS_PER_FP_MUL = 288


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=1_000_000, help="rounds per GPU (configs[1]: 1M)")
    ap.add_argument("--seg-len", type=int, default=64)
    ap.add_argument("--corrupt-rate", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["per-round", "rlc"], default="per-round",
                    help="per-round: configs[1]; rlc: configs[2] (random linear combination + bisection)")
    ap.add_argument("--rlc-seed", type=int, default=3)
    return ap.parse_args()


def fp_ops_per_round():
    """Fp mul+sqr count per round of the executed per-round algorithm, from
    profiles/op_counts.json (counted by the instrumented host build)."""
    p = os.path.join(ROOT, "profiles", "op_counts.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        return d["per_round_verify"]["fp_mul"] + d["per_round_verify"]["fp_sqr"], d
    return None, None


# stage name (dgpu_stage_times) -> op_counts.json stages it executes
STAGE_OPS = {"hash_to_g2": ["hash_to_g2"], "decode_g2": ["decode_g2"], "pairing_check": ["miller_loop", "final_exp"]}


def roofline_for(stage_ms, n, mode):
    """Roofline of the dominant kernel: achieved = algorithmic 32x32 products
    per launch (Fp mul+sqr count x 288) / measured launch time
    (HIP events on the launch stream); traffic = PMC FETCH+WRITE bytes per
    round (profiles/*_traffic.json) x rounds per launch."""
    if not stage_ms:
        return None
    name = max(stage_ms, key=stage_ms.get)
    ms = stage_ms[name]
    ops, counts = fp_ops_per_round()
    out = {"bound": "valu-int32", "unit": "T mad_u64_u32/s", "kernel": name, "launch_ms": ms,
           "peak": PEAK_MAD_U64_PER_S / 1e12, "achieved": None, "frac": None, "traffic": None,
           "stage_ms": stage_ms}
    if counts and mode == "per-round" and name in STAGE_OPS:
        st = counts["per_round_verify"]["stages"]
        k_ops = sum(st[s]["fp_mul"] + st[s]["fp_sqr"] for s in STAGE_OPS[name])
        achieved = n * k_ops * PRODUCTS_PER_FP_MUL / (ms * 1e-3)
        out.update(achieved=achieved / 1e12, frac=achieved / PEAK_MAD_U64_PER_S,
                   work_per_round_products=k_ops * PRODUCTS_PER_FP_MUL,
                   pipeline_products_per_round=ops * PRODUCTS_PER_FP_MUL)
    import glob
    tr = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    if tr:
        with open(tr[-1]) as f:
            t = json.load(f)["kernels"]
        kname = {"hash_to_g2": "dgpu::k_hash_to_g2_beacons", "decode_g2": "dgpu::k_decode_g2_sigs",
                 "pairing_check": "dgpu::k_pairing_check"}.get(name)
        if kname in t:
            out["traffic"] = n * (t[kname]["fetch_bytes_per_round"] + t[kname]["write_bytes_per_round"])
            out["traffic_unit"] = "bytes per launch (PMC FETCH_SIZE+WRITE_SIZE, " + os.path.basename(tr[-1]) + ")"
    return out


def cpu_baseline(chain, seconds, cores, expect_valid):
    """Oracle timed on this host over a bounded sample of the same chain."""
    from oracle import cpu_baseline as cb
    return cb.run(chain, seconds, cores, expect_valid)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import corrupt, make_chain

    n = args.rounds
    t_gen = time.time()
    chain = make_chain(args.seed, n, _lib.SCHEME_CHAINED, seg_len=args.seg_len, device=local,
                       start_round=rank * n + 1)
    bad = corrupt(chain, args.seed + rank, rate=args.corrupt_rate)
    t_gen = time.time() - t_gen

    dev = torch.device("cuda", local)
    d_rounds = torch.from_numpy(chain.rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(chain.sigs).to(dev)
    d_sig_len = torch.from_numpy(chain.sig_len.view(np.int32)).to(dev)
    d_prev = torch.from_numpy(chain.prev).to(dev)
    d_prev_len = torch.from_numpy(chain.prev_len.view(np.int32)).to(dev)
    d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
    ctx = get_context(local)
    lib = ctx.lib
    _lib.check(lib.dgpu_set_pubkey(ctx.handle, _lib.SCHEME_CHAINED, chain.pk, 48))
    stream = torch.cuda.current_stream(dev)
    mode = _lib.MODE_RLC if args.mode == "rlc" else _lib.MODE_PER_ROUND

    def step():
        _lib.check(lib.dgpu_verify_batch_device(
            ctx.handle, _lib.SCHEME_CHAINED, n, d_rounds.data_ptr(), d_sigs.data_ptr(), 96, d_sig_len.data_ptr(),
            d_prev.data_ptr(), 96, d_prev_len.data_ptr(), mode, args.rlc_seed, d_bits.data_ptr(), None,
            ctypes.c_void_p(stream.cuda_stream)))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # per-stage kernel timing (HIP events on the launch stream), one profiled pass
    _lib.check(lib.dgpu_set_profiling(ctx.handle, 1))
    step()
    ms = (ctypes.c_float * 8)()
    names = (ctypes.c_char_p * 8)()
    ns = lib.dgpu_stage_times(ctx.handle, ms, 8, names)
    stage_ms = {names[i].decode(): float(ms[i]) for i in range(max(ns, 0))}
    _lib.check(lib.dgpu_set_profiling(ctx.handle, 0))
    torch.cuda.synchronize()

    from drand_amd.dist import gather_verdict_bits

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    # the one exchange step: every rank's verdict bitmap to every rank (RCCL)
    verdicts = gather_verdict_bits(d_bits, n, n * world, world, rank)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # verdicts vs construction (each rank knows its own corrupted rounds)
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    mine = verdicts[rank * n:(rank + 1) * n] if world > 1 else verdicts
    mism_local = torch.tensor([int((mine != expect).sum())], device=dev)
    if world > 1:
        dist.all_reduce(mism_local)
    mismatches = int(mism_local.item())

    if rank == 0:
        total_rounds = n * world * args.steps
        value = total_rounds / elapsed
        roofline = roofline_for(stage_ms, n, args.mode)
        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(chain, args.cpu_seconds, min(16, os.cpu_count() or 1), expect)
            except Exception as e:  # reported, never fatal
                cpu = {"error": repr(e)}
        out = {
            "metric": "verified beacon rounds/sec, chained BLS12-381 chain",
            "value": value,
            "unit": "rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (14x28-bit limb Fp, int32 VALU)",
            "data": "synthetic chained chain generated on GPU (seeded), 0.1% corrupted",
            "config": {"workload": ("configs[1]: chained G2 chain, per-round pairing verify" if args.mode == "per-round"
                                    else "configs[2]: chained G2 chain, RLC batch verify + bisection, 0.1% corrupted"),
                       "rounds_per_gpu": n, "seg_len": args.seg_len, "scheme": "pedersen-bls-chained",
                       "mode": args.mode, "parallelism": f"shard{world}"},
            "stage_ms": stage_ms,
            "verdict_mismatches": mismatches,
            "corrupted_rounds_per_gpu": len(bad),
            "chain_gen_s": t_gen,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
