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
    ap.add_argument("--rounds", type=int, default=None,
                    help="rounds per GPU (default: 1M per-round/rlc as configs[1-2], 100k for recover)")
    ap.add_argument("--seg-len", type=int, default=64)
    ap.add_argument("--corrupt-rate", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["per-round", "rlc", "recover"], default="per-round",
                    help="per-round: configs[1]; rlc: configs[2] (random linear combination + bisection); "
                         "recover: configs[4] (t-of-n threshold recovery, n=32, t=17)")
    ap.add_argument("--t", type=int, default=17)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--bad-rate", type=float, default=0.1, help="recover: fraction of rounds with one invalid partial")
    ap.add_argument("--rlc-seed", type=int, default=3)
    ap.add_argument("--scheme", default="pedersen-bls-chained",
                    choices=["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1",
                             "bls-unchained-g1-rfc9380"],
                    help="per-round/rlc modes: the chain's scheme (configs[3]: unchained and on-g1)")
    return ap.parse_args()


def engine_work():
    """Exact per-item work of the pairing-engine kernels (tools/engine_work.py
    -> profiles/engine_work.json: product terms + reductions of the generated
    programs, x 196 v_mad_u64_u32 each)."""
    p = os.path.join(ROOT, "profiles", "engine_work.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)["kernels"]


def legacy_stage_ops():
    """Fp mul+sqr counts per round of the legacy stages, from
    profiles/op_counts.json (counted by the instrumented host build)."""
    p = os.path.join(ROOT, "profiles", "op_counts.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)["per_round_verify"]["stages"]
    return None


# stage name (dgpu_stage_times) -> kernel symbol / op_counts.json stages
STAGE_KERNEL = {"eng_lines": "k_eng_lines", "eng_miller": "k_eng_miller", "eng_inv": "k_eng_inv", "eng_fe": "k_eng_fe",
                "eng_lines_fixed": "k_eng_lines_fixed", "hash_to_g2": "k_hash_to_g2_beacons",
                "decode_g2": "k_decode_g2_sigs", "hash_to_g1": "k_hash_to_g1_beacons", "decode_g1": "k_decode_g1_sigs"}
STAGE_OPS = {"hash_to_g2": ["hash_to_g2"], "decode_g2": ["decode_g2"]}


def roofline_for(stage_ms, items):
    """Roofline of the dominant kernel (largest summed launch time; chunked
    stages are summed over their launches): achieved = algorithmic
    v_mad_u64_u32 products over the launches / measured time (HIP events on
    the launch stream) vs the measured int32 mad peak; traffic = PMC
    FETCH_SIZE+WRITE_SIZE bytes per item (profiles/*_traffic.json) x items.
    items = pairing checks per step (None when data-dependent, as in RLC)."""
    if not stage_ms:
        return None
    name = max(stage_ms, key=stage_ms.get)
    ms = stage_ms[name]
    kern = STAGE_KERNEL.get(name, name)
    out = {"bound": "valu-int32", "unit": "T mad_u64_u32/s", "kernel": kern, "launch_ms_total": ms,
           "items": items, "peak": PEAK_MAD_U64_PER_S / 1e12, "achieved": None, "frac": None, "traffic": None}
    if not items:
        return out
    work = engine_work()
    per_item = None
    if kern in work:
        per_item = work[kern]["mads"]
        out["work_source"] = "profiles/engine_work.json"
    elif name in STAGE_OPS and legacy_stage_ops():
        st = legacy_stage_ops()
        per_item = sum(st[s]["fp_mul"] + st[s]["fp_sqr"] for s in STAGE_OPS[name]) * PRODUCTS_PER_FP_MUL
        out["work_source"] = "profiles/op_counts.json"
    if per_item:
        achieved = items * per_item / (ms * 1e-3)
        out.update(achieved=achieved / 1e12, frac=achieved / PEAK_MAD_U64_PER_S, work_per_item_mads=per_item)
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        with open(path) as f:
            t = json.load(f)["kernels"]
        key = next((k for k in t if k.split("::")[-1] == kern), None)
        if key:
            per = t[key]
            out["traffic"] = items * (per["fetch_bytes_per_round"] + per["write_bytes_per_round"])
            out["traffic_unit"] = "bytes over the launches (PMC FETCH_SIZE+WRITE_SIZE, " + os.path.basename(path) + ")"
            break
    return out


def cpu_baseline(chain, seconds, cores, expect_valid):
    """Oracle timed on this host over a bounded sample of the same chain."""
    from oracle import cpu_baseline as cb
    return cb.run(chain, seconds, cores, expect_valid)


def timed(step, steps, world, dev):
    """barrier + synchronize, K steps, synchronize + barrier; max over ranks."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def stage_times(lib, ctx, step):
    """One profiled pass: HIP-event stage times summed per stage name."""
    import torch
    _lib_mod = sys.modules["drand_amd._lib"]
    _lib_mod.check(lib.dgpu_set_profiling(ctx.handle, 1))
    step()
    ms = (ctypes.c_float * 32)()
    names = (ctypes.c_char_p * 32)()
    ns = lib.dgpu_stage_times(ctx.handle, ms, 32, names)
    _lib_mod.check(lib.dgpu_set_profiling(ctx.handle, 0))
    torch.cuda.synchronize()
    return {names[i].decode(): float(ms[i]) for i in range(max(ns, 0))}


def main_recover(args, world, rank, local):
    """configs[4]: batch threshold recovery (kyber tbls.Recover as the
    aggregator calls it, chain/beacon/chain.go:158-168): per round t partials
    (one invalid in --bad-rate of the rounds), VerifyPartial of each on the
    pairing engine, selection + Lagrange + G2 MSM, VerifyRecovered.  Inputs
    resident in HBM (dgpu_recover_batch_device).  Shards: contiguous round
    ranges per rank (weak scaling); each rank checks its own outputs."""
    import torch
    import torch.distributed as dist
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import group_signatures, make_group, make_recovery_batch

    n = args.rounds or 100_000
    dev = torch.device("cuda", local)
    t_gen = time.time()
    grp = make_group(args.seed, args.t, args.n, device=local)
    msgs, parts, expect_ok = make_recovery_batch(grp, n, args.seed + 7919 * rank, args.bad_rate,
                                                 first_round=rank * n + 1, device=local)
    expect = group_signatures(grp, msgs, device=local)
    t_gen = time.time() - t_gen
    ctx = get_context(local)
    lib = ctx.lib
    cbuf = np.frombuffer(b"".join(grp.commits), dtype=np.uint8).copy()
    _lib.check(lib.dgpu_set_group(ctx.handle, grp.t, grp.n, _lib.ptr(cbuf)))
    m = parts.shape[1]
    d_msgs = torch.from_numpy(msgs).to(dev)
    d_parts = torch.from_numpy(parts.reshape(n * m, 98)).to(dev)
    d_plen = torch.full((n * m,), 98, dtype=torch.int32, device=dev)
    d_out = torch.zeros((n, 96), dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        _lib.check(lib.dgpu_recover_batch_device(ctx.handle, n, d_msgs.data_ptr(), m, d_parts.data_ptr(), 98,
                                                 d_plen.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(), None,
                                                 ctypes.c_void_p(stream.cuda_stream)))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    stage_ms = stage_times(lib, ctx, step)
    elapsed = timed(step, args.steps, world, dev)

    ok = d_ok.cpu().numpy().astype(bool)
    out = d_out.cpu().numpy()
    mism = int((ok != expect_ok).sum()) + int((out[ok & expect_ok] != expect[ok & expect_ok]).any(axis=1).sum())
    mism_t = torch.tensor([mism], device=dev)
    if world > 1:
        dist.all_reduce(mism_t)
    if rank == 0:
        items = n * m
        roof = roofline_for({k: v for k, v in stage_ms.items() if k.startswith("eng_")}, items + n)
        cpu = None
        if not args.no_cpu_baseline:
            try:
                from oracle import cpu_baseline as cb
                exp_sigs = [bytes(expect[i]) if expect_ok[i] else None for i in range(n)]
                cpu = cb.run_recover(grp.commits, grp.t, grp.n, msgs, parts, exp_sigs, args.cpu_seconds,
                                     min(16, os.cpu_count() or 1))
            except Exception as e:  # reported, never fatal
                cpu = {"error": repr(e)}
        print(json.dumps({
            "metric": "recovered beacon rounds/sec, t-of-n threshold recovery (VerifyPartial x t, Lagrange, "
                      "G2 MSM, VerifyRecovered)",
            "value": n * world * args.steps / elapsed, "unit": "rounds/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (14x28-bit limb Fp, 10x28-bit limb Fr, int32 VALU)",
            "data": f"synthetic {args.t}-of-{args.n} group and partials generated on GPU (seeded), "
                    f"{args.bad_rate:.0%} of rounds with one invalid partial",
            "config": {"workload": "configs[4]: threshold recovery, n=%d, t=%d" % (args.n, args.t),
                       "rounds_per_gpu": n, "partials_per_round": m, "pairings_per_round": m + 1,
                       "mode": "recover", "parallelism": f"shard{world}"},
            "stage_ms": stage_ms, "verdict_mismatches": int(mism_t.item()),
            "unrecoverable_rounds_per_gpu": int((~expect_ok).sum()), "gen_s": t_gen,
            "roofline": roof, "cpu_baseline": cpu}))


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
    if args.mode == "recover":
        main_recover(args, world, rank, local)
        if world > 1:
            dist.destroy_process_group()
        return

    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import corrupt, make_chain

    n = args.rounds or 1_000_000
    t_gen = time.time()
    code = _lib.scheme_from_name(args.scheme) if hasattr(_lib, "scheme_from_name") else {
        "pedersen-bls-chained": _lib.SCHEME_CHAINED, "pedersen-bls-unchained": _lib.SCHEME_UNCHAINED,
        "bls-unchained-on-g1": _lib.SCHEME_UNCHAINED_G1, "bls-unchained-g1-rfc9380": _lib.SCHEME_G1_RFC9380}[args.scheme]
    on_g1 = code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)
    chain = make_chain(args.seed, n, code, seg_len=args.seg_len, device=local,
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
    _lib.check(lib.dgpu_set_pubkey(ctx.handle, code, chain.pk, len(chain.pk)))
    stream = torch.cuda.current_stream(dev)
    mode = _lib.MODE_RLC if args.mode == "rlc" else _lib.MODE_PER_ROUND

    def step():
        _lib.check(lib.dgpu_verify_batch_device(
            ctx.handle, code, n, d_rounds.data_ptr(), d_sigs.data_ptr(), 96, d_sig_len.data_ptr(),
            d_prev.data_ptr(), 96, d_prev_len.data_ptr(), mode, args.rlc_seed, d_bits.data_ptr(), None,
            ctypes.c_void_p(stream.cuda_stream)))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # per-stage kernel timing (HIP events on the launch stream), one profiled
    # pass; the first (discarded) absorbs the single-lane buffer growth
    _lib.check(lib.dgpu_set_profiling(ctx.handle, 1))
    step()
    step()
    ms = (ctypes.c_float * 32)()
    names = (ctypes.c_char_p * 32)()
    ns = lib.dgpu_stage_times(ctx.handle, ms, 32, names)
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
        roofline = roofline_for(stage_ms, n if args.mode == "per-round" else None)
        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(chain, args.cpu_seconds, min(16, os.cpu_count() or 1), expect)
            except Exception as e:  # reported, never fatal
                cpu = {"error": repr(e)}
        out = {
            "metric": "verified beacon rounds/sec, chained BLS12-381 chain" if code == _lib.SCHEME_CHAINED
                      else f"verified beacon rounds/sec, {args.scheme} chain",
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
            "data": f"synthetic {args.scheme} chain generated on GPU (seeded), {args.corrupt_rate:.1%} corrupted",
            "config": {"workload": (f"configs[3]: {args.scheme} chain, per-round pairing verify" if code != _lib.SCHEME_CHAINED
                                    else "configs[1]: chained G2 chain, per-round pairing verify" if args.mode == "per-round"
                                    else "configs[2]: chained G2 chain, RLC batch verify + bisection, 0.1% corrupted"),
                       "rounds_per_gpu": n, "seg_len": args.seg_len, "scheme": args.scheme,
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
