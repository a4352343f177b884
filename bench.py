#!/usr/bin/env python3
"""Benchmark: verified drand beacon rounds/s on MI355X (BASELINE.json metric:
"verified beacon rounds/sec, 10M-round chained BLS12-381 chain, 1/2/4/8 MI355X").

One step = one pass of the verify hot path (DigestMessage -> hash-to-G2 ->
signature decode + subgroup check -> pairing check -> verdict bitmap) over
the WHOLE 10M-round chain, with every input already resident in HBM.  With N
GPUs the same chain is split into N contiguous round shards (strong scaling,
the bulk check-chain loop chain/beacon/sync_manager.go:188-222 sharded as
SURVEY.md 8(e)); each rank verifies its shard, and the per-rank verdict
bitmaps are all-gathered over RCCL (the one exchange step) inside the timed
region, then checked against the construction.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rounds R]

With --gpus N > 1 and no torch.distributed environment, bench.py starts the
N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before
anything touches the GPU; under torch.distributed.run it is one rank.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# measured on MI355X: profiles/r01_microbench_intmul.txt (v_mad_u64_u32, 32x32->64 products/s)
PEAK_MAD_U64_PER_S = 33.48e12


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=None,
                    help="rounds in the whole chain, split over the GPUs (default: 10M as BASELINE.json's metric; "
                         "100k for recover)")
    ap.add_argument("--seg-len", type=int, default=64)
    ap.add_argument("--corrupt-rate", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (H2D-inclusive) pass")
    ap.add_argument("--no-rlc", action="store_true",
                    help="per-round mode: skip the RLC batch-verify pass over the same resident chain (configs[2])")
    ap.add_argument("--mode", choices=["per-round", "rlc", "recover"], default="per-round",
                    help="per-round: configs[1] / the metric; rlc: configs[2] (random linear combination + "
                         "bisection); recover: configs[4] (t-of-n threshold recovery, n=32, t=17)")
    ap.add_argument("--t", type=int, default=17)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--bad-rate", type=float, default=0.1, help="recover: fraction of rounds with one invalid partial")
    ap.add_argument("--rlc-seed", type=int, default=3)
    ap.add_argument("--scheme", default="pedersen-bls-chained",
                    choices=["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1",
                             "bls-unchained-g1-rfc9380"],
                    help="per-round/rlc modes: the chain's scheme (configs[3]: unchained and on-g1)")
    return ap.parse_args(argv)


def log(*a):
    """Progress on stderr (rank-tagged): long GPU runs stay visibly alive."""
    print(f"[bench rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def launch_ranks(args):
    """--gpus N without a torch.distributed environment: start N rank
    processes (this process never touches the GPU) and exit with the worst
    status.  Rank 0 prints the JSON line."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def engine_work():
    """Exact per-item work of the pairing-engine kernels (tools/engine_work.py
    -> profiles/engine_work.json: product terms + reductions of the generated
    programs, x 196 v_mad_u64_u32 each)."""
    p = os.path.join(ROOT, "profiles", "engine_work.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)["kernels"]


def hash_work():
    """Per-round v_mad_u64_u32 counts of the hash / decode kernels of the
    chained per-round pipeline (tools/count_ops.py -> profiles/op_counts.json,
    counted by the host build of the same device functions)."""
    p = os.path.join(ROOT, "profiles", "op_counts.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f).get("kernels", {})


# stage name (dgpu_stage_times) -> kernel symbol
STAGE_KERNEL = {"eng_lines": "k_eng_lines", "eng_miller": "k_eng_miller", "eng_inv": "k_eng_inv", "eng_fe": "k_eng_fe",
                "eng_lines_fixed": "k_eng_lines_fixed", "hash_to_g2": "hash_to_g2", "decode_g2": "k_decode_g2_sigs",
                "hash_to_g1": "k_hash_to_g1_beacons", "decode_g1": "k_decode_g1_sigs"}


def traffic_for(kern, items):
    """PMC FETCH_SIZE + WRITE_SIZE per item of this build (profiles/r02*_traffic.json)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "r02*_traffic.json"), recursive=True), reverse=True):
        with open(path) as f:
            t = json.load(f)["kernels"]
        key = next((k for k in t if k.split("::")[-1].split("(")[0] == kern), None)
        if key:
            per = t[key]
            return items * (per["fetch_bytes_per_round"] + per["write_bytes_per_round"]), os.path.basename(path)
    return None, None


def roofline_for(stage_ms, items):
    """Roofline of the dominant kernel (largest summed launch time; chunked
    stages are summed over their launches): achieved = algorithmic
    v_mad_u64_u32 products over the launches / measured time (HIP events on
    the launch stream) vs the measured int32 mad peak; traffic = PMC bytes of
    this build over the same launches.  items = pairing checks per pass
    (None when data-dependent, as in RLC)."""
    if not stage_ms:
        return None
    name = max(stage_ms, key=stage_ms.get)
    ms = stage_ms[name]
    kern = STAGE_KERNEL.get(name, name)
    out = {"bound": "valu-int32", "unit": "T mad_u64_u32/s", "kernel": kern, "launch_ms_total": ms,
           "items": items, "peak": PEAK_MAD_U64_PER_S / 1e12, "achieved": None, "frac": None, "traffic": None}
    if not items:
        return out
    work = dict(hash_work(), **engine_work())
    if kern in work:
        per_item = work[kern]["mads"]
        achieved = items * per_item / (ms * 1e-3)
        out.update(achieved=achieved / 1e12, frac=achieved / PEAK_MAD_U64_PER_S, work_per_item_mads=per_item,
                   work_source="profiles/engine_work.json" if kern in engine_work() else "profiles/op_counts.json")
    # the same fraction for every stage that has a work figure (hash and decode
    # from profiles/op_counts.json, the engine from profiles/engine_work.json)
    out["stage_frac"] = {s: items * work[STAGE_KERNEL.get(s, s)]["mads"] / (t * 1e-3) / PEAK_MAD_U64_PER_S
                         for s, t in stage_ms.items() if STAGE_KERNEL.get(s, s) in work and t > 0}
    traffic, src = traffic_for(kern, items)
    if traffic is not None:
        out["traffic"] = traffic
        out["traffic_unit"] = "bytes over the launches (PMC FETCH_SIZE+WRITE_SIZE, %s)" % src
    return out


def stage_times(lib, ctx, step, passes=1):
    """Profiled passes (the last one counts): HIP-event stage times summed per stage name."""
    import torch
    from drand_amd import _lib
    _lib.check(lib.dgpu_set_profiling(ctx.handle, 1))
    for _ in range(passes):
        step()
    ms = (ctypes.c_float * 32)()
    names = (ctypes.c_char_p * 32)()
    ns = lib.dgpu_stage_times(ctx.handle, ms, 32, names)
    _lib.check(lib.dgpu_set_profiling(ctx.handle, 0))
    torch.cuda.synchronize()
    return {names[i].decode(): float(ms[i]) for i in range(max(ns, 0))}


def timed(step, steps, world, dev, after=None):
    """barrier + synchronize, K steps (+ `after`, the exchange step),
    synchronize + barrier; max over ranks."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    res = after() if after else None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), res


def shard_chain(args, code, n_total, lo, hi, device):
    """This rank's rounds [lo + 1, hi] of the global chain: whole seg_len
    segments are generated (segment s covers rounds s*seg_len + 1 ..; its seed
    depends only on s), so every rank sees the same chain whatever N is."""
    from drand_amd.synth import make_chain
    seg = args.seg_len
    s0 = lo // seg
    s1 = (hi + seg - 1) // seg
    ch = make_chain(args.seed, (s1 - s0) * seg, code, seg_len=seg, device=device, start_round=s0 * seg + 1)
    a, b = lo - s0 * seg, hi - s0 * seg
    for name in ("rounds", "sigs", "sig_len", "prev", "prev_len"):
        setattr(ch, name, np.ascontiguousarray(getattr(ch, name)[a:b]))
    return ch


def main_recover(args, world, rank, local):
    """configs[4]: batch threshold recovery (kyber tbls.Recover as the
    aggregator calls it, chain/beacon/chain.go:158-168): per round t partials
    (one invalid in --bad-rate of the rounds), VerifyPartial of each on the
    pairing engine, selection + Lagrange + G2 MSM, VerifyRecovered.  Inputs
    resident in HBM (dgpu_recover_batch_device).  The --rounds batch is split
    into contiguous round shards (strong scaling); each rank checks its own
    outputs."""
    import torch
    import torch.distributed as dist
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.dist import shard_range
    from drand_amd.synth import group_signatures, make_group, make_recovery_batch

    n_total = args.rounds or 100_000
    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    dev = torch.device("cuda", local)
    t_gen = time.time()
    grp = make_group(args.seed, args.t, args.n, device=local)
    msgs, parts, expect_ok = make_recovery_batch(grp, n, args.seed + 7919 * rank, args.bad_rate,
                                                 first_round=lo + 1, device=local)
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
    elapsed, _ = timed(step, args.steps, world, dev)

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
        if not args.no_cpu_baseline and world == 1:
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
            "value": n_total * args.steps / elapsed, "unit": "rounds/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32 (14x28-bit limb Fp, 10x28-bit limb Fr, int32 VALU)",
            "data": f"synthetic {args.t}-of-{args.n} group and partials generated on GPU (seeded), "
                    f"{args.bad_rate:.0%} of rounds with one invalid partial",
            "config": {"workload": "configs[4]: threshold recovery, n=%d, t=%d" % (args.n, args.t),
                       "rounds_total": n_total, "rounds_per_gpu": n, "partials_per_round": m,
                       "pairings_per_round": m + 1, "mode": "recover", "parallelism": f"shard{world}"},
            "stage_ms": stage_ms, "verdict_mismatches": int(mism_t.item()),
            "unrecoverable_rounds_rank0": int((~expect_ok).sum()), "gen_s": t_gen,
            "roofline": roof, "cpu_baseline": cpu}))


def main_verify(args, world, rank, local):
    import torch
    import torch.distributed as dist
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.dist import gather_verdict_bits, shard_range
    from drand_amd.synth import corrupt_global

    n_total = args.rounds or 10_000_000
    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    code = _lib.load().dgpu_scheme_from_name(args.scheme.encode())
    t_gen = time.time()
    log(f"generating rounds [{lo + 1}, {hi}] of a {n_total}-round {args.scheme} chain")
    chain = shard_chain(args, code, n_total, lo, hi, local)
    bad = corrupt_global(chain, args.seed, n_total, lo, rate=args.corrupt_rate)
    t_gen = time.time() - t_gen
    log(f"chain ready in {t_gen:.1f} s")

    dev = torch.device("cuda", local)
    d_rounds = torch.from_numpy(chain.rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(chain.sigs).to(dev)
    d_sig_len = torch.from_numpy(chain.sig_len.view(np.int32)).to(dev)
    d_prev = torch.from_numpy(chain.prev).to(dev)
    d_prev_len = torch.from_numpy(chain.prev_len.view(np.int32)).to(dev)
    d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
    ctx = get_context(local)
    lib = ctx.lib
    pk = np.frombuffer(chain.pk, dtype=np.uint8).copy()
    stream = torch.cuda.current_stream(dev)
    mode = _lib.MODE_RLC if args.mode == "rlc" else _lib.MODE_PER_ROUND
    seed = args.rlc_seed + 7 * rank

    def step():
        _lib.check(lib.dgpu_verify_beacons_device(
            ctx.handle, code, _lib.ptr(pk), pk.size, n, d_rounds.data_ptr(), d_sigs.data_ptr(), 96,
            d_sig_len.data_ptr(), d_prev.data_ptr(), 96, d_prev_len.data_ptr(), mode, seed, d_bits.data_ptr(),
            None, ctypes.c_void_p(stream.cuda_stream)))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    log("warmup done")
    # per-stage kernel timing (HIP events on the launch stream), single lane;
    # the first of the two passes absorbs the single-lane buffer growth
    stage_ms = stage_times(lib, ctx, step, passes=2)
    log("stage times", json.dumps(stage_ms))

    # the exchange step: every rank's verdict bitmap to every rank (RCCL)
    elapsed, verdicts = timed(step, args.steps, world, dev,
                              after=lambda: gather_verdict_bits(d_bits, n, n_total, world, rank))

    log(f"timed: {args.steps} steps in {elapsed:.3f} s")
    # verdicts vs construction (the corruption catalog is global, seeded)
    expect = np.ones(n_total, dtype=bool)
    expect[list(bad.keys())] = False
    mism = int((verdicts != expect).sum())

    # end to end: host records through dgpu_verify_beacons (H2D + D2H inside)
    e2e = None
    if not args.no_e2e:
        h_bits = np.zeros((n + 7) // 8, dtype=np.uint8)

        def step_host():
            _lib.check(lib.dgpu_verify_beacons(
                ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(chain.rounds), _lib.ptr(chain.sigs), 96,
                _lib.ptr(chain.sig_len), _lib.ptr(chain.prev), 96, _lib.ptr(chain.prev_len), mode, seed,
                _lib.ptr(h_bits), None))

        e2e_steps = max(1, min(args.steps, 2))
        t_host, _ = timed(step_host, e2e_steps, world, dev)
        host_ok = np.unpackbits(h_bits, bitorder="little")[:n].astype(bool)
        e2e = {"value": n_total * e2e_steps / t_host, "unit": "rounds/s", "ms_per_step": t_host / e2e_steps * 1e3,
               "steps": e2e_steps, "api": "dgpu_verify_beacons (pageable host records: H2D, verify, D2H)",
               "verdicts_equal_device_path": bool(np.array_equal(host_ok, verdicts[lo:hi]))}

    # configs[2] beside the metric: RLC batch verification (one multi-Miller
    # loop + one final exponentiation per checked node, root first, exact
    # per-round verdicts by bisection) over the same resident chain
    rlc = None
    if args.mode == "per-round" and not args.no_rlc and code in (_lib.SCHEME_CHAINED, _lib.SCHEME_UNCHAINED):
        def step_rlc():
            _lib.check(lib.dgpu_verify_beacons_device(
                ctx.handle, code, _lib.ptr(pk), pk.size, n, d_rounds.data_ptr(), d_sigs.data_ptr(), 96,
                d_sig_len.data_ptr(), d_prev.data_ptr(), 96, d_prev_len.data_ptr(), _lib.MODE_RLC, seed + 1,
                d_bits.data_ptr(), None, ctypes.c_void_p(stream.cuda_stream)))

        step_rlc()
        rlc_ms = stage_times(lib, ctx, step_rlc)
        rlc_steps = max(1, min(args.steps, 3))
        t_rlc, v_rlc = timed(step_rlc, rlc_steps, world, dev,
                             after=lambda: gather_verdict_bits(d_bits, n, n_total, world, rank))
        rlc = {"value": n_total * rlc_steps / t_rlc, "unit": "rounds/s", "ms_per_step": t_rlc / rlc_steps * 1e3,
               "steps": rlc_steps, "verdict_mismatches": int((v_rlc != expect).sum()), "stage_ms": rlc_ms,
               "workload": "configs[2] on the same chain: RLC batch verify, root first, per-round verdicts by "
                           "bisection (dgpu_verify_beacons_device mode DGPU_MODE_RLC)"}
        log(f"rlc: {rlc['value']:.0f} rounds/s")

    if rank == 0:
        value = n_total * args.steps / elapsed
        roofline = roofline_for(stage_ms, n if args.mode == "per-round" else None)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                from oracle import cpu_baseline as cb
                cpu = cb.run(chain, args.cpu_seconds, min(16, os.cpu_count() or 1), expect[lo:hi])
            except Exception as e:  # reported, never fatal
                cpu = {"error": repr(e)}
        log("cpu baseline done" if cpu else "no cpu baseline")
        chained = code == _lib.SCHEME_CHAINED
        nm = f"{n_total / 1e6:g}M"
        out = {
            "metric": (f"verified beacon rounds/sec, {nm}-round chained BLS12-381 chain" if chained
                       else f"verified beacon rounds/sec, {nm}-round {args.scheme} chain"),
            "value": value,
            "unit": "rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32 (14x28-bit limb Fp, int32 VALU)",
            "data": f"synthetic {args.scheme} chain generated on GPU (seeded), {args.corrupt_rate:.1%} corrupted",
            "config": {"workload": ("configs[1] shape at the metric's size: chained G2 chain, per-round pairing "
                                    "verify" if chained and args.mode == "per-round"
                                    else "configs[2]: chained G2 chain, RLC batch verify + bisection"
                                    if args.mode == "rlc" else f"configs[3]: {args.scheme} chain, per-round verify"),
                       "rounds_total": n_total, "rounds_per_gpu": n, "seg_len": args.seg_len, "scheme": args.scheme,
                       "mode": args.mode, "parallelism": f"shard{world}"},
            "stage_ms": stage_ms,
            "verdict_mismatches": mism,
            "corrupted_rounds_total": len(bad),
            "chain_gen_s": t_gen,
            "end_to_end": e2e,
            "rlc": rlc,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)


def dryrun(args):
    """DRAND_BENCH_DRYRUN=1 (CPU tests): the rank plumbing alone, over gloo
    with no GPU -- every rank reports its shard of the chain; rank 0 prints
    them as one JSON line."""
    import torch.distributed as dist
    from drand_amd.dist import shard_range
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n_total = args.rounds or 10_000_000
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "shard": shard_range(n_total, world, rank)}
    if world > 1:
        dist.init_process_group("gloo")
        got = [None] * world
        dist.all_gather_object(got, me)
        dist.destroy_process_group()
    else:
        got = [me]
    if rank == 0:
        print(json.dumps({"dryrun": True, "n_gpus": world, "rounds_total": n_total, "ranks": got}), flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if os.environ.get("DRAND_BENCH_DRYRUN"):
        return dryrun(args)
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
    try:
        if args.mode == "recover":
            main_recover(args, world, rank, local)
        else:
            main_verify(args, world, rank, local)
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
