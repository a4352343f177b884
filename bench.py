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

The default run also measures every other BASELINE.json configuration at its
stated size, each with its own verdict check, roofline and CPU baseline:
  rlc            configs[2]: RLC batch verify of the same resident chain
  configs3       configs[3]: 10M-round pedersen-bls-unchained and
                 bls-unchained-on-g1 chains, per-round verify and the
                 per-GPU RLC fold (G2 / G1 bucket-MSM roots) of each
  recover        configs[4]: threshold recovery, n=32, t=17, 100k rounds
  multi_abi      the product multi-GPU boundary (dgpu_verify_multi: one
                 process drives all N GPUs, host records, RCCL gathers), run
                 in a child process while the ranks wait
    python bench.py [--gpus N] [--steps K] [--warmup W] [--rounds R] [--no-legs]
    python bench.py --driver abi [--gpus N]   # the value through dgpu_verify_multi

With --gpus N > 1 and no torch.distributed environment, bench.py starts the
N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before
anything touches the GPU; under torch.distributed.run it is one rank.
"""
import argparse
import ctypes
import gc
import json
import os
import struct
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
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the configs[3] / configs[4] / multi_abi legs of the default run")
    ap.add_argument("--leg-steps", type=int, default=2, help="timed steps of each extra leg")
    ap.add_argument("--no-ingest", action="store_true", help="skip the bolt-store check-chain ingest leg")
    ap.add_argument("--ingest-rounds", type=int, default=1_000_000)
    ap.add_argument("--ingest-only", action="store_true",
                    help="only the bolt-store ingest leg, once per window size in --ingest-windows")
    ap.add_argument("--ingest-windows", default="262144", help="comma-separated CheckPastBeacons window sizes")
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
    ap.add_argument("--driver", choices=["dist", "abi"], default="dist",
                    help="dist: one process per GPU over torch.distributed (RCCL); abi: one process, "
                         "dgpu_verify_multi / dgpu_recover_multi over all GPUs (the Go caller's boundary)")
    ap.add_argument("--abi-devices", default=None,
                    help="abi driver: comma-separated device list (default 0..N-1; a repeated device needs "
                         "DGPU_MULTI_ALLOW_SAME_DEVICE=1)")
    ap.add_argument("--abi-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-small-batch", action="store_true", help="skip the small-batch latency leg")
    ap.add_argument("--small-batch-sizes", default=None,
                    help="comma-separated call sizes for the small-batch leg (default 1,8,64,500,4096)")
    ap.add_argument("--small-batch-only", action="store_true",
                    help="only the small-batch latency leg (host records, n = 1 .. 4096) on a 4096-round chain")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the chosen driver, the rank count and each rank's shard, touch no GPU")
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


def _load_json(*parts):
    p = os.path.join(ROOT, *parts)
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def engine_work():
    """Exact per-item work of the pairing-engine kernels (tools/engine_work.py
    -> profiles/engine_work.json: product terms + reductions of the generated
    programs, x 196 v_mad_u64_u32 each)."""
    return _load_json("profiles", "engine_work.json").get("kernels", {})


def hash_work():
    """Per-round v_mad_u64_u32 counts of the hash / decode / RLC / on-G1
    kernels (tools/count_ops.py -> profiles/op_counts.json, counted by the host
    build of the same device functions)."""
    return _load_json("profiles", "op_counts.json").get("kernels", {})


# stage name (dgpu_stage_times) -> work key (profiles/*.json), per pipeline
STAGE_WORK = {
    "g2": {"eng_lines": "k_eng_lines", "eng_miller": "k_eng_miller", "eng_inv": "k_eng_inv", "eng_fe": "k_eng_fe",
           "hash_to_g2": "hash_to_g2", "decode_g2": "k_decode_g2_sigs", "h_affine": "k_g2_batch_affine"},
    "g1": {"eng_miller": "k_eng_miller_fixed", "eng_inv": "k_eng_inv", "eng_fe": "k_eng_fe",
           "eng_lines_fixed": "k_eng_lines_fixed", "hash_to_g1": "k_hash_to_g1_beacons",
           "decode_g1": "k_decode_g1_sigs", "h_affine": "k_g1_batch_affine"},
    # RLC: the per-round stages only (node checks are data-dependent: 1 at 0% corruption)
    "rlc": {"rlc_hash_to_g2_raw": "rlc_hash_to_g2_raw", "decode_g2": "k_decode_g2_sigs+subgroup",
            "rlc_affine": "k_g2_batch_affine", "rlc_root_msm": "rlc_root_msm", "rlc_leaves_tree": "rlc_leaves_tree",
            "rlc_plain_tree": "rlc_plain_tree"},
    # RLC for the G1-signature schemes (configs[3]'s per-GPU fold)
    "rlc_g1": {"rlc_hash_to_g1_raw": "rlc_hash_to_g1_raw", "decode_g1": "k_decode_g1_sigs",
               "rlc_affine": "k_g1_batch_affine", "rlc_root_msm": "rlc_root_msm_g1",
               "rlc_leaves_tree": "rlc_leaves_tree_g1", "rlc_plain_tree": "rlc_plain_tree_g1"},
    # recovery (batched check): per round, one pairing check and the MSMs
    "recover": {"eng_lines": "k_eng_lines", "eng_miller": "k_eng_miller", "eng_inv": "k_eng_inv",
                "eng_fe": "k_eng_fe", "recover_msm": "recover_msm", "recover_rlc_g1": "recover_rlc_g1"},
}


def recover_work(t, slices=5):
    """Per-round v_mad_u64_u32 of the recovery MSM kernels, composed from the
    counted group-law ops (profiles/op_counts.json group_ops) along the code's
    operation sequence (recover.cuh): k_recover_msm_w4, per slice, a table
    [1..8] sig_j (1 doubling + 6 mixed additions per point) then 17 signed
    radix-16 windows of 4 doublings (16 of them) + t full additions; k_recover_rlc_g1
    64 G1 doublings + 17 t mixed additions + C_0."""
    go = _load_json("profiles", "op_counts.json").get("group_ops")
    if not go:
        return {}
    m = lambda k: go[k]["mads"]  # noqa: E731
    slice_mads = t * (m("g2_dbl") + 6 * m("g2_add_affine")) + 64 * m("g2_dbl") + 17 * t * m("g2_add")
    g1 = 64 * m("g1_dbl") + (17 * t + 1) * m("g1_add_affine")
    return {"recover_msm": {"mads": slices * slice_mads}, "recover_rlc_g1": {"mads": g1}}
# the Karabina FE's stages (libdrand_gpu eng_fe_kb_locked): the 12-lane
# program segments (+ the flagged-block fallback), the 8-lane compressed
# chains, the norms' inversion and the decompression
KB_STAGE_WORK = {"eng_fe": "k_eng_fe_seg", "eng_fe_chain": "k_eng_kb_chain", "eng_fe_kbinv": "k_eng_kb_inv"}


# the T-steps run per thread (k_lines_thr) unless DGPU_LINES=engine selects
# the 12-lane engine program (k_eng_lines)
if os.environ.get("DGPU_LINES") != "engine":
    for _p in ("g2", "recover"):
        STAGE_WORK[_p]["eng_lines"] = "k_lines_thr"
# likewise the compressed chains (k_kb_chain_thr; DGPU_KB_CHAIN=lanes: k_eng_kb_chain)
if os.environ.get("DGPU_KB_CHAIN") != "lanes":
    KB_STAGE_WORK["eng_fe_chain"] = "k_kb_chain_thr"


# stage -> kernel symbol for the traffic lookup
STAGE_KERNEL = {"eng_lines": STAGE_WORK["g2"]["eng_lines"], "eng_miller": "k_eng_miller", "eng_inv": "k_eng_inv", "eng_fe": "k_eng_fe",
                "eng_lines_fixed": "k_eng_lines_fixed", "hash_to_g2": "hash_to_g2", "decode_g2": "k_decode_g2_sigs",
                "hash_to_g1": "k_hash_to_g1_beacons", "decode_g1": "k_decode_g1_sigs",
                "rlc_leaves_tree": "k_rlc_leaves"}


def traffic_for(kern, items):
    """PMC FETCH_SIZE + WRITE_SIZE per item of this build (latest profiles/**/r0*_traffic.json)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "r0*_traffic.json"), recursive=True),
                       key=os.path.basename, reverse=True):
        with open(path) as f:
            t = json.load(f)["kernels"]
        key = next((k for k in t if k.split("::")[-1].split("(")[0] == kern), None)
        if key:
            per = t[key]
            return items * (per["fetch_bytes_per_round"] + per["write_bytes_per_round"]), os.path.basename(path)
    return None, None


def roofline_for(stage_ms, items, pipeline="g2", stage_items=None, extra_work=None):
    """Roofline of the dominant stage (largest summed launch time among the
    stages with a work figure; chunked stages are summed over their
    launches): achieved = algorithmic v_mad_u64_u32 products over the launches
    / measured time (HIP events on the launch stream) vs the measured int32
    mad peak; traffic = PMC bytes of this build over the same launches.
    items = work items per pass (rounds, or pairing checks); stage_items
    overrides it per stage."""
    if not stage_ms or not items:
        return None
    wmap = dict(STAGE_WORK[pipeline])
    # Karabina FE (default; DGPU_FE=gs runs k_eng_fe alone under "eng_fe"), on
    # the pipelines whose engine stages run once per item (not RLC's node checks)
    if "eng_fe_chain" in stage_ms and "eng_fe" in wmap:
        wmap.update(KB_STAGE_WORK)
    work = dict(hash_work(), **engine_work())
    work.update(extra_work or {})
    have = {s: t for s, t in stage_ms.items() if s in wmap and wmap[s] in work and t > 0}
    if not have:
        return None
    stage_items = stage_items or {}
    name = max(have, key=have.get)
    ms = have[name]
    key = wmap[name]
    it = stage_items.get(name, items)
    per_item = work[key]["mads"]
    achieved = it * per_item / (ms * 1e-3)
    out = {"bound": "valu-int32", "unit": "T mad_u64_u32/s", "kernel": key, "stage": name, "launch_ms_total": ms,
           "items": it, "peak": PEAK_MAD_U64_PER_S / 1e12, "achieved": achieved / 1e12,
           "frac": achieved / PEAK_MAD_U64_PER_S, "traffic": None, "work_per_item_mads": per_item,
           "work_source": ("profiles/engine_work.json" if key in engine_work() else
                           "profiles/op_counts.json group_ops (bench.recover_work)" if key in (extra_work or {}) else
                           "profiles/op_counts.json")}
    out["stage_frac"] = {s: stage_items.get(s, items) * work[wmap[s]]["mads"] / (t * 1e-3) / PEAK_MAD_U64_PER_S
                         for s, t in have.items()}
    kb = "eng_fe_chain" in stage_ms and name in KB_STAGE_WORK
    traffic, src = traffic_for(key if kb else STAGE_KERNEL.get(name, key), it)
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
    try:
        out = _lib.stage_times(ctx)
    finally:
        _lib.check(lib.dgpu_set_profiling(ctx.handle, 0))
    torch.cuda.synchronize()
    return out


def coll_device(dev):
    """Where the bench's own small collectives run: the GPU over RCCL, the CPU
    when the process group is gloo (DRAND_BENCH_BACKEND=gloo: several ranks
    rehearsed on one GPU)."""
    import torch.distributed as dist
    return "cpu" if dist.is_initialized() and dist.get_backend() == "gloo" else dev


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
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll_device(dev))
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), res


def shard_chain(seed, seg, code, lo, hi, device):
    """This rank's rounds [lo + 1, hi] of the global chain: whole seg_len
    segments are generated (segment s covers rounds s*seg_len + 1 ..; its seed
    depends only on s), so every rank sees the same chain whatever N is."""
    from drand_amd.synth import make_chain
    s0 = lo // seg
    s1 = (hi + seg - 1) // seg
    ch = make_chain(seed, (s1 - s0) * seg, code, seg_len=seg, device=device, start_round=s0 * seg + 1)
    a, b = lo - s0 * seg, hi - s0 * seg
    for name in ("rounds", "sigs", "sig_len", "prev", "prev_len"):
        setattr(ch, name, np.ascontiguousarray(getattr(ch, name)[a:b]))
    return ch


def cpu_threads():
    """cpu_baseline threads: every core this process may run on (GOMAXPROCS =
    the host's cores, as north_star asks; host and cgroup views are reported)."""
    return len(os.sched_getaffinity(0))


# ---------------------------------------------------------------- configs[4]
def recover_leg(args, world, rank, local, n_total, steps, warmup, cpu_seconds):
    """configs[4]: batch threshold recovery (kyber tbls.Recover as the
    aggregator calls it, chain/beacon/chain.go:158-168): per round t partials
    (one invalid in --bad-rate of the rounds), VerifyPartial, selection +
    Lagrange + G2 MSM, VerifyRecovered.  Inputs resident in HBM
    (dgpu_recover_batch_device).  The batch is split into contiguous round
    shards (strong scaling); each rank checks its own outputs."""
    import torch
    import torch.distributed as dist
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.dist import shard_range
    from drand_amd.synth import group_signatures, make_group, make_recovery_batch

    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    dev = torch.device("cuda", local)
    t_gen = time.time()
    grp = make_group(args.seed, args.t, args.n, device=local)
    msgs, parts, expect_ok = make_recovery_batch(grp, n, args.seed + 7919 * rank, args.bad_rate,
                                                 first_round=lo + 1, device=local)
    expect = group_signatures(grp, msgs, device=local)
    t_gen = time.time() - t_gen
    log(f"recover: {n} rounds generated in {t_gen:.1f} s")
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

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    stage_ms = stage_times(lib, ctx, step)
    elapsed, _ = timed(step, steps, world, dev)
    # per-step wall times (diagnostic: host-side gaps between the kernels)
    step_ms = []
    for _ in range(2):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        step_ms.append((time.perf_counter() - t0) * 1e3)

    ok = d_ok.cpu().numpy().astype(bool)
    out = d_out.cpu().numpy()
    mism = int((ok != expect_ok).sum()) + int((out[ok & expect_ok] != expect[ok & expect_ok]).any(axis=1).sum())
    mism_t = torch.tensor([mism], device=coll_device(dev))
    if world > 1:
        dist.all_reduce(mism_t)
    res = {"metric": "recovered beacon rounds/sec, t-of-n threshold recovery (VerifyPartial x t, Lagrange, "
                     "G2 MSM, VerifyRecovered)",
           "value": n_total * steps / elapsed, "unit": "rounds/s", "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True, "scaling": "strong",
           "dtype": "u32 (14x28-bit limb Fp, 10x28-bit limb Fr, int32 VALU)",
           "data": f"synthetic {args.t}-of-{args.n} group and partials generated on GPU (seeded), "
                   f"{args.bad_rate:.0%} of rounds with one invalid partial",
           "config": {"workload": "configs[4]: threshold recovery, n=%d, t=%d" % (args.n, args.t),
                      "rounds_total": n_total, "rounds_per_gpu": n, "partials_per_round": m, "mode": "recover",
                      "parallelism": f"shard{world}"},
           "stage_ms": stage_ms, "stage_ms_total": sum(stage_ms.values()), "extra_step_ms": step_ms,
           "verdict_mismatches": int(mism_t.item()),
           "unrecoverable_rounds_rank0": int((~expect_ok).sum()), "gen_s": t_gen}
    if rank == 0:
        res["roofline"] = roofline_for(stage_ms, n, "recover", extra_work=recover_work(args.t))
        if res["roofline"]:
            res["roofline"]["items_note"] = ("rounds per pass (the batched check: one pairing and the MSMs per "
                                             "round; rounds on the exact path add engine items)")
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                from oracle import cpu_baseline as cb
                exp_sigs = [bytes(expect[i]) if expect_ok[i] else None for i in range(n)]
                cpu = cb.run_recover(grp.commits, grp.t, grp.n, msgs, parts, exp_sigs, cpu_seconds, cpu_threads())
            except Exception as e:  # reported, never fatal
                cpu = {"error": repr(e)}
        res["cpu_baseline"] = cpu
    del d_msgs, d_parts, d_plen, d_out, d_ok
    return res


# ---------------------------------------------------------------- latency callers
SMALL_BATCH_SIZES = (1, 8, 64, 500, 4096)


def small_batch_leg(chain, scheme, sizes=SMALL_BATCH_SIZES, budget_s=20.0):
    """The latency-bound callers: tryNode verifies a peer stream buffered
    MaxSyncBuffer = 500 beacons deep (net/client_grpc.go:220, verify at
    chain/beacon/sync_manager.go:397), the client walk verifies a fetched
    range (client/verify.go:149-169), the gossip validator one beacon per
    message (lp2p/client/validator.go:64-66).  Each size n: wall time of one
    dgpu_verify_beacons call on n host records (H2D, verify, D2H; the
    library's default kernel thresholds), median and p90 over repeated calls,
    beside the C port's single-core time for the same n beacons (the
    reference's loops are one goroutine).  The crossover is the smallest n
    where the GPU call beats the single core."""
    from drand_amd import _lib
    from drand_amd.chain import get_context
    ctx = get_context(0)
    lib = ctx.lib
    code = lib.dgpu_scheme_from_name(scheme.encode())
    pk = np.frombuffer(chain.pk, dtype=np.uint8).copy()
    cpu_ms_per_round = None
    try:
        from oracle import c_ref
        c_ref.load()
        k = min(8, len(chain))  # a chain of fewer records (--small-batch-sizes 1) times what it has
        sub = [np.ascontiguousarray(a[:k]) for a in (chain.rounds, chain.sigs, chain.sig_len, chain.prev,
                                                     chain.prev_len)]
        g1 = code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)

        def cpu():
            if g1:  # G1 signatures: the restatement's own entry (G2 key, RFC 9380 or drand DST)
                return c_ref.verify_batch_g1(code == _lib.SCHEME_G1_RFC9380, chain.pk, sub[0], sub[1], sub[2], 1)
            return c_ref.verify_batch(code == _lib.SCHEME_CHAINED, chain.pk, *sub, 1)
        cpu()  # warm
        t0 = time.perf_counter()
        ref = cpu()
        cpu_ms_per_round = (time.perf_counter() - t0) * 1e3 / k
        if int((ref != 0).sum()) > k // 2:  # a timing of rejected records would be meaningless
            raise RuntimeError("C port rejected the sample")
    except Exception as e:  # reported, never fatal
        log(f"small-batch: no C port timing ({e!r})")
    rows = []
    per_size = budget_s / len(sizes)
    for n in sizes:
        n = min(n, len(chain))
        cols = [np.ascontiguousarray(a[:n]) for a in (chain.rounds, chain.sigs, chain.sig_len, chain.prev,
                                                        chain.prev_len)]
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)

        def call():
            _lib.check(lib.dgpu_verify_beacons(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(cols[0]),
                                               _lib.ptr(cols[1]), 96, _lib.ptr(cols[2]), _lib.ptr(cols[3]), 96,
                                               _lib.ptr(cols[4]), _lib.MODE_PER_ROUND, 0, _lib.ptr(bits), None))
        for _ in range(3):  # buffers sized, kernels loaded
            call()
        ts = []
        t_end = time.perf_counter() + per_size
        while len(ts) < 5 or (time.perf_counter() < t_end and len(ts) < 200):
            t0 = time.perf_counter()
            call()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        row = {"n": n, "gpu_ms_median": ts[len(ts) // 2], "gpu_ms_p90": ts[int(len(ts) * 0.9)], "calls": len(ts),
               "gpu_rounds_per_s": n / (ts[len(ts) // 2] * 1e-3)}
        if cpu_ms_per_round:
            row["cpu_1core_ms"] = n * cpu_ms_per_round
            row["gpu_faster"] = row["gpu_ms_median"] < row["cpu_1core_ms"]
        rows.append(row)
        log(f"small-batch n={n}: {row['gpu_ms_median']:.2f} ms")
    cross = next((r["n"] for r in rows if r.get("gpu_faster")), None)
    return {"api": "dgpu_verify_beacons (host records, per-round mode, default thresholds)", "scheme": scheme,
            "rows": rows, "cpu_1core_ms_per_round": cpu_ms_per_round,
            "cpu_kind": "port (oracle/c/bls381_ref.c, one thread; kilic's x86 asm is not available here)",
            "crossover_n": cross,
            "callers": "tryNode windows of <= 500 (net/client_grpc.go:220), gossip validator 1 per message "
                       "(lp2p/client/validator.go:64-66)"}


# ---------------------------------------------------------------- check-chain ingest
def _hex_rows(a, lens):
    """numpy (n, stride) bytes -> lowercase hex of each row's first lens[i] bytes"""
    table = np.frombuffer(b"".join(b"%02x" % v for v in range(256)), dtype=np.uint8).reshape(256, 2)
    hx = table[a].reshape(a.shape[0], -1)
    return [bytes(hx[i, :2 * int(lens[i])]) for i in range(a.shape[0])]


def ingest_leg(chain, n_rows, scheme, window=1 << 18, windows=None):
    """The bulk check-chain path end to end from a drand bolt store: n_rows
    rounds of the bench chain written (outside the timed region, with the
    test writer tests/bolt_writer.py) as Beacon.Marshal rows keyed by
    RoundToBytes (chain/boltdb/store.go:72-86), then CheckPastBeacons
    (chain/beacon/sync_manager.go:171-232) timed over the file: native B+tree
    walk + hexjson decode of each window overlapped with the GPU verify of the
    previous one (drand_amd/sync.py, drand_amd/ingest.py)."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from bolt_writer import write_bolt
    from drand_amd import ingest
    from drand_amd.boltstore import BoltStore
    from drand_amd.chain import Verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.sync import check_past_beacons
    n = min(n_rows, len(chain))
    t0 = time.perf_counter()
    sig_hex = _hex_rows(chain.sigs[:n], chain.sig_len[:n])
    prev_hex = _hex_rows(chain.prev[:n], chain.prev_len[:n])
    kv = {struct.pack(">Q", 0): b'{"PreviousSig":null,"Round":0,"Signature":"' + chain.genesis.hex().encode() + b'"}'}
    for i in range(n):
        r = int(chain.rounds[i])
        p = b'"' + prev_hex[i] + b'"' if chain.prev_len[i] else b"null"
        kv[struct.pack(">Q", r)] = (b'{"PreviousSig":' + p + b',"Round":' + str(r).encode() + b',"Signature":"' +
                                   sig_hex[i] + b'"}')
    del sig_hex, prev_hex
    d = tempfile.mkdtemp(prefix="drand_ingest_")
    path = os.path.join(d, "drand.db")
    write_bolt(path, kv)
    del kv
    t_write = time.perf_counter() - t0
    log(f"ingest: {n}-round bolt file written in {t_write:.1f} s")
    bs = BoltStore(path)
    v = Verifier(get_scheme_by_id_with_default(scheme))
    try:
        check_past_beacons(bs, v, chain.pk, 1 << 16, window=1 << 16)  # warm: key decode, buffers, page cache
        sweep = {}
        for w in windows or ():  # --ingest-only: the same file at other window sizes
            check_past_beacons(bs, v, chain.pk, 10 ** 12, window=w)
            t0 = time.perf_counter()
            check_past_beacons(bs, v, chain.pk, 10 ** 12, window=w)
            sweep[w] = n / (time.perf_counter() - t0)
            log(f"ingest window {w}: {sweep[w]:.0f} rounds/s")
        t0 = time.perf_counter()
        faulty = check_past_beacons(bs, v, chain.pk, 10 ** 12, window=window)
        el = time.perf_counter() - t0
        t0 = time.perf_counter()
        for lo in range(1, n + 1, window):
            ingest.window_records(bs, lo, min(n + 1, lo + window))
        t_dec = time.perf_counter() - t0
        expect = [int(chain.rounds[i]) for i in range(n) if not _valid_by_construction(chain, i)]
        res = {"value": n / el, "unit": "rounds/s", "rounds": n, "seconds": el, "window": window,
               "faulty_rounds": len(faulty or []), "faulty_equal_construction": (faulty or []) == expect,
               "decode_only_rounds_per_s": n / t_dec, "file_bytes": os.path.getsize(path),
               "write_s": t_write, "decode_threads": ingest.DECODE_THREADS,
               "api": "sync.check_past_beacons(BoltStore) -> native scan/decode -> dgpu_verify_beacons"}
        if sweep:
            res["window_sweep"] = {str(k): v for k, v in sweep.items()}
    finally:
        bs.close()
        os.remove(path)
        os.rmdir(d)
    return res


_EXPECT = {}


def _valid_by_construction(chain, i):
    return _EXPECT.get(id(chain), {}).get(i, True)


# ---------------------------------------------------------------- configs[1..3]
def verify_leg(args, world, rank, local, scheme, n_total, steps, warmup, mode="per-round", e2e=False, rlc=False,
               cpu_seconds=None, main=False):
    """One chain of `scheme`, n_total rounds sharded over the ranks, verified
    `steps` times with inputs resident in HBM (dgpu_verify_beacons_device),
    verdicts all-gathered (RCCL) and checked against the construction; plus
    optionally the host-record pass (e2e) and the RLC pass over the same chain."""
    import torch
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.dist import gather_verdict_bits, shard_range, verify_rlc_sharded
    from drand_amd.synth import corrupt_global

    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    code = _lib.load().dgpu_scheme_from_name(scheme.encode())
    t_gen = time.time()
    log(f"generating rounds [{lo + 1}, {hi}] of a {n_total}-round {scheme} chain")
    chain = shard_chain(args.seed, args.seg_len, code, lo, hi, local)
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
    mcode = _lib.MODE_RLC if mode == "rlc" else _lib.MODE_PER_ROUND
    seed = args.rlc_seed + 7 * rank

    def step_mode(md, sd):
        if md == _lib.MODE_RLC and world > 1:  # the per-rank RLC protocol: roots all-gathered, one node check
            verify_rlc_sharded(ctx, code, pk, n, d_rounds, d_sigs, d_sig_len, d_prev, d_prev_len, sd, d_bits, stream,
                               world, rank)
            return
        _lib.check(lib.dgpu_verify_beacons_device(
            ctx.handle, code, _lib.ptr(pk), pk.size, n, d_rounds.data_ptr(), d_sigs.data_ptr(), 96,
            d_sig_len.data_ptr(), d_prev.data_ptr(), 96, d_prev_len.data_ptr(), md, sd, d_bits.data_ptr(),
            None, ctypes.c_void_p(stream.cuda_stream)))

    step = lambda: step_mode(mcode, seed)  # noqa: E731
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    log(f"{scheme} warmup done")
    # per-stage kernel timing (HIP events on the launch stream), single lane;
    # the first of the two passes absorbs the single-lane buffer growth
    stage_ms = stage_times(lib, ctx, step, passes=2 if main else 1)
    log("stage times", json.dumps(stage_ms))
    # the exchange step: every rank's verdict bitmap to every rank (RCCL)
    elapsed, verdicts = timed(step, steps, world, dev,
                              after=lambda: gather_verdict_bits(d_bits, n, n_total, world, rank))
    log(f"{scheme}: {steps} steps in {elapsed:.3f} s")
    expect = np.ones(n_total, dtype=bool)
    expect[list(bad.keys())] = False
    res = {"value": n_total * steps / elapsed, "unit": "rounds/s", "steps": steps, "warmup": warmup,
           "ms_per_step": elapsed / steps * 1e3, "stage_ms": stage_ms,
           "verdict_mismatches": int((verdicts != expect).sum()), "corrupted_rounds_total": len(bad),
           "chain_gen_s": t_gen, "scheme": scheme, "rounds_total": n_total, "rounds_per_gpu": n}
    g1 = code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)
    rlc_pipe = "rlc_g1" if g1 else "rlc"
    pipeline = rlc_pipe if mode == "rlc" else ("g1" if g1 else "g2")
    if rank == 0:
        res["roofline"] = roofline_for(stage_ms, n, pipeline)

    if e2e:  # host records through dgpu_verify_beacons (H2D + D2H inside)
        h_bits = np.zeros((n + 7) // 8, dtype=np.uint8)

        def step_host():
            _lib.check(lib.dgpu_verify_beacons(
                ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(chain.rounds), _lib.ptr(chain.sigs), 96,
                _lib.ptr(chain.sig_len), _lib.ptr(chain.prev), 96, _lib.ptr(chain.prev_len), mcode, seed,
                _lib.ptr(h_bits), None))

        e2e_steps = max(1, min(steps, 2))
        t_host, _ = timed(step_host, e2e_steps, world, dev)
        host_ok = np.unpackbits(h_bits, bitorder="little")[:n].astype(bool)
        st_ms, st_host_ms, st_bytes = _lib.staging_stats(ctx)
        res["end_to_end"] = {"value": n_total * e2e_steps / t_host, "unit": "rounds/s",
                             "ms_per_step": t_host / e2e_steps * 1e3, "steps": e2e_steps,
                             "api": "dgpu_verify_beacons (pageable caller records through the library's pinned ring, "
                                    "slice by slice beside the verification; verdicts D2H)",
                             "staging": {"ms": round(st_ms, 2), "host_ms": round(st_host_ms, 2), "bytes": st_bytes,
                                         "GB_per_s": round(st_bytes / max(st_ms, 1e-6) / 1e6, 2)},
                             "vs_resident": (n_total * e2e_steps / t_host) / res["value"] if res.get("value") else None,
                             "verdicts_equal_device_path": bool(np.array_equal(host_ok, verdicts[lo:hi]))}

    # configs[2] beside the metric: RLC batch verification (one multi-Miller
    # loop + one final exponentiation per checked node, root first, exact
    # per-round verdicts by bisection) over the same resident chain
    if rlc and mode == "per-round":
        step_rlc = lambda: step_mode(_lib.MODE_RLC, seed + 1)  # noqa: E731
        step_rlc()
        rlc_ms = stage_times(lib, ctx, step_rlc)
        rlc_steps = max(1, min(steps, 3))
        t_rlc, v_rlc = timed(step_rlc, rlc_steps, world, dev,
                             after=lambda: gather_verdict_bits(d_bits, n, n_total, world, rank))
        res["rlc"] = {"value": n_total * rlc_steps / t_rlc, "unit": "rounds/s", "ms_per_step": t_rlc / rlc_steps * 1e3,
                      "steps": rlc_steps, "verdict_mismatches": int((v_rlc != expect).sum()), "stage_ms": rlc_ms,
                      "roofline": roofline_for(rlc_ms, n, rlc_pipe) if rank == 0 else None,
                      "workload": ("configs[3] per-GPU fold on the same chain: RLC batch verify of G1 signatures "
                                   "(G1 bucket-MSM root, one 2-pair check on the key's fixed-Q lines), root first, "
                                   "per-round verdicts by bisection (dgpu_verify_beacons_device mode DGPU_MODE_RLC)"
                                   if g1 else
                                   "configs[2] on the same chain: RLC batch verify, root first, per-round verdicts by "
                                   "bisection (dgpu_verify_beacons_device mode DGPU_MODE_RLC)")}
        log(f"rlc: {res['rlc']['value']:.0f} rounds/s")

    if main and rank == 0 and world == 1 and not args.no_small_batch:
        try:
            res["small_batch"] = small_batch_leg(chain, scheme)
        except Exception as e:  # reported, never fatal
            res["small_batch"] = {"error": repr(e)}
    if main and rank == 0 and world == 1 and not args.no_ingest:
        _EXPECT[id(chain)] = {gi - lo: False for gi in bad if lo <= gi < hi}
        try:
            res["ingest"] = ingest_leg(chain, args.ingest_rounds, scheme)
            log(f"ingest: {res['ingest']['value']:.0f} rounds/s")
        except Exception as e:  # reported, never fatal
            res["ingest"] = {"error": repr(e)}
    if rank == 0 and cpu_seconds and not args.no_cpu_baseline and world == 1:
        try:
            from oracle import cpu_baseline as cb
            res["cpu_baseline"] = cb.run(chain, cpu_seconds, cpu_threads(), expect[lo:hi])
        except Exception as e:  # reported, never fatal
            res["cpu_baseline"] = {"error": repr(e)}
        log("cpu baseline done")
        if "rlc" in res and "value" in res["cpu_baseline"]:
            # the reference has no batch mode: its CPU path verifies every round with
            # its own pairing whatever the GPU's mode, so the leg's baseline stands
            res["rlc"]["cpu_baseline"] = dict(res["cpu_baseline"], note="same CPU run as this leg's cpu_baseline "
                                              "(the reference verifies each round with its own pairing check)")
    del d_rounds, d_sigs, d_sig_len, d_prev, d_prev_len, d_bits, chain
    gc.collect()
    torch.cuda.empty_cache()
    return res


# ---------------------------------------------------------------- the product multi-GPU boundary
def abi_devices(args, ngpu):
    if args.abi_devices:
        return [int(x) for x in args.abi_devices.split(",")]
    return list(range(ngpu))


def multi_staging(mctx, ndev):
    """Per device of a dgpu_verify_multi handle: the last call's host-record
    staging through that context's pinned ring (dgpu_staging_stats: span on
    its copy stream, bytes) -- the concurrent H2D of every shard from one
    process, which the per-GPU compute has to hide."""
    from drand_amd import _lib

    class _C:  # a device context of the handle, as _lib.staging_stats takes it
        pass
    out = []
    for k in range(ndev):
        h = ctypes.c_void_p()
        _lib.check(mctx.lib.dgpu_multi_context(mctx.handle, k, ctypes.byref(h)))
        c = _C()
        c.lib, c.handle = mctx.lib, h
        ms, hms, nb = _lib.staging_stats(c)
        out.append({"ms": round(ms, 2), "host_ms": round(hms, 2), "bytes": nb,
                    "GB_per_s": round(nb / max(ms, 1e-6) / 1e6, 2)})
    return {"per_device": out, "max_ms": max(d["ms"] for d in out), "max_host_ms": max(d["host_ms"] for d in out),
            "note": "ms: span on each context's copy stream, first ring piece to last DMA of its shard; host_ms: "
                    "its staging thread's wall time, first memcpy into the ring to the last DMA enqueued"}


def main_abi(args):
    """One process drives every GPU through the C ABI as a Go caller of
    crypto/gpu would: dgpu_verify_multi over host records
    (per-device staging, verify, RCCL all-gather of the verdict bitmaps), and
    dgpu_recover_multi for --mode recover.  No torch in this process."""
    from drand_amd import _lib
    from drand_amd.multi import MultiThresholdGroup, MultiVerifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.synth import corrupt_global, group_signatures, make_chain, make_group, make_recovery_batch
    devs = abi_devices(args, args.gpus)
    mctx = _lib.MultiContext(devs)
    wall = lambda: time.perf_counter()  # noqa: E731
    if args.mode == "recover":
        n_total = args.rounds or 100_000
        grp = make_group(args.seed, args.t, args.n, device=devs[0])
        msgs, parts, expect_ok = make_recovery_batch(grp, n_total, args.seed, args.bad_rate, device=devs[0])
        expect = group_signatures(grp, msgs, device=devs[0])
        mg = MultiThresholdGroup(grp.commits, grp.n, mctx=mctx)
        nr, m = parts.shape[:2]
        mb = np.ascontiguousarray(msgs).reshape(-1)
        plen = np.full((nr, m), 98, dtype=np.uint32)
        run = lambda: mg.recover_records(mb, parts, plen)  # noqa: E731
        for _ in range(args.warmup):
            run()
        t0 = wall()
        for _ in range(args.steps):
            sigs, _ = run()
        el = wall() - t0
        okv = np.array([s is not None for s in sigs])
        mism = int((okv != expect_ok).sum()) + sum(1 for i, s in enumerate(sigs) if s is not None and expect_ok[i]
                                                  and s != bytes(expect[i]))
        res = {"value": n_total * args.steps / el, "unit": "rounds/s", "ms_per_step": el / args.steps * 1e3,
               "rounds_total": n_total, "verdict_mismatches": mism, "workload": "configs[4] through dgpu_recover_multi"}
    else:
        n_total = args.rounds or 10_000_000
        code = _lib.load().dgpu_scheme_from_name(args.scheme.encode())
        t_gen = wall()
        chain = make_chain(args.seed, n_total, code, seg_len=args.seg_len, device=devs[0])
        bad = corrupt_global(chain, args.seed, n_total, 0, rate=args.corrupt_rate)
        t_gen = wall() - t_gen
        log(f"abi: {n_total}-round chain in {t_gen:.1f} s")
        mv = MultiVerifier(get_scheme_by_id_with_default(args.scheme), mctx=mctx)
        mcode = _lib.MODE_RLC if args.mode == "rlc" else _lib.MODE_PER_ROUND
        run = lambda: mv.verify_records(chain.pk, chain.rounds, chain.sigs, chain.sig_len, chain.prev,  # noqa: E731
                                        chain.prev_len, mcode, args.rlc_seed)
        for _ in range(args.warmup):
            run()
        t0 = wall()
        for _ in range(args.steps):
            reason = run()
        el = wall() - t0
        expect = np.ones(n_total, dtype=bool)
        expect[list(bad.keys())] = False
        res = {"value": n_total * args.steps / el, "unit": "rounds/s", "ms_per_step": el / args.steps * 1e3,
               "rounds_total": n_total, "verdict_mismatches": int(((reason == 0) != expect).sum()),
               "chain_gen_s": t_gen, "scheme": args.scheme, "mode": args.mode,
               "workload": "dgpu_verify_multi over host records (per-device H2D staging, verify, RCCL verdict "
                           "all-gather, D2H)",
               "staging": multi_staging(mctx, len(devs))}
    res.update({"n_gpus": len(devs), "devices": devs, "steps": args.steps, "warmup": args.warmup,
                "driver": "abi (one process, libdrand_gpu.so multi-GPU handle)",
                "gather": "in-library device copies (DGPU_MULTI_ALLOW_SAME_DEVICE)" if os.environ.get(
                    "DGPU_MULTI_ALLOW_SAME_DEVICE") == "1" else "RCCL ncclAllGather"})
    mctx.close()
    return res


def multi_abi_leg(args, world, rank):
    """The abi driver in a child process (this rank's GPU state stays as is;
    the other ranks wait on a CPU barrier), bounded by a timeout: reported
    beside the main line, never fatal."""
    n_total = args.rounds or 10_000_000
    cmd = [sys.executable, os.path.abspath(__file__), "--abi-child", "--gpus", str(world), "--rounds", str(n_total),
           "--steps", str(args.leg_steps), "--warmup", "1", "--seed", str(args.seed)]
    log("multi_abi: " + " ".join(cmd[2:]))
    try:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, text=True)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            return {"error": f"rc {p.returncode}", "stderr_tail": p.stderr[-800:]}
        return json.loads(lines[-1])
    except subprocess.TimeoutExpired:
        return {"error": "timeout (300 s)"}


# ---------------------------------------------------------------- main
def main_verify(args, world, rank, local):
    import torch.distributed as dist
    n_total = args.rounds or 10_000_000
    main = verify_leg(args, world, rank, local, args.scheme, n_total, args.steps, args.warmup, mode=args.mode,
                      e2e=not args.no_e2e, rlc=not args.no_rlc, cpu_seconds=args.cpu_seconds, main=True)
    legs = {}
    default_run = args.mode == "per-round" and args.scheme == "pedersen-bls-chained" and not args.no_legs
    if default_run:
        # configs[3]: the two unchained schemes at their stated size
        legs["configs3"] = {}
        for sch in ("pedersen-bls-unchained", "bls-unchained-on-g1"):
            legs["configs3"][sch] = verify_leg(args, world, rank, local, sch, n_total, args.leg_steps, 1,
                                               rlc=not args.no_rlc, cpu_seconds=args.cpu_seconds / 2)
        # configs[4]: threshold recovery at its stated shape
        legs["recover"] = recover_leg(args, world, rank, local, 100_000, max(args.leg_steps, 3), 1,
                                      args.cpu_seconds / 2)
        # the product multi-GPU boundary over all ranks' GPUs, in a child process
        gl = dist.new_group(backend="gloo") if world > 1 else None
        if rank == 0:
            legs["multi_abi"] = multi_abi_leg(args, world, rank)
        if gl is not None:
            dist.barrier(group=gl)
    if rank != 0:
        return
    chained = args.scheme == "pedersen-bls-chained"
    nm = f"{n_total / 1e6:g}M"
    out = {
        "metric": (f"verified beacon rounds/sec, {nm}-round chained BLS12-381 chain" if chained
                   else f"verified beacon rounds/sec, {nm}-round {args.scheme} chain"),
        "value": main["value"],
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32 (14x28-bit limb Fp, int32 VALU)",
        "data": f"synthetic {args.scheme} chain generated on GPU (seeded), {args.corrupt_rate:.1%} corrupted",
        "config": {"workload": ("configs[1] shape at the metric's size: chained G2 chain, per-round pairing "
                                "verify" if chained and args.mode == "per-round"
                                else "configs[2]: chained G2 chain, RLC batch verify + bisection"
                                if args.mode == "rlc" else f"configs[3]: {args.scheme} chain, per-round verify"),
                   "rounds_total": n_total, "rounds_per_gpu": main["rounds_per_gpu"], "seg_len": args.seg_len,
                   "scheme": args.scheme, "mode": args.mode, "parallelism": f"shard{world}"},
        "stage_ms": main["stage_ms"],
        "verdict_mismatches": main["verdict_mismatches"],
        "corrupted_rounds_total": main["corrupted_rounds_total"],
        "chain_gen_s": main["chain_gen_s"],
        "end_to_end": main.get("end_to_end"),
        "rlc": main.get("rlc"),
        "ingest": main.get("ingest"),
        "small_batch": main.get("small_batch"),
        "roofline": main.get("roofline"),
        "cpu_baseline": main.get("cpu_baseline"),
    }
    out["driver"] = driver_info(world)
    out.update(legs)
    print(json.dumps(out), flush=True)


def driver_info(world):
    """How the run drove the GPUs: one process per GPU over torch.distributed
    (every rank calls the C ABI's per-device entry points; the exchange steps
    -- verdict bitmaps, and in RLC mode the per-rank roots of the
    dgpu_rlc_root_device / dgpu_rlc_finish_device protocol -- over the
    process group), with the world size the process group initialised."""
    info = {"name": "dist", "api": "dgpu_verify_beacons_device per rank; RLC: dgpu_rlc_root_device + all-gather of "
                                   "roots + dgpu_rlc_finish_device", "ranks": world}
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            info.update(rccl_world_size=dist.get_world_size(), backend=str(dist.get_backend()))
    except Exception:  # reported, never fatal
        pass
    return info


def main_recover(args, world, rank, local):
    res = recover_leg(args, world, rank, local, args.rounds or 100_000, args.steps, args.warmup, args.cpu_seconds)
    if rank == 0:
        res["vs_baseline"] = None
        print(json.dumps(res), flush=True)


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
    if args.driver == "abi":  # one process: the library shards over the devices itself
        world = args.gpus
        got = [{"device": k, "shard": shard_range(n_total, world, k)} for k in range(world)]
    elif world > 1:
        dist.init_process_group("gloo")
        got = [None] * world
        dist.all_gather_object(got, me)
        dist.destroy_process_group()
    else:
        got = [me]
    if rank == 0:
        driver = ("abi: one process, dgpu_verify_multi over %d devices" % args.gpus if args.driver == "abi" else
                  "dist: %d rank processes over torch.distributed (nccl = RCCL on GPUs), dgpu_verify_beacons_device "
                  "per rank, RLC roots via dgpu_rlc_root_device / dgpu_rlc_finish_device" % world)
        print(json.dumps({"dryrun": True, "driver": args.driver, "driver_detail": driver, "n_gpus": world,
                          "rounds_total": n_total, "ranks": got}), flush=True)


def main():
    args = parse()
    if args.dry_run:
        os.environ["DRAND_BENCH_DRYRUN"] = "1"
        if args.driver == "abi":
            return dryrun(args)
    if args.abi_child or (args.driver == "abi" and "WORLD_SIZE" not in os.environ):
        # one process over all GPUs (never under a rank launcher)
        res = main_abi(args)
        if not args.abi_child:
            res.update({"metric": "verified beacon rounds/sec through dgpu_verify_multi", "higher_is_better": True,
                        "scaling": "strong", "vs_baseline": None})
        print(json.dumps(res), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.small_batch_only:
        from drand_amd import _lib
        from drand_amd.synth import corrupt, make_chain
        code = _lib.load().dgpu_scheme_from_name(args.scheme.encode())
        sizes = tuple(int(x) for x in args.small_batch_sizes.split(",")) if args.small_batch_sizes else SMALL_BATCH_SIZES
        ch = make_chain(args.seed, max(max(sizes), 8), code, seg_len=args.seg_len)  # >= 8 for the CPU sample
        corrupt(ch, args.seed, rate=args.corrupt_rate)
        print(json.dumps(small_batch_leg(ch, args.scheme, sizes=sizes)), flush=True)
        return
    if args.ingest_only:
        from drand_amd import _lib
        from drand_amd.synth import corrupt, make_chain
        code = _lib.load().dgpu_scheme_from_name(args.scheme.encode())
        ch = make_chain(args.seed, args.ingest_rounds, code, seg_len=args.seg_len)
        _EXPECT[id(ch)] = {i: False for i in corrupt(ch, args.seed, rate=args.corrupt_rate)}
        ws = [int(x) for x in args.ingest_windows.split(",")]
        print(json.dumps(ingest_leg(ch, args.ingest_rounds, args.scheme, window=ws[0], windows=ws)), flush=True)
        return
    if os.environ.get("DRAND_BENCH_DRYRUN"):
        return dryrun(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DRAND_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # devices round-robin; collectives over gloo on the CPU); the default is
    # one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("DRAND_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
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
