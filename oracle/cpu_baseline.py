"""cpu_baseline leg of bench.py (TEST INFRASTRUCTURE: the oracle timed on the
host cores as a reported baseline, never the measured product).

Verifies a bounded random sample of the bench's own chain with the C
restatement (oracle/c, pthreads) -- or the pure-Python oracle in a process
pool if the C build is unavailable -- checks the sample's verdicts against
the chain's construction, and reports rounds/s.
"""
import os
import time

import numpy as np


SCHEME_BY_CODE = {0: "pedersen-bls-chained", 1: "pedersen-bls-unchained", 2: "bls-unchained-on-g1",
                  3: "bls-unchained-g1-rfc9380"}


def host_cores():
    """The box's CPU view, stated with every baseline: all host cores
    (os.cpu_count), the cores this process may run on (sched_getaffinity),
    and the cgroup CPU quota when one is set (cpu.max, in cores)."""
    info = {"host_cores": os.cpu_count(), "affinity_cores": len(os.sched_getaffinity(0))}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            info["cgroup_quota_cores"] = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return info


def quota_threads(info):
    """Threads that match the CPU time the box actually grants (the cgroup
    quota), when that is below the affinity count."""
    q = info.get("cgroup_quota_cores")
    return max(1, min(info["affinity_cores"], int(q))) if q else info["affinity_cores"]


def _quota_and_projection(out, run_k, seconds, rate_hint):
    """Beside the all-affinity-threads figure: (a) the same sample size run on
    quota_threads threads when a cgroup quota caps the box below its
    affinity count (oversubscribed threads only add switching), and (b) the
    single-core rate times every host core -- the ideal-scaling upper bound of
    the reference's verifier with GOMAXPROCS = the host core count."""
    out["projected_all_host_cores_value"] = out["single_core_value"] * out["host_cores"]
    qt = quota_threads(out)
    if qt >= out["threads"]:
        return
    k = int(max(qt, seconds / 2 * rate_hint))
    _, wall, cpu_s = _timed(lambda: run_k(k))
    out["quota_threads"] = {"threads": qt, "value": k / wall, "wall_s": wall, "effective_parallelism": cpu_s / wall}


def _label_cores(out, threads):
    """`cores` is the parallelism the run measurably got (CPU seconds / wall:
    ~15.9 under the GPU box's 16-core cgroup quota, whatever the thread
    count); the threads started and the host / affinity / quota views are
    kept beside it."""
    out["threads"] = threads
    out["cores"] = round(out["effective_parallelism"], 2)


def _timed(fn):
    """wall and process CPU seconds (all threads) of fn()"""
    c0, t0 = time.process_time(), time.perf_counter()
    out = fn()
    return out, time.perf_counter() - t0, time.process_time() - c0


def sample_size(n, seconds, cores, per_round_1core, calib_rate=None):
    """Rounds for ~`seconds` of wall time: from a measured parallel rate when
    there is one (quota-limited boxes run fewer cores than threads), capped
    at the cgroup quota's rate -- a sub-second calibration burst runs above
    the quota before the throttle engages (r06: a 12 s budget ran 48 s)."""
    rate = calib_rate if calib_rate else cores / max(per_round_1core, 1e-6)
    q = host_cores().get("cgroup_quota_cores")
    if q:
        rate = min(rate, q / max(per_round_1core, 1e-6))
    return int(max(cores, min(n, seconds * rate)))


def run(chain, seconds, cores, expect_valid=None):
    """`cores` threads of the C restatement over a bounded uniform sample of
    the chain: calibrated single-threaded (the reference's bulk loop is one
    goroutine, chain/beacon/sync_manager.go:188) and on all threads, then
    timed; reports wall rate, CPU seconds used and the effective parallelism."""
    n = len(chain)
    chained = chain.scheme_code == 0
    on_g1 = chain.scheme_code >= 2
    try:
        from oracle import c_ref
        c_ref.load()
        if on_g1:  # bls-unchained-on-g1 (G2 suite's DST) / bls-unchained-g1-rfc9380 (G1 DST)
            rfc = chain.scheme_code == 3
            impl = ("oracle/c/bls381_ref.c (C restatement, 6x64-bit limbs: RFC 9380 hash to G1, [r]P subgroup test, "
                    "e(H, pk) e(-sig, g2))")
            verify = lambda sub, thr: c_ref.verify_batch_g1(rfc, chain.pk, sub[0], sub[1], sub[2], thr)  # noqa: E731
        else:
            impl = "oracle/c/bls381_ref.c (C restatement, 6x64-bit limbs, [r]Q subgroup test as kilic (R))"
            verify = lambda sub, thr: c_ref.verify_batch(chained, chain.pk, *sub, thr)  # noqa: E731
        cols = (chain.rounds, chain.sigs, chain.sig_len, chain.prev, chain.prev_len)
        rng = np.random.default_rng(12345)
        pick = lambda k: np.sort(rng.choice(n, size=min(n, k), replace=False))  # noqa: E731
        sub_of = lambda idx: [np.ascontiguousarray(a[idx]) for a in cols]  # noqa: E731
        # single-threaded calibration, then a short all-threads calibration
        idx0 = pick(4)
        _, w1, _ = _timed(lambda: verify(sub_of(idx0), 1))
        per = w1 / len(idx0)
        idxc = pick(2 * cores)
        _, wc, _ = _timed(lambda: verify(sub_of(idxc), cores))
        sample = sample_size(n, seconds, cores, per, len(idxc) / max(wc, 1e-6))
        idx = pick(sample)
        sub = sub_of(idx)
        reason, wall, cpu_s = _timed(lambda: verify(sub, cores))
    except Exception as e:  # C build unavailable: pure-Python oracle
        return _run_py(chain, seconds, cores, repr(e))
    out = {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port", "impl": impl,
           "sample": f"{sample} uniformly sampled rounds of the bench chain", "wall_s": wall,
           "cpu_s": cpu_s, "effective_parallelism": cpu_s / wall,
           "single_core_ms_per_round": per * 1e3, "single_core_value": 1.0 / per}
    out.update(host_cores())
    _label_cores(out, cores)
    _quota_and_projection(out, lambda k: verify(sub_of(pick(k)), quota_threads(out)), seconds, sample / wall)
    if expect_valid is not None:
        out["sample_verdict_mismatches"] = int(((reason == 0) != expect_valid[idx]).sum())
    return out


def _verify_py(args):
    from oracle import bls12381 as B
    from oracle import drand_ref as D
    scheme, pk, items = args
    pkp = B.g2_decompress(pk) if scheme in D.SIG_ON_G1_DST else B.g1_decompress(pk)
    return [D.verify_beacon(scheme, pkp, r, prev, sig) for r, prev, sig in items]


def _run_py(chain, seconds, cores, why, expect_valid=None):
    from concurrent.futures import ProcessPoolExecutor
    n = len(chain)
    items = lambda idx: [(int(chain.rounds[i]), bytes(chain.prev[i, : chain.prev_len[i]]),  # noqa: E731
                          bytes(chain.sigs[i, : chain.sig_len[i]])) for i in idx]
    scheme = SCHEME_BY_CODE[chain.scheme_code]
    t = time.perf_counter()
    _verify_py((scheme, chain.pk, items([0])))
    per = time.perf_counter() - t
    sample = max(cores, min(n, int(seconds * cores / max(per, 1e-6))))
    idx = sorted(np.random.default_rng(12345).choice(n, size=sample, replace=False).tolist())
    chunks = [idx[k::cores] for k in range(cores)]
    t = time.perf_counter()
    with ProcessPoolExecutor(max_workers=cores) as ex:
        got = list(ex.map(_verify_py, [(scheme, chain.pk, items(c)) for c in chunks]))
    wall = time.perf_counter() - t
    out = {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port",
           "impl": f"oracle/bls12381.py (pure Python; C restatement not used: {why})",
           "sample": f"{sample} uniformly sampled rounds of the bench chain", "wall_s": wall,
           "single_core_ms_per_round": per * 1e3}
    if expect_valid is not None:
        mism = sum(int(v != bool(expect_valid[i])) for c, g in zip(chunks, got) for i, v in zip(c, g))
        out["sample_verdict_mismatches"] = mism
    return out


# ---------------------------------------------------------------- configs[4]: threshold recovery
_REC = {}


def _rec_init(commits, t, n):
    from oracle import bls12381 as B
    from oracle import c_ref
    from oracle import drand_ref as D
    c_ref.load(build=False)
    pts = [B.g1_decompress(c) for c in commits]
    _REC.update(t=t, n=n, pts=pts, c0=commits[0],
                evals=[B.g1_compress(D.pub_poly_eval(pts, i)) for i in range(n)])


def _rec_round(args):
    """Recover (kyber tbls.Recover restated in oracle/drand_ref.recover) with
    VerifyPartial on the C restatement, then VerifyRecovered."""
    from oracle import bls12381 as B
    from oracle import c_ref
    from oracle import drand_ref as D
    msg, parts = args
    L = c_ref.load(build=False)

    def verify(i, sig):
        pk = _REC["evals"][i] if i < _REC["n"] else B.g1_compress(D.pub_poly_eval(_REC["pts"], i))
        return L.ref_verify_msg(pk, msg, sig, len(sig)) == 0

    sig = D.recover(_REC["pts"], msg, parts, _REC["t"], _REC["n"], verify=verify)
    if sig is not None and L.ref_verify_msg(_REC["c0"], msg, sig, len(sig)) != 0:
        sig = None
    return sig


def run_recover(commits, t, n, msgs, parts, expect_sigs, seconds, cores):
    """Bounded sample of the bench's recovery batch on `cores` threads of the
    C restatement (oracle/c ref_recover: t VerifyPartial pairings, Lagrange in
    Fr, G2 MSM, VerifyRecovered), checked against the expected recovered
    signatures (None = failure).  Falls back to the Python Lagrange/MSM with
    C pairings if the C recovery is unavailable."""
    nr = len(msgs)
    try:
        from oracle import c_ref
        c_ref.load()
        rng = np.random.default_rng(12345)
        pick = lambda k: np.sort(rng.choice(nr, size=min(nr, k), replace=False))  # noqa: E731
        run_idx = lambda idx, thr: c_ref.recover_batch(  # noqa: E731
            commits, t, np.ascontiguousarray(msgs[idx]), np.ascontiguousarray(parts[idx]), thr)
        _, w1, _ = _timed(lambda: run_idx(pick(1), 1))
        idxc = pick(cores)
        _, wc, _ = _timed(lambda: run_idx(idxc, cores))
        sample = sample_size(nr, seconds, cores, w1, len(idxc) / max(wc, 1e-6))
        idx = pick(sample)
        (sigs, ok), wall, cpu_s = _timed(lambda: run_idx(idx, cores))
        mism = sum(1 for k, i in enumerate(idx) if (bytes(sigs[k]) if ok[k] else None) != expect_sigs[i])
        out = {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port",
               "impl": "oracle/c/bls381_ref.c ref_recover (C restatement of kyber tbls.Recover (R): VerifyPartial x t, "
                       "Lagrange in Fr, G2 MSM, VerifyRecovered)",
               "sample": f"{sample} uniformly sampled rounds of the bench batch", "wall_s": wall, "cpu_s": cpu_s,
               "effective_parallelism": cpu_s / wall, "single_core_ms_per_round": w1 * 1e3,
               "single_core_value": 1.0 / w1, "sample_mismatches": mism}
        out.update(host_cores())
        _label_cores(out, cores)
        _quota_and_projection(out, lambda k: run_idx(pick(k), quota_threads(out)), seconds, sample / wall)
        return out
    except (OSError, AttributeError):
        return _run_recover_py(commits, t, n, msgs, parts, expect_sigs, seconds, cores)


def _run_recover_py(commits, t, n, msgs, parts, expect_sigs, seconds, cores):
    """Python selection / Lagrange / MSM with C pairings (fallback)."""
    from concurrent.futures import ProcessPoolExecutor
    nr = len(msgs)
    _rec_init(commits, t, n)
    job = lambda i: (bytes(msgs[i]), [bytes(p) for p in parts[i]])  # noqa: E731
    t0 = time.perf_counter()
    _rec_round(job(0))
    per = time.perf_counter() - t0
    sample = int(max(cores, min(nr, seconds * cores / max(per, 1e-6))))
    idx = sorted(np.random.default_rng(12345).choice(nr, size=sample, replace=False).tolist())
    t0 = time.perf_counter()
    with ProcessPoolExecutor(max_workers=cores, initializer=_rec_init, initargs=(commits, t, n)) as ex:
        got = list(ex.map(_rec_round, [job(i) for i in idx], chunksize=max(1, sample // (4 * cores))))
    wall = time.perf_counter() - t0
    mism = sum(1 for i, g in zip(idx, got) if g != expect_sigs[i])
    return {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port",
            "impl": "oracle/drand_ref.recover (Python: selection, Lagrange, G2 MSM) + oracle/c pairings "
                    "(VerifyPartial, VerifyRecovered)",
            "sample": f"{sample} uniformly sampled rounds of the bench batch", "wall_s": wall,
            "single_core_ms_per_round": per * 1e3, "sample_mismatches": mism}
