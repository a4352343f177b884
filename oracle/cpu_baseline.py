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


def run(chain, seconds, cores, expect_valid=None):
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
        # calibrate on a few rounds single-threaded
        idx0 = np.arange(min(4, n))
        t = time.perf_counter()
        verify([np.ascontiguousarray(a[idx0]) for a in cols], 1)
        per = (time.perf_counter() - t) / len(idx0)
        sample = int(max(cores, min(n, seconds * cores / max(per, 1e-6))))
        rng = np.random.default_rng(12345)
        idx = np.sort(rng.choice(n, size=sample, replace=False))
        sub = [np.ascontiguousarray(a[idx]) for a in cols]
        t = time.perf_counter()
        reason = verify(sub, cores)
        wall = time.perf_counter() - t
    except Exception as e:  # C build unavailable: pure-Python oracle
        return _run_py(chain, seconds, cores, repr(e))
    out = {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port", "impl": impl,
           "sample": f"{sample} uniformly sampled rounds of the bench chain", "wall_s": wall,
           "single_core_ms_per_round": per * 1e3}
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
        t0 = time.perf_counter()
        c_ref.recover_batch(commits, t, msgs[:1], parts[:1], 1)
        per = time.perf_counter() - t0
        sample = int(max(cores, min(nr, seconds * cores / max(per, 1e-6))))
        idx = np.sort(np.random.default_rng(12345).choice(nr, size=sample, replace=False))
        t0 = time.perf_counter()
        sigs, ok = c_ref.recover_batch(commits, t, np.ascontiguousarray(msgs[idx]), np.ascontiguousarray(parts[idx]),
                                       cores)
        wall = time.perf_counter() - t0
        mism = sum(1 for k, i in enumerate(idx) if (bytes(sigs[k]) if ok[k] else None) != expect_sigs[i])
        return {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port",
                "impl": "oracle/c/bls381_ref.c ref_recover (C restatement of kyber tbls.Recover (R): VerifyPartial x t, "
                        "Lagrange in Fr, G2 MSM, VerifyRecovered)",
                "sample": f"{sample} uniformly sampled rounds of the bench batch", "wall_s": wall,
                "single_core_ms_per_round": per * 1e3, "sample_mismatches": mism}
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
