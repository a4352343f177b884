"""cpu_baseline leg of bench.py (TEST INFRASTRUCTURE: the oracle timed on the
host cores as a reported baseline, never the measured product).

Verifies a bounded sample of the bench's own chain with the CPU oracle in a
process pool, checks the sample's verdicts against construction, and reports
rounds/s.  Uses the C restatement (oracle/c, built into oracle/build) when
present, else the pure-Python oracle.
"""
import os
import time
from concurrent.futures import ProcessPoolExecutor


def _verify_py(args):
    from oracle import bls12381 as B
    from oracle import drand_ref as D
    pk, items = args
    pkp = B.g1_decompress(pk)
    return [D.verify_beacon(D.SCHEME_CHAINED, pkp, r, prev, sig) for r, prev, sig in items]


def _items(chain, idx):
    return [(int(chain.rounds[i]), bytes(chain.prev[i, : chain.prev_len[i]]), bytes(chain.sigs[i, : chain.sig_len[i]]))
            for i in idx]


def run(chain, seconds, cores):
    import numpy as np
    n = len(chain)
    # calibrate on one round, then size the sample to ~`seconds` of CPU work
    t = time.perf_counter()
    _verify_py((chain.pk, _items(chain, [0])))
    per = time.perf_counter() - t
    sample = max(cores, min(n, int(seconds * cores / max(per, 1e-6))))
    rng = np.random.default_rng(12345)
    idx = sorted(rng.choice(n, size=sample, replace=False).tolist())
    chunks = [idx[k::cores] for k in range(cores)]
    t = time.perf_counter()
    with ProcessPoolExecutor(max_workers=cores) as ex:
        res = list(ex.map(_verify_py, [(chain.pk, _items(chain, c)) for c in chunks]))
    wall = time.perf_counter() - t
    verdicts = {}
    for c, r in zip(chunks, res):
        verdicts.update(dict(zip(c, r)))
    return {"value": sample / wall, "unit": "rounds/s", "cores": cores, "kind": "port",
            "impl": "oracle/bls12381.py (pure Python)", "sample": f"{sample} rounds of the bench chain (uniform)",
            "sample_verdicts_valid": int(sum(verdicts.values())), "wall_s": wall}
