"""The shipped kernel-selection thresholds: tests/conftest.py
sets DGPU_THR_MIN=0, DGPU_RLC_MIN=0, DGPU_COF_ENGINE_MAX=0 and DGPU_FE_GS_MAX=0
for the suite so that its small batches run the per-thread kernels, the RLC
pipeline, k_h2c_finish and the Karabina FE the bulk path uses.
These tests open fresh contexts at the library's defaults instead
(DGPU_THR_MIN=65536: pairing chunks under 64Ki items on the 12-lane lines and
8-lane chain; DGPU_RLC_MIN=131072: smaller RLC-mode calls on the per-round
path; DGPU_COF_ENGINE_MAX=16384 / DGPU_FE_GS_MAX=16384: small calls clear the
hash cofactor on the engine ladder and take the Granger-Scott FE) for the pipelines the chained-G2 default tests in test_gpu_parity.py
do not cover: G1 signatures per round and in RLC mode (a call above the RLC
threshold, so the combination runs with its node checks on the lane
kernels), and threshold recovery.  Verdicts equal the construction / golden
fixtures.  Marked gpu.

Tests elsewhere that pin the defaults: test_gpu_parity.py
test_small_batches_on_lane_kernels, test_rlc_small_batches_take_per_round_path,
test_rlc_node_checks_on_either_kernel_family."""
import contextlib

import numpy as np
import pytest

from conftest import load_golden, open_ctx

pytestmark = pytest.mark.gpu

DEFAULTS = {"DGPU_THR_MIN": "65536", "DGPU_RLC_MIN": "131072", "DGPU_COF_ENGINE_MAX": "16384",
            "DGPU_FE_GS_MAX": "16384"}


@contextlib.contextmanager
def _default_ctx(extra=None):
    from drand_amd import _lib
    ctx = open_ctx(dict(DEFAULTS, **(extra or {})))
    try:
        yield ctx
    finally:
        ctx.close()


def _verify(ctx, code, c, mode, seed=777):
    from drand_amd import _lib
    n = len(c)
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    reason = np.zeros(n, dtype=np.uint8)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    _lib.check(ctx.lib.dgpu_verify_beacons(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(c.rounds),
                                           _lib.ptr(c.sigs), c.sigs.shape[1], _lib.ptr(c.sig_len), _lib.ptr(c.prev),
                                           c.prev.shape[1], _lib.ptr(c.prev_len), mode, seed, _lib.ptr(bits),
                                           _lib.ptr(reason)))
    assert np.array_equal(np.unpackbits(bits, bitorder="little")[:n].astype(bool), reason == 0)
    return reason


@pytest.mark.parametrize("code_name", ["SCHEME_UNCHAINED_G1", "SCHEME_G1_RFC9380"])
def test_g1_per_round_and_small_rlc_at_defaults(code_name):
    """5,003-round G1 chains, 1% corrupted: per-round mode (lane kernels under
    64Ki) and RLC mode under 128Ki rounds (the per-round path) give the same
    reasons, equal to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    code = getattr(_lib, code_name)
    c = make_chain(91, 5003, code, seg_len=64)
    bad = corrupt(c, 91, rate=1e-2)
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    with _default_ctx() as ctx:
        per = _verify(ctx, code, c, _lib.MODE_PER_ROUND)
        rlc = _verify(ctx, code, c, _lib.MODE_RLC)
    assert np.array_equal(per == 0, expect)
    assert rlc.tolist() == per.tolist()


def test_g1_rlc_above_threshold_at_defaults():
    """A 140,000-round bls-unchained-on-g1 chain (above DGPU_RLC_MIN) in RLC
    mode at the defaults: bucket-MSM root, plain-sum localization with node
    checks under 64Ki items on the lane kernels, confirmation -- verdicts
    equal the construction and per-round mode."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    code = _lib.SCHEME_UNCHAINED_G1
    c = make_chain(93, 140000, code, seg_len=64)
    bad = corrupt(c, 93, rate=2e-4)
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    with _default_ctx() as ctx:
        rlc = _verify(ctx, code, c, _lib.MODE_RLC)
        per = _verify(ctx, code, c, _lib.MODE_PER_ROUND)
    assert np.array_equal(rlc == 0, expect)
    assert rlc.tolist() == per.tolist()


@pytest.mark.parametrize("name", ["recover_t3_n8.json", "recover_t17_n32.json"])
def test_recover_at_defaults(name):
    """Threshold recovery on a context at the shipped thresholds (its
    VerifyPartial / VerifyRecovered pairings are small batches, so they run on
    the lane kernels): recovered signatures and per-partial statuses equal the
    golden fixtures."""
    from drand_amd import _lib
    from drand_amd.threshold import pack_partials, unpack_recovered
    g = load_golden(name)
    commits = np.frombuffer(b"".join(bytes.fromhex(x) for x in g["commits"]), dtype=np.uint8).copy()
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    partials = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
    mb, buf, plen, m, stride = pack_partials(msgs, partials)
    nr = len(msgs)
    out = np.zeros(nr * 96, dtype=np.uint8)
    ok = np.zeros((nr + 7) // 8, dtype=np.uint8)
    pv = np.zeros(nr * m, dtype=np.uint8)
    with _default_ctx() as ctx:
        _lib.check(ctx.lib.dgpu_set_group(ctx.handle, len(g["commits"]), g["n"], _lib.ptr(commits)))
        _lib.check(ctx.lib.dgpu_recover_batch(ctx.handle, nr, _lib.ptr(mb), m, _lib.ptr(buf), stride, _lib.ptr(plen),
                                              _lib.ptr(out), _lib.ptr(ok), _lib.ptr(pv)))
    sigs, valid = unpack_recovered(out, ok, pv, partials, m)
    for c, s, v in zip(g["cases"], sigs, valid):
        assert v == c["valid"], c["kind"]
        assert (s.hex() if s else None) == c["recovered"], c["kind"]


@pytest.mark.parametrize("rows", ["0", "1"])
def test_recover_batched_check_table_layouts(rows):
    """The batched recovery check (no per-partial statuses requested) with its
    window tables gathered from SoA planes or from 224-byte rows
    (DGPU_RECOVER_ROWS): recovered signatures equal the t=17-of-32 and
    t=12-of-20 fixtures case by case."""
    from drand_amd import _lib
    from drand_amd.threshold import pack_partials, unpack_recovered
    for name in ("recover_t17_n32.json", "recover_t12_n20.json"):
        g = load_golden(name)
        commits = np.frombuffer(b"".join(bytes.fromhex(x) for x in g["commits"]), dtype=np.uint8).copy()
        msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
        partials = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
        mb, buf, plen, m, stride = pack_partials(msgs, partials)
        nr = len(msgs)
        out = np.zeros(nr * 96, dtype=np.uint8)
        ok = np.zeros((nr + 7) // 8, dtype=np.uint8)
        # the SoA layout is an A/B variant: only the A/B build reads the knob
        with _default_ctx({"DGPU_RECOVER_ROWS": rows} if rows == "0" else None) as ctx:
            _lib.check(ctx.lib.dgpu_set_group(ctx.handle, len(g["commits"]), g["n"], _lib.ptr(commits)))
            _lib.check(ctx.lib.dgpu_recover_batch(ctx.handle, nr, _lib.ptr(mb), m, _lib.ptr(buf), stride,
                                                  _lib.ptr(plen), _lib.ptr(out), _lib.ptr(ok), None))
        sigs, _ = unpack_recovered(out, ok, None, partials, m)
        assert [s.hex() if s else None for s in sigs] == [c["recovered"] for c in g["cases"]], name


@pytest.mark.parametrize("cof_max,fe_max", [("0", "0"), ("16384", "0"), ("0", "16384"), ("16384", "16384")])
@pytest.mark.parametrize("n", [1, 7, 4099])
def test_small_calls_latency_paths(cof_max, fe_max, n):
    """The small-call latency paths, each on and off: per-round calls up to
    DGPU_COF_ENGINE_MAX rounds clear the hash's cofactor on the 12-lane
    ladder (pairing_engine.cuh k_cof_*) instead of k_h2c_finish, and pairing
    calls up to DGPU_FE_GS_MAX items take the Granger-Scott FE instead of the
    Karabina side.  A chained chain with 1% corrupted rounds gives the
    construction's verdicts in every combination."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(97 + n, n, _lib.SCHEME_CHAINED, seg_len=min(64, n))
    bad = corrupt(c, 97, rate=1e-2) if n > 50 else {}
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    with _default_ctx({"DGPU_COF_ENGINE_MAX": cof_max, "DGPU_FE_GS_MAX": fe_max}) as ctx:
        per = _verify(ctx, _lib.SCHEME_CHAINED, c, _lib.MODE_PER_ROUND)
    assert np.array_equal(per == 0, expect)
