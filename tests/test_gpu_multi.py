"""The multi-GPU product entry points (dgpu_verify_multi, dgpu_recover_multi;
include/drand_gpu.h) with D = 2 and 3 contexts on one GPU
(DGPU_MULTI_ALLOW_SAME_DEVICE=1: the all-gathers become in-library device
copies, every other line is the production D >= 2 path -- per-device RLC
seeds, the root all-gather + sum + single check on the first context, the
descent on each device when the node root fails, short and empty shard
padding, the grouped bitmap / reason gathers).  Verdicts, reasons and
recovered signatures must equal the single-context calls and the
construction.  The bulk caller is chain/beacon/sync_manager.go:188-222, the
aggregator chain/beacon/chain.go:158-168.  Marked gpu."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sch(name="pedersen-bls-chained"):
    from drand_amd.scheme import get_scheme_by_id_with_default
    return get_scheme_by_id_with_default(name)


@pytest.fixture(scope="module")
def chain5003():
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(61, 5003, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 61, rate=2e-3)
    beacons = [c.beacon(i) for i in range(len(c))]
    single = Verifier(_sch()).verify_reasons(beacons, c.pk)
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(single == 0, expect)
    return c, bad, beacons, single


@pytest.mark.parametrize("ndev", [2, 3])
def test_verify_multi_same_device_equals_single(ndev, chain5003, monkeypatch):
    from drand_amd import _lib
    from drand_amd.multi import MultiVerifier
    c, bad, beacons, single = chain5003
    monkeypatch.setenv("DGPU_MULTI_ALLOW_SAME_DEVICE", "1")
    mv = MultiVerifier(_sch(), [0] * ndev)
    try:
        lo_hi = [_lib.shard_range(len(c), ndev, k) for k in range(ndev)]
        assert lo_hi[-1][1] - lo_hi[-1][0] < lo_hi[0][1] - lo_hi[0][0]  # a short last shard
        for mode in (_lib.MODE_PER_ROUND, _lib.MODE_RLC):
            got = mv.verify_reasons(beacons, c.pk, mode, rlc_seed=12345)
            assert got.tolist() == single.tolist(), mode
            # clean batch: RLC passes with the node root (sum of the device roots) alone
            clean = [b for i, b in enumerate(beacons[:1500]) if i not in bad]
            assert not mv.verify_reasons(clean, c.pk, mode).any()
            # an empty last shard: 8 (D - 1) rounds -> shards of 8, the last one empty
            n_e = 8 * (ndev - 1)
            assert _lib.shard_range(n_e, ndev, ndev - 1) == (n_e, n_e)
            assert mv.verify_reasons(beacons[:n_e], c.pk, mode).tolist() == single[:n_e].tolist()
            # a batch smaller than one shard
            assert mv.verify_reasons(beacons[3:8], c.pk, mode).tolist() == single[3:8].tolist()
    finally:
        mv.close()


def test_verify_multi_same_device_unchained_and_on_g1(monkeypatch):
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.multi import MultiVerifier
    from drand_amd.synth import corrupt, make_chain
    monkeypatch.setenv("DGPU_MULTI_ALLOW_SAME_DEVICE", "1")
    for name, code in (("pedersen-bls-unchained", _lib.SCHEME_UNCHAINED),
                       ("bls-unchained-on-g1", _lib.SCHEME_UNCHAINED_G1),
                       ("bls-unchained-g1-rfc9380", _lib.SCHEME_G1_RFC9380)):
        c = make_chain(62, 997, code, seg_len=64)
        corrupt(c, 62, rate=5e-3)
        beacons = [c.beacon(i) for i in range(len(c))]
        single = Verifier(_sch(name)).verify_reasons(beacons, c.pk)
        mv = MultiVerifier(_sch(name), [0, 0])
        try:
            assert mv.verify_reasons(beacons, c.pk).tolist() == single.tolist(), name
            # RLC at D = 2: per-device roots (G2 or G1 Jacobian sums) gathered and
            # summed on device 0; descent per shard when the node fails
            assert mv.verify_reasons(beacons, c.pk, _lib.MODE_RLC).tolist() == single.tolist(), name
            clean = [b for b, r in zip(beacons, single) if r == 0]
            assert not mv.verify_reasons(clean, c.pk, _lib.MODE_RLC).any(), name
        finally:
            mv.close()


@pytest.mark.parametrize("ndev", [2, 3])
def test_recover_multi_same_device_equals_single(ndev, monkeypatch):
    from conftest import load_golden
    from drand_amd.multi import MultiThresholdGroup
    from drand_amd.threshold import ThresholdGroup
    monkeypatch.setenv("DGPU_MULTI_ALLOW_SAME_DEVICE", "1")
    g = load_golden("recover_t17_n32.json")
    commits = [bytes.fromhex(x) for x in g["commits"]]
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]] * 5   # 30 rounds: D=2 shards 16 + 14, D=3 16 + 14 + empty
    parts = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]] * 5
    single = ThresholdGroup(commits, g["n"]).recover_batch(msgs, parts)
    mg = MultiThresholdGroup(commits, g["n"], [0] * ndev)
    try:
        got = mg.recover_batch(msgs, parts)
    finally:
        mg.close()
    ThresholdGroup._active = None
    assert got == single
    assert [s.hex() if s else None for s in got[0]] == [c["recovered"] for c in g["cases"]] * 5
