"""Threshold recovery (kyber tbls.Recover (R), chain/beacon/chain.go:158-168).

CPU: the oracle's restatement against the reference's own round-trip pin
(chain/beacon/node_test.go:88-105: a signature recovered from t partials is
the group secret's signature and verifies under the group key) on the
committed fixtures, and the partial-index rule.  GPU: the batch C-ABI call
reproduces every fixture bit-exactly (recovered bytes, failure verdicts,
per-partial validity)."""
import struct

import pytest

from conftest import load_golden
from oracle import bls12381 as B
from oracle import drand_ref as D

# t = 3, 12, 17, 32: every MSM table bucket of k_recover_msm_w4 (TMAX 8 / 16 / 24 / 32)
FIXTURES = ["recover_t3_n8.json", "recover_t12_n20.json", "recover_t17_n32.json", "recover_t32_n40.json"]


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_recovered_is_group_signature(name):
    g = load_golden(name)
    sk = D.share_poly(g["seed"], g["t"])[0]
    assert [bytes.fromhex(c) for c in g["commits"]] == D.pub_poly_commits(D.share_poly(g["seed"], g["t"]))
    kinds = {c["kind"]: c for c in g["cases"]}
    assert kinds["exact_t"]["recovered"] and kinds["one_bad_short"]["recovered"] is None
    assert kinds["duplicate_index"]["recovered"] is None  # kyber stops at t good, duplicates count once
    for c in g["cases"]:
        if c["recovered"] is not None:
            assert bytes.fromhex(c["recovered"]) == B.sign_g2(sk, bytes.fromhex(c["msg"]))


def test_oracle_recover_small_group_real_verification():
    """The oracle's full path (with pairings) on one small fixture case."""
    g = load_golden("recover_t3_n8.json")
    cpts = [B.g1_decompress(bytes.fromhex(c)) for c in g["commits"]]
    c = next(x for x in g["cases"] if x["kind"] == "three_bad_enough")
    parts = [bytes.fromhex(p) for p in c["partials"]]
    got = D.recover(cpts, bytes.fromhex(c["msg"]), parts, g["t"], g["n"])
    assert got.hex() == c["recovered"]


def test_index_of():
    from drand_amd.threshold import index_of
    assert index_of(b"") == -1 and index_of(b"\x01") == -1
    assert index_of(struct.pack(">H", 513) + b"x") == 513


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_recover_matches_fixtures(name):
    from drand_amd.threshold import ThresholdGroup
    g = load_golden(name)
    grp = ThresholdGroup([bytes.fromhex(c) for c in g["commits"]], g["n"])
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    parts = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
    sigs, valid = grp.recover_batch(msgs, parts)
    for c, s, v in zip(g["cases"], sigs, valid):
        assert v == c["valid"], c["kind"]
        assert (s.hex() if s else None) == c["recovered"], c["kind"]


@pytest.mark.gpu
def test_gpu_recover_stage_count_within_max_stages():
    """The recovery pipeline records the most stages of any call (hash,
    decode, engine stages, MSM, verdicts): dgpu_stage_times' count (the
    count needed) stays within DGPU_MAX_STAGES (_lib.stage_times asserts it)."""
    from drand_amd import _lib
    from drand_amd.threshold import ThresholdGroup
    g = load_golden("recover_t17_n32.json")
    grp = ThresholdGroup([bytes.fromhex(c) for c in g["commits"]], g["n"])
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    parts = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
    lib = grp.ctx.lib
    _lib.check(lib.dgpu_set_profiling(grp.ctx.handle, 1))
    try:
        grp.recover_batch(msgs, parts)
        st = _lib.stage_times(grp.ctx)
    finally:
        _lib.check(lib.dgpu_set_profiling(grp.ctx.handle, 0))
    assert 8 < len(st) <= _lib.MAX_STAGES, st


@pytest.mark.gpu
def test_gpu_recover_many_rounds_property():
    """Size-independent property at a larger batch: every round with >= t good
    partials recovers the group signature (sk * H(msg)); rounds with t - 1
    good fail."""
    import hashlib
    import random
    from drand_amd.threshold import ThresholdGroup
    t, n, seed = 5, 9, 11
    co = D.share_poly(seed, t)
    grp = ThresholdGroup(D.pub_poly_commits(co), n)
    rng = random.Random(3)
    msgs, parts, expect = [], [], []
    for r in range(24):
        m = hashlib.sha256(b"round" + bytes([r])).digest()
        k = t if r % 3 else t - 1
        idx = rng.sample(range(n), k)
        msgs.append(m)
        parts.append([D.partial_sign(i, D.poly_eval(co, i + 1), m) for i in idx])
        expect.append(B.sign_g2(co[0], m) if k >= t else None)
    sigs, _ = grp.recover_batch(msgs, parts)
    assert sigs == expect


def test_synth_group_matches_oracle_poly():
    """The bench's synthetic group (drand_amd.synth) uses the oracle's
    coefficient derivation, so fixtures and bench batches share one group."""
    from drand_amd import synth
    assert synth.share_coeffs(5, 4) == D.share_poly(5, 4)
    co = D.share_poly(5, 4)
    assert [synth.poly_eval(co, x) for x in (1, 7, 33)] == [D.poly_eval(co, x) for x in (1, 7, 33)]


@pytest.mark.gpu
def test_gpu_synthetic_partials_match_oracle():
    """dgpu_make_partials (bench data tool) == tbls.Sign restated in the oracle;
    group_signatures == bls.Sign with the group secret; commitments derived on
    the GPU == the oracle's."""
    import hashlib
    import numpy as np
    from drand_amd import synth
    grp = synth.make_group(9, 3, 5)
    co = D.share_poly(9, 3)
    assert grp.commits == D.pub_poly_commits(co)
    msgs = np.stack([np.frombuffer(hashlib.sha256(bytes([k])).digest(), dtype=np.uint8) for k in range(2)])
    idx = np.array([[0, 4, 2], [3, 1, 0]], dtype=np.uint32)
    lab = idx.copy()
    lab[1, 2] = 2
    parts = synth.sign_partials(grp, msgs, idx, lab)
    for r in range(2):
        for j in range(3):
            sig = B.sign_g2(D.poly_eval(co, int(idx[r, j]) + 1), bytes(msgs[r]))
            assert bytes(parts[r, j]) == struct.pack(">H", int(lab[r, j])) + sig
    gs = synth.group_signatures(grp, msgs)
    assert [bytes(g) for g in gs] == [B.sign_g2(co[0], bytes(m)) for m in msgs]


@pytest.mark.gpu
def test_gpu_recover_device_entry_point_bench_batch():
    """The bench's configs[4] workload at small size through
    dgpu_recover_batch_device: recovered == group signature on rounds with t
    good partials, failure (zeros) on rounds with one invalid partial."""
    import ctypes
    import numpy as np
    import torch
    from drand_amd import _lib, synth
    from drand_amd.chain import get_context
    grp = synth.make_group(4, 5, 8)
    msgs, parts, expect_ok = synth.make_recovery_batch(grp, 96, seed=1, bad_rate=0.25)
    assert 0 < int((~expect_ok).sum()) < 96
    expect = synth.group_signatures(grp, msgs)
    ctx = get_context(0)
    cb = np.frombuffer(b"".join(grp.commits), dtype=np.uint8).copy()
    _lib.check(ctx.lib.dgpu_set_group(ctx.handle, grp.t, grp.n, _lib.ptr(cb)))
    from drand_amd.threshold import ThresholdGroup
    ThresholdGroup._active = None  # group replaced behind ThresholdGroup's cache
    n, m = parts.shape[:2]
    dev = torch.device("cuda", 0)
    d_msgs = torch.from_numpy(msgs).to(dev)
    d_parts = torch.from_numpy(parts.reshape(n * m, 98).copy()).to(dev)
    d_plen = torch.full((n * m,), 98, dtype=torch.int32, device=dev)
    d_out = torch.zeros((n, 96), dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_st = torch.full((n * m,), 0xFF, dtype=torch.uint8, device=dev)
    _lib.check(ctx.lib.dgpu_recover_batch_device(ctx.handle, n, d_msgs.data_ptr(), m, d_parts.data_ptr(), 98,
                                                 d_plen.data_ptr(), d_out.data_ptr(), d_ok.data_ptr(),
                                                 d_st.data_ptr(), ctypes.c_void_p(0)))
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy().astype(bool)
    out = d_out.cpu().numpy()
    st = d_st.cpu().numpy().reshape(n, m)
    assert (ok == expect_ok).all()
    assert (out[ok] == expect[ok]).all() and not out[~ok].any()
    assert ((st != 0).sum(axis=1) == (~expect_ok).astype(int)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_recover_batched_check_matches_fixtures(name):
    """Without per-partial statuses the library checks each round's first t
    decodable partials and the recovered signature with one pairing
    (recover.cuh, batched check) and sends the undecided rounds down the
    exact per-partial path: recovered bytes and failures equal the fixture
    for every case kind (bad partials, duplicates, short ones, index >= n)."""
    from drand_amd.threshold import ThresholdGroup
    g = load_golden(name)
    grp = ThresholdGroup([bytes.fromhex(c) for c in g["commits"]], g["n"])
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    parts = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
    sigs, valid = grp.recover_batch(msgs, parts, statuses=False)
    assert valid is None
    assert [s.hex() if s else None for s in sigs] == [c["recovered"] for c in g["cases"]]


def _cancelling_partials(t=3, n=8, seed=3):
    """Partials whose errors cancel in the Lagrange combination: sig_1 + l_2 D
    and sig_2 - l_1 D (l_j the Lagrange coefficients of the chosen indices),
    so sum_j l_j sig_j is still the group signature, yet both partials fail
    VerifyPartial and the reference (chain/beacon/chain.go:160 -> Recover)
    skips them."""
    import hashlib
    co = D.share_poly(seed, t)
    msg = hashlib.sha256(b"drand-mi355x/cancel").digest()
    idx = [1, 4, 6, 2, 7]
    parts = [D.partial_sign(i, D.poly_eval(co, i + 1), msg) for i in idx]
    lam = D.lagrange_at_zero([i + 1 for i in idx[:t]])
    Dp = B.g2_mul(B.G2_GEN, 0x1234567)
    s1 = B.g2_add(B.g2_decompress(parts[0][2:]), B.g2_mul(Dp, lam[1]))
    s2 = B.g2_add(B.g2_decompress(parts[1][2:]), B.g2_neg(B.g2_mul(Dp, lam[0])))
    parts[0] = parts[0][:2] + B.g2_compress(s1)
    parts[1] = parts[1][:2] + B.g2_compress(s2)
    return co, msg, parts


def test_cancelling_partials_fail_the_reference():
    """CPU: the crafted set recovers the group signature under plain
    interpolation, but the reference's walk rejects both bad partials."""
    co, msg, parts = _cancelling_partials()
    cpts = [B.g1_decompress(c) for c in D.pub_poly_commits(co)]
    sig = B.sign_g2(co[0], msg)
    lam = D.lagrange_at_zero([struct.unpack(">H", p[:2])[0] + 1 for p in parts[:3]])
    acc = None
    for lj, p in zip(lam, parts[:3]):
        acc = B.g2_add(acc, B.g2_mul(B.g2_decompress(p[2:]), lj))
    assert B.g2_compress(acc) == sig                      # the errors cancel
    assert D.recover(cpts, msg, parts[:3], 3, 8) is None  # yet the reference fails the round
    assert D.recover(cpts, msg, parts, 3, 8) == sig       # and recovers from the three good ones


@pytest.mark.gpu
def test_gpu_recover_cancelling_partials_rejected():
    """GPU, batched check: the random coefficients expose the cancelling
    errors (the round with only these three partials fails like the
    reference); with two more good partials the round recovers through the
    exact path; per-partial statuses mark exactly the two crafted ones."""
    from drand_amd.threshold import ThresholdGroup
    co, msg, parts = _cancelling_partials()
    grp = ThresholdGroup(D.pub_poly_commits(co), 8)
    sig = B.sign_g2(co[0], msg)
    for _ in range(3):  # fresh coefficients per call
        got, _ = grp.recover_batch([msg, msg], [parts[:3], parts], statuses=False)
        assert got == [None, sig]
    got, valid = grp.recover_batch([msg, msg], [parts[:3], parts], statuses=True)
    assert got == [None, sig]
    assert valid == [[False, False, True], [False, False, True, True, True]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("statuses", [True, False])
def test_gpu_recover_generic_redo_paths_match_fixtures(name, statuses):
    """The fast group-law paths' generic redo, forced on every item (A/B
    build test hook DGPU_TEST_FORCE_EXC=1): the partials' membership test
    (g2_in_subgroup in place of the ladder) and the recovery MSM's windows
    (the generic mixed addition redoing each slice) -- recovered bytes and
    failures equal the fixture, per-partial statuses and batched check."""
    from conftest import open_ctx
    from drand_amd import _lib
    from drand_amd.threshold import pack_partials, unpack_recovered
    import numpy as np
    g = load_golden(name)
    commits = [bytes.fromhex(c) for c in g["commits"]]
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    parts = [[bytes.fromhex(p) for p in c["partials"]] for c in g["cases"]]
    ctx = open_ctx({"DGPU_TEST_FORCE_EXC": "1"})
    try:
        buf = np.frombuffer(b"".join(commits), dtype=np.uint8).copy()
        _lib.check(ctx.lib.dgpu_set_group(ctx.handle, len(commits), g["n"], _lib.ptr(buf)))
        mb, pb, plen, m, stride = pack_partials(msgs, parts)
        nr = len(msgs)
        out = np.zeros(nr * 96, dtype=np.uint8)
        ok = np.zeros((nr + 7) // 8, dtype=np.uint8)
        pv = np.zeros(nr * m, dtype=np.uint8) if statuses else None
        _lib.check(ctx.lib.dgpu_recover_batch(ctx.handle, nr, _lib.ptr(mb), m, _lib.ptr(pb), stride, _lib.ptr(plen),
                                              _lib.ptr(out), _lib.ptr(ok), _lib.ptr(pv)))
        sigs, valid = unpack_recovered(out, ok, pv, parts, m)
    finally:
        ctx.close()
    assert [s.hex() if s else None for s in sigs] == [c["recovered"] for c in g["cases"]]
    if statuses:
        assert [v for v in valid] == [c["valid"] for c in g["cases"]]
