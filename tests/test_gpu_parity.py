"""GPU parity: the HIP path through the C-ABI against the oracle and the
committed golden fixtures (bit-exact), plus size-independent properties at
larger sizes.  Marked gpu."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden, open_ctx
from oracle import bls12381 as B
from oracle import drand_ref as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def chained():
    from drand_amd.chain import Verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    return Verifier(get_scheme_by_id_with_default("pedersen-bls-chained"))


@pytest.fixture(scope="module")
def unchained():
    from drand_amd.chain import Verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    return Verifier(get_scheme_by_id_with_default("pedersen-bls-unchained"))


def test_hash_to_g2_golden(gpu_ctx):
    from drand_amd.chain import hash_to_g2
    cases = load_golden("hash_to_g2.json")["cases"]
    out = hash_to_g2([bytes.fromhex(c["msg"]) for c in cases])
    assert [o.hex() for o in out] == [c["h"] for c in cases]


def test_kat_on_device(gpu_ctx):
    """key/curve_test.go:10-30 reproduced on the GPU: AuthScheme.Sign of the
    18-byte message with the KAT secret gives sigExp bit for bit, the
    signature verifies (VerifyRecovered over the raw message), the public key
    derived on the device is sk * g1, and H(msg) = sk^-1 * sig."""
    from drand_amd.chain import hash_to_curve, sign, verify_recovered
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.synth import R_ORDER
    k = load_golden("kat_bls12381_compat_v112.json")
    msg, sk, sig, pk = (bytes.fromhex(k[f]) for f in ("msg", "sk", "sig", "pk"))
    assert len(msg) == 18
    sch = get_scheme_by_id_with_default("")
    assert sign(sk, [msg], sch) == [sig]
    assert verify_recovered(sch, pk, [msg, msg + b"!", b""], [sig, sig, sig]).tolist() == [0, 3, 3]
    from drand_amd import _lib
    out = np.zeros(48, dtype=np.uint8)
    skb = np.frombuffer(sk, dtype=np.uint8).copy()
    _lib.check(gpu_ctx.lib.dgpu_derive_pubkey(gpu_ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(skb), _lib.ptr(out), 48))
    assert bytes(out) == pk
    h = B.g2_decompress(hash_to_curve([msg], sch)[0])
    inv = pow(int.from_bytes(sk, "big"), -1, R_ORDER)
    assert B.g2_compress(B.g2_mul(B.g2_decompress(sig), inv)) == B.g2_compress(h)


def test_digest_matches_reference_rule(chained, unchained):
    rng = np.random.default_rng(1)
    prevs = [bytes(rng.integers(0, 256, size=n, dtype=np.uint8)) for n in (0, 32, 96, 55, 56, 120)]
    rounds = [1, 2, 1969, 184348345343, 0xA1B2C3D4E5F6A7B8, 0]
    got = chained.digest_messages(rounds, prevs)
    for r, p, g in zip(rounds, prevs, got):
        assert g == hashlib.sha256(p + D.round_to_bytes(r)).digest()
    got = unchained.digest_messages(rounds, prevs)
    for r, g in zip(rounds, got):
        assert g == hashlib.sha256(D.round_to_bytes(r)).digest()


@pytest.mark.parametrize("name", ["chain_chained_s1.json", "chain_unchained_s1.json"])
def test_golden_chain_verdicts(name, chained, unchained):
    from drand_amd.chain import Beacon
    g = load_golden(name)
    v = chained if g["scheme"] == "pedersen-bls-chained" else unchained
    pk = bytes.fromhex(g["pk"])
    beacons = [Beacon(bytes.fromhex(r["prev"]), r["round"], bytes.fromhex(r["sig"])) for r in g["rounds"]]
    beacons += [Beacon(bytes.fromhex(c["prev"]), c["round"], bytes.fromhex(c["sig"])) for c in g["corrupted"]]
    expect = [True] * len(g["rounds"]) + [c["valid"] for c in g["corrupted"]]
    errs = v.verify_beacons(beacons, pk)
    assert [e is None for e in errs] == expect
    # single-beacon API: VerifyBeacon returns nil / error
    v.verify_beacon(beacons[0], pk)
    with pytest.raises(Exception):
        v.verify_beacon(beacons[-1], pk)


def test_gpu_chain_generator_matches_oracle(gpu_ctx):
    """dgpu_make_chain (one segment) reproduces the oracle's chain bit-exactly."""
    from drand_amd import _lib
    from drand_amd.synth import make_chain
    pk, ch = D.make_chain(1, 6)
    c = make_chain(1, 6, _lib.SCHEME_CHAINED, seg_len=6)
    assert c.pk == pk
    for i, (r, prev, sig) in enumerate(ch):
        assert int(c.rounds[i]) == r
        assert bytes(c.prev[i, : c.prev_len[i]]) == prev
        assert bytes(c.sigs[i]) == sig


@pytest.mark.parametrize("name", ["chain_chained_s1.json", "chain_unchained_s1.json"])
def test_reasons_match_oracle(name, chained, unchained):
    """Per-round reason codes equal the oracle's kyber error class (R)."""
    from drand_amd.chain import Beacon
    g = load_golden(name)
    v = chained if g["scheme"] == "pedersen-bls-chained" else unchained
    beacons = [Beacon(bytes.fromhex(c["prev"]), c["round"], bytes.fromhex(c["sig"])) for c in g["corrupted"]]
    reasons = v.verify_reasons(beacons, bytes.fromhex(g["pk"])).tolist()
    assert {c["kind"]: r for c, r in zip(g["corrupted"], reasons)} == {c["kind"]: c["reason"] for c in g["corrupted"]}


def test_non_subgroup_signature(chained):
    from drand_amd import _lib
    from drand_amd.chain import Beacon
    rnd = np.random.default_rng(4)
    u = (int.from_bytes(rnd.bytes(64), "big") % B.P, int.from_bytes(rnd.bytes(64), "big") % B.P)
    q = B.iso_map_g2(B.map_to_curve_sswu_g2(u))
    g = load_golden("chain_chained_s1.json")
    r = g["rounds"][0]
    reasons = chained.verify_reasons([Beacon(bytes.fromhex(r["prev"]), r["round"], B.g2_compress(q))],
                                     bytes.fromhex(g["pk"]))
    assert reasons.tolist() == [_lib.REASON_SUBGROUP]


def test_bad_pubkey_rejected(chained):
    from drand_amd import _lib
    from drand_amd.chain import Beacon
    with pytest.raises(_lib.DrandGPUError):
        chained.verify_beacons([Beacon(b"", 1, bytes(96))], bytes([0x80]) + bytes(47))


def test_large_chain_by_construction(chained):
    """4096 GPU-generated rounds, 0.5% corrupted across the whole catalog:
    verdicts equal construction; a sample re-checked with the oracle."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(7, 4096, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 7, rate=5e-3)
    beacons = [c.beacon(i) for i in range(len(c))]
    errs = chained.verify_beacons(beacons, c.pk)
    got = np.array([e is None for e in errs])
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(got, expect)
    pk = B.g1_decompress(c.pk)
    for i in list(bad.keys())[:3] + [0, 1, 64, 4095]:
        b = beacons[i]
        assert D.verify_beacon(D.SCHEME_CHAINED, pk, b.round, b.previous_sig, b.signature) == bool(got[i])


@pytest.mark.parametrize("name", ["chain_chained_s1.json", "chain_unchained_s1.json"])
def test_rlc_mode_equals_per_round_golden(name, chained, unchained):
    from drand_amd import _lib
    from drand_amd.chain import Beacon
    g = load_golden(name)
    v = chained if g["scheme"] == "pedersen-bls-chained" else unchained
    pk = bytes.fromhex(g["pk"])
    beacons = [Beacon(bytes.fromhex(r["prev"]), r["round"], bytes.fromhex(r["sig"])) for r in g["rounds"]]
    beacons += [Beacon(bytes.fromhex(c["prev"]), c["round"], bytes.fromhex(c["sig"])) for c in g["corrupted"]]
    per = v.verify_reasons(beacons, pk).tolist()
    for seed in (1, 0xDEADBEEF):
        assert v.verify_reasons(beacons, pk, mode=_lib.MODE_RLC, rlc_seed=seed).tolist() == per
    # edge cases: single beacon, all valid, all invalid-by-pairing, decode failures only
    for sub in (beacons[:1], beacons[: len(g["rounds"])], beacons[-3:], [beacons[-1]]):
        assert (v.verify_reasons(sub, pk, mode=_lib.MODE_RLC, rlc_seed=5).tolist()
                == v.verify_reasons(sub, pk).tolist())


def test_rlc_mode_large_chain(chained):
    """3000 rounds (not a power of two), 1% corrupted: RLC verdicts/reasons ==
    per-round verdicts/reasons == construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(11, 3000, _lib.SCHEME_CHAINED, seg_len=32)
    bad = corrupt(c, 11, rate=1e-2)
    beacons = [c.beacon(i) for i in range(len(c))]
    per = chained.verify_reasons(beacons, c.pk)
    rlc = chained.verify_reasons(beacons, c.pk, mode=_lib.MODE_RLC, rlc_seed=12345)
    assert rlc.tolist() == per.tolist()
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(per == 0, expect)


def test_rlc_node_checks_on_either_kernel_family():
    """RLC mode's node checks below DGPU_THR_MIN (default 65,536) run on the
    12-lane lines and 8-lane chain kernels; DGPU_THR_MIN=0 puts every check on
    the per-thread kernels (what the 10M bench's 64Ki-node top level uses).
    20,011 rounds, 1% corrupted: identical reasons either way, equal to
    per-round mode and to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(23, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 23, rate=1e-2)
    per = _verify_with_env(c, {})
    lanes = _verify_with_env(c, {"DGPU_THR_MIN": "65536"}, mode=_lib.MODE_RLC)
    thread = _verify_with_env(c, {"DGPU_THR_MIN": "0"}, mode=_lib.MODE_RLC)
    assert lanes.tolist() == thread.tolist() == per.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(per == 0, expect)


def test_small_batches_on_lane_kernels():
    """Per-round batches under DGPU_THR_MIN (default 65,536 items per pairing
    chunk) run the 12-lane lines and the 8-lane chain; DGPU_THR_MIN=0 (the
    suite's setting) the per-thread kernels.  5,003 rounds, 1% corrupted:
    identical reasons, equal to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 5003
    c = make_chain(31, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 31, rate=1e-2)
    lanes = _verify_with_env(c, {"DGPU_THR_MIN": "65536"})
    thread = _verify_with_env(c, {"DGPU_THR_MIN": "0"})
    assert lanes.tolist() == thread.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(thread == 0, expect)


def test_rlc_small_batches_take_per_round_path():
    """Below DGPU_RLC_MIN rounds (default 131,072) an RLC-mode call runs the
    per-round path: same reasons as RLC mode on the RLC path
    (DGPU_RLC_MIN=0, the test suite's setting) and as per-round mode."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 5003
    c = make_chain(29, n, _lib.SCHEME_CHAINED, seg_len=64)
    corrupt(c, 29, rate=1e-2)
    per = _verify_with_env(c, {})
    small = _verify_with_env(c, {"DGPU_RLC_MIN": "131072"}, mode=_lib.MODE_RLC)
    rlc = _verify_with_env(c, {"DGPU_RLC_MIN": "0"}, mode=_lib.MODE_RLC)
    assert small.tolist() == rlc.tolist() == per.tolist()


def _verify_with_env(c, env, mode=None):
    """Verify chain c on a fresh context opened under the environment `env`
    (the library reads its A/B and test knobs at dgpu_open); returns reasons."""
    import os
    from drand_amd import _lib
    n = len(c.rounds)
    ctx = open_ctx(env)
    try:
        lib = ctx.lib
        _lib.check(lib.dgpu_set_pubkey(ctx.handle, _lib.SCHEME_CHAINED, c.pk, len(c.pk)))
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        _lib.check(lib.dgpu_verify_batch(ctx.handle, _lib.SCHEME_CHAINED, n, _lib.ptr(c.rounds),
                                         _lib.ptr(c.sigs), c.sigs.shape[1], _lib.ptr(c.sig_len),
                                         _lib.ptr(c.prev), c.prev.shape[1], _lib.ptr(c.prev_len),
                                         _lib.MODE_PER_ROUND if mode is None else mode, 0, _lib.ptr(bits),
                                         _lib.ptr(reason)))
        assert np.array_equal(np.unpackbits(bits, bitorder="little")[:n].astype(bool), reason == 0)
        return reason
    finally:
        ctx.close()


def test_karabina_fe_equals_granger_scott_and_fallback():
    """The Karabina FE (default) against the Granger-Scott kernel (DGPU_FE=gs)
    and against the Karabina path with every 7th item of each chunk forced
    onto the fallback list (DGPU_KB_TEST_FLAG=7, a test hook of the A/B build:
    flagged as if f1 = 0, its FE re-run on prog_fe by k_eng_fe_fb), with the
    8-lane compressed chain (DGPU_KB_CHAIN=lanes) in place of the per-thread
    one, and with the norms read from the planes instead of written by the
    chain (DGPU_KB_NORM=planes, A/B build, fallback forced).  20,011 rounds (a
    ragged last block), 1% corrupted: identical reasons, equal to the
    construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(21, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 21, rate=1e-2)
    kb = _verify_with_env(c, {})
    gs = _verify_with_env(c, {"DGPU_FE": "gs"})
    fb = _verify_with_env(c, {"DGPU_KB_TEST_FLAG": "7"})
    lanes = _verify_with_env(c, {"DGPU_KB_CHAIN": "lanes"})
    norm_planes = _verify_with_env(c, {"DGPU_KB_NORM": "planes", "DGPU_KB_TEST_FLAG": "7"})
    assert kb.tolist() == gs.tolist() == fb.tolist() == lanes.tolist() == norm_planes.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(kb == 0, expect)


def test_karabina_fallback_on_natural_input():
    """The fallback without a test hook: under the key sk = 1 (pk = g1) a valid
    signature is H itself, so the two Miller loops are f(g1, H) and f(-g1, H)
    = conj f(g1, H) up to Fp factors; their product lies in Fp6 and the easy
    part maps it to m = 1, whose compressed form has f1 = 0: every valid round
    is flagged by the norms kernel and decided by k_eng_fe_fb, while
    corrupted rounds (m != 1) take the Karabina path in the same chunks.  The
    shipped library's reasons equal the construction and the Granger-Scott
    kernel's (DGPU_FE=gs), per chunk size (one chunk, and 4Ki-round chunks)."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    from oracle import bls12381 as B
    from oracle import drand_ref as D
    n = 9001
    c = make_chain(25, n, _lib.SCHEME_CHAINED, seg_len=64, sk=1)
    assert bytes(c.pk) == B.g1_compress(B.G1_GEN)
    # the oracle agrees that such a round verifies (pk = g1, sig = H(msg))
    assert D.verify_beacon(D.SCHEME_CHAINED, B.g1_decompress(bytes(c.pk)), int(c.rounds[0]),
                           bytes(c.prev[0, :c.prev_len[0]]), bytes(c.sigs[0]))
    bad = corrupt(c, 25, rate=2e-2)
    kb = _verify_with_env(c, {})
    kb4 = _verify_with_env(c, {"DGPU_ENG_CHUNK": "4096"})
    gs = _verify_with_env(c, {"DGPU_FE": "gs"})
    assert kb.tolist() == kb4.tolist() == gs.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(kb == 0, expect)


def test_thread_lines_equal_engine_lines():
    """The per-thread T-steps (k_lines_thr, default) against the 12-lane
    engine's lines program (DGPU_LINES=engine) and the pair-per-wave variant
    (A/B build, DGPU_LINES_WAVE=1): 20,011 rounds (ragged last
    block), 1% corrupted -- identical reasons (x-bit flips that stay on the
    curve exercise the fused membership test: REASON_SUBGROUP from both),
    equal to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(23, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 23, rate=1e-2)
    thr = _verify_with_env(c, {})
    eng = _verify_with_env(c, {"DGPU_LINES": "engine"})
    wave = _verify_with_env(c, {"DGPU_LINES_WAVE": "1"})  # A/B: a pair per wave, P in SGPRs
    assert thr.tolist() == eng.tolist() == wave.tolist()
    assert (thr == _lib.REASON_SUBGROUP).any()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(thr == 0, expect)


def test_fast_group_law_generic_redo_equals_default():
    """The fast group-law paths' generic redo forced on every item (A/B build
    test hook DGPU_TEST_FORCE_EXC=1): the hash's cofactor ladder redone by
    g2_clear_cofactor from P, the decoders' membership ladder by
    g2_in_subgroup, the RLC root MSM's bucket sums by the generic mixed
    addition (each thread's emits overwritten) -- per round and in RLC mode
    (DGPU_RLC_MIN=0), 20,011 rounds, 1% corrupted: reasons identical to the
    default paths' and equal to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(31, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 31, rate=1e-2)
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    for mode in (_lib.MODE_PER_ROUND, _lib.MODE_RLC):
        ref = _verify_with_env(c, {"DGPU_RLC_MIN": "0"}, mode=mode)
        red = _verify_with_env(c, {"DGPU_RLC_MIN": "0", "DGPU_TEST_FORCE_EXC": "1"}, mode=mode)
        assert red.tolist() == ref.tolist()
        assert np.array_equal(red == 0, expect)


def test_karabina_chain_on_two_lanes_equals_default():
    """The Karabina chain with each round's compressed element split over two
    lanes (k_kb_chain_pair, A/B build DGPU_KB_PAIR=1: the lanes swap (q, k)
    once per squaring) against the one-thread chain: 20,011 rounds (odd, a
    ragged last block), 1% corrupted, on two engine chunk sizes and with the
    Karabina fallback forced on every 7th item -- identical reasons, equal to
    the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(29, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 29, rate=1e-2)
    ref = _verify_with_env(c, {"DGPU_KB_PAIR": "0"})
    pair = _verify_with_env(c, {"DGPU_KB_PAIR": "1"})
    pair_small = _verify_with_env(c, {"DGPU_KB_PAIR": "1", "DGPU_ENG_CHUNK": "4099"})
    pair_fb = _verify_with_env(c, {"DGPU_KB_PAIR": "1", "DGPU_KB_TEST_FLAG": "7"})
    assert pair.tolist() == ref.tolist() == pair_small.tolist() == pair_fb.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(pair == 0, expect)


def test_engine_without_idle_lanes_equals_default():
    """The Miller loop and the Karabina FE segments on 16-group 192-thread
    blocks (k_eng_miller_xw, k_eng_fe_seg_xw: groups 5 and 10 span two waves,
    sub-ops ordered by barriers, the verdict vote through LDS) against the
    five-group wave kernels: 20,011 rounds (a ragged last block of 11 items,
    and a chunk count that is not a multiple of 16), 1% corrupted, on two
    engine chunk sizes, and with the Karabina fallback forced on every 7th
    item (its list names 5-round blocks once each) -- identical reasons,
    equal to the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 20011
    c = make_chain(27, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 27, rate=1e-2)
    ref = _verify_with_env(c, {"DGPU_ENG_XW": "0"})
    miller = _verify_with_env(c, {"DGPU_ENG_XW": "1"})
    xw = _verify_with_env(c, {"DGPU_ENG_XW": "3"})
    xw_small = _verify_with_env(c, {"DGPU_ENG_XW": "3", "DGPU_ENG_CHUNK": "4099"})
    xw_fb = _verify_with_env(c, {"DGPU_ENG_XW": "3", "DGPU_KB_TEST_FLAG": "7"})
    assert xw.tolist() == ref.tolist() == miller.tolist() == xw_small.tolist() == xw_fb.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(xw == 0, expect)


def test_two_lane_per_round_large_chain():
    """A batch spanning two engine chunks runs on two lanes (streams, half the
    batch each, capi.hip verify_status_locked), its host records staged slice
    by slice through the pinned ring beside the verification
    (verify_status_host_locked): 2*131072 + 1001 rounds (odd split), 0.1%
    corrupted -- reasons equal the one-lane context's (DGPU_LANES=1,
    64Ki-round engine chunks: five chunks), five slices alternating between
    the lanes (A/B build), the round-5 whole-batch pageable staging (A/B
    build, DGPU_STAGE=pageable) and the construction."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 2 * 131072 + 1001
    c = make_chain(13, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 13, rate=1e-3)

    two = _verify_with_env(c, {"DGPU_LANES": "2"})
    one = _verify_with_env(c, {"DGPU_LANES": "1", "DGPU_ENG_CHUNK": "65536"})
    five = _verify_with_env(c, {"DGPU_LANES": "2", "DGPU_LANE_SLICES": "5"})  # slices alternating between lanes
    page = _verify_with_env(c, {"DGPU_STAGE": "pageable"})
    assert two.tolist() == one.tolist() == five.tolist() == page.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(two == 0, expect)
