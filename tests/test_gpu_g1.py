"""GPU parity for the signatures-on-G1 schemes (bls-unchained-on-g1 and
bls-unchained-g1-rfc9380) through the C-ABI: hash-to-G1 vs the oracle's
fixture (pinned by RFC 9380 J.9.1), per-round verdicts and reasons on the
committed G1 chain fixtures and their corruption catalog, a synthetic GPU
chain with injected corruptions vs construction, and the scheme/key-group
mismatch error.  Parity against the reference is unpinned (scheme absent
from the snapshot); these pin the oracle's restatement."""
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

FIXTURES = ["chain_on_g1_s1.json", "chain_g1_rfc9380_s2.json"]


def _scheme(g):
    from drand_amd.scheme import get_scheme_by_id_with_default
    return get_scheme_by_id_with_default(g["scheme"])


def test_hash_to_g1_matches_fixture():
    from drand_amd import _lib
    from drand_amd.chain import hash_to_g1
    cases = [c for c in load_golden("hash_to_g1.json")["cases"] if c["msg"]]
    for code, tag in ((_lib.SCHEME_UNCHAINED_G1, "G2"), (_lib.SCHEME_G1_RFC9380, "G1")):
        sub = [c for c in cases if f"BLS12381{tag}_XMD" in c["dst"]]
        got = hash_to_g1([bytes.fromhex(c["msg"]) for c in sub], code)
        assert [g.hex() for g in got] == [c["h"] for c in sub]


@pytest.mark.parametrize("name", FIXTURES)
def test_g1_chain_fixture_verdicts(name):
    from drand_amd.chain import Beacon, new_verifier
    g = load_golden(name)
    v = new_verifier(_scheme(g))
    pk = bytes.fromhex(g["pk"])
    beacons = [Beacon(b"", r["round"], bytes.fromhex(r["sig"])) for r in g["rounds"]]
    beacons += [Beacon(b"", c["round"], bytes.fromhex(c["sig"])) for c in g["corrupted"]]
    reasons = v.verify_reasons(beacons, pk)
    expect = [0] * len(g["rounds"]) + [c["reason"] for c in g["corrupted"]]
    assert list(map(int, reasons)) == expect


@pytest.mark.parametrize("code_name", ["SCHEME_UNCHAINED_G1", "SCHEME_G1_RFC9380"])
def test_g1_synthetic_chain_with_corruptions(code_name):
    import numpy as np
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import corrupt, make_chain
    from oracle import bls12381 as B
    from oracle import drand_ref as D
    code = getattr(_lib, code_name)
    ch = make_chain(4, 3000, code, seg_len=50)
    scheme = D.SCHEME_UNCHAINED_G1 if code == _lib.SCHEME_UNCHAINED_G1 else D.SCHEME_G1_RFC9380
    pkp = B.g2_decompress(ch.pk)
    for i in (0, 1777):  # the generator agrees with the oracle's signer
        assert D.verify_beacon(scheme, pkp, int(ch.rounds[i]), b"", bytes(ch.sigs[i, :48]))
    bad = corrupt(ch, 9, rate=0.01)
    ctx = get_context(0)
    n = len(ch)
    _lib.check(ctx.lib.dgpu_set_pubkey(ctx.handle, code, ch.pk, 96))
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_verify_batch(ctx.handle, code, n, _lib.ptr(ch.rounds), _lib.ptr(ch.sigs), 96,
                                         _lib.ptr(ch.sig_len), None, 0, None, _lib.MODE_PER_ROUND, 0,
                                         _lib.ptr(bits), None))
    valid = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
    expect = np.ones(n, dtype=bool)
    expect[list(bad)] = False
    assert (valid == expect).all()


def test_key_group_mismatch_is_an_error():
    from drand_amd import _lib
    from drand_amd.chain import Beacon, new_verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    g1 = load_golden("chain_on_g1_s1.json")
    v = new_verifier(get_scheme_by_id_with_default("pedersen-bls-unchained"))
    with pytest.raises(_lib.DrandGPUError):
        v.verify_beacons([Beacon(b"", 1, bytes(96))], bytes.fromhex(g1["pk"]))  # 96-byte key for a G1-key scheme


@pytest.mark.parametrize("name", FIXTURES)
def test_g1_rlc_equals_per_round_fixture(name):
    """RLC mode for the G1-signature schemes (rlc_msm.cuh over G1Ops: bucket-MSM
    root, the key's fixed-Q lines for every node check, leaves + tree only
    when the root fails) gives the per-round reasons on the fixture and its
    corruption catalog, and a clean batch passes on the root alone."""
    from drand_amd import _lib
    from drand_amd.chain import Beacon, new_verifier
    g = load_golden(name)
    v = new_verifier(_scheme(g))
    pk = bytes.fromhex(g["pk"])
    clean = [Beacon(b"", r["round"], bytes.fromhex(r["sig"])) for r in g["rounds"]]
    beacons = clean + [Beacon(b"", c["round"], bytes.fromhex(c["sig"])) for c in g["corrupted"]]
    expect = [0] * len(g["rounds"]) + [c["reason"] for c in g["corrupted"]]
    for seed in (1, 2, 0xFFFFFFFFFFFFFFFF):
        assert v.verify_reasons(beacons, pk, _lib.MODE_RLC, rlc_seed=seed).tolist() == expect
    lib = v.ctx.lib
    _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 1))
    try:
        assert not v.verify_reasons(clean, pk, _lib.MODE_RLC).any()
        stages = set(_lib.stage_times(v.ctx))
    finally:
        _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 0))
    assert {"rlc_hash_to_g1_raw", "decode_g1", "rlc_root_msm"} <= stages and "rlc_leaves_tree" not in stages, stages
    # one round alone: its leaf is the root
    assert v.verify_reasons(beacons[-1:], pk, _lib.MODE_RLC).tolist() == expect[-1:]
    assert v.verify_reasons(clean[:1], pk, _lib.MODE_RLC).tolist() == [0]


@pytest.mark.parametrize("code_name", ["SCHEME_UNCHAINED_G1", "SCHEME_G1_RFC9380"])
def test_g1_rlc_large_chain_every_corruption_kind(code_name):
    """20,011 rounds (ragged engine blocks), 1% corrupted with every kind
    (x-bit flips that land on the curve are off-subgroup G1 points), plus
    signatures moved off the subgroup by a point of order 3 ((0, 2) on
    y^2 = x^3 + 4: a combination without the membership test would accept
    them whenever the coefficient is 0 mod 3): RLC reasons == per-round
    reasons == construction."""
    import numpy as np
    from drand_amd import _lib
    from drand_amd.chain import get_context
    from drand_amd.synth import corrupt, make_chain
    from oracle import bls12381 as B
    code = getattr(_lib, code_name)
    n = 20011
    ch = make_chain(31, n, code, seg_len=64)
    bad = corrupt(ch, 31, rate=0.01)
    T3 = (0, 2)
    assert B.g1_on_curve(T3) and B.g1_mul(T3, 3) is None
    off = [i for i in range(5, n, 4001) if i not in bad]
    for i in off:
        s = B.g1_decompress(bytes(ch.sigs[i, :48]))
        ch.sigs[i, :48] = np.frombuffer(B.g1_compress(B.g1_add(s, T3)), dtype=np.uint8)
    ctx = get_context(0)
    _lib.check(ctx.lib.dgpu_set_pubkey(ctx.handle, code, ch.pk, 96))

    def run(mode, seed=0):
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        _lib.check(ctx.lib.dgpu_verify_batch(ctx.handle, code, n, _lib.ptr(ch.rounds), _lib.ptr(ch.sigs), 96,
                                             _lib.ptr(ch.sig_len), None, 0, None, mode, seed, _lib.ptr(bits),
                                             _lib.ptr(reason)))
        return reason

    per = run(_lib.MODE_PER_ROUND)
    rlc = run(_lib.MODE_RLC, 0x1234)
    assert rlc.tolist() == per.tolist()
    assert all(per[i] == _lib.REASON_SUBGROUP for i in off)
    assert (per == _lib.REASON_SUBGROUP).sum() > len(off)  # x-bit flips onto the curve, off the subgroup
    expect = np.ones(n, dtype=bool)
    expect[list(bad) + off] = False
    assert np.array_equal(per == 0, expect)
