"""The oracle against the reference's own known answers (CPU)."""
import hashlib

import pytest

from conftest import load_golden
from oracle import bls12381 as B
from oracle import drand_ref as D
from oracle import pairing_formulas as PF


def test_kat_bls12381_compat_v112():
    """key/curve_test.go:10-30: pins DST, hash-to-G2, G2 mul and compression."""
    k = load_golden("kat_bls12381_compat_v112.json")
    sig = B.sign_g2(int(k["sk"], 16), bytes.fromhex(k["msg"]))
    assert sig.hex() == "9940ca447bab3bab393c3a07866349343630437167eaeab063ef1e47acedc51e85c513121cf319a8832c3d136d7f36490fa7241194b403a3bbbba9e7d5e73c9a86f67a9585c6fe077cd6576b2f76560efbab3550d9d5124242c728e3a7ef6989"
    pk = B.g1_mul(B.G1_GEN, int(k["sk"], 16))
    assert B.verify_g2(pk, bytes.fromhex(k["msg"]), sig)


def test_round_to_bytes():
    """chain/store_test.go:9-14"""
    assert D.round_to_bytes(0) == bytes(8)
    assert D.round_to_bytes(1) == bytes(7) + b"\x01"
    assert D.round_to_bytes(184348345343) == bytes([0, 0, 0, 0x2A, 0xEC, 0x04, 0x83, 0xFF])
    assert D.round_to_bytes(0xA1B2C3D4E5F6A7B8) == bytes([0xA1, 0xB2, 0xC3, 0xD4, 0xE5, 0xF6, 0xA7, 0xB8])


def test_digest_message_rules():
    """chain/verify.go:24-32"""
    prev = bytes(range(96))
    assert D.digest_message(D.SCHEME_CHAINED, 7, prev) == hashlib.sha256(prev + D.round_to_bytes(7)).digest()
    assert D.digest_message(D.SCHEME_UNCHAINED, 7, prev) == hashlib.sha256(D.round_to_bytes(7)).digest()
    assert D.digest_message(D.SCHEME_CHAINED, 7, b"") == hashlib.sha256(D.round_to_bytes(7)).digest()


def test_generators_and_constants():
    assert B.g1_on_curve(B.G1_GEN) and B.g2_on_curve(B.G2_GEN)
    assert B.g1_in_subgroup(B.G1_GEN) and B.g2_in_subgroup(B.G2_GEN)
    assert B.g1_compress(B.G1_GEN).hex().startswith("97f1d3a7")
    assert B.g2_compress(B.G2_GEN).hex().startswith("93e02b60")
    x, p, r = B.BLS_X, B.P, B.R
    assert (p ** 4 - p ** 2 + 1) % r == 0
    assert 3 * (p ** 4 - p ** 2 + 1) // r == (x - 1) ** 2 * (x + p) * (x * x + p * p - 1) + 3


def test_pairing_bilinear():
    a, b = 5, 11
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert not B.f12_is_one(e)
    assert B.f12_eq(B.pairing(B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)), B.f12_pow(e, a * b))
    assert B.f12_is_one(B.f12_pow(e, B.R))


def test_projective_miller_matches_generic():
    P1 = B.g1_mul(B.G1_GEN, 7)
    Q1 = B.g2_mul(B.G2_GEN, 13)
    ref = B.pairing(P1, Q1)
    assert B.f12_eq(B.final_exponentiation(PF.miller_loop_multi([(P1, Q1)])), ref)
    assert B.f12_eq(PF.final_exp_chain(PF.miller_loop_multi([(P1, Q1)])), ref)


def test_psi_subgroup_criterion_matches_r_mult():
    q = B.hash_to_g2(b"abc")
    assert B.g2_psi(q) == B.g2_mul(q, B.BLS_X)
    import random
    rnd = random.Random(5)
    for _ in range(3):
        pt = B.iso_map_g2(B.map_to_curve_sswu_g2((rnd.randrange(B.P), rnd.randrange(B.P))))
        assert not B.g2_in_subgroup(pt)
        assert B.g2_psi(pt) != B.g2_mul(pt, B.BLS_X)


def test_clear_cofactor_psi_equals_h_eff():
    import random
    rnd = random.Random(9)
    pt = B.iso_map_g2(B.map_to_curve_sswu_g2((rnd.randrange(B.P), rnd.randrange(B.P))))
    assert B.clear_cofactor_g2(pt) == B.g2_mul(pt, B.H_EFF_G2)


def test_hash_to_g2_golden():
    g = load_golden("hash_to_g2.json")
    for c in g["cases"][:6]:
        assert B.g2_compress(B.hash_to_g2(bytes.fromhex(c["msg"]))).hex() == c["h"]


def test_group_toml_keys_decode():
    """deploy/latest/group.toml public keys: decode-only fixtures."""
    g = load_golden("group_toml_keys.json")
    assert len(g["keys"]) > 0
    for k in g["keys"][:4]:
        pt = B.g1_decompress(bytes.fromhex(k["pk"]))
        assert B.g1_compress(pt).hex() == k["pk"]


def test_reference_legacy_encodings_decode():
    """The reference's decode-only G1-layout encodings (test/test-integration/
    test.json, demo/docker/data keys; tests/golden/make_golden.py
    legacy_encodings): stored forms decode and recompress to the same bytes,
    mutated forms keep their class."""
    g = load_golden("reference_legacy_encodings.json")
    srcs = {c["source"] for c in g["cases"]}
    assert len(srcs) >= 4 and any("test.json:Public" in s for s in srcs)
    for c in g["cases"]:
        raw = bytes.fromhex(c["hex"])
        g2 = c["group"] == "g2"
        if c["kind"] == "as_stored":
            assert c["decodes"] and c["recompressed"] == c["hex"]
        if c["decodes"]:
            pt = B.g2_decompress(raw) if g2 else B.g1_decompress(raw)
            assert (B.g2_compress(pt) if g2 else B.g1_compress(pt)).hex() == c["recompressed"]
        else:
            with pytest.raises(B.DecodeError):
                B.g2_decompress(raw) if g2 else B.g1_decompress(raw)


@pytest.mark.parametrize("name", ["chain_chained_s1.json", "chain_unchained_s1.json"])
def test_golden_chain_verifies(name):
    g = load_golden(name)
    pk = B.g1_decompress(bytes.fromhex(g["pk"]))
    for r in g["rounds"][:2]:
        assert D.verify_beacon(g["scheme"], pk, r["round"], bytes.fromhex(r["prev"]), bytes.fromhex(r["sig"]))
    for c in g["corrupted"][:4]:
        assert D.verify_beacon(g["scheme"], pk, c["round"], bytes.fromhex(c["prev"]), bytes.fromhex(c["sig"])) == c["valid"]


def test_empty_and_wrong_round_rejected():
    """lp2p/client/validator_test.go:125-145 (empty sig) and
    test/mock/grpcserver.go:150-155 (round-1 must fail)."""
    g = load_golden("chain_chained_s1.json")
    pk = B.g1_decompress(bytes.fromhex(g["pk"]))
    r = g["rounds"][3]
    prev, sig = bytes.fromhex(r["prev"]), bytes.fromhex(r["sig"])
    assert not D.verify_beacon(D.SCHEME_CHAINED, pk, r["round"], prev, b"")
    assert not D.verify_beacon(D.SCHEME_CHAINED, pk, r["round"] - 1, prev, sig)


def test_check_past_beacons_semantics():
    """sync_manager.go:171-232: missing rows shorten the scan; faulty list."""
    store = {0: (0, b"", b"g"), 1: (1, b"", b"a"), 2: (2, b"", b"bad"), 4: (4, b"", b"a"), 5: (5, b"", b"a")}
    faulty, progress = D.check_past_beacons(store, 10, lambda b: b[2] != b"bad")
    # Len = 5 -> i in 1..4; row 3 missing -> faulty 3; upTo clamps to last = 5
    assert faulty == [2, 3]
    assert progress == [(1, 5), (2, 5), (3, 5), (4, 5)]
    assert D.check_past_beacons({0: (0, b"", b"")}, 3, lambda b: True) == (None, [])
