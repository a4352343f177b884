"""Oracle for the signatures-on-G1 schemes (bls-unchained-on-g1 and
bls-unchained-g1-rfc9380): hash-to-G1 pinned by RFC 9380's test vector J.9.1
(the isogeny constants are derived in tools/derive_iso11.py, which checks the
RFC's published k_(1,0) and this vector), the committed chain fixtures, and
the endomorphism G1-membership test the kernels use against [r]P == O.
The schemes themselves are absent from the reference snapshot (SURVEY.md
section 8c): their DST choice is parity-unpinned."""
import random

from conftest import load_golden
from oracle import bls12381 as B
from oracle import drand_ref as D

P = B.P
TV_DST = b"QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_"


def test_hash_to_g1_rfc9380_vector():
    h = B.hash_to_g1(b"", TV_DST)
    assert h == (0x052926ADD2207B76CA4FA57A8734416C8DC95E24501772C814278700EED6D1E4E8CF62D9C09DB0FAC349612B759E79A1,
                 0x08BA738453BFED09CB546DBB0783DBB3A5F1F566ED67BB6BE0E8C67E2E81A4CC68EE29813BB7994998F3EAE0C9C6A265)
    assert B.g1_in_subgroup(h)


def test_hash_to_g1_fixture_consistent():
    for c in load_golden("hash_to_g1.json")["cases"][:6]:
        assert B.g1_compress(B.hash_to_g1(bytes.fromhex(c["msg"]), c["dst"].encode())).hex() == c["h"]


def test_g1_chain_fixtures_verify():
    for name in ("chain_on_g1_s1.json", "chain_g1_rfc9380_s2.json"):
        g = load_golden(name)
        pk = B.g2_decompress(bytes.fromhex(g["pk"]))
        for rd in g["rounds"][:3]:
            assert D.verify_beacon(g["scheme"], pk, rd["round"], b"", bytes.fromhex(rd["sig"]))
        kinds = {c["kind"]: c["reason"] for c in g["corrupted"]}
        assert kinds["not_in_subgroup"] == D.REASON_SUBGROUP and kinds["infinity"] == D.REASON_INFINITY
        assert kinds["y_sign_flip"] == D.REASON_PAIRING and kinds["g2_sized_sig"] == D.REASON_DECODE


def test_schemes_differ_only_in_dst():
    m = D.digest_message(D.SCHEME_UNCHAINED_G1, 7, b"")
    assert m == D.digest_message(D.SCHEME_G1_RFC9380, 7, b"")
    assert B.hash_to_g1(m, B.DST_G2) != B.hash_to_g1(m, B.DST_G1)


def test_endomorphism_membership_matches_order_test():
    """phi(P) = (beta x, y) == -[x^2] P  <=>  [r] P == O on E1(Fp) (Scott)."""
    beta = 0x5F19672FDF76CE51BA69C6076A0F77EADDB3A93BE6F89688DE17D813620A00022E01FFFFFFFEFFFE
    assert pow(beta, 3, P) == 1 and beta != 1
    rng = random.Random(9)
    cof = 0x396C8C005555E1568C00AAAB0000AAAB
    for k in range(12):
        while True:
            x = rng.randrange(P)
            y = B.fp_sqrt(x ** 3 + 4)
            if y is not None:
                break
        pt = B.g1_mul((x, y), cof) if k % 2 else (x, y)
        phi = (beta * pt[0] % P, pt[1])
        assert (phi == B.g1_mul(pt, -B.BLS_X * B.BLS_X)) == B.g1_in_subgroup(pt)
