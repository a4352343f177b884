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

FIXTURES = ["recover_t3_n8.json", "recover_t17_n32.json"]


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
