"""CheckPastBeacons batch mirror (drand_amd/sync.py) against the oracle's
restatement of chain/beacon/sync_manager.go:171-232: identical faulty lists,
progress callbacks and stopping rule for every window size.  The CPU tests
use a stand-in verifier (verdict = a marker in the signature bytes); the GPU
test runs the real HIP verifier over a golden chain with missing rows."""
import random

import numpy as np
import pytest

from conftest import load_golden
from drand_amd.chain import Beacon
from drand_amd.sync import MemoryStore, beacon_marshal, beacon_unmarshal, check_past_beacons
from oracle import drand_ref as D


class MarkerVerifier:
    """Stand-in for chain.Verifier in CPU tests: a beacon is valid iff its
    signature does not start with b"BAD"."""

    def __init__(self):
        self.calls = 0

    def verify_reasons(self, beacons, pubkey, mode=0):
        self.calls += 1
        return np.array([3 if b.signature.startswith(b"BAD") else 0 for b in beacons], dtype=np.uint8)

    def verify_records(self, pubkey, rounds, sigs, sig_len, prev, prev_len, mode=0):
        """The fixed-stride form (native bolt ingest, drand_amd/ingest.py)."""
        self.calls += 1
        return np.array([3 if sig_len[i] > sigs.shape[1] or bytes(sigs[i, :3]) == b"BAD" and sig_len[i] >= 3 else 0
                         for i in range(len(rounds))], dtype=np.uint8)


def _random_store(rng, n):
    st = MemoryStore()
    table = {}
    st.put(Beacon(b"", 0, b"genesis"))
    table[0] = (0, b"", b"genesis")
    for r in range(1, n + 1):
        if rng.random() < 0.05:
            continue  # missing row
        rr = r if rng.random() > 0.03 else r + 1000  # stored beacon with a different Round field
        sig = (b"BAD" if rng.random() < 0.1 else b"ok") + bytes([r & 0xFF])
        st.put_raw(r, beacon_marshal(Beacon(b"p", rr, sig)))
        table[r] = (rr, b"p", sig)
    return st, table


def test_hexjson_roundtrip():
    b = Beacon(bytes(range(96)), 184348345343, bytes(range(96, 192)))
    enc = beacon_marshal(b)
    assert b'"Round":184348345343' in enc and bytes(range(4)).hex().encode() in enc
    assert beacon_unmarshal(enc) == b
    assert beacon_unmarshal(b'{"Round":7}') == Beacon(b"", 7, b"")


@pytest.mark.parametrize("bad", ["ab cd", " abcd", "abcd ", "abc", "zz", "0xab", "ab\ncd", "١٢", "ab\tcd"])
def test_hexjson_rejects_what_go_hex_rejects(bad):
    """hexjson decodes []byte fields with Go's hex.DecodeString, which refuses
    odd lengths and any non-hex byte (whitespace included) -- the row is an
    Unmarshal error, so CheckPastBeacons counts it faulty."""
    import json
    for field in ("Signature", "PreviousSig"):
        with pytest.raises(ValueError):
            beacon_unmarshal(json.dumps({"Round": 3, field: bad}).encode())
    assert beacon_unmarshal(b'{"Round":3,"Signature":"ABcd"}') == Beacon(b"", 3, b"\xab\xcd")


@pytest.mark.parametrize("window", [1, 3, 16, 1 << 16])
def test_check_past_beacons_matches_oracle(window):
    rng = random.Random(window)
    for trial in range(40):
        n = rng.randint(1, 60)
        st, table = _random_store(rng, n)
        last = st.last().round
        for up_to in (0, 1, rng.randint(1, n + 5), n, n + 10, last + 5):
            calls = []
            got = check_past_beacons(st, MarkerVerifier(), b"pk", up_to, cb=lambda i, u: calls.append((i, u)),
                                     window=window)
            exp, progress = D.check_past_beacons(table, up_to, lambda b: not b[2].startswith(b"BAD"))
            assert got == exp, (trial, up_to)
            assert calls == progress, (trial, up_to)


def test_check_past_beacons_batches():
    st, table = _random_store(random.Random(5), 200)
    v = MarkerVerifier()
    check_past_beacons(st, v, b"pk", 10**9, window=64)
    assert v.calls == -(-(st.len() - 1) // 64)  # one GPU batch per window, not one call per round


@pytest.mark.gpu
def test_check_past_beacons_gpu_golden():
    """Real verifier: a golden chained chain with corrupted rows and holes;
    the faulty list equals the oracle restatement's."""
    from drand_amd.chain import Verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    g = load_golden("chain_chained_s1.json")
    pk = bytes.fromhex(g["pk"])
    st = MemoryStore()
    table = {0: (0, b"", bytes.fromhex(g["genesis"]))}
    st.put(Beacon(b"", 0, bytes.fromhex(g["genesis"])))
    bad = {c["round"]: c for c in g["corrupted"] if c["kind"] in ("x_bit_flip", "y_sign", "other_round_sig")}
    for r in g["rounds"]:
        if r["round"] == 5:
            continue  # hole
        src = bad.get(r["round"], r)
        b = Beacon(bytes.fromhex(src["prev"]), r["round"], bytes.fromhex(src["sig"]))
        st.put(b)
        table[r["round"]] = (b.round, b.previous_sig, b.signature)
    v = Verifier(get_scheme_by_id_with_default("pedersen-bls-chained"))
    got = check_past_beacons(st, v, pk, 10**9, window=7)
    exp, _ = D.check_past_beacons(table, 10**9, lambda b: b[2] == bytes.fromhex(
        next(x["sig"] for x in g["rounds"] if x["round"] == b[0])))
    assert got == exp and 5 in got


# ---------------------------------------------------------------- tryNode / client walk mirrors
def _packets(rng, n, start=1):
    out = []
    for r in range(start, start + n):
        sig = (b"BAD" if rng.random() < 0.04 else b"ok") + r.to_bytes(4, "big")
        bid = "other" if rng.random() < 0.02 else ("main" if rng.random() < 0.5 else None)
        out.append((Beacon(b"", r, sig), bid))
    return out


@pytest.mark.parametrize("window", [1, 4, 500])
def test_try_node_matches_oracle(window):
    from drand_amd.sync import try_node
    rng = random.Random(7 + window)
    for trial in range(60):
        pk = _packets(rng, rng.randint(0, 40))
        up_to = rng.randint(0, 45)
        fail_put = rng.choice([None, rng.randint(1, 45)])
        stored_a, stored_b = [], []

        class Store:
            def __init__(self, sink):
                self.sink = sink

            def put(self, b):
                if b.round == fail_put:
                    raise ValueError("put failed")
                self.sink.append(b.round)

        ok, last = try_node(pk, MarkerVerifier(), b"pk", Store(stored_a), up_to, beacon_id="main", window=window)

        def put_ref(b):
            if b[0] == fail_put:
                raise ValueError("put failed")
            stored_b.append(b[0])
        ok_r, last_r = D.try_node([((b.round, b.previous_sig, b.signature), bid) for b, bid in pk],
                                  lambda b: not b[2].startswith(b"BAD"), put_ref, up_to, beacon_id="main")
        assert (ok, stored_a) == (ok_r, stored_b)
        assert (last.round if last else None) == (last_r[0] if last_r else None)


def test_scheme_store_linkage():
    from drand_amd.sync import SchemeStore
    st = MemoryStore()
    st.put(Beacon(b"", 0, b"g"))
    ss = SchemeStore(st, decouple_prev_sig=False)
    ss.put(Beacon(b"g", 1, b"s1"))
    with pytest.raises(ValueError):
        ss.put(Beacon(b"xx", 2, b"s2"))
    ss.put(Beacon(b"s1", 2, b"s2"))
    uns = SchemeStore(MemoryStore(), decouple_prev_sig=True)
    uns.put(Beacon(b"anything", 5, b"s5"))
    assert uns.get(5).previous_sig == b""


@pytest.mark.parametrize("window", [1, 3, 1 << 14])
def test_trusted_previous_signature_matches_oracle(window):
    from drand_amd.chain import VerifyError
    from drand_amd.sync import trusted_previous_signature
    rng = random.Random(window)
    for trial in range(40):
        n = rng.randint(1, 30)
        sigs = {r: (b"BAD" if rng.random() < 0.03 else b"ok") + bytes([r]) for r in range(1, n + 2)}
        pot = rng.choice([None, (rng.randint(1, n), None)])
        if pot:
            pot = (pot[0], sigs[pot[0]])
        target = rng.randint(1, n + 1)
        try:
            ref = D.trusted_previous_signature(lambda r, p, s: not s.startswith(b"BAD"), sigs.__getitem__,
                                               b"seed", target, pot)
        except ValueError:
            ref = "error"
        try:
            got = trusted_previous_signature(MarkerVerifier(), b"pk", sigs.__getitem__, b"seed", target, pot,
                                             window=window)
        except VerifyError:
            got = "error"
        assert got == ref


@pytest.mark.gpu
def test_client_walk_and_try_node_gpu_golden():
    """The batch client walk and tryNode mirrors with the real HIP verifier on
    the golden chained chain: the walk returns round r-1's signature (and the
    new point of trust), a corrupted round in the walk raises; tryNode stores
    up to the first invalid beacon."""
    from drand_amd.chain import VerifyError, new_verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.sync import SchemeStore, trusted_previous_signature, try_node
    g = load_golden("chain_chained_s1.json")
    v = new_verifier(get_scheme_by_id_with_default(g["scheme"]))
    pk = bytes.fromhex(g["pk"])
    sig = {r["round"]: bytes.fromhex(r["sig"]) for r in g["rounds"]}
    seed = bytes.fromhex(g["genesis"])
    prev, pot = trusted_previous_signature(v, pk, sig.__getitem__, seed, 20, point_of_trust=(5, sig[5]), window=7)
    assert prev == sig[19] and pot == (19, sig[19])
    bad = dict(sig)
    bad[10] = sig[11]
    with pytest.raises(VerifyError):
        trusted_previous_signature(v, pk, bad.__getitem__, seed, 20, point_of_trust=(5, sig[5]), window=7)
    # without a point of trust the reference walks from (1, GenesisSeed) and
    # verifies round 2 against the genesis seed (client/verify.go:129-160), so
    # a chained walk fails at round 2 -- reproduced, not corrected
    with pytest.raises(VerifyError) as e:
        trusted_previous_signature(v, pk, sig.__getitem__, seed, 20, window=7)
    assert e.value.round == 2
    st = MemoryStore()
    st.put(Beacon(b"", 0, seed))
    packets = [(Beacon(bytes.fromhex(r["prev"]), r["round"], bad[r["round"]]), None) for r in g["rounds"]]
    ok, last = try_node(packets, v, pk, SchemeStore(st, False), up_to=24, window=5)
    assert not ok and last.round == 9 and st.len() == 10
