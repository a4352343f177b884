"""Regression for the round-3 ragged-block fault (DESIGN.md 2b' "r03i").

An uncommitted step between 141d92b and 787950a put the Karabina state
planes in the engine's wave-blocked layout (blocks of 5 rounds) while still
sizing and carving the chunk's scratch per round (cap x bytes, pbuf at
xbuf + planes x cap).  When a chunk's capacity was not a multiple of 5 -- any
batch smaller than one chunk whose size is not -- the last, partial block's
planes ran into pbuf / ebuf / the fallback list: that block's stored values
were overwritten by the norm kernel (pairing failures for exactly the last
n mod 5 items) and k_eng_fe_fb walked a garbage fallback list (illegal memory
access on the on-G1 path).  The 20,011-round tests never saw it (their
failures would have hit 1 item of 20k and were masked by the next step).

Here: batch sizes around the 5-item engine block, the 8-item compressed-chain
wave and the 64-item wave, per-round verify of the golden chained and on-G1
chains (items cycled from the fixture, so the last items are valid and
corrupted ones alike) and dgpu_verify_recovered over their digests, on
contexts with the Karabina fallback forced on every 3rd item and off.
Expected reasons come from the fixtures (tests/golden/make_golden.py)."""
import hashlib
import struct

import numpy as np
import pytest

from conftest import load_golden, open_ctx

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 8, 9, 15, 16, 17, 41]
FIXTURES = ["chain_chained_s1.json", "chain_on_g1_s1.json", "chain_g1_rfc9380_s2.json"]


def _items(g):
    """(prev, round, sig, reason) of the fixture's rounds and corruption catalog."""
    out = [(bytes.fromhex(r["prev"]), r["round"], bytes.fromhex(r["sig"]), 0) for r in g["rounds"]]
    out += [(bytes.fromhex(c["prev"]), c["round"], bytes.fromhex(c["sig"]), c["reason"]) for c in g["corrupted"]]
    return out


def _digest(chained, prev, rnd):
    """chain/verify.go:24-32 DigestMessage (host restatement for the test)."""
    h = hashlib.sha256()
    if chained:
        h.update(prev)
    h.update(struct.pack(">Q", rnd))
    return h.digest()


@pytest.fixture(scope="module", params=["default", "fallback3"])
def ctx(request):
    c = open_ctx({} if request.param == "default" else {"DGPU_KB_TEST_FLAG": "3"})
    yield c
    c.close()


@pytest.mark.parametrize("name", FIXTURES)
def test_ragged_batches_verify_and_verify_recovered(name, ctx):
    from drand_amd import _lib
    from drand_amd.chain import _pack_msgs, pack_beacons, Beacon
    from drand_amd.scheme import get_scheme_by_id_with_default
    from drand_amd.chain import scheme_code
    g = load_golden(name)
    sch = get_scheme_by_id_with_default(g["scheme"])
    code = scheme_code(sch)
    chained = not sch.decouple_prev_sig
    items = _items(g)
    pk = np.frombuffer(bytes.fromhex(g["pk"]), dtype=np.uint8).copy()
    lib = ctx.lib
    for n in SIZES:
        pick = [items[(n + i) % len(items)] for i in range(n)]  # the start moves with n
        expect = [it[3] for it in pick]
        beacons = [Beacon(p if chained else b"", r, s) for p, r, s, _ in pick]
        rounds, sigs, sig_len, prev, prev_len = pack_beacons(beacons)
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        _lib.check(lib.dgpu_verify_beacons(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(rounds),
                                           _lib.ptr(sigs), sigs.shape[1], _lib.ptr(sig_len), _lib.ptr(prev),
                                           prev.shape[1], _lib.ptr(prev_len), _lib.MODE_PER_ROUND, 0,
                                           _lib.ptr(bits), _lib.ptr(reason)))
        assert reason.tolist() == expect, (name, n)
        assert np.array_equal(np.unpackbits(bits, bitorder="little")[:n].astype(bool), reason == 0)
        # the same items as raw VerifyRecovered(pk, DigestMessage(...), sig)
        mb, ml = _pack_msgs([_digest(chained, p, r) for p, r, _, _ in pick])
        sb, sl = _pack_msgs([s for _, _, s, _ in pick])
        width = 96 if code in (_lib.SCHEME_CHAINED, _lib.SCHEME_UNCHAINED) else 48
        if sb.shape[1] < width:
            sb = np.pad(sb, ((0, 0), (0, width - sb.shape[1])))
        reason2 = np.zeros(n, dtype=np.uint8)
        bits[:] = 0
        _lib.check(lib.dgpu_verify_recovered(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(mb), mb.shape[1],
                                             _lib.ptr(ml), _lib.ptr(sb), sb.shape[1], _lib.ptr(sl),
                                             _lib.MODE_PER_ROUND, 0, _lib.ptr(bits), _lib.ptr(reason2)))
        assert reason2.tolist() == expect, (name, n, "recovered")
