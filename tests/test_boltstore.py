"""Read-only bolt beacon store (drand_amd/boltstore.py) for check-chain ingest:
the read side of chain/boltdb/store.go (Len / Last / Get) over bbolt files,
and CheckPastBeacons fed from it.  The files come from tests/bolt_writer.py
(Go and bbolt are absent, so parity with bbolt-written files is unpinned);
the semantics are checked against the in-memory store and the oracle's
restatement of the loop."""
import random
import struct

import pytest

from bolt_writer import write_bolt
from drand_amd.boltstore import BoltFormatError, BoltStore, fnv1a64
from drand_amd.chain import Beacon
from drand_amd.sync import ErrNoBeaconSaved, MemoryStore, beacon_marshal, check_past_beacons
from oracle import drand_ref as D
from test_sync import MarkerVerifier


def _kv(st: MemoryStore):
    return dict(st._kv)


def _random_store(rng, n, big=None):
    st = MemoryStore()
    table = {0: (0, b"", b"genesis")}
    st.put(Beacon(b"", 0, b"genesis"))
    for r in range(1, n + 1):
        if rng.random() < 0.04:
            continue  # missing row
        if rng.random() < 0.01:
            st.put_raw(r, b"not json")  # unmarshal error: faulty, like the reference's Get
            table[r] = None
            continue
        rr = r if rng.random() > 0.02 else r + 7  # stored beacon with a different Round field
        sig = (b"BAD" if rng.random() < 0.1 else b"ok") + r.to_bytes(4, "big")
        prev = bytes(rng.randrange(256) for _ in range(big if big and r % 97 == 0 else 96))
        st.put_raw(r, beacon_marshal(Beacon(prev, rr, sig)))
        table[r] = (rr, prev, sig)
    return st, table


def test_reference_store_test_semantics(tmp_path):
    """chain/boltdb/store_test.go TestStoreBolt / TestStoreBoltOrder: Len counts
    keys, Last is the highest round whatever the insertion order, Get returns
    the stored beacon, a missing round is ErrNoBeaconSaved."""
    b1 = Beacon(bytes([1, 2, 3]), 145, bytes([2, 3, 4]))
    b2 = Beacon(bytes([2, 3, 4]), 146, bytes([1, 2, 3]))
    for order in ((b2, b1), (b1, b2)):
        st = MemoryStore()
        for b in order:
            st.put(b)
        p = tmp_path / "drand.db"
        write_bolt(p, _kv(st))
        bs = BoltStore(p)
        assert bs.len() == 2 and bs.last() == b2
        assert bs.get(145) == b1 and bs.get(146) == b2
        with pytest.raises(ErrNoBeaconSaved):
            bs.get(147)
        bs.close()


@pytest.mark.parametrize("n,inline,big", [(3, True, None), (40, False, None), (3000, False, None), (600, False, 9000)])
def test_bolt_store_equals_memory_store(tmp_path, n, inline, big):
    """Inline bucket, one leaf, a three-level tree, and leaves with overflow
    pages (a 9,000-byte PreviousSig): Len / Last / Get / scan agree with the
    in-memory store row for row."""
    st, _ = _random_store(random.Random(n), n, big)
    p = tmp_path / "drand.db"
    write_bolt(p, _kv(st), inline=inline)
    bs = BoltStore(p)
    assert bs.len() == st.len()
    assert bs.last() == st.last()
    for r in range(0, n + 3):
        try:
            want = st.get(r)
        except (ErrNoBeaconSaved, ValueError) as e:
            want = type(e)
        try:
            got = bs.get(r)
        except (ErrNoBeaconSaved, ValueError) as e:
            got = type(e)
        assert got == want, r
    lo, hi = n // 3, 2 * n // 3 + 1
    assert list(bs.scan(lo, hi)) == [(r, v) for r, v in sorted(
        (struct.unpack(">Q", k)[0], v) for k, v in _kv(st).items()) if lo <= r < hi]
    bs.close()


@pytest.mark.parametrize("window", [1, 5, 64, 1 << 16])
def test_check_past_beacons_from_bolt(tmp_path, window):
    """CheckPastBeacons over the bolt file (windowed ordered scans) gives the
    same faulty list and progress callbacks as over the in-memory store and
    as the oracle's restatement of chain/beacon/sync_manager.go:171-232."""
    rng = random.Random(window)
    st, table = _random_store(rng, 700)
    p = tmp_path / "drand.db"
    write_bolt(p, _kv(st))
    bs = BoltStore(p)
    for up_to in (0, 1, 350, 10 ** 9):  # 0: round 1 is still checked (the loop breaks after it)
        c1, c2 = [], []
        got = check_past_beacons(bs, MarkerVerifier(), b"pk", up_to, cb=lambda i, u: c1.append((i, u)), window=window)
        mem = check_past_beacons(st, MarkerVerifier(), b"pk", up_to, cb=lambda i, u: c2.append((i, u)), window=window)
        tab = {r: v for r, v in table.items() if v is not None}
        for r in (r for r, v in table.items() if v is None):
            tab[r] = (r, b"", b"BAD-unmarshal")  # the oracle's table has no raw rows: faulty either way
        exp, progress = D.check_past_beacons(tab, up_to, lambda b: not b[2].startswith(b"BAD"))
        assert got == mem == exp
        assert c1 == c2 == progress
    bs.close()


def test_meta_selection_and_errors(tmp_path):
    """The valid meta page with the larger txid is current; a bad checksum on
    it falls back to the other; no valid meta, a missing bucket or an empty
    bucket are reported like bbolt / the store do."""
    st, _ = _random_store(random.Random(1), 50)
    p = tmp_path / "drand.db"
    write_bolt(p, _kv(st))
    raw = bytearray(p.read_bytes())
    assert BoltStore(p).txid == 1
    raw[4096 + 16 + 40] ^= 1  # page 1's txid: checksum no longer matches
    p.write_bytes(bytes(raw))
    bs = BoltStore(p)
    assert bs.txid == 0 and bs.last() == st.last()
    bs.close()
    raw[16 + 40] ^= 1
    p.write_bytes(bytes(raw))
    with pytest.raises(BoltFormatError):
        BoltStore(p)
    q = tmp_path / "other.db"
    write_bolt(q, _kv(st), bucket=b"other")
    with pytest.raises(BoltFormatError):
        BoltStore(q)
    e = tmp_path / "empty.db"
    write_bolt(e, {})
    be = BoltStore(e)
    assert be.len() == 0
    with pytest.raises(ErrNoBeaconSaved):
        be.last()
    be.close()
    assert fnv1a64(b"") == 0xCBF29CE484222325 and fnv1a64(b"a") == 0xAF63DC4C8601EC8C  # FNV-1a-64 test vectors


def test_torn_meta0_opens_from_meta1(tmp_path):
    """bbolt v1.3.4 Open: when meta 0 fails validation its page size is not
    trusted (the OS page size is assumed) and the file opens from meta 1
    (ADVICE r02).  Page 0's checksum broken, then its page-size field
    garbage as well: both open from page 1 (txid 1)."""
    st, _ = _random_store(random.Random(2), 80)
    p = tmp_path / "drand.db"
    write_bolt(p, _kv(st))
    raw = bytearray(p.read_bytes())
    raw[16 + 40] ^= 1  # page 0's txid: checksum mismatch
    p.write_bytes(bytes(raw))
    bs = BoltStore(p)
    assert bs.txid == 1 and bs.page_size == 4096 and bs.last() == st.last() and bs.len() == st.len()
    bs.close()
    raw[16 + 8:16 + 12] = struct.pack("<I", 123457)  # page 0's pageSize: garbage
    p.write_bytes(bytes(raw))
    bs = BoltStore(p)
    assert bs.txid == 1 and bs.last() == st.last() and bs.len() == st.len()
    bs.close()
    # a 16 KiB-page file whose meta 0 is torn: bbolt v1.3.4 looks for meta 1
    # one OS page in only and refuses it; the opt-in lenient mode
    # (a documented deviation) also probes 16 KiB and opens it
    q = tmp_path / "big.db"
    write_bolt(q, _kv(st), page_size=16384)
    raw = bytearray(q.read_bytes())
    raw[16 + 40] ^= 1
    q.write_bytes(bytes(raw))
    import mmap
    if mmap.PAGESIZE != 16384:
        with pytest.raises(BoltFormatError):
            BoltStore(q)
    bq = BoltStore(q, lenient_page_size=True)
    assert bq.txid == 1 and bq.page_size == 16384 and bq.last() == st.last()
    bq.close()


# hexjson rows the native decoder must leave to beacon_unmarshal (or decode
# identically): whitespace, key order and case, null fields, uppercase hex,
# Round edge cases, escapes, odd / non-hex strings, lengths past the stride
MALFORMED = [
    b'{"PreviousSig":"aa","Round":5,"Signature":"bb"}',
    b'{"PreviousSig":null,"Round":6,"Signature":"CC"}',
    b'{"PreviousSig":"","Round":7,"Signature":null}',
    b'{"Round":8,"PreviousSig":"aa","Signature":"bb"}',
    b'{"previoussig":"aa","round":9,"signature":"bb"}',
    b'{ "PreviousSig":"aa","Round":10,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":011,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":12.0,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":-13,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":18446744073709551615,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":18446744073709551616,"Signature":"bb"}',
    b'{"PreviousSig":"a","Round":15,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":16,"Signature":"b b"}',
    b'{"PreviousSig":"aa","Round":17,"Signature":"zz"}',
    b'{"PreviousSig":"\\u0061a","Round":18,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":19,"Signature":"bb"}  ',
    b'{"PreviousSig":"aa","Round":20,"Signature":"bb","Extra":1}',
    b'{"PreviousSig":"aa","Round":21,"Round":22,"Signature":"bb"}',
    b'{"PreviousSig":"aa","Round":23,"Signature":"bb"',
    b'not json',
    b'[1,2,3]',
    b'{"PreviousSig":"' + b"ab" * 200 + b'","Round":24,"Signature":"' + b"cd" * 96 + b'"}',
    b'{"PreviousSig":"ab","Round":25,"Signature":"' + b"cd" * 150 + b'"}',
    b'{"PreviousSig":"ab","Round":26,"Signature":7}',
    b'{"PreviousSig":"ab","Round":true,"Signature":"cd"}',
    b'{}',
    b'{"PreviousSig":"AbCd","Round":0,"Signature":"' + b"Ef" * 96 + b'"}',
]


def test_native_decoder_equals_beacon_unmarshal(tmp_path):
    """The native window decode (drand_amd/ingest.py over libdrand_ingest.so)
    gives, row for row, what beacon_unmarshal gives: the same record, or an
    Unmarshal error for the same rows."""
    import numpy as np
    from drand_amd import ingest
    from drand_amd.sync import beacon_unmarshal
    assert ingest.load() is not None, "libdrand_ingest.so not built"
    kv = {struct.pack(">Q", 100 + i): v for i, v in enumerate(MALFORMED)}
    kv[struct.pack(">Q", 0)] = b'{"PreviousSig":null,"Round":0,"Signature":"00"}'
    p = tmp_path / "drand.db"
    write_bolt(p, kv)
    bs = BoltStore(p)
    rec = ingest.window_records(bs, 100, 100 + len(MALFORMED))
    bad = set(rec.bad.tolist())
    got = {int(j): k for k, j in enumerate(rec.index)}
    for i, v in enumerate(MALFORMED):
        try:
            want = beacon_unmarshal(v)
        except ValueError:
            assert i in bad and i not in got, v
            continue
        assert i in got, v
        k = got[i]
        assert int(rec.rounds[k]) == want.round, v
        sl = int(rec.sig_len[k])
        if len(want.signature) > rec.sigs.shape[1]:
            assert sl == 0xFFFFFFFF
        else:
            assert bytes(rec.sigs[k, :sl]) == want.signature and not rec.sigs[k, sl:].any(), v
        assert bytes(rec.prev[k, :rec.prev_len[k]]) == want.previous_sig, v
    assert len(got) + len(bad) == len(MALFORMED)
    bs.close()


def test_native_scan_equals_python_scan(tmp_path):
    """The native B+tree walk returns the Python reader's rows (multi-level
    tree, overflow pages, a missing row range at both window ends)."""
    import numpy as np
    from drand_amd import ingest
    st, _ = _random_store(random.Random(7), 3000, 9000)
    p = tmp_path / "drand.db"
    write_bolt(p, _kv(st))
    bs = BoltStore(p)
    assert bs._b.inline is None
    buf = bs.buffer()
    for lo, hi in ((0, 3001), (1, 2), (500, 1500), (2990, 4000), (5000, 6000)):
        rr, off, ln = ingest.scan(buf, bs.page_size, bs._b.root, lo, hi)
        want = list(bs.scan(lo, hi))
        assert rr.tolist() == [r for r, _ in want]
        assert [bytes(buf[o:o + n]) for o, n in zip(off, ln)] == [v for _, v in want]
    bs.close()


@pytest.mark.timeout(60)
def test_native_walk_rejects_self_referencing_branch_page():
    """A crafted branch page whose 254 children all point back to itself (a
    cycle, never produced by bbolt) must be rejected as malformed by the
    native walk and count instead of taking 254^64 steps: the
    walk stops after as many page visits as the file has pages."""
    import numpy as np
    from drand_amd import ingest
    ps, pg = 4096, 2
    f = bytearray(3 * ps)
    count = 254
    base = pg * ps
    struct.pack_into("<QHHI", f, base, pg, 0x01, count, 0)  # branch page, no overflow
    key_off = base + 16 + count * 16  # one 8-byte key shared by every element
    struct.pack_into(">Q", f, key_off, 1)
    for i in range(count):
        e = base + 16 + 16 * i
        struct.pack_into("<IIQ", f, e, key_off - e, 8, pg)  # pos, ksize, child = this page
    buf = np.frombuffer(bytes(f), dtype=np.uint8)
    with pytest.raises(BoltFormatError):
        ingest.scan(buf, ps, pg, 0, 1 << 16)
    with pytest.raises(BoltFormatError):
        ingest.count(buf, ps, pg)
