"""Native ingest for the bulk check-chain path:
libdrand_ingest.so (drand_amd/csrc/ingest.cpp) walks a bolt bucket's B+tree
in key order and decodes canonical Beacon.Marshal rows straight into the
C ABI's fixed-stride records; every other row is decoded by
sync.beacon_unmarshal (hexjson's rules restated), so a window's records and
its undecodable rounds are exactly what Get + Unmarshal give
(chain/boltdb/store.go:113-132, chain/beacon.go:34-37).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdrand_ingest.so")
_lib = None
DECODE_THREADS = max(1, min(8, len(os.sched_getaffinity(0)) // 2))
_decode_pool = None


def _pool():
    global _decode_pool
    if _decode_pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _decode_pool = ThreadPoolExecutor(DECODE_THREADS)
    return _decode_pool


def load():
    """The native ingest library, or None when it is not built."""
    global _lib
    if _lib is None and os.path.exists(LIB_PATH):
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        L.dgpu_ingest_scan.restype = c.c_long
        L.dgpu_ingest_scan.argtypes = [c.c_void_p, c.c_size_t, c.c_size_t, c.c_uint64, c.c_uint64, c.c_uint64,
                                       c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
        L.dgpu_ingest_count.restype = c.c_long
        L.dgpu_ingest_count.argtypes = [c.c_void_p, c.c_size_t, c.c_size_t, c.c_uint64]
        L.dgpu_ingest_decode.restype = c.c_size_t
        L.dgpu_ingest_decode.argtypes = [c.c_size_t, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p,
                                         c.c_size_t, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p]
        _lib = L
    return _lib


class Records:
    """One window of decoded rows: `index` (position of each record's row in
    the window, i.e. round - lo), the fixed-stride records, and the window
    positions whose row is missing or does not unmarshal (faulty rounds)."""

    __slots__ = ("lo", "hi", "index", "rounds", "sigs", "sig_len", "prev", "prev_len", "bad")

    def __init__(self, lo, hi, index, rounds, sigs, sig_len, prev, prev_len, bad):
        self.lo, self.hi = lo, hi
        self.index, self.rounds, self.sigs, self.sig_len = index, rounds, sigs, sig_len
        self.prev, self.prev_len, self.bad = prev, prev_len, bad


def scan(buf, page_size, root_pgid, lo, hi):
    """(rounds, value offsets, value lengths) of the bucket's rows with lo <=
    round < hi, in key order (native B+tree walk over the mapped file)."""
    L = load()
    cap = max(0, hi - lo)
    rounds = np.zeros(cap, dtype=np.uint64)
    off = np.zeros(cap, dtype=np.uint64)
    ln = np.zeros(cap, dtype=np.uint32)
    n = L.dgpu_ingest_scan(buf.ctypes.data, buf.size, page_size, root_pgid, lo, hi, rounds.ctypes.data,
                           off.ctypes.data, ln.ctypes.data, cap)
    if n < 0:
        from .boltstore import BoltFormatError
        raise BoltFormatError("malformed bbolt page in the beacon bucket" if n == -1 else "scan overflow")
    return rounds[:n], off[:n], ln[:n]


def count(buf, page_size, root_pgid):
    """bucket.Stats().KeyN (every leaf element of the bucket's tree), natively."""
    n = load().dgpu_ingest_count(buf.ctypes.data, buf.size, page_size, root_pgid)
    if n < 0:
        from .boltstore import BoltFormatError
        raise BoltFormatError("malformed bbolt page in the beacon bucket")
    return n


def decode(buf, off, ln, raw=None, sig_stride=96, prev_stride=96):
    """Rows at buf[off:off+ln] -> fixed-stride records + ok mask.  Rows the
    native decoder leaves (ok = 0) are decoded by sync.beacon_unmarshal:
    decodable ones fill their record (sig longer than the stride -> length
    0xFFFFFFFF, a decode failure like pack_beacons; a longer PreviousSig
    widens the prev stride); the rest stay ok = 0 (Unmarshal error)."""
    from .sync import beacon_unmarshal
    L = load()
    n = len(off)
    rounds = np.zeros(n, dtype=np.uint64)
    sigs = np.zeros((n, sig_stride), dtype=np.uint8)
    sig_len = np.zeros(n, dtype=np.uint32)
    prev = np.zeros((n, prev_stride), dtype=np.uint8)
    prev_len = np.zeros(n, dtype=np.uint32)
    ok = np.zeros(n, dtype=np.uint8)
    if n:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ln = np.ascontiguousarray(ln, dtype=np.uint32)
    if n and L is not None:
        def part(a, b):
            L.dgpu_ingest_decode(b - a, buf.ctypes.data, off[a:].ctypes.data, ln[a:].ctypes.data,
                                 rounds[a:].ctypes.data, sigs[a:].ctypes.data, sig_stride, sig_len[a:].ctypes.data,
                                 prev[a:].ctypes.data, prev_stride, prev_len[a:].ctypes.data, ok[a:].ctypes.data)
        # the ctypes call releases the GIL: large windows decode on DECODE_THREADS threads
        k = max(1, min(DECODE_THREADS, n // 8192))
        cuts = [n * j // k for j in range(k + 1)]
        if k == 1:
            part(0, n)
        else:
            list(_pool().map(lambda j: part(cuts[j], cuts[j + 1]), range(k)))
    for i in np.nonzero(ok == 0)[0].tolist():
        try:
            b = beacon_unmarshal(bytes(buf[off[i]:off[i] + ln[i]]))
        except ValueError:
            continue
        ok[i] = 1
        rounds[i] = b.round
        s = b.signature
        if len(s) <= sig_stride:
            sigs[i, :len(s)] = np.frombuffer(s, dtype=np.uint8)
            sig_len[i] = len(s)
        else:
            sig_len[i] = 0xFFFFFFFF
        p = b.previous_sig
        if len(p) > prev.shape[1]:
            prev = np.pad(prev, ((0, 0), (0, len(p) - prev.shape[1])))
        prev[i, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        prev_len[i] = len(p)
    return rounds, sigs, sig_len, prev, prev_len, ok.astype(bool)


def window_records(store, lo, hi):
    """Records of rounds [lo, hi) of a BoltStore (native scan + decode)."""
    rr, off, ln, buf = store.scan_offsets(lo, hi)
    rounds, sigs, sig_len, prev, prev_len, ok = decode(buf, off, ln)
    present = np.zeros(hi - lo, dtype=bool)
    pos = (rr - np.uint64(lo)).astype(np.int64)
    present[pos] = True
    bad = ~present
    bad[pos[~ok]] = True
    keep = np.nonzero(ok)[0]
    return Records(lo, hi, pos[keep], rounds[keep], sigs[keep], sig_len[keep], prev[keep], prev_len[keep],
                   np.nonzero(bad)[0])
