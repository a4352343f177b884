"""Read-only reader of drand's bolt beacon store, for check-chain ingest
(SURVEY.md 8(f) row 2): a drand node's `drand.db` walked straight into the
batched CheckPastBeacons mirror (drand_amd/sync.py) without a Go process.

Mirrors the read side of chain/boltdb/store.go:
  NewBoltStore / bucket "beacons"        chain/boltdb/store.go:20-50
  Len  (bucket.Stats().KeyN)             :52-63
  Last (cursor.Last, Beacon.Unmarshal)   :90-108
  Get  (bucket.Get(RoundToBytes(round))) :110-128
Keys are RoundToBytes(round) = BE64 (chain/store.go:42-46), so key order is
round order; values are Beacon.Marshal JSON (chain/beacon.go:29-37).

The file format is go.etcd.io/bbolt v1.3.4's (go.mod:37; the module is not in
the reference snapshot): pages of `page_size` bytes, each with a 16-byte
header (id u64, flags u16, count u16, overflow u32) -- a page with overflow k
spans k + 1 pages; meta pages 0 and 1 (magic 0xED0CDAED, version 2, page
size, flags, root bucket {root pgid, sequence}, freelist pgid, high-water
pgid, txid, FNV-1a-64 checksum of the preceding 56 bytes), the valid one with
the larger txid is current; branch elements (pos u32, ksize u32, pgid u64)
and leaf elements (flags u32, pos u32, ksize u32, vsize u32), 16 bytes each,
with pos relative to the element; a leaf element with flags & 1 is a nested
bucket whose value starts with {root pgid u64, sequence u64} and, when root
is 0, holds the bucket's single page inline right after it.

Reads go through mmap; nothing is written.  `scan(lo, hi)` walks the B+tree
in key order and is what the windowed ingest uses (one pass over the leaves,
not one tree search per round).
"""
import mmap
import struct

from .sync import ErrNoBeaconSaved, beacon_unmarshal

MAGIC = 0xED0CDAED
VERSION = 2
PAGE_HEADER = 16
ELEMENT = 16
BUCKET_HEADER = 16
BRANCH_PAGE, LEAF_PAGE, META_PAGE, FREELIST_PAGE = 0x01, 0x02, 0x04, 0x10
BUCKET_LEAF_FLAG = 0x01


class BoltFormatError(ValueError):
    """The file is not a bbolt database this reader understands."""


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for b in data:
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


class _Node:
    """One B+tree page (or an inline bucket's page): its kind and elements."""
    __slots__ = ("leaf", "keys", "vals", "flags", "children")

    def __init__(self, buf, off):
        _pid, flags, count, _ovf = struct.unpack_from("<QHHI", buf, off)
        base = off + PAGE_HEADER
        self.keys = []
        if flags & LEAF_PAGE:
            self.leaf = True
            self.vals, self.flags, self.children = [], [], None
            for i in range(count):
                e = base + i * ELEMENT
                fl, pos, ks, vs = struct.unpack_from("<IIII", buf, e)
                k0 = e + pos
                self.keys.append(bytes(buf[k0:k0 + ks]))
                self.vals.append(bytes(buf[k0 + ks:k0 + ks + vs]))
                self.flags.append(fl)
        elif flags & BRANCH_PAGE:
            self.leaf = False
            self.vals = self.flags = None
            self.children = []
            for i in range(count):
                e = base + i * ELEMENT
                pos, ks, pgid = struct.unpack_from("<IIQ", buf, e)
                self.keys.append(bytes(buf[e + pos:e + pos + ks]))
                self.children.append(pgid)
        else:
            raise BoltFormatError(f"page at offset {off}: flags 0x{flags:x} is neither a branch nor a leaf")


class _Bucket:
    def __init__(self, db, value: bytes):
        if len(value) < BUCKET_HEADER:
            raise BoltFormatError("bucket value shorter than its header")
        self.db = db
        self.root, self.sequence = struct.unpack_from("<QQ", value, 0)
        self.inline = _Node(value, BUCKET_HEADER) if self.root == 0 else None

    def node(self, pgid=None):
        if pgid is None and self.inline is not None:
            return self.inline
        return self.db.page_node(self.root if pgid is None else pgid)

    def items(self, lo=None):
        """(key, value, flags) in key order, starting at the first key >= lo."""
        stack = [self.node()]
        # descend to the first leaf that can hold lo
        while not stack[-1].leaf:
            n = stack[-1]
            i = 0
            if lo is not None:
                while i + 1 < len(n.keys) and n.keys[i + 1] <= lo:
                    i += 1
            stack[-1] = (n, i)
            stack.append(self.node(n.children[i]))
        leaf = stack.pop()
        path = stack  # [(branch, index)]
        while True:
            for k, v, f in zip(leaf.keys, leaf.vals, leaf.flags):
                if lo is None or k >= lo:
                    yield k, v, f
            # next leaf: climb to the first branch with a right sibling
            while path and path[-1][1] + 1 >= len(path[-1][0].children):
                path.pop()
            if not path:
                return
            n, i = path.pop()
            path.append((n, i + 1))
            nxt = self.node(n.children[i + 1])
            while not nxt.leaf:
                path.append((nxt, 0))
                nxt = self.node(nxt.children[0])
            leaf = nxt
            lo = None

    def get(self, key: bytes):
        n = self.node()
        while not n.leaf:
            i = 0
            while i + 1 < len(n.keys) and n.keys[i + 1] <= key:
                i += 1
            n = self.node(n.children[i])
        for k, v, f in zip(n.keys, n.vals, n.flags):
            if k == key:
                return None if f & BUCKET_LEAF_FLAG else v
        return None

    def last(self):
        n = self.node()
        while not n.leaf:
            n = self.node(n.children[-1])
        return (n.keys[-1], n.vals[-1]) if n.keys else None

    def key_n(self):
        """bucket.Stats().KeyN: every leaf element of this bucket's tree."""
        def count(n):
            if n.leaf:
                return len(n.keys)
            return sum(count(self.node(c)) for c in n.children)
        return count(self.node())


class BoltStore:
    """chain.Store's read side over a drand bolt file (read-only)."""

    def __init__(self, path, bucket=b"beacons", lenient_page_size=False):
        """lenient_page_size (opt-in DEVIATION from bbolt v1.3.4): when meta 0
        is torn, also try 4/8/16/64 KiB for meta 1 instead of only the OS
        page size -- opens files the reference refuses (a file written with
        another page size whose meta 0 is damaged)."""
        self._lenient = lenient_page_size
        self._f = open(path, "rb")
        try:
            self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        except ValueError:
            self._f.close()
            raise BoltFormatError(f"{path}: empty file") from None
        self._cache = {}
        meta = self._meta()
        self.page_size = meta["page_size"]
        self.txid = meta["txid"]
        root = _Bucket(self, struct.pack("<QQ", meta["root"], meta["sequence"]))
        v = None
        for k, val, f in root.items():
            if k == bucket and f & BUCKET_LEAF_FLAG:
                v = val
                break
        if v is None:
            raise BoltFormatError(f"{path}: no bucket {bucket!r}")
        self._b = _Bucket(self, v)
        self._buf = None

    def _read_meta(self, off):
        """The meta at byte offset `off` (a page start), or None if it fails
        bbolt's meta.validate (magic, version, checksum)."""
        mm = self._mm
        off += PAGE_HEADER
        if off + 64 > len(mm):
            return None
        magic, ver, psize, flags, root, seq, freelist, hw, txid, chk = struct.unpack_from("<IIIIQQQQQQ", mm, off)
        if magic != MAGIC or ver != VERSION or chk != fnv1a64(mm[off:off + 56]):
            return None
        return {"page_size": psize, "root": root, "sequence": seq, "freelist": freelist, "hw": hw, "txid": txid}

    def _meta(self):
        """bbolt v1.3.4 DB.Open + DB.meta: the page size comes from meta 0 only
        if meta 0 validates; otherwise bbolt assumes the OS page size (the
        size the file was created with) and finds meta 1 one page later.
        Then the valid meta with the larger txid is current.  Like bbolt,
        only the OS page size is tried for meta 1 when meta 0 is torn (a
        file with another page size then fails to open, as in the
        reference) unless the store was opened with lenient_page_size."""
        mm = self._mm
        if len(mm) < 2 * 1024:
            raise BoltFormatError("file shorter than two meta pages")
        m0 = self._read_meta(0)
        if m0 is not None:
            sizes = [m0["page_size"]]
        else:
            sizes = [mmap.PAGESIZE]
            if self._lenient:
                sizes += [s for s in (4096, 8192, 16384, 65536) if s != mmap.PAGESIZE]
        best = m0
        for ps in sizes:
            m1 = self._read_meta(ps)
            if m1 is None or (m0 is None and m1["page_size"] != ps):
                continue
            if best is None or m1["txid"] > best["txid"]:
                best = m1
            break
        if best is None:
            raise BoltFormatError("no valid meta page")
        return best

    def page_node(self, pgid):
        n = self._cache.get(pgid)
        if n is None:
            off = pgid * self.page_size
            if off + PAGE_HEADER > len(self._mm):
                raise BoltFormatError(f"page {pgid} past the end of the file")
            n = _Node(self._mm, off)
            if len(self._cache) > 4096:
                self._cache.clear()
            self._cache[pgid] = n
        return n

    def close(self):
        self._cache.clear()
        self._buf = None
        try:
            self._mm.close()
        except BufferError:  # arrays over the mapping still alive: it closes with them
            pass
        self._f.close()

    def buffer(self):
        """The mapped file as a read-only uint8 array (native ingest input)."""
        if self._buf is None:
            import numpy as np
            self._buf = np.frombuffer(self._mm, dtype=np.uint8)
        return self._buf

    def scan_offsets(self, lo, hi):
        """(rounds, value offsets, value lengths, buffer) of the rows with
        lo <= round < hi in key order: the native B+tree walk over the
        mapped file (drand_amd/ingest.py) when the bucket has its own pages,
        else this reader's walk with the values copied into a small buffer."""
        import numpy as np
        from . import ingest
        if self._b.inline is None and ingest.load() is not None:
            rr, off, ln = ingest.scan(self.buffer(), self.page_size, self._b.root, lo, hi)
            return rr, off, ln, self.buffer()
        rows = list(self.scan(lo, hi))
        ln = np.array([len(v) for _, v in rows], dtype=np.uint32)
        off = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)[:-1]]).astype(np.uint64) if rows else \
            np.zeros(0, dtype=np.uint64)
        buf = np.frombuffer(b"".join(v for _, v in rows) or b"\0", dtype=np.uint8)
        return np.array([r for r, _ in rows], dtype=np.uint64), off, ln, buf

    # ---- chain.Store (read side)
    def len(self):
        from . import ingest
        if self._b.inline is None and ingest.load() is not None:
            return ingest.count(self.buffer(), self.page_size, self._b.root)
        return self._b.key_n()

    def last(self):
        kv = self._b.last()
        if kv is None:
            raise ErrNoBeaconSaved("no beacon saved")
        return beacon_unmarshal(kv[1])

    def get(self, round_):
        v = self._b.get(struct.pack(">Q", round_))
        if v is None:
            raise ErrNoBeaconSaved(round_)
        return beacon_unmarshal(v)

    def scan(self, lo, hi):
        """Stored (round, raw value) for lo <= round < hi, in round order."""
        for k, v, f in self._b.items(struct.pack(">Q", lo)):
            if f & BUCKET_LEAF_FLAG or len(k) != 8:
                continue
            r = struct.unpack(">Q", k)[0]
            if r >= hi:
                return
            yield r, v
