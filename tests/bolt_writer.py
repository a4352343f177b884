"""Test-only writer of bbolt v1.3.4 database files (the format
drand_amd/boltstore.py reads; see its header), for fixtures of drand's bolt
beacon store: meta pages 0/1 (FNV-1a checksums), an empty freelist page, the
root bucket's leaf page naming the "beacons" bucket, and the bucket's B+tree
(leaves packed in key order, branch levels above them, overflow pages for
elements larger than a page) -- or the bucket inline in its root element when
it is small, as bbolt stores small buckets.  Go and bbolt are absent here, so
files bbolt itself wrote are not available: this writer and the reader share
one reading of the format ("parity unpinned" against bbolt)."""
import struct

from drand_amd.boltstore import (BRANCH_PAGE, BUCKET_LEAF_FLAG, ELEMENT, FREELIST_PAGE, LEAF_PAGE, MAGIC,
                                 META_PAGE, PAGE_HEADER, VERSION, fnv1a64)


def _page_bytes(pgid, flags, elems, page_size, branch):
    """One page (plus overflow pages if needed) holding `elems`:
    leaf: (flags, key, value); branch: (key, child pgid)."""
    n = len(elems)
    hdr_end = PAGE_HEADER + n * ELEMENT
    data = bytearray()
    ehdrs = bytearray()
    for i, e in enumerate(elems):
        pos = hdr_end + len(data) - (PAGE_HEADER + i * ELEMENT)
        if branch:
            key, child = e
            ehdrs += struct.pack("<IIQ", pos, len(key), child)
            data += key
        else:
            fl, key, val = e
            ehdrs += struct.pack("<IIII", fl, pos, len(key), len(val))
            data += key + val
    size = hdr_end + len(data)
    npages = -(-size // page_size)
    body = struct.pack("<QHHI", pgid, flags, n, npages - 1) + bytes(ehdrs) + bytes(data)
    return body + bytes(npages * page_size - len(body)), npages


def _inline_page(elems):
    body, _ = _page_bytes(0, LEAF_PAGE, elems, 1, False)
    size = PAGE_HEADER + len(elems) * ELEMENT + sum(len(k) + len(v) for _, k, v in elems)
    return body[:size]


def write_bolt(path, items, page_size=4096, bucket=b"beacons", fill=0.5, inline=None):
    """items: {key bytes: value bytes}; writes a bbolt file with one bucket."""
    keys = sorted(items)
    elems = [(0, k, items[k]) for k in keys]
    size = PAGE_HEADER + sum(ELEMENT + len(k) + len(v) for _, k, v in elems)
    if inline is None:
        inline = size <= page_size // 4
    pages = {}  # pgid -> bytes (multi-page blobs allowed)
    next_pg = 4
    if inline:
        bucket_val = struct.pack("<QQ", 0, 0) + _inline_page(elems)
    else:
        # leaves: pack elements until the page is `fill` full (always >= 1 element)
        level = []
        cur, cur_size = [], PAGE_HEADER
        for e in elems:
            esz = ELEMENT + len(e[1]) + len(e[2])
            if cur and cur_size + esz > page_size * fill:
                level.append(cur)
                cur, cur_size = [], PAGE_HEADER
            cur.append(e)
            cur_size += esz
        if cur or not level:
            level.append(cur)
        nodes = []
        for leaf in level:
            blob, npg = _page_bytes(next_pg, LEAF_PAGE, leaf, page_size, False)
            pages[next_pg] = blob
            nodes.append(((leaf[0][1] if leaf else b""), next_pg))
            next_pg += npg
        while len(nodes) > 1:
            per = max(2, int(page_size * fill) // (ELEMENT + 8))
            up = []
            for j in range(0, len(nodes), per):
                grp = nodes[j:j + per]
                blob, npg = _page_bytes(next_pg, BRANCH_PAGE, grp, page_size, True)
                pages[next_pg] = blob
                up.append((grp[0][0], next_pg))
                next_pg += npg
            nodes = up
        bucket_val = struct.pack("<QQ", nodes[0][1], 0)
    root_blob, _ = _page_bytes(3, LEAF_PAGE, [(BUCKET_LEAF_FLAG, bucket, bucket_val)], page_size, False)
    free_blob = struct.pack("<QHHI", 2, FREELIST_PAGE, 0, 0) + bytes(page_size - PAGE_HEADER)
    high_water = next_pg

    def meta(pgid, txid):
        m = struct.pack("<IIIIQQQQQ", MAGIC, VERSION, page_size, 0, 3, 0, 2, high_water, txid)
        m += struct.pack("<Q", fnv1a64(m))
        return (struct.pack("<QHHI", pgid, META_PAGE, 0, 0) + m).ljust(page_size, b"\0")

    out = bytearray(meta(0, 0) + meta(1, 1) + free_blob + root_blob)
    for pg in sorted(pages):
        assert len(out) == pg * page_size
        out += pages[pg]
    with open(path, "wb") as f:
        f.write(out)
