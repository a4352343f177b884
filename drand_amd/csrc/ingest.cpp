// libdrand_ingest.so: host-side ingest for the bulk check-chain path
//  -- the rows of a drand bolt beacon store walked and
// decoded natively, straight into the fixed-stride records of the C ABI
// (include/drand_gpu.h), so that feeding the GPU is not bound by Python.
//
// Mirrors the read side of chain/boltdb/store.go:
//   Cursor walk of bucket "beacons"      :141-151 (key = RoundToBytes(round), chain/store.go:42-46)
//   Get + Beacon.Unmarshal               :113-132, chain/beacon.go:34-37 (hexjson)
// over the bbolt v1.3.4 page format (go.mod:37; restated in drand_amd/boltstore.py,
// which keeps the meta / bucket lookup and every non-canonical row).
//
// dgpu_ingest_decode accepts only the canonical Beacon.Marshal layout
//   {"PreviousSig":<hex or null>,"Round":<uint64>,"Signature":<hex or null>}
// (Go's encoding order, no whitespace); any other row -- whitespace, escapes,
// other key order or case, odd or non-hex strings, bytes beyond the stride,
// a Round that is not a canonical uint64 -- is left to the Python decoder
// (drand_amd/sync.py beacon_unmarshal), which mirrors hexjson's rules.
// Nothing here links HIP; the library is plain C++.
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace {

constexpr int PAGE_HEADER = 16, ELEMENT = 16;
constexpr uint16_t BRANCH_PAGE = 0x01, LEAF_PAGE = 0x02;
constexpr uint32_t BUCKET_LEAF_FLAG = 0x01;

inline uint16_t rd16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

// byte-wise key order (bbolt compares keys with bytes.Compare)
inline int key_cmp(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
  const size_t n = na < nb ? na : nb;
  const int c = memcmp(a, b, n);
  if (c) return c;
  return na < nb ? -1 : na > nb ? 1 : 0;
}

struct scan_state {
  const uint8_t* file;
  size_t file_len, page_size;
  uint8_t lo[8], hi[8];
  uint64_t* rounds;
  uint64_t* off;
  uint32_t* len;
  size_t cap, n;
  int depth;
  bool done;
  size_t visits;  // page visits left: a well-formed tree visits each page at most once
};

// -1: malformed file; -2: output full; 0: ok
int scan_page(scan_state& S, uint64_t pgid) {
  if (S.done) return 0;
  if (++S.depth > 64) return -1;
  // a crafted branch page pointing back into the tree (itself, an ancestor)
  // would make the walk exponential: more visits than the file has pages is
  // a malformed file
  if (S.visits == 0) return -1;
  --S.visits;
  if (pgid > (S.file_len - PAGE_HEADER) / S.page_size) return -1;
  const size_t po = (size_t)pgid * S.page_size;
  const uint8_t* p = S.file + po;
  const uint16_t flags = rd16(p + 8), count = rd16(p + 10);
  const uint64_t span = ((uint64_t)rd32(p + 12) + 1) * S.page_size;
  if (po + span > S.file_len || (size_t)PAGE_HEADER + (size_t)count * ELEMENT > span) return -1;
  const uint8_t* base = p + PAGE_HEADER;
  if (flags & BRANCH_PAGE) {
    for (int i = 0; i < count && !S.done; ++i) {
      const uint8_t* e = base + (size_t)i * ELEMENT;
      const size_t ko = (size_t)(e - S.file) + rd32(e), ks = rd32(e + 4);
      if (ko + ks > S.file_len) return -1;
      // child i holds keys in [key_i, key_{i+1}): skip it when key_{i+1} <= lo
      if (i + 1 < count) {
        const uint8_t* e2 = e + ELEMENT;
        const size_t ko2 = (size_t)(e2 - S.file) + rd32(e2), ks2 = rd32(e2 + 4);
        if (ko2 + ks2 > S.file_len) return -1;
        if (key_cmp(S.file + ko2, ks2, S.lo, 8) <= 0) continue;
      }
      if (i > 0 && key_cmp(S.file + ko, ks, S.hi, 8) >= 0) {
        S.done = true;
        break;
      }
      const int rc = scan_page(S, rd64(e + 8));
      if (rc) return rc;
    }
  } else if (flags & LEAF_PAGE) {
    for (int i = 0; i < count; ++i) {
      const uint8_t* e = base + (size_t)i * ELEMENT;
      const uint32_t fl = rd32(e), pos = rd32(e + 4), ks = rd32(e + 8), vs = rd32(e + 12);
      const size_t ko = (size_t)(e - S.file) + pos;
      if (ko + (size_t)ks + vs > S.file_len) return -1;
      const uint8_t* k = S.file + ko;
      if (key_cmp(k, ks, S.lo, 8) < 0) continue;
      if (key_cmp(k, ks, S.hi, 8) >= 0) {
        S.done = true;
        break;
      }
      if ((fl & BUCKET_LEAF_FLAG) || ks != 8) continue;
      if (S.n == S.cap) return -2;
      uint64_t r = 0;
      for (int b = 0; b < 8; ++b) r = (r << 8) | k[b];
      S.rounds[S.n] = r;
      S.off[S.n] = ko + ks;
      S.len[S.n] = vs;
      ++S.n;
    }
  } else {
    return -1;
  }
  --S.depth;
  return 0;
}

// hex digit value, -1 for any other byte
struct hex_lut {
  int8_t v[256];
  constexpr hex_lut() : v() {
    for (int i = 0; i < 256; ++i) v[i] = -1;
    for (int i = 0; i < 10; ++i) v['0' + i] = (int8_t)i;
    for (int i = 0; i < 6; ++i) {
      v['a' + i] = (int8_t)(10 + i);
      v['A' + i] = (int8_t)(10 + i);
    }
  }
};
constexpr hex_lut HEX{};

inline bool lit(const uint8_t*& p, const uint8_t* end, const char* s, size_t n) {
  if ((size_t)(end - p) < n || memcmp(p, s, n)) return false;
  p += n;
  return true;
}
#define LIT(p, end, s) lit(p, end, s, sizeof(s) - 1)

// "<hex>" or null -> out (stride bytes), *len; false = not canonical
inline bool hex_field(const uint8_t*& p, const uint8_t* end, uint8_t* out, size_t stride, uint32_t* len) {
  if (LIT(p, end, "null")) {
    *len = 0;
    return true;
  }
  if (p >= end || *p != '"') return false;
  ++p;
  size_t k = 0;
  while (p + 1 < end) {
    const int a = HEX.v[p[0]];
    if (a < 0) break;
    const int b = HEX.v[p[1]];
    if (b < 0 || k == stride) return false;
    out[k++] = (uint8_t)(a << 4 | b);
    p += 2;
  }
  if (p >= end || *p != '"') return false;  // odd length, a non-hex byte, or no closing quote
  *len = (uint32_t)k;
  ++p;
  return true;
}

// leaf elements under page pgid (bucket.Stats().KeyN counts every leaf
// element of the bucket's tree); -1: malformed
long count_page(const uint8_t* file, size_t file_len, size_t ps, uint64_t pgid, int depth, size_t& visits) {
  if (depth > 64 || pgid > (file_len - PAGE_HEADER) / ps) return -1;
  if (visits == 0) return -1;  // more page visits than pages: a cycle (see scan_page)
  --visits;
  const uint8_t* p = file + (size_t)pgid * ps;
  const uint16_t flags = rd16(p + 8), count = rd16(p + 10);
  if ((size_t)pgid * ps + PAGE_HEADER + (size_t)count * ELEMENT > file_len) return -1;
  if (flags & LEAF_PAGE) return count;
  if (!(flags & BRANCH_PAGE)) return -1;
  long total = 0;
  for (int i = 0; i < count; ++i) {
    const long c = count_page(file, file_len, ps, rd64(p + PAGE_HEADER + (size_t)i * ELEMENT + 8), depth + 1, visits);
    if (c < 0) return -1;
    total += c;
  }
  return total;
}

}  // namespace

extern "C" {

// bucket.Stats().KeyN of the bucket rooted at root_pgid (chain/boltdb/store.go
// Len, :51-62); -1 for a malformed file.
long dgpu_ingest_count(const uint8_t* file, size_t file_len, size_t page_size, uint64_t root_pgid) {
  if (!file || page_size < 64 || file_len < 2 * page_size) return -1;
  size_t visits = file_len / page_size;
  return count_page(file, file_len, page_size, root_pgid, 0, visits);
}

// In-order walk of a bucket's B+tree (bbolt pages of page_size bytes in the
// mapped file, root page root_pgid) collecting the elements whose key k
// satisfies BE64(lo) <= k < BE64(hi), skipping nested buckets and keys that
// are not 8 bytes: rounds_out[i] = the key as a round, val_off[i] / val_len[i]
// = the value's byte range in the file.  Returns the row count, -1 for a
// malformed file, -2 when more than cap rows fall in the range.
long dgpu_ingest_scan(const uint8_t* file, size_t file_len, size_t page_size, uint64_t root_pgid, uint64_t lo,
                      uint64_t hi, uint64_t* rounds_out, uint64_t* val_off, uint32_t* val_len, size_t cap) {
  if (!file || page_size < 64 || file_len < 2 * page_size) return -1;
  scan_state S{};
  S.file = file;
  S.file_len = file_len;
  S.page_size = page_size;
  S.visits = file_len / page_size;
  for (int b = 0; b < 8; ++b) {
    S.lo[b] = (uint8_t)(lo >> (56 - 8 * b));
    S.hi[b] = (uint8_t)(hi >> (56 - 8 * b));
  }
  S.rounds = rounds_out;
  S.off = val_off;
  S.len = val_len;
  S.cap = cap;
  const int rc = scan_page(S, root_pgid);
  return rc ? rc : (long)S.n;
}

// Canonical Beacon.Marshal rows -> fixed-stride records.  Row i is
// val_len[i] bytes at base + val_off[i].  ok[i] = 1: decoded into rounds[i],
// sigs + i*sig_stride (sig_len[i]), prev + i*prev_stride (prev_len[i]);
// ok[i] = 0: not canonical, the caller decodes it (record left zeroed).
// Returns the number of decoded rows.
size_t dgpu_ingest_decode(size_t n, const uint8_t* base, const uint64_t* val_off, const uint32_t* val_len,
                          uint64_t* rounds, uint8_t* sigs, size_t sig_stride, uint32_t* sig_len, uint8_t* prev,
                          size_t prev_stride, uint32_t* prev_len, uint8_t* ok) {
  size_t good = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* p = base + val_off[i];
    const uint8_t* end = p + val_len[i];
    uint8_t* so = sigs + i * sig_stride;
    uint8_t* po = prev + i * prev_stride;
    bool g = LIT(p, end, "{\"PreviousSig\":") && hex_field(p, end, po, prev_stride, prev_len + i) &&
             LIT(p, end, ",\"Round\":");
    uint64_t r = 0;
    if (g) {
      const uint8_t* d = p;
      while (p < end && *p >= '0' && *p <= '9') ++p;
      const size_t nd = (size_t)(p - d);
      g = nd >= 1 && nd <= 20 && !(nd > 1 && d[0] == '0');
      for (size_t k = 0; g && k < nd; ++k) {
        const uint64_t dig = (uint64_t)(d[k] - '0');
        if (r > (UINT64_MAX - dig) / 10) g = false;
        else r = r * 10 + dig;
      }
    }
    g = g && LIT(p, end, ",\"Signature\":") && hex_field(p, end, so, sig_stride, sig_len + i) && LIT(p, end, "}") &&
        p == end;
    if (!g) {
      memset(so, 0, sig_stride);
      memset(po, 0, prev_stride);
      sig_len[i] = prev_len[i] = 0;
      rounds[i] = 0;
    } else {
      rounds[i] = r;
      if (sig_len[i] < sig_stride) memset(so + sig_len[i], 0, sig_stride - sig_len[i]);
      if (prev_len[i] < prev_stride) memset(po + prev_len[i], 0, prev_stride - prev_len[i]);
      ++good;
    }
    ok[i] = g ? 1 : 0;
  }
  return good;
}

}  // extern "C"
