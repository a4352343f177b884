/*
 * drand_ingest.h -- host-side ingest helpers (libdrand_ingest.so, plain C++,
 * drand_amd/csrc/ingest.cpp) for the bulk check-chain path
 * (SURVEY.md 8(f) row 2): a drand bolt beacon store walked and decoded
 * straight into the fixed-stride records of dgpu_verify_beacons
 * (include/drand_gpu.h).
 *
 * Replaces, for a caller without Go's bbolt / hexjson:
 *   bucket cursor walk of "beacons"      chain/boltdb/store.go:141-151
 *   bucket.Stats().KeyN (Len)            chain/boltdb/store.go:51-62
 *   Get + Beacon.Unmarshal (hexjson)     chain/boltdb/store.go:113-132, chain/beacon.go:34-37
 * A Go caller already has these; the Python mirror (drand_amd/boltstore.py,
 * drand_amd/ingest.py) uses them.  Meta-page selection and bucket lookup stay
 * with the caller (drand_amd/boltstore.py): these functions take the mapped
 * file, its page size and the bucket's root page.
 */
#ifndef DRAND_INGEST_H
#define DRAND_INGEST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Rows with BE64(lo) <= key < BE64(hi) of the bucket rooted at root_pgid, in
 * key order (nested buckets and keys that are not 8 bytes skipped):
 * rounds_out[i] = the key, val_off[i] / val_len[i] = the value's bytes in
 * file.  Returns the count, -1 for a malformed file, -2 if more than cap. */
long dgpu_ingest_scan(const uint8_t *file, size_t file_len, size_t page_size, uint64_t root_pgid, uint64_t lo,
                      uint64_t hi, uint64_t *rounds_out, uint64_t *val_off, uint32_t *val_len, size_t cap);

/* bucket.Stats().KeyN of the bucket rooted at root_pgid; -1: malformed. */
long dgpu_ingest_count(const uint8_t *file, size_t file_len, size_t page_size, uint64_t root_pgid);

/* Canonical Beacon.Marshal rows {"PreviousSig":<hex|null>,"Round":<u64>,
 * "Signature":<hex|null>} -> records (ok[i] = 1); any other row -> ok[i] = 0
 * and a zeroed record, for the caller's full hexjson decoder.  Returns the
 * number of decoded rows. */
size_t dgpu_ingest_decode(size_t n, const uint8_t *base, const uint64_t *val_off, const uint32_t *val_len,
                          uint64_t *rounds, uint8_t *sigs, size_t sig_stride, uint32_t *sig_len, uint8_t *prev,
                          size_t prev_stride, uint32_t *prev_len, uint8_t *ok);

#ifdef __cplusplus
}
#endif
#endif /* DRAND_INGEST_H */
