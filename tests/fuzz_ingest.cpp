// Test infrastructure (tests/test_ingest_fuzz.py): mutation fuzzing of the
// native bolt-store parsers (drand_amd/csrc/ingest.cpp: dgpu_ingest_count,
// dgpu_ingest_scan, dgpu_ingest_decode) built together with them under
// AddressSanitizer / UBSan.  Every mutated file is handed over in a heap
// buffer of exactly its length, so any read past it is reported.
//
//   fuzz_ingest <db file> <page size> <root pgid> <iterations> <seed>
//
// Mutations: random byte flips, truncation, random 8-byte runs, extreme
// values written over page-header and element fields, and a random root
// page.  Decoded rows are checked against their file ranges; the decoder is
// also fed mutated canonical rows.  Exit 0 = no finding (the sanitizers
// abort on the first one).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/drand_ingest.h"

namespace {

std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

void mutate(std::vector<uint8_t>& f, std::mt19937_64& rng, size_t page_size) {
  const int kind = (int)(rng() % 5);
  if (f.empty()) return;
  if (kind == 0) {  // byte flips
    const int k = 1 + (int)(rng() % 16);
    for (int i = 0; i < k; ++i) f[rng() % f.size()] ^= (uint8_t)(1 + rng() % 255);
  } else if (kind == 1) {  // truncation
    f.resize(rng() % (f.size() + 1));
  } else if (kind == 2) {  // random 8-byte runs
    const int k = 1 + (int)(rng() % 4);
    for (int i = 0; i < k && f.size() >= 8; ++i) {
      const size_t o = rng() % (f.size() - 7);
      const uint64_t v = rng();
      memcpy(&f[o], &v, 8);
    }
  } else {  // extreme values over a page header or an element field
    const size_t pages = f.size() / page_size;
    if (!pages) return;
    const size_t pg = rng() % pages;
    const size_t field = kind == 3 ? 8 + 2 * (rng() % 4)                         // flags, count, overflow
                                   : 16 + 16 * (rng() % 8) + 4 * (rng() % 4);   // element words
    const size_t o = pg * page_size + field;
    if (o + 4 > f.size()) return;
    static const uint32_t ext[] = {0u, 1u, 2u, 0x7FFFu, 0xFFFFu, 0x10000u, 0x7FFFFFFFu, 0xFFFFFFFFu};
    const uint32_t v = ext[rng() % 8];
    memcpy(&f[o], &v, (kind == 3 && field < 12) ? 2 : 4);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s db page_size root iterations seed\n", argv[0]);
    return 2;
  }
  const std::vector<uint8_t> base = read_file(argv[1]);
  const size_t page_size = strtoull(argv[2], nullptr, 10);
  const uint64_t root = strtoull(argv[3], nullptr, 10);
  const long iters = strtol(argv[4], nullptr, 10);
  std::mt19937_64 rng(strtoull(argv[5], nullptr, 10));
  if (base.empty()) return 2;
  const size_t cap = 1 << 14, stride = 96;
  std::vector<uint64_t> rounds(cap), off(cap), drounds(cap);
  std::vector<uint32_t> len(cap), slen(cap), plen(cap);
  std::vector<uint8_t> sigs(cap * stride), prev(cap * stride), ok(cap);
  long scans = 0, rows = 0;
  for (long it = 0; it < iters; ++it) {
    std::vector<uint8_t> f = base;
    const int nmut = 1 + (int)(rng() % 3);
    for (int m = 0; m < nmut; ++m) mutate(f, rng, page_size);
    uint8_t* buf = (uint8_t*)malloc(f.size() ? f.size() : 1);
    if (!f.empty()) memcpy(buf, f.data(), f.size());
    const uint64_t r = (rng() % 8 == 0) ? rng() % (2 + f.size() / page_size) : root;
    const size_t ps = (rng() % 16 == 0) ? 64u << (rng() % 8) : page_size;
    (void)dgpu_ingest_count(buf, f.size(), ps, r);
    const uint64_t lo = rng() % 4 == 0 ? rng() : 0, hi = rng() % 4 == 0 ? rng() : ~0ull;
    const long n = dgpu_ingest_scan(buf, f.size(), ps, r, lo, hi, rounds.data(), off.data(), len.data(), cap);
    ++scans;
    if (n > 0) {
      for (long i = 0; i < n; ++i)
        if (off[i] + len[i] > f.size()) {
          fprintf(stderr, "row %ld outside the file: %llu + %u > %zu\n", i, (unsigned long long)off[i], len[i], f.size());
          return 1;
        }
      rows += n;
      dgpu_ingest_decode((size_t)n, buf, off.data(), len.data(), drounds.data(), sigs.data(), stride, slen.data(),
                         prev.data(), stride, plen.data(), ok.data());
    }
    free(buf);
  }
  // the decoder on mutated canonical rows, each in its own exact-size buffer
  const std::string good =
      "{\"PreviousSig\":\"" + std::string(192, 'a') + "\",\"Round\":18446744073709551615,\"Signature\":\"" +
      std::string(192, 'F') + "\"}";
  long decoded = 0;
  for (long it = 0; it < iters; ++it) {
    std::string row = good;
    const int k = (int)(rng() % 6);
    for (int i = 0; i < k && !row.empty(); ++i) {
      const int op = (int)(rng() % 3);
      const size_t o = rng() % row.size();
      if (op == 0) row[o] = (char)(rng() % 256);
      else if (op == 1) row.erase(o, 1 + rng() % 8);
      else row.insert(o, 1 + rng() % 8, "0a\",:{}n9"[rng() % 9]);
    }
    uint8_t* buf = (uint8_t*)malloc(row.size() ? row.size() : 1);
    memcpy(buf, row.data(), row.size());
    const uint64_t o0 = 0;
    const uint32_t l0 = (uint32_t)row.size();
    decoded += (long)dgpu_ingest_decode(1, buf, &o0, &l0, drounds.data(), sigs.data(), stride, slen.data(), prev.data(),
                                        stride, plen.data(), ok.data());
    if (ok[0] && (slen[0] > stride || plen[0] > stride)) return 1;
    free(buf);
  }
  printf("scans=%ld rows=%ld decoded=%ld\n", scans, rows, decoded);
  return 0;
}
