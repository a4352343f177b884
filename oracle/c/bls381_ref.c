/*
 * C restatement of drand's beacon verification (TEST INFRASTRUCTURE / CPU
 * baseline).  Never linked into the product (libdrand_gpu.so); used by
 * tests/ and by bench.py's cpu_baseline leg through ctypes.
 *
 * An independent implementation of the same published algorithms as the
 * reference's third-party crypto (kyber-bls12381 v0.2.1 / kilic bls12-381,
 * absent from /root/reference): 6 x 64-bit Montgomery limbs (R = 2^384, a
 * different representation from the GPU's 14 x 28-bit), RFC 9380
 * hash-to-G2, ZCash decode with the reference's [r]Q == O subgroup test,
 * optimal-ate pairing check.  Restates:
 *   chain/verify.go:24-32   DigestMessage (SHA-256(prev || BE64(round)))
 *   chain/verify.go:38-45   VerifyBeacon -> key.Scheme.VerifyRecovered
 *   key/curve.go:24-39      keys on G1, signatures on G2
 * and is checked against the golden vectors of the pure-Python oracle,
 * itself pinned by key/curve_test.go:10-30.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

#include "consts.h"

/* ------------------------------------------------------------------ SHA-256 */
static const uint32_t SK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_block(uint32_t h[8], const uint8_t* b) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
  }
  h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* one-shot SHA-256 over up to 4 concatenated segments */
static void sha256_segs(uint8_t out[32], const uint8_t* s[], const size_t len[], int nseg) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t fill = 0, total = 0;
  for (int k = 0; k < nseg; ++k) {
    for (size_t i = 0; i < len[k]; ++i) {
      blk[fill++] = s[k][i];
      if (fill == 64) { sha_block(h, blk); fill = 0; }
    }
    total += len[k];
  }
  blk[fill++] = 0x80;
  if (fill > 56) { while (fill < 64) blk[fill++] = 0; sha_block(h, blk); fill = 0; }
  while (fill < 56) blk[fill++] = 0;
  u64 bits = (u64)total * 8;
  for (int i = 0; i < 8; ++i) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_block(h, blk);
  for (int i = 0; i < 8; ++i) { out[4 * i] = h[i] >> 24; out[4 * i + 1] = h[i] >> 16; out[4 * i + 2] = h[i] >> 8; out[4 * i + 3] = h[i]; }
}

/* ------------------------------------------------------------------ Fp */
typedef struct { u64 v[6]; } fp;

static fp fpc(const u64* c) { fp r; memcpy(r.v, c, 48); return r; }
static int fp_geq_p(const fp* a) {
  for (int i = 5; i >= 0; --i) { if (a->v[i] > P_[i]) return 1; if (a->v[i] < P_[i]) return 0; }
  return 1;
}
static void fp_subp(fp* a) {
  u64 br = 0;
  for (int i = 0; i < 6; ++i) { u128 d = (u128)a->v[i] - P_[i] - br; a->v[i] = (u64)d; br = (u64)(d >> 64) & 1; }
}
static fp fp_add(fp a, fp b) {
  fp r; u64 c = 0;
  for (int i = 0; i < 6; ++i) { u128 s = (u128)a.v[i] + b.v[i] + c; r.v[i] = (u64)s; c = (u64)(s >> 64); }
  if (c || fp_geq_p(&r)) fp_subp(&r);
  return r;
}
static fp fp_sub(fp a, fp b) {
  fp r; u64 br = 0;
  for (int i = 0; i < 6; ++i) { u128 d = (u128)a.v[i] - b.v[i] - br; r.v[i] = (u64)d; br = (u64)(d >> 64) & 1; }
  if (br) { u64 c = 0; for (int i = 0; i < 6; ++i) { u128 s = (u128)r.v[i] + P_[i] + c; r.v[i] = (u64)s; c = (u64)(s >> 64); } }
  return r;
}
static fp fp_neg(fp a) { fp z = {{0}}; return fp_sub(z, a); }
static fp fp_mul(fp a, fp b) { /* CIOS */
  u64 t[8] = {0};
  for (int i = 0; i < 6; ++i) {
    u64 c = 0;
    for (int j = 0; j < 6; ++j) { u128 s = (u128)a.v[j] * b.v[i] + t[j] + c; t[j] = (u64)s; c = (u64)(s >> 64); }
    u128 s = (u128)t[6] + c; t[6] = (u64)s; t[7] = (u64)(s >> 64);
    u64 m = t[0] * PINV;
    s = (u128)m * P_[0] + t[0]; c = (u64)(s >> 64);
    for (int j = 1; j < 6; ++j) { s = (u128)m * P_[j] + t[j] + c; t[j - 1] = (u64)s; c = (u64)(s >> 64); }
    s = (u128)t[6] + c; t[5] = (u64)s; t[6] = t[7] + (u64)(s >> 64);
  }
  fp r; memcpy(r.v, t, 48);
  if (t[6] || fp_geq_p(&r)) fp_subp(&r);
  return r;
}
static fp fp_sqr(fp a) { return fp_mul(a, a); }
static int fp_is_zero(fp a) { u64 z = 0; for (int i = 0; i < 6; ++i) z |= a.v[i]; return z == 0; }
static int fp_eq(fp a, fp b) { return memcmp(a.v, b.v, 48) == 0; }
static fp fp_one(void) { return fpc(ONE_); }
static fp fp_pow(fp a, const u64* e, int nbits) {
  fp r = fp_one();
  for (int i = nbits - 1; i >= 0; --i) { r = fp_sqr(r); if ((e[i >> 6] >> (i & 63)) & 1) r = fp_mul(r, a); }
  return r;
}
static fp fp_inv(fp a) { return fp_pow(a, E_PM2, E_PM2_NBITS); }
static fp fp_from_mont(fp a) { fp one = {{1, 0, 0, 0, 0, 0}}; return fp_mul(a, one); }
static fp fp_to_mont(fp a) { return fp_mul(a, fpc(R2_)); }
static int fp_sgn0(fp a) { return fp_from_mont(a).v[0] & 1; }
/* standard value > (p-1)/2 */
static int fp_gt_half(fp a) {
  fp s = fp_from_mont(a), d; u64 c = 0;
  for (int i = 0; i < 6; ++i) { u128 t = (u128)s.v[i] + s.v[i] + c; d.v[i] = (u64)t; c = (u64)(t >> 64); }
  return c || fp_geq_p(&d);
}
static fp fp_from_be48(const uint8_t* b) { fp r; for (int i = 0; i < 6; ++i) { u64 w = 0; for (int k = 0; k < 8; ++k) w = w << 8 | b[8 * (5 - i) + k]; r.v[i] = w; } return r; }
static void fp_to_be48(fp a, uint8_t* b) { fp s = fp_from_mont(a); for (int i = 0; i < 6; ++i) for (int k = 0; k < 8; ++k) b[8 * (5 - i) + k] = (uint8_t)(s.v[i] >> (56 - 8 * k)); }

/* ------------------------------------------------------------------ Fp2 */
typedef struct { fp c0, c1; } fp2;
static fp2 f2c(const u64 c[2][6]) { fp2 r = {fpc(c[0]), fpc(c[1])}; return r; }
static fp2 f2_add(fp2 a, fp2 b) { fp2 r = {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; return r; }
static fp2 f2_sub(fp2 a, fp2 b) { fp2 r = {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; return r; }
static fp2 f2_neg(fp2 a) { fp2 r = {fp_neg(a.c0), fp_neg(a.c1)}; return r; }
static fp2 f2_dbl(fp2 a) { return f2_add(a, a); }
static fp2 f2_mul(fp2 a, fp2 b) {
  fp t0 = fp_mul(a.c0, b.c0), t1 = fp_mul(a.c1, b.c1);
  fp2 r = {fp_sub(t0, t1), fp_sub(fp_sub(fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1)), t0), t1)};
  return r;
}
static fp2 f2_sqr(fp2 a) { fp2 r = {fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_mul(fp_add(a.c0, a.c0), a.c1)}; return r; }
static fp2 f2_mulfp(fp2 a, fp s) { fp2 r = {fp_mul(a.c0, s), fp_mul(a.c1, s)}; return r; }
static fp2 f2_xi(fp2 a) { fp2 r = {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; return r; }
static fp2 f2_conj(fp2 a) { fp2 r = {a.c0, fp_neg(a.c1)}; return r; }
static int f2_is_zero(fp2 a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
static int f2_eq(fp2 a, fp2 b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
static fp2 f2_zero(void) { fp2 r; memset(&r, 0, sizeof r); return r; }
static fp2 f2_one(void) { fp2 r = {fp_one(), {{0}}}; return r; }
static fp f2_norm(fp2 a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }
static fp2 f2_inv(fp2 a) { fp t = fp_inv(f2_norm(a)); fp2 r = {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))}; return r; }
static int fp_is_square(fp a) { fp t = fp_pow(a, E_LEG, E_LEG_NBITS); return fp_is_zero(a) || fp_eq(t, fp_one()); }
static fp fp_sqrt_cand(fp a) { return fp_pow(a, E_SQRT, E_SQRT_NBITS); }
static fp fp_half(fp a) { /* a/2 */
  fp s = a; u64 c = 0;
  if (s.v[0] & 1) for (int i = 0; i < 6; ++i) { u128 t = (u128)s.v[i] + P_[i] + c; s.v[i] = (u64)t; c = (u64)(t >> 64); }
  for (int i = 0; i < 5; ++i) s.v[i] = s.v[i] >> 1 | s.v[i + 1] << 63;
  s.v[5] = s.v[5] >> 1 | c << 63;
  return s;
}
static int f2_sqrt(fp2* out, fp2 a) {
  if (fp_is_zero(a.c1)) {
    fp s = fp_sqrt_cand(a.c0);
    if (fp_eq(fp_sqr(s), a.c0)) { out->c0 = s; memset(&out->c1, 0, sizeof(fp)); return 1; }
    fp na = fp_neg(a.c0); s = fp_sqrt_cand(na);
    memset(&out->c0, 0, sizeof(fp)); out->c1 = s;
    return fp_eq(fp_sqr(s), na);
  }
  fp al = f2_norm(a), g = fp_sqrt_cand(al);
  if (!fp_eq(fp_sqr(g), al)) return 0;
  fp d = fp_half(fp_add(a.c0, g)), x0 = fp_sqrt_cand(d);
  if (!fp_eq(fp_sqr(x0), d)) { d = fp_half(fp_sub(a.c0, g)); x0 = fp_sqrt_cand(d); }
  fp x1 = fp_mul(a.c1, fp_inv(fp_add(x0, x0)));
  out->c0 = x0; out->c1 = x1;
  return f2_eq(f2_sqr(*out), a);
}
static int f2_sgn0(fp2 a) { int s0 = fp_sgn0(a.c0), z0 = fp_is_zero(a.c0), s1 = fp_sgn0(a.c1); return s0 | (z0 & s1); }
static int f2_lexi(fp2 y) { return fp_is_zero(y.c1) ? fp_gt_half(y.c0) : fp_gt_half(y.c1); }

/* ------------------------------------------------------------------ Fp6, Fp12 */
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
static fp6 f6_add(fp6 a, fp6 b) { fp6 r = {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; return r; }
static fp6 f6_sub(fp6 a, fp6 b) { fp6 r = {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; return r; }
static fp6 f6_neg(fp6 a) { fp6 r = {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; return r; }
static fp6 f6_mul(fp6 a, fp6 b) {
  fp2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
  fp6 r;
  r.c0 = f2_add(t0, f2_xi(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), f2_add(t1, t2))));
  r.c1 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), f2_add(t0, t1)), f2_xi(t2));
  r.c2 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), f2_add(t0, t2)), t1);
  return r;
}
static fp6 f6_mulv(fp6 a) { fp6 r = {f2_xi(a.c2), a.c0, a.c1}; return r; }
static fp6 f6_inv(fp6 a) {
  fp2 t0 = f2_sub(f2_sqr(a.c0), f2_xi(f2_mul(a.c1, a.c2)));
  fp2 t1 = f2_sub(f2_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  fp2 t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  fp2 d = f2_inv(f2_add(f2_mul(a.c0, t0), f2_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2)))));
  fp6 r = {f2_mul(t0, d), f2_mul(t1, d), f2_mul(t2, d)};
  return r;
}
static fp12 f12_mul(fp12 a, fp12 b) {
  fp6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  fp12 r = {f6_add(t0, f6_mulv(t1)), f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), f6_add(t0, t1))};
  return r;
}
static fp12 f12_sqr(fp12 a) { return f12_mul(a, a); }
static fp12 f12_conj(fp12 a) { fp12 r = {a.c0, f6_neg(a.c1)}; return r; }
static fp12 f12_inv(fp12 a) {
  fp6 t = f6_inv(f6_sub(f6_mul(a.c0, a.c0), f6_mulv(f6_mul(a.c1, a.c1))));
  fp12 r = {f6_mul(a.c0, t), f6_neg(f6_mul(a.c1, t))};
  return r;
}
static fp12 f12_one(void) { fp12 r; memset(&r, 0, sizeof r); r.c0.c0 = f2_one(); return r; }
static int f12_is_one(fp12 a) {
  fp12 o = f12_one();
  return f2_eq(a.c0.c0, o.c0.c0) && f2_is_zero(a.c0.c1) && f2_is_zero(a.c0.c2) && f2_is_zero(a.c1.c0) &&
         f2_is_zero(a.c1.c1) && f2_is_zero(a.c1.c2);
}
/* Frobenius on basis w^i: 1->c0.c0, w->c1.c0, w^2->c0.c1, w^3->c1.c1, w^4->c0.c2, w^5->c1.c2 */
static fp12 f12_frob(fp12 a, int k) {
  const u64(*G)[2][6] = k == 1 ? FROB1 : FROB2;
  fp2* c[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
  for (int i = 0; i < 6; ++i) { fp2 x = k == 1 ? f2_conj(*c[i]) : *c[i]; *c[i] = i ? f2_mul(x, f2c(G[i])) : x; }
  return a;
}
/* a * (b0 + b1 v) and a * (b1 v) in Fp6 (sparse factors of a line) */
static fp6 f6_mul01(fp6 a, fp2 b0, fp2 b1) {
  fp2 t0 = f2_mul(a.c0, b0), t1 = f2_mul(a.c1, b1);
  fp6 r = {f2_add(t0, f2_xi(f2_mul(a.c2, b1))), f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b0, b1)), f2_add(t0, t1)),
           f2_add(f2_mul(a.c2, b0), t1)};
  return r;
}
static fp6 f6_mul1(fp6 a, fp2 b1) { fp6 r = {f2_xi(f2_mul(a.c2, b1)), f2_mul(a.c0, b1), f2_mul(a.c1, b1)}; return r; }
/* f * l with l = c0 + c2 w^2 + c3 w^3 = (c0 + c2 v) + (c3 v) w */
static fp12 f12_mul_line(fp12 f, fp2 c0, fp2 c2, fp2 c3) {
  fp6 a = f6_mul01(f.c0, c0, c2), b = f6_mul1(f.c1, c3);
  fp12 r = {f6_add(a, f6_mulv(b)), f6_sub(f6_mul01(f6_add(f.c0, f.c1), c0, f2_add(c2, c3)), f6_add(a, b))};
  return r;
}
/* Granger-Scott squaring on the cyclotomic subgroup */
static void f4_sqr(fp2* r0, fp2* r1, fp2 x0, fp2 x1) {
  fp2 t0 = f2_sqr(x0), t1 = f2_sqr(x1);
  *r0 = f2_add(t0, f2_xi(t1));
  *r1 = f2_sub(f2_sqr(f2_add(x0, x1)), f2_add(t0, t1));
}
static fp2 f2_3m2(fp2 a, fp2 b) { return f2_add(f2_dbl(f2_sub(a, b)), a); }
static fp2 f2_3p2(fp2 a, fp2 b) { return f2_add(f2_dbl(f2_add(a, b)), a); }
static fp12 f12_cyc_sqr(fp12 f) {
  fp2 a0, a1, b0, b1, c0, c1;
  f4_sqr(&a0, &a1, f.c0.c0, f.c1.c1);
  f4_sqr(&b0, &b1, f.c1.c0, f.c0.c2);
  f4_sqr(&c0, &c1, f.c0.c1, f.c1.c2);
  fp12 r;
  r.c0.c0 = f2_3m2(a0, f.c0.c0); r.c1.c1 = f2_3p2(a1, f.c1.c1);
  r.c1.c0 = f2_3p2(f2_xi(c1), f.c1.c0); r.c0.c2 = f2_3m2(c0, f.c0.c2);
  r.c0.c1 = f2_3m2(b0, f.c0.c1); r.c1.c2 = f2_3p2(b1, f.c1.c2);
  return r;
}

/* ------------------------------------------------------------------ G2 (Jacobian) */
typedef struct { fp2 x, y, z; } g2;
static int g2_inf(const g2* p) { return f2_is_zero(p->z); }
static g2 g2_infinity(void) { g2 r = {f2_one(), f2_one(), f2_zero()}; return r; }
static g2 g2_dbl(g2 p) {
  fp2 A = f2_sqr(p.x), B = f2_sqr(p.y), C = f2_sqr(B);
  fp2 D = f2_dbl(f2_sub(f2_sqr(f2_add(p.x, B)), f2_add(A, C)));
  fp2 E = f2_add(f2_dbl(A), A), F = f2_sqr(E);
  g2 r;
  r.x = f2_sub(F, f2_dbl(D));
  r.y = f2_sub(f2_mul(E, f2_sub(D, r.x)), f2_dbl(f2_dbl(f2_dbl(C))));
  r.z = f2_dbl(f2_mul(p.y, p.z));
  return r;
}
static g2 g2_add(g2 p, g2 q) {
  if (g2_inf(&p)) return q;
  if (g2_inf(&q)) return p;
  fp2 z1z1 = f2_sqr(p.z), z2z2 = f2_sqr(q.z);
  fp2 u1 = f2_mul(p.x, z2z2), u2 = f2_mul(q.x, z1z1);
  fp2 s1 = f2_mul(f2_mul(p.y, q.z), z2z2), s2 = f2_mul(f2_mul(q.y, p.z), z1z1);
  fp2 h = f2_sub(u2, u1), rr = f2_dbl(f2_sub(s2, s1));
  if (f2_is_zero(h)) return f2_is_zero(rr) ? g2_dbl(p) : g2_infinity();
  fp2 i = f2_sqr(f2_dbl(h)), j = f2_mul(h, i), v = f2_mul(u1, i);
  g2 r;
  r.x = f2_sub(f2_sub(f2_sqr(rr), j), f2_dbl(v));
  r.y = f2_sub(f2_mul(rr, f2_sub(v, r.x)), f2_dbl(f2_mul(s1, j)));
  r.z = f2_mul(f2_sub(f2_sqr(f2_add(p.z, q.z)), f2_add(z1z1, z2z2)), h);
  return r;
}
static g2 g2_neg(g2 p) { p.y = f2_neg(p.y); return p; }
static g2 g2_mul_u64s(g2 p, const u64* k, int nbits) {
  g2 r = g2_infinity();
  for (int i = nbits - 1; i >= 0; --i) { r = g2_dbl(r); if ((k[i >> 6] >> (i & 63)) & 1) r = g2_add(r, p); }
  return r;
}
static const u64 XABS = 0xd201000000010000ULL;
static g2 g2_mul_x(g2 p) { return g2_neg(g2_mul_u64s(p, &XABS, 64)); } /* x < 0 */
static g2 g2_psi(g2 p) { g2 r = {f2_mul(f2_conj(p.x), f2c(PSI_CX)), f2_mul(f2_conj(p.y), f2c(PSI_CY)), f2_conj(p.z)}; return r; }
static void g2_affine(const g2* p, fp2* x, fp2* y) {
  fp2 zi = f2_inv(p->z), zi2 = f2_sqr(zi);
  *x = f2_mul(p->x, zi2); *y = f2_mul(p->y, f2_mul(zi2, zi));
}

/* ------------------------------------------------------------------ hash to G2 (RFC 9380) */
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
static const char DST_G1[] = "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_";
/* expand_message_xmd (RFC 9380 5.3.1): len_out = 32 ell bytes of a 32-byte msg under a 43-byte DST */
static void expand_xmd_dst(uint8_t* out, int ell, const uint8_t msg[32], const char* dst) {
  uint8_t zpad[64] = {0}, dstp[44], b0[32], bi[32], tmp[32];
  memcpy(dstp, dst, 43); dstp[43] = 43;
  uint8_t lib0[3] = {(uint8_t)((32 * ell) >> 8), (uint8_t)(32 * ell), 0};
  const uint8_t* s0[4] = {zpad, msg, lib0, dstp};
  size_t l0[4] = {64, 32, 3, 44};
  sha256_segs(b0, s0, l0, 4);
  memset(bi, 0, 32);
  for (int i = 1; i <= ell; ++i) {
    for (int k = 0; k < 32; ++k) tmp[k] = b0[k] ^ bi[k];
    uint8_t idx = (uint8_t)i;
    const uint8_t* s[3] = {tmp, &idx, dstp};
    size_t l[3] = {32, 1, 44};
    sha256_segs(bi, s, l, 3);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}
static void expand_xmd(uint8_t out[256], const uint8_t msg[32]) { expand_xmd_dst(out, 8, msg, DST); }
static fp fp_from_be64(const uint8_t* b) { /* 64-byte BE mod p in Montgomery form */
  uint8_t hi[48] = {0};
  memcpy(hi + 32, b, 16);
  fp lo = fp_from_be48(b + 16), h = fp_from_be48(hi);
  return fp_add(fp_to_mont(lo), fp_mul(h, fpc(K384_)));
}
static void sswu(fp2* ox, fp2* oy, fp2 u) {
  fp2 A = f2c(SSWU_A), B = f2c(SSWU_B), Z = f2c(SSWU_Z);
  fp2 zu2 = f2_mul(Z, f2_sqr(u)), den = f2_add(f2_sqr(zu2), zu2), x1;
  if (f2_is_zero(den)) x1 = f2c(SSWU_BZA);
  else x1 = f2_mul(f2c(SSWU_MBA), f2_add(f2_one(), f2_inv(den)));
  fp2 gx1 = f2_add(f2_mul(f2_add(f2_sqr(x1), A), x1), B);
  fp2 x2 = f2_mul(zu2, x1), gx2 = f2_add(f2_mul(f2_add(f2_sqr(x2), A), x2), B), y;
  if (fp_is_square(f2_norm(gx1))) { *ox = x1; f2_sqrt(&y, gx1); }
  else { *ox = x2; f2_sqrt(&y, gx2); }
  if (f2_sgn0(u) != f2_sgn0(y)) y = f2_neg(y);
  *oy = y;
}
static fp2 poly(const u64 (*k)[2][6], int n, fp2 x) {
  fp2 acc = f2c(k[n - 1]);
  for (int i = n - 2; i >= 0; --i) acc = f2_add(f2_mul(acc, x), f2c(k[i]));
  return acc;
}
static g2 iso3(fp2 x, fp2 y) {
  fp2 xn = poly(ISO_XNUM, 4, x), xd = poly(ISO_XDEN, 3, x), yn = poly(ISO_YNUM, 4, x), yd = poly(ISO_YDEN, 4, x);
  if (f2_is_zero(xd) || f2_is_zero(yd)) return g2_infinity();
  g2 r = {f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))), f2_one()};
  return r;
}
static g2 clear_cofactor(g2 p) {
  g2 t1 = g2_mul_x(p), t2 = g2_psi(p), t3 = g2_psi(g2_psi(g2_dbl(p)));
  t3 = g2_add(t3, g2_neg(t2));
  t2 = g2_mul_x(g2_add(t1, t2));
  t3 = g2_add(g2_add(t3, t2), g2_neg(t1));
  return g2_add(t3, g2_neg(p));
}
static g2 hash_to_g2(const uint8_t msg[32]) {
  uint8_t u[256];
  expand_xmd(u, msg);
  fp2 u0 = {fp_from_be64(u), fp_from_be64(u + 64)}, u1 = {fp_from_be64(u + 128), fp_from_be64(u + 192)}, x, y;
  sswu(&x, &y, u0);
  g2 q0 = iso3(x, y);
  sswu(&x, &y, u1);
  g2 q1 = iso3(x, y);
  return clear_cofactor(g2_add(q0, q1));
}

/* ------------------------------------------------------------------ decode */
enum { R_OK = 0, R_DECODE = 1, R_SUBGROUP = 2, R_PAIRING = 3, R_INFINITY = 4 };
static int g2_decode(fp2* x, fp2* y, const uint8_t* in, size_t len) {
  if (len != 96) return R_DECODE;
  if (!(in[0] & 0x80)) return R_DECODE;
  if (in[0] & 0x40) {
    int nz = in[0] & 0x3f;
    for (int i = 1; i < 96; ++i) nz |= in[i];
    return nz ? R_DECODE : R_INFINITY;
  }
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  fp x1 = fp_from_be48(b), x0 = fp_from_be48(in + 48);
  if (fp_geq_p(&x0) || fp_geq_p(&x1)) return R_DECODE;
  x->c0 = fp_to_mont(x0); x->c1 = fp_to_mont(x1);
  if (!f2_sqrt(y, f2_add(f2_mul(f2_sqr(*x), *x), f2c(B2)))) return R_DECODE;
  if (f2_lexi(*y) != !!(in[0] & 0x20)) *y = f2_neg(*y);
  g2 q = {*x, *y, f2_one()};
  g2 t = g2_mul_u64s(q, R_ORDER, 256); /* reference semantics: [r]Q == O (R) */
  return g2_inf(&t) ? R_OK : R_SUBGROUP;
}
static int g1_decode(fp* x, fp* y, const uint8_t* in) {
  if (!(in[0] & 0x80) || (in[0] & 0x40)) return R_DECODE;
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  fp xs = fp_from_be48(b);
  if (fp_geq_p(&xs)) return R_DECODE;
  *x = fp_to_mont(xs);
  fp rhs = fp_add(fp_mul(fp_sqr(*x), *x), fpc(B1));
  *y = fp_sqrt_cand(rhs);
  if (!fp_eq(fp_sqr(*y), rhs)) return R_DECODE;
  if (fp_gt_half(*y) != !!(in[0] & 0x20)) *y = fp_neg(*y);
  return R_OK; /* subgroup of the (trusted, decoded-once) group key is checked by the callers' tests */
}

/* ------------------------------------------------------------------ G1 (Jacobian), hash to G1, G1 signatures */
typedef struct { fp x, y, z; } g1;
static int g1_inf(const g1* p) { return fp_is_zero(p->z); }
static g1 g1_infinity(void) { g1 r = {fp_one(), fp_one(), {{0}}}; return r; }
static g1 g1_dbl(g1 p) {
  fp A = fp_sqr(p.x), B = fp_sqr(p.y), C = fp_sqr(B);
  fp D = fp_sub(fp_sqr(fp_add(p.x, B)), fp_add(A, C));
  D = fp_add(D, D);
  fp E = fp_add(fp_add(A, A), A), F = fp_sqr(E);
  g1 r;
  r.x = fp_sub(F, fp_add(D, D));
  fp C8 = fp_add(C, C); C8 = fp_add(C8, C8); C8 = fp_add(C8, C8);
  r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), C8);
  r.z = fp_mul(fp_add(p.y, p.y), p.z);
  return r;
}
static g1 g1_add(g1 p, g1 q) {
  if (g1_inf(&p)) return q;
  if (g1_inf(&q)) return p;
  fp z1z1 = fp_sqr(p.z), z2z2 = fp_sqr(q.z);
  fp u1 = fp_mul(p.x, z2z2), u2 = fp_mul(q.x, z1z1);
  fp s1 = fp_mul(fp_mul(p.y, q.z), z2z2), s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  fp h = fp_sub(u2, u1), rr = fp_sub(s2, s1);
  rr = fp_add(rr, rr);
  if (fp_is_zero(h)) return fp_is_zero(rr) ? g1_dbl(p) : g1_infinity();
  fp i = fp_sqr(fp_add(h, h)), j = fp_mul(h, i), v = fp_mul(u1, i);
  g1 r;
  r.x = fp_sub(fp_sub(fp_sqr(rr), j), fp_add(v, v));
  fp s1j = fp_mul(s1, j);
  r.y = fp_sub(fp_mul(rr, fp_sub(v, r.x)), fp_add(s1j, s1j));
  r.z = fp_mul(fp_sub(fp_sqr(fp_add(p.z, q.z)), fp_add(z1z1, z2z2)), h);
  return r;
}
static g1 g1_mul_u64s(g1 p, const u64* k, int nbits) {
  g1 r = g1_infinity();
  for (int i = nbits - 1; i >= 0; --i) { r = g1_dbl(r); if ((k[i >> 6] >> (i & 63)) & 1) r = g1_add(r, p); }
  return r;
}
static void g1_affine(const g1* p, fp* x, fp* y) {
  fp zi = fp_inv(p->z), zi2 = fp_sqr(zi);
  *x = fp_mul(p->x, zi2); *y = fp_mul(p->y, fp_mul(zi2, zi));
}
/* simplified SWU on E1' (RFC 9380 6.6.2), then the 11-isogeny to E1 */
static void sswu1(fp* ox, fp* oy, fp u) {
  fp A = fpc(SSWU1_A), B = fpc(SSWU1_B), Z = fpc(SSWU1_Z);
  fp zu2 = fp_mul(Z, fp_sqr(u)), den = fp_add(fp_sqr(zu2), zu2), x1;
  if (fp_is_zero(den)) x1 = fpc(SSWU1_BZA);
  else x1 = fp_mul(fpc(SSWU1_MBA), fp_add(fp_one(), fp_inv(den)));
  fp gx1 = fp_add(fp_mul(fp_add(fp_sqr(x1), A), x1), B);
  fp x2 = fp_mul(zu2, x1), gx2 = fp_add(fp_mul(fp_add(fp_sqr(x2), A), x2), B), y;
  if (fp_is_square(gx1)) { *ox = x1; y = fp_sqrt_cand(gx1); }
  else { *ox = x2; y = fp_sqrt_cand(gx2); }
  if (fp_sgn0(u) != fp_sgn0(y)) y = fp_neg(y);
  *oy = y;
}
static fp fpoly(const u64 (*k)[6], int n, fp x) {
  fp acc = fpc(k[n - 1]);
  for (int i = n - 2; i >= 0; --i) acc = fp_add(fp_mul(acc, x), fpc(k[i]));
  return acc;
}
static g1 iso11(fp x, fp y) {
  fp xd = fpoly(ISO11_XDEN, 11, x), yd = fpoly(ISO11_YDEN, 16, x);
  if (fp_is_zero(xd) || fp_is_zero(yd)) return g1_infinity();
  g1 r = {fp_mul(fpoly(ISO11_XNUM, 12, x), fp_inv(xd)), fp_mul(y, fp_mul(fpoly(ISO11_YNUM, 16, x), fp_inv(yd))), fp_one()};
  return r;
}
/* RFC 9380 BLS12381G1_XMD:SHA-256_SSWU_RO_ of a 32-byte digest; h_eff = 1 - x */
static g1 hash_to_g1(const uint8_t msg[32], const char* dst) {
  uint8_t u[128];
  expand_xmd_dst(u, 4, msg, dst);
  fp x, y;
  sswu1(&x, &y, fp_from_be64(u));
  g1 q0 = iso11(x, y);
  sswu1(&x, &y, fp_from_be64(u + 64));
  g1 q1 = iso11(x, y);
  static const u64 HEFF1 = 0xd201000000010001ULL;
  return g1_mul_u64s(g1_add(q0, q1), &HEFF1, 64);
}
/* 48-byte compressed G1 signature, kilic FromCompressed semantics (R): flags,
   x < p, on the curve, [r]P == O */
static int g1_decode_sig(fp* x, fp* y, const uint8_t* in, size_t len) {
  if (len != 48) return R_DECODE;
  if (!(in[0] & 0x80)) return R_DECODE;
  if (in[0] & 0x40) {
    int nz = in[0] & 0x3f;
    for (int i = 1; i < 48; ++i) nz |= in[i];
    return nz ? R_DECODE : R_INFINITY;
  }
  int rc = g1_decode(x, y, in);
  if (rc != R_OK) return rc;
  g1 q = {*x, *y, fp_one()};
  g1 t = g1_mul_u64s(q, R_ORDER, 256);
  return g1_inf(&t) ? R_OK : R_SUBGROUP;
}

/* ------------------------------------------------------------------ Fr (4 x 64-bit Montgomery, R = 2^256) */
typedef struct { u64 v[4]; } fr;
static int fr_geq(const fr* a) {
  for (int i = 3; i >= 0; --i) { if (a->v[i] > FR_[i]) return 1; if (a->v[i] < FR_[i]) return 0; }
  return 1;
}
static void fr_subr(fr* a) {
  u128 b = 0;
  for (int i = 0; i < 4; ++i) { u128 d = (u128)a->v[i] - FR_[i] - b; a->v[i] = (u64)d; b = (d >> 64) & 1; }
}
static fr fr_mul(fr a, fr b) { /* CIOS */
  u64 t[6] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a.v[j] * b.v[i] + t[j]; t[j] = (u64)c; c >>= 64; }
    c += t[4]; t[4] = (u64)c; t[5] = (u64)(c >> 64);
    u64 m = t[0] * FR_INV;
    c = (u128)m * FR_[0] + t[0]; c >>= 64;
    for (int j = 1; j < 4; ++j) { c += (u128)m * FR_[j] + t[j]; t[j - 1] = (u64)c; c >>= 64; }
    c += t[4]; t[3] = (u64)c; t[4] = t[5] + (u64)(c >> 64);
  }
  fr r; memcpy(r.v, t, 32);
  if (t[4] || fr_geq(&r)) fr_subr(&r);
  return r;
}
static fr fr_from_u64(u64 x) { fr a = {{x, 0, 0, 0}}, r2; memcpy(r2.v, FR_R2, 32); return fr_mul(a, r2); }
static fr fr_sub(fr a, fr b) {
  u128 br = 0; fr r;
  for (int i = 0; i < 4; ++i) { u128 d = (u128)a.v[i] - b.v[i] - br; r.v[i] = (u64)d; br = (d >> 64) & 1; }
  if (br) { u128 c = 0; for (int i = 0; i < 4; ++i) { c += (u128)r.v[i] + FR_[i]; r.v[i] = (u64)c; c >>= 64; } }
  return r;
}
static fr fr_inv(fr a) {
  fr r = fr_from_u64(1);
  for (int i = 254; i >= 0; --i) { r = fr_mul(r, r); if ((FR_EM2[i >> 6] >> (i & 63)) & 1) r = fr_mul(r, a); }
  return r;
}
static void fr_to_u64s(fr a, u64 out[4]) { fr one = {{1, 0, 0, 0}}; fr s = fr_mul(a, one); memcpy(out, s.v, 32); }

/* ------------------------------------------------------------------ pairing check */
typedef struct { fp2 x, y, z; } g2p;
static void dbl_step(g2p* T, fp nxp, fp yp, fp2* c0, fp2* c2, fp2* c3) {
  fp2 t0 = f2_sqr(T->y), t1 = f2_sqr(T->z), t2 = f2_mul(t1, f2c(B2_3)), t3 = f2_add(f2_dbl(t2), t2);
  fp2 xy = f2_mul(T->x, T->y);
  xy.c0 = fp_half(xy.c0); xy.c1 = fp_half(xy.c1);
  fp2 yz2 = f2_sub(f2_sqr(f2_add(T->y, T->z)), f2_add(t0, t1)), x2 = f2_sqr(T->x);
  *c0 = f2_sub(t0, t2);
  *c2 = f2_mulfp(f2_add(f2_dbl(x2), x2), nxp);
  *c3 = f2_mulfp(yz2, yp);
  fp2 h = f2_add(t0, t3);
  h.c0 = fp_half(h.c0); h.c1 = fp_half(h.c1);
  fp2 t2s = f2_sqr(t2);
  T->x = f2_mul(xy, f2_sub(t0, t3));
  T->y = f2_sub(f2_sqr(h), f2_add(f2_dbl(t2s), t2s));
  T->z = f2_mul(t0, yz2);
}
static void add_step(g2p* T, fp2 qx, fp2 qy, fp nxp, fp yp, fp2* c0, fp2* c2, fp2* c3) {
  fp2 th = f2_sub(T->y, f2_mul(qy, T->z)), la = f2_sub(T->x, f2_mul(qx, T->z));
  fp2 C = f2_sqr(th), D = f2_sqr(la), E = f2_mul(la, D), F = f2_mul(T->z, C), G = f2_mul(T->x, D);
  fp2 H = f2_sub(f2_add(E, F), f2_dbl(G));
  *c0 = f2_sub(f2_mul(th, qx), f2_mul(la, qy));
  *c2 = f2_mulfp(th, nxp);
  *c3 = f2_mulfp(la, yp);
  fp2 ye = f2_mul(T->y, E);
  T->x = f2_mul(la, H);
  T->y = f2_sub(f2_mul(th, f2_sub(G, H)), ye);
  T->z = f2_mul(T->z, E);
}
static fp12 miller2(fp2 q1x, fp2 q1y, fp p1x, fp p1y, fp2 q2x, fp2 q2y, fp p2x, fp p2y) {
  g2p T1 = {q1x, q1y, f2_one()}, T2 = {q2x, q2y, f2_one()};
  fp n1 = fp_neg(p1x), n2 = fp_neg(p2x);
  fp12 f = f12_one();
  fp2 a, b, c;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = f12_sqr(f);
    dbl_step(&T1, n1, p1y, &a, &b, &c); f = f12_mul_line(f, a, b, c);
    dbl_step(&T2, n2, p2y, &a, &b, &c); f = f12_mul_line(f, a, b, c);
    if ((XABS >> i) & 1) {
      add_step(&T1, q1x, q1y, n1, p1y, &a, &b, &c); f = f12_mul_line(f, a, b, c);
      add_step(&T2, q2x, q2y, n2, p2y, &a, &b, &c); f = f12_mul_line(f, a, b, c);
    }
  }
  return f12_conj(f);
}
static fp12 pow_absx(fp12 a) { fp12 r = a; for (int i = 62; i >= 0; --i) { r = f12_cyc_sqr(r); if ((XABS >> i) & 1) r = f12_mul(r, a); } return r; }
static fp12 exp_x(fp12 a) { return f12_conj(pow_absx(a)); }
static fp12 final_exp(fp12 f) {
  fp12 t = f12_mul(f12_conj(f), f12_inv(f));
  t = f12_mul(f12_frob(t, 2), t);
  fp12 t0 = f12_mul(exp_x(t), f12_conj(t));
  fp12 t1 = f12_mul(exp_x(t0), f12_conj(t0));
  fp12 t2 = f12_mul(exp_x(t1), f12_frob(t1, 1));
  fp12 t3 = f12_mul(f12_mul(exp_x(exp_x(t2)), f12_frob(t2, 2)), f12_conj(t2));
  return f12_mul(t3, f12_mul(f12_sqr(t), t));
}

/* ------------------------------------------------------------------ public (ctypes) API */
int ref_verify_msg(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig, size_t sig_len) {
  fp px, py;
  if (g1_decode(&px, &py, pk48) != R_OK) return 100;
  fp2 sx, sy;
  int rc = g2_decode(&sx, &sy, sig, sig_len);
  if (rc != R_OK) return rc;
  g2 h = hash_to_g2(msg32);
  fp2 hx, hy;
  g2_affine(&h, &hx, &hy);
  fp12 f = miller2(hx, hy, px, py, sx, sy, fpc(G1X), fp_neg(fpc(G1Y)));
  return f12_is_one(final_exp(f)) ? R_OK : R_PAIRING;
}

void ref_digest(int chained, const uint8_t* prev, size_t prev_len, u64 round, uint8_t out[32]) {
  uint8_t be[8];
  for (int i = 0; i < 8; ++i) be[i] = (uint8_t)(round >> (56 - 8 * i));
  const uint8_t* s[2] = {prev, be};
  size_t l[2] = {chained ? prev_len : 0, 8};
  sha256_segs(out, s + (l[0] ? 0 : 1), l + (l[0] ? 0 : 1), l[0] ? 2 : 1);
}

int ref_verify_beacon(int chained, const uint8_t* pk48, u64 round, const uint8_t* prev, size_t prev_len,
                      const uint8_t* sig, size_t sig_len) {
  uint8_t m[32];
  ref_digest(chained, prev, prev_len, round, m);
  return ref_verify_msg(pk48, m, sig, sig_len);
}

void ref_hash_to_g2(const uint8_t* msg32, uint8_t* out96) {
  g2 h = hash_to_g2(msg32);
  fp2 x, y;
  g2_affine(&h, &x, &y);
  fp_to_be48(x.c1, out96);
  fp_to_be48(x.c0, out96 + 48);
  out96[0] |= 0x80;
  if (f2_lexi(y)) out96[0] |= 0x20;
}

typedef struct {
  int chained; const uint8_t* pk; size_t lo, hi; const u64* rounds; const uint8_t* sigs; size_t sig_stride;
  const uint32_t* sig_len; const uint8_t* prev; size_t prev_stride; const uint32_t* prev_len; uint8_t* reason;
} job_t;
static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->reason[i] = (uint8_t)ref_verify_beacon(j->chained, j->pk, j->rounds[i], j->prev ? j->prev + i * j->prev_stride : NULL,
                                              j->prev ? j->prev_len[i] : 0, j->sigs + i * j->sig_stride, j->sig_len[i]);
  return NULL;
}
/* n beacons over `threads` pthreads; reason[i] = 0 valid, else the error class */
int ref_verify_batch(int chained, const uint8_t* pk48, size_t n, const u64* rounds, const uint8_t* sigs,
                     size_t sig_stride, const uint32_t* sig_len, const uint8_t* prev, size_t prev_stride,
                     const uint32_t* prev_len, int threads, uint8_t* reason) {
  if (threads < 1) threads = 1;
  pthread_t tid[256];
  job_t jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_t){chained, pk48, n * t / threads, n * (t + 1) / threads, rounds, sigs, sig_stride, sig_len,
                      chained ? prev : NULL, prev_stride, prev_len, reason};
    pthread_create(&tid[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  return 0;
}

/* ------------------------------------------------------------------ signatures on G1 (bls-unchained-on-g1 and its RFC DST) */
/* VerifyBeacon for the G1-signature schemes: msg = SHA-256(BE64(round)) hashed
   to G1 (legacy: the G2 suite's DST; rfc: the G1 suite's), signature 48-byte
   G1, key 96-byte G2: e(H, pk) e(-sig, g2) == 1.  Reason codes as above;
   100 = bad key. */
int ref_verify_beacon_g1(int rfc_dst, const uint8_t* pk96, u64 round, const uint8_t* sig, size_t sig_len) {
  fp2 kx, ky;
  if (g2_decode(&kx, &ky, pk96, 96) != R_OK) return 100;
  fp sx, sy;
  int rc = g1_decode_sig(&sx, &sy, sig, sig_len);
  if (rc != R_OK) return rc;
  uint8_t m[32];
  ref_digest(0, NULL, 0, round, m);
  g1 h = hash_to_g1(m, rfc_dst ? DST_G1 : DST);
  fp hx, hy;
  g1_affine(&h, &hx, &hy);
  fp12 f = miller2(kx, ky, hx, hy, f2c(G2X), f2c(G2Y), sx, fp_neg(sy));
  return f12_is_one(final_exp(f)) ? R_OK : R_PAIRING;
}

void ref_hash_to_g1(int rfc_dst, const uint8_t* msg32, uint8_t* out48) {
  g1 h = hash_to_g1(msg32, rfc_dst ? DST_G1 : DST);
  fp x, y;
  g1_affine(&h, &x, &y);
  fp_to_be48(x, out48);
  out48[0] |= 0x80;
  if (fp_gt_half(y)) out48[0] |= 0x20;
}

typedef struct { int rfc; const uint8_t* pk; size_t lo, hi; const u64* rounds; const uint8_t* sigs; size_t sig_stride;
                 const uint32_t* sig_len; uint8_t* reason; } job_g1_t;
static void* worker_g1(void* arg) {
  job_g1_t* j = (job_g1_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->reason[i] = (uint8_t)ref_verify_beacon_g1(j->rfc, j->pk, j->rounds[i], j->sigs + i * j->sig_stride, j->sig_len[i]);
  return NULL;
}
int ref_verify_batch_g1(int rfc_dst, const uint8_t* pk96, size_t n, const u64* rounds, const uint8_t* sigs,
                        size_t sig_stride, const uint32_t* sig_len, int threads, uint8_t* reason) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job_g1_t jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_g1_t){rfc_dst, pk96, n * t / threads, n * (t + 1) / threads, rounds, sigs, sig_stride, sig_len, reason};
    pthread_create(&tid[t], NULL, worker_g1, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  return 0;
}

/* ------------------------------------------------------------------ threshold recovery (kyber tbls.Recover (R)) */
/* Restates oracle/drand_ref.recover: walk the partials in order, keep those
   whose index is readable and that pass VerifyPartial against
   PubPoly.Eval(index) = sum_j C_j (index + 1)^j, stop at t; sort by index,
   first t distinct; Lagrange at 0 over x = index + 1 (Fr); G2 MSM; then
   VerifyRecovered under C_0.  Returns 1 and the 96-byte signature, or 0. */
static int verify_pt(fp px, fp py, const uint8_t* msg32, const uint8_t* sig, size_t len, fp2* sx, fp2* sy) {
  int rc = g2_decode(sx, sy, sig, len);
  if (rc != R_OK) return rc;
  g2 h = hash_to_g2(msg32);
  fp2 hx, hy;
  g2_affine(&h, &hx, &hy);
  fp12 f = miller2(hx, hy, px, py, *sx, *sy, fpc(G1X), fp_neg(fpc(G1Y)));
  return f12_is_one(final_exp(f)) ? R_OK : R_PAIRING;
}
int ref_recover(const uint8_t* commits48, int t, const uint8_t* msg32, const uint8_t* partials, size_t pstride,
                const uint32_t* plen, int m, uint8_t* out96) {
  if (t < 1 || t > 64) return 0;
  g1 C[64];
  for (int j = 0; j < t; ++j) {
    fp x, y;
    if (g1_decode(&x, &y, commits48 + 48 * j) != R_OK) return 0;
    C[j] = (g1){x, y, fp_one()};
  }
  int idx[64], cnt = 0;
  fp2 sx[64], sy[64];
  for (int k = 0; k < m && cnt < t; ++k) {
    const uint8_t* pp = partials + (size_t)k * pstride;
    if (plen[k] < 2) continue;
    int i = (pp[0] << 8) | pp[1];
    u64 xv = (u64)i + 1;
    g1 e = C[t - 1];
    for (int j = t - 2; j >= 0; --j) e = g1_add(g1_mul_u64s(e, &xv, 17), C[j]);
    if (g1_inf(&e)) continue;
    fp ex, ey;
    g1_affine(&e, &ex, &ey);
    if (verify_pt(ex, ey, msg32, pp + 2, plen[k] - 2, &sx[cnt], &sy[cnt]) != R_OK) continue;
    idx[cnt++] = i;
  }
  /* sort by index (stable), first t distinct */
  for (int a = 1; a < cnt; ++a)
    for (int b = a; b > 0 && idx[b - 1] > idx[b]; --b) {
      int ti = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = ti;
      fp2 tx = sx[b]; sx[b] = sx[b - 1]; sx[b - 1] = tx;
      fp2 ty = sy[b]; sy[b] = sy[b - 1]; sy[b - 1] = ty;
    }
  int sel[64], ns = 0;
  for (int a = 0; a < cnt && ns < t; ++a)
    if (ns == 0 || idx[sel[ns - 1]] != idx[a]) sel[ns++] = a;
  if (ns < t) return 0;
  g2 acc = g2_infinity();
  for (int a = 0; a < ns; ++a) {
    fr xa = fr_from_u64((u64)idx[sel[a]] + 1), num = fr_from_u64(1), den = fr_from_u64(1);
    for (int b = 0; b < ns; ++b) {
      if (b == a) continue;
      fr xb = fr_from_u64((u64)idx[sel[b]] + 1);
      num = fr_mul(num, xb);
      den = fr_mul(den, fr_sub(xb, xa));
    }
    u64 lam[4];
    fr_to_u64s(fr_mul(num, fr_inv(den)), lam);
    g2 q = {sx[sel[a]], sy[sel[a]], f2_one()};
    acc = g2_add(acc, g2_mul_u64s(q, lam, 256));
  }
  if (g2_inf(&acc)) return 0;
  fp2 x, y;
  g2_affine(&acc, &x, &y);
  fp_to_be48(x.c1, out96);
  fp_to_be48(x.c0, out96 + 48);
  out96[0] |= 0x80;
  if (f2_lexi(y)) out96[0] |= 0x20;
  fp cx, cy;
  g1_affine(&C[0], &cx, &cy);
  fp2 rx, ry;
  return verify_pt(cx, cy, msg32, out96, 96, &rx, &ry) == R_OK;
}

typedef struct { const uint8_t* commits; int t; const uint8_t* msgs; const uint8_t* parts; size_t pstride;
                 const uint32_t* plen; int m; size_t lo, hi; uint8_t* out; uint8_t* ok; } job_rec_t;
static void* worker_rec(void* arg) {
  job_rec_t* j = (job_rec_t*)arg;
  for (size_t r = j->lo; r < j->hi; ++r)
    j->ok[r] = (uint8_t)ref_recover(j->commits, j->t, j->msgs + 32 * r, j->parts + r * j->m * j->pstride, j->pstride,
                                    j->plen + r * j->m, j->m, j->out + 96 * r);
  return NULL;
}
int ref_recover_batch(const uint8_t* commits48, int t, size_t n_rounds, const uint8_t* msgs32, const uint8_t* partials,
                      size_t pstride, const uint32_t* plen, int m, int threads, uint8_t* out96, uint8_t* ok) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job_rec_t jobs[256];
  for (int k = 0; k < threads; ++k) {
    jobs[k] = (job_rec_t){commits48, t, msgs32, partials, pstride, plen, m, n_rounds * k / threads,
                          n_rounds * (k + 1) / threads, out96, ok};
    pthread_create(&tid[k], NULL, worker_rec, &jobs[k]);
  }
  for (int k = 0; k < threads; ++k) pthread_join(tid[k], NULL);
  return 0;
}
