// Scalar field Fr of BLS12-381 (r = 0x73eda753...00000001, 255 bits) for the
// Lagrange coefficients of threshold recovery (kyber share.RecoverCommit (R)):
// 10 x 28-bit limbs, Montgomery form with R = 2^280.  Values are kept
// normalized and < 2r; fr_canon gives [0, r).  Constants derived in
// tools/gen_constants.py terms: FR_RINV = -r^-1 mod 2^28, FR_ONE = R mod r,
// FR_R2 = R^2 mod r (checked by tests/test_hostsim.py).
#pragma once
#include "fp.cuh"

namespace dgpu {

constexpr int FR_LIMBS = 10;
constexpr uint32_t FR_P[FR_LIMBS] = {0x1, 0xffffff0, 0xe5bfeff, 0xa402fff, 0x80553bd,
                                     0x809a1d, 0x83339d8, 0x299d7d4, 0x3eda753, 0x7};
constexpr uint32_t FR_RINV = 0xfffffff;
constexpr uint32_t FR_R2[FR_LIMBS] = {0xc31bba9, 0x3b3440e, 0xe045fb0, 0x8929657, 0x57c6e1a,
                                      0x2d645cf, 0x12ecf5, 0xea6a1c5, 0xc7b9d12, 0x3};
constexpr uint32_t FR_ONE_M[FR_LIMBS] = {0xdcaaf6c, 0x355093f, 0x8209402, 0x41e37a6, 0x135587d,
                                         0x26172ba, 0x6854f56, 0x3973f39, 0xbc66e55, 0x6};
// r - 2, little-endian 32-bit words (Fermat inversion exponent)
constexpr uint32_t FR_EXP_INV[8] = {0xffffffff, 0xfffffffe, 0xfffe5bfe, 0x53bda402,
                                    0x9a1d805, 0x3339d808, 0x299d7d48, 0x73eda753};

struct fr {
  uint32_t l[FR_LIMBS];
};

DG_FN fr fr_from_limbs(const uint32_t* v) {
  fr a;
#pragma unroll
  for (int i = 0; i < FR_LIMBS; ++i) a.l[i] = v[i];
  return a;
}

// a, b normalized, < 2^281; result (a b + m r) / R < 2r for a, b < 2r.
DG_FN fr fr_mul(const fr& a, const fr& b) {
  uint32_t t[2 * FR_LIMBS];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * FR_LIMBS - 1; ++k) {
#pragma unroll
    for (int i = (k < FR_LIMBS ? 0 : k - FR_LIMBS + 1); i <= (k < FR_LIMBS ? k : FR_LIMBS - 1); ++i)
      acc += (uint64_t)a.l[i] * b.l[k - i];
    t[k] = (uint32_t)acc & FP_MASK;
    acc >>= FP_BITS;
  }
  t[2 * FR_LIMBS - 1] = (uint32_t)acc;
  uint32_t m[FR_LIMBS];
  fr r;
  acc = 0;
#pragma unroll
  for (int k = 0; k < FR_LIMBS; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * FR_P[k - i];
    acc += t[k];
    m[k] = ((uint32_t)acc * FR_RINV) & FP_MASK;
    acc += (uint64_t)m[k] * FR_P[0];
    acc >>= FP_BITS;
  }
#pragma unroll
  for (int k = FR_LIMBS; k < 2 * FR_LIMBS; ++k) {
#pragma unroll
    for (int i = k - FR_LIMBS + 1; i < FR_LIMBS; ++i) acc += (uint64_t)m[i] * FR_P[k - i];
    acc += t[k];
    if (k < 2 * FR_LIMBS - 1) {
      r.l[k - FR_LIMBS] = (uint32_t)acc & FP_MASK;
      acc >>= FP_BITS;
    } else {
      r.l[k - FR_LIMBS] = (uint32_t)acc;
    }
  }
  return r;
}

// canonical representative in [0, r) of a normalized value < 2r
DG_FN fr fr_canon(const fr& a) {
  fr d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < FR_LIMBS; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)FR_P[i] + c;
    d.l[i] = (uint32_t)s & FP_MASK;
    c = s >> FP_BITS;
  }
  return c < 0 ? a : d;
}

// small non-negative integer -> Montgomery form
DG_FN fr fr_from_u32(uint32_t x) {
  fr a{};
  a.l[0] = x & FP_MASK;
  a.l[1] = x >> FP_BITS;
  return fr_mul(a, fr_from_limbs(FR_R2));
}

// r - a for canonical a in [0, r) (a != 0), normalized
DG_FN fr fr_neg(const fr& a) {
  fr d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < FR_LIMBS; ++i) {
    int32_t s = (int32_t)FR_P[i] - (int32_t)a.l[i] + c;
    d.l[i] = (uint32_t)s & FP_MASK;
    c = s >> FP_BITS;
  }
  return d;
}

DG_FN fr fr_inv(const fr& a) {
  fr r = fr_from_limbs(FR_ONE_M);
  for (int i = 254; i >= 0; --i) {
    r = fr_mul(r, r);
    if ((FR_EXP_INV[i >> 5] >> (i & 31)) & 1u) r = fr_mul(r, a);
  }
  return r;
}

// Montgomery -> canonical integer as 8 little-endian 32-bit words
DG_FN void fr_to_words(const fr& a, uint32_t* w) {
  fr one{};
  one.l[0] = 1;
  fr s = fr_canon(fr_mul(a, one));
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = 0;
#pragma unroll
  for (int i = 0; i < FR_LIMBS; ++i) {
    const int bit = i * FP_BITS;
    w[bit >> 5] |= s.l[i] << (bit & 31);
    if ((bit & 31) > 32 - FP_BITS && (bit >> 5) + 1 < 8) w[(bit >> 5) + 1] |= s.l[i] >> (32 - (bit & 31));
  }
}

// Lagrange basis coefficient at 0 for point j of the distinct points xs[0..t)
// (x_i = share index + 1):  prod_{m != j} x_m / (x_m - x_j)  (mod r), as words.
DG_FN void fr_lagrange_at_zero(const uint32_t* xs, int t, int j, uint32_t* out_words) {
  fr num = fr_from_limbs(FR_ONE_M), den = fr_from_limbs(FR_ONE_M);
  bool negative = false;
  for (int m = 0; m < t; ++m) {
    if (m == j) continue;
    num = fr_mul(num, fr_from_u32(xs[m]));
    const int64_t d = (int64_t)xs[m] - (int64_t)xs[j];
    den = fr_mul(den, fr_from_u32((uint32_t)(d < 0 ? -d : d)));
    negative ^= d < 0;
  }
  fr l = fr_canon(fr_mul(num, fr_inv(den)));
  if (negative) {
    bool zero = true;
    for (int i = 0; i < FR_LIMBS; ++i) zero = zero && l.l[i] == 0;
    if (!zero) l = fr_neg(l);
  }
  fr_to_words(l, out_words);
}

}  // namespace dgpu
