// Fp arithmetic for BLS12-381 on gfx950: 14 x 28-bit unsaturated limbs held
// in 32-bit VGPRs, Montgomery form with R = 2^392.
//
// Why this shape (measured, profiles/r01_microbench_*.txt): on gfx950
// v_mad_u64_u32 issues at ~half rate (33.5 T/s chip-wide) and carry-chained
// v_add_co/v_addc pairs serialize on VCC, while plain v_add_u32 is full rate.
// 28-bit limbs leave 4 bits of headroom per limb, so a 14-term product column
// (each term < 2^60) accumulates in one 64-bit register pair with a single
// v_mad_u64_u32 per partial product and no carry flags at all, and field
// additions are 14 carry-free v_add_u32 (normalized lazily).
//
// Value invariant of every public op ("CI"): limbs normalized (< 2^28 each),
// value < 2.01 p.  fp_mul / fp_sqr accept any inputs whose limbs are < 2^30
// and whose values multiply to < R*p (~2600 p^2), and return CI (< 1.01 p).
// Functions with the suffix _lz are lazy (unnormalized) and document the
// bounds their callers rely on.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "constants.h"

#ifndef DG_FN
#define DG_FN __host__ __device__ __forceinline__
#endif
// Out-of-line on the device: keeps loop bodies small enough for the
// instruction cache and the compile tractable (args/returns stay in VGPRs
// for Fp-sized values).
#ifndef DG_NOINL
#define DG_NOINL __host__ __device__ __noinline__
#endif
// The Fp multiply/square/reduce kernels: out of line by default; with
// DG_INLINE_FP they are inlined into their (out-of-line) callers.
#ifdef DG_INLINE_FP
#define DG_FPK DG_FN
#else
#define DG_FPK DG_NOINL
#endif

// Operation counters for the test-only host build (tests/hostsim, tools/count_ops.py):
// the executed algorithm's Fp mul/sqr counts feed the roofline's work figure.
#if defined(DG_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long dg_count_mul, dg_count_sqr;
#define DG_COUNT(x) (++(x))
#define DG_COUNT_N(x, n) ((x) += (n))
#else
#define DG_COUNT(x)
#define DG_COUNT_N(x, n)
#endif

namespace dgpu {

struct fp {
  uint32_t l[FP_LIMBS];
};
#define FP_CONST(...) ::dgpu::fp{{__VA_ARGS__}}

DG_FN fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = 0;
  return r;
}

DG_FN fp fp_one() { return FP_ONE_MONT; }

// ---------------------------------------------------------------- Montgomery
// Separated operand scanning in product-scanning order: the full product as
// 27 unnormalized 64-bit columns (one v_mad_u64_u32 per partial product, no
// carry handling), then the Montgomery reduction over the columns into a
// running 64-bit accumulator.  Column bound: 14 products of limbs < 2^30 are
// < 14 * 2^60, plus the reduction's 14 m * p terms (< 2^56 each) and carry:
// < 2^64.  (Round 1 normalized the columns first: 540 VALU instructions per
// multiplication and 484 per squaring, against 490 and 422 in this form.)
#define DG_LIMB_PARAMS(x)                                                                                     \
  uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, uint32_t x##6,   \
      uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11, uint32_t x##12, uint32_t x##13
#define DG_LIMB_ARGS(v)                                                                                       \
  (v).l[0], (v).l[1], (v).l[2], (v).l[3], (v).l[4], (v).l[5], (v).l[6], (v).l[7], (v).l[8], (v).l[9], (v).l[10], \
      (v).l[11], (v).l[12], (v).l[13]
#define DG_LIMB_PACK(x) fp{{x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11, x##12, x##13}}

// The out-of-line Fp kernels take limbs as scalar arguments: the AMDGPU
// calling convention passes a second 14-dword struct byval through scratch,
// which would put a store/load round trip (and an exposed wait) in front of
// every multiplication.  28 scalars travel in v0..v27.
// Montgomery reduction of unnormalized product columns t[k] (< 2^64 - 2^60):
// T / R mod p, normalized limbs, < T/R + p.
DG_FN fp fp_redc_cols(const uint64_t* t) {
  fp r;
  uint32_t m[FP_LIMBS];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * FP_P[k - i];
    acc += t[k];
    m[k] = ((uint32_t)acc * FP_PINV) & FP_MASK;
    acc += (uint64_t)m[k] * FP_P[0];
    acc >>= FP_BITS;
  }
#pragma unroll
  for (int k = FP_LIMBS; k < 2 * FP_LIMBS; ++k) {
#pragma unroll
    for (int i = k - FP_LIMBS + 1; i < FP_LIMBS; ++i) acc += (uint64_t)m[i] * FP_P[k - i];
    acc += t[k];
    if (k < 2 * FP_LIMBS - 1) {
      r.l[k - FP_LIMBS] = (uint32_t)acc & FP_MASK;
      acc >>= FP_BITS;
    } else {
      r.l[k - FP_LIMBS] = (uint32_t)acc;
    }
  }
  return r;
}

#if defined(DG_FP_SOS)
// Product columns left unnormalized (each < 14 * 2^60 for limbs < 2^30)
// and fed straight to the reduction.
DG_FPK fp fp_mul_r(DG_LIMB_PARAMS(x), DG_LIMB_PARAMS(y)) {
  const fp a = DG_LIMB_PACK(x), b = DG_LIMB_PACK(y);
  DG_COUNT(dg_count_mul);
  uint64_t t[2 * FP_LIMBS];
#pragma unroll
  for (int k = 0; k < 2 * FP_LIMBS - 1; ++k) {
    uint64_t c = 0;
#pragma unroll
    for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); i <= (k < FP_LIMBS ? k : FP_LIMBS - 1); ++i)
      c += (uint64_t)a.l[i] * b.l[k - i];
    t[k] = c;
  }
  t[2 * FP_LIMBS - 1] = 0;
  return fp_redc_cols(t);
}

// Squaring: cross products once, doubled per column.
DG_FPK fp fp_sqr_r(DG_LIMB_PARAMS(x)) {
  const fp a = DG_LIMB_PACK(x);
  DG_COUNT(dg_count_sqr);
  uint64_t t[2 * FP_LIMBS];
#pragma unroll
  for (int k = 0; k < 2 * FP_LIMBS - 1; ++k) {
    uint64_t c = 0;
#pragma unroll
    for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); 2 * i < k; ++i) c += (uint64_t)a.l[i] * a.l[k - i];
    c <<= 1;
    if ((k & 1) == 0) c += (uint64_t)a.l[k / 2] * a.l[k / 2];
    t[k] = c;
  }
  t[2 * FP_LIMBS - 1] = 0;
  return fp_redc_cols(t);
}
#else
// Finely integrated product scanning (FIPS): column k of the product and of
// the reduction's m * p go into one running 64-bit accumulator (same bound
// as above: < 14 * 2^60 + 14 * 2^56 + carry < 2^64), so no 27-column array
// is held: ~50 VGPRs instead of 81 for the separated form.  These functions
// are called out of line from loops whose live state must survive the calls
// in the registers a call does not clobber, so their register footprint
// matters as much as their instruction count.
DG_FPK fp fp_mul_r(DG_LIMB_PARAMS(x), DG_LIMB_PARAMS(y)) {
  const fp a = DG_LIMB_PACK(x), b = DG_LIMB_PACK(y);
  DG_COUNT(dg_count_mul);
  uint32_t m[FP_LIMBS];
  fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * FP_LIMBS; ++k) {
#pragma unroll
    for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); i <= (k < FP_LIMBS ? k : FP_LIMBS - 1); ++i)
      if (k < 2 * FP_LIMBS - 1) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); i < (k < FP_LIMBS ? k : FP_LIMBS); ++i)
      acc += (uint64_t)m[i] * FP_P[k - i];
    if (k < FP_LIMBS) {
      m[k] = ((uint32_t)acc * FP_PINV) & FP_MASK;
      acc += (uint64_t)m[k] * FP_P[0];
      acc >>= FP_BITS;
    } else if (k < 2 * FP_LIMBS - 1) {
      r.l[k - FP_LIMBS] = (uint32_t)acc & FP_MASK;
      acc >>= FP_BITS;
    } else {
      r.l[k - FP_LIMBS] = (uint32_t)acc;
    }
  }
  return r;
}

// Squaring: cross products once, doubled per column, then the column's
// reduction terms (FIPS as fp_mul_r).
DG_FPK fp fp_sqr_r(DG_LIMB_PARAMS(x)) {
  const fp a = DG_LIMB_PACK(x);
  DG_COUNT(dg_count_sqr);
  uint32_t m[FP_LIMBS];
  fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * FP_LIMBS; ++k) {
    if (k < 2 * FP_LIMBS - 1) {
      uint64_t c = 0;
#pragma unroll
      for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); 2 * i < k; ++i) c += (uint64_t)a.l[i] * a.l[k - i];
      acc += c << 1;
      if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
    }
#pragma unroll
    for (int i = (k < FP_LIMBS ? 0 : k - FP_LIMBS + 1); i < (k < FP_LIMBS ? k : FP_LIMBS); ++i)
      acc += (uint64_t)m[i] * FP_P[k - i];
    if (k < FP_LIMBS) {
      m[k] = ((uint32_t)acc * FP_PINV) & FP_MASK;
      acc += (uint64_t)m[k] * FP_P[0];
      acc >>= FP_BITS;
    } else if (k < 2 * FP_LIMBS - 1) {
      r.l[k - FP_LIMBS] = (uint32_t)acc & FP_MASK;
      acc >>= FP_BITS;
    } else {
      r.l[k - FP_LIMBS] = (uint32_t)acc;
    }
  }
  return r;
}
#endif

// ---------------------------------------------------------------- normalization
// Carry-propagate: limbs < 2^28 except the top one.  Input limbs < 2^31.
DG_FN fp fp_norm(const fp& a) {
  fp r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS - 1; ++i) {
    uint32_t s = a.l[i] + c;
    r.l[i] = s & FP_MASK;
    c = s >> FP_BITS;
  }
  r.l[FP_LIMBS - 1] = a.l[FP_LIMBS - 1] + c;
  return r;
}

// Input normalized, value < 2^392.  Output CI (< 2.01p): subtract q*p with
// q = floor(top / (floor(p / 2^364) + 1)) <= floor(value / p).
DG_FPK fp fp_reduce_r(DG_LIMB_PARAMS(x)) {
  const fp a = DG_LIMB_PACK(x);
  constexpr uint32_t PTOP1 = FP_P[FP_LIMBS - 1] + 1;
  uint32_t q = a.l[FP_LIMBS - 1] / PTOP1;
  fp r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS - 1; ++i) {
    int64_t s = (int64_t)a.l[i] - (int64_t)((uint64_t)q * FP_P[i]) + c;
    r.l[i] = (uint32_t)s & FP_MASK;
    c = s >> FP_BITS;  // arithmetic
  }
  r.l[FP_LIMBS - 1] = (uint32_t)((int64_t)a.l[FP_LIMBS - 1] - (int64_t)q * FP_P[FP_LIMBS - 1] + c);
  return r;
}

DG_FN fp fp_mul(const fp& a, const fp& b) { return fp_mul_r(DG_LIMB_ARGS(a), DG_LIMB_ARGS(b)); }
DG_FN fp fp_sqr(const fp& a) { return fp_sqr_r(DG_LIMB_ARGS(a)); }
DG_FN fp fp_reduce(const fp& a) { return fp_reduce_r(DG_LIMB_ARGS(a)); }

// ---------------------------------------------------------------- lazy add/sub
DG_FN fp fp_add_lz(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = a.l[i] + b.l[i];
  return r;
}

// a - b + 8p; b normalized with value < 7.99p.  Limbs of result < a_i + 2^29.6.
DG_FN fp fp_sub_lz(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = a.l[i] + FP_SUBK[i] - b.l[i];
  return r;
}

// a - b + 32p; b = unnormalized sum of two normalized values (value < 31.9p).
DG_FN fp fp_sub2_lz(const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = a.l[i] + FP_SUBK2[i] - b.l[i];
  return r;
}

// ---------------------------------------------------------------- safe ops (CI in, CI out)
DG_FN fp fp_add(const fp& a, const fp& b) { return fp_reduce(fp_norm(fp_add_lz(a, b))); }
DG_FN fp fp_sub(const fp& a, const fp& b) { return fp_reduce(fp_norm(fp_sub_lz(a, b))); }
DG_FN fp fp_neg(const fp& a) { return fp_sub(fp_zero(), a); }
DG_FN fp fp_dbl(const fp& a) { return fp_add(a, a); }

// a / 2 mod p.  a CI.  If odd add p (value < 3.01p), then shift right.
DG_NOINL fp fp_half(fp a) {
  uint32_t odd = a.l[0] & 1u;
  uint32_t mask = 0u - odd;
  fp t;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) t.l[i] = a.l[i] + (FP_P[i] & mask);
  t = fp_norm(t);
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS - 1; ++i) r.l[i] = (t.l[i] >> 1) | ((t.l[i + 1] & 1u) << (FP_BITS - 1));
  r.l[FP_LIMBS - 1] = t.l[FP_LIMBS - 1] >> 1;
  return r;
}

DG_FN fp fp_cmov(const fp& a, const fp& b, bool take_b) {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = take_b ? b.l[i] : a.l[i];
  return r;
}

// ---------------------------------------------------------------- canonical form
// Exact reduction of a normalized value < 2p into [0, p).
DG_NOINL fp fp_csub_p(fp a) {
  fp d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)FP_P[i] + c;
    d.l[i] = (uint32_t)s & FP_MASK;
    c = s >> FP_BITS;
  }
  // c < 0 <=> a < p
  return fp_cmov(d, a, c < 0);
}

// Montgomery -> standard canonical integer in [0, p).
DG_FN fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_csub_p(fp_mul(a, one));  // < p + 2^-10 p
}

// standard integer (limbs normalized, value < 2^384) -> Montgomery (CI)
DG_FN fp fp_to_mont(const fp& a) { return fp_mul(a, FP_R2); }

DG_FN bool fp_is_zero_std(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) acc |= a.l[i];
  return acc == 0;
}

// a == 0 mod p for a CI value (normalized, < 2.01p): a is one of 0, p, 2p.
DG_FN bool fp_is_zero(const fp& a) {
  uint32_t z = 0, zp = 0, z2p = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    z |= a.l[i];
    zp |= a.l[i] ^ FP_P[i];
    z2p |= a.l[i] ^ FP_2P[i];
  }
  return z == 0 || zp == 0 || z2p == 0;
}

DG_FN bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

// ---------------------------------------------------------------- exponentiation
// Fixed 4-bit-window exponentiation by a public constant exponent (uniform
// control flow; the window table index is wave-uniform).
DG_NOINL fp fp_pow(fp a, const uint32_t* e, int nbits) {
  fp tbl[16];
  tbl[1] = a;
#pragma unroll 1
  for (int i = 2; i < 16; ++i) tbl[i] = fp_mul(tbl[i - 1], a);
  int nwin = (nbits + 3) / 4;
  int top = nwin - 1;
  uint32_t w = (e[(4 * top) >> 5] >> ((4 * top) & 31)) & 15u;
  fp r = tbl[w];  // top window is non-zero (nbits is the exact bit length)
  for (int k = top - 1; k >= 0; --k) {
    r = fp_sqr(fp_sqr(fp_sqr(fp_sqr(r))));
    w = (e[(4 * k) >> 5] >> ((4 * k) & 31)) & 15u;
    if (w) r = fp_mul(r, tbl[w]);
  }
  return r;
}

// Sliding-window (width 5) exponentiation by a public constant exponent from
// its generated schedule (tools/gen_constants.py sliding_schedule): the odd
// powers x, x^3, .., x^31 in a 16-entry table, then per step `squarings`
// squarings and one multiplication by a table entry -- about 82
// multiplications per 381-bit exponent instead of the fixed 4-bit window's
// 103.  Wave-uniform control flow (the schedule is a constant).
DG_NOINL fp fp_pow_sched(fp a, const uint32_t* sched, int nsteps, int tail) {
  fp tbl[16];
  tbl[0] = a;
  const fp a2 = fp_sqr(a);
#pragma unroll 1
  for (int i = 1; i < 16; ++i) tbl[i] = fp_mul(tbl[i - 1], a2);
  fp r = tbl[sched[0] & 0xFFu];
#pragma unroll 1
  for (int s = 1; s < nsteps; ++s) {
    const uint32_t w = sched[s];
#pragma unroll 1
    for (uint32_t q = w >> 8; q; --q) r = fp_sqr(r);
    r = fp_mul(r, tbl[w & 0xFFu]);
  }
#pragma unroll 1
  for (int q = 0; q < tail; ++q) r = fp_sqr(r);
  return r;
}
#define DG_POW(a, NAME) fp_pow_sched((a), NAME##_SCHED, (int)(sizeof(NAME##_SCHED) / sizeof(uint32_t)), NAME##_SCHED_TAIL)

// a^-1 by Fermat (a^(p-2)): 381 squarings and ~82 multiplications.
DG_FN fp fp_inv_pow(const fp& a) { return DG_POW(a, EXP_P_MINUS_2); }

// ---------------------------------------------------------------- inversion by divsteps
// Bernstein-Yang "safegcd" with half-delta divsteps (the variant whose
// iteration bound for d-bit inputs is floor((45907 d + 26313) / 19929): 879
// for d = 381), run in 32 batches of 28 on the low limb -- 896 divsteps --
// with each batch's 2x2 transition matrix applied to the full-width (f, g)
// and to the cofactors (d, e) at once.  Invariant: f = d x, g = e x (mod p),
// starting from (f, g, d, e) = (p, x, 0, 1); at the end g = 0, f = +-1 and
// x^-1 = +-d.  About 25k VALU operations against ~230k for the Fermat chain,
// and no data-dependent control flow (the batch count is the bound).
//
// Signed numbers in radix 2^28: limbs 0..12 in [0, 2^28), limb 13 signed.
struct fp_s {
  int32_t l[FP_LIMBS];
};

// 28 divsteps on the low words f, g (only their low 28 bits are read):
// returns (uf, vf; ug, vg) with 2^28 (f', g') = (uf f + vf g, ug f + vg g).
// eta = 2 delta.  The swap case (delta > 0, g odd: f' = g, g' = (g - f) / 2)
// is a swap with negation (f, g) <- (g, -f) followed by the g-odd case.
DG_FN void fp_divsteps28(int32_t& eta, int32_t f, int32_t g, int32_t& uf, int32_t& vf, int32_t& ug, int32_t& vg) {
  uf = 1, vf = 0, ug = 0, vg = 1;
#pragma unroll 4
  for (int k = 0; k < FP_BITS; ++k) {
    const bool odd = g & 1;
    const bool sw = odd && eta > 0;
    const int32_t f0 = f, uf0 = uf, vf0 = vf;
    f = sw ? g : f, uf = sw ? ug : uf, vf = sw ? vg : vf;
    g = sw ? -f0 : g, ug = sw ? -uf0 : ug, vg = sw ? -vf0 : vg;
    eta = sw ? -eta : eta;
    g += odd ? f : 0, ug += odd ? uf : 0, vg += odd ? vf : 0;
    g >>= 1, uf *= 2, vf *= 2, eta += 2;
  }
}

// (a, b) <- ((ua a + va b) / 2^28, (ub a + vb b) / 2^28), exact (the low
// 28 bits of both combinations vanish).  |u| + |v| <= 2^28, so every column
// sum stays below 2^58.
DG_FN void fp_s_apply(fp_s& a, fp_s& b, int32_t ua, int32_t va, int32_t ub, int32_t vb) {
  int64_t ca = ((int64_t)ua * a.l[0] + (int64_t)va * b.l[0]) >> FP_BITS;
  int64_t cb = ((int64_t)ub * a.l[0] + (int64_t)vb * b.l[0]) >> FP_BITS;
#pragma unroll
  for (int i = 1; i < FP_LIMBS; ++i) {
    ca += (int64_t)ua * a.l[i] + (int64_t)va * b.l[i];
    cb += (int64_t)ub * a.l[i] + (int64_t)vb * b.l[i];
    a.l[i - 1] = (int32_t)(ca & FP_MASK), b.l[i - 1] = (int32_t)(cb & FP_MASK);
    ca >>= FP_BITS, cb >>= FP_BITS;
  }
  a.l[FP_LIMBS - 1] = (int32_t)ca, b.l[FP_LIMBS - 1] = (int32_t)cb;
}

// The cofactors: (d, e) <- ((ud d + vd e + md p) / 2^28, (ue d + ve e + me p)
// / 2^28) with md, me in [0, 2^28) chosen so that the divisions are exact,
// i.e. the matrix applied mod p with the factor 2^-28.  |d|, |e| grow by < p
// per batch: < 33p after 32 (top limb < 2^24).
DG_FN void fp_s_apply_mod(fp_s& d, fp_s& e, int32_t ud, int32_t vd, int32_t ue, int32_t ve) {
  const uint32_t md = (((uint32_t)ud * (uint32_t)d.l[0] + (uint32_t)vd * (uint32_t)e.l[0]) * FP_PINV) & FP_MASK;
  const uint32_t me = (((uint32_t)ue * (uint32_t)d.l[0] + (uint32_t)ve * (uint32_t)e.l[0]) * FP_PINV) & FP_MASK;
  int64_t cd = ((int64_t)ud * d.l[0] + (int64_t)vd * e.l[0] + (int64_t)md * FP_P[0]) >> FP_BITS;
  int64_t ce = ((int64_t)ue * d.l[0] + (int64_t)ve * e.l[0] + (int64_t)me * FP_P[0]) >> FP_BITS;
#pragma unroll
  for (int i = 1; i < FP_LIMBS; ++i) {
    cd += (int64_t)ud * d.l[i] + (int64_t)vd * e.l[i] + (int64_t)md * FP_P[i];
    ce += (int64_t)ue * d.l[i] + (int64_t)ve * e.l[i] + (int64_t)me * FP_P[i];
    d.l[i - 1] = (int32_t)(cd & FP_MASK), e.l[i - 1] = (int32_t)(ce & FP_MASK);
    cd >>= FP_BITS, ce >>= FP_BITS;
  }
  d.l[FP_LIMBS - 1] = (int32_t)cd, e.l[FP_LIMBS - 1] = (int32_t)ce;
}

// r = a^-1 (Montgomery in, Montgomery out; 0 -> 0).  The Montgomery value
// x = a R is inverted as an integer (x^-1 = a^-1 R^-1) and multiplied by R^3
// through the Montgomery product: a^-1 R.  false if g has not reached 0
// (excluded by the divstep bound); fp_inv then takes the Fermat chain.
DG_FN bool fp_inv_ds(const fp& a, fp& r) {
  // work counters (tools/count_ops.py): the batches' 32 x 140 signed 32x32->64
  // mads, 4,480, as 11 multiplications' worth (392 each); fp_mul by R^3 counts itself
  DG_COUNT_N(dg_count_mul, 11);
  const fp x = fp_csub_p(fp_csub_p(a));  // CI (< 2.01p) -> [0, p)
  fp_s f, g, d, e;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    f.l[i] = (int32_t)FP_P[i], g.l[i] = (int32_t)x.l[i];
    d.l[i] = 0, e.l[i] = 0;
  }
  e.l[0] = 1;
  int32_t eta = 1;
#pragma unroll 1
  for (int b = 0; b < 32; ++b) {
    int32_t uf, vf, ug, vg;
    fp_divsteps28(eta, f.l[0], g.l[0], uf, vf, ug, vg);
    fp_s_apply(f, g, uf, vf, ug, vg);
    fp_s_apply_mod(d, e, uf, vf, ug, vg);
  }
  int32_t gz = 0, pos = f.l[0] ^ 1, neg = f.l[0] ^ (int32_t)FP_MASK;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) gz |= g.l[i];
#pragma unroll
  for (int i = 1; i < FP_LIMBS - 1; ++i) pos |= f.l[i], neg |= f.l[i] ^ (int32_t)FP_MASK;
  pos |= f.l[FP_LIMBS - 1], neg |= f.l[FP_LIMBS - 1] + 1;
  if (gz != 0) return false;
  if (pos != 0 && neg != 0) {  // gcd(p, x) = p: x = 0
    r = fp_zero();
    return true;
  }
  // +-d + 34p in (p, 67p), carried into normalized limbs; times R^3
  const int64_t sgn = pos == 0 ? 1 : -1;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    c += sgn * d.l[i] + 34 * (int64_t)FP_P[i];
    r.l[i] = (uint32_t)(c & FP_MASK);
    c >>= FP_BITS;
  }
  r.l[FP_LIMBS - 1] += (uint32_t)c << FP_BITS;
  r = fp_mul(r, FP_R3);
  return true;
}
DG_NOINL fp fp_inv(const fp& a) {
  fp r;
  if (!fp_inv_ds(a, r)) r = fp_inv_pow(a);
  return r;
}

// candidate square root a^((p+1)/4); caller checks (r^2 == a)
DG_FN fp fp_sqrt_cand(const fp& a) { return DG_POW(a, EXP_P_PLUS_1_DIV_4); }

// Legendre-style test: a is a square (or zero)
DG_FN bool fp_is_square(const fp& a) {
  fp t = DG_POW(a, EXP_P_MINUS_1_DIV_2);
  return fp_is_zero(t) || fp_eq(t, fp_one());
}

// ---------------------------------------------------------------- bytes <-> fp
// 48 big-endian bytes (value < 2^384) -> standard limbs (not Montgomery)
DG_FN fp fp_std_from_be48(const uint8_t* b) {
  fp r = fp_zero();
#pragma unroll
  for (int byte = 0; byte < 48; ++byte) {
    uint32_t v = b[47 - byte];
    int bit = byte * 8;
    r.l[bit / FP_BITS] |= (v << (bit % FP_BITS)) & FP_MASK;
    if (bit % FP_BITS > FP_BITS - 8) r.l[bit / FP_BITS + 1] |= v >> (FP_BITS - bit % FP_BITS);
  }
  return r;
}

// standard canonical limbs -> 48 big-endian bytes
DG_FN void fp_std_to_be48(const fp& a, uint8_t* b) {
#pragma unroll
  for (int byte = 0; byte < 48; ++byte) {
    int bit = byte * 8;
    uint32_t v = a.l[bit / FP_BITS] >> (bit % FP_BITS);
    if (bit % FP_BITS > FP_BITS - 8) v |= a.l[bit / FP_BITS + 1] << (FP_BITS - bit % FP_BITS);
    b[47 - byte] = (uint8_t)v;
  }
}

// a < p for standard normalized limbs
DG_FN bool fp_std_lt_p(const fp& a) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)FP_P[i] + c;
    c = s >> FP_BITS;
  }
  return c < 0;
}

// a > (p-1)/2 for standard canonical limbs, i.e. 2a > p-1, i.e. 2a >= p
DG_FN bool fp_std_gt_half(const fp& a) {
  fp d;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) d.l[i] = a.l[i] << 1;
  d = fp_norm(d);
  return !fp_std_lt_p(d);
}

}  // namespace dgpu
