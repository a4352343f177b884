// Extension tower for BLS12-381:
//   Fp2  = Fp[u]  / (u^2 + 1)
//   Fp6  = Fp2[v] / (v^3 - xi),  xi = 1 + u
//   Fp12 = Fp6[w] / (w^2 - v)
// Same tower and basis as the oracle (oracle/bls12381.py), so intermediate
// values can be compared element by element.
#pragma once
#include "fp.cuh"

namespace dgpu {

struct fp2 {
  fp c0, c1;
};
#define FP2_CONST(a, b) ::dgpu::fp2{a, b}

struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ================================================================ Fp2
DG_FN fp2 fp2_zero() { return fp2{fp_zero(), fp_zero()}; }
DG_FN fp2 fp2_one() { return fp2{fp_one(), fp_zero()}; }
DG_FN fp2 fp2_add(const fp2& a, const fp2& b) { return fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
DG_FN fp2 fp2_sub(const fp2& a, const fp2& b) { return fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
DG_FN fp2 fp2_neg(const fp2& a) { return fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
DG_FN fp2 fp2_dbl(const fp2& a) { return fp2_add(a, a); }
DG_FN fp2 fp2_conj(const fp2& a) { return fp2{a.c0, fp_neg(a.c1)}; }
DG_FN fp2 fp2_half(const fp2& a) { return fp2{fp_half(a.c0), fp_half(a.c1)}; }

// Karatsuba: 3 Fp multiplications.  Lazy sums feed the third product
// (limbs < 2^29, values < 4.02p: inside fp_mul's bounds); c1's subtrahend is
// an unnormalized sum of two CI values, handled by fp_sub2_lz.
DG_FN fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp t0 = fp_mul(a.c0, b.c0);
  fp t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add_lz(a.c0, a.c1), fp_add_lz(b.c0, b.c1));
  fp2 r;
  r.c0 = fp_sub(t0, t1);
  r.c1 = fp_reduce(fp_norm(fp_sub2_lz(t2, fp_add_lz(t0, t1))));
  return r;
}

// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u
DG_FN fp2 fp2_sqr(const fp2& a) {
  fp2 r;
  r.c0 = fp_mul(fp_add_lz(a.c0, a.c1), fp_sub_lz(a.c0, a.c1));
  r.c1 = fp_mul(fp_add_lz(a.c0, a.c0), a.c1);
  return r;
}

DG_FN fp2 fp2_mul_fp(const fp2& a, const fp& s) { return fp2{fp_mul(a.c0, s), fp_mul(a.c1, s)}; }

// ---- lazy Fp2 steps for the group law: each caller states the bounds it
// relies on (fp_mul / fp2_mul / fp2_sqr inputs: limbs < 2^30 after their own
// internal lazy sums, value products < ~2600 p^2; fp2_sqr's second coefficient
// normalized < 7.99p).  An fp2_add + fp2_dbl chain of CI ops costs a carry
// pass and a reduction per coefficient per step; these defer both.
DG_FN fp2 fp2_add_lz(const fp2& a, const fp2& b) { return fp2{fp_add_lz(a.c0, b.c0), fp_add_lz(a.c1, b.c1)}; }
// carry propagation only (input limbs < 2^31): normalized, value unchanged
DG_FN fp2 fp2_carry(const fp2& a) { return fp2{fp_norm(a.c0), fp_norm(a.c1)}; }
// k a limb-wise (k a < 2^31 per limb), unnormalized
DG_FN fp2 fp2_mulk_lz(const fp2& a, uint32_t k) {
  fp2 r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.c0.l[i] = k * a.c0.l[i], r.c1.l[i] = k * a.c1.l[i];
  return r;
}
// a - b reduced (CI): a CI, b normalized with value < 31.9p or an unnormalized
// sum of two normalized values (fp_sub2_lz's precondition)
DG_FN fp2 fp2_sub32(const fp2& a, const fp2& b) {
  return fp2{fp_reduce(fp_norm(fp_sub2_lz(a.c0, b.c0))), fp_reduce(fp_norm(fp_sub2_lz(a.c1, b.c1)))};
}

// multiply by xi = 1 + u: (a0 - a1) + (a0 + a1) u
DG_FN fp2 fp2_mul_xi(const fp2& a) { return fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

DG_FN fp2 fp2_cmov(const fp2& a, const fp2& b, bool take_b) {
  return fp2{fp_cmov(a.c0, b.c0, take_b), fp_cmov(a.c1, b.c1, take_b)};
}

DG_FN bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
DG_FN bool fp2_eq(const fp2& a, const fp2& b) { return fp2_is_zero(fp2_sub(a, b)); }

DG_FN fp fp2_norm(const fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

DG_NOINL fp2 fp2_inv(const fp2& a) {
  fp t = fp_inv(fp2_norm(a));
  return fp2{fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}

// square test in Fp2: a is a square iff its norm is a square in Fp
DG_FN bool fp2_is_square(const fp2& a) { return fp_is_square(fp2_norm(a)); }

// sqrt(w) / m^2 for w in Fp2 whose norm is g^2 (g a square root of the norm),
// m in Fp nonzero: one exponentiation, no inversion.  With d = (w0 + g) / 2
// (or (w0 - g) / 2 when that is 0, i.e. w1 = 0) and t = (d m^4)^((p-3)/4):
// d square -> d t + (w1 t / 2) u, else (w1 t / 2) - d t u.
// Derivation and model: tools/sswu_model.py (sqrt_scaled).
// fp2_sqrt_scaled in two halves around its exponentiation t = dm4^((p-3)/4)
// (the staged SSWU runs that exponentiation as its own launch): _pre returns
// d and dm4 = d m^4, _post the root from t.
DG_FN fp fp2_sqrt_scaled_pre(const fp2& w, const fp& g, const fp& m, fp& dm4) {
  fp d = fp_half(fp_add(w.c0, g));
  d = fp_cmov(d, fp_half(fp_sub(w.c0, g)), fp_is_zero(d));
  const fp m2 = fp_sqr(m);
  dm4 = fp_mul(d, fp_sqr(m2));
  return d;
}
DG_FN fp2 fp2_sqrt_scaled_post(const fp2& w, const fp& d, const fp& dm4, const fp& t) {
  const bool sq = fp_eq(fp_mul(dm4, fp_sqr(t)), fp_one());
  const fp dt = fp_mul(d, t);
  const fp wt = fp_half(fp_mul(w.c1, t));
  return sq ? fp2{dt, wt} : fp2{wt, fp_neg(dt)};
}
DG_NOINL fp2 fp2_sqrt_scaled(const fp2& w, const fp& g, const fp& m) {
  fp dm4;
  const fp d = fp2_sqrt_scaled_pre(w, g, m, dm4);
  return fp2_sqrt_scaled_post(w, d, dm4, DG_POW(dm4, EXP_P_MINUS_3_DIV_4));
}

// Square root in Fp2 (p = 3 mod 4) by the norm method in two exponentiations
// (the square test of the norm and fp2_sqrt_scaled).  Returns false if a is
// not a square.  Which of the two roots is returned does not matter: every
// caller fixes the sign afterwards (RFC 9380 sgn0 / ZCash sign bit).
DG_NOINL bool fp2_sqrt(fp2& out, const fp2& a) {
  const fp alpha = fp2_norm(a);
  const fp g = fp_sqrt_cand(alpha);
  if (!fp_eq(fp_sqr(g), alpha)) return false;
  out = fp2_sqrt_scaled(a, g, fp_one());
  return true;
}

// canonical (non-Montgomery) components
DG_FN void fp2_from_mont(fp& c0, fp& c1, const fp2& a) {
  c0 = fp_from_mont(a.c0);
  c1 = fp_from_mont(a.c1);
}

// RFC 9380 sgn0 for Fp2
DG_NOINL uint32_t fp2_sgn0(const fp2& a) {
  fp c0, c1;
  fp2_from_mont(c0, c1, a);
  uint32_t s0 = c0.l[0] & 1u;
  uint32_t z0 = fp_is_zero_std(c0) ? 1u : 0u;
  uint32_t s1 = c1.l[0] & 1u;
  return s0 | (z0 & s1);
}

// ZCash "lexicographically largest" for Fp2 y
DG_NOINL bool fp2_lexi_largest(const fp2& a) {
  fp c0, c1;
  fp2_from_mont(c0, c1, a);
  if (!fp_is_zero_std(c1)) return fp_std_gt_half(c1);
  return fp_std_gt_half(c0);
}

DG_FN fp2 fp2_frob(const fp2& a) { return fp2_conj(a); }

// ================================================================ Fp6
DG_FN fp6 fp6_zero() { return fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
DG_FN fp6 fp6_one() { return fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
DG_NOINL fp6 fp6_add(const fp6& a, const fp6& b) {
  return fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)};
}
DG_NOINL fp6 fp6_sub(const fp6& a, const fp6& b) {
  return fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)};
}
DG_NOINL fp6 fp6_neg(const fp6& a) { return fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }

// Karatsuba-style, 6 Fp2 multiplications (same formula as the oracle's f6_mul)
DG_NOINL fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp6 r;
  r.c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
  r.c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  r.c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return r;
}

DG_FN fp6 fp6_sqr(const fp6& a) { return fp6_mul(a, a); }

// multiply by v: (a0, a1, a2) -> (xi a2, a0, a1)
DG_FN fp6 fp6_mul_v(const fp6& a) { return fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }

DG_FN fp6 fp6_mul_fp2(const fp6& a, const fp2& s) {
  return fp6{fp2_mul(a.c0, s), fp2_mul(a.c1, s), fp2_mul(a.c2, s)};
}

// a * (b0 + b1 v)   (sparse: b2 = 0)
DG_NOINL fp6 fp6_mul_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = fp2_mul(a.c0, b0);
  fp2 t1 = fp2_mul(a.c1, b1);
  fp6 r;
  // c0 = t0 + xi * (a2 * b1)
  r.c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(a.c2, b1)));
  // c1 = (a0 + a1)(b0 + b1) - t0 - t1
  r.c1 = fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), fp2_add(t0, t1));
  // c2 = a2 * b0 + t1
  r.c2 = fp2_add(fp2_mul(a.c2, b0), t1);
  return r;
}

// a * (b1 v)   (sparse: only b1)
DG_NOINL fp6 fp6_mul_1(const fp6& a, const fp2& b1) {
  return fp6{fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

DG_NOINL fp6 fp6_inv(const fp6& a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return fp6{fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ================================================================ Fp12
DG_FN fp12 fp12_one() { return fp12{fp6_one(), fp6_zero()}; }

DG_NOINL fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp12 r;
  r.c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
  r.c0 = fp6_add(t0, fp6_mul_v(t1));
  return r;
}

// complex squaring: 2 Fp6 multiplications
DG_NOINL fp12 fp12_sqr(const fp12& a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp12 r;
  r.c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  r.c1 = fp6_add(ab, ab);
  return r;
}

DG_FN fp12 fp12_conj(const fp12& a) { return fp12{a.c0, fp6_neg(a.c1)}; }

DG_NOINL fp12 fp12_inv(const fp12& a) {
  fp6 t = fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1)));
  fp6 ti = fp6_inv(t);
  return fp12{fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti))};
}

// (x0 + x1 s)^2 in Fp4 = Fp2[s]/(s^2 - xi): 3 Fp2 squarings
DG_FN void fp4_sqr(fp2& r0, fp2& r1, const fp2& x0, const fp2& x1) {
  fp2 t0 = fp2_sqr(x0);
  fp2 t1 = fp2_sqr(x1);
  r0 = fp2_add(t0, fp2_mul_xi(t1));
  r1 = fp2_sub(fp2_sqr(fp2_add(x0, x1)), fp2_add(t0, t1));
}

// 3a - 2b and 3a + 2b in Fp2
DG_FN fp2 fp2_3a_m_2b(const fp2& a, const fp2& b) { fp2 t = fp2_sub(a, b); return fp2_add(fp2_dbl(t), a); }
DG_FN fp2 fp2_3a_p_2b(const fp2& a, const fp2& b) { fp2 t = fp2_add(a, b); return fp2_add(fp2_dbl(t), a); }

// Granger-Scott squaring, valid on the cyclotomic subgroup (after the easy
// part of the final exponentiation): view Fp12 = Fp4[w]/(w^3 - s), s = w^3,
// f = A + B w + C w^2 with A = (f0, f3), B = (f1, f4), C = (f2, f5):
//   A' = 3A^2 - 2 conj(A),  B' = 3 s C^2 + 2 conj(B),  C' = 3B^2 - 2 conj(C).
// 9 Fp2 squarings instead of 2 Fp6 multiplications (checked in tests).
DG_NOINL fp12 fp12_cyclo_sqr(const fp12& f) {
  fp2 a0, a1, b0, b1, c0, c1;
  fp4_sqr(a0, a1, f.c0.c0, f.c1.c1);
  fp4_sqr(b0, b1, f.c1.c0, f.c0.c2);
  fp4_sqr(c0, c1, f.c0.c1, f.c1.c2);
  fp12 r;
  r.c0.c0 = fp2_3a_m_2b(a0, f.c0.c0);
  r.c1.c1 = fp2_3a_p_2b(a1, f.c1.c1);
  r.c1.c0 = fp2_3a_p_2b(fp2_mul_xi(c1), f.c1.c0);
  r.c0.c2 = fp2_3a_m_2b(c0, f.c0.c2);
  r.c0.c1 = fp2_3a_m_2b(b0, f.c0.c1);
  r.c1.c2 = fp2_3a_p_2b(b1, f.c1.c2);
  return r;
}

// Multiply by a Miller-loop line l = c0 + c2 w^2 + c3 w^3
//   = (c0 + c2 v) + (c3 v) w   in the Fp6[w] basis.
DG_NOINL fp12 fp12_mul_line(const fp12& f, const fp2& c0, const fp2& c2, const fp2& c3) {
  // (f0 + f1 w)(L0 + L1 w) = (f0 L0 + v f1 L1) + (f0 L1 + f1 L0) w,  L0 = c0 + c2 v, L1 = c3 v
  fp6 a = fp6_mul_01(f.c0, c0, c2);
  fp6 b = fp6_mul_1(f.c1, c3);
  fp12 r;
  // (f0 + f1)(L0 + L1) - a - b
  fp2 s1 = fp2_add(c2, c3);
  r.c1 = fp6_sub(fp6_mul_01(fp6_add(f.c0, f.c1), c0, s1), fp6_add(a, b));
  r.c0 = fp6_add(a, fp6_mul_v(b));
  return r;
}

// Frobenius maps f -> f^(p^k), k = 1, 2, 3, on the w-basis coefficients.
// Basis order: 1 -> c0.c0, w -> c1.c0, w^2 -> c0.c1, w^3 -> c1.c1, w^4 -> c0.c2, w^5 -> c1.c2
DG_NOINL fp12 fp12_frob1(const fp12& a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), C_FROB1_1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), C_FROB1_2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), C_FROB1_3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), C_FROB1_4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), C_FROB1_5);
  return r;
}

DG_NOINL fp12 fp12_frob2(const fp12& a) {
  fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul_fp(a.c1.c0, fp2(C_FROB2_1).c0);
  r.c0.c1 = fp2_mul_fp(a.c0.c1, fp2(C_FROB2_2).c0);
  r.c1.c1 = fp2_mul_fp(a.c1.c1, fp2(C_FROB2_3).c0);
  r.c0.c2 = fp2_mul_fp(a.c0.c2, fp2(C_FROB2_4).c0);
  r.c1.c2 = fp2_mul_fp(a.c1.c2, fp2(C_FROB2_5).c0);
  return r;
}

DG_NOINL fp12 fp12_frob3(const fp12& a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), C_FROB3_1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), C_FROB3_2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), C_FROB3_3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), C_FROB3_4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), C_FROB3_5);
  return r;
}

DG_NOINL bool fp12_is_one(const fp12& a) {
  return fp2_eq(a.c0.c0, fp2_one()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}

}  // namespace dgpu
