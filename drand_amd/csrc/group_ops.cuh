// The signature group's law behind one interface, so the RLC batch pipeline
// (rlc_msm.cuh: bucket-MSM root, leaves, segment tree, node preparation) is
// written once for both signature groups: G2 (pedersen-bls-chained /
// -unchained, common/scheme/scheme.go:9-48) and G1 (bls-unchained-on-g1 and
// its RFC 9380 DST variant, the short-signature schemes north_star names).
//
// Each group has an efficient endomorphism that acts on the prime-order
// subgroup as a scalar, which the RLC coefficients r = a + b*lambda (a, b the
// 32-bit halves of a 64-bit draw) use to halve the doublings:
//   G2: psi (untwist-Frobenius-twist), psi = [x] on G2 (p == x mod r);
//   G1: phi(x, y) = (beta x, y), beta a cube root of unity in Fp; phi = [-x^2]
//       on G1 (the same beta as the membership test of g1sig.cuh:
//       (beta x, y) == -[x^2] P).
// Both endomorphisms are group automorphisms of the whole curve (not only of
// the subgroup), so they commute with the cofactor multiplication h_eff: for a
// pre-cofactor hash point R, h_eff ([a] R + [b] endo(R)) = [a + b lambda] H
// with H = h_eff R the hash point.  2^64 distinct (a, b) give 2^64 distinct
// coefficients mod r (|a|, |b| < 2^32 and the lattice {(a, b): a + b lambda
// == 0 mod r} has no vector that short: lambda ~ 2^64 (G2) or 2^127 (G1) with
// r ~ 2^255), the soundness of uniform 64-bit coefficients.
#pragma once
#include "curve.cuh"

namespace dgpu {

DG_NOINL g1j g1_phi(const g1j& p) { return g1j{fp_mul(C_G1_BETA, p.x), p.y, p.z}; }

DG_NOINL bool g1_eq(const g1j& p, const g1j& q) {
  const bool pi = g1_is_inf(p), qi = g1_is_inf(q);
  if (pi || qi) return pi && qi;
  const fp z1z1 = fp_sqr(p.z), z2z2 = fp_sqr(q.z);
  const bool ex = fp_eq(fp_mul(p.x, z2z2), fp_mul(q.x, z1z1));
  const bool ey = fp_eq(fp_mul(fp_mul(p.y, q.z), z2z2), fp_mul(fp_mul(q.y, p.z), z1z1));
  return ex && ey;
}

// h_eff = 1 - x = 1 + |x| (RFC 9380 8.8.1): P + [|x|] P
DG_NOINL g1j g1_clear_cofactor(const g1j& p) {
  g1j r = p;
  for (int i = 62; i >= 0; --i) {
    r = g1_dbl(r);
    if ((BLS_X_ABS >> i) & 1ull) r = g1_add(r, p);
  }
  return g1_add(r, p);
}

struct G2Ops {
  using aff = g2a;
  using jac = g2j;
  static DG_FN jac inf() { return g2_infinity(); }
  static DG_FN bool is_inf(const jac& p) { return g2_is_inf(p); }
  static DG_FN bool aff_is_zero(const aff& q) { return fp2_is_zero(q.x) && fp2_is_zero(q.y); }
  static DG_FN jac from_aff(const aff& q) { return g2_from_affine(q); }
  static DG_FN jac neg(const jac& p) { return g2_neg(p); }
  static DG_FN jac cneg(const jac& p, bool c) { return jac{p.x, fp2_cmov(p.y, fp2_neg(p.y), c), p.z}; }
  static DG_FN jac cmov(const jac& a, const jac& b, bool take_b) { return g2_cmov(a, b, take_b); }
  static DG_FN jac dbl_body(const jac& p) { return g2_dbl_body(p); }
  static DG_FN jac add_body(const jac& p, const jac& q) { return g2_add_body(p, q); }
  static DG_FN jac add_aff_body(const jac& p, const aff& q) { return g2_add_affine_body(p, q); }
  static DG_FN jac dbl(const jac& p) { return g2_dbl(p); }
  static DG_FN jac add(const jac& p, const jac& q) { return g2_add(p, q); }
  static DG_FN jac endo(const jac& p) { return g2_psi(p); }
  static DG_FN jac clear_cofactor(const jac& p) { return g2_clear_cofactor(p); }
  static DG_FN aff to_aff(const jac& p) { return g2_to_affine(p); }
  static DG_FN aff aff_zero() { return aff{fp2_zero(), fp2_zero()}; }
};

struct G1Ops {
  using aff = g1a;
  using jac = g1j;
  static DG_FN jac inf() { return g1_infinity(); }
  static DG_FN bool is_inf(const jac& p) { return g1_is_inf(p); }
  static DG_FN bool aff_is_zero(const aff& q) { return fp_is_zero(q.x) && fp_is_zero(q.y); }
  static DG_FN jac from_aff(const aff& q) { return jac{q.x, q.y, fp_one()}; }
  static DG_FN jac neg(const jac& p) { return g1_neg(p); }
  static DG_FN jac cneg(const jac& p, bool c) { return jac{p.x, fp_cmov(p.y, fp_neg(p.y), c), p.z}; }
  static DG_FN jac cmov(const jac& a, const jac& b, bool take_b) { return g1_cmov(a, b, take_b); }
  static DG_FN jac dbl_body(const jac& p) { return g1_dbl_body(p); }
  static DG_FN jac add_body(const jac& p, const jac& q) { return g1_add_body(p, q); }
  static DG_FN jac add_aff_body(const jac& p, const aff& q) { return g1_add_affine_body(p, q); }
  static DG_FN jac dbl(const jac& p) { return g1_dbl(p); }
  static DG_FN jac add(const jac& p, const jac& q) { return g1_add(p, q); }
  static DG_FN jac endo(const jac& p) { return g1_phi(p); }
  static DG_FN jac clear_cofactor(const jac& p) { return g1_clear_cofactor(p); }
  static DG_FN aff to_aff(const jac& p) { return g1_to_affine(p); }
  static DG_FN aff aff_zero() { return aff{fp_zero(), fp_zero()}; }
};

// [a] q + [b] endo(q) for an affine q (not the identity) and 32-bit a, b with
// the same operation sequence in every lane (see g2_mul2_win4_affine, of which
// this is the group-generic form): signed radix-16 windows of both scalars
// over T[m] = [m + 1] q, 8 windows of 4 doublings + 2 additions.
template <class Gr>
DG_FN typename Gr::jac mul2_win4_affine(const typename Gr::aff& q, uint32_t a, uint32_t b) {
  using J = typename Gr::jac;
  const uint64_t da = win4_recode32(a), db = win4_recode32(b);
  J T[8];
  T[0] = Gr::from_aff(q);
  T[1] = Gr::dbl_body(T[0]);
#pragma unroll 1
  for (int m = 2; m < 8; ++m) T[m] = Gr::add_aff_body(T[m - 1], q);
  J acc = Gr::cmov(Gr::inf(), T[0], (da >> 40) & 1u);
  acc = Gr::cmov(acc, Gr::add_body(acc, Gr::endo(T[0])), (db >> 40) & 1u);
#pragma unroll 1
  for (int j = 7; j >= 0; --j) {
#pragma unroll 1
    for (int s = 0; s < 4; ++s) acc = Gr::dbl_body(acc);
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      const uint32_t dg = (uint32_t)(((s ? db : da) >> (5 * j)) & 31u), mag = dg & 15u;
      J t = T[(mag - 1u) & 7u];
      if (s) t = Gr::endo(t);
      t = Gr::cneg(t, (dg & 16u) != 0);
      acc = Gr::cmov(acc, Gr::add_body(acc, t), mag != 0);
    }
  }
  return acc;
}

}  // namespace dgpu
