// Optimal-ate pairing pieces for BLS12-381 on gfx950: projective Miller-loop
// steps with line evaluation, the shared-squaring 2-pair Miller loop and the
// final exponentiation.  Formulas (and their derivation) are mirrored in
// oracle/pairing_formulas.py and checked there against the generic pairing.
//
// Reference path: chain/verify.go:44 -> kyber bls.Verify ->
// Suite.ValidatePairing(pk, H(m), g1, sig) -> kilic Engine AddPair /
// AddPairInv / Check (R): e(pk, H(m)) * e(-g1, sig) == 1.
#pragma once
#include "curve.cuh"

namespace dgpu {

struct g2p {  // homogeneous projective (x = X/Z, y = Y/Z)
  fp2 x, y, z;
};
struct line3 {  // l = c0 + c2 w^2 + c3 w^3
  fp2 c0, c2, c3;
};

// P given as (-xP, yP) in Montgomery form
DG_NOINL line3 miller_dbl_step(g2p& T, const fp& neg_xp, const fp& yp) {
  fp2 t0 = fp2_sqr(T.y);
  fp2 t1 = fp2_sqr(T.z);
  fp2 t2 = fp2_mul(t1, C_B2_3);                  // 3 b' Z^2
  fp2 t3 = fp2_add(fp2_dbl(t2), t2);             // 9 b' Z^2
  fp2 xy = fp2_half(fp2_mul(T.x, T.y));          // XY/2
  fp2 yz2 = fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), fp2_add(t0, t1));  // 2YZ
  fp2 x2 = fp2_sqr(T.x);
  line3 l;
  l.c0 = fp2_sub(t0, t2);
  l.c2 = fp2_mul_fp(fp2_add(fp2_dbl(x2), x2), neg_xp);
  l.c3 = fp2_mul_fp(yz2, yp);
  fp2 t2sq = fp2_sqr(t2);
  T.x = fp2_mul(xy, fp2_sub(t0, t3));
  T.y = fp2_sub(fp2_sqr(fp2_half(fp2_add(t0, t3))), fp2_add(fp2_dbl(t2sq), t2sq));
  T.z = fp2_mul(t0, yz2);
  return l;
}

DG_NOINL line3 miller_add_step(g2p& T, const g2a& Q, const fp& neg_xp, const fp& yp) {
  fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  fp2 lam = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  fp2 C = fp2_sqr(theta);
  fp2 D = fp2_sqr(lam);
  fp2 E = fp2_mul(lam, D);
  fp2 F = fp2_mul(T.z, C);
  fp2 G = fp2_mul(T.x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  line3 l;
  l.c0 = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y));
  l.c2 = fp2_mul_fp(theta, neg_xp);
  l.c3 = fp2_mul_fp(lam, yp);
  fp2 ye = fp2_mul(T.y, E);
  T.x = fp2_mul(lam, H);
  T.y = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), ye);
  T.z = fp2_mul(T.z, E);
  return l;
}

// f_{|x|} for two pairs with one shared Fp12 squaring per bit, conjugated (x < 0).
DG_NOINL fp12 miller_loop_2(const g2a& Q1, const fp& nx1, const fp& y1, const g2a& Q2, const fp& nx2, const fp& y2) {
  g2p T1{Q1.x, Q1.y, fp2_one()};
  g2p T2{Q2.x, Q2.y, fp2_one()};
  fp12 f = fp12_one();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    line3 l = miller_dbl_step(T1, nx1, y1);
    f = fp12_mul_line(f, l.c0, l.c2, l.c3);
    l = miller_dbl_step(T2, nx2, y2);
    f = fp12_mul_line(f, l.c0, l.c2, l.c3);
    if ((BLS_X_ABS >> i) & 1ull) {
      l = miller_add_step(T1, Q1, nx1, y1);
      f = fp12_mul_line(f, l.c0, l.c2, l.c3);
      l = miller_add_step(T2, Q2, nx2, y2);
      f = fp12_mul_line(f, l.c0, l.c2, l.c3);
    }
  }
  return fp12_conj(f);
}

// a^|x| (square-and-multiply over the public constant), a in the cyclotomic subgroup
DG_NOINL fp12 fp12_pow_absx(const fp12& a) {
  fp12 r = a;
  for (int i = 62; i >= 0; --i) {
    r = fp12_cyclo_sqr(r);
    if ((BLS_X_ABS >> i) & 1ull) r = fp12_mul(r, a);
  }
  return r;
}

// a^x, x < 0, for a in the cyclotomic subgroup (inverse == conjugate)
DG_FN fp12 fp12_exp_x(const fp12& a) { return fp12_conj(fp12_pow_absx(a)); }

// f^(3 (p^12 - 1) / r): easy part, then the hard-part chain
// 3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3.
DG_NOINL fp12 final_exponentiation(const fp12& f) {
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));  // f^(p^6 - 1)
  t = fp12_mul(fp12_frob2(t), t);                // ^(p^2 + 1)
  fp12 t0 = fp12_mul(fp12_exp_x(t), fp12_conj(t));
  fp12 t1 = fp12_mul(fp12_exp_x(t0), fp12_conj(t0));
  fp12 t2 = fp12_mul(fp12_exp_x(t1), fp12_frob1(t1));
  fp12 t3 = fp12_mul(fp12_mul(fp12_exp_x(fp12_exp_x(t2)), fp12_frob2(t2)), fp12_conj(t2));
  return fp12_mul(t3, fp12_mul(fp12_sqr(t), t));
}

}  // namespace dgpu
