// G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+u) over Fp2)
// group law in Jacobian coordinates (x = X/Z^2, y = Y/Z^3, Z = 0 is the point
// at infinity), the psi endomorphism, the psi-based G2 membership test, and
// ZCash compressed encodings (the format kyber-bls12381 / kilic read and
// write: chain/verify.go:44 -> key.Scheme.VerifyRecovered (R)).
#pragma once
#include "tower.cuh"

namespace dgpu {

struct g2a {  // affine
  fp2 x, y;
};
struct g2j {  // Jacobian
  fp2 x, y, z;
};
struct g1a {
  fp x, y;
};
struct g1j {
  fp x, y, z;
};

// ================================================================ G2
DG_FN g2j g2_from_affine(const g2a& a) { return g2j{a.x, a.y, fp2_one()}; }
DG_FN g2j g2_infinity() { return g2j{fp2_one(), fp2_one(), fp2_zero()}; }
DG_FN bool g2_is_inf(const g2j& a) { return fp2_is_zero(a.z); }
DG_FN g2j g2_neg(const g2j& a) { return g2j{a.x, fp2_neg(a.y), a.z}; }

DG_FN g2j g2_cmov(const g2j& a, const g2j& b, bool take_b) {
  return g2j{fp2_cmov(a.x, b.x, take_b), fp2_cmov(a.y, b.y, take_b), fp2_cmov(a.z, b.z, take_b)};
}

// dbl-2009-l (a = 0): 2M + 5S.  Infinity stays infinity (Z3 = 2YZ).
// (*_body: the same code force-inlined, for loops that keep the point in
// registers instead of passing it through the stack to an out-of-line call)
// Lazy linear steps (bounds in units of p; CI = normalized, < 2.01p):
//   X + B carried (< 4.02p) into fp2_sqr; D/2 = (X+B)^2 - A - C reduced;
//   E = 3A carried (< 6.03p); X3 = F - 4(D/2) (4(D/2) carried, < 8.04p);
//   D - X3 = 2(D/2) + 8p - X3 carried (< 12.02p) into fp2_mul with E
//   (sum products 12.06p x 24.04p); 8C carried (< 16.08p);
//   Z3 = (2Y) Z with 2Y lazy (limbs < 2^29, fp2_mul's sum < 2^30).
// Evaluation order keeps at most five Fp2 values live across the
// out-of-line Fp calls (Z3 first frees Z, B frees Y, X + B frees X, ...).
DG_FN g2j g2_dbl_body(const g2j& p) {
  g2j r;
  r.z = fp2_mul(fp2_add_lz(p.y, p.y), p.z);
  const fp2 B = fp2_sqr(p.y);
  const fp2 A = fp2_sqr(p.x);
  const fp2 XB = fp2_carry(fp2_add_lz(p.x, B));
  const fp2 C = fp2_sqr(B);
  const fp2 Dh = fp2_sub32(fp2_sqr(XB), fp2_add_lz(A, C));
  const fp2 E = fp2_carry(fp2_add_lz(fp2_add_lz(A, A), A));
  r.x = fp2_sub32(fp2_sqr(E), fp2_carry(fp2_mulk_lz(Dh, 4)));
  const fp2 D2 = fp2_add_lz(Dh, Dh);
  const fp2 DX = fp2_carry(fp2{fp_sub_lz(D2.c0, r.x.c0), fp_sub_lz(D2.c1, r.x.c1)});
  r.y = fp2_sub32(fp2_mul(E, DX), fp2_carry(fp2_mulk_lz(C, 8)));
  return r;
}

DG_NOINL g2j g2_dbl(const g2j& p) { return g2_dbl_body(p); }

// fp2_mul with its outputs normalized but not reduced -- c0 = t0 + 8p - t1,
// c1 = t2 + 32p - (t0 + t1) -- for a consumer that reduces anyway (or, as Z
// of the ladder below, feeds another fp2_mul).  With t0, t1 < 1.05p and
// t2 < 1.2p (operand sums < 4.02p x 4.02p, or the bounds stated by the
// caller): c0 < 9.1p, c1 < 33.3p, limbs < 2^28 (top limb < 2^23).
DG_FN fp2 fp2_mul_nr(const fp2& a, const fp2& b) {
  const fp t0 = fp_mul(a.c0, b.c0);
  const fp t1 = fp_mul(a.c1, b.c1);
  const fp t2 = fp_mul(fp_add_lz(a.c0, a.c1), fp_add_lz(b.c0, b.c1));
  return fp2{fp_norm(fp_sub_lz(t0, t1)), fp_norm(fp_sub2_lz(t2, fp_add_lz(t0, t1)))};
}

// g2_dbl_body with four reductions fewer, for the cofactor ladder: Y3's
// product is left unreduced into fp2_sub32 (65.3p + 32p bound: reduced once),
// and Z is carried unreduced from doubling to doubling -- Z3 = (2Y) Z with
// Z.c0 < 9.1p, Z.c1 < 33.3p: operand sums 8.04p x 42.4p = 341 p^2 (fp_mul
// bound ~2600 p^2), t2 < 1.13p, so Z3 keeps the same bounds.  Z must be
// reduced (g2_z_reduce) before an addition or any other consumer.
DG_FN g2j g2_dbl_lz(const g2j& p) {
  g2j r;
  r.z = fp2_mul_nr(fp2_add_lz(p.y, p.y), p.z);
  const fp2 B = fp2_sqr(p.y);
  const fp2 A = fp2_sqr(p.x);
  const fp2 XB = fp2_carry(fp2_add_lz(p.x, B));
  const fp2 C = fp2_sqr(B);
  const fp2 Dh = fp2_sub32(fp2_sqr(XB), fp2_add_lz(A, C));
  const fp2 E = fp2_carry(fp2_add_lz(fp2_add_lz(A, A), A));
  r.x = fp2_sub32(fp2_sqr(E), fp2_carry(fp2_mulk_lz(Dh, 4)));
  const fp2 D2 = fp2_add_lz(Dh, Dh);
  const fp2 DX = fp2_carry(fp2{fp_sub_lz(D2.c0, r.x.c0), fp_sub_lz(D2.c1, r.x.c1)});
  r.y = fp2_sub32(fp2_mul_nr(E, DX), fp2_carry(fp2_mulk_lz(C, 8)));
  return r;
}
DG_FN g2j g2_z_reduce(g2j r) {
  r.z = fp2{fp_reduce(r.z.c0), fp_reduce(r.z.c1)};
  return r;
}

// add-2007-bl with the exceptional cases resolved (P == Q -> dbl,
// P == -Q -> infinity, either operand infinity -> the other).
// Lazy linear steps: rr = 2(s2 - s1) and 2h carried (< 4.02p); X3 = rr^2 -
// (J + 2V), the sum carried (< 6.03p); V - X3 = V + 8p - X3 carried (< 10.02p)
// into fp2_mul with rr (sum products 8.04p x 20.04p); 2 s1 J = (2 s1) J with
// 2 s1 lazy; Z1 + Z2 carried into fp2_sqr, minus the lazy z1z1 + z2z2.
DG_FN g2j g2_add_body(const g2j& p, const g2j& q) {
  const fp2 z1z1 = fp2_sqr(p.z);
  const fp2 z2z2 = fp2_sqr(q.z);
  const fp2 u1 = fp2_mul(p.x, z2z2);
  const fp2 u2 = fp2_mul(q.x, z1z1);
  const fp2 s1 = fp2_mul(fp2_mul(p.y, q.z), z2z2);
  const fp2 s2 = fp2_mul(fp2_mul(q.y, p.z), z1z1);
  const fp2 h = fp2_sub(u2, u1);
  const fp2 rh = fp2_sub(s2, s1);
  const bool p_inf = g2_is_inf(p), q_inf = g2_is_inf(q);
  const bool h0 = fp2_is_zero(h), r0 = fp2_is_zero(rh);
  const fp2 rr = fp2_carry(fp2_add_lz(rh, rh));
  const fp2 i = fp2_sqr(fp2_carry(fp2_add_lz(h, h)));
  const fp2 j = fp2_mul(h, i);
  const fp2 v = fp2_mul(u1, i);
  g2j r;
  r.x = fp2_sub32(fp2_sqr(rr), fp2_carry(fp2_add_lz(fp2_add_lz(j, v), v)));
  const fp2 VX = fp2_carry(fp2{fp_sub_lz(v.c0, r.x.c0), fp_sub_lz(v.c1, r.x.c1)});
  r.y = fp2_sub(fp2_mul(rr, VX), fp2_mul(fp2_add_lz(s1, s1), j));
  r.z = fp2_mul(fp2_sub32(fp2_sqr(fp2_carry(fp2_add_lz(p.z, q.z))), fp2_add_lz(z1z1, z2z2)), h);
  if (h0 && !p_inf && !q_inf) r = r0 ? g2_dbl(p) : g2_infinity();
  if (p_inf) r = q;
  if (q_inf) r = p;
  return r;
}

DG_NOINL g2j g2_add(const g2j& p, const g2j& q) { return g2_add_body(p, q); }

// Mixed addition p + q with q affine (madd-2007-bl: 7M + 4S), exceptional
// cases resolved (p == q -> dbl, p == -q -> infinity, p infinity -> q).
DG_FN g2j g2_add_affine_body(const g2j& p, const g2a& q) {
  // lazy linear steps as g2_add_body; I = 4 HH carried (< 8.04p)
  const fp2 z1z1 = fp2_sqr(p.z);
  const fp2 u2 = fp2_mul(q.x, z1z1);
  const fp2 s2 = fp2_mul(fp2_mul(q.y, p.z), z1z1);
  const fp2 h = fp2_sub(u2, p.x);
  const fp2 rh = fp2_sub(s2, p.y);
  const bool p_inf = g2_is_inf(p);
  const bool h0 = fp2_is_zero(h), r0 = fp2_is_zero(rh);
  const fp2 rr = fp2_carry(fp2_add_lz(rh, rh));
  const fp2 hh = fp2_sqr(h);
  const fp2 i = fp2_carry(fp2_mulk_lz(hh, 4));
  const fp2 j = fp2_mul(h, i);
  const fp2 v = fp2_mul(p.x, i);
  g2j r;
  r.x = fp2_sub32(fp2_sqr(rr), fp2_carry(fp2_add_lz(fp2_add_lz(j, v), v)));
  const fp2 VX = fp2_carry(fp2{fp_sub_lz(v.c0, r.x.c0), fp_sub_lz(v.c1, r.x.c1)});
  r.y = fp2_sub(fp2_mul(rr, VX), fp2_mul(fp2_add_lz(p.y, p.y), j));
  r.z = fp2_sub32(fp2_sqr(fp2_carry(fp2_add_lz(p.z, h))), fp2_add_lz(z1z1, hh));
  if (h0 && !p_inf) r = r0 ? g2_dbl(g2_from_affine(q)) : g2_infinity();
  if (p_inf) r = g2_from_affine(q);
  return r;
}

DG_NOINL g2j g2_add_affine(const g2j& p, const g2a& q) { return g2_add_affine_body(p, q); }

// [|x|] p with the group law inlined (register-resident loop state)
DG_FN g2j g2_mul_absx_inl(const g2j& p) {
  g2j r = p;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = g2_dbl_body(r);
    if ((BLS_X_ABS >> i) & 1ull) r = g2_add_body(r, p);
  }
  return r;
}

// [|x|] p for the BLS parameter |x| = 0xd201000000010000 (MSB-first double-and-add)
DG_NOINL g2j g2_mul_absx(const g2j& p) {
  g2j r = p;
  for (int i = 62; i >= 0; --i) {
    r = g2_dbl(r);
    if ((BLS_X_ABS >> i) & 1ull) r = g2_add(r, p);
  }
  return r;
}

// generic [k] p, k given as little-endian 32-bit words (MSB-first double-and-add)
DG_NOINL g2j g2_mul_words(const g2j& p, const uint32_t* k, int nwords) {
  g2j r = g2_infinity();
  for (int i = nwords * 32 - 1; i >= 0; --i) {
    r = g2_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = g2_add(r, p);
  }
  return r;
}

// Non-adjacent form of a 64-bit scalar: k = (3k >> 1) - (k >> 1), and digit j
// of NAF(k) is bit j of (3k >> 1) minus bit j of (k >> 1).  pos / neg hold the
// +1 / -1 digits at positions 0..63, top the digit at position 64 (0 or +1).
DG_FN void naf64(uint64_t k, uint64_t& pos, uint64_t& neg, uint32_t& top) {
  const uint64_t lo = k + (k << 1);  // 3k = hi:lo
  const uint64_t hi = (k >> 63) + (lo < k ? 1ull : 0ull);
  const uint64_t h = (lo >> 1) | (hi << 63);  // (3k >> 1) mod 2^64
  const uint64_t kk = k >> 1;
  const uint64_t c = h ^ kk;
  pos = h & c;
  neg = kk & c;
  top = (uint32_t)(hi >> 1);
}

// [k] q for an affine q and a 64-bit k: MSB-first signed double-and-add over
// NAF(k) (about 21 mixed additions instead of 32), group law inlined so the
// accumulator stays in registers (RLC leaves).
DG_FN g2j g2_mul64_naf_affine(const g2a& q, uint64_t k) {
  uint64_t pos, neg;
  uint32_t top;
  naf64(k, pos, neg, top);
  const uint64_t any = pos | neg;
  g2j r = top ? g2_from_affine(q) : g2_infinity();
#pragma unroll 1
  for (int i = 63; i >= 0; --i) {
    r = g2_dbl_body(r);
    if ((any >> i) & 1ull) {
      const g2a t{q.x, fp2_cmov(q.y, fp2_neg(q.y), (neg >> i) & 1ull)};
      r = g2_add_affine_body(r, t);
    }
  }
  return r;
}

// NAF of a 32-bit scalar (digits 0..32) as +1 / -1 masks (see naf64).
DG_FN void naf32(uint32_t k, uint64_t& pos, uint64_t& neg) {
  const uint64_t h = (3ull * k) >> 1, kk = (uint64_t)(k >> 1), c = h ^ kk;
  pos = h & c;
  neg = kk & c;
}

// psi of an affine point: (conj(x) cx, conj(y) cy)
DG_FN g2a g2a_psi(const g2a& q) {
  return g2a{fp2_mul(fp2_conj(q.x), C_PSI_CX), fp2_mul(fp2_conj(q.y), C_PSI_CY)};
}

// [a] q + [b] pq for affine q, pq and 32-bit a, b: one shared ladder of at
// most 33 doublings over NAF(a) and NAF(b) (Straus), mixed additions, group
// law inlined.  With pq = psi(q) and q in G2 this is [a + b x] q (psi acts as
// [x] on G2); the RLC leaves draw their coefficients as r = a + b x.
// PSI_ON_DEMAND: pq is ignored and psi(q) recomputed at each of its digits
// (2 Fp2 products each) instead of being held live across the ladder.
template <bool PSI_ON_DEMAND = false>
DG_FN g2j g2_mul2_naf32_affine(const g2a& q, const g2a& pq, uint32_t a, uint32_t b) {
  uint64_t ap, an, bp, bn;
  naf32(a, ap, an);
  naf32(b, bp, bn);
  const uint64_t am = ap | an, bm = bp | bn;
  g2j r = g2_infinity();
#pragma unroll 1
  for (int i = 63 - __builtin_clzll(am | bm | 1ull); i >= 0; --i) {
    r = g2_dbl_body(r);
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      if ((((s ? bm : am) >> i) & 1ull) == 0) continue;
      g2a t;
      if (PSI_ON_DEMAND) {
        t = s ? g2a_psi(q) : q;
      } else {
        t = g2a{fp2_cmov(q.x, pq.x, s != 0), fp2_cmov(q.y, pq.y, s != 0)};
      }
      const bool negd = (((s ? bn : an) >> i) & 1ull) != 0;
      t.y = fp2_cmov(t.y, fp2_neg(t.y), negd);
      r = g2_add_affine_body(r, t);
    }
  }
  return r;
}

// [x] p with x < 0
DG_FN g2j g2_mul_x(const g2j& p) { return g2_neg(g2_mul_absx(p)); }

// psi(x, y) = (conj(x) cx, conj(y) cy); on Jacobian coordinates Z -> conj(Z)
DG_NOINL g2j g2_psi(const g2j& p) {
  return g2j{fp2_mul(fp2_conj(p.x), C_PSI_CX), fp2_mul(fp2_conj(p.y), C_PSI_CY), fp2_conj(p.z)};
}
DG_NOINL g2j g2_psi2(const g2j& p) {
  return g2j{fp2_mul_fp(p.x, fp2(C_PSI2_CX).c0), fp2_mul_fp(p.y, fp2(C_PSI2_CY).c0), p.z};
}

// Signed radix-16 digits of a 32-bit k: k = sum_j d_j 16^j with d_j in
// [-8, 7] for j < 8 and d_8 in {0, 1}; digit j packed at bits 5j..5j+4 as
// |d_j| (4 bits) and its sign (bit 4).
DG_FN uint64_t win4_recode32(uint32_t k) {
  uint64_t out = 0;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t w = ((k >> (4 * j)) & 15u) + c;
    c = w >= 8u ? 1u : 0u;
    const uint32_t mag = c ? 16u - w : w;
    out |= (uint64_t)(mag | (c && mag ? 16u : 0u)) << (5 * j);
  }
  return out | ((uint64_t)c << 40);
}

// [a] q + [b] psi(q) for an affine q (not the identity) and 32-bit a, b with
// the same operation sequence in every lane.  In k_rlc_leaves the lanes of a
// wave hold unrelated coefficients, so a digit-driven ladder (the NAF form
// above) runs the union of its lanes' additions -- about two per bit.  Here:
// signed radix-16 windows of both scalars over the table T[m] = [m + 1] q
// (Jacobian, private memory, built with 1 doubling + 6 mixed additions); 8
// windows of 4 doublings + 2 additions (psi applied to b's entry), a zero
// digit's addition computed and discarded: 33 doublings, 17 additions.
DG_FN g2j g2_mul2_win4_affine(const g2a& q, uint32_t a, uint32_t b) {
  const uint64_t da = win4_recode32(a), db = win4_recode32(b);
  g2j T[8];
  T[0] = g2_from_affine(q);
  T[1] = g2_dbl_body(T[0]);
#pragma unroll 1
  for (int m = 2; m < 8; ++m) T[m] = g2_add_affine_body(T[m - 1], q);
  // top digits (0 or 1): acc = [d_8(a)] q + [d_8(b)] psi(q)
  g2j acc = g2_cmov(g2_infinity(), T[0], (da >> 40) & 1u);
  acc = g2_cmov(acc, g2_add_body(acc, g2_psi(T[0])), (db >> 40) & 1u);
#pragma unroll 1
  for (int j = 7; j >= 0; --j) {
#pragma unroll 1
    for (int s = 0; s < 4; ++s) acc = g2_dbl_body(acc);
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      const uint32_t dg = (uint32_t)(((s ? db : da) >> (5 * j)) & 31u), mag = dg & 15u;
      g2j t = T[(mag - 1u) & 7u];
      if (s) t = g2_psi(t);
      t.y = fp2_cmov(t.y, fp2_neg(t.y), (dg & 16u) != 0);
      acc = g2_cmov(acc, g2_add_body(acc, t), mag != 0);
    }
  }
  return acc;
}

DG_NOINL bool g2_eq(const g2j& p, const g2j& q) {
  bool pi = g2_is_inf(p), qi = g2_is_inf(q);
  if (pi || qi) return pi && qi;
  fp2 z1z1 = fp2_sqr(p.z), z2z2 = fp2_sqr(q.z);
  bool ex = fp2_eq(fp2_mul(p.x, z2z2), fp2_mul(q.x, z1z1));
  bool ey = fp2_eq(fp2_mul(fp2_mul(p.y, q.z), z2z2), fp2_mul(fp2_mul(q.y, p.z), z1z1));
  return ex && ey;
}

// G2 membership: psi(Q) == [x] Q  (Scott, "A note on group membership tests
// for G1, G2 and GT on BLS pairing-friendly curves"); same verdict as the
// reference's [r] Q == O test (R), checked against it in tests.
DG_FN bool g2_in_subgroup(const g2j& p) { return g2_eq(g2_psi(p), g2_neg(g2_mul_absx_inl(p))); }

DG_NOINL g2a g2_to_affine(const g2j& p) {
  fp2 zi = fp2_inv(p.z);
  fp2 zi2 = fp2_sqr(zi);
  return g2a{fp2_mul(p.x, zi2), fp2_mul(p.y, fp2_mul(zi2, zi))};
}

DG_FN bool g2_on_curve_affine(const g2a& a) {
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(a.x), a.x), C_B2);
  return fp2_eq(fp2_sqr(a.y), rhs);
}

// add-2007-bl for operands that are neither equal, opposite nor the identity:
// g2_add_body without its exceptional branches (whose out-of-line g2_dbl call
// is a call site in the caller's loop); `exc` is set when one of those cases
// arises, and the caller redoes the whole computation on the generic path.
// The second operand comes through `q` (q.x(), q.y(), q.z()), each coordinate
// fetched where it is used -- from HBM in the cofactor ladders -- and the
// products ordered so p's coordinates die early: at most six Fp2 values live.
// Z3 = 2 Z1 Z2 H (the same value as ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H), 2 Z1Z2
// lazy into fp2_mul (limbs < 2^29).
template <class Q>
DG_FN g2j g2_add_nx_q(const g2j& p, const Q& q, bool& exc) {
  fp2 u1, s1, z1z2;
  {
    const fp2 qz = q.z();
    exc = exc || fp2_is_zero(qz);
    const fp2 z2z2 = fp2_sqr(qz);
    u1 = fp2_mul(p.x, z2z2);
    s1 = fp2_mul(fp2_mul(p.y, qz), z2z2);
    z1z2 = fp2_mul(p.z, qz);
  }
  fp2 h, rh;
  {
    const fp2 z1z1 = fp2_sqr(p.z);
    h = fp2_sub(fp2_mul(q.x(), z1z1), u1);
    rh = fp2_sub(fp2_mul(fp2_mul(q.y(), p.z), z1z1), s1);
  }
  exc = exc || g2_is_inf(p) || fp2_is_zero(h);
  g2j r;
  r.z = fp2_mul(fp2_add_lz(z1z2, z1z2), h);
  const fp2 rr = fp2_carry(fp2_add_lz(rh, rh));
  const fp2 i = fp2_sqr(fp2_carry(fp2_add_lz(h, h)));
  const fp2 j = fp2_mul(h, i);
  const fp2 v = fp2_mul(u1, i);
  r.x = fp2_sub32(fp2_sqr(rr), fp2_carry(fp2_add_lz(fp2_add_lz(j, v), v)));
  const fp2 VX = fp2_carry(fp2{fp_sub_lz(v.c0, r.x.c0), fp_sub_lz(v.c1, r.x.c1)});
  r.y = fp2_sub(fp2_mul(rr, VX), fp2_mul(fp2_add_lz(s1, s1), j));
  return r;
}
struct g2j_q {  // an in-register second operand
  const g2j& p;
  DG_FN fp2 x() const { return p.x; }
  DG_FN fp2 y() const { return p.y; }
  DG_FN fp2 z() const { return p.z; }
};
DG_FN g2j g2_add_nx(const g2j& p, const g2j& q, bool& exc) { return g2_add_nx_q(p, g2j_q{q}, exc); }
DG_FN g2j g2_psi_body(const g2j& p) {
  return g2j{fp2_mul(fp2_conj(p.x), C_PSI_CX), fp2_mul(fp2_conj(p.y), C_PSI_CY), fp2_conj(p.z)};
}
DG_FN g2j g2_psi2_body(const g2j& p) {
  return g2j{fp2_mul_fp(p.x, fp2(C_PSI2_CX).c0), fp2_mul_fp(p.y, fp2(C_PSI2_CY).c0), p.z};
}

#ifdef DG_LADDER_DBL_PLAIN  // A/B: every doubling fully reduced (g2_dbl_body)
#define G2_LADDER_DBL g2_dbl_body
#define G2_LADDER_ZRED(r) (r)
#else
#define G2_LADDER_DBL g2_dbl_lz
#define G2_LADDER_ZRED(r) g2_z_reduce(r)
#endif
// [|x|] of the point in stash slot k, |x| = 0xd201000000010000 (bits 63, 62,
// 60, 57, 48, 16): runs of 1, 2, 3, 9 and 32 doublings, each closed by an
// addition of the point reloaded from the slot, then 16 doublings -- only the
// accumulator lives across the loops.
template <class Stash>
DG_FN g2j g2_mul_absx_stash(Stash& st, int k, bool& exc) {
  g2j r = st.get(k);
#pragma unroll 1
  for (int a = 0; a < 5; ++a) {
    const int nd = a == 0 ? 1 : a == 1 ? 2 : a == 2 ? 3 : a == 3 ? 9 : 32;
#pragma unroll 1
    for (int d = 0; d < nd; ++d) r = G2_LADDER_DBL(r);
    r = g2_add_nx_q(G2_LADDER_ZRED(r), st.at(k), exc);
  }
#pragma unroll 1
  for (int d = 0; d < 16; ++d) r = G2_LADDER_DBL(r);
  return G2_LADDER_ZRED(r);
}

// madd-2007-bl (g2_add_affine_body) for operands that are neither equal,
// opposite nor the identity, the affine operand fetched through q (q.x(),
// q.y()) where used; `exc` as g2_add_nx_q.
template <class Q>
DG_FN g2j g2_madd_nx_q(const g2j& p, const Q& q, bool& exc) {
  const fp2 z1z1 = fp2_sqr(p.z);
  const fp2 h = fp2_sub(fp2_mul(q.x(), z1z1), p.x);
  const fp2 rh = fp2_sub(fp2_mul(fp2_mul(q.y(), p.z), z1z1), p.y);
  exc = exc || g2_is_inf(p) || fp2_is_zero(h);
  const fp2 rr = fp2_carry(fp2_add_lz(rh, rh));
  const fp2 hh = fp2_sqr(h);
  const fp2 i = fp2_carry(fp2_mulk_lz(hh, 4));
  const fp2 j = fp2_mul(h, i);
  const fp2 v = fp2_mul(p.x, i);
  g2j r;
  r.x = fp2_sub32(fp2_sqr(rr), fp2_carry(fp2_add_lz(fp2_add_lz(j, v), v)));
  const fp2 VX = fp2_carry(fp2{fp_sub_lz(v.c0, r.x.c0), fp_sub_lz(v.c1, r.x.c1)});
  r.y = fp2_sub(fp2_mul(rr, VX), fp2_mul(fp2_add_lz(p.y, p.y), j));
  r.z = fp2_sub32(fp2_sqr(fp2_carry(fp2_add_lz(p.z, h))), fp2_add_lz(z1z1, hh));
  return r;
}

// G2 membership psi(P) == -[|x|]P (g2_in_subgroup) for an affine P (not the
// identity) on the cofactor ladder's structure: runs of lazy doublings, each
// closed by a fast mixed addition of P fetched through q -- only the
// accumulator lives across the loops.  exc: an exceptional addition (P of
// small order); the caller then decides with g2_in_subgroup.
template <class Q>
DG_FN bool g2_in_subgroup_ladder(const g2a& p, const Q& q, bool& exc) {
  g2j r = g2_from_affine(p);
#pragma unroll 1
  for (int a = 0; a < 5; ++a) {
    const int nd = a == 0 ? 1 : a == 1 ? 2 : a == 2 ? 3 : a == 3 ? 9 : 32;
#pragma unroll 1
    for (int d = 0; d < nd; ++d) r = G2_LADDER_DBL(r);
    r = g2_madd_nx_q(G2_LADDER_ZRED(r), q, exc);
  }
#pragma unroll 1
  for (int d = 0; d < 16; ++d) r = G2_LADDER_DBL(r);
  return g2_eq(g2_psi(g2_from_affine(q.get())), g2_neg(G2_LADDER_ZRED(r)));
}

// h_eff (Q0 + Q1) in the order of g2_clear_cofactor (RFC 9380 G.3) with the
// cold operands parked in three point slots of `st` (k_h2c_finish: the
// round's own SoA slots in HBM) so the two [|x|] ladders hold one point each:
//   slot 0: P = Q0 + Q1 (generic addition);  slot 1: R = psi^2(2P) - psi(P) - P,
//   then R - [x]P;  slot 2: U = [x]P + psi(P);  result R + [x]U.
// exc: an exceptional addition arose on the fast path (the caller recomputes
// with g2_clear_cofactor).
template <class Stash>
DG_FN g2j g2_clear_cofactor_stash(const g2j& q0, const g2j& q1, Stash& st, bool& exc) {
  {
    const g2j P = g2_add_body(q0, q1);
    st.put(0, P);
    const g2j t = g2_add_nx(g2_psi2_body(g2_dbl_body(P)), g2_neg(g2_psi_body(P)), exc);
    st.put(1, g2_add_nx(t, g2_neg(P), exc));
  }
  const g2j nA = g2_mul_absx_stash(st, 0, exc);  // -[x]P
  st.put(2, g2_add_nx(g2_neg(nA), g2_psi_body(st.get(0)), exc));
  st.put(1, g2_add_nx(st.get(1), nA, exc));
  const g2j nB = g2_mul_absx_stash(st, 2, exc);  // -[x]U
  return g2_add_nx(st.get(1), g2_neg(nB), exc);
}

// Clear cofactor with the whole computation inlined (k_h2c_finish).
DG_FN g2j g2_clear_cofactor_inl(const g2j& p) {
  g2j t1 = g2_neg(g2_mul_absx_inl(p));
  g2j t2 = g2_psi(p);
  g2j t3 = g2_psi2(g2_dbl_body(p));
  t3 = g2_add_body(t3, g2_neg(t2));
  t2 = g2_add_body(t1, t2);
  t2 = g2_neg(g2_mul_absx_inl(t2));
  t3 = g2_add_body(t3, t2);
  t3 = g2_add_body(t3, g2_neg(t1));
  return g2_add_body(t3, g2_neg(p));
}

// Clear cofactor: h_eff * P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)
// (RFC 9380 appendix G.3 sequence).
DG_NOINL g2j g2_clear_cofactor_generic(const g2j& p) {
  g2j t1 = g2_mul_x(p);
  g2j t2 = g2_psi(p);
  g2j t3 = g2_psi2(g2_dbl(p));
  t3 = g2_add(t3, g2_neg(t2));
  t2 = g2_add(t1, t2);
  t2 = g2_mul_x(t2);
  t3 = g2_add(t3, t2);
  t3 = g2_add(t3, g2_neg(t1));
  return g2_add(t3, g2_neg(p));
}

// [|x|] p in registers on the ladder's structure (lazy doublings, fast
// additions; exc as g2_add_nx).
DG_FN g2j g2_mul_absx_fast(const g2j& p, bool& exc) {
  g2j r = p;
#pragma unroll 1
  for (int a = 0; a < 5; ++a) {
    const int nd = a == 0 ? 1 : a == 1 ? 2 : a == 2 ? 3 : a == 3 ? 9 : 32;
#pragma unroll 1
    for (int d = 0; d < nd; ++d) r = G2_LADDER_DBL(r);
    r = g2_add_nx(G2_LADDER_ZRED(r), p, exc);
  }
#pragma unroll 1
  for (int d = 0; d < 16; ++d) r = G2_LADDER_DBL(r);
  return G2_LADDER_ZRED(r);
}

// h_eff P (the sequence above) for the one-off callers -- the RLC node
// checks (k_rlc_prep), the hash's exceptional redo, hash_to_g2: the ladder
// form in registers (round 6), the generic form when an addition is
// exceptional or P is the identity.
DG_NOINL g2j g2_clear_cofactor(const g2j& p) {
#ifndef DG_COFACTOR_GENERIC
  bool exc = g2_is_inf(p);
  const g2j nt1 = g2_mul_absx_fast(p, exc);  // -[x]P
  const g2j t2 = g2_psi_body(p);
  g2j t3 = g2_add_nx(g2_psi2_body(g2_dbl_body(p)), g2_neg(t2), exc);
  const g2j u = g2_add_nx(g2_neg(nt1), t2, exc);
  const g2j nt2 = g2_mul_absx_fast(u, exc);  // -[x]U
  t3 = g2_add_nx(t3, g2_neg(nt2), exc);
  t3 = g2_add_nx(t3, nt1, exc);
  t3 = g2_add_nx(t3, g2_neg(p), exc);
  if (!exc) return t3;
#endif
  return g2_clear_cofactor_generic(p);
}

// ---------------------------------------------------------------- ZCash G2 codec
enum : int {
  DEC_OK = 0,
  DEC_ERR_LENGTH = 1,
  DEC_ERR_FLAG = 2,
  DEC_ERR_INFINITY_NONCANON = 3,
  DEC_INFINITY = 4,
  DEC_ERR_X_RANGE = 5,
  DEC_ERR_NOT_ON_CURVE = 6,
  DEC_ERR_SUBGROUP = 7,
};

// Decode a 96-byte compressed G2 point (c1 || c0 big-endian, flags in byte 0).
// Returns DEC_OK (affine point in *out), DEC_INFINITY, or an error code.
DG_NOINL int g2_decompress(g2a* out, const uint8_t* in, bool check_subgroup) {
  uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return DEC_ERR_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= in[i];
    return acc ? DEC_ERR_INFINITY_NONCANON : DEC_INFINITY;
  }
  bool sign = (b0 & 0x20) != 0;
  uint8_t buf[48];
  for (int i = 0; i < 48; ++i) buf[i] = in[i];
  buf[0] &= 0x1f;
  fp x1 = fp_std_from_be48(buf);
  fp x0 = fp_std_from_be48(in + 48);
  if (!fp_std_lt_p(x0) || !fp_std_lt_p(x1)) return DEC_ERR_X_RANGE;
  fp2 x{fp_to_mont(x0), fp_to_mont(x1)};
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), C_B2);
  fp2 y;
  if (!fp2_sqrt(y, rhs)) return DEC_ERR_NOT_ON_CURVE;
  if (fp2_lexi_largest(y) != sign) y = fp2_neg(y);
  out->x = x;
  out->y = y;
  if (check_subgroup && !g2_in_subgroup(g2_from_affine(*out))) return DEC_ERR_SUBGROUP;
  return DEC_OK;
}

DG_NOINL void g2_compress(uint8_t* out, const g2a& a, bool infinity) {
  if (infinity) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out[i] = 0;
    return;
  }
  fp x0, x1;
  fp2_from_mont(x0, x1, a.x);
  fp_std_to_be48(x1, out);
  fp_std_to_be48(x0, out + 48);
  out[0] |= 0x80;
  if (fp2_lexi_largest(a.y)) out[0] |= 0x20;
}

// ================================================================ G1
DG_FN g1j g1_infinity() { return g1j{fp_one(), fp_one(), fp_zero()}; }
DG_FN bool g1_is_inf(const g1j& a) { return fp_is_zero(a.z); }
DG_FN g1j g1_neg(const g1j& a) { return g1j{a.x, fp_neg(a.y), a.z}; }

// a limb-wise multiple k a (k a < 2^31 per limb), unnormalized
DG_FN fp fp_mulk_lz(const fp& a, uint32_t k) {
  fp r;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) r.l[i] = k * a.l[i];
  return r;
}

#ifndef DG_G1_DBL_PLAIN
// dbl-2009-l (a = 0) with g2_dbl_body's lazy linear steps, in Fp (round 6;
// 7 products and 3 reductions where the form below, every step reduced, makes
// 14).  CI in, CI out; bounds in units of p: 2Y lazy (< 4.02p, limbs < 2^29)
// into the product with Z; X + B normalized (< 3.02p); D/2 = (X + B)^2 - A - C
// (+32p, < 33.1p) reduced; E = 3A normalized (< 3.03p); X3 = E^2 - 4 (D/2) with
// 4 (D/2) normalized (< 8.04p); D - X3 = 2 (D/2) + 8p - X3 normalized
// (< 12.1p) into the product with E (36 p^2); Y3 = E (D - X3) - 8C with 8C
// normalized (< 8.08p, limbs 8 x 2^28 < 2^31).
DG_FN g1j g1_dbl_body(const g1j& p) {
  g1j r;
  r.z = fp_mul(fp_add_lz(p.y, p.y), p.z);
  const fp B = fp_sqr(p.y);
  const fp A = fp_sqr(p.x);
  const fp XB = fp_norm(fp_add_lz(p.x, B));
  const fp C = fp_sqr(B);
  const fp Dh = fp_reduce(fp_norm(fp_sub2_lz(fp_sqr(XB), fp_add_lz(A, C))));
  const fp E = fp_norm(fp_add_lz(fp_add_lz(A, A), A));
  r.x = fp_reduce(fp_norm(fp_sub2_lz(fp_sqr(E), fp_norm(fp_mulk_lz(Dh, 4)))));
  const fp DX = fp_norm(fp_sub_lz(fp_add_lz(Dh, Dh), r.x));
  r.y = fp_reduce(fp_norm(fp_sub2_lz(fp_mul(E, DX), fp_norm(fp_mulk_lz(C, 8)))));
  return r;
}
#else  // A/B: rounds 1-5, every step reduced
DG_FN g1j g1_dbl_body(const g1j& p) {
  fp A = fp_sqr(p.x);
  fp B = fp_sqr(p.y);
  fp C = fp_sqr(B);
  fp D = fp_dbl(fp_sub(fp_sqr(fp_add(p.x, B)), fp_add(A, C)));
  fp E = fp_add(fp_dbl(A), A);
  fp F = fp_sqr(E);
  g1j r;
  r.x = fp_sub(F, fp_dbl(D));
  r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), fp_dbl(fp_dbl(fp_dbl(C))));
  r.z = fp_dbl(fp_mul(p.y, p.z));
  return r;
}
#endif

DG_NOINL g1j g1_dbl(const g1j& p) { return g1_dbl_body(p); }

#ifndef DG_G1_ADD_PLAIN
// add-2007-bl with g2_add_body's lazy linear steps, in Fp (round 6: 4
// reductions where the every-step-reduced form makes 13; same bounds as the G2
// form: rr = 2(s2 - s1) and 2h normalized (< 4.02p); X3 = rr^2 - (J + 2V)
// with the sum normalized (< 6.03p); V - X3 = V + 8p - X3 normalized
// (< 10.02p) into the product with rr; 2 s1 J = (2 s1) J with 2 s1 lazy;
// Z1 + Z2 normalized into the square, minus the lazy z1z1 + z2z2).
DG_FN g1j g1_add_body(const g1j& p, const g1j& q) {
  const fp z1z1 = fp_sqr(p.z), z2z2 = fp_sqr(q.z);
  const fp u1 = fp_mul(p.x, z2z2), u2 = fp_mul(q.x, z1z1);
  const fp s1 = fp_mul(fp_mul(p.y, q.z), z2z2), s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  const fp h = fp_sub(u2, u1);
  const fp rh = fp_sub(s2, s1);
  const bool p_inf = g1_is_inf(p), q_inf = g1_is_inf(q);
  const bool h0 = fp_is_zero(h), r0 = fp_is_zero(rh);
  const fp rr = fp_norm(fp_add_lz(rh, rh));
  const fp i = fp_sqr(fp_norm(fp_add_lz(h, h)));
  const fp j = fp_mul(h, i);
  const fp v = fp_mul(u1, i);
  g1j r;
  r.x = fp_reduce(fp_norm(fp_sub2_lz(fp_sqr(rr), fp_norm(fp_add_lz(fp_add_lz(j, v), v)))));
  const fp VX = fp_norm(fp_sub_lz(v, r.x));
  r.y = fp_sub(fp_mul(rr, VX), fp_mul(fp_add_lz(s1, s1), j));
  r.z = fp_mul(fp_norm(fp_sub2_lz(fp_sqr(fp_norm(fp_add_lz(p.z, q.z))), fp_add_lz(z1z1, z2z2))), h);  // 66.6 p^2
  if (h0 && !p_inf && !q_inf) r = r0 ? g1_dbl(p) : g1_infinity();
  if (p_inf) r = q;
  if (q_inf) r = p;
  return r;
}
#else  // A/B: rounds 1-5, every step reduced
DG_FN g1j g1_add_body(const g1j& p, const g1j& q) {
  fp z1z1 = fp_sqr(p.z), z2z2 = fp_sqr(q.z);
  fp u1 = fp_mul(p.x, z2z2), u2 = fp_mul(q.x, z1z1);
  fp s1 = fp_mul(fp_mul(p.y, q.z), z2z2), s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  fp h = fp_sub(u2, u1);
  fp rr = fp_dbl(fp_sub(s2, s1));
  bool p_inf = g1_is_inf(p), q_inf = g1_is_inf(q);
  bool h0 = fp_is_zero(h), r0 = fp_is_zero(rr);
  fp i = fp_sqr(fp_dbl(h));
  fp j = fp_mul(h, i);
  fp v = fp_mul(u1, i);
  g1j r;
  r.x = fp_sub(fp_sub(fp_sqr(rr), j), fp_dbl(v));
  r.y = fp_sub(fp_mul(rr, fp_sub(v, r.x)), fp_dbl(fp_mul(s1, j)));
  r.z = fp_mul(fp_sub(fp_sqr(fp_add(p.z, q.z)), fp_add(z1z1, z2z2)), h);
  if (h0 && !p_inf && !q_inf) r = r0 ? g1_dbl(p) : g1_infinity();
  if (p_inf) r = q;
  if (q_inf) r = p;
  return r;
}
#endif

DG_NOINL g1j g1_add(const g1j& p, const g1j& q) { return g1_add_body(p, q); }

// Mixed addition p + q, q affine (madd-2007-bl, a = 0: 7M + 4S), exceptional
// cases resolved (p == q -> dbl, p == -q -> infinity, p infinity -> q).
#ifndef DG_G1_ADD_PLAIN
// madd-2007-bl with g2_add_affine_body's lazy linear steps, in Fp (4
// reductions where the every-step-reduced form makes 12; I = 4 HH normalized,
// < 4.04p).
DG_FN g1j g1_add_affine_body(const g1j& p, const g1a& q) {
  const fp z1z1 = fp_sqr(p.z);
  const fp u2 = fp_mul(q.x, z1z1);
  const fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  const fp h = fp_sub(u2, p.x);
  const fp rh = fp_sub(s2, p.y);
  const bool p_inf = g1_is_inf(p);
  const bool h0 = fp_is_zero(h), r0 = fp_is_zero(rh);
  const fp rr = fp_norm(fp_add_lz(rh, rh));
  const fp hh = fp_sqr(h);
  const fp i = fp_norm(fp_mulk_lz(hh, 4));
  const fp j = fp_mul(h, i);
  const fp v = fp_mul(p.x, i);
  g1j r;
  r.x = fp_reduce(fp_norm(fp_sub2_lz(fp_sqr(rr), fp_norm(fp_add_lz(fp_add_lz(j, v), v)))));
  const fp VX = fp_norm(fp_sub_lz(v, r.x));
  r.y = fp_sub(fp_mul(rr, VX), fp_mul(fp_add_lz(p.y, p.y), j));
  r.z = fp_reduce(fp_norm(fp_sub2_lz(fp_sqr(fp_norm(fp_add_lz(p.z, h))), fp_add_lz(z1z1, hh))));
  if (h0 && !p_inf) r = r0 ? g1_dbl(g1j{q.x, q.y, fp_one()}) : g1_infinity();
  if (p_inf) r = g1j{q.x, q.y, fp_one()};
  return r;
}
#else
DG_FN g1j g1_add_affine_body(const g1j& p, const g1a& q) {
  const fp z1z1 = fp_sqr(p.z);
  const fp u2 = fp_mul(q.x, z1z1);
  const fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  const fp h = fp_sub(u2, p.x);
  const fp rr = fp_dbl(fp_sub(s2, p.y));
  const bool p_inf = g1_is_inf(p);
  const bool h0 = fp_is_zero(h), r0 = fp_is_zero(rr);
  const fp hh = fp_sqr(h);
  const fp i = fp_dbl(fp_dbl(hh));
  const fp j = fp_mul(h, i);
  const fp v = fp_mul(p.x, i);
  g1j r;
  r.x = fp_sub(fp_sub(fp_sqr(rr), j), fp_dbl(v));
  r.y = fp_sub(fp_mul(rr, fp_sub(v, r.x)), fp_dbl(fp_mul(p.y, j)));
  r.z = fp_sub(fp_sqr(fp_add(p.z, h)), fp_add(z1z1, hh));
  if (h0 && !p_inf) r = r0 ? g1_dbl(g1j{q.x, q.y, fp_one()}) : g1_infinity();
  if (p_inf) r = g1j{q.x, q.y, fp_one()};
  return r;
}
#endif

DG_FN g1j g1_cmov(const g1j& a, const g1j& b, bool take_b) {
  return g1j{fp_cmov(a.x, b.x, take_b), fp_cmov(a.y, b.y, take_b), fp_cmov(a.z, b.z, take_b)};
}

// generic scalar multiplication by a little-endian 32-bit-word scalar
DG_NOINL g1j g1_mul_words(const g1j& p, const uint32_t* k, int nwords) {
  g1j r = g1_infinity();
  for (int i = nwords * 32 - 1; i >= 0; --i) {
    r = g1_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = g1_add(r, p);
  }
  return r;
}

DG_FN g1a g1_to_affine(const g1j& p) {
  fp zi = fp_inv(p.z);
  fp zi2 = fp_sqr(zi);
  return g1a{fp_mul(p.x, zi2), fp_mul(p.y, fp_mul(zi2, zi))};
}

DG_NOINL void g1_compress(uint8_t* out, const g1a& a, bool infinity) {
  if (infinity) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; ++i) out[i] = 0;
    return;
  }
  fp_std_to_be48(fp_from_mont(a.x), out);
  out[0] |= 0x80;
  if (fp_std_gt_half(fp_from_mont(a.y))) out[0] |= 0x20;
}

// Decode a 48-byte compressed G1 point; G1 membership by [r] P == O (r as words).
DG_NOINL int g1_decompress(g1a* out, const uint8_t* in, const uint32_t* r_words) {
  uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return DEC_ERR_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; ++i) acc |= in[i];
    return acc ? DEC_ERR_INFINITY_NONCANON : DEC_INFINITY;
  }
  bool sign = (b0 & 0x20) != 0;
  uint8_t buf[48];
  for (int i = 0; i < 48; ++i) buf[i] = in[i];
  buf[0] &= 0x1f;
  fp xs = fp_std_from_be48(buf);
  if (!fp_std_lt_p(xs)) return DEC_ERR_X_RANGE;
  fp x = fp_to_mont(xs);
  fp rhs = fp_add(fp_mul(fp_sqr(x), x), C_B1);
  fp y = fp_sqrt_cand(rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return DEC_ERR_NOT_ON_CURVE;
  if (fp_std_gt_half(fp_from_mont(y)) != sign) y = fp_neg(y);
  out->x = x;
  out->y = y;
  g1j t = g1_mul_words(g1j{x, y, fp_one()}, r_words, 8);
  if (!g1_is_inf(t)) return DEC_ERR_SUBGROUP;
  return DEC_OK;
}

}  // namespace dgpu
