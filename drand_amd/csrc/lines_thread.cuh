// Per-thread T-steps of the two Miller loops: one thread per (round, pair),
// the G2 point T in registers, 68 steps of line coefficients written to the
// engine's blocked line buffer (pairing_engine.cuh: [b][step][limb][g][6p+e]),
// where k_eng_miller consumes them.  Same contract as k_eng_lines (which stays
// for the on-G1 fixed-line table): pairs (pk, H_i) and (-g1, S_i), and the
// fused G2 membership test of S_i on pair 1's final T = [|x|] S_i.
//
// Why per thread: the T-steps carry no Fp12 state, so a thread holds one pair's
// point (6 Fp) and runs the step formulas with every Fp product on its own
// lanes -- no LDS slot round trips or per-sub-op waits of the 12-lane engine.
//
// Reference: chain/verify.go:44 -> kyber bls.Verify -> kilic Engine
// (miller loop line evaluations, R).  Line convention as pairing.cuh
// miller_dbl_step / miller_add_step: l = c0 + c2 w^2 + c3 w^3 with c2 linear in
// -xP and c3 in yP; each line may carry any Fp2 scale (killed by the final
// exponentiation), so the doubling below runs a 4x-scaled T with no halvings.
#pragma once
#include "pairing.cuh"

namespace dgpu {

// Doubling with its tangent line, homogeneous projective T (x = X/Z, y = Y/Z),
// E': y^2 = x^3 + b', b' = 4 xi.  With t0 = Y^2, t2 = 3 b' Z^2 = 12 xi Z^2,
// t3 = 3 t2:
//   X' = 2XY (t0 - t3), Y' = (t0 + t3)^2 - 12 t2^2, Z' = 4 t0 (2YZ)
//   (4x the classical (XY/2 (t0 - t3), ((t0 + t3)/2)^2 - 3 t2^2, t0 2YZ)),
//   line: c0 = t0 - t2, c2 = 3 X^2 (-xP), c3 = 2YZ yP.
// 2XY and 2YZ as (X + Y)^2 - X^2 - Y^2 and (Y + Z)^2 - Y^2 - Z^2, left
// unreduced (lt_sub32_nr: they only feed products).
// Bounds (units of p; CI = normalized, < 2.01p; fp_mul outputs < 1.01p here):
//   X + Y, Y + Z carried (< 4.02p) into fp2_sqr; t2 = 12 (xi Z^2) from the
//   carried lazy xi Z^2 (< 10.01p, limbs < 2^28 so 12x < 2^32) reduced to CI;
//   t3 = 3 t2 carried (< 6.03p); t0 + t3 carried (< 7.04p: fp2_sqr's
//   second coefficient < 7.99p); t0 + 8p - t3 carried (< 9.04p) into fp2_mul;
//   12 t2^2 carried (< 12.1p, fp2_sub32's bound 31.9p); 4 t0 carried (< 4.04p).
// a - b + 32p normalized, not reduced (< 33.2p: top limb < 2^23): only ever a
// multiplication operand (fp2_mul / fp2_mul_fp: sums < 2^29 per limb, value
// products < 70p x 4.1p).
DG_FN fp2 lt_sub32_nr(const fp2& a, const fp2& b) {
  return fp2{fp_norm(fp_sub2_lz(a.c0, b.c0)), fp_norm(fp_sub2_lz(a.c1, b.c1))};
}

// Each coefficient is handed to emit(k, value) (k = 0: c0, 1: c2, 2: c3) as
// soon as it is formed, and the statements run in the order that ends the
// most live ranges first (old X, then Y and Z, then the temporaries), so a
// step's line never waits in registers for the step's end: the kernel's
// stores retire each coefficient at once (the spilled
// live set of k_lines_thr).  Same operations and bounds as before.
// The pair's G1 point (-x_P, y_P) as held in registers (lt_pt_val) or
// reloaded from memory at each use (lt_pt_mem: DG_LINES_PT_RELOAD, which frees
// 28 VGPRs of the T-step loop; an empty asm on the address keeps the loads in
// the loop).
struct lt_pt_val {
  fp nx_, y_;
  DG_FN fp nx() const { return nx_; }
  DG_FN fp y() const { return y_; }
};

// T.x and T.z leave the doubling with their second coefficient reduced and
// the first only normalized (t0 + 8p - t1 < 9.2p; lt_fp2_mul_c1r, round 6):
// every consumer takes that -- fp2_sqr(X), fp2_sqr(Z) and the carried X + Y,
// Y + Z need c1 < 7.99p for their a0 - a1 and see products < 300 p^2; the
// addition step's products and fp2_sub minuends take any normalized operand
// -- and lt_pair_p reduces the final T (the membership test compares it).
// Two reductions fewer per doubling (A/B: -DDG_LINES_DBL_C1R).
DG_FN fp2 lt_fp2_mul_c1r(const fp2& a, const fp2& b) {
  const fp t0 = fp_mul(a.c0, b.c0);
  const fp t1 = fp_mul(a.c1, b.c1);
  const fp t2 = fp_mul(fp_add_lz(a.c0, a.c1), fp_add_lz(b.c0, b.c1));
  return fp2{fp_norm(fp_sub_lz(t0, t1)), fp_reduce(fp_norm(fp_sub2_lz(t2, fp_add_lz(t0, t1))))};
}
// Measured without gain (r06s: eng_lines 128.3 vs 127.6 ms per 2M, noise);
// the A/B build variant -DDG_LINES_DBL_C1R keeps it, both outputs reduced ship.
#ifdef DG_LINES_DBL_C1R
#define LT_MUL_OUT lt_fp2_mul_c1r
#else
#define LT_MUL_OUT fp2_mul
#endif

template <class PT, class Emit>
DG_FN void lt_dbl_p(g2p& T, const PT& P, Emit&& emit) {
  const fp nxp = P.nx();
  const fp2 t0 = fp2_sqr(T.y);
  const fp2 x2 = fp2_sqr(T.x);
  const fp2 xy2 = lt_sub32_nr(fp2_sqr(fp2_carry(fp2_add_lz(T.x, T.y))), fp2_add_lz(x2, t0));
  emit(1, fp2_mul_fp(fp2_carry(fp2_add_lz(fp2_add_lz(x2, x2), x2)), nxp));
  const fp2 t1 = fp2_sqr(T.z);
  const fp2 yz2 = lt_sub32_nr(fp2_sqr(fp2_carry(fp2_add_lz(T.y, T.z))), fp2_add_lz(t0, t1));
  emit(2, fp2_mul_fp(yz2, P.y()));
  const fp2 xt1 = fp2_carry(fp2{fp_sub_lz(t1.c0, t1.c1), fp_add_lz(t1.c0, t1.c1)});
  const fp2 t2 = fp2{fp_reduce(fp_norm(fp2_mulk_lz(xt1, 12).c0)), fp_reduce(fp_norm(fp2_mulk_lz(xt1, 12).c1))};
  emit(0, fp2_sub(t0, t2));
  T.z = LT_MUL_OUT(fp2_carry(fp2_mulk_lz(t0, 4)), yz2);
  const fp2 t3 = fp2_carry(fp2_add_lz(fp2_add_lz(t2, t2), t2));
  T.x = LT_MUL_OUT(xy2, fp2_carry(fp2{fp_sub_lz(t0.c0, t3.c0), fp_sub_lz(t0.c1, t3.c1)}));
  const fp2 t2sq = fp2_sqr(t2);
  T.y = fp2_sub32(fp2_sqr(fp2_carry(fp2_add_lz(t0, t3))), fp2_carry(fp2_mulk_lz(t2sq, 12)));
}

// Mixed addition T + Q (Q affine) with its chord line (pairing.cuh
// miller_add_step's formulas; 5 of the 68 steps), coefficients emitted early.
template <class PT, class Emit>
DG_FN void lt_add_p(g2p& T, const g2a& Q, const PT& P, Emit&& emit) {
  const fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  const fp2 lam = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  emit(1, fp2_mul_fp(theta, P.nx()));
  emit(2, fp2_mul_fp(lam, P.y()));
  emit(0, fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y)));
  const fp2 C = fp2_sqr(theta);
  const fp2 D = fp2_sqr(lam);
  const fp2 E = fp2_mul(lam, D);
  const fp2 F = fp2_mul(T.z, C);
  const fp2 G = fp2_mul(T.x, D);
  const fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  const fp2 ye = fp2_mul(T.y, E);
  T.x = fp2_mul(lam, H);
  T.y = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), ye);
  T.z = fp2_mul(T.z, E);
}

// The same steps returning the whole line (host emulation, tests).
DG_FN line3 lt_dbl(g2p& T, const fp& nxp, const fp& yp) {
  line3 l;
  lt_dbl_p(T, lt_pt_val{nxp, yp}, [&](int k, const fp2& v) { (k == 0 ? l.c0 : k == 1 ? l.c2 : l.c3) = v; });
  return l;
}
DG_FN line3 lt_add(g2p& T, const g2a& Q, const fp& nxp, const fp& yp) {
  line3 l;
  lt_add_p(T, Q, lt_pt_val{nxp, yp}, [&](int k, const fp2& v) { (k == 0 ? l.c0 : k == 1 ? l.c2 : l.c3) = v; });
  return l;
}

// One pair's 68 T-steps with the coefficients emitted one by one:
// emit(step, k, value); returns the final T = [|x|] Q.
// Q: the pair's affine G2 point as a value (lt_q_val) or reloaded at each
// addition (DG_LINES_Q_RELOAD).
struct lt_q_val {
  g2a q;
  DG_FN g2a get() const { return q; }
};

template <class QT, class PT, class Emit>
DG_FN g2p lt_pair_p(const QT& Qs, const PT& P, Emit&& emit) {
  const g2a Q0 = Qs.get();
  g2p T{Q0.x, Q0.y, fp2_one()};
  int step = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    lt_dbl_p(T, P, [&](int k, const fp2& v) { emit(step, k, v); });
    ++step;
    if ((BLS_X_ABS >> i) & 1ull) {
      lt_add_p(T, Qs.get(), P, [&](int k, const fp2& v) { emit(step, k, v); });
      ++step;
    }
  }
  T.x = fp2{fp_reduce(T.x.c0), T.x.c1};  // the last step is a doubling (bit 0 of |x| is 0)
  T.z = fp2{fp_reduce(T.z.c0), T.z.c1};
  return T;
}

// One pair's 68 T-steps (63 doublings, additions at the 5 lower set bits of
// |x|), sink(step, line) per step; returns the final T = [|x|] Q.
template <class Sink>
DG_FN g2p lt_pair(const g2a& Q, const fp& nxp, const fp& yp, Sink&& sink) {
  g2p T{Q.x, Q.y, fp2_one()};
  int step = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    sink(step++, lt_dbl(T, nxp, yp));
    if ((BLS_X_ABS >> i) & 1ull) sink(step++, lt_add(T, Q, nxp, yp));
  }
  T.x = fp2{fp_reduce(T.x.c0), T.x.c1};
  T.z = fp2{fp_reduce(T.z.c0), T.z.c1};
  return T;
}

// psi(S) == -T for T = [|x|] S (homogeneous): X = x_psi Z, Y = -y_psi Z, Z != 0
// (Scott's G2 membership test, as the engine's LSUB op).
DG_FN bool lt_in_g2(const g2p& T, const g2a& S) {
  const g2a ps = g2a_psi(S);
  return !fp2_is_zero(T.z) && fp2_is_zero(fp2_sub(T.x, fp2_mul(ps.x, T.z))) &&
         fp2_is_zero(fp2_add(T.y, fp2_mul(ps.y, T.z)));
}

#ifndef DG_NO_KERNELS
}  // namespace dgpu
#include "pairing_engine.cuh"
namespace dgpu {

#ifndef DG_LINES_OCC
#define DG_LINES_OCC 2
#endif
// Thread t: chunk-local round i = t / 2, pair p = t % 2.  Arguments as
// k_eng_lines (pairing_engine.cuh); consts: the engine constant block (pair
// points (-x, y) in slots ENG_C_NXP0..ENG_C_YP1).  Each step's 6 exports of
// the pair are 6 consecutive words per limb plane, written as 3 dwordx2.
// WAVE (no per-item keys, pk_items == nullptr): a wave holds 64 rounds of one
// pair (waves alternate between the pairs) instead of 32 rounds of both, so
// the pair's G1 point -- the key or -g1, the same for every lane -- is
// wave-uniform and lives in scalar registers (readfirstlane), off the T-step
// loop's VGPR budget.
template <bool WAVE>
__global__ void __launch_bounds__(256, DG_LINES_OCC) k_lines_thr(size_t n, size_t r0, size_t cnt,
                                                                 const uint32_t* __restrict__ h_pts, size_t h_stride,
                                                                 const uint32_t* __restrict__ h_idx,
                                                                 const uint32_t* __restrict__ sig_pts,
                                                                 const uint32_t* __restrict__ pk_items,
                                                                 const uint32_t* __restrict__ consts,
                                                                 uint32_t* __restrict__ lines,
                                                                 uint8_t* __restrict__ status) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i = WAVE ? ((t >> 7) << 6) + (t & 63) : t >> 1;
  const int p = WAVE ? (int)((t >> 6) & 1) : (int)(t & 1);
  if (i >= cnt) return;
  const size_t r = r0 + i;
  const uint32_t* qb = p ? sig_pts : h_pts;
  const size_t qs = p ? n : h_stride;
  const size_t qi = p ? r : (h_idx ? (size_t)h_idx[r] : r);
#ifdef DG_LINES_Q_RELOAD
  struct {
    const uint32_t* qb;
    size_t qs, qi;
    DG_FN g2a get() const {
      const uint32_t* b = qb;
      asm volatile("" : "+v"(b));  // opaque per use: not hoisted out of the loop
      g2a Q;
      Q.x.c0 = ld_soa(b, qs, qi);
      Q.x.c1 = ld_soa(b + (size_t)FP_LIMBS * qs, qs, qi);
      Q.y.c0 = ld_soa(b + (size_t)2 * FP_LIMBS * qs, qs, qi);
      Q.y.c1 = ld_soa(b + (size_t)3 * FP_LIMBS * qs, qs, qi);
      return Q;
    }
  } Qs{qb, qs, qi};
#else
  lt_q_val Qs;
  Qs.q.x.c0 = ld_soa(qb, qs, qi);
  Qs.q.x.c1 = ld_soa(qb + (size_t)FP_LIMBS * qs, qs, qi);
  Qs.q.y.c0 = ld_soa(qb + (size_t)2 * FP_LIMBS * qs, qs, qi);
  Qs.q.y.c1 = ld_soa(qb + (size_t)3 * FP_LIMBS * qs, qs, qi);
#endif
  // the pair's G1 point: words l * stride of pt (nx) and of pt + ystep (y)
  const uint32_t* pt;
  size_t stride, ystep;
  if (p == 0 && pk_items) {
    pt = pk_items + r, stride = n, ystep = (size_t)FP_LIMBS * n;
  } else {
    pt = consts + ((p ? ENG_C_NXP1 : ENG_C_NXP0) - 64) * ENG_SLOT_WORDS, stride = 1, ystep = ENG_SLOT_WORDS;
  }
  const size_t blk = i / ENG_ROUNDS_PER_BLOCK;
  uint32_t* base = lines + eng_blk_off(blk, ENG_LINE_STEPS, 0, (int)(i % ENG_ROUNDS_PER_BLOCK), 6 * p);
#ifdef DG_LINES_PT_RELOAD
  struct {
    const uint32_t* pt;
    size_t stride, ystep;
    DG_FN fp ld(size_t off) const {
      const uint32_t* q = pt + off;
      asm volatile("" : "+v"(q));  // opaque per use: not hoisted out of the loop
      fp v;
#pragma unroll
      for (int l = 0; l < FP_LIMBS; ++l) v.l[l] = q[l * stride];
      return v;
    }
    DG_FN fp nx() const { return ld(0); }
    DG_FN fp y() const { return ld(ystep); }
  } P{pt, stride, ystep};
#else
  lt_pt_val P;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) {
    if constexpr (WAVE) {  // uniform: scalar registers
      P.nx_.l[l] = __builtin_amdgcn_readfirstlane(pt[l * stride]);
      P.y_.l[l] = __builtin_amdgcn_readfirstlane(pt[ystep + l * stride]);
    } else {
      P.nx_.l[l] = pt[l * stride], P.y_.l[l] = pt[ystep + l * stride];
    }
  }
#endif
  const g2p T = lt_pair_p(Qs, P, [&](int step, int k, const fp2& v) {
    uint2* b = reinterpret_cast<uint2*>(base + (size_t)step * FP_LIMBS * ENG_WAVE_WORDS) + k;
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) b[l * (ENG_WAVE_WORDS / 2)] = make_uint2(v.c0.l[l], v.c1.l[l]);
  });
  if (status && p == 1 && !lt_in_g2(T, Qs.get()) && status[r] == ST_OK) status[r] = ST_SUBGROUP;
}
#endif

}  // namespace dgpu
