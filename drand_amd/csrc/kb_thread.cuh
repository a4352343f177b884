// Per-thread Karabina chain: one thread per round squares the compressed
// element (f1, f2, f4, f5) of the exponentiation input m 63 times and stores
// m^(2^s) at the six set bits s of |x| -- the same contract as the 8-lane
// k_eng_kb_chain (pairing_engine.cuh), whose planes and layout it reads and
// writes.  The compressed state is 8 Fp, so it stays in one thread's
// registers and every product runs on the thread's own lanes.
//
// Compressed squaring (Granger-Scott, tower.cuh fp12_cyclo_sqr, restricted to
// the closed outputs; Karabina 2010): with B = (f1, f4), C = (f2, f5) in
// Fp4 = Fp2[s]/(s^2 - xi),
//   B^2 = (f1^2 + xi f4^2, 2 f1 f4),  C^2 = (f2^2 + xi f5^2, 2 f2 f5)
//   f1' = 3 xi (2 f2 f5) + 2 f1,  f4' = 3 (f2^2 + xi f5^2) - 2 f4,
//   f2' = 3 (f1^2 + xi f4^2) - 2 f2,  f5' = 3 (2 f1 f4) + 2 f5.
// Six Fp2 squarings (2 f1 f4 = (f1 + f4)^2 - f1^2 - f4^2): 12 Fp products.
// Reference: the final exponentiation of kilic/bls12-381 (R), via
// chain/verify.go:44 -> kyber bls.Verify; tools/gen_engine.py KbChainModel.
#pragma once
#include "tower.cuh"

namespace dgpu {

// Lazy steps (units of p; inputs CI: normalized, < 2.01p; fp2_sqr outputs
// < 1.01p):
//   f1 + f4, f2 + f5 carried (< 4.02p) into fp2_sqr;
//   x^2 + xi y^2 = (X.re + Y.re + 8p - Y.im, X.im + Y.re + Y.im) carried
//   (< 11.1p, limbs < 2^28), tripled (< 33.3p, limbs < 2^29.6), minus 2 f
//   through fp_sub2_lz (+32p) -> < 65.3p, normalized and reduced to CI;
//   2ab = (a + b)^2 - (a^2 + b^2) through fp_sub2_lz carried (< 33.1p),
//   tripled plus 2 f (< 103.4p) -> CI; the xi-twisted one reduced to CI first
//   (xi needs its subtrahend < 7.99p), xi applied lazily and carried
//   (< 10.01p), tripled plus 2 f1 (< 34.1p) -> CI.
DG_FN fp kb_t_out(const fp& x3, const fp& f, bool minus) {
  fp t = fp_add_lz(fp_add_lz(x3, x3), x3);
  return fp_reduce(fp_norm(minus ? fp_sub2_lz(t, fp_add_lz(f, f)) : fp_add_lz(t, fp_add_lz(f, f))));
}
DG_FN fp2 kb_t_qsum(const fp2& xx, const fp2& yy) {  // xx + xi yy, carried
  return fp2{fp_norm(fp_add_lz(xx.c0, fp_sub_lz(yy.c0, yy.c1))), fp_norm(fp_add_lz(xx.c1, fp_add_lz(yy.c0, yy.c1)))};
}
DG_FN fp2 kb_t_cross(const fp2& ss, const fp2& xx, const fp2& yy) {  // ss - xx - yy, carried
  return fp2{fp_norm(fp_sub2_lz(ss.c0, fp_add_lz(xx.c0, yy.c0))), fp_norm(fp_sub2_lz(ss.c1, fp_add_lz(xx.c1, yy.c1)))};
}

// xi (2 f2 f5) = xi ((f2 + f5)^2 - f2^2 - f5^2) straight from the six product
// components (each < 1.01p, normalized), without reducing 2 f2 f5 first:
//   re = s.re + c2.im + c5.im - s.im - (c2.re + c5.re),
//   im = s.re + s.im - (c2.re + c5.re) - (c2.im + c5.im)
// with the subtrahends as 8p - x and 32p - (x + y) (fp_sub_lz, fp_sub2_lz):
// limbs < 3 (2^28) + 2^29 + 0x30000000 < 2^31, and 2 (2^28) + 2 x 0x30000000
// < 2^31; carried, < 43.1p and < 66.1p.  kb_t_out then triples them (< 2^30.3
// per limb after the carry) and adds 2 f1: < 133p and < 203p, inside
// fp_reduce's < 2^392.  Two reductions fewer per compressed squaring than
// reducing 2 f2 f5 before the twist.
DG_FN fp2 kb_t_xi_cross(const fp2& s, const fp2& c2, const fp2& c5) {
  const fp re = fp_sub2_lz(fp_sub_lz(fp_add_lz(fp_add_lz(s.c0, c2.c1), c5.c1), s.c1), fp_add_lz(c2.c0, c5.c0));
  const fp im = fp_sub2_lz(fp_sub2_lz(fp_add_lz(s.c0, s.c1), fp_add_lz(c2.c0, c5.c0)), fp_add_lz(c2.c1, c5.c1));
  return fp2{fp_norm(re), fp_norm(im)};
}

DG_FN void kb_sqr_thr(fp2& f1, fp2& f2, fp2& f4, fp2& f5) {
  // C side: f1' and f4' (they need the old f1, f4, which the B side squares)
  fp2 n1, n4;
  {
    const fp2 c2 = fp2_sqr(f2), c5 = fp2_sqr(f5);
    const fp2 c25 = fp2_sqr(fp2_carry(fp2_add_lz(f2, f5)));
    const fp2 q = kb_t_qsum(c2, c5);
    n4 = fp2{kb_t_out(q.c0, f4.c0, true), kb_t_out(q.c1, f4.c1, true)};
#ifdef DG_KB_XI_REDUCED  // A/B: 2 f2 f5 reduced before the twist (rounds 3-5)
    const fp2 x = kb_t_cross(c25, c2, c5);
    const fp2 xr{fp_reduce(x.c0), fp_reduce(x.c1)};
    const fp2 xx{fp_norm(fp_sub_lz(xr.c0, xr.c1)), fp_norm(fp_add_lz(xr.c0, xr.c1))};  // xi (2 f2 f5)
#else
    const fp2 xx = kb_t_xi_cross(c25, c2, c5);
#endif
    n1 = fp2{kb_t_out(xx.c0, f1.c0, false), kb_t_out(xx.c1, f1.c1, false)};
  }
  // B side: f2' and f5'
  const fp2 a1 = fp2_sqr(f1), a4 = fp2_sqr(f4);
  const fp2 a14 = fp2_sqr(fp2_carry(fp2_add_lz(f1, f4)));
  const fp2 q = kb_t_qsum(a1, a4);
  f2 = fp2{kb_t_out(q.c0, f2.c0, true), kb_t_out(q.c1, f2.c1, true)};
  const fp2 x = kb_t_cross(a14, a1, a4);
  f5 = fp2{kb_t_out(x.c0, f5.c0, false), kb_t_out(x.c1, f5.c1, false)};
  f1 = n1;
  f4 = n4;
}

// The same squaring split over two lanes (k_kb_chain_pair): the B lane holds
// (x, y) = (f1, f4), the C lane (f2, f5).  Each squares its own pair and forms
// q = x^2 + xi y^2 and k = 2xy (B) or xi 2xy (C), the lanes swap (q, k), and
// each forms its new pair from the partner's:
//   B: f1' = out(k_C, f1, +), f4' = out(q_C, f4, -);  C: f2' = out(q_B, f2, -), f5' = out(k_B, f5, +)
// -- kb_sqr_thr's outputs, term for term (the same bounds: kb_t_out's minus form
// takes a qsum, its plus form a cross or xi cross).  Selects are branch-free
// (the two lanes of a pair sit in one wave).
DG_FN void kb_pair_send(const fp2& x, const fp2& y, bool c, fp2& q, fp2& k) {
  const fp2 sx = fp2_sqr(x), sy = fp2_sqr(y);
  const fp2 sxy = fp2_sqr(fp2_carry(fp2_add_lz(x, y)));
  q = kb_t_qsum(sx, sy);
  const fp2 kb = kb_t_cross(sxy, sx, sy), kc = kb_t_xi_cross(sxy, sx, sy);
  k = fp2{fp_cmov(kb.c0, kc.c0, c), fp_cmov(kb.c1, kc.c1, c)};
}
DG_FN fp kb_t_out_sel(const fp& x3, const fp& f, bool minus) {
  const fp t = fp_add_lz(fp_add_lz(x3, x3), x3), f2 = fp_add_lz(f, f);
  return fp_reduce(fp_norm(fp_cmov(fp_add_lz(t, f2), fp_sub2_lz(t, f2), minus)));
}
DG_FN void kb_pair_recv(fp2& x, fp2& y, bool c, const fp2& rq, const fp2& rk) {
  const fp2 ax{fp_cmov(rk.c0, rq.c0, c), fp_cmov(rk.c1, rq.c1, c)};
  const fp2 ay{fp_cmov(rq.c0, rk.c0, c), fp_cmov(rq.c1, rk.c1, c)};
  x = fp2{kb_t_out_sel(ax.c0, x.c0, c), kb_t_out_sel(ax.c1, x.c1, c)};
  y = fp2{kb_t_out_sel(ay.c0, y.c0, !c), kb_t_out_sel(ay.c1, y.c1, !c)};
}

// 63 compressed squarings of (f1, f2, f4, f5); snap(j, f1, f2, f4, f5) after
// s = 16, 48, 57, 60, 62, 63 of them (sum of 2^s = |x|).
template <class Snap>
DG_FN void kb_chain_thr(fp2 f1, fp2 f2, fp2 f4, fp2 f5, Snap&& snap) {
  int s = 0;
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    const int sj = j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
#pragma unroll 1
    for (; s < sj; ++s) kb_sqr_thr(f1, f2, f4, f5);
    snap(j, f1, f2, f4, f5);
  }
}

}  // namespace dgpu

#ifndef DG_NO_KERNELS
#include "pairing_engine.cuh"
namespace dgpu {

#ifndef DG_KB_THR_OCC
#define DG_KB_THR_OCC 2
#endif
// Fp2 components (comp, comp + 1; comp even) of round i's plane: one dwordx2 per limb.
__device__ __forceinline__ fp2 kb_ld_thr(const uint32_t* xbuf, size_t i, int plane, int comp) {
  return kb_ld2(xbuf, i, plane, comp);
}
__device__ __forceinline__ void kb_st_thr(uint32_t* xbuf, size_t i, int plane, int comp, const fp2& v) {
  kb_st2(xbuf, i, plane, comp, v);
}

// Thread = round i of the chunk: m from plane M, the six stored values to
// planes X0.. (components 2..5, 8..11: f1, f2, f4, f5), dwordx2 per Fp2 limb.
// NORM (DGPU_KB_NORM=chain): at each snap also Norm(4 f1) of the stored value
// -> nbuf ([j][limb][cnt], round-fastest, coalesced), so k_eng_kb_norm_pre
// reads 6 x 56 B per round instead of the values' f1 halves from the blocked
// planes.
template <bool NORM>
__global__ void __launch_bounds__(256, DG_KB_THR_OCC) k_kb_chain_thr(size_t cnt, uint32_t* __restrict__ xbuf,
                                                                     uint32_t* __restrict__ nbuf) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt) return;
  kb_chain_thr(kb_ld_thr(xbuf, i, ENG_KB_PL_M, 2), kb_ld_thr(xbuf, i, ENG_KB_PL_M, 4),
               kb_ld_thr(xbuf, i, ENG_KB_PL_M, 8), kb_ld_thr(xbuf, i, ENG_KB_PL_M, 10),
               [&](int j, const fp2& f1, const fp2& f2, const fp2& f4, const fp2& f5) {
                 const int pl = ENG_KB_PL_X0 + j;
                 kb_st_thr(xbuf, i, pl, 2, f1);
                 kb_st_thr(xbuf, i, pl, 4, f2);
                 kb_st_thr(xbuf, i, pl, 8, f4);
                 kb_st_thr(xbuf, i, pl, 10, f5);
                 if constexpr (NORM) st_soa(nbuf + (size_t)j * FP_LIMBS * cnt, cnt, i, eng_kb_norm(f1));
               });
}

// Two lanes per round (kb_pair_send / _recv): 2 cnt threads, lane 2i the B
// half of round i, lane 2i + 1 the C half; each lane holds 4 Fp of state
// instead of 8, so the kernel fits fewer VGPRs than k_kb_chain_thr (more
// waves per SIMD; tools/engbench/powprobe.hip), for one swap of 4 Fp per
// squaring (quad_perm [1,0,3,2] DPP moves).  Same planes and snaps as
// k_kb_chain_thr; NORM: the B lane writes Norm(4 f1).
#ifndef DG_KB_PAIR_OCC
#define DG_KB_PAIR_OCC 3
#endif
__device__ __forceinline__ fp fp_swap_pair(const fp& a) {
  fp r;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) r.l[l] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.l[l], 0xB1, 0xF, 0xF, false);
  return r;
}
template <bool NORM>
__global__ void __launch_bounds__(256, DG_KB_PAIR_OCC) k_kb_chain_pair(size_t cnt, uint32_t* __restrict__ xbuf,
                                                                       uint32_t* __restrict__ nbuf) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i = t >> 1;
  if (i >= cnt) return;  // both lanes of a pair (same i) leave together
  const bool c = (t & 1) != 0;
  const int cx = c ? 4 : 2, cy = c ? 10 : 8;
  fp2 x = kb_ld_thr(xbuf, i, ENG_KB_PL_M, cx), y = kb_ld_thr(xbuf, i, ENG_KB_PL_M, cy);
  int s = 0;
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    const int sj = j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
#pragma unroll 1
    for (; s < sj; ++s) {
      fp2 q, k;
      kb_pair_send(x, y, c, q, k);
      kb_pair_recv(x, y, c, fp2{fp_swap_pair(q.c0), fp_swap_pair(q.c1)}, fp2{fp_swap_pair(k.c0), fp_swap_pair(k.c1)});
    }
    const int pl = ENG_KB_PL_X0 + j;
    kb_st_thr(xbuf, i, pl, cx, x);
    kb_st_thr(xbuf, i, pl, cy, y);
    if constexpr (NORM) {
      if (!c) st_soa(nbuf + (size_t)j * FP_LIMBS * cnt, cnt, i, eng_kb_norm(x));
    }
  }
}

}  // namespace dgpu
#endif
