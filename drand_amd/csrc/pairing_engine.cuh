// Per-round pairing check e(pk, H) * e(-g1, sig) == 1 on the lane-cooperative
// engine (engine.cuh), as four launches over a chunk of rounds:
//
//   k_eng_lines   T-steps of both Miller loops (pairs (pk, H) and (-g1, sig)):
//                 68 steps x 2 lines x 6 Fp of line coefficients -> HBM
//   k_eng_miller  f = prod of lines (shared squaring), then N1 = Norm(f) in Fp
//   k_eng_inv     batch inversion of N1 (Montgomery's trick, 1 exponentiation
//                 per 64 rounds)
//   k_eng_fe      f^-1 from N1^-1, final exponentiation, f == 1 -> verdict
//
// Reference: chain/verify.go:44 -> kyber bls.Verify -> ValidatePairing ->
// kilic Engine AddPair/AddPairInv/Check (R).  The conjugation of the Miller
// value (x < 0) is skipped: FE(conj f) = FE(f)^-1, equal to 1 iff FE(f) is.
//
// HBM layouts (chunk-local round index i = 5 b + g, block b, chunk capacity cap):
//   lines  [b][step 0..67][limb][g][export 0..11]  (export 6p + e: pair p, l0.re .. l3.im)
//   fbuf   [b][plane 0..1][limb][g][component 0..11] (f, later t and t2 of the FE)
//   n1     [limb][i]
#pragma once
#include "engine.cuh"
#include "kernels.cuh"

namespace dgpu {

constexpr int ENG_BLOCK = 64;                                  // one wave: 5 rounds
constexpr int ENG_ROUNDS_PER_BLOCK = ENG_GROUPS_PER_WAVE;
constexpr int ENG_LINE_STEPS = 68;

// block constant region, host-built (capi.hip: eng_consts_for)
struct eng_const_block {
  uint32_t w[ENG_NCONST * ENG_SLOT_WORDS];
};

struct eng_lane {
  int g, k;      // group in the wave, lane in the group
  size_t i;      // chunk-local round (clamped)
  size_t blk;    // the wave's block of 5 rounds (blockIdx.x, or a listed block: k_eng_fe_fb)
  bool valid;
};

__device__ __forceinline__ eng_lane eng_lane_id(size_t cnt, size_t blk) {
  const int lane = threadIdx.x & 63;
  eng_lane L;
  L.g = lane < 60 ? lane / 12 : 4;
  L.k = lane < 60 ? lane % 12 : lane - 60;
  L.blk = blk;
  const size_t gi = blk * ENG_ROUNDS_PER_BLOCK + L.g;
  L.valid = gi < cnt;
  L.i = L.valid ? gi : cnt - 1;
  return L;
}

__device__ __forceinline__ void eng_load_consts(uint32_t* c, const uint32_t* src) {
  for (int t = threadIdx.x; t < ENG_NCONST * ENG_SLOT_WORDS; t += blockDim.x) c[t] = src[t];
  __syncthreads();
}

__device__ __forceinline__ void st_soa(uint32_t* base, size_t stride, size_t i, const fp& a) {
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) base[(size_t)l * stride + i] = a.l[l];
}
__device__ __forceinline__ fp ld_soa(const uint32_t* base, size_t stride, size_t i) {
  fp a;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) a.l[l] = base[(size_t)l * stride + i];
  return a;
}

// Wave-blocked layout of the line and f buffers: block b (rounds 5b..5b+4)
// owns planes [b][plane][limb][60] with word g*12 + e (group g, export e), so
// every limb access of a wave is one contiguous 240-byte segment (a
// round-fastest SoA would scatter the 60 lanes over 12 planes, 20 bytes each).
constexpr int ENG_WAVE_WORDS = ENG_GROUPS_PER_WAVE * 12;
__device__ __forceinline__ size_t eng_blk_off(size_t blk, int planes, int plane, int g, int e) {
  return (blk * planes + plane) * FP_LIMBS * ENG_WAVE_WORDS + g * 12 + e;
}
__device__ __forceinline__ eng_lane eng_lane_id(size_t cnt) { return eng_lane_id(cnt, blockIdx.x); }
__device__ __forceinline__ void st_blk(uint32_t* base, size_t off, const fp& a) {
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) base[off + l * ENG_WAVE_WORDS] = a.l[l];
}
__device__ __forceinline__ fp ld_blk(const uint32_t* base, size_t off) {
  fp a;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) a.l[l] = base[off + l * ENG_WAVE_WORDS];
  return a;
}

// HBM side of a kernel program (chunk-local buffers).
struct eng_io {
  uint32_t* lines;   // blocked, ENG_LINE_STEPS planes of 12 exports per round
  uint32_t* fbuf;    // blocked, 2 planes of 12 components (f / t, then t2)
  uint32_t* n1;      // [limb][cnt]
  size_t cnt;
  const uint32_t* table = nullptr;  // FIXED: on-G1 line table (k_eng_lines_fixed's layout)
  fp mlt{};                         // FIXED: this lane's export multiplier (P coordinate)
  bool scale = false;               // FIXED: export L.k is linear in a P coordinate
  uint32_t* xbuf = nullptr;         // Karabina FE: LD12 / ST12 address its ENG_KB_PLANES state planes instead of fbuf
};

// The program interpreter (one inlined copy of the op interpreter per kernel).
// FIXED: LDLINE reads the per-key line table and scales it by the lane's P
// coordinate (the on-G1 lines, computed in place of k_eng_lines_fixed).
// CYC: E_CYC runs straight-line (engine.cuh eng_cyc_fast), the FE kernel only.
// FAM: the kernel's family of compiled ops (engine_compiled.h eng_run_c<FAM>:
// 0 lines, 1 Miller, 2 FE), -1 none.
#ifndef DG_ENG_NO_CYC_FAST
constexpr bool ENG_CYC_FAST = true;
#else
constexpr bool ENG_CYC_FAST = false;
#endif
#ifndef DG_ENG_NO_COMPILED
constexpr bool ENG_COMPILED = true;
#else
constexpr bool ENG_COMPILED = false;
#endif
// KB: LD12 / ST12 address the Karabina FE planes (io.xbuf), else fbuf.
// XW: the group's lanes may span waves (eng_sync barriers; k_eng_miller_xw).
template <bool FIXED = false, bool CYC = false, int FAM = -1, bool KB = false, bool XW = false>
__device__ __forceinline__ void eng_exec(const uint32_t* prog, int len, uint32_t* g, const uint32_t* c,
                                         const eng_lane& L, const eng_io& io) {
  int step = 0;
  auto sink = [&](uint32_t e, const fp& v) {
    if (!L.valid) return;
    if (e < 12) st_blk(io.lines, eng_blk_off(L.blk, ENG_LINE_STEPS, step, L.g, (int)e), v);
    else st_soa(io.n1, io.cnt, L.i, v);
  };
#pragma unroll 1
  for (int pc = 0; pc < len; ++pc) {
    const uint32_t ins = prog[pc];
    const uint32_t opc = ins >> 24, a = ins & 0xFFu, b = (ins >> 8) & 0xFFu;
    if (opc == ENG_OPC_RUN) {
      if (CYC && a == OP_E_CYC) {  // the run of E_CYC ops starting here, as one chain
        int n = 1;
        while (pc + n < len && prog[pc + n] == ins) ++n;
        eng_cyc_chain(g, L.k, n);
        pc += n - 1;
        continue;
      }
      bool done = false;
      if constexpr (ENG_COMPILED && FAM == 0) done = eng_run_c0<XW>((int)a, g, c, L.k, sink);
      if constexpr (ENG_COMPILED && FAM == 1) done = eng_run_c1<XW>((int)a, g, c, L.k, sink);
      if constexpr (ENG_COMPILED && FAM == 2) done = eng_run_c2<XW>((int)a, g, c, L.k, sink);
      if (!done) eng_run<XW>((int)a, g, c, L.k, sink);
    } else if (opc == ENG_OPC_STEP) {
      ++step;
    } else if (opc == ENG_OPC_LDLINE) {
      if constexpr (FIXED) {
        fp v = ld_blk(io.table, (size_t)step * FP_LIMBS * ENG_WAVE_WORDS + L.k);
        if (io.scale) v = fp_mul(v, io.mlt);
        eng_st(g + (a + L.k) * ENG_SLOT_WORDS, v);
      } else {
        eng_st(g + (a + L.k) * ENG_SLOT_WORDS, ld_blk(io.lines, eng_blk_off(L.blk, ENG_LINE_STEPS, step, L.g, L.k)));
      }
      ++step;
      // consecutive LDLINEs (l1, l2 of a step) share one barrier
      if (!(pc + 1 < len && (prog[pc + 1] >> 24) == ENG_OPC_LDLINE)) eng_sync<XW>();
    } else if (opc == ENG_OPC_LD12) {
      const int pl = (int)b / 12;
      if constexpr (KB) eng_st(g + (a + L.k) * ENG_SLOT_WORDS, ld_blk(io.xbuf, eng_blk_off(L.blk, ENG_KB_PLANES, pl, L.g, L.k)));
      else eng_st(g + (a + L.k) * ENG_SLOT_WORDS, ld_blk(io.fbuf, eng_blk_off(L.blk, 2, (int)b / 12, L.g, L.k)));
      eng_sync<XW>();
    } else if (opc == ENG_OPC_ST12) {
      if (L.valid) {
        if constexpr (KB) st_blk(io.xbuf, eng_blk_off(L.blk, ENG_KB_PLANES, (int)b / 12, L.g, L.k), eng_ld(g + (a + L.k) * ENG_SLOT_WORDS));
        else st_blk(io.fbuf, eng_blk_off(L.blk, 2, (int)b / 12, L.g, L.k), eng_ld(g + (a + L.k) * ENG_SLOT_WORDS));
      }
      eng_sync<XW>();
    }
    asm volatile("" ::: "memory");
  }
}

// x == K mod p for x < 2.01p (normalized) and a canonical constant K < p
__device__ __forceinline__ bool eng_eq_canon(const fp& x, const fp& K) {
  fp k1 = fp_norm(fp_add_lz(K, fp{{FP_P[0], FP_P[1], FP_P[2], FP_P[3], FP_P[4], FP_P[5], FP_P[6], FP_P[7], FP_P[8],
                                    FP_P[9], FP_P[10], FP_P[11], FP_P[12], FP_P[13]}}));
  fp k2 = fp_norm(fp_add_lz(k1, fp{{FP_P[0], FP_P[1], FP_P[2], FP_P[3], FP_P[4], FP_P[5], FP_P[6], FP_P[7], FP_P[8],
                                     FP_P[9], FP_P[10], FP_P[11], FP_P[12], FP_P[13]}}));
  uint32_t d0 = 0, d1 = 0, d2 = 0;
#pragma unroll
  for (int i = 0; i < FP_LIMBS; ++i) {
    d0 |= x.l[i] ^ K.l[i];
    d1 |= x.l[i] ^ k1.l[i];
    d2 |= x.l[i] ^ k2.l[i];
  }
  return d0 == 0 || d1 == 0 || d2 == 0;
}

// ---------------------------------------------------------------- k_eng_lines
// Item i (chunk-local; global item r0 + i) checks e(P_i, H_i) e(-g1, S_i):
//   H_i = h_pts[h_idx ? h_idx[r0 + i] : r0 + i], S_i = sig_pts[r0 + i]
//   (affine G2 SoA [x.c0, x.c1, y.c0, y.c1][limb][stride]),
//   P_i = pk_items ? pk_items[r0 + i] ((-x, y) SoA [2][limb][n]) : the block constant key.
// status (optional, per item): after the loop T of pair 1 is [|x|] S_i, and
// the program's LSUB op tests psi(S_i) == -T (tools/gen_engine.py
// lines_subgroup_op) -- the G2 membership check of the signature, so the
// decoder can skip its own 63-doubling ladder; a failing item with status
// ST_OK becomes ST_SUBGROUP.
__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_lines(size_t n, size_t r0, size_t cnt,
                                                         const uint32_t* __restrict__ h_pts, size_t h_stride,
                                                         const uint32_t* __restrict__ h_idx,
                                                         const uint32_t* __restrict__ sig_pts,
                                                         const uint32_t* __restrict__ pk_items,
                                                         const uint32_t* __restrict__ consts,
                                                         uint32_t* __restrict__ lines,
                                                         uint8_t* __restrict__ status,
                                                         uint32_t* __restrict__ t_out) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_LINES * ENG_SLOT_WORDS];
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  const eng_lane L = eng_lane_id(cnt);
  uint32_t* g = lds + ENG_GBASE_LINES[L.g] * ENG_SLOT_WORDS;
  const size_t r = r0 + L.i;
  if (L.k < 8) {  // Q coordinates: X, Y of T and the affine copy (xQ, yQ)
    const int p = L.k >> 2, comp = L.k & 3;
    const fp q = p ? ld_soa(sig_pts + (size_t)comp * FP_LIMBS * n, n, r)
                   : ld_soa(h_pts + (size_t)comp * FP_LIMBS * h_stride, h_stride, h_idx ? (size_t)h_idx[r] : r);
    eng_st(g + (p * ENG_LINE_PAIR_SLOTS + comp) * ENG_SLOT_WORDS, q);
    eng_st(g + (p * ENG_LINE_PAIR_SLOTS + 6 + comp) * ENG_SLOT_WORDS, q);
  } else {        // Z = 1
    const int p = (L.k - 8) >> 1, comp = (L.k - 8) & 1;
    eng_st(g + (p * ENG_LINE_PAIR_SLOTS + 4 + comp) * ENG_SLOT_WORDS, comp ? fp_zero() : fp_one());
  }
  if (L.k < 2) {  // pair 0's G1 point
    const fp v = pk_items ? ld_soa(pk_items + (size_t)L.k * FP_LIMBS * n, n, r)
                          : eng_ld(c + (ENG_C_NXP0 + L.k - 64) * ENG_SLOT_WORDS);
    eng_st(g + (ENG_L_NXP0 + L.k) * ENG_SLOT_WORDS, v);
  }
  asm volatile("" ::: "memory");
  eng_exec<false, false, 0>(ENG_PROG_LINES, ENG_PROG_LINES_LEN, g, c, L, eng_io{lines, nullptr, nullptr, cnt});
  if (status) {
    // lanes 0..3 test D1, D2 == 0, lanes 4, 5 test Z (re, im) == 0
    const int sl = L.k < 2 ? ENG_L_SUB_D1 + L.k : L.k < 4 ? ENG_L_SUB_D2 + L.k - 2 : ENG_L_SUB_Z + (L.k & 1);
    const bool zero = eng_eq_canon(eng_ld(g + sl * ENG_SLOT_WORDS), fp_zero());
    const uint64_t gm = (__ballot(zero) >> (12 * L.g)) & 0x3Full;
    const bool in_g2 = (gm & 0xFull) == 0xFull && (gm & 0x30ull) != 0x30ull;
    if (L.valid && L.k == 0 && !in_g2 && status[r0 + L.i] == ST_OK) status[r0 + L.i] = ST_SUBGROUP;
  }
  if (t_out && L.valid) {  // T of both pairs (homogeneous X, Y, Z): [12 fp][cnt], lane k = 6 pair + component
    const int pr = L.k / 6, comp = L.k - 6 * pr;
    st_soa(t_out + (size_t)L.k * FP_LIMBS * cnt, cnt, L.i, eng_ld(g + (pr * ENG_LINE_PAIR_SLOTS + comp) * ENG_SLOT_WORDS));
  }
}

// ---------------------------------------------------------------- small-batch cofactor clearing
// For a call of a few thousand rounds k_h2c_finish is one thread's 126
// sequential doublings per round (~4.4 ms at n = 1).  Its two ladders run
// instead on the 12-lane LINES program, whose T after the loop is [|x|]Q
// (k_eng_lines' t_out; the line coefficients go to a scratch buffer):
//   k_cof_prep   P = Q0 + Q1 (Jacobian kept); P and psi(P) affine
//   k_eng_lines  T0 = [|x|]P, T1 = [|x|]psi(P)            (homogeneous)
//   k_cof_mid    T0 affine: the second pass's input
//   k_eng_lines  T2 = [|x|]T0 = [x^2]P    beside   k_cof_partial  U = T0 - P - T1 - psi(P) + psi^2(2P)
//   k_cof_final  h_eff P = T2 + U
// with [x]P = -T0, [x]psi(P) = -T1: RFC 9380 G.3's [x^2 - x - 1]P +
// [x - 1]psi(P) + psi^2(2P) regrouped, written as k_h2c_finish writes it
// (X, Y to h_out, Z to z_out).  Exceptional ladder steps need P of order
// below 2^64 + 1 -- a hash output is not (every point the ladder meets is
// then a nonzero multiple of a large-order point); the additions here are
// the complete g2_add.
// Scratch planes (stride n): pj [6] | pa [4] | psia [4] | t1 [12] | t0a [4] | t2 [12] | u [6]
constexpr int COF_PLANES = 6 + 4 + 4 + 12 + 4 + 12 + 6;
__device__ __forceinline__ g2j cof_homog_to_jac(const uint32_t* t, size_t n, size_t i, int pr) {
  const uint32_t* b = t + (size_t)pr * 6 * FP_LIMBS * n;
  const fp2 X{ld_soa(b, n, i), ld_soa(b + FP_LIMBS * n, n, i)};
  const fp2 Y{ld_soa(b + 2 * FP_LIMBS * n, n, i), ld_soa(b + 3 * FP_LIMBS * n, n, i)};
  const fp2 Z{ld_soa(b + 4 * FP_LIMBS * n, n, i), ld_soa(b + 5 * FP_LIMBS * n, n, i)};
  return g2j{fp2_mul(X, Z), fp2_mul(Y, fp2_sqr(Z)), Z};  // x = X/Z = XZ/Z^2, y = Y/Z = YZ^2/Z^3
}
__global__ void __launch_bounds__(256) k_cof_prep(size_t n, const uint32_t* __restrict__ q, uint32_t* __restrict__ w) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const g2j P = g2_add(ld_g2j(q, n, i), ld_g2j(q + G2J_WORDS * n, n, i));
  st_g2j(w, n, i, P);
  const g2a a = g2_to_affine(P);
  st_g2a(w + G2J_WORDS * n, n, i, a);
  const g2j s = g2_psi(g2_from_affine(a));  // Z = conj(1) = 1: still affine
  st_g2a(w + (G2J_WORDS + G2A_WORDS) * n, n, i, g2a{s.x, s.y});
}
__global__ void __launch_bounds__(256) k_cof_mid(size_t n, uint32_t* __restrict__ w) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* t1 = w + (G2J_WORDS + 2 * G2A_WORDS) * n;
  const fp2 zi = fp2_inv(fp2{ld_soa(t1 + 4 * FP_LIMBS * n, n, i), ld_soa(t1 + 5 * FP_LIMBS * n, n, i)});
  const fp2 X{ld_soa(t1, n, i), ld_soa(t1 + FP_LIMBS * n, n, i)};
  const fp2 Y{ld_soa(t1 + 2 * FP_LIMBS * n, n, i), ld_soa(t1 + 3 * FP_LIMBS * n, n, i)};
  st_g2a(w + (G2J_WORDS + 2 * G2A_WORDS + 12 * FP_WORDS) * n, n, i, g2a{fp2_mul(X, zi), fp2_mul(Y, zi)});
}
// U = T0 - P - T1 - psi(P) + psi^2(2P): everything but [x^2]P, from the
// first pass alone -- it runs on a second stream beside the second pass
__global__ void __launch_bounds__(256) k_cof_partial(size_t n, uint32_t* __restrict__ w) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* t1 = w + (G2J_WORDS + 2 * G2A_WORDS) * n;
  const g2j P = ld_g2j(w, n, i);
  g2j u = g2_add(cof_homog_to_jac(t1, n, i, 0), g2_neg(P));                       // -[x]P - P
  u = g2_add(u, g2_neg(cof_homog_to_jac(t1, n, i, 1)));                            // + [x]psi(P)
  u = g2_add(u, g2_neg(g2_psi(P)));
  u = g2_add(u, g2_psi2(g2_dbl(P)));
  st_g2j(w + (G2J_WORDS + 3 * G2A_WORDS + 24 * FP_WORDS) * n, n, i, u);
}
// h_eff P = [x^2]P + U
__global__ void __launch_bounds__(256) k_cof_final(size_t n, const uint32_t* __restrict__ w, uint32_t* __restrict__ h_out,
                                                   uint32_t* __restrict__ z_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* t2 = w + (G2J_WORDS + 3 * G2A_WORDS + 12 * FP_WORDS) * n;
  const g2j h = g2_add(cof_homog_to_jac(t2, n, i, 0), ld_g2j(t2 + 12 * FP_WORDS * n, n, i));
  st_g2a(h_out, n, i, g2a{h.x, h.y});
  st_fp(z_out, n, i, h.z.c0);
  st_fp(z_out + FP_WORDS * n, n, i, h.z.c1);
}

// ---------------------------------------------------------------- k_eng_miller
// (4 waves/SIMD measured slower, r02m: the 128-VGPR cap spills)
__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_miller(size_t cnt, const uint32_t* __restrict__ consts,
                                                          uint32_t* __restrict__ lines,
                                                          uint32_t* __restrict__ fbuf, uint32_t* __restrict__ n1) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_MILLER * ENG_SLOT_WORDS];
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  const eng_lane L = eng_lane_id(cnt);
  uint32_t* g = lds + ENG_GBASE_MILLER[L.g] * ENG_SLOT_WORDS;
  eng_st(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS, L.k == 0 ? fp_one() : fp_zero());
  asm volatile("" ::: "memory");
  eng_exec<false, false, 1>(ENG_PROG_MILLER, ENG_PROG_MILLER_LEN, g, c, L, eng_io{lines, fbuf, n1, cnt});
  if (L.valid) st_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k), eng_ld(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS));
}

// ---------------------------------------------------------------- k_eng_miller_xw
// k_eng_miller without idle lanes: a 192-thread block (three waves) holds 16
// groups of 12 lanes, so every lane carries an item (a 64-lane wave holds
// five groups and four idle lanes).  Groups 5 and 10 span two waves, so the
// sub-ops are ordered by barriers (engine.cuh eng_sync).  The DPP partner of
// lane k (k ^ 1) stays in its wave: groups start at even lanes and the wave
// boundaries (64, 128) fall on even k.  Item i = 16 blockIdx.x + group; the
// HBM buffers keep the 5-round blocked layout (block i / 5, group i % 5).
constexpr int ENG_XW_ITEMS = 16;
constexpr int ENG_XW_BLOCK = ENG_XW_ITEMS * 12;  // three waves
static_assert(ENG_XW_BLOCK == 192, "16 groups of 12 lanes");

__device__ __forceinline__ eng_lane eng_lane_xw(size_t cnt, int& grp) {
  grp = (int)threadIdx.x / 12;
  eng_lane L;
  L.k = (int)threadIdx.x - 12 * grp;
  const size_t gi = (size_t)blockIdx.x * ENG_XW_ITEMS + grp;
  L.valid = gi < cnt;
  L.i = L.valid ? gi : cnt - 1;
  L.blk = L.i / ENG_ROUNDS_PER_BLOCK;
  L.g = (int)(L.i - L.blk * ENG_ROUNDS_PER_BLOCK);
  return L;
}

__global__ void __launch_bounds__(ENG_XW_BLOCK, 3) k_eng_miller_xw(size_t cnt, const uint32_t* __restrict__ consts,
                                                                uint32_t* __restrict__ lines,
                                                                uint32_t* __restrict__ fbuf, uint32_t* __restrict__ n1) {
  __shared__ uint32_t lds[(ENG_NCONST + ENG_XW_ITEMS * ENG_SLOTS_MILLER) * ENG_SLOT_WORDS];
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  int grp;
  const eng_lane L = eng_lane_xw(cnt, grp);
  uint32_t* g = lds + (ENG_NCONST + grp * ENG_SLOTS_MILLER) * ENG_SLOT_WORDS;
  eng_st(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS, L.k == 0 ? fp_one() : fp_zero());
  eng_sync<true>();
  eng_exec<false, false, 1, false, true>(ENG_PROG_MILLER, ENG_PROG_MILLER_LEN, g, c, L, eng_io{lines, fbuf, n1, cnt});
  if (L.valid) st_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k), eng_ld(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS));
}

// ---------------------------------------------------------------- k_eng_inv
// Thread t inverts the N1 of rounds t, t + T, t + 2T, ... (T = threads in the
// grid) by Montgomery's trick; prefix products go to `pre` (same layout).
// A zero N1 (f not invertible: FE(f) = 0 != 1) fails its round.
__global__ void __launch_bounds__(256) k_eng_inv(size_t cnt, size_t r0, uint32_t* __restrict__ n1,
                                                 uint32_t* __restrict__ pre, uint8_t* __restrict__ status) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  fp acc = fp_one();
  size_t last = t;
  for (size_t i = t; i < cnt; i += T) {
    fp v = ld_soa(n1, cnt, i);
    if (fp_is_zero(v)) {
      v = fp_one();
      if (status[r0 + i] == ST_OK) status[r0 + i] = ST_PAIRING;
      st_soa(n1, cnt, i, v);
    }
    acc = fp_mul(acc, v);
    st_soa(pre, cnt, i, acc);
    last = i;
  }
  fp inv = fp_inv(acc);
  for (size_t i = last;; i -= T) {
    const fp v = ld_soa(n1, cnt, i);
    const fp out = i >= t + T ? fp_mul(inv, ld_soa(pre, cnt, i - T)) : inv;
    st_soa(n1, cnt, i, out);
    if (i < t + T) break;
    inv = fp_mul(inv, v);
  }
}

// ---------------------------------------------------------------- k_eng_fe
// The Granger-Scott FE (prog_fe) of the block `blk` of 5 rounds.
// only != nullptr: the Karabina path's fallback -- only flagged items take a verdict.
__device__ __forceinline__ void eng_fe_block(size_t blk, size_t cnt, size_t r0, const uint32_t* __restrict__ consts,
                                             uint32_t* __restrict__ fbuf, const uint32_t* __restrict__ n1inv,
                                             uint8_t* __restrict__ status, const uint8_t* __restrict__ only,
                                             uint32_t* lds) {
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  const eng_lane L = eng_lane_id(cnt, blk);
  uint32_t* g = lds + ENG_GBASE_FE[L.g] * ENG_SLOT_WORDS;
  eng_st(g + (ENG_E_F + L.k) * ENG_SLOT_WORDS, ld_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k)));
  if (L.k == 0) eng_st(g + ENG_E_N1I * ENG_SLOT_WORDS, ld_soa(n1inv, cnt, L.i));
  asm volatile("" ::: "memory");
  eng_exec<false, ENG_CYC_FAST, 2>(ENG_PROG_FE, ENG_PROG_FE_LEN, g, c, L, eng_io{nullptr, fbuf, nullptr, cnt});
  const fp v = eng_ld(g + (ENG_E_R + L.k) * ENG_SLOT_WORDS);
  const bool ok = eng_eq_canon(v, L.k == 0 ? fp_one() : fp_zero());
  const uint64_t m = __ballot(ok);
  const bool all = ((m >> (12 * L.g)) & 0xFFFull) == 0xFFFull;
  if (L.valid && L.k == 0 && !all && (!only || only[L.i]) && status[r0 + L.i] == ST_OK) status[r0 + L.i] = ST_PAIRING;
}

__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_fe(size_t cnt, size_t r0, const uint32_t* __restrict__ consts,
                                                      uint32_t* __restrict__ fbuf, const uint32_t* __restrict__ n1inv,
                                                      uint8_t* __restrict__ status) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_FE * ENG_SLOT_WORDS];
  eng_fe_block(blockIdx.x, cnt, r0, consts, fbuf, n1inv, status, nullptr, lds);
}

// ---------------------------------------------------------------- Karabina FE
// Per chunk: k_eng_fe_seg(0), then for each of the five exponentiations by
// |x|: k_eng_kb_chain -> k_eng_kb_norm -> k_eng_inv -> k_eng_kb_dec ->
// k_eng_fe_seg(e); finally k_eng_fe_fb re-runs the listed blocks with a
// flagged item (f1 = 0 at a stored value: practically never) on prog_fe.
//
// State planes (gen_engine.py PL_*: t, t2, the exponentiation input m, the
// six stored m^(2^s)) in fbuf's wave-blocked layout with ENG_KB_PLANES planes:
// [block of 5 rounds][plane][limb][g * 12 + component].
__device__ __forceinline__ size_t kb_off(size_t i, int plane, int comp) {
  const size_t blk = i / ENG_ROUNDS_PER_BLOCK;
  const int g = (int)(i - blk * ENG_ROUNDS_PER_BLOCK);
  return (blk * ENG_KB_PLANES + plane) * FP_LIMBS * ENG_WAVE_WORDS + g * 12 + comp;
}
// Fp2 components (comp, comp + 1; comp even) of round i's plane: one dwordx2
// per limb (8-byte aligned: g * 48 + comp * 4 bytes).  The per-thread
// kernels' accesses; 4-byte loads of each component let a wave's loads of one
// value spread over L2 long enough to be evicted between components (r04q:
// k_eng_kb_norm fetched 22 KB per round for 2.7 KB of f1 values).
__device__ __forceinline__ fp2 kb_ld2(const uint32_t* xbuf, size_t i, int plane, int comp) {
  const uint32_t* b = xbuf + kb_off(i, plane, comp);
  fp2 v;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) {
    const uint2 w = *reinterpret_cast<const uint2*>(b + l * ENG_WAVE_WORDS);
    v.c0.l[l] = w.x, v.c1.l[l] = w.y;
  }
  return v;
}
__device__ __forceinline__ void kb_st2(uint32_t* xbuf, size_t i, int plane, int comp, const fp2& v) {
  uint32_t* b = xbuf + kb_off(i, plane, comp);
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) *reinterpret_cast<uint2*>(b + l * ENG_WAVE_WORDS) = make_uint2(v.c0.l[l], v.c1.l[l]);
}

// Segment [off, off + len) of ENG_PROG_FEK (gen_engine.py prog_fe_kb) on the
// 12-lane engine.  first: read f and 1/N1 as k_eng_fe does, clear the items'
// flags and the fallback list; last: R == 1 -> verdict for unflagged items,
// and the block joins the fallback list fb = [count, blocks...] if any of
// its items is flagged.
__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_fe_seg(int off, int len, bool first, bool last, size_t cnt,
                                                          size_t r0, const uint32_t* __restrict__ consts,
                                                          const uint32_t* __restrict__ fbuf,
                                                          const uint32_t* __restrict__ n1inv, uint32_t* __restrict__ xbuf,
                                                          uint8_t* __restrict__ flags, uint32_t* __restrict__ fb,
                                                          uint8_t* __restrict__ status) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_FE * ENG_SLOT_WORDS];
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  const eng_lane L = eng_lane_id(cnt);
  uint32_t* g = lds + ENG_GBASE_FE[L.g] * ENG_SLOT_WORDS;
  if (first) {
    eng_st(g + (ENG_E_F + L.k) * ENG_SLOT_WORDS, ld_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k)));
    if (L.k == 0) eng_st(g + ENG_E_N1I * ENG_SLOT_WORDS, ld_soa(n1inv, cnt, L.i));
    if (L.valid && L.k == 0) flags[L.i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) fb[0] = 0;
  }
  asm volatile("" ::: "memory");
  eng_io io{nullptr, nullptr, nullptr, cnt};
  io.xbuf = xbuf;
  eng_exec<false, false, 2, true>(ENG_PROG_FEK + off, len, g, c, L, io);
  if (last) {
    const fp v = eng_ld(g + (ENG_E_R + L.k) * ENG_SLOT_WORDS);
    const bool ok = eng_eq_canon(v, L.k == 0 ? fp_one() : fp_zero());
    const uint64_t m = __ballot(ok);
    const bool all = ((m >> (12 * L.g)) & 0xFFFull) == 0xFFFull;
    const bool flagged = L.valid && flags[L.i];
    if (L.valid && L.k == 0 && !all && !flagged && status[r0 + L.i] == ST_OK) status[r0 + L.i] = ST_PAIRING;
    if (__ballot(flagged) != 0 && threadIdx.x == 0) fb[1 + atomicAdd(fb, 1u)] = blockIdx.x;
  }
}

// k_eng_fe_seg on 16-group 192-thread blocks (no idle lanes; see
// k_eng_miller_xw).  SLOTS: the group's LDS slots the segment needs (34 for
// the segments between the chains, 46 for the easy part and the last one;
// tools/gen_engine.py prog_fe_kb), so the in-between segments fit four blocks
// per CU.  The verdict vote of a group spanning waves goes through LDS; the
// fallback list names 5-round blocks (k_eng_fe_fb's unit), each once: by the
// first flagged item of the block.
template <int SLOTS>
__global__ void __launch_bounds__(ENG_XW_BLOCK, 3) k_eng_fe_seg_xw(int off, int len, bool first, bool last, size_t cnt,
                                                                size_t r0, const uint32_t* __restrict__ consts,
                                                                const uint32_t* __restrict__ fbuf,
                                                                const uint32_t* __restrict__ n1inv,
                                                                uint32_t* __restrict__ xbuf, uint8_t* __restrict__ flags,
                                                                uint32_t* __restrict__ fb, uint8_t* __restrict__ status) {
  static_assert(SLOTS <= ENG_SLOTS_FE, "segment slots");
  __shared__ uint32_t lds[(ENG_NCONST + ENG_XW_ITEMS * SLOTS) * ENG_SLOT_WORDS];
  __shared__ uint32_t vote[ENG_XW_ITEMS];
  uint32_t* c = lds;
  if (threadIdx.x < ENG_XW_ITEMS) vote[threadIdx.x] = 0;
  eng_load_consts(c, consts);
  int grp;
  const eng_lane L = eng_lane_xw(cnt, grp);
  uint32_t* g = lds + (ENG_NCONST + grp * SLOTS) * ENG_SLOT_WORDS;
  if (first) {
    eng_st(g + (ENG_E_F + L.k) * ENG_SLOT_WORDS, ld_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k)));
    if (L.k == 0) eng_st(g + ENG_E_N1I * ENG_SLOT_WORDS, ld_soa(n1inv, cnt, L.i));
    if (L.valid && L.k == 0) flags[L.i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) fb[0] = 0;
  }
  eng_sync<true>();
  eng_io io{nullptr, nullptr, nullptr, cnt};
  io.xbuf = xbuf;
  eng_exec<false, false, 2, true, true>(ENG_PROG_FEK + off, len, g, c, L, io);
  if (last) {
    const fp v = eng_ld(g + (ENG_E_R + L.k) * ENG_SLOT_WORDS);
    if (eng_eq_canon(v, L.k == 0 ? fp_one() : fp_zero())) atomicOr(&vote[grp], 1u << L.k);
    eng_sync<true>();
    const bool all = vote[grp] == 0xFFFu;
    const bool flagged = L.valid && flags[L.i];
    if (L.valid && L.k == 0 && !all && !flagged && status[r0 + L.i] == ST_OK) status[r0 + L.i] = ST_PAIRING;
    if (flagged && L.k == 0) {
      bool first_in_blk = true;
      for (int q = 1; q <= L.g; ++q) first_in_blk = first_in_blk && !flags[L.i - q];
      if (first_in_blk) fb[1 + atomicAdd(fb, 1u)] = (uint32_t)L.blk;
    }
  }
}

// The Granger-Scott fallback over the listed blocks (fb = [count, blocks...]).
constexpr unsigned ENG_FB_GRID = 64;
__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_fe_fb(size_t cnt, size_t r0, const uint32_t* __restrict__ consts,
                                                         uint32_t* __restrict__ fbuf,
                                                         const uint32_t* __restrict__ n1inv,
                                                         uint8_t* __restrict__ status,
                                                         const uint8_t* __restrict__ flags,
                                                         const uint32_t* __restrict__ fb) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_FE * ENG_SLOT_WORDS];
  const uint32_t n = fb[0];
  for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
    eng_fe_block(fb[1 + q], cnt, r0, consts, fbuf, n1inv, status, flags, lds);
    __syncthreads();
  }
}

static_assert(ENG_KB_COMP[0] == 2 && ENG_KB_COMP[3] == 5 && ENG_KB_COMP[4] == 8 && ENG_KB_COMP[7] == 11,
              "kb_comp: compressed coordinates f1, f2, f4, f5");
__device__ __forceinline__ int kb_comp(int k) { return k < 4 ? k + 2 : k + 4; }
__device__ __forceinline__ int kb_snap(int j) {
  static_assert(ENG_KB_NSNAP == 6 && ENG_KB_SNAP[0] == 16 && ENG_KB_SNAP[1] == 48 && ENG_KB_SNAP[2] == 57 &&
                    ENG_KB_SNAP[3] == 60 && ENG_KB_SNAP[4] == 62 && ENG_KB_SNAP[5] == 63,
                "kb_snap: the set bits of |x| below the top one");
  return j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
}

// The compressed chain of one exponentiation: 8 lanes per item (8 items per
// wave, all 64 lanes busy), lane k owning component kb_comp(k) of (f1, f2, f4,
// f5); 63 compressed squarings of m (plane M) with m^(2^s) stored to plane
// X0 + j after s = kb_snap(j) squarings.  LDS: 16 slots per item (state, LIN sums).
#ifndef DG_KB_CHAIN_OCC
#define DG_KB_CHAIN_OCC 3
#endif
__global__ void __launch_bounds__(64, DG_KB_CHAIN_OCC) k_eng_kb_chain(size_t cnt, uint32_t* __restrict__ xbuf) {
  __shared__ uint32_t lds[8 * ENG_KB_SLOTS * ENG_SLOT_WORDS];
  const int lane = threadIdx.x & 63, grp = lane >> 3, k = lane & 7;
  const size_t gi = (size_t)blockIdx.x * 8 + grp;
  const bool valid = gi < cnt;
  const size_t i = valid ? gi : cnt - 1;
  uint32_t* g = lds + grp * ENG_KB_SLOTS * ENG_SLOT_WORDS;
  const int comp = kb_comp(k);
  fp own = ld_blk(xbuf, kb_off(i, ENG_KB_PL_M, comp));
  eng_st(g + k * ENG_SLOT_WORDS, own);
  asm volatile("" ::: "memory");
  own = eng_cyc_fast<true, 8>(g, k, own);
  int s = 1;
#pragma unroll 1
  for (int j = 0; j < ENG_KB_NSNAP; ++j) {
    const int sj = kb_snap(j);
#pragma unroll 1
    for (; s < sj; ++s) own = eng_cyc_fast<false, 8>(g, k, own);
    if (valid) st_blk(xbuf, kb_off(i, ENG_KB_PL_X0 + j, comp), own);
  }
}

// Per item: the norms N_j = Norm(4 f1) of the six stored values, their
// product P -> pbuf ([limb][cnt]; k_eng_inv inverts it in place) and the
// excluded products E_j = prod_(k != j) N_k -> ebuf ([j][limb][cnt]), so
// that 1 / N_j = E_j / P.  A zero norm (f1 = 0) flags the item (unless it
// has already failed: its verdict stands); 1 stands in for it.  flag_every
// (test mode, DGPU_KB_TEST_FLAG): also flag every item i with
// i % flag_every == 0, so the fallback runs.
// PRE (DGPU_KB_NORM=chain): the chain already wrote the norms into ebuf's
// planes (k_kb_chain_thr<true>); each thread reads its six before writing E_j.
template <bool PRE>
__global__ void __launch_bounds__(256, 2) k_eng_kb_norm(size_t cnt, size_t r0, const uint32_t* __restrict__ xbuf,
                                                     uint32_t* __restrict__ pbuf, uint32_t* __restrict__ ebuf,
                                                     uint8_t* __restrict__ flags, const uint8_t* __restrict__ status,
                                                     size_t flag_every) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt) return;
  fp nrm[ENG_KB_NSNAP];
  bool zero = flag_every && i % flag_every == 0;
#pragma unroll
  for (int j = 0; j < ENG_KB_NSNAP; ++j) {
    if constexpr (PRE)
      nrm[j] = ld_soa(ebuf + (size_t)j * FP_LIMBS * cnt, cnt, i);
    else
      nrm[j] = eng_kb_norm(kb_ld2(xbuf, i, ENG_KB_PL_X0 + j, 2));
    if (fp_is_zero(nrm[j])) {
      nrm[j] = fp_one();
      zero = true;
    }
  }
  // prefixes into ebuf, then each E_j = prefix_(j-1) * suffix_(j+1)
  fp acc = nrm[0];
#pragma unroll
  for (int j = 1; j < ENG_KB_NSNAP; ++j) {
    st_soa(ebuf + (size_t)j * FP_LIMBS * cnt, cnt, i, acc);
    acc = fp_mul(acc, nrm[j]);
  }
  st_soa(pbuf, cnt, i, acc);
  acc = nrm[ENG_KB_NSNAP - 1];
#pragma unroll
  for (int j = ENG_KB_NSNAP - 2; j >= 0; --j) {
    const fp e = j ? fp_mul(ld_soa(ebuf + (size_t)j * FP_LIMBS * cnt, cnt, i), acc) : acc;
    st_soa(ebuf + (size_t)j * FP_LIMBS * cnt, cnt, i, e);
    acc = fp_mul(acc, nrm[j]);
  }
  if (zero && status[r0 + i] == ST_OK) flags[i] = 1;
}

// Decompression, one thread per stored value j of item i (element e = j cnt
// + i): 1 / N_j = E_j / P (ebuf, pbuf after k_eng_inv), then f0 and f3 of
// plane X0 + j (engine.cuh ENG_KB_DECOMPRESS).  Flagged items are skipped.
// 2 waves/SIMD (13 spilled VGPRs) measured faster than 1 (r03k: the FE's
// inversion + decompression stages 47.3 vs 60.9 ms per 2M rounds).
#ifndef DG_KB_DEC_OCC
#define DG_KB_DEC_OCC 2
#endif
__global__ void __launch_bounds__(256, DG_KB_DEC_OCC) k_eng_kb_dec(size_t cnt, uint32_t* __restrict__ xbuf,
                                                                   const uint32_t* __restrict__ pbuf,
                                                                   const uint32_t* __restrict__ ebuf,
                                                                   const uint8_t* __restrict__ flags) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)ENG_KB_NSNAP * cnt) return;
  const size_t j = e / cnt, i = e - j * cnt;
  if (flags[i]) return;
  const int pl = ENG_KB_PL_X0 + (int)j;
  const fp ninv = fp_mul(ld_soa(pbuf, cnt, i), ld_soa(ebuf + j * FP_LIMBS * cnt, cnt, i));
  fp2 f0, f3;
  ENG_KB_DECOMPRESS(kb_ld2(xbuf, i, pl, 2), kb_ld2(xbuf, i, pl, 4), kb_ld2(xbuf, i, pl, 8), kb_ld2(xbuf, i, pl, 10),
                    ninv, f0, f3);
  kb_st2(xbuf, i, pl, 0, f0);
  kb_st2(xbuf, i, pl, 6, f3);
}

}  // namespace dgpu

namespace dgpu {

// ---------------------------------------------------------------- k_eng_lines_fixed
// Signatures on G1: e(H_i, pk) e(-sig_i, g2) with both G2 arguments fixed per
// key.  `table` holds the LINES program's exports for (pk, g2) evaluated at
// P = (1, 1) (one item, blocked layout of block 0 / group 0; computed by
// dgpu_set_pubkey); every export is linear in its pair's -x_P (exports 2, 3)
// or y_P (4, 5), so item i's lines are the table scaled by P0 = H_i and
// P1 = -sig_i = (x_s, -y_s).  Grid: (blocks of 5 items) x ENG_LINE_STEPS, one
// thread per export; points are affine [x, y][limb][n].
__global__ void __launch_bounds__(64) k_eng_lines_fixed(size_t n, size_t r0, size_t cnt,
                                                        const uint32_t* __restrict__ h_pts,
                                                        const uint32_t* __restrict__ s_pts,
                                                        const uint32_t* __restrict__ table,
                                                        uint32_t* __restrict__ lines) {
  const int lane = threadIdx.x;
  if (lane >= ENG_WAVE_WORDS) return;
  const int g = lane / 12, e = lane % 12;
  const size_t i = (size_t)blockIdx.x * ENG_ROUNDS_PER_BLOCK + g;
  if (i >= cnt) return;
  const int step = blockIdx.y, pair = e / 6, k = e % 6;
  fp v = ld_blk(table, (size_t)step * FP_LIMBS * ENG_WAVE_WORDS + e);
  if (k >= 2) {
    const uint32_t* pts = pair ? s_pts : h_pts;
    const fp c = k < 4 ? fp_neg(ld_fp(pts, n, r0 + i)) : ld_fp(pts + FP_WORDS * n, n, r0 + i);
    v = fp_mul(v, (pair && k >= 4) ? fp_neg(c) : c);
  }
  st_blk(lines, (((size_t)blockIdx.x * ENG_LINE_STEPS + step) * FP_LIMBS) * ENG_WAVE_WORDS + lane, v);
}

// ---------------------------------------------------------------- k_eng_miller_fixed
// On-G1 Miller loop with the fixed-Q lines formed at each LDLINE from the
// per-key table (same scaling as k_eng_lines_fixed: export e = 6 pair + k,
// k in 2..3 scaled by -x, k in 4..5 by y of P0 = H_i / P1 = -sig_i), so the
// 45.7 KB/round line buffer is neither written nor read.
__global__ void __launch_bounds__(ENG_BLOCK, 3) k_eng_miller_fixed(size_t n, size_t r0, size_t cnt,
                                                                const uint32_t* __restrict__ consts,
                                                                const uint32_t* __restrict__ h_pts,
                                                                const uint32_t* __restrict__ s_pts,
                                                                const uint32_t* __restrict__ table,
                                                                uint32_t* __restrict__ fbuf,
                                                                uint32_t* __restrict__ n1) {
  __shared__ uint32_t lds[ENG_LDS_SLOTS_MILLER * ENG_SLOT_WORDS];
  uint32_t* c = lds;
  eng_load_consts(c, consts);
  const eng_lane L = eng_lane_id(cnt);
  uint32_t* g = lds + ENG_GBASE_MILLER[L.g] * ENG_SLOT_WORDS;
  eng_io io{nullptr, fbuf, n1, cnt};
  io.table = table;
  const int pair = L.k / 6, k = L.k % 6;
  io.scale = k >= 2;
  if (io.scale) {
    const uint32_t* pts = pair ? s_pts : h_pts;
    const fp cc = k < 4 ? fp_neg(ld_fp(pts, n, r0 + L.i)) : ld_fp(pts + FP_WORDS * n, n, r0 + L.i);
    io.mlt = (pair && k >= 4) ? fp_neg(cc) : cc;
  }
  eng_st(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS, L.k == 0 ? fp_one() : fp_zero());
  asm volatile("" ::: "memory");
  eng_exec<true, false, 1>(ENG_PROG_MILLER, ENG_PROG_MILLER_LEN, g, c, L, io);
  if (L.valid) st_blk(fbuf, eng_blk_off(L.blk, 2, 0, L.g, L.k), eng_ld(g + (ENG_M_F + L.k) * ENG_SLOT_WORDS));
}

}  // namespace dgpu
