// Batch kernels: one thread per beacon round.  Intermediate points live in
// HBM as structure-of-arrays ([limb][round], round fastest) so every limb
// load/store of a wavefront is one coalesced 256-byte access.
#pragma once
#include <hip/hip_runtime.h>
#include "h2c.cuh"

namespace dgpu {

constexpr int FP_WORDS = FP_LIMBS;          // 14 dwords per Fp in HBM
constexpr int G2A_WORDS = 4 * FP_WORDS;     // affine G2 point

__device__ __forceinline__ void st_fp(uint32_t* base, size_t n, size_t i, const fp& a) {
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) base[(size_t)k * n + i] = a.l[k];
}
__device__ __forceinline__ fp ld_fp(const uint32_t* base, size_t n, size_t i) {
  fp a;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) a.l[k] = base[(size_t)k * n + i];
  return a;
}
__device__ __forceinline__ void st_g2a(uint32_t* base, size_t n, size_t i, const g2a& p) {
  st_fp(base, n, i, p.x.c0);
  st_fp(base + FP_WORDS * n, n, i, p.x.c1);
  st_fp(base + 2 * FP_WORDS * n, n, i, p.y.c0);
  st_fp(base + 3 * FP_WORDS * n, n, i, p.y.c1);
}
__device__ __forceinline__ g2a ld_g2a(const uint32_t* base, size_t n, size_t i) {
  g2a p;
  p.x.c0 = ld_fp(base, n, i);
  p.x.c1 = ld_fp(base + FP_WORDS * n, n, i);
  p.y.c0 = ld_fp(base + 2 * FP_WORDS * n, n, i);
  p.y.c1 = ld_fp(base + 3 * FP_WORDS * n, n, i);
  return p;
}

constexpr int G2J_WORDS = 6 * FP_WORDS;

__device__ __forceinline__ void st_g2j(uint32_t* base, size_t n, size_t i, const g2j& p) {
  st_fp(base, n, i, p.x.c0);
  st_fp(base + FP_WORDS * n, n, i, p.x.c1);
  st_fp(base + 2 * FP_WORDS * n, n, i, p.y.c0);
  st_fp(base + 3 * FP_WORDS * n, n, i, p.y.c1);
  st_fp(base + 4 * FP_WORDS * n, n, i, p.z.c0);
  st_fp(base + 5 * FP_WORDS * n, n, i, p.z.c1);
}
__device__ __forceinline__ g2j ld_g2j(const uint32_t* base, size_t n, size_t i) {
  g2j p;
  p.x.c0 = ld_fp(base, n, i);
  p.x.c1 = ld_fp(base + FP_WORDS * n, n, i);
  p.y.c0 = ld_fp(base + 2 * FP_WORDS * n, n, i);
  p.y.c1 = ld_fp(base + 3 * FP_WORDS * n, n, i);
  p.z.c0 = ld_fp(base + 4 * FP_WORDS * n, n, i);
  p.z.c1 = ld_fp(base + 5 * FP_WORDS * n, n, i);
  return p;
}

// Test hook of the A/B build (DGPU_TEST_FORCE_EXC=1 at dgpu_open): the fast
// group-law paths (cofactor ladder, membership ladder, MSM additions) take
// their generic redo as if an exceptional addition had occurred, so the redo
// code runs on every item.  Always false in the shipped build.
#ifdef DG_AB_KNOBS
__device__ int g_dg_force_exc = 0;
#define DG_FORCE_EXC (g_dg_force_exc != 0)
#else
#define DG_FORCE_EXC false
#endif

// per-round status codes carried between kernels (also the public `reason`)
enum : uint8_t {
  ST_OK = 0,
  ST_DECODE = 1,    // wrong length / flags / x >= p / not on curve / non-canonical infinity
  ST_SUBGROUP = 2,  // point not in the r-order subgroup
  ST_PAIRING = 3,   // e(pk, H(m)) != e(g1, sig)
  ST_INFINITY = 4,  // signature is the point at infinity (pairing check fails)
};

struct g1_key {  // public key prepared for line evaluation: (-x, y), Montgomery
  fp neg_x, y;
};

// Where a batch item's message comes from: drand's DigestMessage of a beacon
// record (chain/verify.go:24-32: SHA-256(prev || BE64(round)), prev ignored
// unless chained), or raw message bytes (msgs != nullptr: key.Scheme.
// VerifyRecovered(pk, msg, sig) with any msg, key/curve.go:36-39,
// chain/beacon/chain.go:165).  A record whose length exceeds its stride
// (prev_len > prev_stride, msg_len > msg_stride) is never read past the
// stride and fails verification (msg_bad_record -> ST_DECODE).
struct msg_src {
  const uint64_t* rounds;
  const uint8_t* prev;
  size_t prev_stride;
  const uint32_t* prev_len;
  int chained;
  const uint8_t* msgs;
  size_t msg_stride;
  const uint32_t* msg_len;
};

__device__ __forceinline__ uint32_t clamp_len(uint32_t len, size_t stride) {
  return (size_t)len > stride ? (uint32_t)stride : len;
}

__device__ __forceinline__ bool msg_bad_record(const msg_src& m, size_t i) {
  if (m.msgs) return (size_t)m.msg_len[i] > m.msg_stride;
  return m.chained && (size_t)m.prev_len[i] > m.prev_stride;
}

// drand digest of a beacon record (32 bytes as 8 big-endian words)
__device__ __forceinline__ void msg_digest(const msg_src& m, size_t i, uint32_t msg[8]) {
  const uint32_t plen = m.chained ? clamp_len(m.prev_len[i], m.prev_stride) : 0u;
  drand_digest(msg, m.chained ? m.prev + i * m.prev_stride : nullptr, plen, m.rounds[i]);
}

// expand_message_xmd of item i's message under DST G1DST with ELL 32-byte blocks
template <bool G1DST, int ELL>
__device__ __forceinline__ void msg_expand(const msg_src& m, size_t i, uint32_t* uni) {
  if (m.msgs) {
    expand_xmd_var<G1DST, ELL>(uni, m.msgs + i * m.msg_stride, clamp_len(m.msg_len[i], m.msg_stride));
  } else {
    uint32_t msg[8];
    msg_digest(m, i, msg);
    expand_xmd<G1DST, ELL>(uni, msg);
  }
}

// ---------------------------------------------------------------- kernels
// The per-round hash to G2 as three launches (the fused kernel needs 512
// registers per lane -- one wave per SIMD -- and 6 KB of scratch; each stage
// alone is far lighter, and the SSWU stage has 2n independent items):
//   k_h2c_field   message (DigestMessage or raw) + expand_message_xmd -> u0, u1 ([4 fp][n])
//   k_h2c_sswu    SSWU + 3-isogeny of each of the 2n field elements -> Jacobian ([2][6 fp][n])
//   k_h2c_finish  Q0 + Q1, cofactor clearing -> X, Y (h_out) and Z (z_out)
__global__ void __launch_bounds__(256) k_h2c_field(size_t n, msg_src m, uint32_t* __restrict__ u_out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t uni[64];
  msg_expand<false, 8>(m, i, uni);
#pragma unroll 1
  for (int k = 0; k < 4; ++k) st_fp(u_out + (size_t)k * FP_WORDS * n, n, i, fp_from_be64_words(uni + 16 * k));
}

// Minimum blocks per CU of the two heavy hash kernels (A/B knobs).
#ifndef DG_SSWU_OCC
#define DG_SSWU_OCC 2
#endif
#ifndef DG_FINISH_OCC
#define DG_FINISH_OCC 2
#endif
__global__ void __launch_bounds__(256, DG_SSWU_OCC) k_h2c_sswu(size_t n, const uint32_t* __restrict__ u,
                                                   uint32_t* __restrict__ q_out) {
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const size_t which = j / n, i = j % n;
  const uint32_t* ub = u + which * 2 * FP_WORDS * n;
  const fp2 uu{ld_fp(ub, n, i), ld_fp(ub + FP_WORDS * n, n, i)};
  st_g2j(q_out + which * G2J_WORDS * n, n, i, map_to_curve_sswu_iso3_body(uu));
}

// A/B (-DDG_SSWU_STAGED, capi.hip launch_sswu; measured slower in the bulk
// pass, r06i): the SSWU stage in five launches, the two exponentiations of
// each item (~85% of its products) alone in k_fp_pow_planes, whose 90 VGPRs
// let 5 waves share a SIMD, where the fused k_h2c_sswu holds 256 VGPRs (2
// waves).  In isolation the out-of-line Fp calls issue ~1.3x faster at 5-8
// waves than at 2 (`tools/engbench/powprobe.hip`, profiles/r06/
// r06h_powprobe.json); in the pass that did not carry over.  Item j of 2n
// (which = j / n, i = j % n):
//   k_sswu_a   u -> N, D, w into the item's q slot (x, y, z words), Norm(w) -> plane 3 which
//   pow        plane 3 which: alpha -> g = alpha^((p+1)/4)
//   k_sswu_b   square test (x2 if not), N, w updated in the slot; d -> plane 3 which + 1,
//              dm4 -> plane 3 which + 2
//   pow        plane 3 which + 2: dm4 -> t = dm4^((p-3)/4)
//   k_sswu_c   y, sign, 3-isogeny -> the Jacobian point over the slot (k_h2c_sswu's output)
// The arithmetic is map_to_curve_sswu_iso3_body's, stage by stage (h2c.cuh).
struct sswu_planes {
  uint32_t* p[6];  // [3 which + k]: FP_WORDS x n words each
};
__global__ void __launch_bounds__(256, 2) k_sswu_a(size_t n, const uint32_t* __restrict__ u, uint32_t* __restrict__ q,
                                                sswu_planes aux) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const size_t which = j / n, i = j % n;
  const uint32_t* ub = u + which * 2 * FP_WORDS * n;
  fp2 N, D, w;
  sswu_pre(fp2{ld_fp(ub, n, i), ld_fp(ub + FP_WORDS * n, n, i)}, N, D, w);
  st_g2j(q + which * G2J_WORDS * n, n, i, g2j{N, D, w});
  st_fp(aux.p[3 * which], n, i, fp2_norm(w));
}
template <int E>
__global__ void __launch_bounds__(256) k_fp_pow_planes(size_t n, sswu_planes aux, int k) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const size_t which = j / n, i = j % n;
  uint32_t* pl = aux.p[3 * which + k];
  const fp a = ld_fp(pl, n, i);
  st_fp(pl, n, i, E == 0 ? fp_sqrt_cand(a) : DG_POW(a, EXP_P_MINUS_3_DIV_4));
}
__global__ void __launch_bounds__(256, 2) k_sswu_b(size_t n, const uint32_t* __restrict__ u, uint32_t* __restrict__ q,
                                                sswu_planes aux) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const size_t which = j / n, i = j % n;
  const uint32_t* ub = u + which * 2 * FP_WORDS * n;
  uint32_t* qs = q + which * G2J_WORDS * n;
  const g2j s = ld_g2j(qs, n, i);
  fp2 N = s.x, w = s.z;
  fp dm4;
  const fp2 uu{ld_fp(ub, n, i), ld_fp(ub + FP_WORDS * n, n, i)};
  const fp d = sswu_mid(uu, sswu_zu2(uu), fp2_norm(w), N, s.y, w, ld_fp(aux.p[3 * which], n, i), dm4);
  st_g2j(qs, n, i, g2j{N, s.y, w});
  st_fp(aux.p[3 * which + 1], n, i, d);
  st_fp(aux.p[3 * which + 2], n, i, dm4);
}
__global__ void __launch_bounds__(256, DG_SSWU_OCC) k_sswu_c(size_t n, const uint32_t* __restrict__ u,
                                                             uint32_t* __restrict__ q, sswu_planes aux) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const size_t which = j / n, i = j % n;
  const uint32_t* ub = u + which * 2 * FP_WORDS * n;
  uint32_t* qs = q + which * G2J_WORDS * n;
  const g2j s = ld_g2j(qs, n, i);
  const fp d = ld_fp(aux.p[3 * which + 1], n, i);
  const fp m2 = fp_sqr(fp2_norm(s.y));  // dm4 = d Norm(D)^4 again, as fp2_sqrt_scaled_pre forms it
  const fp dm4 = fp_mul(d, fp_sqr(m2));
  st_g2j(qs, n, i, sswu_post(fp2{ld_fp(ub, n, i), ld_fp(ub + FP_WORDS * n, n, i)}, s.x, s.y, s.z, d, dm4,
                             ld_fp(aux.p[3 * which + 2], n, i)));
}

// An affine point at item i of an SoA array ([x.c0, x.c1, y.c0, y.c1][limb][n]),
// each coordinate loaded where the ladder uses it (the base passes through an
// empty asm per fetch so the loads stay in the loop instead of being hoisted
// and spilled).
struct g2a_soa_fetch {
  const uint32_t* base;
  size_t n, i;
  __device__ __forceinline__ const uint32_t* b() const {
    const uint32_t* p = base;
    __asm__ volatile("" : "+s"(p));
    return p;
  }
  __device__ __forceinline__ fp2 x() const {
    const uint32_t* p = b();
    return fp2{ld_fp(p, n, i), ld_fp(p + FP_WORDS * n, n, i)};
  }
  __device__ __forceinline__ fp2 y() const {
    const uint32_t* p = b();
    return fp2{ld_fp(p + 2 * FP_WORDS * n, n, i), ld_fp(p + 3 * FP_WORDS * n, n, i)};
  }
  __device__ __forceinline__ g2a get() const { return g2a{x(), y()}; }
};
// G2 membership of a decoded signature p, stored first at item i of pts (its
// output slot): the ladder form, the generic test on an exceptional addition.
__device__ __forceinline__ bool g2_in_subgroup_stored(const g2a& p, uint32_t* pts, size_t n, size_t i) {
  st_g2a(pts, n, i, p);
#ifdef DG_SUBGROUP_GENERIC  // A/B: rounds 1-5, g2_in_subgroup with the point in registers
  return g2_in_subgroup(g2_from_affine(p));
#endif
  bool exc = false;
  const g2a_soa_fetch f{pts, n, i};
  const bool in = g2_in_subgroup_ladder(p, f, exc);
  return exc || DG_FORCE_EXC ? g2_in_subgroup(g2_from_affine(f.get())) : in;
}

// Point slots of g2_clear_cofactor_stash in the round's own SoA words: 0, 1 =
// the two SSWU outputs' slots of q (each read once, before it is written),
// 2 = the output slot (X, Y in h_out, Z in z_out).
struct h2c_finish_stash {
  uint32_t* q;
  uint32_t* h_out;
  uint32_t* z_out;
  size_t n, i;
  __device__ __forceinline__ void put(int k, const g2j& p) {
    if (k < 2) {
      st_g2j(q + (size_t)k * G2J_WORDS * n, n, i, p);
    } else {
      st_g2a(h_out, n, i, g2a{p.x, p.y});
      st_fp(z_out, n, i, p.z.c0);
      st_fp(z_out + FP_WORDS * n, n, i, p.z.c1);
    }
  }
  struct fetch {  // slot k's coordinates, each loaded where g2_add_nx_q uses it
    const uint32_t* xy;
    const uint32_t* zp;
    size_t n, i;
    __device__ __forceinline__ fp2 x() const { return fp2{ld_fp(xy, n, i), ld_fp(xy + FP_WORDS * n, n, i)}; }
    __device__ __forceinline__ fp2 y() const {
      return fp2{ld_fp(xy + 2 * FP_WORDS * n, n, i), ld_fp(xy + 3 * FP_WORDS * n, n, i)};
    }
    __device__ __forceinline__ fp2 z() const { return fp2{ld_fp(zp, n, i), ld_fp(zp + FP_WORDS * n, n, i)}; }
  };
  // (the bases pass through an empty asm: the slot is re-read at each
  // addition instead of hoisted out of the ladder and spilled)
  __device__ __forceinline__ fetch at(int k) const {
    const uint32_t* qb = q;
    const uint32_t* hb = h_out;
    const uint32_t* zb = z_out;
#ifdef __HIP_DEVICE_COMPILE__
    __asm__ volatile("" : "+s"(qb), "+s"(hb), "+s"(zb));
#endif
    const uint32_t* xy = k < 2 ? qb + (size_t)k * G2J_WORDS * n : hb;
    return fetch{xy, k < 2 ? xy + 4 * FP_WORDS * n : zb, n, i};
  }
  __device__ __forceinline__ g2j get(int k) const {
    if (k < 2) return ld_g2j(q + (size_t)k * G2J_WORDS * n, n, i);
    const g2a a = ld_g2a(h_out, n, i);
    return g2j{a.x, a.y, fp2{ld_fp(z_out, n, i), ld_fp(z_out + FP_WORDS * n, n, i)}};
  }
};

// Q0 + Q1 and the cofactor clearing, its cold points parked in HBM (one
// point live per [|x|] ladder, no call sites in the loops; VERDICT r05 item
// 3).  An exceptional addition on the fast path (Q0 = +-Q1, a small-order
// point, ...) redoes the round with the generic g2_clear_cofactor from P,
// which slot 0 still holds.  Overwrites q.
__global__ void __launch_bounds__(256, DG_FINISH_OCC) k_h2c_finish(size_t n, uint32_t* __restrict__ q,
                                                     uint32_t* __restrict__ h_out, uint32_t* __restrict__ z_out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
#ifdef DG_FINISH_INL  // A/B: rounds 1-5, the whole ladder in registers (4 KB of scratch per lane)
  const g2j hh = g2_clear_cofactor_inl(g2_add_body(ld_g2j(q, n, i), ld_g2j(q + G2J_WORDS * n, n, i)));
  st_g2a(h_out, n, i, g2a{hh.x, hh.y});
  st_fp(z_out, n, i, hh.z.c0);
  st_fp(z_out + FP_WORDS * n, n, i, hh.z.c1);
  return;
#endif
  h2c_finish_stash st{q, h_out, z_out, n, i};
  bool exc = false;
  g2j h = g2_clear_cofactor_stash(ld_g2j(q, n, i), ld_g2j(q + G2J_WORDS * n, n, i), st, exc);
  if (exc || DG_FORCE_EXC) h = DG_FORCE_EXC ? g2_clear_cofactor_generic(st.get(0)) : g2_clear_cofactor(st.get(0));
  st.put(2, h);
}

// RLC mode's pre-cofactor hash point R = Q0 + Q1 (Jacobian, [6 fp][n]) from
// k_h2c_sswu's output: the cofactor is cleared once per checked tree node.
__global__ void __launch_bounds__(256, 2) k_h2c_sum(size_t n, const uint32_t* __restrict__ q,
                                                  uint32_t* __restrict__ r_out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_g2j(r_out, n, i, g2_add_body(ld_g2j(q, n, i), ld_g2j(q + G2J_WORDS * n, n, i)));
}

// Jacobian -> affine for n G2 points in place (X, Y in pts; Z in z) with one
// Fp inversion per thread: thread t takes points t, t + T, ... (T threads in
// the grid) and inverts the norms N(Z_i) by Montgomery's trick (prefix
// products in `pre`); 1/Z = conj(Z) / N(Z).  Z = 0 (the identity) gives (0, 0)
// like g2_to_affine.
__global__ void __launch_bounds__(256) k_g2_batch_affine(size_t n, uint32_t* __restrict__ pts,
                                                         const uint32_t* __restrict__ z, uint32_t* __restrict__ pre) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  auto ldz = [&](size_t i) { return fp2{ld_fp(z, n, i), ld_fp(z + FP_WORDS * n, n, i)}; };
  fp acc = fp_one();
  size_t last = t;
  for (size_t i = t; i < n; i += T) {
    const fp nz = fp2_norm(ldz(i));
    acc = fp_mul(acc, fp_cmov(nz, fp_one(), fp_is_zero(nz)));
    st_fp(pre, n, i, acc);
    last = i;
  }
  fp inv = fp_inv(acc);
  for (size_t i = last;; i -= T) {
    const fp2 zi = ldz(i);
    const fp nz = fp2_norm(zi);
    const bool inf = fp_is_zero(nz);
    const fp ninv = i >= t + T ? fp_mul(inv, ld_fp(pre, n, i - T)) : inv;  // 1 / N(Z_i)
    const fp2 zinv = fp2_mul_fp(fp2_conj(zi), ninv);
    const fp2 zinv2 = fp2_sqr(zinv);
    g2a a = ld_g2a(pts, n, i);
    a.x = fp2_mul(a.x, zinv2);
    a.y = fp2_mul(a.y, fp2_mul(zinv2, zinv));
    st_g2a(pts, n, i, inf ? g2a{fp2_zero(), fp2_zero()} : a);
    if (i < t + T) break;
    if (!inf) inv = fp_mul(inv, nz);
  }
}

// H(m) for raw messages of any length, compressed (parity surface:
// dgpu_hash_to_g2 / dgpu_hash_to_curve)
__global__ void __launch_bounds__(256) k_hash_to_g2_msgs(size_t n, msg_src m, uint8_t* __restrict__ out96) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t uni[64];
  msg_expand<false, 8>(m, i, uni);
  const fp2 u0{fp_from_be64_words(uni), fp_from_be64_words(uni + 16)};
  const fp2 u1{fp_from_be64_words(uni + 32), fp_from_be64_words(uni + 48)};
  g2j h = g2_clear_cofactor(g2_add(map_to_curve_sswu_iso3(u0), map_to_curve_sswu_iso3(u1)));
  bool inf = g2_is_inf(h);
  g2a a = inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(h);
  g2_compress(out96 + i * 96, a, inf);
}

// drand digests only (parity/debug: dgpu_digest)
__global__ void __launch_bounds__(256) k_digest(size_t n, const uint64_t* __restrict__ rounds,
                                                 const uint8_t* __restrict__ prev, size_t prev_stride,
                                                 const uint32_t* __restrict__ prev_len, int chained,
                                                 uint8_t* __restrict__ out32) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8];
  drand_digest(msg, chained ? prev + i * prev_stride : nullptr, chained ? prev_len[i] : 0u, rounds[i]);
  for (int w = 0; w < 8; ++w) {
    out32[i * 32 + 4 * w] = (uint8_t)(msg[w] >> 24);
    out32[i * 32 + 4 * w + 1] = (uint8_t)(msg[w] >> 16);
    out32[i * 32 + 4 * w + 2] = (uint8_t)(msg[w] >> 8);
    out32[i * 32 + 4 * w + 3] = (uint8_t)msg[w];
  }
}

// Signature decode (kilic G2.FromCompressed semantics (R)) + G2 membership.
// A record whose message part overruns its stride (msg_bad_record) fails as a
// decode error without its signature being read.  check_subgroup = 0: the
// membership test is left to the pairing engine's lines kernel (the Miller
// loop's ladder of the signature gives [x] sig for free, k_eng_lines).
__global__ void __launch_bounds__(256, 4) k_decode_g2_sigs(size_t n, const uint8_t* __restrict__ sigs, size_t sig_stride,
                                                         const uint32_t* __restrict__ sig_len, msg_src m,
                                                         int check_subgroup, uint32_t* __restrict__ sig_out,
                                                         uint8_t* __restrict__ status) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st;
  g2a p{fp2_zero(), fp2_zero()};
  if (sig_len[i] != 96 || msg_bad_record(m, i)) {
    st = ST_DECODE;
  } else {
    uint8_t buf[96];
    const uint8_t* src = sigs + i * sig_stride;
    for (int k = 0; k < 96; ++k) buf[k] = src[k];
    int rc = g2_decompress(&p, buf, check_subgroup != 0);
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  }
  st_g2a(sig_out, n, i, p);
  status[i] = st;
}

// The same decode with the G2 membership check (RLC mode and recovery need
// it up front; DGPU_SUBGROUP=decode): the 63-doubling ladder inlined into
// the kernel at 2 waves/SIMD -- out of line in g2_decompress its registers
// escaped the kernel's budget (4.6 KB of scratch at 4 waves/SIMD): 389.6 ->
// 360.2 ms per 10M (tools/engbench/dec_g2.hip, profiles/r04/r04f_dec_g2_variants.txt).
__global__ void __launch_bounds__(256, 2) k_decode_g2_sigs_sub(size_t n, const uint8_t* __restrict__ sigs,
                                                             size_t sig_stride, const uint32_t* __restrict__ sig_len,
                                                             msg_src m, uint32_t* __restrict__ sig_out,
                                                             uint8_t* __restrict__ status) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st;
  g2a p{fp2_zero(), fp2_zero()};
  if (sig_len[i] != 96 || msg_bad_record(m, i)) {
    st = ST_DECODE;
    st_g2a(sig_out, n, i, p);
  } else {
    uint8_t buf[96];
    const uint8_t* src = sigs + i * sig_stride;
    for (int k = 0; k < 96; ++k) buf[k] = src[k];
    int rc = g2_decompress(&p, buf, false);
    if (rc == DEC_OK) {  // p is stored by the membership test (not kept live across its ladder)
      if (!g2_in_subgroup_stored(p, sig_out, n, i)) rc = DEC_ERR_SUBGROUP;
    } else {
      st_g2a(sig_out, n, i, p);
    }
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  }
  status[i] = st;
}

// Synthetic-chain generator (test-data tool, not the verify path): one step
// of S independent chained segments, following the reference's fixture
// generator client/test/result/mock/result.go:86-130 (msg = DigestMessage,
// sig = sk * H(msg), previous = sig).  Segment s signs round first_round[s] + step
// over prev (prev_len[s] bytes at prev + s*96) and writes the 96-byte
// signature to sig_out + s*96 and to prev (for the next step).
struct scalar256 {
  uint32_t w[8];
};
__global__ void __launch_bounds__(256) k_sign_step(size_t S, const uint64_t* __restrict__ first_round, uint64_t step,
                                                    uint8_t* __restrict__ prev, uint32_t* __restrict__ prev_len,
                                                    int chained, scalar256 sk, uint8_t* __restrict__ sig_out,
                                                    size_t sig_stride) {
  size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  uint32_t msg[8];
  uint8_t pb[96];
  uint32_t plen = chained ? prev_len[s] : 0u;
  for (uint32_t k = 0; k < plen && k < 96; ++k) pb[k] = prev[s * 96 + k];
  drand_digest(msg, pb, plen, first_round[s] + step);
  g2j h = hash_to_g2(msg);
  g2j sg = g2_mul_words(h, sk.w, 8);
  bool inf = g2_is_inf(sg);
  g2a a = inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(sg);
  uint8_t out[96];
  g2_compress(out, a, inf);
  for (int k = 0; k < 96; ++k) {
    sig_out[s * sig_stride + k] = out[k];
    prev[s * 96 + k] = out[k];
  }
  prev_len[s] = 96;
}

// pk = sk * g1, compressed (synthetic-chain tool)
__global__ void k_derive_pubkey(scalar256 sk, uint8_t* __restrict__ out48) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  g1j g{C_G1_X, C_G1_Y, fp_one()};
  g1j p = g1_mul_words(g, sk.w, 8);
  bool inf = g1_is_inf(p);
  g1a a = inf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(p);
  uint8_t out[48];
  g1_compress(out, a, inf);
  for (int k = 0; k < 48; ++k) out48[k] = out[k];
}

// ================================================================ RLC batching
// Shared-key collapse of the random linear combination:
//   prod_i d_i^{r_i} = e(pk, h_eff * sum_i r_i R_i) * e(-g1, sum_i r_i sig_i),
// with R_i the pre-cofactor hash point (h_eff applied once per checked node,
// by linearity) and d_i = e(pk, H_i) e(-g1, sig_i).  Jacobian G2 arrays are
// SoA [6 Fp][limb][index].
// SplitMix64-derived nonzero 64-bit coefficient for batch position `idx`
// under `seed`.  Keyed on the position, never on the record's Round field:
// two records with equal Round (duplicated store rows) must get independent
// coefficients, or a +D / -D pair of corruptions cancels in every node.
__device__ __forceinline__ uint64_t rlc_coeff(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z ? z : 1ull;
}

// Node status of a trivially passing candidate (both points at infinity;
// rlc_msm.cuh k_rlc_prep).
constexpr uint8_t RLC_TRIVIAL = 0x80;

// Engine verdicts of the candidates -> fail flags.
__global__ void __launch_bounds__(256) k_rlc_fail(size_t n_cand, const uint8_t* __restrict__ st,
                                                  uint8_t* __restrict__ fail) {
  size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cand) return;
  fail[c] = (st[c] == ST_OK || st[c] == RLC_TRIVIAL) ? 0 : 1;
}

// Mark the rounds of failing leaves.
__global__ void k_rlc_mark(size_t n_cand, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ fail,
                           uint8_t* __restrict__ status) {
  size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cand) return;
  if (fail[c]) status[idx[c]] = ST_PAIRING;
}

// status -> verdict bitmap (bit = 1 valid), one thread per output byte
__global__ void k_pack_verdicts(size_t n, const uint8_t* __restrict__ status, uint8_t* __restrict__ bits) {
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j * 8 >= n) return;
  uint8_t b = 0;
  for (int k = 0; k < 8; ++k) {
    size_t i = j * 8 + k;
    if (i < n && status[i] == ST_OK) b |= (uint8_t)(1u << k);
  }
  bits[j] = b;
}

// nonzero bytes -> bitmap (bit = 1 where ok[i] != 0): recovery verdicts
__global__ void k_pack_ok(size_t n, const uint8_t* __restrict__ ok, uint8_t* __restrict__ bits) {
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j * 8 >= n) return;
  uint8_t b = 0;
  for (int k = 0; k < 8; ++k) {
    size_t i = j * 8 + k;
    if (i < n && ok[i]) b |= (uint8_t)(1u << k);
  }
  bits[j] = b;
}

// Public key decode (48-byte compressed G1, kilic G1.FromCompressed (R)) on one thread.
__global__ void k_decode_g1_pk(const uint8_t* __restrict__ in48, uint32_t* __restrict__ out, int* __restrict__ rc) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint8_t buf[48];
  for (int k = 0; k < 48; ++k) buf[k] = in48[k];
  g1a p{fp_zero(), fp_zero()};
  int r = g1_decompress(&p, buf, GROUP_ORDER_WORDS);
  fp nx = fp_neg(p.x);
  for (int k = 0; k < FP_LIMBS; ++k) {
    out[k] = nx.l[k];
    out[FP_LIMBS + k] = p.y.l[k];
  }
  *rc = r;
}

// Decoded points (SoA, nfp Fp coordinates of stride n, Montgomery) -> canonical
// big-endian 48-byte coordinates, item-major: out + (i nfp + j) 48.  neg_first:
// coordinate 0 is stored negated (k_decode_g1_pk's (-x, y)).  The decode
// entry points' readout (dgpu_decode_signatures / dgpu_decode_pubkey).
__global__ void __launch_bounds__(256) k_fp_soa_to_be48(size_t n, int nfp, const uint32_t* __restrict__ pts,
                                                        int neg_first, uint8_t* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (size_t)nfp) return;
  const size_t i = t / (size_t)nfp;
  const int j = (int)(t - i * (size_t)nfp);
  fp v = ld_fp(pts + (size_t)j * FP_WORDS * n, n, i);
  if (neg_first && j == 0) v = fp_neg(v);
  fp_std_to_be48(fp_from_mont(v), out + t * 48);
}

}  // namespace dgpu
