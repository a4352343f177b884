// RLC root by bucket MSM (Pippenger), configs[2]: the whole batch's
// random-linear-combination root
//   P = sum_i r_i R_i,   S = sum_i r_i sig_i      (r_i = a_i + b_i x, kernels.cuh rlc_coeff)
// without a per-point scalar multiplication.  With the psi split of the
// leaves (P = sum a_i R_i + psi(sum b_i R_i), psi a group endomorphism of E')
// the root is four MSMs with 32-bit scalars over the batch's affine points,
// each in two 16-bit windows: every (MSM, window, digit) is a bucket, so a
// point costs one mixed addition per MSM and window -- 8 per round instead
// of the two window ladders of k_rlc_leaves (~32 doublings + 16 additions
// each).  The tree of leaves is built only when this root fails
// (capi.hip verify_status_locked).
//
// Pipeline (one launch each; the bucket order is a counting sort, so the
// sums do not depend on the order the atomics hand out positions -- point
// addition is associative and commutative, the results are exact):
//   k_msm_aos     R_i, sig_i affine SoA -> AoS (224 B per point: gathers
//                 read two cache lines instead of 56) + usable flags
//   k_msm_count   bucket sizes (atomics)
//   k_msm_scan    exclusive prefix sums (one block)
//   k_msm_scatter point indices into their buckets (atomics on cursors)
//   k_msm_bucket  one thread per bucket: sum of its points (mixed additions)
//   k_msm_window  one thread per run of 64 buckets: sum_k k B_k of the run
//   k_g2_sum_level  pairwise tree over the runs of each (MSM, window)
//   k_msm_root    MSM_m = W_m0 + 2^16 W_m1; P = MSM_0 + psi(MSM_1), S = MSM_2 + psi(MSM_3)
#pragma once
#include "kernels.cuh"

namespace dgpu {

constexpr int MSM_C = 16;                         // window bits
constexpr int MSM_BUCKETS = 1 << MSM_C;           // per (MSM, window); digit 0 unused
constexpr int MSM_MW = 8;                         // 4 MSMs x 2 windows
constexpr size_t MSM_KEYS = (size_t)MSM_MW * MSM_BUCKETS;
constexpr int MSM_RUN = 64;                       // buckets per k_msm_window thread
constexpr int MSM_RUNS = MSM_BUCKETS / MSM_RUN;   // runs per (MSM, window)
constexpr int MSM_AOS_WORDS = G2A_WORDS;          // 56 words per affine point

__device__ __forceinline__ g2a ld_aos(const uint32_t* __restrict__ base, size_t i) {
  const uint32_t* p = base + i * MSM_AOS_WORDS;
  g2a a;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) {
    a.x.c0.l[l] = p[l];
    a.x.c1.l[l] = p[FP_LIMBS + l];
    a.y.c0.l[l] = p[2 * FP_LIMBS + l];
    a.y.c1.l[l] = p[3 * FP_LIMBS + l];
  }
  return a;
}

// R (affine SoA in r_aff, (0, 0) = identity) and sig (affine SoA) -> AoS
// [R | sig][i]; flags[i]: bit 0 R usable, bit 1 sig usable (status ST_OK and
// not the identity; the leaves kernel skips the same points).
__global__ void __launch_bounds__(256) k_msm_aos(size_t n, const uint32_t* __restrict__ r_aff,
                                                 const uint32_t* __restrict__ sig_pts,
                                                 const uint8_t* __restrict__ status, uint32_t* __restrict__ aos,
                                                 uint8_t* __restrict__ flags) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t f = 0;
  for (int which = 0; which < 2; ++which) {
    const g2a q = ld_g2a(which ? sig_pts : r_aff, n, i);
    uint32_t* o = aos + ((size_t)which * n + i) * MSM_AOS_WORDS;
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) {
      o[l] = q.x.c0.l[l];
      o[FP_LIMBS + l] = q.x.c1.l[l];
      o[2 * FP_LIMBS + l] = q.y.c0.l[l];
      o[3 * FP_LIMBS + l] = q.y.c1.l[l];
    }
    if (status[i] == ST_OK && !(fp2_is_zero(q.x) && fp2_is_zero(q.y))) f |= (uint8_t)(1u << which);
  }
  flags[i] = f;
}

// bucket of point i in (MSM m, window w), or -1: m = 0 a R, 1 b R, 2 a sig, 3 b sig
__device__ __forceinline__ int msm_bucket(uint64_t z, uint8_t flags, int m, int w) {
  if (!((flags >> (m >> 1)) & 1)) return -1;
  const uint32_t k = (m & 1) ? (uint32_t)(z >> 32) : (uint32_t)z;
  const uint32_t d = (k >> (MSM_C * w)) & (MSM_BUCKETS - 1);
  return d ? (int)(((uint32_t)(m * 2 + w) << MSM_C) | d) : -1;
}

__global__ void __launch_bounds__(256) k_msm_count(size_t n, uint64_t seed, const uint8_t* __restrict__ flags,
                                                   uint32_t* __restrict__ counts) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t z = rlc_coeff(seed, i);
  const uint8_t f = flags[i];
#pragma unroll
  for (int mw = 0; mw < MSM_MW; ++mw) {
    const int b = msm_bucket(z, f, mw >> 1, mw & 1);
    if (b >= 0) atomicAdd(counts + b, 1u);
  }
}

// exclusive prefix sums of MSM_KEYS counts -> offsets (and a cursor copy);
// one block of 1024 threads, 512 consecutive buckets each
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t* __restrict__ counts, uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  constexpr int PER = (int)(MSM_KEYS / 1024);
  const size_t b0 = (size_t)t * PER;
  uint32_t sum = 0;
  for (int k = 0; k < PER; ++k) sum += counts[b0 + k];
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int k = 0; k < PER; ++k) {
    offsets[b0 + k] = run;
    cursor[b0 + k] = run;
    run += counts[b0 + k];
  }
}

__global__ void __launch_bounds__(256) k_msm_scatter(size_t n, uint64_t seed, const uint8_t* __restrict__ flags,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ list) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t z = rlc_coeff(seed, i);
  const uint8_t f = flags[i];
#pragma unroll
  for (int mw = 0; mw < MSM_MW; ++mw) {
    const int b = msm_bucket(z, f, mw >> 1, mw & 1);
    if (b >= 0) list[atomicAdd(cursor + b, 1u)] = (uint32_t)i;
  }
}

// B_b = sum of the bucket's points (Jacobian SoA, stride MSM_KEYS)
__global__ void __launch_bounds__(256, 2) k_msm_bucket(size_t n, const uint32_t* __restrict__ offsets,
                                                     const uint32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ aos, uint32_t* __restrict__ buckets) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= MSM_KEYS) return;
  const int m = (int)(b >> (MSM_C + 1));
  const uint32_t* src = aos + (m >> 1 ? n * MSM_AOS_WORDS : 0);
  const uint32_t o = offsets[b], cnt = counts[b];
  g2j acc = g2_infinity();
#pragma unroll 1
  for (uint32_t p = 0; p < cnt; ++p) acc = g2_add_affine_body(acc, ld_aos(src, list[o + p]));
  st_g2j(buckets, MSM_KEYS, b, acc);
}

// Per run of MSM_RUN buckets [lo, lo + MSM_RUN) of one (MSM, window):
// sum_k k B_k = T + (lo - 1) R with R = sum_k B_k and T = sum_k (k - lo + 1) B_k
// (running sums from the top).  Output [mw][run] (stride MSM_MW * MSM_RUNS).
__global__ void __launch_bounds__(256, 2) k_msm_window(const uint32_t* __restrict__ buckets, uint32_t* __restrict__ runs) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)MSM_MW * MSM_RUNS) return;
  const size_t mw = g / MSM_RUNS, run = g % MSM_RUNS;
  const uint32_t lo = (uint32_t)(run * MSM_RUN);
  const size_t base = mw * MSM_BUCKETS + lo;
  g2j R = g2_infinity(), T = g2_infinity();
#pragma unroll 1
  for (int k = MSM_RUN - 1; k >= 0; --k) {
    R = g2_add_body(R, ld_g2j(buckets, MSM_KEYS, base + k));
    T = g2_add_body(T, R);
  }
  if (lo == 0) {  // digits 0..63: T counts every bucket once too often
    T = g2_add(T, g2_neg(R));
  } else if (lo > 1) {
    const uint32_t s = lo - 1;
    T = g2_add(T, g2_mul_words(R, &s, 1));
  }
  st_g2j(runs, (size_t)MSM_MW * MSM_RUNS, g, T);
}

// One level of pairwise sums over `groups` independent arrays of n_in
// Jacobian points each (group-major, stride total_in / total_out).
__global__ void __launch_bounds__(256) k_g2_sum_level(int groups, size_t n_in, const uint32_t* __restrict__ in,
                                                      size_t n_out, uint32_t* __restrict__ out) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)groups * n_out) return;
  const size_t grp = g / n_out, j = g % n_out;
  const size_t tin = (size_t)groups * n_in, tout = (size_t)groups * n_out;
  g2j P = ld_g2j(in, tin, grp * n_in + 2 * j);
  if (2 * j + 1 < n_in) P = g2_add_body(P, ld_g2j(in, tin, grp * n_in + 2 * j + 1));
  st_g2j(out, tout, g, P);
}

// The root: W[mw] (one point per (MSM, window), stride MSM_MW) ->
// P, S (stride-1 Jacobian SoA, the node layout rlc_check_locked reads).
__global__ void k_msm_root(const uint32_t* __restrict__ w, uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  if (blockIdx.x != 0 || threadIdx.x >= 2) return;
  const int tree = threadIdx.x;  // 0: P (MSMs 0, 1 over R), 1: S (MSMs 2, 3 over sig)
  g2j msm[2];
  for (int h = 0; h < 2; ++h) {
    const int m = 2 * tree + h;
    g2j hi = ld_g2j(w, MSM_MW, 2 * m + 1);
    for (int k = 0; k < MSM_C; ++k) hi = g2_dbl(hi);
    msm[h] = g2_add(ld_g2j(w, MSM_MW, 2 * m), hi);
  }
  st_g2j(tree ? s_out : p_out, 1, 0, g2_add(msm[0], g2_psi(msm[1])));
}

}  // namespace dgpu
