// RLC batch verification (configs[2], and configs[3]'s per-GPU fold for the
// G1-signature schemes), written once over the signature group (group_ops.cuh:
// G2Ops for pedersen-bls-*, G1Ops for bls-unchained-on-g1 / -g1-rfc9380).
//
// With d_i = e(pk, H_i) e(-g1, sig_i) (G2 signatures) or e(H_i, pk) e(-sig_i, g2)
// (G1 signatures), the whole batch collapses to one pairing check by
//   prod_i d_i^(r_i) = e(h_eff sum_i r_i R_i, .) e(sum_i r_i sig_i, .)
// with R_i the pre-cofactor hash point (h_eff applied once per checked node,
// by linearity) and r_i = a_i + b_i lambda (group_ops.cuh).  The root
//   P = sum_i a_i R_i + endo(sum_i b_i R_i),  S = sum_i a_i sig_i + endo(sum_i b_i sig_i)
// is four MSMs with 32-bit scalars over the batch's affine points, each in two
// 16-bit windows: every (MSM, window, digit) is a bucket, so a point costs one
// mixed addition per MSM and window -- 8 per round instead of the two window
// ladders of k_rlc_leaves (~32 doublings + 16 additions each).  The tree of
// leaves is built only when this root fails (capi.hip verify_status_locked).
//
// Pipeline (one launch each; the bucket order is a counting sort, so the
// sums do not depend on the order the atomics hand out positions -- point
// addition is associative and commutative, the results are exact):
//   k_msm_aos     R_i, sig_i affine SoA -> AoS (G2: 224 B contiguous per point,
//                 gathers read two cache lines instead of 56) + usable flags
//   k_msm_count   bucket sizes (atomics)
//   k_msm_scan    exclusive prefix sums (one block)
//   k_msm_scatter point indices (and keys) into their buckets (atomics on cursors)
//   k_msm_bucket_seg  equal ranges of the sorted list per thread: sums of its runs of
//                 equal key (mixed additions); k_msm_fixup joins runs cut by a range
//                 boundary (DGPU_MSM_SEG=0: k_msm_bucket, one thread per bucket)
//   k_msm_window  one thread per run of MSM_RUN buckets: sum_k k B_k of the run
//   k_sum_level   pairwise tree over the runs of each (MSM, window)
//   k_msm_root    MSM_m = W_m0 + 2^16 W_m1; P = MSM_0 + endo(MSM_1), S = MSM_2 + endo(MSM_3)
#pragma once
#include <type_traits>
#include "kernels.cuh"
#include "group_ops.cuh"

namespace dgpu {

constexpr int G1A_WORDS = 2 * FP_WORDS;  // affine G1 point
constexpr int G1J_WORDS = 3 * FP_WORDS;  // Jacobian G1 point

__device__ __forceinline__ void st_g1j(uint32_t* base, size_t n, size_t i, const g1j& p) {
  st_fp(base, n, i, p.x);
  st_fp(base + FP_WORDS * n, n, i, p.y);
  st_fp(base + 2 * FP_WORDS * n, n, i, p.z);
}
__device__ __forceinline__ g1j ld_g1j(const uint32_t* base, size_t n, size_t i) {
  return g1j{ld_fp(base, n, i), ld_fp(base + FP_WORDS * n, n, i), ld_fp(base + 2 * FP_WORDS * n, n, i)};
}
__device__ __forceinline__ void st_g1a(uint32_t* base, size_t n, size_t i, const g1a& p) {
  st_fp(base, n, i, p.x);
  st_fp(base + FP_WORDS * n, n, i, p.y);
}
__device__ __forceinline__ g1a ld_g1a(const uint32_t* base, size_t n, size_t i) {
  return g1a{ld_fp(base, n, i), ld_fp(base + FP_WORDS * n, n, i)};
}

// HBM layouts of one group's points: SoA [coordinate Fp][limb][index] (AFF /
// JAC words per point), AoS rows of AFF words (the MSM's gather side).
template <class Gr>
struct GrMem;
template <>
struct GrMem<G2Ops> {
  static constexpr int AFF = G2A_WORDS, JAC = G2J_WORDS;
  static __device__ __forceinline__ g2a ld_aff(const uint32_t* b, size_t n, size_t i) { return ld_g2a(b, n, i); }
  static __device__ __forceinline__ void st_aff(uint32_t* b, size_t n, size_t i, const g2a& p) { st_g2a(b, n, i, p); }
  static __device__ __forceinline__ g2j ld_jac(const uint32_t* b, size_t n, size_t i) { return ld_g2j(b, n, i); }
  static __device__ __forceinline__ void st_jac(uint32_t* b, size_t n, size_t i, const g2j& p) { st_g2j(b, n, i, p); }
  static __device__ __forceinline__ g2a ld_row(const uint32_t* __restrict__ p) {
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
  static __device__ __forceinline__ void st_row(uint32_t* __restrict__ o, const g2a& q) {
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) {
      o[l] = q.x.c0.l[l];
      o[FP_LIMBS + l] = q.x.c1.l[l];
      o[2 * FP_LIMBS + l] = q.y.c0.l[l];
      o[3 * FP_LIMBS + l] = q.y.c1.l[l];
    }
  }
};
template <>
struct GrMem<G1Ops> {
  static constexpr int AFF = G1A_WORDS, JAC = G1J_WORDS;
  static __device__ __forceinline__ g1a ld_aff(const uint32_t* b, size_t n, size_t i) { return ld_g1a(b, n, i); }
  static __device__ __forceinline__ void st_aff(uint32_t* b, size_t n, size_t i, const g1a& p) { st_g1a(b, n, i, p); }
  static __device__ __forceinline__ g1j ld_jac(const uint32_t* b, size_t n, size_t i) { return ld_g1j(b, n, i); }
  static __device__ __forceinline__ void st_jac(uint32_t* b, size_t n, size_t i, const g1j& p) { st_g1j(b, n, i, p); }
  static __device__ __forceinline__ g1a ld_row(const uint32_t* __restrict__ p) {
    g1a a;
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) {
      a.x.l[l] = p[l];
      a.y.l[l] = p[FP_LIMBS + l];
    }
    return a;
  }
  static __device__ __forceinline__ void st_row(uint32_t* __restrict__ o, const g1a& q) {
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) {
      o[l] = q.x.l[l];
      o[FP_LIMBS + l] = q.y.l[l];
    }
  }
};

constexpr int MSM_C = 16;                         // window bits
constexpr int MSM_BUCKETS = 1 << MSM_C;           // per (MSM, window); digit 0 unused
constexpr int MSM_MW = 8;                         // 4 MSMs x 2 windows
constexpr size_t MSM_KEYS = (size_t)MSM_MW * MSM_BUCKETS;
// Buckets per k_msm_window thread: 8 (64Ki threads for the 8 (MSM, window)
// pairs, short serial runs) measured faster than 64 (8Ki threads, 512 waves
// for 1,024 SIMDs): root MSM 96.2 -> 87.2 ms per 10M G2 points, 37.8 -> 35.6
// for G1 (profiles/r04/r04p_msm_run_ab.txt).
#ifndef DG_MSM_RUN
#define DG_MSM_RUN 8
#endif
constexpr int MSM_RUN = DG_MSM_RUN;
constexpr int MSM_RUNS = MSM_BUCKETS / MSM_RUN;   // runs per (MSM, window)

// R (affine SoA in r_aff, (0, 0) = identity) and sig (affine SoA) -> AoS
// [R | sig][i]; flags[i]: bit 0 R usable, bit 1 sig usable (status ST_OK and
// not the identity; the leaves kernel skips the same points).
template <class Gr>
__global__ void __launch_bounds__(256) k_msm_aos(size_t n, const uint32_t* __restrict__ r_aff,
                                                 const uint32_t* __restrict__ sig_pts,
                                                 const uint8_t* __restrict__ status, uint32_t* __restrict__ aos,
                                                 uint8_t* __restrict__ flags) {
  using M = GrMem<Gr>;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t f = 0;
  for (int which = 0; which < 2; ++which) {
    const typename Gr::aff q = M::ld_aff(which ? sig_pts : r_aff, n, i);
    M::st_row(aos + ((size_t)which * n + i) * M::AFF, q);
    if (status[i] == ST_OK && !Gr::aff_is_zero(q)) f |= (uint8_t)(1u << which);
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
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ list,
                                                     uint32_t* __restrict__ keys) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t z = rlc_coeff(seed, i);
  const uint8_t f = flags[i];
#pragma unroll
  for (int mw = 0; mw < MSM_MW; ++mw) {
    const int b = msm_bucket(z, f, mw >> 1, mw & 1);
    if (b >= 0) {
      const uint32_t pos = atomicAdd(cursor + b, 1u);
      list[pos] = (uint32_t)i;
      if (keys) keys[pos] = (uint32_t)b;  // the load-balanced sums read the key per entry
    }
  }
}

// B_b = sum of the bucket's points (Jacobian SoA, stride MSM_KEYS)
template <class Gr>
__global__ void __launch_bounds__(256, 2) k_msm_bucket(size_t n, const uint32_t* __restrict__ offsets,
                                                     const uint32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ aos, uint32_t* __restrict__ buckets) {
  using M = GrMem<Gr>;
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= MSM_KEYS) return;
  const int m = (int)(b >> (MSM_C + 1));
  const uint32_t* src = aos + (m >> 1 ? n * M::AFF : 0);
  const uint32_t o = offsets[b], cnt = counts[b];
  typename Gr::jac acc = Gr::inf();
#pragma unroll 1
  for (uint32_t p = 0; p < cnt; ++p) acc = Gr::add_aff_body(acc, M::ld_row(src + (size_t)list[o + p] * M::AFF));
  M::st_jac(buckets, MSM_KEYS, b, acc);
}

// Load-balanced bucket sums (the default).  One thread per bucket leaves a
// wave running as long as its largest bucket: at 10M rounds the bucket sizes
// are Poisson(~153), and the maximum over a wave's 64 buckets is ~183, so
// about 16% of the lanes' addition slots are idle.  Here the sorted list
// (keys ascending, k_msm_scatter) is cut into T equal ranges of
// S = ceil(L / T) entries, T = one resident wave per SIMD slot, and every
// thread runs exactly S mixed additions over the runs of equal key in its
// range.  A run that is a whole bucket goes to buckets[key]; a run cut by the
// range's start goes to part slot A[t], one cut only by its end to B[t]
// (at most one of each per thread); k_msm_fixup joins the pieces:
// bucket = B[t0] + A[t0 + 1] + ... + A[t1] with t0, t1 the ranges holding the
// bucket's first and last entries.
template <class Gr>
__device__ __forceinline__ void msm_seg_emit(uint32_t key, size_t s, size_t e, size_t t, size_t T,
                                             const uint32_t* __restrict__ offsets,
                                             const uint32_t* __restrict__ counts, const typename Gr::jac& acc,
                                             uint32_t* __restrict__ buckets, uint32_t* __restrict__ part) {
  using M = GrMem<Gr>;
  const size_t o = offsets[key], c = counts[key];
  const bool whole = s <= o && e >= o + c;
  // cut at the start: A[t]; cut at the end only: B[t]; else the whole bucket (one store sequence)
  M::st_jac(whole ? buckets : part, whole ? MSM_KEYS : 2 * T, whole ? key : (s > o ? t : T + t), acc);
}

// A G2 row (x.c0, x.c1, y.c0, y.c1 limbs, 224 bytes), each coordinate loaded
// where the addition uses it (empty asm on the address per fetch).
struct g2_row_fetch {
  const uint32_t* row;
  __device__ __forceinline__ const uint32_t* b() const {
    const uint32_t* p = row;
    __asm__ volatile("" : "+v"(p));
    return p;
  }
  __device__ __forceinline__ fp2 x() const {
    const uint32_t* p = b();
    fp2 v;
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) v.c0.l[l] = p[l], v.c1.l[l] = p[FP_LIMBS + l];
    return v;
  }
  __device__ __forceinline__ fp2 y() const {
    const uint32_t* p = b() + 2 * FP_LIMBS;
    fp2 v;
#pragma unroll
    for (int l = 0; l < FP_LIMBS; ++l) v.c0.l[l] = p[l], v.c1.l[l] = p[FP_LIMBS + l];
    return v;
  }
  __device__ __forceinline__ g2a get() const { return g2a{x(), y()}; }
};

// G2 (round 6): the runs are summed with fast mixed additions of the fetched
// row (no call site in the loop; a run's first point is taken as is), and an
// exceptional addition (the running sum = +-the next point, e.g. a batch
// holding one signature twice) redoes the thread's range with the generic
// addition -- the emits are plain stores, so the redo overwrites them.
template <class Gr>
__global__ void __launch_bounds__(256, 2) k_msm_bucket_seg(size_t n, size_t T, const uint32_t* __restrict__ offsets,
                                                         const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ aos,
                                                         uint32_t* __restrict__ buckets, uint32_t* __restrict__ part) {
  using M = GrMem<Gr>;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const size_t L = (size_t)offsets[MSM_KEYS - 1] + counts[MSM_KEYS - 1];
  const size_t S = (L + T - 1) / T;
  const size_t p0 = t * S;
  if (p0 >= L) return;
  const size_t p1 = p0 + S < L ? p0 + S : L;
  bool exc = false;
#ifndef DG_MSM_GENERIC
  if constexpr (std::is_same<Gr, G2Ops>::value) {
    uint32_t key = keys[p0];
    size_t s = p0;
    g2j acc = g2_infinity();
    bool first = true;
#pragma unroll 1
    for (size_t p = p0; p < p1; ++p) {
      const uint32_t k = keys[p];
      if (k != key) {
        msm_seg_emit<Gr>(key, s, p, t, T, offsets, counts, acc, buckets, part);
        key = k;
        s = p;
        first = true;
      }
      const uint32_t* src = aos + ((key >> (MSM_C + 2)) ? n * M::AFF : 0);  // MSMs 2, 3: the signatures
      const g2_row_fetch f{src + (size_t)list[p] * M::AFF};
      if (first) {
        acc = g2_from_affine(f.get());
        first = false;
      } else {
        acc = g2_madd_nx_q(acc, f, exc);
      }
    }
    msm_seg_emit<Gr>(key, s, p1, t, T, offsets, counts, acc, buckets, part);
    if (!exc && !DG_FORCE_EXC) return;
  }
#endif
  uint32_t key = keys[p0];
  size_t s = p0;
  typename Gr::jac acc = Gr::inf();
#pragma unroll 1
  for (size_t p = p0; p < p1; ++p) {
    const uint32_t k = keys[p];
    if (k != key) {
      msm_seg_emit<Gr>(key, s, p, t, T, offsets, counts, acc, buckets, part);
      key = k;
      s = p;
      acc = Gr::inf();
    }
    const uint32_t* src = aos + ((key >> (MSM_C + 2)) ? n * M::AFF : 0);  // MSMs 2, 3: the signatures
    acc = Gr::add_aff_body(acc, M::ld_row(src + (size_t)list[p] * M::AFF));
  }
  msm_seg_emit<Gr>(key, s, p1, t, T, offsets, counts, acc, buckets, part);
}

// One thread per bucket: empty -> identity; a bucket spread over ranges
// t0 < t1 -> B[t0] + A[t0 + 1] + ... + A[t1]; a bucket inside one range was
// written whole by k_msm_bucket_seg.
template <class Gr>
__global__ void __launch_bounds__(256) k_msm_fixup(size_t T, const uint32_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ part, uint32_t* __restrict__ buckets) {
  using M = GrMem<Gr>;
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= MSM_KEYS) return;
  const size_t c = counts[b];
  if (c == 0) {
    M::st_jac(buckets, MSM_KEYS, b, Gr::inf());
    return;
  }
  const size_t L = (size_t)offsets[MSM_KEYS - 1] + counts[MSM_KEYS - 1];
  const size_t S = (L + T - 1) / T;
  const size_t o = offsets[b], t0 = o / S, t1 = (o + c - 1) / S;
  if (t0 == t1) return;
  typename Gr::jac acc = M::ld_jac(part, 2 * T, T + t0);
#pragma unroll 1
  for (size_t t = t0 + 1; t <= t1; ++t) acc = Gr::add(acc, M::ld_jac(part, 2 * T, t));
  M::st_jac(buckets, MSM_KEYS, b, acc);
}

// Per run of MSM_RUN buckets [lo, lo + MSM_RUN) of one (MSM, window):
// sum_k k B_k = T + (lo - 1) R with R = sum_k B_k and T = sum_k (k - lo + 1) B_k
// (running sums from the top).  Output [mw][run] (stride MSM_MW * MSM_RUNS).
template <class Gr>
__global__ void __launch_bounds__(256, 2) k_msm_window(const uint32_t* __restrict__ buckets, uint32_t* __restrict__ runs) {
  using M = GrMem<Gr>;
  using J = typename Gr::jac;
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)MSM_MW * MSM_RUNS) return;
  const size_t mw = g / MSM_RUNS, run = g % MSM_RUNS;
  const uint32_t lo = (uint32_t)(run * MSM_RUN);
  const size_t base = mw * MSM_BUCKETS + lo;
  J R = Gr::inf(), T = Gr::inf();
#pragma unroll 1
  for (int k = MSM_RUN - 1; k >= 0; --k) {
    R = Gr::add_body(R, M::ld_jac(buckets, MSM_KEYS, base + k));
    T = Gr::add_body(T, R);
  }
  if (lo == 0) {  // digits 0..MSM_RUN-1: T counts every bucket once too often
    T = Gr::add(T, Gr::neg(R));
  } else if (lo > 1) {  // + [lo - 1] R, double-and-add over the 16-bit multiplier
    const uint32_t s = lo - 1;
    J acc = Gr::inf();
#pragma unroll 1
    for (int i = 31 - __builtin_clz(s); i >= 0; --i) {
      acc = Gr::dbl(acc);
      if ((s >> i) & 1u) acc = Gr::add(acc, R);
    }
    T = Gr::add(T, acc);
  }
  M::st_jac(runs, (size_t)MSM_MW * MSM_RUNS, g, T);
}

// One level of pairwise sums over `groups` independent arrays of n_in
// Jacobian points each (group-major, stride total_in / total_out).
template <class Gr>
__global__ void __launch_bounds__(256) k_sum_level(int groups, size_t n_in, const uint32_t* __restrict__ in,
                                                   size_t n_out, uint32_t* __restrict__ out) {
  using M = GrMem<Gr>;
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)groups * n_out) return;
  const size_t grp = g / n_out, j = g % n_out;
  const size_t tin = (size_t)groups * n_in, tout = (size_t)groups * n_out;
  typename Gr::jac P = M::ld_jac(in, tin, grp * n_in + 2 * j);
  if (2 * j + 1 < n_in) P = Gr::add_body(P, M::ld_jac(in, tin, grp * n_in + 2 * j + 1));
  M::st_jac(out, tout, g, P);
}

// The root: W[mw] (one point per (MSM, window), stride MSM_MW) ->
// P, S (stride-1 Jacobian SoA, the node layout rlc_check_locked reads).
template <class Gr>
__global__ void k_msm_root(const uint32_t* __restrict__ w, uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  if (blockIdx.x != 0 || threadIdx.x >= 2) return;
  const int tree = threadIdx.x;  // 0: P (MSMs 0, 1 over R), 1: S (MSMs 2, 3 over sig)
  typename Gr::jac msm[2];
  for (int h = 0; h < 2; ++h) {
    const int m = 2 * tree + h;
    typename Gr::jac hi = M::ld_jac(w, MSM_MW, 2 * m + 1);
    for (int k = 0; k < MSM_C; ++k) hi = Gr::dbl(hi);
    msm[h] = Gr::add(M::ld_jac(w, MSM_MW, 2 * m), hi);
  }
  M::st_jac(tree ? s_out : p_out, 1, 0, Gr::add(msm[0], Gr::endo(msm[1])));
}

// ---------------------------------------------------------------- leaves, tree, nodes
// Leaves of the RLC tree: P_i = [a_i] R_i + [b_i] endo(R_i), S_i = [a_i] sig_i +
// [b_i] endo(sig_i) with (a_i, b_i) the two halves of rlc_coeff (infinity for
// rounds whose decode verdict is already final).  R_i is affine here (batch
// affine ran on the pre-cofactor hash points; (0, 0) marks the identity).
// 2n threads: j < n computes P_j, j >= n computes S_{j-n}.  The scalar
// multiplication is the window form (every lane runs the same sequence).
template <class Gr>
__global__ void __launch_bounds__(256, 2) k_rlc_leaves(size_t n, uint64_t seed, const uint32_t* __restrict__ r_aff,
                                                       const uint32_t* __restrict__ sig_pts,
                                                       const uint8_t* __restrict__ status,
                                                       uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const bool sig = j >= n;
  const size_t i = sig ? j - n : j;
  typename Gr::jac acc = Gr::inf();
  if (status[i] == ST_OK) {
    const typename Gr::aff q = M::ld_aff(sig ? sig_pts : r_aff, n, i);
    if (!Gr::aff_is_zero(q)) {
      const uint64_t z = rlc_coeff(seed, i);
      if constexpr (std::is_same<Gr, G2Ops>::value)
        acc = g2_mul2_win4_affine(q, (uint32_t)z, (uint32_t)(z >> 32));
      else
        acc = mul2_win4_affine<Gr>(q, (uint32_t)z, (uint32_t)(z >> 32));
    }
  }
  M::st_jac(sig ? s_out : p_out, n, i, acc);
}

// Leaves of the localization tree (coefficients 1): P_i = R_i, S_i = sig_i
// as Jacobian points (infinity for rounds whose verdict is already final).
// A leaf check of this tree is the round's own pairing check (exact); an
// internal node can only hide bad rounds whose errors cancel in a plain sum,
// which the confirmation check with fresh random coefficients catches
// (capi.hip rlc_resolve_locked).
template <class Gr>
__global__ void __launch_bounds__(256) k_rlc_leaves_plain(size_t n, const uint32_t* __restrict__ r_aff,
                                                          const uint32_t* __restrict__ sig_pts,
                                                          const uint8_t* __restrict__ status,
                                                          uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const bool sig = j >= n;
  const size_t i = sig ? j - n : j;
  typename Gr::jac acc = Gr::inf();
  if (status[i] == ST_OK) {
    const typename Gr::aff q = M::ld_aff(sig ? sig_pts : r_aff, n, i);
    if (!Gr::aff_is_zero(q)) acc = Gr::from_aff(q);
  }
  M::st_jac(sig ? s_out : p_out, n, i, acc);
}

// Leaves of listed rounds (the localization's failing leaves), whatever
// their status now: P_k = [a] R_i + [b] endo(R_i), S_k likewise, i = list[k]
// -- the terms those rounds contributed to the shard's root.
template <class Gr>
__global__ void __launch_bounds__(256, 2) k_rlc_leaves_list(size_t m, const uint32_t* __restrict__ list, size_t n,
                                                            uint64_t seed, const uint32_t* __restrict__ r_aff,
                                                            const uint32_t* __restrict__ sig_pts,
                                                            uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * m) return;
  const bool sig = j >= m;
  const size_t k = sig ? j - m : j, i = list[k];
  typename Gr::jac acc = Gr::inf();
  const typename Gr::aff q = M::ld_aff(sig ? sig_pts : r_aff, n, i);
  if (!Gr::aff_is_zero(q)) {
    const uint64_t z = rlc_coeff(seed, i);
    if constexpr (std::is_same<Gr, G2Ops>::value)
      acc = g2_mul2_win4_affine(q, (uint32_t)z, (uint32_t)(z >> 32));
    else
      acc = mul2_win4_affine<Gr>(q, (uint32_t)z, (uint32_t)(z >> 32));
  }
  M::st_jac(sig ? s_out : p_out, m, k, acc);
}

// Compaction of the failing candidates: out[atomic] = idx[k] where fail[k]
// (order irrelevant: the listed leaves are summed).
__global__ void __launch_bounds__(256) k_rlc_compact_fail(size_t m, const uint32_t* __restrict__ idx,
                                                          const uint8_t* __restrict__ fail, uint32_t* __restrict__ out,
                                                          uint32_t* __restrict__ count) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < m && fail[k]) out[atomicAdd(count, 1u)] = idx[k];
}

// root - F (each a stride-1 (P, S) pair of Jacobian points) -> out
template <class Gr>
__global__ void k_rlc_sub_root(const uint32_t* __restrict__ root, const uint32_t* __restrict__ fp_,
                               const uint32_t* __restrict__ fs, uint32_t* __restrict__ out) {
  using M = GrMem<Gr>;
  if (blockIdx.x != 0 || threadIdx.x >= 2) return;
  const int w = threadIdx.x;  // 0: P, 1: S
  const typename Gr::jac r = M::ld_jac(root + w * M::JAC, 1, 0);
  const typename Gr::jac f = M::ld_jac(w ? fs : fp_, 1, 0);
  M::st_jac(out + w * M::JAC, 1, 0, Gr::add(r, Gr::neg(f)));
}

// One tree level: out[j] = in[2j] + in[2j+1] (odd tail copied); 2 n_out
// threads, the first n_out on the P tree, the rest on the S tree.
template <class Gr>
// (bounded at 2 waves/SIMD it spills 233 VGPRs for G2 and gains nothing:
// profiles/r04/r04s_rlc_level_occ_ab.txt)
__global__ void __launch_bounds__(256) k_rlc_level(size_t n_in, const uint32_t* __restrict__ p_in,
                                                   const uint32_t* __restrict__ s_in, size_t n_out,
                                                   uint32_t* __restrict__ p_out, uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n_out) return;
  const bool sig = t >= n_out;
  const size_t j = sig ? t - n_out : t;
  const uint32_t* in = sig ? s_in : p_in;
  const size_t a = 2 * j, b = 2 * j + 1;
  typename Gr::jac P = M::ld_jac(in, n_in, a);
  if (b < n_in) P = Gr::add_body(P, M::ld_jac(in, n_in, b));
  M::st_jac(sig ? s_out : p_out, n_out, j, P);
}

// Candidate nodes for the pairing engine: h[c] = affine h_eff * P, sg[c] =
// affine S, st[c] = ST_OK when both are finite (the engine then decides),
// RLC_TRIVIAL when both are infinity (passes), ST_PAIRING when exactly one is
// (e(Q, .) of a non-trivial prime-order point alone is never 1).
template <class Gr>
__global__ void __launch_bounds__(64) k_rlc_prep(size_t n_cand, const uint32_t* __restrict__ idx, size_t n_level,
                                                 const uint32_t* __restrict__ p_lvl,
                                                 const uint32_t* __restrict__ s_lvl, uint32_t* __restrict__ h_out,
                                                 uint32_t* __restrict__ s_out, uint8_t* __restrict__ st) {
  using M = GrMem<Gr>;
  size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cand) return;
  size_t j = idx[c];
  const typename Gr::jac P = Gr::clear_cofactor(M::ld_jac(p_lvl, n_level, j));
  const typename Gr::jac S = M::ld_jac(s_lvl, n_level, j);
  const bool pi = Gr::is_inf(P), si = Gr::is_inf(S);
  M::st_aff(h_out, n_cand, c, pi ? Gr::aff_zero() : Gr::to_aff(P));
  M::st_aff(s_out, n_cand, c, si ? Gr::aff_zero() : Gr::to_aff(S));
  st[c] = (pi && si) ? RLC_TRIVIAL : (pi || si) ? (uint8_t)ST_PAIRING : (uint8_t)ST_OK;
}

// Multi-GPU RLC: the per-device roots (P, S), gathered over RCCL as
// [dev][P (JAC words), S (JAC words)] (each a stride-1 Jacobian SoA), summed
// into one node (stride 1) that is checked once for the whole node.
template <class Gr>
__global__ void k_rlc_sum_roots(int ndev, const uint32_t* __restrict__ roots, uint32_t* __restrict__ p_out,
                                uint32_t* __restrict__ s_out) {
  using M = GrMem<Gr>;
  if (blockIdx.x != 0 || threadIdx.x >= 2) return;
  const int w = threadIdx.x;  // 0: P, 1: S
  typename Gr::jac acc = M::ld_jac(roots + w * M::JAC, 1, 0);
  for (int d = 1; d < ndev; ++d) acc = Gr::add(acc, M::ld_jac(roots + (size_t)d * 2 * M::JAC + w * M::JAC, 1, 0));
  M::st_jac(w ? s_out : p_out, 1, 0, acc);
}

}  // namespace dgpu
