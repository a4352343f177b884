// RLC leaves [a] q + [b] psi(q) over G2 (k_rlc_leaves<G2Ops>'s arithmetic):
// the library's signed radix-16 window ladder (table [1..8] q) against a
// radix-8 form (table [1..4] q: half the private table, 22 additions instead
// of 16 + 4 more table entries), same results checked point by point.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o leaves_bin leaves.hip
#include <cstdio>
#include <vector>
#include "../../drand_amd/csrc/rlc_msm.cuh"
using namespace dgpu;

// signed radix-8 digits of a 32-bit k: 11 digits in [-4, 3] (bits 4j..4j+3:
// |d| in 3 bits, sign in bit 3) and a top digit (0 or 1) at bit 44
DG_FN uint64_t win3_recode32(uint32_t k) {
  uint64_t out = 0;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 11; ++j) {
    const uint32_t w = (j < 10 ? ((k >> (3 * j)) & 7u) : (k >> 30)) + c;
    c = w >= 4u ? 1u : 0u;
    const uint32_t mag = c ? 8u - w : w;
    out |= (uint64_t)(mag | (c && mag ? 8u : 0u)) << (4 * j);
  }
  return out | ((uint64_t)c << 44);
}

DG_FN g2j g2_mul2_win3_affine(const g2a& q, uint32_t a, uint32_t b) {
  const uint64_t da = win3_recode32(a), db = win3_recode32(b);
  g2j T[4];
  T[0] = g2_from_affine(q);
  T[1] = g2_dbl_body(T[0]);
  T[2] = g2_add_affine_body(T[1], q);
  T[3] = g2_dbl_body(T[1]);
  g2j acc = g2_cmov(g2_infinity(), T[0], (da >> 44) & 1u);
  acc = g2_cmov(acc, g2_add_body(acc, g2_psi(T[0])), (db >> 44) & 1u);
#pragma unroll 1
  for (int j = 10; j >= 0; --j) {
#pragma unroll 1
    for (int s = 0; s < 3; ++s) acc = g2_dbl_body(acc);
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      const uint32_t dg = (uint32_t)(((s ? db : da) >> (4 * j)) & 15u), mag = dg & 7u;
      g2j t = T[(mag - 1u) & 3u];
      if (s) t = g2_psi(t);
      t.y = fp2_cmov(t.y, fp2_neg(t.y), (dg & 8u) != 0);
      acc = g2_cmov(acc, g2_add_body(acc, t), mag != 0);
    }
  }
  return acc;
}

template <int V>
__global__ void __launch_bounds__(256, 2) k_leaves_v(size_t n, uint64_t seed, const uint32_t* __restrict__ r_aff,
                                                     uint32_t* __restrict__ p_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const g2a q = ld_g2a(r_aff, n, i);
  const uint64_t z = rlc_coeff(seed, i);
  const g2j acc = V == 0 ? g2_mul2_win4_affine(q, (uint32_t)z, (uint32_t)(z >> 32))
                         : g2_mul2_win3_affine(q, (uint32_t)z, (uint32_t)(z >> 32));
  st_g2j(p_out, n, i, acc);
}

__global__ void k_make_pts(size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8];
  for (int k = 0; k < 8; ++k) msg[k] = (uint32_t)(i * 2654435761u + k);
  st_g2a(out, n, i, g2_to_affine(hash_to_g2(msg)));
}

__global__ void k_eq(size_t n, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, unsigned* bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (!g2_eq(ld_g2j(a, n, i), ld_g2j(b, n, i))) atomicAdd(bad, 1u);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
template <class K>
float timeit(K launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : (1u << 20);
  uint32_t *pts, *o0, *o1;
  CK(hipMalloc(&pts, n * G2A_WORDS * 4));
  CK(hipMalloc(&o0, n * G2J_WORDS * 4));
  CK(hipMalloc(&o1, n * G2J_WORDS * 4));
  hipLaunchKernelGGL(k_make_pts, dim3((n + 63) / 64), dim3(64), 0, 0, n, pts);
  CK(hipDeviceSynchronize());
  const dim3 g((n + 255) / 256), b(256);
  const float t0 = timeit([&] { hipLaunchKernelGGL(k_leaves_v<0>, g, b, 0, 0, n, (uint64_t)7, pts, o0); }, 3);
  const float t1 = timeit([&] { hipLaunchKernelGGL(k_leaves_v<1>, g, b, 0, 0, n, (uint64_t)7, pts, o1); }, 3);
  unsigned* bad;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_eq, g, b, 0, 0, n, o0, o1, bad);
  unsigned nb = 0;
  CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("mismatching points: %u\n", nb);
  printf("win4 (library) %8.3f ms per %zu  (%.1f ms per 10M points)\n", t0, n, t0 * 1e7 / n);
  printf("win3           %8.3f ms per %zu  (%.1f ms per 10M points)\n", t1, n, t1 * 1e7 / n);
  return 0;
}
