// Unsaturated-limb Montgomery multiply variants (no carry flags): W-bit limbs in
// 32-bit registers, 64-bit column accumulators via v_mad_u64_u32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "consts.h"

template <int W, int N>
__device__ __forceinline__ void mont_mul_sos(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr uint32_t M = (1u << W) - 1;
  const uint32_t* P = (W == 30) ? P30 : P28;
  const uint32_t PINV = (W == 30) ? PINV30 : PINV28;
  uint32_t t[2 * N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); ++i) acc += (uint64_t)a[i] * b[k - i];
    t[k] = (uint32_t)acc & M;
    acc >>= W;
  }
  t[2 * N - 1] = (uint32_t)acc;
  uint32_t m[N];
  acc = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) acc += (uint64_t)m[i] * P[k - i];
    acc += t[k];
    m[k] = ((uint32_t)acc * PINV) & M;
    acc += (uint64_t)m[k] * P[0];
    acc >>= W;
  }
#pragma unroll
  for (int k = N; k < 2 * N; ++k) {
#pragma unroll
    for (int i = k - N + 1; i < N; ++i) acc += (uint64_t)m[i] * P[k - i];
    acc += t[k];
    if (k < 2 * N - 1) { r[k - N] = (uint32_t)acc & M; acc >>= W; }
    else r[k - N] = (uint32_t)acc;
  }
}

template <int W, int N, int NDEP>
__global__ void __launch_bounds__(256) k_fpmul(uint32_t* out, int iters) {
  constexpr uint32_t M = (1u << W) - 1;
  uint32_t x[NDEP][N], y[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    y[j] = (0x12345678u * (j + 1) ^ threadIdx.x) & M;
#pragma unroll
    for (int d = 0; d < NDEP; ++d) x[d][j] = ((0x9abcdef1u * (j + 3 + d)) ^ blockIdx.x) & M;
  }
  y[N - 1] &= 0xfffff;
#pragma unroll
  for (int d = 0; d < NDEP; ++d) x[d][N - 1] &= 0xfffff;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < NDEP; ++d) mont_mul_sos<W, N>(x[d], x[d], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int d = 0; d < NDEP; ++d)
#pragma unroll
    for (int j = 0; j < N; ++j) s ^= x[d][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int W, int N, int NDEP>
static void run(int blocks) {
  int threads = 256, iters = 256;
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipLaunchKernelGGL((k_fpmul<W, N, NDEP>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_fpmul<W, N, NDEP>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double muls = (double)blocks * threads * iters * NDEP * 5;
  printf("fpmul W=%d N=%d ndep=%d blocks=%d: %.3f ms  %.2f G Fp-mul/s  (%.2f T mads/s)\n", W, N, NDEP, blocks, ms,
         muls / (ms * 1e-3) / 1e9, muls * (2 * N * N) / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  run<30, 13, 1>(16384); run<30, 13, 2>(16384); run<30, 13, 4>(16384);
  run<28, 14, 1>(16384); run<28, 14, 2>(16384); run<28, 14, 4>(16384);
  return 0;
}
