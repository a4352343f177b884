// Fp mul (14 x 28-bit) ILP variants at low occupancy (1 wave/SIMD) vs high.
// NACC independent column accumulators per product column.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../drand_amd/csrc/constants.h"
using namespace dgpu;

template <int NACC>
__device__ __forceinline__ void mulk(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr int N = 14, W = 28;
  constexpr uint32_t M = (1u << W) - 1;
  uint32_t t[2 * N];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) {
    uint64_t acc[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = 0;
    acc[0] = carry;
    int lo = k < N ? 0 : k - N + 1, hi = k < N ? k : N - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc[(i - lo) % NACC] += (uint64_t)a[i] * b[k - i];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) s += acc[q];
    t[k] = (uint32_t)s & M;
    carry = s >> W;
  }
  t[2 * N - 1] = (uint32_t)carry;
  uint32_t m[N];
  carry = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    uint64_t acc[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = 0;
    acc[0] = carry + t[k];
#pragma unroll
    for (int i = 0; i < k; ++i) acc[i % NACC] += (uint64_t)m[i] * FP_P[k - i];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) s += acc[q];
    m[k] = ((uint32_t)s * FP_PINV) & M;
    s += (uint64_t)m[k] * FP_P[0];
    carry = s >> W;
  }
#pragma unroll
  for (int k = N; k < 2 * N; ++k) {
    uint64_t acc[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[q] = 0;
    acc[0] = carry + t[k];
#pragma unroll
    for (int i = k - N + 1; i < N; ++i) acc[i % NACC] += (uint64_t)m[i] * FP_P[k - i];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) s += acc[q];
    r[k - N] = k < 2 * N - 1 ? ((uint32_t)s & M) : (uint32_t)s;
    carry = s >> W;
  }
}

template <int NACC>
__global__ void __launch_bounds__(256) k_mul(uint32_t* out, int iters) {
  uint32_t x[14], y[14];
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    y[j] = (0x12345678u * (j + 1) ^ threadIdx.x) & 0xfffffff;
    x[j] = ((0x9abcdef1u * (j + 3)) ^ blockIdx.x) & 0xfffffff;
  }
  y[13] &= 0xffff; x[13] &= 0xffff;
  for (int i = 0; i < iters; ++i) mulk<NACC>(x, x, y);
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) s ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(64) k_madlat(uint32_t* out, int iters) {
  uint64_t acc = threadIdx.x;
  uint32_t a = threadIdx.x * 7 + 1, b = blockIdx.x + 3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)acc;
}

template <int NACC>
static void run(int blocks, int threads) {
  int iters = 128;
  uint32_t* out;
  hipMalloc(&out, 4 * blocks * threads);
  hipLaunchKernelGGL((k_mul<NACC>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_mul<NACC>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double muls = 3.0 * blocks * threads * iters;
  printf("nacc=%d blocks=%d threads=%d (waves/SIMD=%.1f): %.2f G Fp-mul/s\n", NACC, blocks, threads,
         blocks * threads / 64.0 / 1024.0, muls / (ms * 1e-3) / 1e9);
  hipFree(out);
}

int main() {
  // latency: one wave per SIMD, dependent chain of 16 mads per iteration
  uint32_t* out; hipMalloc(&out, 4 * 1024 * 64);
  int iters = 4096;
  hipLaunchKernelGGL(k_madlat, dim3(1024), dim3(64), 0, 0, out, iters); hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0); hipLaunchKernelGGL(k_madlat, dim3(1024), dim3(64), 0, 0, out, iters); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("dependent v_mad_u64_u32 chain, 1 wave/SIMD: %.2f ns per mad (%.1f cycles @2.4GHz)\n", ms * 1e6 / (iters * 16.0), ms * 1e6 / (iters * 16.0) * 2.4);
  for (int t : {256}) {
    run<1>(256, t); run<2>(256, t); run<3>(256, t); run<4>(256, t);      // 1 wave/SIMD
    run<1>(512, t); run<2>(512, t); run<4>(512, t);                      // 2 waves/SIMD
    run<1>(8192, t); run<2>(8192, t); run<4>(8192, t);                   // many
  }
  return 0;
}
