// Throughput of a thread-per-element 12x32-bit-limb Montgomery multiply (CIOS)
// on gfx950, two code shapes.  Sets expectations for the Fp layer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__constant__ uint32_t P[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,
                               0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
#define PINV 0xfffcfffdu

__device__ __forceinline__ void mont_mul_cios(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t t[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      uint64_t s = (uint64_t)a[j] * b[i] + t[j] + (c & 0xffffffffu);
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    uint64_t s = (uint64_t)t[12] + c;
    t[12] = (uint32_t)s;
    t[13] = (uint32_t)(s >> 32);
    uint32_t m = t[0] * PINV;
    s = (uint64_t)m * P[0] + t[0];
    c = s >> 32;
#pragma unroll
    for (int j = 1; j < 12; ++j) {
      s = (uint64_t)m * P[j] + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[12] + c;
    t[11] = (uint32_t)s;
    t[12] = t[13] + (uint32_t)(s >> 32);
  }
  // final conditional subtraction
  uint32_t d[12];
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    int64_t s = (int64_t)t[j] - P[j] + br;
    d[j] = (uint32_t)s;
    br = s >> 32;
  }
  bool ge = (t[12] != 0) || (br == 0);
#pragma unroll
  for (int j = 0; j < 12; ++j) r[j] = ge ? d[j] : t[j];
}


// Product-scanning (Comba) Montgomery: 96-bit column accumulator (u64 + u32 carry word)
__device__ __forceinline__ void mont_mul_comba(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[12];
  uint64_t acc = 0; uint32_t acc2 = 0;
#define MAC(x, y) asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(acc), "+v"(acc2) : "v"(x), "v"(y) : "vcc")
#pragma unroll
  for (int k = 0; k < 12; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) { MAC(a[i], b[k - i]); MAC(m[i], P[k - i]); }
    MAC(a[k], b[0]);
    m[k] = (uint32_t)acc * PINV;
    MAC(m[k], P[0]);
    acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
  }
  uint32_t t[13];
#pragma unroll
  for (int k = 12; k < 23; ++k) {
#pragma unroll
    for (int i = k - 11; i < 12; ++i) { MAC(a[i], b[k - i]); MAC(m[i], P[k - i]); }
    t[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
  }
  t[11] = (uint32_t)acc; t[12] = (uint32_t)(acc >> 32);
  uint32_t d[12];
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    int64_t s = (int64_t)t[j] - P[j] + br;
    d[j] = (uint32_t)s;
    br = s >> 32;
  }
  bool ge = (t[12] != 0) || (br == 0);
#pragma unroll
  for (int j = 0; j < 12; ++j) r[j] = ge ? d[j] : t[j];
}

template <int NDEP, int V>
__global__ void __launch_bounds__(256) k_fpmul(uint32_t* out, int iters) {
  uint32_t x[NDEP][12], y[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    y[j] = 0x12345678u * (j + 1) ^ threadIdx.x;
#pragma unroll
    for (int d = 0; d < NDEP; ++d) x[d][j] = (0x9abcdef1u * (j + 3 + d)) ^ blockIdx.x;
  }
  y[11] &= 0x0fffffff;
#pragma unroll
  for (int d = 0; d < NDEP; ++d) x[d][11] &= 0x0fffffff;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < NDEP; ++d) { if (V == 0) mont_mul_cios(x[d], x[d], y); else mont_mul_comba(x[d], x[d], y); }
  }
  uint32_t s = 0;
#pragma unroll
  for (int d = 0; d < NDEP; ++d)
#pragma unroll
    for (int j = 0; j < 12; ++j) s ^= x[d][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NDEP, int V>
static void run(int blocks) {
  int threads = 256, iters = 256;
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipLaunchKernelGGL((k_fpmul<NDEP, V>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_fpmul<NDEP, V>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double muls = (double)blocks * threads * iters * NDEP * 5;
  printf("fpmul v=%d ndep=%d blocks=%d: %.3f ms  %.2f G Fp-mul/s  (%.3f T 32x32 products/s @288/mul)\n", V, NDEP, blocks, ms,
         muls / (ms * 1e-3) / 1e9, muls * 288 / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  run<1,0>(4096); run<1,0>(16384); run<2,0>(16384); run<4,0>(16384);
  run<1,1>(4096); run<1,1>(16384); run<2,1>(16384); run<4,1>(16384);
  return 0;
}
