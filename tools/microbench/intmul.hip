// Integer-multiply throughput microbenchmark for gfx950 (sets the roofline
// denominator for the big-number kernels).  Each lane runs NCHAIN independent
// chains of one instruction kind; the result is folded into an output so the
// compiler cannot drop the work.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define NCHAIN 8
#define ITERS 4096

__global__ void __launch_bounds__(256) k_mad_u64(uint32_t* out, uint32_t seed) {
  uint64_t acc[NCHAIN];
  uint32_t a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCHAIN; ++c) {
      uint64_t r;
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b + c), "v"(acc[c]) : "vcc");
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

#define DEF_BINOP(NAME, INSN)                                                              \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {              \
    uint32_t acc[NCHAIN];                                                                  \
    uint32_t b = seed * 3 + blockIdx.x;                                                    \
    _Pragma("unroll") for (int c = 0; c < NCHAIN; ++c) acc[c] = seed ^ (threadIdx.x + c); \
    for (int i = 0; i < ITERS; ++i) {                                                      \
      _Pragma("unroll") for (int c = 0; c < NCHAIN; ++c) {                                 \
        uint32_t r;                                                                        \
        asm volatile(INSN " %0, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b));                 \
        acc[c] = r;                                                                        \
      }                                                                                    \
    }                                                                                      \
    uint32_t s = 0;                                                                        \
    _Pragma("unroll") for (int c = 0; c < NCHAIN; ++c) s ^= acc[c];                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
  }

DEF_BINOP(k_mul_lo, "v_mul_lo_u32")
DEF_BINOP(k_mul_hi, "v_mul_hi_u32")
DEF_BINOP(k_mul_u24, "v_mul_u32_u24")
DEF_BINOP(k_mul_hi_u24, "v_mul_hi_u32_u24")
DEF_BINOP(k_add_u32, "v_add_u32")

__global__ void __launch_bounds__(256) k_add_co(uint32_t* out, uint32_t seed) {
  uint32_t acc[NCHAIN];
  uint32_t b = seed * 3 + blockIdx.x;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) acc[c] = seed ^ (threadIdx.x + c);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCHAIN; c += 2) {
      uint32_t r0, r1;
      asm volatile("v_add_co_u32 %0, vcc, %2, %3\n\tv_addc_co_u32 %1, vcc, %4, %3, vcc"
                   : "=&v"(r0), "=v"(r1) : "v"(acc[c]), "v"(b), "v"(acc[c + 1]) : "vcc");
      acc[c] = r0; acc[c + 1] = r1;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fma_f64(uint32_t* out, uint32_t seed) {
  double acc[NCHAIN];
  double b = 1.0000001 + seed * 1e-9;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) acc[c] = (double)(threadIdx.x + c);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCHAIN; ++c) {
      double r;
      asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(acc[c]), "v"(b), "v"(b));
      acc[c] = r;
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

typedef void (*kfn)(uint32_t*, uint32_t);

static void run(const char* name, kfn k, int insn_per_chain_iter) {
  int blocks = 256 * 8 * 4;  // 8 waves per SIMD with 256-thread blocks
  int threads = 256;
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * threads * ITERS * NCHAIN * insn_per_chain_iter * reps;
  printf("%-14s %8.3f ms  %8.3f Tlane-ops/s\n", name, ms, ops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run("mad_u64_u32", k_mad_u64, 1);
  run("mul_lo_u32", k_mul_lo, 1);
  run("mul_hi_u32", k_mul_hi, 1);
  run("mul_u32_u24", k_mul_u24, 1);
  run("mul_hi_u24", k_mul_hi_u24, 1);
  run("add_u32", k_add_u32, 1);
  run("add_co+addc", k_add_co, 1);
  run("fma_f64", k_fma_f64, 1);
  return 0;
}
