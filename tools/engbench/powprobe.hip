// Occupancy probe for the per-thread kernels' out-of-line Fp calls: one
// fp_sqrt_cand (the SSWU's exponentiation, fp_pow_sched over fp_sqr_r /
// fp_mul_r calls) per thread and repetition, with exactly `wps` waves per SIMD
// resident (256 x wps blocks of 4 waves; the kernel itself needs few VGPRs).
// The per-thread hash, lines and chain kernels run at 2 waves per SIMD (256
// VGPRs); this measures what the same call-bound code issues at 1..8.
// Prints pows/s chip-wide and the rate relative to 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../drand_amd/csrc/fp.cuh"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

using namespace dgpu;

__global__ void __launch_bounds__(256) k_pow(int reps, const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  fp a;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) a.l[k] = in[k] ^ (uint32_t)(t & 0xFFFu);
#pragma unroll 1
  for (int r = 0; r < reps; ++r) a = fp_sqrt_cand(a);
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) x ^= a.l[k];
  out[t] = x;
}

int main() {
  uint32_t *din, *dout;
  uint32_t h[FP_LIMBS];
  for (int k = 0; k < FP_LIMBS; ++k) h[k] = (0x1234567u * (k + 1)) & FP_MASK;
  h[FP_LIMBS - 1] &= 0xFFFFu;
  CK(hipMalloc(&din, sizeof(h)));
  CK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, (size_t)256 * 8 * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 8;
  double base = 0;
  const int w[] = {2, 1, 3, 4, 6, 8};
  for (int wps : w) {
    const int blocks = 256 * wps;
    hipLaunchKernelGGL(k_pow, dim3(blocks), dim3(256), 0, 0, 1, din, dout);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_pow, dim3(blocks), dim3(256), 0, 0, reps, din, dout);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double rate = (double)blocks * 256 * reps / (ms * 1e-3);
    if (wps == 2) base = rate;
    printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"pows_per_s\": %.4g, \"vs_2_waves\": %.3f}\n", wps, ms, rate,
           rate / base);
  }
  return 0;
}
