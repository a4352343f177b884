// Issue-rate probe for the VALU instructions the engine's inner loops use
// (v_mad_u64_u32, 64-bit shift/add/move, 32-bit and/add/cndmask) at 1, 2 and
// 4 waves per SIMD, 8 independent chains per lane.  Prints ns per
// wave-instruction per SIMD (chip: 256 CUs x 4 SIMDs).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

template <int KIND>
__global__ void __launch_bounds__(256) k_probe(int iters, uint32_t y, uint64_t* __restrict__ out) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b0 = threadIdx.x, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
  const uint64_t y64 = ((uint64_t)y << 32) | y;
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (KIND == 0) {
#define S(i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a##i) : "v"(b##i), "v"(y) : "s40", "s41");
        BODY8(S)
#undef S
      } else if constexpr (KIND == 1) {
#define S(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a##i) : "v"(y64));
        BODY8(S)
#undef S
      } else if constexpr (KIND == 2) {
#define S(i) asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(a##i));
        BODY8(S)
#undef S
      } else if constexpr (KIND == 3) {
#define S(i) asm volatile("v_mov_b64 %0, %1" : "=v"(a##i) : "v"(y64));
        BODY8(S)
#undef S
      } else if constexpr (KIND == 4) {
#define S(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(b##i) : "v"(y));
        BODY8(S)
#undef S
      } else if constexpr (KIND == 5) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(b##i) : "v"(y));
        BODY8(S)
#undef S
      } else if constexpr (KIND == 6) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(b##i) : "v"(y) : "vcc");
        BODY8(S)
#undef S
      }
    }
  }
  out[(size_t)blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
}

int main() {
  uint64_t* d;
  CK(hipMalloc(&d, (size_t)256 * 256 * 4 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"v_mad_u64_u32", "v_lshl_add_u64", "v_lshrrev_b64", "v_mov_b64", "v_and_b32", "v_mul_lo_u32", "v_add_co_u32"};
  void (*kern[])(int, uint32_t, uint64_t*) = {k_probe<0>, k_probe<1>, k_probe<2>, k_probe<3>, k_probe<4>, k_probe<5>, k_probe<6>};
  const int iters = 2048;
  for (int k = 0; k < 7; ++k) {
    for (int wps = 1; wps <= 4; wps *= 2) {
      const int blocks = 256 * wps;  // 4 waves per block: wps waves per SIMD
      hipLaunchKernelGGL(kern[k], dim3(blocks), dim3(256), 0, 0, 8, 3u, d);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern[k], dim3(blocks), dim3(256), 0, 0, iters, 3u, d);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double winst_per_simd = (double)iters * 64 * wps;
      printf("{\"inst\": \"%s\", \"waves_per_simd\": %d, \"ns_per_wave_inst_per_simd\": %.4f}\n", names[k], wps,
             ms * 1e6 / winst_per_simd);
    }
  }
  return 0;
}
