// G2 signature decode with the membership check (RLC mode's decode_g2 stage)
// in variants of register budget / inlining, timed against the library's
// k_decode_g2_sigs(check_subgroup = 1) on valid signatures hashed on the
// device.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o dec_g2_bin dec_g2.hip
#include <cstdio>
#include <vector>
#include "../../drand_amd/csrc/kernels.cuh"
using namespace dgpu;

// decode without the check (out of line, as the library), membership inline
// in the kernel (the 63-doubling ladder then obeys the kernel's launch bounds)
template <int OCC, bool INL_LAW>
__global__ void __launch_bounds__(256, OCC) k_dec2_v(size_t n, const uint8_t* __restrict__ sigs, size_t sig_stride,
                                                     const uint32_t* __restrict__ sig_len, uint32_t* __restrict__ sig_out,
                                                     uint8_t* __restrict__ status) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st;
  g2a p{fp2_zero(), fp2_zero()};
  if (sig_len[i] != 96) {
    st = ST_DECODE;
  } else {
    uint8_t buf[96];
    const uint8_t* src = sigs + i * sig_stride;
    for (int k = 0; k < 96; ++k) buf[k] = src[k];
    int rc = g2_decompress(&p, buf, false);
    if (rc == DEC_OK) {
      const g2j q = g2_from_affine(p);
      const bool in = INL_LAW ? g2_eq(g2_psi(q), g2_neg(g2_mul_absx_inl(q))) : g2_eq(g2_psi(q), g2_neg(g2_mul_absx(q)));
      if (!in) rc = DEC_ERR_SUBGROUP;
    }
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  }
  st_g2a(sig_out, n, i, p);
  status[i] = st;
}

__global__ void k_make_sigs(size_t n, uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8];
  for (int k = 0; k < 8; ++k) msg[k] = (uint32_t)(i * 2654435761u + k);
  const g2j h = hash_to_g2(msg);
  g2_compress(out + i * 96, g2_to_affine(h), false);
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
  uint8_t *sigs, *st;
  uint32_t *len, *out;
  CK(hipMalloc(&sigs, n * 96));
  CK(hipMalloc(&st, n));
  CK(hipMalloc(&len, n * 4));
  CK(hipMalloc(&out, n * G2A_WORDS * 4));
  std::vector<uint32_t> l(n, 96);
  CK(hipMemcpy(len, l.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_make_sigs, dim3((n + 63) / 64), dim3(64), 0, 0, n, sigs);
  CK(hipDeviceSynchronize());
  msg_src m{};
  const dim3 g((n + 255) / 256), b(256);
  std::vector<uint8_t> ref(n), got(n);
  float t = timeit([&] { hipLaunchKernelGGL(k_decode_g2_sigs, g, b, 0, 0, n, sigs, (size_t)96, len, m, 1, out, st); }, 5);
  CK(hipMemcpy(ref.data(), st, n, hipMemcpyDeviceToHost));
  size_t ok = 0;
  for (size_t i = 0; i < n; ++i) ok += ref[i] == ST_OK;
  printf("library k_decode_g2_sigs(1)  %8.3f ms per %zu  (%.1f ms per 10M)  valid %zu\n", t, n, t * 1e7 / n, ok);
  auto check = [&](const char* name, float ms) {
    CK(hipMemcpy(got.data(), st, n, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += got[i] != ref[i];
    printf("%-28s %8.3f ms per %zu  (%.1f ms per 10M)  status mismatches %zu\n", name, ms, n, ms * 1e7 / n, bad);
    return 0;
  };
#define RUNV(O, L) check("v<" #O "," #L ">", timeit([&] { hipLaunchKernelGGL((k_dec2_v<O, L>), g, b, 0, 0, n, sigs, (size_t)96, len, out, st); }, 5));
  RUNV(2, true) RUNV(3, true) RUNV(4, true) RUNV(2, false) RUNV(4, false)
  return 0;
}
