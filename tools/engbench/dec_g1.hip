// G1 signature decode variants (register budget / group-law inlining) timed
// against the library's k_decode_g1_sigs on valid signatures hashed on the
// device.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o dec_g1_bin dec_g1.hip
#include <cstdio>
#include <vector>
#include "../../drand_amd/csrc/g1sig.cuh"
using namespace dgpu;
// V1: everything force-inlined into the kernel (launch bounds apply)
template <bool INL_LAW>
DG_FN g1j mul_absx_v(const g1j& p) {
  g1j r = p;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = INL_LAW ? g1_dbl_body(r) : g1_dbl(r);
    if ((BLS_X_ABS >> i) & 1ull) r = INL_LAW ? g1_add_body(r, p) : g1_add(r, p);
  }
  return r;
}
template <bool INL_LAW>
DG_FN bool in_sub_v(const g1a& p) {
  const g1j t = mul_absx_v<INL_LAW>(mul_absx_v<INL_LAW>(g1j{p.x, p.y, fp_one()}));
  if (g1_is_inf(t)) return false;
  const fp z2 = fp_sqr(t.z);
  return fp_eq(fp_mul(fp_mul(C_G1_BETA, p.x), z2), t.x) && fp_is_zero(fp_add(fp_mul(p.y, fp_mul(z2, t.z)), t.y));
}
template <bool INL_LAW>
DG_FN int dec_v(g1a* out, const uint8_t* in) {
  const uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return DEC_ERR_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; ++i) acc |= in[i];
    return acc ? DEC_ERR_INFINITY_NONCANON : DEC_INFINITY;
  }
  const bool sign = (b0 & 0x20) != 0;
  uint8_t buf[48];
  for (int i = 0; i < 48; ++i) buf[i] = in[i];
  buf[0] &= 0x1f;
  const fp xs = fp_std_from_be48(buf);
  if (!fp_std_lt_p(xs)) return DEC_ERR_X_RANGE;
  const fp x = fp_to_mont(xs);
  const fp rhs = fp_add(fp_mul(fp_sqr(x), x), C_B1);
  fp y = fp_sqrt_cand(rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return DEC_ERR_NOT_ON_CURVE;
  if (fp_std_gt_half(fp_from_mont(y)) != sign) y = fp_neg(y);
  out->x = x;
  out->y = y;
  return in_sub_v<INL_LAW>(*out) ? DEC_OK : DEC_ERR_SUBGROUP;
}
template <int OCC, bool INL_LAW>
__global__ void __launch_bounds__(256, OCC) k_dec_v(size_t n, const uint8_t* __restrict__ sigs, size_t sig_stride,
                                                         const uint32_t* __restrict__ sig_len, msg_src m,
                                                         uint32_t* __restrict__ sig_out, uint8_t* __restrict__ status) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st;
  g1a p{fp_zero(), fp_zero()};
  if (sig_len[i] != 48 || msg_bad_record(m, i)) {
    st = ST_DECODE;
  } else {
    uint8_t buf[48];
    const uint8_t* src = sigs + i * sig_stride;
    for (int k = 0; k < 48; ++k) buf[k] = src[k];
    const int rc = dec_v<INL_LAW>(&p, buf);
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  }
  st_fp(sig_out, n, i, p.x);
  st_fp(sig_out + FP_WORDS * n, n, i, p.y);
  status[i] = st;
}

__global__ void k_make_sigs(size_t n, uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8];
  for (int k = 0; k < 8; ++k) msg[k] = (uint32_t)(i * 2654435761u + k);
  const g1j h = hash_to_g1(msg, false);
  g1_compress(out + i * 48, g1_to_affine(h), false);
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
  CK(hipMalloc(&sigs, n * 48));
  CK(hipMalloc(&st, n));
  CK(hipMalloc(&len, n * 4));
  CK(hipMalloc(&out, n * 2 * FP_WORDS * 4));
  std::vector<uint32_t> l(n, 48);
  CK(hipMemcpy(len, l.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_make_sigs, dim3((n + 255) / 256), dim3(256), 0, 0, n, sigs);
  CK(hipDeviceSynchronize());
  msg_src m{};
  const dim3 g((n + 255) / 256), b(256);
  std::vector<uint8_t> ref(n), got(n);
  auto check = [&](const char* name, float ms) {
    CK(hipMemcpy(got.data(), st, n, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += got[i] != ref[i];
    printf("%-28s %8.3f ms per %zu  (%.1f ms per 10M)  status mismatches %zu\n", name, ms, n, ms * 1e7 / n, bad);
    return 0;
  };
  float t = timeit([&] { hipLaunchKernelGGL(k_decode_g1_sigs, g, b, 0, 0, n, sigs, (size_t)48, len, m, out, st); }, 5);
  CK(hipMemcpy(ref.data(), st, n, hipMemcpyDeviceToHost));
  size_t ok = 0;
  for (size_t i = 0; i < n; ++i) ok += ref[i] == ST_OK;
  printf("library k_decode_g1_sigs     %8.3f ms per %zu  (%.1f ms per 10M)  valid %zu\n", t, n, t * 1e7 / n, ok);
#define RUNV(O, L) check("v<" #O "," #L ">", timeit([&] { hipLaunchKernelGGL((k_dec_v<O, L>), g, b, 0, 0, n, sigs, (size_t)48, len, m, out, st); }, 5));
  RUNV(2, true) RUNV(3, true) RUNV(4, true) RUNV(2, false) RUNV(4, false)
  return 0;
}
