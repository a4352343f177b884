// Per-op cost microbenchmark of the lane-cooperative pairing engine
// (drand_amd/csrc/engine.cuh).  Every wave runs one engine op `reps` times on
// random field elements in its groups' LDS slots (the op's own kernel slot
// count, so occupancy matches the production kernel), and the host reports
// ms per 1M group-ops (one op on 1M pairing items).  Used to A/B engine
// variants (compile-time macros) op by op before touching the full pipeline.
//
//   engbench [reps]         -> one JSON line per op
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../drand_amd/csrc/engine.cuh"

using namespace dgpu;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

#ifndef ENGBENCH_PAD_WORDS
#define ENGBENCH_PAD_WORDS 0   // extra LDS per block: occupancy sweep
#endif
// the production kernels' LDS layout per family (0 lines, 1 Miller, 2 FE)
constexpr int bench_lds_slots(int fam) {
  return fam == 0 ? ENG_LDS_SLOTS_LINES : fam == 1 ? ENG_LDS_SLOTS_MILLER : ENG_LDS_SLOTS_FE;
}
__device__ __forceinline__ int bench_gbase(int fam, int g) {
  return fam == 0 ? ENG_GBASE_LINES[g] : fam == 1 ? ENG_GBASE_MILLER[g] : ENG_GBASE_FE[g];
}
template <int FAM>
__global__ void __launch_bounds__(64, 3) k_bench(int op, int reps, const uint32_t* __restrict__ init,
                                                 uint32_t* __restrict__ out, int sub_first, int sub_count) {
  constexpr int NSLOTS = FAM == 0 ? ENG_SLOTS_LINES : FAM == 1 ? ENG_SLOTS_MILLER : ENG_SLOTS_FE;
  __shared__ uint32_t lds[bench_lds_slots(FAM) * ENG_SLOT_WORDS + ENGBENCH_PAD_WORDS];
#ifdef ENGBENCH_LDS_RECORDS   // the op's records staged in LDS instead of read from global memory
  __shared__ __attribute__((aligned(16))) uint32_t rec[528];  // largest op's record span
  const uint32_t s0 = ENG_OP_TAB[op][0], sl = s0 + ENG_OP_TAB[op][1] - 1;
  const uint32_t w0 = ENG_SUB_TAB[s0][0];
  const uint32_t w1 = ENG_SUB_TAB[sl][0] + 12 * eng_rec_words(ENG_SUB_TAB[sl][1] & 0xFFu);
  for (uint32_t t = threadIdx.x; t < w1 - w0; t += blockDim.x) rec[t] = ENG_WORDS[w0 + t];
#define ENGBENCH_RUN_ARGS , rec, w0
#elif defined(ENGBENCH_LDS_PAD)   // same LDS footprint, records from global memory
  __shared__ uint32_t pad[528];
  if (reps < 0) pad[threadIdx.x] = op;
  if (reps < 0) out[threadIdx.x] = pad[(threadIdx.x + 1) & 63];
#define ENGBENCH_RUN_ARGS
#else
#define ENGBENCH_RUN_ARGS
#endif
  constexpr int W = bench_lds_slots(FAM) * ENG_SLOT_WORDS;
  const uint32_t* src = init + (size_t)(blockIdx.x & 63) * W;
  for (int t = threadIdx.x; t < W; t += blockDim.x) lds[t] = src[t];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int gi = lane < 60 ? lane / 12 : 4;
  const int k = lane < 60 ? lane % 12 : lane - 60;
  uint32_t* c = lds;
  uint32_t* g = lds + bench_gbase(FAM, gi) * ENG_SLOT_WORDS;
  uint32_t sink_acc = 0;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    if (op == -1) {  // E_CYC with its LIN sub-op
      eng_cyc_fast<true>(g, k, fp{});
      continue;
    }
    if (op == -2) {  // one chain of reps E_CYC (fused LIN epilogue, post operand in registers)
      eng_cyc_chain(g, k, reps);
      break;
    }
    if (op >= 1000) {  // compiled form (engine_compiled.h)
      auto snk = [&](uint32_t e, const fp& v) { sink_acc += v.l[0] ^ e; };
      if (!(eng_run_c0(op - 1000, g, c, k, snk) || eng_run_c1(op - 1000, g, c, k, snk) ||
            eng_run_c2(op - 1000, g, c, k, snk)))
        sink_acc += 1;
      continue;
    }
#ifdef ENGBENCH_LDS_RECORDS
    eng_run(op, g, c, k, [&](uint32_t e, const fp& v) { sink_acc += v.l[0] ^ e; } ENGBENCH_RUN_ARGS);
#else
    eng_run(op, g, c, k, [&](uint32_t e, const fp& v) { sink_acc += v.l[0] ^ e; }, ENG_WORDS, 0,
            (uint32_t)sub_first, (uint32_t)sub_count);
#endif
  }
  asm volatile("" ::: "memory");
  uint32_t h = sink_acc;
  for (int i = 0; i < NSLOTS * ENG_SLOT_WORDS; i += 64) h ^= g[(i + lane) % (NSLOTS * ENG_SLOT_WORDS)];
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = h;
}

// v_mad_u64_u32 latency / throughput probe: 4 waves per block (one per SIMD),
// NCH independent accumulation chains per lane, each a dependent mad chain.
template <int NCH>
__global__ void __launch_bounds__(256) k_mad(int iters, uint32_t y, uint64_t* __restrict__ out) {
  uint64_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = threadIdx.x + c;
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 64 / NCH; ++u) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[c] = (uint64_t)(uint32_t)acc[c] * y + acc[c];
    }
  }
  uint64_t h = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) h ^= acc[c];
  out[(size_t)blockIdx.x * 256 + threadIdx.x] = h;
}

struct OpDesc {
  const char* name;
  int op;
  int fam;  // 0 lines, 1 miller, 2 fe
  int sub_first = 0, sub_count = 255;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 64;
  const int blocks = 256 * 11 * 4;
  const char* only = getenv("ENGBENCH_ONLY");
  const OpDesc ops[] = {
      {"LDBL", OP_LDBL, 0},       {"LADD", OP_LADD, 0},       {"M_XIF", OP_M_XIF, 1},     {"M_SQR", OP_M_SQR, 1},
      {"M_XIL", OP_M_XIL, 1},     {"M_LM1", OP_M_LM1, 1},     {"E_CYC", OP_E_CYC, 2},     {"E_MUL", OP_E_MUL, 2},
      {"E_MULCJ", OP_E_MULCJ, 2}, {"E_XIA", OP_E_XIA, 2},     {"E_FROB1", OP_E_FROB1, 2},
      {"E_CYC_lin", OP_E_CYC, 2, 0, 1}, {"E_CYC_prod", OP_E_CYC, 2, 1, 1}, {"E_CYC_fast", -1, 2}, {"E_CYC_chain", -2, 2},
      {"LDBL_c", 1000 + OP_LDBL, 0}, {"LADD_c", 1000 + OP_LADD, 0}, {"M_SQR_c", 1000 + OP_M_SQR, 1},
      {"M_XIF_c", 1000 + OP_M_XIF, 1}, {"M_LM1_c", 1000 + OP_M_LM1, 1}, {"E_MUL_c", 1000 + OP_E_MUL, 2}, {"E_XIA_c", 1000 + OP_E_XIA, 2},
  };
  constexpr int WMAX = (ENG_NCONST + ENG_GROUPS_PER_WAVE * 64) * ENG_SLOT_WORDS;
  std::vector<uint32_t> h((size_t)64 * WMAX);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < h.size(); ++i) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    const int limb = (int)((i % ENG_SLOT_WORDS));
    h[i] = limb == FP_LIMBS - 1 ? (uint32_t)(s % FP_P[FP_LIMBS - 1]) : (uint32_t)(s & FP_MASK);
  }
  uint32_t *d_init, *d_out;
  CK(hipMalloc(&d_init, h.size() * 4));
  CK(hipMalloc(&d_out, (size_t)blocks * 64 * 4));
  CK(hipMemcpy(d_init, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (!only || strstr(only, "MAD")) {
    uint64_t* d_mo;
    CK(hipMalloc(&d_mo, (size_t)256 * 256 * 8));
    const int iters = 4096;
    auto mad_run = [&](auto kern, const char* name) {
      hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, 16, 3u, d_mo);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, iters, 3u, d_mo);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      // one wave per SIMD, 64 mads per iteration per wave: ns per mad per wave
      printf("{\"op\": \"%s\", \"ms\": %.3f, \"ns_per_mad_per_wave\": %.4f}\n", name, ms, ms * 1e6 / (iters * 64.0));
    };
    mad_run(k_mad<1>, "MAD_chains1");
    mad_run(k_mad<2>, "MAD_chains2");
    mad_run(k_mad<4>, "MAD_chains4");
    mad_run(k_mad<8>, "MAD_chains8");
    CK(hipFree(d_mo));
  }
  for (const OpDesc& o : ops) {
    if (only && !strstr(only, o.name)) continue;
    auto launch = [&](int r) {
      if (o.fam == 0) hipLaunchKernelGGL(k_bench<0>, dim3(blocks), dim3(64), 0, 0, o.op, r, d_init, d_out, o.sub_first, o.sub_count);
      else if (o.fam == 1) hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(64), 0, 0, o.op, r, d_init, d_out, o.sub_first, o.sub_count);
      else hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(64), 0, 0, o.op, r, d_init, d_out, o.sub_first, o.sub_count);
    };
    launch(2);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int it = 0; it < 3; ++it) {
      CK(hipEventRecord(e0));
      launch(reps);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double group_ops = (double)blocks * ENG_GROUPS_PER_WAVE * reps;
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"ms_per_1M_items\": %.4f}\n", o.name, best, best * 1e6 / group_ops);
    fflush(stdout);
  }
  return 0;
}
