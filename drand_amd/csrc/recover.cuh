// Batch threshold recovery: kyber tbls.Recover + share.RecoverCommit (R), as
// called by drand's aggregator chain/beacon/chain.go:158-168 (and the
// partial check node.go:117-125 -> VerifyPartial).
//
// Per round: walk the partials in order, keep those whose index parses
// (>= 2 bytes) and that verify against PubPoly.Eval(index) (decode +
// subgroup + pairing: the pairing runs on the lane-cooperative engine over
// all partial "items" of the batch), stop after t good ones; dedup by index
// (xyCommit); fewer than t distinct -> failure; otherwise Lagrange at 0 over
// Fr (x_i = index + 1) and the G2 multi-scalar multiplication
// sum_j lambda_j sig_j (4-way split by the psi endomorphism, Straus, mixed additions),
// compressed to 96 bytes; then VerifyRecovered (chain.go:165) of every
// recovered signature under C_0 on the engine.
//
// Batched check (the default path, capi.hip recover_device_locked): all
// partials of a round sign the same H(msg), so instead of t VerifyPartial
// pairings the round's first t decodable partials (the candidates) are
// checked together with the recovered signature in ONE two-pair pairing:
//   e(C_0 + sum_j r_j Eval(i_j), H) * e(-g1, sigma + sum_j r_j sig_j) == 1
// with fresh uniform 64-bit r_j.  With E_j = sig_j - s_j H the error of
// candidate j, sigma - sk H = sum_j lambda_j E_j, so the check holds iff
// sum_j (r_j + lambda_j) E_j = 0: always when every candidate is valid (then
// the selection is exactly the reference's "first t good"), and with
// probability <= 2^-64 otherwise.  A failing round is decided without
// pairings when no decodable partial is left beyond the candidates (the
// reference cannot reach t good ones either); otherwise it, and every round
// whose per-partial statuses are requested, takes the exact per-partial path
// above.
#pragma once
#include "fr.cuh"
#include "kernels.cuh"

namespace dgpu {

constexpr int RECOVER_MAX_T = 32;
// digits per (round, j): the four base-|x| digits of lambda_j, then the RLC
// coefficient r_j of the batched check
constexpr int RECOVER_SLOTS = 5;

// recovery class of a round (k_recover_cand; REC_MORE flags a decodable
// partial beyond the candidates)
enum : uint8_t { REC_RLC = 0, REC_FAIL = 1, REC_EXACT = 2, REC_MORE = 0x10 };

// Group commitments C_j (48-byte compressed G1) -> affine SoA [x, y][limb][t]
// (Montgomery); rc[j] = decode code.  kyber UnmarshalBinary semantics (R).
__global__ void k_decode_commits(int t, const uint8_t* __restrict__ in48, uint32_t* __restrict__ pts,
                                 int* __restrict__ rc) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= t) return;
  uint8_t buf[48];
  for (int k = 0; k < 48; ++k) buf[k] = in48[(size_t)j * 48 + k];
  g1a p{fp_zero(), fp_zero()};
  int r = g1_decompress(&p, buf, GROUP_ORDER_WORDS);
  st_fp(pts, t, j, p.x);
  st_fp(pts + FP_LIMBS * t, t, j, p.y);
  rc[j] = r;
}

// PubPoly.Eval(i) = sum_j C_j (i+1)^j by Horner (kyber share/poly.go (R)),
// returned as the pairing engine wants it: (-x, y), Montgomery.
__device__ void pubpoly_eval(const uint32_t* commits, int t, uint32_t i, fp& neg_x, fp& y) {
  const uint32_t x = i + 1;
  g1j acc = g1_infinity();
  for (int j = t - 1; j >= 0; --j) {
    acc = g1_mul_words(acc, &x, 1);
    const g1a cj{ld_fp(commits, t, j), ld_fp(commits + FP_LIMBS * t, t, j)};
    acc = g1_add(acc, g1j{cj.x, cj.y, fp_one()});
  }
  const g1a a = g1_to_affine(acc);
  neg_x = fp_neg(a.x);
  y = a.y;
}

// Table of PubPoly.Eval(i) for i < n: SoA [(-x), y][limb][n]
__global__ void k_pubpoly_table(int n, int t, const uint32_t* __restrict__ commits, uint32_t* __restrict__ table) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp nx, y;
  pubpoly_eval(commits, t, (uint32_t)i, nx, y);
  st_fp(table, n, i, nx);
  st_fp(table + FP_LIMBS * n, n, i, y);
}

// Partials -> engine items.  Item i = partial i (round i / m, slot i % m):
// index (BE16 of the first two bytes; 0xFFFFFFFF if fewer than 2), the
// signature decoded (96 bytes after the index; any other length, including
// one above the stride, is a decode error; at most 98 bytes are read), the share key PubPoly.Eval(index) (table for index < n, else
// evaluated here), status ST_* (ST_OK -> still to be pairing-checked).
// (the membership ladder inlined at 2 waves/SIMD, as k_decode_g2_sigs_sub:
// out of line in g2_decompress its registers escape the kernel's budget)
__global__ void __launch_bounds__(256, 2) k_decode_partials(size_t n_items, const uint8_t* __restrict__ partials,
                                                          size_t stride, const uint32_t* __restrict__ plen, int n_group,
                                                          int t, const uint32_t* __restrict__ table,
                                                          const uint32_t* __restrict__ commits,
                                                          uint32_t* __restrict__ sig_pts, uint32_t* __restrict__ pk_items,
                                                          uint32_t* __restrict__ idx_out, uint8_t* __restrict__ status) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint8_t* src = partials + i * stride;
  const uint32_t len = plen[i];
  uint32_t idx = 0xFFFFFFFFu;
  uint8_t st = ST_DECODE;
  g2a p{fp2_zero(), fp2_zero()};
  if (len >= 2) idx = ((uint32_t)src[0] << 8) | src[1];
  if (len == 98) {
    uint8_t buf[96];
    for (int k = 0; k < 96; ++k) buf[k] = src[2 + k];
    int rc = g2_decompress(&p, buf, false);
    if (rc == DEC_OK) {  // p is stored by the membership test (not kept live across its ladder)
      if (!g2_in_subgroup_stored(p, sig_pts, n_items, i)) rc = DEC_ERR_SUBGROUP;
    } else {
      st_g2a(sig_pts, n_items, i, p);
    }
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  } else {
    st_g2a(sig_pts, n_items, i, p);
  }
  fp nx = fp_zero(), y = fp_zero();
  if (st == ST_OK) {
    if (idx < (uint32_t)n_group) {
      nx = ld_fp(table, n_group, idx);
      y = ld_fp(table + FP_LIMBS * n_group, n_group, idx);
    } else {
      pubpoly_eval(commits, t, idx, nx, y);
    }
  }
  st_fp(pk_items, n_items, i, nx);
  st_fp(pk_items + FP_LIMBS * n_items, n_items, i, y);
  idx_out[i] = idx;
  status[i] = st;
}

// Round of every partial item (engine h_idx): item / m.
__global__ void __launch_bounds__(256) k_round_of_item(size_t n_items, size_t m, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_items) out[i] = (uint32_t)(i / m);
}

// Affine hash points H(msg) of raw 32-byte messages (SoA, stride n).
__global__ void __launch_bounds__(256) k_hash_to_g2_msgs_pts(size_t n, const uint8_t* __restrict__ msgs,
                                                              uint32_t* __restrict__ h_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8];
  for (int w = 0; w < 8; ++w) {
    const uint8_t* b = msgs + i * 32 + 4 * w;
    msg[w] = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  }
  st_g2a(h_out, n, i, g2_to_affine(hash_to_g2(msg)));
}

// Synthetic partials (test/bench data tool, tbls.Sign (R)): item i of round
// i / m is BE16(label[i]) || compress(share[sign_idx[i]] * H(msg of round)).
// A label different from the signing share makes an invalid partial.
__global__ void __launch_bounds__(64) k_sign_partials(size_t n_items, size_t m, size_t n_rounds,
                                                      const uint32_t* __restrict__ h_pts,
                                                      const uint32_t* __restrict__ sign_idx,
                                                      const uint32_t* __restrict__ label,
                                                      const scalar256* __restrict__ shares,
                                                      uint8_t* __restrict__ out98) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const g2a h = ld_g2a(h_pts, n_rounds, i / m);
  const scalar256 k = shares[sign_idx[i]];
  const g2j sg = g2_mul_words(g2_from_affine(h), k.w, 8);
  const bool inf = g2_is_inf(sg);
  uint8_t* o = out98 + i * 98;
  o[0] = (uint8_t)(label[i] >> 8);
  o[1] = (uint8_t)label[i];
  g2_compress(o + 2, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(sg), inf);
}

// Recovery after the VerifyPartial pairings, in four launches (one thread per
// round ran only n_rounds threads, at one wave per SIMD):
//   k_recover_select    per round: the first t good partials in input order,
//                       deduplicated by index (sel = items, xs = index + 1);
//                       failures are final here (zero output, ok = 0)
//   k_recover_lagrange  per (round, j): the Lagrange coefficient at 0 over Fr
//                       as base-|x| digits, lambda = d0 + d1|x| + d2|x|^2 + d3|x|^3
//   k_recover_msm       per (round, i < 4): P_i = sum_j d_{j,i} sig_j (Straus, 64 bits)
//   k_recover_finish    per round: sum_j lambda_j sig_j = P0 - psi(P1) + psi^2(P2)
//                       - psi^3(P3) (psi = [x] on G2, x < 0: [|x|] = -psi), compressed
constexpr uint64_t RECOVER_ABSX_ODD = 0xd20100000001ull;  // |x| = 2^16 RECOVER_ABSX_ODD

// w (little-endian 32-bit words of v < 2^256) <- v / |x|; returns v mod |x|.
DG_FN uint64_t div_absx(uint32_t w[8]) {
  const uint32_t low = w[0] & 0xFFFFu;
  uint32_t q[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  uint64_t rem = 0;
  for (int k = 14; k >= 0; --k) {  // 16-bit digit k of v >> 16, most significant first
    const int bit = 16 * k + 16;
    rem = (rem << 16) | ((w[bit >> 5] >> (bit & 31)) & 0xFFFFu);
    const uint64_t qd = rem / RECOVER_ABSX_ODD;
    rem -= qd * RECOVER_ABSX_ODD;
    q[(16 * k) >> 5] |= (uint32_t)qd << ((16 * k) & 31);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = q[i];
  return (rem << 16) | low;
}

__global__ void __launch_bounds__(64) k_recover_select(size_t n_rounds, size_t m, int t,
                                                       const uint32_t* __restrict__ idx,
                                                       const uint8_t* __restrict__ status, uint32_t* __restrict__ sel,
                                                       uint32_t* __restrict__ xs, uint8_t* __restrict__ out96,
                                                       uint8_t* __restrict__ ok, const uint32_t* __restrict__ commits,
                                                       uint32_t* __restrict__ rec_pts, uint32_t* __restrict__ rec_pk,
                                                       uint8_t* __restrict__ rec_st) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds) return;
  // VerifyRecovered operands: key = PubPoly.Commit() = C_0
  st_fp(rec_pk, n_rounds, r, fp_neg(ld_fp(commits, t, 0)));
  st_fp(rec_pk + FP_LIMBS * n_rounds, n_rounds, r, ld_fp(commits + FP_LIMBS * t, t, 0));
  uint32_t sel_idx[RECOVER_MAX_T];
  uint32_t* sl = sel + r * RECOVER_MAX_T;
  uint32_t* xr = xs + r * RECOVER_MAX_T;
  int good = 0, distinct = 0;
  for (size_t j = 0; j < m && good < t; ++j) {
    const size_t item = r * m + j;
    if (status[item] != ST_OK) continue;
    ++good;
    const uint32_t id = idx[item];
    bool dup = false;
    for (int q = 0; q < distinct; ++q) dup = dup || sel_idx[q] == id;
    if (!dup) {
      sel_idx[distinct] = id;
      sl[distinct] = (uint32_t)item;
      xr[distinct] = id + 1;
      ++distinct;
    }
  }
  if (distinct < t) {
    for (int k = 0; k < 96; ++k) out96[r * 96 + k] = 0;
    ok[r] = 0;
    st_g2a(rec_pts, n_rounds, r, g2a{fp2_zero(), fp2_zero()});
    rec_st[r] = ST_DECODE;
    return;
  }
  ok[r] = 1;
}

// rlc_seed != 0: slot 4 = r_j of the batched check (SplitMix64 of the seed
// and the (round, j) position, as the beacon RLC's rlc_coeff)
__global__ void __launch_bounds__(256) k_recover_lagrange(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                          const uint32_t* __restrict__ xs,
                                                          uint64_t* __restrict__ digits, uint64_t rlc_seed) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rounds * RECOVER_MAX_T) return;
  const size_t r = g / RECOVER_MAX_T;
  const int j = (int)(g % RECOVER_MAX_T);
  if (j >= t || !ok[r]) return;
  uint32_t w[8];
  fr_lagrange_at_zero(xs + r * RECOVER_MAX_T, t, j, w);
  uint64_t* d = digits + g * RECOVER_SLOTS;
  d[0] = div_absx(w);
  d[1] = div_absx(w);
  d[2] = div_absx(w);
  d[3] = ((uint64_t)w[1] << 32) | w[0];  // the last quotient, < |x| since lambda < r < |x|^4
  d[4] = rlc_seed ? rlc_coeff(rlc_seed, g) : 0;
}

__global__ void __launch_bounds__(256, 2) k_recover_msm(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                     const uint32_t* __restrict__ sel,
                                                     const uint64_t* __restrict__ digits,
                                                     const uint32_t* __restrict__ sig_pts, size_t n_items,
                                                     uint32_t* __restrict__ part) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 4 * n_rounds) return;
  const size_t r = g >> 2;
  const int i = (int)(g & 3);
  if (!ok[r]) return;
  const uint64_t* d = digits + r * RECOVER_MAX_T * RECOVER_SLOTS + i;
  const uint32_t* sl = sel + r * RECOVER_MAX_T;
  g2j acc = g2_infinity();
  for (int b = 63; b >= 0; --b) {
    acc = g2_dbl_body(acc);
    for (int j = 0; j < t; ++j)
      if ((d[RECOVER_SLOTS * j] >> b) & 1ull) acc = g2_add_affine_body(acc, ld_g2a(sig_pts, n_items, sl[j]));
  }
  st_g2j(part + (size_t)i * G2J_WORDS * n_rounds, n_rounds, r, acc);
}

// Signed radix-16 digit j (0..16) of a 64-bit k: d_j = w_j + b_{4j-1} - 16
// b_{4j+3} (w_j the 4-bit window, b the bits of k), in [-8, 8];
// k = sum_j d_j 16^j.
DG_FN int win4_digit64(uint64_t k, int j) {
  const int w = j < 16 ? (int)((k >> (4 * j)) & 15u) : 0;
  const int cin = j ? (int)((k >> (4 * j - 1)) & 1u) : 0;
  const int cout = j < 16 ? (int)((k >> (4 * j + 3)) & 1u) : 0;
  return w + cin - 16 * cout;
}

// k_recover_msm with the same operation sequence in every lane.  The lanes
// of a wave hold different rounds, whose signer sets (so Lagrange digits)
// differ; the bit-driven loop above runs an addition whenever any lane's bit
// is set, i.e. about 64 t per thread.  Here: per point j a table
// [1..8] sig_j (Jacobian, private memory, 1 doubling + 6 mixed additions),
// then 17 signed radix-16 windows of 4 doublings + t additions (a zero
// digit's addition computed and discarded): 16 t + 7 t additions in all.
// TMAX bounds t (private table TMAX x 8 points).  `slices` threads per
// round: the four digit slices of lambda, and (slices = 5) the batched
// check's sum_j r_j sig_j.
template <int TMAX>
__global__ void __launch_bounds__(256, 2) k_recover_msm_w4(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                         const uint32_t* __restrict__ sel,
                                                         const uint64_t* __restrict__ digits,
                                                         const uint32_t* __restrict__ sig_pts, size_t n_items,
                                                         uint32_t* __restrict__ part, int slices) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)slices * n_rounds) return;
  const size_t r = g / slices;
  const int i = (int)(g % slices);
  if (!ok[r] || t > TMAX) return;
  const uint64_t* d = digits + r * RECOVER_MAX_T * RECOVER_SLOTS + i;
  const uint32_t* sl = sel + r * RECOVER_MAX_T;
  g2j T[TMAX][8];
#pragma unroll 1
  for (int j = 0; j < t; ++j) {
    const g2a q = ld_g2a(sig_pts, n_items, sl[j]);
    T[j][0] = g2_from_affine(q);
    T[j][1] = g2_dbl_body(T[j][0]);
#pragma unroll 1
    for (int m = 2; m < 8; ++m) T[j][m] = g2_add_affine_body(T[j][m - 1], q);
  }
  g2j acc = g2_infinity();
#pragma unroll 1
  for (int w = 16; w >= 0; --w) {
    if (w < 16) {
#pragma unroll 1
      for (int s = 0; s < 4; ++s) acc = g2_dbl_body(acc);
    }
#pragma unroll 1
    for (int j = 0; j < t; ++j) {
      const int dg = win4_digit64(d[RECOVER_SLOTS * j], w);
      const int mag = dg < 0 ? -dg : dg;
      g2j e = T[j][(mag - 1) & 7];
      e.y = fp2_cmov(e.y, fp2_neg(e.y), dg < 0);
      acc = g2_cmov(acc, g2_add_body(acc, e), mag != 0);
    }
  }
  st_g2j(part + (size_t)i * G2J_WORDS * n_rounds, n_rounds, r, acc);
}

// Batched-check MSM with shared window tables.  k_recover_tables: one
// thread per (round, candidate j) builds [1..8] sig_j once (1 doubling + 6
// mixed additions, Jacobian; rounds not on the batched check write the
// identity-free placeholder (0, 0, 1) so the batch inversion stays sound),
// k_g2_batch_affine turns every entry affine, and k_recover_msm_aff's
// `slices` threads per round (the four base-|x| slices of lambda and the RLC
// coefficients) run their signed radix-16 windows with mixed additions over
// the shared affine entries -- the table is built once per point instead
// of once per slice, and every window addition is a mixed one.
// Table layout: entry (r, j, m) = [m + 1] sig_j at index (r * t + j) * 8 + m
// of a G2 SoA (X, Y in tab, Z in tabz).
__global__ void __launch_bounds__(256, 2) k_recover_tables(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                        const uint32_t* __restrict__ sel,
                                                        const uint32_t* __restrict__ sig_pts, size_t n_items,
                                                        uint32_t* __restrict__ tab, uint32_t* __restrict__ tabz) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rounds * (size_t)t) return;
  const size_t r = g / t;
  const int j = (int)(g % t);
  const size_t N = n_rounds * (size_t)t * 8;
  auto put = [&](int m, const g2j& p) {
    const size_t e = g * 8 + m;
    st_g2a(tab, N, e, g2a{p.x, p.y});
    st_fp(tabz, N, e, p.z.c0);
    st_fp(tabz + FP_WORDS * N, N, e, p.z.c1);
  };
  if (!ok[r]) {
    const g2j ph{fp2_zero(), fp2_zero(), fp2_one()};
#pragma unroll 1
    for (int m = 0; m < 8; ++m) put(m, ph);
    return;
  }
  const g2a q = ld_g2a(sig_pts, n_items, sel[r * RECOVER_MAX_T + j]);
  g2j acc = g2_from_affine(q);
  put(0, acc);
  acc = g2_dbl_body(acc);
  put(1, acc);
#pragma unroll 1
  for (int m = 2; m < 8; ++m) {
    acc = g2_add_affine_body(acc, q);
    put(m, acc);
  }
}

// The affine table entries transposed to rows (AoS, G2A_WORDS = 56 words,
// 224 contiguous bytes: x.c0, x.c1, y.c0, y.c1), one thread per entry: the
// window additions gather one row (two cache lines) per entry instead of
// one word from each of 56 SoA planes (the RLC root MSM's layout, k_msm_aos).
__global__ void __launch_bounds__(256) k_recover_tab_rows(size_t ne, const uint32_t* __restrict__ tab,
                                                          uint32_t* __restrict__ rows) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  const g2a q = ld_g2a(tab, ne, e);
  uint4* o = reinterpret_cast<uint4*>(rows + e * G2A_WORDS);
  const fp* c[4] = {&q.x.c0, &q.x.c1, &q.y.c0, &q.y.c1};
#pragma unroll
  for (int k = 0; k < G2A_WORDS / 4; ++k) {
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = c[(4 * k + u) / FP_LIMBS]->l[(4 * k + u) % FP_LIMBS];
    o[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
__device__ __forceinline__ g2a recover_ld_row(const uint32_t* __restrict__ rows, size_t e) {
  const uint4* p = reinterpret_cast<const uint4*>(rows + e * G2A_WORDS);
  g2a q;
  fp* c[4] = {&q.x.c0, &q.x.c1, &q.y.c0, &q.y.c1};
#pragma unroll
  for (int k = 0; k < G2A_WORDS / 4; ++k) {
    const uint4 v = p[k];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) c[(4 * k + u) / FP_LIMBS]->l[(4 * k + u) % FP_LIMBS] = w[u];
  }
  return q;
}

// One window-table entry of the recovery MSM, signed, each coordinate loaded
// where the addition uses it (the base passes through an empty asm per fetch:
// not hoisted and spilled).  ROWS: 224-byte rows, else the SoA planes.
template <bool ROWS>
struct rec_entry_fetch {
  const uint32_t* tab;
  size_t N, ei;
  bool neg;
  __device__ __forceinline__ const uint32_t* b() const {
    const uint32_t* p = tab;
    __asm__ volatile("" : "+s"(p));
    return p;
  }
  __device__ __forceinline__ fp2 x() const {
    if (ROWS) {
      const g2a q = recover_ld_row(b(), ei);
      return q.x;
    }
    return fp2{ld_fp(b(), N, ei), ld_fp(b() + FP_WORDS * N, N, ei)};
  }
  __device__ __forceinline__ fp2 y() const {
    fp2 y;
    if (ROWS) {
      y = recover_ld_row(b(), ei).y;
    } else {
      y = fp2{ld_fp(b() + 2 * FP_WORDS * N, N, ei), ld_fp(b() + 3 * FP_WORDS * N, N, ei)};
    }
    return fp2_cmov(y, fp2_neg(y), neg);
  }
  __device__ __forceinline__ g2a get() const { return g2a{x(), y()}; }
};

// ROWS: the table as rows (k_recover_tab_rows), else the SoA planes.
// FAST (round 6): the cofactor ladder's structure -- lazy doublings (Z
// reduced once per window), fast mixed additions of the fetched entry (the
// identity accumulator handled by a select: acc = e), no call site in the
// loops; an exceptional addition (acc = +-e) redoes the slice with the
// generic mixed addition.
template <bool ROWS>
__global__ void __launch_bounds__(256, 2) k_recover_msm_aff(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                          const uint64_t* __restrict__ digits,
                                                          const uint32_t* __restrict__ tab,
                                                          uint32_t* __restrict__ part, int slices) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)slices * n_rounds) return;
  const size_t r = g / slices;
  const int i = (int)(g % slices);
  if (!ok[r]) return;
  const uint64_t* d = digits + r * RECOVER_MAX_T * RECOVER_SLOTS + i;
  const size_t N = n_rounds * (size_t)t * 8;
  const size_t base = r * (size_t)t * 8;
  bool exc = false;
  g2j acc = g2_infinity();
#ifndef DG_RECOVER_MSM_GENERIC
#pragma unroll 1
  for (int w = 16; w >= 0; --w) {
    if (w < 16) {
#pragma unroll 1
      for (int s = 0; s < 4; ++s) acc = G2_LADDER_DBL(acc);
      acc = G2_LADDER_ZRED(acc);
    }
#pragma unroll 1
    for (int j = 0; j < t; ++j) {
      const int dg = win4_digit64(d[RECOVER_SLOTS * j], w);
      const int mag = dg < 0 ? -dg : dg;
      const rec_entry_fetch<ROWS> f{tab, N, base + (size_t)j * 8 + ((mag - 1) & 7), dg < 0};
      const bool ainf = g2_is_inf(acc);
      bool ex = false;
      g2j sum = g2_madd_nx_q(acc, f, ex);
      if (ainf) sum = g2_from_affine(f.get());  // only before the slice's first nonzero digit
      exc = exc || (ex && !ainf && mag != 0);
      acc = g2_cmov(acc, sum, mag != 0);
    }
  }
#else
  exc = true;
#endif
  if (exc || DG_FORCE_EXC) {  // the generic mixed addition (rounds 2-5): exceptional cases resolved
    acc = g2_infinity();
#pragma unroll 1
    for (int w = 16; w >= 0; --w) {
      if (w < 16) {
#pragma unroll 1
        for (int s = 0; s < 4; ++s) acc = g2_dbl_body(acc);
      }
#pragma unroll 1
      for (int j = 0; j < t; ++j) {
        const int dg = win4_digit64(d[RECOVER_SLOTS * j], w);
        const int mag = dg < 0 ? -dg : dg;
        const size_t ei = base + (size_t)j * 8 + ((mag - 1) & 7);
        g2a e = ROWS ? recover_ld_row(tab, ei) : ld_g2a(tab, N, ei);
        e.y = fp2_cmov(e.y, fp2_neg(e.y), dg < 0);
        acc = g2_cmov(acc, g2_add_affine_body(acc, e), mag != 0);
      }
    }
  }
  st_g2j(part + (size_t)i * G2J_WORDS * n_rounds, n_rounds, r, acc);
}

// slices = 5 (batched check): rec_pts gets B = sigma + sum_j r_j sig_j
// instead of sigma, and rec_st whether B is the identity.
__global__ void __launch_bounds__(64) k_recover_finish(size_t n_rounds, const uint8_t* __restrict__ ok,
                                                       const uint32_t* __restrict__ part, uint8_t* __restrict__ out96,
                                                       uint32_t* __restrict__ rec_pts, uint8_t* __restrict__ rec_st,
                                                       int slices) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds || !ok[r]) return;
  const g2j p0 = ld_g2j(part, n_rounds, r);
  const g2j p1 = ld_g2j(part + G2J_WORDS * n_rounds, n_rounds, r);
  const g2j p2 = ld_g2j(part + 2 * G2J_WORDS * n_rounds, n_rounds, r);
  const g2j p3 = ld_g2j(part + 3 * G2J_WORDS * n_rounds, n_rounds, r);
  g2j acc = g2_add(p0, g2_neg(g2_psi(p1)));
  acc = g2_add(acc, g2_psi2(p2));
  acc = g2_add(acc, g2_neg(g2_psi(g2_psi2(p3))));
  const bool inf = g2_is_inf(acc);
  const g2a a = inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(acc);
  g2_compress(out96 + r * 96, a, inf);
  if (slices == 5) {
    const g2j b = g2_add(acc, ld_g2j(part + 4 * G2J_WORDS * n_rounds, n_rounds, r));
    const bool binf = g2_is_inf(b);
    st_g2a(rec_pts, n_rounds, r, binf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(b));
    rec_st[r] = binf ? (uint8_t)ST_INFINITY : (uint8_t)ST_OK;
    return;
  }
  st_g2a(rec_pts, n_rounds, r, a);
  rec_st[r] = inf ? (uint8_t)ST_INFINITY : (uint8_t)ST_OK;
}

// VerifyRecovered verdicts (chain/beacon/chain.go:165): a recovered signature
// that does not verify under C_0 is dropped like a failed recovery.
__global__ void __launch_bounds__(256) k_recover_verdict(size_t n_rounds, const uint8_t* __restrict__ rec_st,
                                                         uint8_t* __restrict__ out96, uint8_t* __restrict__ ok) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds || !ok[r] || rec_st[r] == ST_OK) return;
  ok[r] = 0;
  for (int k = 0; k < 96; ++k) out96[r * 96 + k] = 0;
}

// ================================================================ batched check
// Window table of the share keys for the batched check: entry (i, m) =
// [m + 1] PubPoly.Eval(i) affine, i < n (AoS: x limbs then y limbs), from
// the (-x, y) Eval table; an identity Eval (y = 0 marks it: G1 has no 2-torsion)
// stores zeros.  One thread per entry, once per group (dgpu_set_group).
constexpr int REC_WTAB_WORDS = 2 * FP_LIMBS;
__global__ void k_pubpoly_wtable(int n, const uint32_t* __restrict__ table, uint32_t* __restrict__ wtab) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 8 * n) return;
  const int i = g >> 3;
  const uint32_t k = (uint32_t)(g & 7) + 1;
  const fp nx = ld_fp(table, n, i), y = ld_fp(table + FP_LIMBS * n, n, i);
  g1a a{fp_zero(), fp_zero()};
  if (!fp_is_zero(y)) {
    const g1j q = g1_mul_words(g1j{fp_neg(nx), y, fp_one()}, &k, 1);
    if (!g1_is_inf(q)) a = g1_to_affine(q);
  }
  uint32_t* o = wtab + (size_t)g * REC_WTAB_WORDS;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) {
    o[l] = a.x.l[l];
    o[FP_LIMBS + l] = a.y.l[l];
  }
}

// Per round: the candidates = the first t partials that decode (status
// ST_OK after k_decode_partials), in input order, duplicates included (the
// reference counts every verified partial towards t), and the class:
//   fewer than t candidates      -> REC_FAIL (the reference finds fewer than t
//                                   good ones whatever the pairings say)
//   t candidates, an index twice -> REC_FAIL if nothing decodable is left,
//                                   else REC_EXACT (validity decides which)
//   t distinct candidates        -> REC_RLC (batched check), ok = 1 for now
// with want_status every round whose per-partial statuses need pairings
// (decodable partials that are not checked candidates) goes REC_EXACT.
__global__ void __launch_bounds__(64) k_recover_cand(size_t n_rounds, size_t m, int t, int want_status,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint8_t* __restrict__ status, uint32_t* __restrict__ sel,
                                                     uint32_t* __restrict__ xs, uint8_t* __restrict__ cls,
                                                     uint8_t* __restrict__ ok, uint8_t* __restrict__ out96) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds) return;
  uint32_t ids[RECOVER_MAX_T];
  uint32_t* sl = sel + r * RECOVER_MAX_T;
  int cnt = 0;
  bool more = false;
  for (size_t j = 0; j < m; ++j) {
    const size_t item = r * m + j;
    if (status[item] != ST_OK) continue;
    if (cnt == t) {
      more = true;
      break;
    }
    sl[cnt] = (uint32_t)item;
    ids[cnt] = idx[item];
    ++cnt;
  }
  bool distinct = cnt == t;
  for (int a = 0; a < cnt && distinct; ++a)
    for (int b = 0; b < a; ++b) distinct = distinct && ids[a] != ids[b];
  uint8_t c;
  if (cnt < t)
    c = (want_status && cnt > 0) ? REC_EXACT : REC_FAIL;
  else if (!distinct)
    c = (more || want_status) ? REC_EXACT : REC_FAIL;
  else
    c = (want_status && more) ? REC_EXACT : REC_RLC;
  if (c == REC_RLC)
    for (int k = 0; k < t; ++k) xs[r * RECOVER_MAX_T + k] = ids[k] + 1;
  cls[r] = c | (more ? REC_MORE : 0);
  ok[r] = c == REC_RLC ? 1 : 0;
  if (c == REC_FAIL)
    for (int k = 0; k < 96; ++k) out96[r * 96 + k] = 0;
}

// The batched check's G1 side, per REC_RLC round: A = C_0 + sum_j r_j
// Eval(i_j) (Straus, signed radix-16 windows over the group's window table,
// the same operation sequence in every lane), stored as the engine's pair-0
// key (-x, y); rec_st combines A with B's identity flag from
// k_recover_finish (both identity: trivially equal; one: fails).  A
// candidate index without a table entry (i >= n) sends the round REC_EXACT.
__global__ void __launch_bounds__(64, 2) k_recover_rlc_g1(size_t n_rounds, int t, int n_group,
                                                       const uint32_t* __restrict__ sel,
                                                       const uint32_t* __restrict__ idx,
                                                       const uint64_t* __restrict__ digits,
                                                       const uint32_t* __restrict__ wtab,
                                                       const uint32_t* __restrict__ commits, uint8_t* __restrict__ cls,
                                                       uint8_t* __restrict__ ok, uint32_t* __restrict__ rec_pk,
                                                       uint8_t* __restrict__ rec_st) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds || (cls[r] & 0x0F) != REC_RLC) return;
  const uint32_t* sl = sel + r * RECOVER_MAX_T;
  const uint64_t* d = digits + r * RECOVER_MAX_T * RECOVER_SLOTS + 4;
  bool table_ok = true;
  for (int j = 0; j < t; ++j) table_ok = table_ok && idx[sl[j]] < (uint32_t)n_group;
  if (!table_ok) {
    cls[r] = (uint8_t)((cls[r] & REC_MORE) | REC_EXACT);
    ok[r] = 0;
    rec_st[r] = ST_DECODE;
    return;
  }
  g1j acc = g1_infinity();
#pragma unroll 1
  for (int w = 16; w >= 0; --w) {
    if (w < 16) {
#pragma unroll 1
      for (int s = 0; s < 4; ++s) acc = g1_dbl_body(acc);
    }
#pragma unroll 1
    for (int j = 0; j < t; ++j) {
      const int dg = win4_digit64(d[RECOVER_SLOTS * j], w);
      const int mag = dg < 0 ? -dg : dg;
      const uint32_t* e = wtab + ((size_t)idx[sl[j]] * 8 + ((mag - 1) & 7)) * REC_WTAB_WORDS;
      g1a q;
#pragma unroll
      for (int l = 0; l < FP_LIMBS; ++l) {
        q.x.l[l] = e[l];
        q.y.l[l] = e[FP_LIMBS + l];
      }
      const bool qinf = fp_is_zero(q.y);
      q.y = fp_cmov(q.y, fp_neg(q.y), dg < 0);
      acc = g1_cmov(acc, g1_add_affine_body(acc, q), mag != 0 && !qinf);
    }
  }
  const g1a c0{ld_fp(commits, t, 0), ld_fp(commits + FP_LIMBS * t, t, 0)};
  acc = g1_add_affine_body(acc, c0);
  const bool ainf = g1_is_inf(acc);
  const bool binf = rec_st[r] == ST_INFINITY;
  const g1a a = ainf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(acc);
  st_fp(rec_pk, n_rounds, r, fp_neg(a.x));
  st_fp(rec_pk + FP_LIMBS * n_rounds, n_rounds, r, a.y);
  rec_st[r] = (ainf && binf) ? RLC_TRIVIAL : (ainf || binf) ? (uint8_t)ST_PAIRING : (uint8_t)ST_OK;
}

// The batched check's verdict per REC_RLC round: pass -> recovered (out96
// already holds sigma); fail -> REC_EXACT when a decodable partial is left
// beyond the candidates (the reference walks on to it) or the per-partial
// statuses are wanted (which candidate failed), else a failure.
__global__ void __launch_bounds__(256) k_recover_rlc_verdict(size_t n_rounds, int want_status,
                                                             const uint8_t* __restrict__ rec_st,
                                                             uint8_t* __restrict__ cls, uint8_t* __restrict__ ok,
                                                             uint8_t* __restrict__ out96) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rounds || (cls[r] & 0x0F) != REC_RLC) return;
  if (rec_st[r] == ST_OK || rec_st[r] == RLC_TRIVIAL) return;
  ok[r] = 0;
  if ((cls[r] & REC_MORE) || want_status) {
    cls[r] = REC_MORE | REC_EXACT;
    return;
  }
  cls[r] = REC_FAIL;
  for (int k = 0; k < 96; ++k) out96[r * 96 + k] = 0;
}

// Rounds list[0..nx) of a recovery batch -> a compact batch (messages,
// partial slots, lengths): one thread per (round, slot).
__global__ void __launch_bounds__(256) k_gather_rounds(size_t nx, const uint32_t* __restrict__ list, size_t m,
                                                       size_t stride, const uint8_t* __restrict__ msgs,
                                                       const uint8_t* __restrict__ parts,
                                                       const uint32_t* __restrict__ plen, uint8_t* __restrict__ x_msgs,
                                                       uint8_t* __restrict__ x_parts, uint32_t* __restrict__ x_plen) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nx * m) return;
  const size_t k = g / m, j = g % m, r = list[k];
  const uint8_t* src = parts + (r * m + j) * stride;
  uint8_t* dst = x_parts + g * stride;
  for (size_t b = 0; b < stride; ++b) dst[b] = src[b];
  x_plen[g] = plen[r * m + j];
  if (j == 0)
    for (int b = 0; b < 32; ++b) x_msgs[k * 32 + b] = msgs[r * 32 + b];
}

// The compact batch's results back to their rounds (status optional).
__global__ void __launch_bounds__(256) k_scatter_rounds(size_t nx, const uint32_t* __restrict__ list, size_t m,
                                                        const uint8_t* __restrict__ x_out, const uint8_t* __restrict__ x_ok,
                                                        const uint8_t* __restrict__ x_st, uint8_t* __restrict__ out96,
                                                        uint8_t* __restrict__ ok, uint8_t* __restrict__ status) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nx * m) return;
  const size_t k = g / m, j = g % m, r = list[k];
  if (status) status[r * m + j] = x_st[g];
  if (j == 0) {
    ok[r] = x_ok[k];
    for (int b = 0; b < 96; ++b) out96[r * 96 + b] = x_out[k * 96 + b];
  }
}

}  // namespace dgpu
