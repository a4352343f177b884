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
#pragma once
#include "fr.cuh"
#include "kernels.cuh"

namespace dgpu {

constexpr int RECOVER_MAX_T = 32;

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
__global__ void __launch_bounds__(256) k_decode_partials(size_t n_items, const uint8_t* __restrict__ partials,
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
  if (len >= 2) {
    idx = ((uint32_t)src[0] << 8) | src[1];
    if (len == 98) {
      uint8_t buf[96];
      for (int k = 0; k < 96; ++k) buf[k] = src[2 + k];
      const int rc = g2_decompress(&p, buf, true);
      st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
    }
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
  st_g2a(sig_pts, n_items, i, p);
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

__global__ void __launch_bounds__(256) k_recover_lagrange(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                          const uint32_t* __restrict__ xs,
                                                          uint64_t* __restrict__ digits) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rounds * RECOVER_MAX_T) return;
  const size_t r = g / RECOVER_MAX_T;
  const int j = (int)(g % RECOVER_MAX_T);
  if (j >= t || !ok[r]) return;
  uint32_t w[8];
  fr_lagrange_at_zero(xs + r * RECOVER_MAX_T, t, j, w);
  uint64_t* d = digits + g * 4;
  d[0] = div_absx(w);
  d[1] = div_absx(w);
  d[2] = div_absx(w);
  d[3] = ((uint64_t)w[1] << 32) | w[0];  // the last quotient, < |x| since lambda < r < |x|^4
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
  const uint64_t* d = digits + r * RECOVER_MAX_T * 4 + i;
  const uint32_t* sl = sel + r * RECOVER_MAX_T;
  g2j acc = g2_infinity();
  for (int b = 63; b >= 0; --b) {
    acc = g2_dbl_body(acc);
    for (int j = 0; j < t; ++j)
      if ((d[4 * j] >> b) & 1ull) acc = g2_add_affine_body(acc, ld_g2a(sig_pts, n_items, sl[j]));
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
// TMAX bounds t (private table TMAX x 8 points).
template <int TMAX>
__global__ void __launch_bounds__(256, 2) k_recover_msm_w4(size_t n_rounds, int t, const uint8_t* __restrict__ ok,
                                                         const uint32_t* __restrict__ sel,
                                                         const uint64_t* __restrict__ digits,
                                                         const uint32_t* __restrict__ sig_pts, size_t n_items,
                                                         uint32_t* __restrict__ part) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 4 * n_rounds) return;
  const size_t r = g >> 2;
  const int i = (int)(g & 3);
  if (!ok[r] || t > TMAX) return;
  const uint64_t* d = digits + r * RECOVER_MAX_T * 4 + i;
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
      const int dg = win4_digit64(d[4 * j], w);
      const int mag = dg < 0 ? -dg : dg;
      g2j e = T[j][(mag - 1) & 7];
      e.y = fp2_cmov(e.y, fp2_neg(e.y), dg < 0);
      acc = g2_cmov(acc, g2_add_body(acc, e), mag != 0);
    }
  }
  st_g2j(part + (size_t)i * G2J_WORDS * n_rounds, n_rounds, r, acc);
}

__global__ void __launch_bounds__(64) k_recover_finish(size_t n_rounds, const uint8_t* __restrict__ ok,
                                                       const uint32_t* __restrict__ part, uint8_t* __restrict__ out96,
                                                       uint32_t* __restrict__ rec_pts, uint8_t* __restrict__ rec_st) {
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

}  // namespace dgpu
