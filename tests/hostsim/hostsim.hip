// TEST-ONLY host build of the kernels' arithmetic (drand_amd/csrc/*.cuh are
// __host__ __device__).  Lets the CPU test suite check the exact code the
// GPU runs against the oracle without a GPU.  Not part of the product:
// libdrand_gpu.so never links or loads this; it is built into
// tests/hostsim/libdrand_hostsim.so by __graft_entry__.build().
#include <cstring>
#include "../../drand_amd/csrc/h2c.cuh"
#include "../../drand_amd/csrc/pairing.cuh"
#define DG_NO_KERNELS
#include "../../drand_amd/csrc/g1sig.cuh"
#include "../../drand_amd/csrc/group_ops.cuh"
#include "../../drand_amd/csrc/lines_thread.cuh"
#include "../../drand_amd/csrc/kb_thread.cuh"

using namespace dgpu;

#ifdef DG_COUNT_OPS
unsigned long long dg_count_mul = 0, dg_count_sqr = 0;
#endif

static void fp_to_be(const fp& a, uint8_t* out) { fp_std_to_be48(fp_from_mont(a), out); }
static fp fp_from_be(const uint8_t* in) { return fp_to_mont(fp_std_from_be48(in)); }

// k_h2c_finish's point slots (kernels.cuh h2c_finish_stash) in host memory
struct hs_stash {
  g2j s[3];
  void put(int k, const g2j& p) { s[k] = p; }
  g2j get(int k) const { return s[k]; }
  g2j_q at(int k) const { return g2j_q{s[k]}; }
};

extern "C" {

// per-stage Fp mul/sqr counts of one per-round verification (DG_COUNT_OPS builds)
int hs_count_stages(const uint8_t* pk48, const uint8_t* prev, uint32_t prev_len, uint64_t round,
                    const uint8_t* sig96, unsigned long long* out /* 8: mul,sqr for hash,decode,miller,fexp */) {
#ifdef DG_COUNT_OPS
  g1a pk;
  if (g1_decompress(&pk, pk48, GROUP_ORDER_WORDS) != DEC_OK) return -1;
  uint32_t m[8];
  dg_count_mul = dg_count_sqr = 0;
  drand_digest(m, prev, prev_len, round);
  g2a h = g2_to_affine(hash_to_g2(m));
  out[0] = dg_count_mul; out[1] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  g2a s;
  int rc = g2_decompress(&s, sig96, true);
  out[2] = dg_count_mul; out[3] = dg_count_sqr;
  if (rc != DEC_OK) return -2;
  dg_count_mul = dg_count_sqr = 0;
  fp12 f = miller_loop_2(h, fp_neg(pk.x), pk.y, s, fp_neg(C_G1_X), C_G1_NEG_Y);
  out[4] = dg_count_mul; out[5] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  bool ok = fp12_is_one(final_exponentiation(f));
  out[6] = dg_count_mul; out[7] = dg_count_sqr;
  return ok ? 0 : 3;
#else
  return -100;
#endif
}

// Fp mul/sqr counts of k_lines_thr per round (DG_COUNT_OPS builds): both
// pairs' 68 T-steps (lines_thread.cuh lt_pair) and the fused membership test.
int hs_count_lines_thr(const uint8_t* sig96, unsigned long long* out) {
#ifdef DG_COUNT_OPS
  g2a s;
  if (g2_decompress(&s, sig96, false) != DEC_OK) return -1;
  const g2a h{C_G2_X, C_G2_Y};
  dg_count_mul = dg_count_sqr = 0;
  lt_pair(h, fp_neg(C_G1_X), C_G1_Y, [](int, const line3&) {});
  const g2p T = lt_pair(s, fp_neg(C_G1_X), C_G1_NEG_Y, [](int, const line3&) {});
  const bool in = lt_in_g2(T, s);
  out[0] = dg_count_mul; out[1] = dg_count_sqr;
  return in ? 0 : -2;
#else
  return -100;
#endif
}

// Fp mul/sqr counts of k_kb_chain_thr per exponentiation (DG_COUNT_OPS builds).
int hs_count_kb_chain_thr(unsigned long long* out) {
#ifdef DG_COUNT_OPS
  const fp2 a{fp_one(), fp_one()};
  dg_count_mul = dg_count_sqr = 0;
  kb_chain_thr(a, a, a, a, [](int, const fp2&, const fp2&, const fp2&, const fp2&) {});
  out[0] = dg_count_mul; out[1] = dg_count_sqr;
  return 0;
#else
  return -100;
#endif
}

// Per-kernel Fp mul/sqr counts of the per-round pipeline as the device runs
// it (DG_COUNT_OPS builds): out[0..7] = mul,sqr of k_h2c_field, k_h2c_sswu
// (both of a round's items), k_h2c_finish, k_decode_g2_sigs (membership left
// to k_eng_lines, check_subgroup = 0).
int hs_count_kernels(const uint8_t* prev, uint32_t prev_len, uint64_t round, const uint8_t* sig96,
                     unsigned long long* out) {
#ifdef DG_COUNT_OPS
  uint32_t m[8];
  drand_digest(m, prev, prev_len, round);
  fp2 u0, u1;
  dg_count_mul = dg_count_sqr = 0;
  hash_to_field_g2(u0, u1, m);
  out[0] = dg_count_mul; out[1] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  const g2j q0 = map_to_curve_sswu_iso3_body(u0), q1 = map_to_curve_sswu_iso3_body(u1);
  out[2] = dg_count_mul; out[3] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  hs_stash st;
  bool exc = false;
  const g2j h = g2_clear_cofactor_stash(q0, q1, st, exc);
  out[4] = dg_count_mul; out[5] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  g2a s;
  const int rc = g2_decompress(&s, sig96, false);
  out[6] = dg_count_mul; out[7] = dg_count_sqr;
  return rc == DEC_OK && !g2_is_inf(h) ? 0 : -1;
#else
  return -100;
#endif
}

static void msg_words(const uint8_t* msg32, uint32_t m[8]);

// Per-item Fp mul/sqr counts of the RLC and on-G1 pipelines' kernels
// (DG_COUNT_OPS builds), out[2k], out[2k+1] = mul, sqr of:
//   k=0 rlc hash: k_h2c_field + k_h2c_sswu (both items) + k_h2c_sum
//   k=1 k_decode_g2_sigs with the membership check (RLC needs it up front)
//   k=2 one RLC leaf: g2_mul2_win4_affine (k_rlc_leaves; two per round)
//   k=3 one tree node: g2_add_body (k_rlc_level; about two per round)
//   k=4 k_g2_batch_affine per point (a 16-point group's share of the inversion)
//   k=5 k_hash_to_g1_beacons (expand under the G2 suite's DST + SSWU/iso-11 + h_eff)
//   k=6 k_decode_g1_sigs (decode + endomorphism membership)
//   k=7 k_g1_batch_affine per point
//   k=8 k_hash_to_g1_raw (RLC, G1 signatures: no cofactor clearing)
//   k=9 one G1 RLC leaf: mul2_win4_affine<G1Ops> (k_rlc_leaves<G1Ops>; two per round)
//   k=10 one G1 tree node: g1_add_body (k_rlc_level<G1Ops>; about two per round)
int hs_count_extra(const uint8_t* msg32, const uint8_t* sig96, const uint8_t* sig48, uint64_t coeff,
                   unsigned long long* out) {
#ifdef DG_COUNT_OPS
  uint32_t m[8];
  msg_words(msg32, m);
  fp2 u0, u1;
  dg_count_mul = dg_count_sqr = 0;
  hash_to_field_g2(u0, u1, m);
  const g2j R = g2_add_body(map_to_curve_sswu_iso3_body(u0), map_to_curve_sswu_iso3_body(u1));
  out[0] = dg_count_mul; out[1] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  g2a s;
  if (g2_decompress(&s, sig96, true) != DEC_OK) return -1;
  out[2] = dg_count_mul; out[3] = dg_count_sqr;
  const g2a Ra = g2_to_affine(R);
  dg_count_mul = dg_count_sqr = 0;
  const g2j leaf = g2_mul2_win4_affine(Ra, (uint32_t)coeff, (uint32_t)(coeff >> 32));
  out[4] = dg_count_mul; out[5] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  (void)g2_add_body(leaf, leaf);
  out[6] = dg_count_mul; out[7] = dg_count_sqr;
  // k_g2_batch_affine over a 16-point group: prefix products, one inversion,
  // the backward pass (the kernel's loop bodies)
  {
    const int G = 16;
    fp2 zs[G];
    for (int i = 0; i < G; ++i) zs[i] = fp2_add(R.z, fp2{fp_one(), fp_zero()});
    dg_count_mul = dg_count_sqr = 0;
    fp pre[G], acc = fp_one();
    for (int i = 0; i < G; ++i) { acc = fp_mul(acc, fp2_norm(zs[i])); pre[i] = acc; }
    fp inv = fp_inv(acc);
    for (int i = G - 1; i >= 0; --i) {
      const fp nz = fp2_norm(zs[i]);
      const fp ninv = i ? fp_mul(inv, pre[i - 1]) : inv;
      const fp2 zinv = fp2_mul_fp(fp2_conj(zs[i]), ninv);
      const fp2 zinv2 = fp2_sqr(zinv);
      (void)fp2_mul(Ra.x, zinv2);
      (void)fp2_mul(Ra.y, fp2_mul(zinv2, zinv));
      if (i) inv = fp_mul(inv, nz);
    }
    out[8] = (dg_count_mul + G / 2) / G; out[9] = (dg_count_sqr + G / 2) / G;
  }
  dg_count_mul = dg_count_sqr = 0;
  uint32_t uni[32];
  expand_xmd<false, 4>(uni, m);
  const g1j h1 = hash_to_g1_from_uni<true>(uni);
  out[10] = dg_count_mul; out[11] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  g1a s1;
  if (g1_decompress_sig(&s1, sig48) != DEC_OK) return -2;
  out[12] = dg_count_mul; out[13] = dg_count_sqr;
  {
    const int G = 16;
    dg_count_mul = dg_count_sqr = 0;
    fp pre[G], acc = fp_one();
    for (int i = 0; i < G; ++i) { acc = fp_mul(acc, h1.z); pre[i] = acc; }
    fp inv = fp_inv(acc);
    for (int i = G - 1; i >= 0; --i) {
      const fp zinv = i ? fp_mul(inv, pre[i - 1]) : inv;
      const fp zinv2 = fp_sqr(zinv);
      (void)fp_mul(h1.x, zinv2);
      (void)fp_mul(h1.y, fp_mul(zinv2, zinv));
      if (i) inv = fp_mul(inv, h1.z);
    }
    out[14] = (dg_count_mul + G / 2) / G; out[15] = (dg_count_sqr + G / 2) / G;
  }
  dg_count_mul = dg_count_sqr = 0;
  const g1j R1 = g1_add_body(map_to_curve_sswu_iso11_body(fp_from_be64_words(uni)),
                             map_to_curve_sswu_iso11_body(fp_from_be64_words(uni + 16)));
  out[16] = dg_count_mul; out[17] = dg_count_sqr;
  const g1a R1a = g1_to_affine(R1);
  dg_count_mul = dg_count_sqr = 0;
  const g1j leaf1 = mul2_win4_affine<G1Ops>(R1a, (uint32_t)coeff, (uint32_t)(coeff >> 32));
  out[18] = dg_count_mul; out[19] = dg_count_sqr;
  dg_count_mul = dg_count_sqr = 0;
  (void)g1_add_body(leaf1, R1);
  out[20] = dg_count_mul; out[21] = dg_count_sqr;
  return 0;
#else
  (void)msg32; (void)sig96; (void)sig48; (void)coeff; (void)out;
  return -100;
#endif
}

// Group-law op counts (DG_COUNT_OPS builds): out[2k], out[2k+1] = mul, sqr of
// k=0 g2_dbl_body, 1 g2_add_body, 2 g2_add_affine_body, 3 g1_dbl_body,
// 4 g1_add_affine_body, 5 g2_psi, 6 g2_to_affine -- the terms of the recovery
// MSM's work figure (recover.cuh k_recover_msm_w4 / k_recover_rlc_g1).
int hs_count_group_ops(const uint8_t* msg32, unsigned long long* out) {
#ifdef DG_COUNT_OPS
  uint32_t m[8];
  msg_words(msg32, m);
  const g2j P = hash_to_g2(m);
  const g2j Q = g2_dbl(P);
  const g2a Qa = g2_to_affine(Q);
  const g1j G{C_G1_X, C_G1_Y, fp_one()};
  const g1j G2x = g1_dbl(G);
  const g1a Ga = g1_to_affine(G2x);
#define CNT(k, expr) dg_count_mul = dg_count_sqr = 0; (void)(expr); out[2 * (k)] = dg_count_mul; out[2 * (k) + 1] = dg_count_sqr;
  CNT(0, g2_dbl_body(Q));
  CNT(1, g2_add_body(P, Q));
  CNT(2, g2_add_affine_body(P, Qa));
  CNT(3, g1_dbl_body(G));
  CNT(4, g1_add_affine_body(G, Ga));
  CNT(5, g2_psi(Q));
  CNT(6, g2_to_affine(Q));
#undef CNT
  return 0;
#else
  (void)msg32; (void)out;
  return -100;
#endif
}

// a*b, a+b, a-b, a^2 on canonical 48-byte big-endian inputs
int hs_fp_ops(const uint8_t* a48, const uint8_t* b48, uint8_t* mul, uint8_t* add, uint8_t* sub, uint8_t* sqr,
              uint8_t* inv) {
  fp a = fp_from_be(a48), b = fp_from_be(b48);
  fp_to_be(fp_mul(a, b), mul);
  fp_to_be(fp_add(a, b), add);
  fp_to_be(fp_sub(a, b), sub);
  fp_to_be(fp_sqr(a), sqr);
  fp_to_be(fp_inv(a), inv);
  return 0;
}

// fp_inv (divsteps) against fp_inv_pow (Fermat) on n pseudo-random CI inputs
// (values up to 2.01p, not reduced) and the edge values 0, p, 2p, 1, p - 1,
// 2^k (Montgomery words); returns the number of disagreements.
int hs_fp_inv_check(int n, uint64_t seed) {
  uint64_t s = seed | 1;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return s;
  };
  int bad = 0;
  auto check = [&](const fp& x) {
    fp a;
    if (!fp_inv_ds(x, a)) ++bad;  // the divstep path itself, no fallback
    const fp b = fp_inv_pow(x);
    if (!fp_is_zero(fp_sub(a, b))) ++bad;
    if (!fp_is_zero(x) && !fp_is_zero(fp_sub(fp_mul(a, x), fp_one()))) ++bad;
  };
  fp e = fp_zero();
  check(e);
  for (int i = 0; i < FP_LIMBS; ++i) e.l[i] = FP_P[i];
  check(e);
  for (int i = 0; i < FP_LIMBS; ++i) e.l[i] = FP_2P[i];
  check(e);
  e = fp_zero(), e.l[0] = 1;
  check(e);
  e = fp_zero(), e.l[0] = FP_P[0] - 1;
  for (int i = 1; i < FP_LIMBS; ++i) e.l[i] = FP_P[i];
  check(e);
  for (int k = 0; k < 381; k += 7) {
    e = fp_zero(), e.l[k / FP_BITS] = 1u << (k % FP_BITS);
    check(e);
  }
  for (int t = 0; t < n; ++t) {
    fp x;
    for (int i = 0; i < FP_LIMBS; ++i) x.l[i] = (uint32_t)next() & FP_MASK;
    x.l[FP_LIMBS - 1] &= (t & 1) ? 0x1FFFFu : 0x3FFFFu;  // < 2^381 or < 2^382 ...
    x = fp_reduce(x);                                     // ... into CI (< 2.01p)
    check(x);
  }
  return bad;
}

int hs_fp2_ops(const uint8_t* a96, const uint8_t* b96, uint8_t* mul, uint8_t* sqr, uint8_t* inv, uint8_t* sqrt_out,
               int* sqrt_ok) {
  fp2 a{fp_from_be(a96), fp_from_be(a96 + 48)}, b{fp_from_be(b96), fp_from_be(b96 + 48)};
  fp2 m = fp2_mul(a, b), s = fp2_sqr(a), iv = fp2_inv(a), r;
  fp_to_be(m.c0, mul); fp_to_be(m.c1, mul + 48);
  fp_to_be(s.c0, sqr); fp_to_be(s.c1, sqr + 48);
  fp_to_be(iv.c0, inv); fp_to_be(iv.c1, inv + 48);
  *sqrt_ok = fp2_sqrt(r, a) ? 1 : 0;
  fp_to_be(r.c0, sqrt_out); fp_to_be(r.c1, sqrt_out + 48);
  return 0;
}

void hs_digest(const uint8_t* prev, uint32_t prev_len, uint64_t round, uint8_t* out32) {
  uint32_t m[8];
  drand_digest(m, prev, prev_len, round);
  for (int w = 0; w < 8; ++w)
    for (int k = 0; k < 4; ++k) out32[4 * w + k] = (uint8_t)(m[w] >> (24 - 8 * k));
}

static void msg_words(const uint8_t* msg32, uint32_t m[8]) {
  for (int w = 0; w < 8; ++w)
    m[w] = ((uint32_t)msg32[4 * w] << 24) | ((uint32_t)msg32[4 * w + 1] << 16) | ((uint32_t)msg32[4 * w + 2] << 8) |
           msg32[4 * w + 3];
}

void hs_expand_xmd(const uint8_t* msg32, uint8_t* out256) {
  uint32_t m[8], o[64];
  msg_words(msg32, m);
  expand_xmd_g2(o, m);
  for (int w = 0; w < 64; ++w)
    for (int k = 0; k < 4; ++k) out256[4 * w + k] = (uint8_t)(o[w] >> (24 - 8 * k));
}

// u0, u1 (4 x 48 bytes canonical: u0.c0 u0.c1 u1.c0 u1.c1)
void hs_hash_to_field(const uint8_t* msg32, uint8_t* out192) {
  uint32_t m[8];
  msg_words(msg32, m);
  fp2 u0, u1;
  hash_to_field_g2(u0, u1, m);
  fp_to_be(u0.c0, out192); fp_to_be(u0.c1, out192 + 48); fp_to_be(u1.c0, out192 + 96); fp_to_be(u1.c1, out192 + 144);
}

// iso3(SSWU(u)) of u (96 bytes) -> affine x, y on E2 (4 x 48)
void hs_sswu(const uint8_t* u96, uint8_t* out192) {
  fp2 u{fp_from_be(u96), fp_from_be(u96 + 48)};
  g2a q = g2_to_affine(map_to_curve_sswu_iso3(u));
  fp_to_be(q.x.c0, out192); fp_to_be(q.x.c1, out192 + 48); fp_to_be(q.y.c0, out192 + 96); fp_to_be(q.y.c1, out192 + 144);
}

// hash to G1 (g1dst: RFC 9380 G1 DST, else the G2 suite's DST), compressed
void hs_hash_to_g1(const uint8_t* msg32, int g1dst, uint8_t* out48) {
  uint32_t m[8];
  msg_words(msg32, m);
  g1j h = hash_to_g1(m, g1dst != 0);
  bool inf = g1_is_inf(h);
  g1_compress(out48, inf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(h), inf);
}

// G1 signature decode (endomorphism membership test); recompressed on success
int hs_decompress_g1(const uint8_t* in48, uint8_t* recompressed) {
  g1a p{fp_zero(), fp_zero()};
  int rc = g1_decompress_sig(&p, in48);
  if (rc == DEC_OK) g1_compress(recompressed, p, false);
  return rc;
}

void hs_hash_to_g2(const uint8_t* msg32, uint8_t* out96) {
  uint32_t m[8];
  msg_words(msg32, m);
  g2j h = hash_to_g2(m);
  bool inf = g2_is_inf(h);
  g2a a = inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(h);
  g2_compress(out96, a, inf);
}

// k_h2c_finish's sequence (g2_clear_cofactor_stash, the generic
// g2_clear_cofactor from slot 0 when it flags an exceptional addition) on
// Q0, Q1 = SSWU(u0), SSWU(u1) of msg, with Q1 replaced by Q0 (mode 1) or -Q0
// (compared with g2_clear_cofactor_generic; hs_hash_to_g2 runs the register
// ladder form of g2_clear_cofactor)
// (mode 2, P = O) -- H compressed to out96 (the generic path's to gen96);
// returns the exceptional flag.
int hs_h2c_finish_check(const uint8_t* msg32, int mode, uint8_t* out96, uint8_t* gen96) {
  uint32_t m[8];
  msg_words(msg32, m);
  fp2 u0, u1;
  hash_to_field_g2(u0, u1, m);
  const g2j q0 = map_to_curve_sswu_iso3_body(u0);
  g2j q1 = map_to_curve_sswu_iso3_body(u1);
  if (mode == 1) q1 = q0;
  if (mode == 2) q1 = g2_neg(q0);
  hs_stash st;
  bool exc = false;
  g2j h = g2_clear_cofactor_stash(q0, q1, st, exc);
  if (exc) h = g2_clear_cofactor(st.get(0));
  const g2j g = g2_clear_cofactor_generic(g2_add(q0, q1));  // the round-5 form, every case resolved
  bool inf = g2_is_inf(h);
  g2_compress(out96, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(h), inf);
  inf = g2_is_inf(g);
  g2_compress(gen96, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(g), inf);
  return exc ? 1 : 0;
}

int hs_decompress_g2(const uint8_t* in96, uint8_t* recompressed) {
  g2a p{fp2_zero(), fp2_zero()};
  int rc = g2_decompress(&p, in96, true);
  if (rc == DEC_OK) g2_compress(recompressed, p, false);
  return rc;
}

// full verification of one signature: returns status code (0 = valid)
int hs_verify(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig96) {
  g1a pk;
  int rc = g1_decompress(&pk, pk48, GROUP_ORDER_WORDS);
  if (rc != DEC_OK) return 100 + rc;
  g2a s;
  rc = g2_decompress(&s, sig96, true);
  if (rc == DEC_INFINITY) return 4;
  if (rc == DEC_ERR_SUBGROUP) return 2;
  if (rc != DEC_OK) return 1;
  uint32_t m[8];
  msg_words(msg32, m);
  g2a h = g2_to_affine(hash_to_g2(m));
  fp12 f = miller_loop_2(h, fp_neg(pk.x), pk.y, s, fp_neg(C_G1_X), C_G1_NEG_Y);
  return fp12_is_one(final_exponentiation(f)) ? 0 : 3;
}

// reduced pairing e(P, Q) = FE(f) (with the 3x hard-part exponent), as 12 x 48 bytes
// in the oracle's f12_to_ints order
void hs_pairing(const uint8_t* p48, const uint8_t* q96, uint8_t* out576) {
  g1a p;
  g1_decompress(&p, p48, GROUP_ORDER_WORDS);
  g2a q;
  g2_decompress(&q, q96, false);
  // single pair: use the 2-pair loop with the second pair's line contribution
  // neutralized is not possible; instead run pair 2 as (P, Q) too and take sqrt? No:
  // compute f for (P,Q) twice -> e^2; callers compare against e(P,Q)^2.
  fp12 f = miller_loop_2(q, fp_neg(p.x), p.y, q, fp_neg(p.x), p.y);
  fp12 e = final_exponentiation(f);
  const fp2* c[12 / 2] = {&e.c0.c0, &e.c0.c1, &e.c0.c2, &e.c1.c0, &e.c1.c1, &e.c1.c2};
  for (int i = 0; i < 6; ++i) {
    fp_to_be(c[i]->c0, out576 + 96 * i);
    fp_to_be(c[i]->c1, out576 + 96 * i + 48);
  }
}

}  // extern "C"

extern "C" int hs_cyclo_sqr_check(const uint8_t* p48, const uint8_t* q96) {
  // easy-part output is cyclotomic: compare Granger-Scott against the generic squaring
  g1a p;
  g1_decompress(&p, p48, GROUP_ORDER_WORDS);
  g2a q;
  g2_decompress(&q, q96, false);
  fp12 f = miller_loop_2(q, fp_neg(p.x), p.y, q, fp_neg(p.x), p.y);
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));
  t = fp12_mul(fp12_frob2(t), t);
  fp12 a = fp12_cyclo_sqr(t), b = fp12_sqr(t);
  const fp2* x[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  const fp2* y[6] = {&b.c0.c0, &b.c0.c1, &b.c0.c2, &b.c1.c0, &b.c1.c1, &b.c1.c2};
  for (int i = 0; i < 6; ++i)
    if (!fp2_eq(*x[i], *y[i])) return 1;
  return 0;
}

// The RLC leaves' window ladder against plain double-and-add on a hashed
// point R (not in G2: psi is applied, not [x]) for the scalar pairs given.
extern "C" int hs_g2_mul2_win4_check(const uint8_t* msg32, const uint32_t* ab, int n) {
  uint32_t m[8];
  msg_words(msg32, m);
  fp2 u0, u1;
  hash_to_field_g2(u0, u1, m);
  const g2j R = g2_add(map_to_curve_sswu_iso3(u0), map_to_curve_sswu_iso3(u1));
  const g2a Ra = g2_to_affine(R);
  for (int i = 0; i < n; ++i) {
    const uint32_t a = ab[2 * i], b = ab[2 * i + 1];
    const g2j want = g2_add(g2_mul_words(R, &a, 1), g2_mul_words(g2_psi(R), &b, 1));
    if (!g2_eq(g2_mul2_win4_affine(Ra, a, b), want)) return i + 1;
  }
  return 0;
}

// RLC collapse check over a whole batch (same device functions as k_rlc_*):
// returns 0 if e(pk, h_eff * sum r_i R_i) * e(-g1, sum r_i sig_i) == 1.
extern "C" int hs_rlc_batch_check(const uint8_t* pk48, const uint8_t* msgs32, const uint8_t* sigs96, int n,
                                  uint64_t seed, const uint64_t* rounds) {
  g1a pk;
  if (g1_decompress(&pk, pk48, GROUP_ORDER_WORDS) != DEC_OK) return -1;
  g2j P = g2_infinity(), S = g2_infinity();
  for (int i = 0; i < n; ++i) {
    uint32_t m[8];
    msg_words(msgs32 + 32 * i, m);
    fp2 u0, u1;
    hash_to_field_g2(u0, u1, m);
    g2j R = g2_add(map_to_curve_sswu_iso3(u0), map_to_curve_sswu_iso3(u1));
    g2a s;
    if (g2_decompress(&s, sigs96 + 96 * i, true) != DEC_OK) return -2;
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (rounds[i] + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (!z) z = 1;
    // the device's leaf arithmetic (k_rlc_leaves: R affine, psi split of the
    // coefficient, joint NAF ladder), checked against plain double-and-add
    const uint32_t a = (uint32_t)z, b = (uint32_t)(z >> 32);
    const g2a Ra = g2_to_affine(R);
    g2j rR = g2_mul2_naf32_affine<true>(Ra, Ra, a, b);
    if (!g2_eq(rR, g2_add(g2_mul_words(R, &a, 1), g2_mul_words(g2_psi(R), &b, 1)))) return -3;
    if (!g2_eq(rR, g2_mul2_naf32_affine<false>(Ra, g2a_psi(Ra), a, b))) return -5;
    if (!g2_eq(rR, g2_mul2_win4_affine(Ra, a, b))) return -6;
    const uint32_t kw[2] = {a, b};
    if (!g2_eq(g2_mul64_naf_affine(Ra, z), g2_mul_words(R, kw, 2))) return -4;
    P = g2_add(P, rR);
    S = g2_add(S, g2_mul2_win4_affine(s, a, b));
  }
  g2a Pa = g2_to_affine(g2_clear_cofactor(P)), Sa = g2_to_affine(S);
  fp12 f = miller_loop_2(Pa, fp_neg(pk.x), pk.y, Sa, fp_neg(C_G1_X), C_G1_NEG_Y);
  return fp12_is_one(final_exponentiation(f)) ? 0 : 1;
}

// G1-signature RLC (rlc_msm.cuh over G1Ops): for a pre-cofactor hash point R
// on E1 (not in G1), the group-generic window ladder [a] R + [b] phi(R) equals
// plain double-and-add for the scalar pairs given; phi acts on H = h_eff R as
// [-x^2]; and h_eff ([a] R + [b] phi(R)) == [a] H + [b] phi(H).
extern "C" int hs_g1_mul2_win4_check(const uint8_t* msg32, const uint32_t* ab, int n) {
  uint32_t m[8];
  msg_words(msg32, m);
  uint32_t uni[32];
  expand_xmd<false, 4>(uni, m);
  const g1j R = g1_add(map_to_curve_sswu_iso11(fp_from_be64_words(uni)),
                       map_to_curve_sswu_iso11(fp_from_be64_words(uni + 16)));
  const g1a Ra = g1_to_affine(R);
  const g1j H = g1_clear_cofactor(R);
  // phi(H) == -[x^2] H
  const uint32_t absx[2] = {(uint32_t)BLS_X_ABS, (uint32_t)(BLS_X_ABS >> 32)};
  if (!g1_eq(g1_phi(H), g1_neg(g1_mul_words(g1_mul_words(H, absx, 2), absx, 2)))) return -1;
  // phi on R (outside G1) is not [-x^2]: the endomorphism is used as a map
  if (g1_eq(g1_phi(R), g1_neg(g1_mul_words(g1_mul_words(R, absx, 2), absx, 2)))) return -2;
  for (int i = 0; i < n; ++i) {
    const uint32_t a = ab[2 * i], b = ab[2 * i + 1];
    const g1j want = g1_add(g1_mul_words(R, &a, 1), g1_mul_words(g1_phi(R), &b, 1));
    const g1j got = mul2_win4_affine<G1Ops>(Ra, a, b);
    if (!g1_eq(got, want)) return i + 1;
    const g1j lhs = g1_clear_cofactor(got);
    const g1j rhs = g1_add(g1_mul_words(H, &a, 1), g1_mul_words(g1_phi(H), &b, 1));
    if (!g1_eq(lhs, rhs)) return 1000 + i;
  }
  return 0;
}

// RLC collapse check for G1 signatures over a batch signed here with sk
// (sig_i = [sk] H_i; sig_i of the `bad` index signs the next message instead):
// returns 0 if e(h_eff sum r_i R_i, pk) e(-sum r_i sig_i, g2) == 1 with the
// leaves computed as the device does (mul2_win4_affine<G1Ops>, r = a + b lambda).
extern "C" int hs_g1_rlc_batch_check(const uint8_t* msgs32, int n, uint64_t sk, uint64_t seed, int bad, int g1dst) {
  const uint32_t skw[2] = {(uint32_t)sk, (uint32_t)(sk >> 32)};
  const g2j pk = g2_mul_words(g2_from_affine(g2a{C_G2_X, C_G2_Y}), skw, 2);
  g1j P = g1_infinity(), S = g1_infinity();
  for (int i = 0; i < n; ++i) {
    auto raw = [&](int k) {
      uint32_t m[8], uni[32];
      msg_words(msgs32 + 32 * k, m);
      if (g1dst)
        expand_xmd<true, 4>(uni, m);
      else
        expand_xmd<false, 4>(uni, m);
      return g1_add(map_to_curve_sswu_iso11(fp_from_be64_words(uni)),
                    map_to_curve_sswu_iso11(fp_from_be64_words(uni + 16)));
    };
    const g1j R = raw(i);
    const g1j sig = g1_mul_words(g1_clear_cofactor(i == bad ? raw((i + 1) % n) : R), skw, 2);
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * ((uint64_t)i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (!z) z = 1;
    P = g1_add(P, mul2_win4_affine<G1Ops>(g1_to_affine(R), (uint32_t)z, (uint32_t)(z >> 32)));
    S = g1_add(S, mul2_win4_affine<G1Ops>(g1_to_affine(sig), (uint32_t)z, (uint32_t)(z >> 32)));
  }
  const g1a Pa = g1_to_affine(g1_clear_cofactor(P)), Sa = g1_to_affine(S);
  // e(Pa, pk) e(-Sa, g2): miller_loop_2 takes each G1 point as (-x, y)
  fp12 f = miller_loop_2(g2_to_affine(pk), fp_neg(Pa.x), Pa.y, g2a{C_G2_X, C_G2_Y}, fp_neg(Sa.x), fp_neg(Sa.y));
  return fp12_is_one(final_exponentiation(f)) ? 0 : 1;
}

// ---------------------------------------------------------------- pairing engine (host emulation)
// The device interpreter's per-lane compute (eng_compute) run for the 12
// lanes of one group in turn: all lanes of a sub-op read, then all write --
// the semantics the device gets from one wavefront's in-order LDS queue.
#define DG_HOSTSIM
#include <vector>
#include "../../drand_amd/csrc/engine.cuh"

namespace {
struct HostGroup {
  uint32_t s[64 * ENG_SLOT_WORDS];
  uint32_t c[ENG_NCONST * ENG_SLOT_WORDS];
  std::vector<fp> lines = std::vector<fp>(68 * 12);
  fp fbuf[12 * ENG_KB_PLANES];   // k_eng_fe's two planes, or the Karabina FE's planes
  fp n1;
  int step = 0;
  bool cyc_ready = false;   // eng_exec's cyc_lin_ready
  fp get(int slot) const { return eng_ld(s + slot * ENG_SLOT_WORDS); }
  void set(int slot, const fp& v) { eng_st(s + slot * ENG_SLOT_WORDS, v); }
};

bool g_cyc_fast = false;
bool g_kb_thread = false;  // the per-thread compressed chain (kb_thread.cuh) instead of the 8-lane rows
bool g_fe_kb = false;     // the Karabina FE (k_eng_fe_seg / k_eng_kb_*) instead of prog_fe
bool g_compiled = false;   // compiled ops (engine_compiled.h) instead of the interpreter

// eng_cyc_fast for the 12 lanes (read all, then write all); `lin`: run the
// LIN sub-op (else the previous E_CYC's fused epilogue wrote its outputs)
void host_cyc_fast(HostGroup& G, bool lin) {
  fp outs[ENG_LANES], fused[ENG_LANES];
  if (lin) {
    for (int k = 0; k < ENG_LANES; ++k) outs[k] = eng_cyc_lin(G.s, ENG_CYC_PAR[k]);
    for (int k = 0; k < ENG_LANES; ++k) eng_st(G.s + (ENG_CYC_PAR[k][0] & 0xFFFFu), outs[k]);
  }
  for (int k = 0; k < ENG_LANES; ++k) outs[k] = eng_cyc_prod(G.s, ENG_CYC_PAR[k]);
  for (int k = 0; k < ENG_LANES; ++k) fused[k] = eng_cyc_fused_lin(outs[k], outs[k ^ 1], k);
  for (int k = 0; k < ENG_LANES; ++k) {
    eng_st(G.s + (ENG_CYC_PAR[k][5] >> 16), outs[k]);
    eng_st(G.s + ENG_CYC_PAR[k][7], fused[k]);
  }
}

void host_run_op(HostGroup& G, int op) {
  if (g_cyc_fast && op == OP_E_CYC) {
    host_cyc_fast(G, !G.cyc_ready);
    G.cyc_ready = true;
    return;
  }
  G.cyc_ready = false;
  const uint32_t s0 = ENG_OP_TAB[op][0], ns = ENG_OP_TAB[op][1];
  for (uint32_t sb = s0; sb < s0 + ns; ++sb) {
    const uint32_t off = ENG_SUB_TAB[sb][0], ntw = ENG_SUB_TAB[sb][1], nt = ntw & 0xFFu;
    fp outs[ENG_LANES];
    for (int k = 0; k < ENG_LANES; ++k) {
      const uint32_t* rec = ENG_WORDS + off + k * eng_rec_words(nt);
      if (!(g_compiled && eng_sub_c_host(op, (int)(sb - s0), G.s, G.c, rec, outs[k]))) outs[k] = eng_compute(G.s, G.c, rec, ntw);
    }
    for (int k = 0; k < ENG_LANES; ++k) {
      const uint32_t* rec = ENG_WORDS + off + k * eng_rec_words(nt);
      if (eng_dst(rec) != 0xFF) G.set(eng_dst(rec), outs[k]);
      const uint32_t e = eng_exp(rec);
      if (e != 0xFF) {
        if (e < 12) G.lines[G.step * 12 + e] = outs[k];
        else G.n1 = outs[k];
      }
    }
    const uint32_t fz = (ntw >> 21) & 0xFFu;  // fused epilogue (engine.cuh eng_fuse_epilogue)
    if (fz) {
      for (int k = 0; k < ENG_LANES; ++k) {
        const uint32_t w = ENG_FUSE_TAB[fz - 1][k], mode = w >> 16;
        if (mode) G.set((int)(w & 0xFFFFu), mode == 1 ? eng_cyc_sum(outs[k], outs[k ^ 1], false)
                                                      : eng_cyc_sum(outs[k ^ 1], outs[k], true));
      }
    }
  }
}

void host_exec(HostGroup& G, const uint32_t* prog, int len) {
  for (int pc = 0; pc < len; ++pc) {
    const uint32_t ins = prog[pc], opc = ins >> 24, a = ins & 0xFF, b = (ins >> 8) & 0xFF;
    if (opc != ENG_OPC_RUN) G.cyc_ready = false;
    if (opc == ENG_OPC_RUN) host_run_op(G, (int)a);
    else if (opc == ENG_OPC_STEP) G.step++;
    else if (opc == ENG_OPC_LDLINE) {
      for (int k = 0; k < 12; ++k) G.set(a + k, G.lines[G.step * 12 + k]);
      G.step++;
    } else if (opc == ENG_OPC_LD12) {
      for (int k = 0; k < 12; ++k) G.set(a + k, G.fbuf[b + k]);
    } else if (opc == ENG_OPC_ST12) {
      for (int k = 0; k < 12; ++k) G.fbuf[b + k] = G.get(a + k);
    }
  }
}

void host_consts(HostGroup& G, const g1a& pk) {
  const fp2 g1c[5] = {C_FROB1_1, C_FROB1_2, C_FROB1_3, C_FROB1_4, C_FROB1_5};
  const fp2 g2c[5] = {C_FROB2_1, C_FROB2_2, C_FROB2_3, C_FROB2_4, C_FROB2_5};
  auto put = [&](int slot, const fp& v) { eng_st(G.c + (slot - 64) * ENG_SLOT_WORDS, v); };
  put(ENG_C_ONE, fp_one());
  put(ENG_C_NXP0, fp_neg(pk.x));
  put(ENG_C_YP0, pk.y);
  put(ENG_C_NXP1, fp_neg(C_G1_X));
  put(ENG_C_YP1, C_G1_NEG_Y);
  for (int k = 0; k < 5; ++k) {
    put(ENG_C_G1 + 2 * k, g1c[k].c0);
    put(ENG_C_G1 + 2 * k + 1, g1c[k].c1);
    put(ENG_C_G2 + k, g2c[k].c0);
  }
  const fp2 cx = C_PSI_CX, cy = C_PSI_CY;
  put(ENG_C_PSI, cx.c0);
  put(ENG_C_PSI + 1, cx.c1);
  put(ENG_C_PSI + 2, cy.c0);
  put(ENG_C_PSI + 3, cy.c1);
}

// The 8-lane compressed squaring (k_eng_kb_chain: eng_cyc_fast<., 8> over
// ENG_CYC8_PAR) for one item: all lanes read, then all write.  own: each
// lane's output of the previous squaring (its post operand when !lin).
void host_kb_square(uint32_t* s, bool lin, fp own[8]) {
  fp outs[8], fused[8];
  if (lin) {
    for (int k = 0; k < 8; ++k) outs[k] = eng_cyc_lin(s, ENG_CYC8_PAR[k]);
    for (int k = 0; k < 8; ++k) eng_st(s + (ENG_CYC8_PAR[k][0] & 0xFFFFu), outs[k]);
  }
  for (int k = 0; k < 8; ++k) outs[k] = eng_cyc_prod<ENG_CYC8_XF>(s, ENG_CYC8_PAR[k], lin ? nullptr : &own[k]);
  for (int k = 0; k < 8; ++k) fused[k] = eng_cyc_fused_lin(outs[k], outs[k ^ 1], k);
  for (int k = 0; k < 8; ++k) {
    eng_st(s + (ENG_CYC8_PAR[k][5] >> 16), outs[k]);
    eng_st(s + ENG_CYC8_PAR[k][7], fused[k]);
    own[k] = outs[k];
  }
}

// Fill a group's slots with normalized garbage (a fresh kernel's LDS): a
// program segment that read a slot it had not written would change the result.
void host_scramble(HostGroup& G, uint64_t x) {
  for (int i = 0; i < 64 * ENG_SLOT_WORDS; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    G.s[i] = (i % ENG_SLOT_WORDS) == FP_LIMBS - 1 ? (uint32_t)(x % FP_P[FP_LIMBS - 1]) : (uint32_t)(x & FP_MASK);
  }
}

// The Karabina FE of one item on the host, kernel by kernel (pairing_engine.cuh
// eng_fe_kb sequence): segments of ENG_PROG_FEK, the compressed chain per
// exponentiation, the norms' inversion and the decompression.  R ends in G's
// slots ENG_E_R.  Returns false if the item would be flagged (f1 = 0).
bool host_fe_kb(HostGroup& G, const fp f[12], const fp& n1inv) {
  auto seg = [&](int j) {
    host_exec(G, ENG_PROG_FEK + ENG_PROG_FEK_OFF[j], ENG_PROG_FEK_OFF[j + 1] - ENG_PROG_FEK_OFF[j]);
  };
  host_scramble(G, 0x1234567);
  for (int k = 0; k < 12; ++k) G.set(ENG_E_F + k, f[k]);
  G.set(ENG_E_N1I, n1inv);
  seg(0);
  for (int e = 1; e <= 5; ++e) {
    if (g_kb_thread) {  // kb_thread.cuh (k_kb_chain_thr)
      const fp* m = G.fbuf + 12 * ENG_KB_PL_M;
      kb_chain_thr(fp2{m[2], m[3]}, fp2{m[4], m[5]}, fp2{m[8], m[9]}, fp2{m[10], m[11]},
                   [&](int j, const fp2& f1, const fp2& f2, const fp2& f4, const fp2& f5) {
                     fp* x = G.fbuf + 12 * (ENG_KB_PL_X0 + j);
                     x[2] = f1.c0, x[3] = f1.c1, x[4] = f2.c0, x[5] = f2.c1;
                     x[8] = f4.c0, x[9] = f4.c1, x[10] = f5.c0, x[11] = f5.c1;
                   });
    } else {
      uint32_t ks[ENG_KB_SLOTS * ENG_SLOT_WORDS];
      memset(ks, 0, sizeof ks);
      fp own[8];
      for (int k = 0; k < 8; ++k) {
        own[k] = G.fbuf[12 * ENG_KB_PL_M + ENG_KB_COMP[k]];
        eng_st(ks + k * ENG_SLOT_WORDS, own[k]);
      }
      host_kb_square(ks, true, own);
      int s = 1;
      for (int j = 0; j < ENG_KB_NSNAP; ++j) {
        for (; s < ENG_KB_SNAP[j]; ++s) host_kb_square(ks, false, own);
        for (int k = 0; k < 8; ++k) G.fbuf[12 * (ENG_KB_PL_X0 + j) + ENG_KB_COMP[k]] = own[k];
      }
    }
    for (int j = 0; j < ENG_KB_NSNAP; ++j) {
      fp* x = G.fbuf + 12 * (ENG_KB_PL_X0 + j);
      const fp nrm = eng_kb_norm(fp2{x[2], x[3]});
      if (fp_is_zero(nrm)) return false;
      fp2 f0, f3;
      ENG_KB_DECOMPRESS(fp2{x[2], x[3]}, fp2{x[4], x[5]}, fp2{x[8], x[9]}, fp2{x[10], x[11]}, fp_inv(nrm), f0, f3);
      x[0] = f0.c0, x[1] = f0.c1, x[6] = f3.c0, x[7] = f3.c1;
    }
    host_scramble(G, 0x9E3779B9ull * (uint64_t)e + 1);
    seg(e);
  }
  return true;
}

// x == 0 mod p for a slot value (< 2.01p)
bool host_slot_zero(const fp& x) { return fp_is_zero(x); }
}  // namespace

// G2 membership of a decodable 96-byte point through the lines program's
// fused test (k_eng_lines status, tools/gen_engine.py lines_subgroup_op):
// the point is pair 1's Q (pair 0 a dummy copy).  Returns 1 in G2, 0 not,
// -1 undecodable.
extern "C" void hs_eng_set_cyc_fast(int on) { g_cyc_fast = on != 0; }
extern "C" void hs_eng_set_fe_kb(int on) { g_fe_kb = on != 0; }
bool g_lines_thread = false;  // T-steps from lines_thread.cuh lt_pair (k_lines_thr) instead of the LINES program
extern "C" void hs_eng_set_lines_thread(int on) { g_lines_thread = on != 0; }
extern "C" void hs_eng_set_kb_thread(int on) { g_kb_thread = on != 0; }
extern "C" void hs_eng_set_compiled(int on) { g_compiled = on != 0; }

// every compiled op vs the interpreter on the same random slots: 0 iff all
// outputs (slots and exports) are identical words
extern "C" int hs_eng_compiled_compare(uint64_t seed) {
  static const int ops[] = {OP_LDBL, OP_LADD, OP_M_XIF, OP_M_SQR, OP_M_LM1, OP_M_LM2, OP_E_MUL, OP_E_MULCJ, OP_E_XIA};
  int n = 0;
  for (int op : ops) {
    HostGroup A;
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + (uint64_t)op + 1;
    for (int i = 0; i < 64 * ENG_SLOT_WORDS; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      const int limb = i % ENG_SLOT_WORDS;
      A.s[i] = limb == FP_LIMBS - 1 ? (uint32_t)(x % FP_P[FP_LIMBS - 1]) : (uint32_t)(x & FP_MASK);
    }
    for (int i = 0; i < ENG_NCONST * ENG_SLOT_WORDS; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      const int limb = i % ENG_SLOT_WORDS;
      A.c[i] = limb == FP_LIMBS - 1 ? (uint32_t)(x % FP_P[FP_LIMBS - 1]) : (uint32_t)(x & FP_MASK);
    }
    HostGroup B = A;
    g_compiled = false;
    host_run_op(A, op);
    g_compiled = true;
    host_run_op(B, op);
    g_compiled = false;
    if (memcmp(A.s, B.s, sizeof A.s) != 0) return 100 + op;
    for (size_t i = 0; i < A.lines.size(); ++i)
      if (memcmp(&A.lines[i], &B.lines[i], sizeof(fp)) != 0) return 200 + op;
    ++n;
  }
  return n == (int)(sizeof ops / sizeof ops[0]) ? 0 : -1;
}

// canonical residue of a normalized value < 2^392
static fp host_canon(fp a) {
  for (int i = 0; i < 12; ++i) a = fp_csub_p(a);
  return a;
}

// E_CYC interpreted vs straight-line (fused LIN epilogue from the second
// squaring on) on the same random group slots (values < p, normalized limbs),
// `reps` squarings in a row: 0 iff the state (R) and LIN (TMP) slots hold the
// same residues after every squaring.
extern "C" int hs_eng_cyc_compare(uint64_t seed, int reps) {
  HostGroup A, B;
  uint64_t x = seed | 1;
  for (int i = 0; i < 64 * ENG_SLOT_WORDS; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const int limb = i % ENG_SLOT_WORDS;
    A.s[i] = limb == FP_LIMBS - 1 ? (uint32_t)(x % FP_P[FP_LIMBS - 1]) : (uint32_t)(x & FP_MASK);
  }
  memset(A.c, 0, sizeof A.c);
  B = A;
  for (int r = 0; r < reps; ++r) {
    g_cyc_fast = false;
    host_run_op(A, OP_E_CYC);
    g_cyc_fast = true;
    host_run_op(B, OP_E_CYC);
    g_cyc_fast = false;
    for (int sl = 0; sl < 12; ++sl) {
      const fp x = host_canon(A.get(sl)), y = host_canon(B.get(sl));
      if (memcmp(&x, &y, sizeof x) != 0) return 1000 * (r + 1) + sl;
    }
    // the fused epilogue's LIN slots == the LIN sub-op over the new state
    for (int k = 0; k < ENG_LANES; ++k) {
      const fp x = host_canon(eng_cyc_lin(B.s, ENG_CYC_PAR[k]));
      const fp y = host_canon(eng_ld(B.s + (ENG_CYC_PAR[k][0] & 0xFFFFu)));
      if (memcmp(&x, &y, sizeof x) != 0) return 1000 * (r + 1) + 100 + k;
    }
  }
  return 0;
}

extern "C" int hs_eng_subgroup(const uint8_t* sig96) {
  g2a s;
  if (g2_decompress(&s, sig96, false) != DEC_OK) return -1;
  static HostGroup G;
  G = HostGroup();
  g1a dummy{C_G1_X, C_G1_Y};
  host_consts(G, dummy);
  for (int p = 0; p < 2; ++p) {
    const fp v[4] = {s.x.c0, s.x.c1, s.y.c0, s.y.c1};
    for (int comp = 0; comp < 4; ++comp) {
      G.set(p * ENG_LINE_PAIR_SLOTS + comp, v[comp]);
      G.set(p * ENG_LINE_PAIR_SLOTS + 6 + comp, v[comp]);
    }
    G.set(p * ENG_LINE_PAIR_SLOTS + 4, fp_one());
    G.set(p * ENG_LINE_PAIR_SLOTS + 5, fp_zero());
  }
  G.set(ENG_L_NXP0, fp_neg(C_G1_X));
  G.set(ENG_L_YP0, C_G1_Y);
  G.step = 0;
  if (g_lines_thread) {
    const g2p T = lt_pair(s, fp_neg(C_G1_X), C_G1_NEG_Y, [](int, const line3&) {});
    return lt_in_g2(T, s) ? 1 : 0;
  }
  host_exec(G, ENG_PROG_LINES, ENG_PROG_LINES_LEN);
  const bool d0 = host_slot_zero(G.get(ENG_L_SUB_D1)) && host_slot_zero(G.get(ENG_L_SUB_D1 + 1)) &&
                  host_slot_zero(G.get(ENG_L_SUB_D2)) && host_slot_zero(G.get(ENG_L_SUB_D2 + 1));
  const bool z0 = host_slot_zero(G.get(ENG_L_SUB_Z)) && host_slot_zero(G.get(ENG_L_SUB_Z + 1));
  return d0 && !z0 ? 1 : 0;
}

// Engine pairing check e(pk, H(msg)) e(-g1, sig) == 1 through the generated
// programs (k_eng_lines -> k_eng_miller -> inversion -> k_eng_fe).  out576:
// FE(f) as 12 canonical 48-byte Fp (w-basis order).  Returns 1 valid, 0 invalid.
extern "C" int hs_eng_pairing(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig96, uint8_t* out576) {
  g1a pk;
  if (g1_decompress(&pk, pk48, GROUP_ORDER_WORDS) != DEC_OK) return -1;
  g2a s;
  if (g2_decompress(&s, sig96, true) != DEC_OK) return -2;
  uint32_t m[8];
  for (int w = 0; w < 8; ++w)
    m[w] = ((uint32_t)msg32[4 * w] << 24) | ((uint32_t)msg32[4 * w + 1] << 16) | ((uint32_t)msg32[4 * w + 2] << 8) | msg32[4 * w + 3];
  g2a h = g2_to_affine(hash_to_g2(m));
  static HostGroup G;
  G = HostGroup();
  host_consts(G, pk);
  const g2a q[2] = {h, s};
  for (int p = 0; p < 2; ++p) {
    const fp v[4] = {q[p].x.c0, q[p].x.c1, q[p].y.c0, q[p].y.c1};
    for (int comp = 0; comp < 4; ++comp) {
      G.set(p * ENG_LINE_PAIR_SLOTS + comp, v[comp]);
      G.set(p * ENG_LINE_PAIR_SLOTS + 6 + comp, v[comp]);
    }
    G.set(p * ENG_LINE_PAIR_SLOTS + 4, fp_one());
    G.set(p * ENG_LINE_PAIR_SLOTS + 5, fp_zero());
  }
  G.set(ENG_L_NXP0, fp_neg(pk.x));
  G.set(ENG_L_YP0, pk.y);
  G.step = 0;
  if (g_lines_thread) {
    const fp nx[2] = {fp_neg(pk.x), fp_neg(C_G1_X)}, yv[2] = {pk.y, C_G1_NEG_Y};
    for (int p = 0; p < 2; ++p)
      lt_pair(q[p], nx[p], yv[p], [&](int step, const line3& l) {
        const fp v[6] = {l.c0.c0, l.c0.c1, l.c2.c0, l.c2.c1, l.c3.c0, l.c3.c1};
        for (int e = 0; e < 6; ++e) G.lines[step * 12 + 6 * p + e] = v[e];
      });
  } else {
    host_exec(G, ENG_PROG_LINES, ENG_PROG_LINES_LEN);
  }
  for (int k = 0; k < 12; ++k) G.set(ENG_M_F + k, k == 0 ? fp_one() : fp_zero());
  G.step = 0;
  host_exec(G, ENG_PROG_MILLER, ENG_PROG_MILLER_LEN);
  fp f[12];
  for (int k = 0; k < 12; ++k) f[k] = G.get(ENG_M_F + k);
  const fp n1inv = fp_inv(G.n1);
  if (g_fe_kb) {
    if (!host_fe_kb(G, f, n1inv)) return -3;
  } else {
    for (int k = 0; k < 12; ++k) G.set(ENG_E_F + k, f[k]);
    G.set(ENG_E_N1I, n1inv);
    host_exec(G, ENG_PROG_FE, ENG_PROG_FE_LEN);
  }
  bool one = true;
  for (int k = 0; k < 12; ++k) {
    fp v = fp_csub_p(fp_csub_p(G.get(ENG_E_R + k)));
    fp_to_be(v, out576 + 48 * k);
    fp cv = fp_from_mont(G.get(ENG_E_R + k));
    bool want_one = k == 0;
    fp_std_to_be48(cv, out576 + 48 * k);
    uint32_t acc = 0;
    for (int i = 0; i < FP_LIMBS; ++i) acc |= cv.l[i] ^ (want_one && i == 0 ? 1u : 0u);
    one = one && acc == 0;
  }
  return one ? 1 : 0;
}

// One pass of the LINES program over the pairs (a, b) (k_eng_lines with
// t_out): T of each pair after the loop, homogeneous (X, Y, Z) in the pair's
// slots 0..5, as Jacobian (XZ, YZ^2, Z) -- pairing_engine.cuh cof_homog_to_jac.
static void host_lines_T(const g2a& a, const g2a& b, g2j out[2]) {
  static HostGroup G;
  G = HostGroup();
  g1a dummy{C_G1_X, C_G1_Y};
  host_consts(G, dummy);
  const g2a q[2] = {a, b};
  for (int p = 0; p < 2; ++p) {
    const fp v[4] = {q[p].x.c0, q[p].x.c1, q[p].y.c0, q[p].y.c1};
    for (int comp = 0; comp < 4; ++comp) {
      G.set(p * ENG_LINE_PAIR_SLOTS + comp, v[comp]);
      G.set(p * ENG_LINE_PAIR_SLOTS + 6 + comp, v[comp]);
    }
    G.set(p * ENG_LINE_PAIR_SLOTS + 4, fp_one());
    G.set(p * ENG_LINE_PAIR_SLOTS + 5, fp_zero());
  }
  G.set(ENG_L_NXP0, fp_neg(C_G1_X));
  G.set(ENG_L_YP0, C_G1_Y);
  G.step = 0;
  host_exec(G, ENG_PROG_LINES, ENG_PROG_LINES_LEN);
  for (int p = 0; p < 2; ++p) {
    auto at = [&](int comp) { return G.get(p * ENG_LINE_PAIR_SLOTS + comp); };
    const fp2 X{at(0), at(1)}, Y{at(2), at(3)}, Z{at(4), at(5)};
    out[p] = g2j{fp2_mul(X, Z), fp2_mul(Y, fp2_sqr(Z)), Z};
  }
}

// The small-call cofactor clearing (capi.hip g2_lane_hash_locked with
// consts: k_cof_prep -> k_eng_lines -> k_cof_mid -> k_eng_lines beside
// k_cof_partial -> k_cof_final) on the host emulation: H(msg) compressed, to
// compare with hs_hash_to_g2 (k_h2c_finish's per-thread ladders).
extern "C" void hs_eng_cof_hash_to_g2(const uint8_t* msg32, uint8_t* out96) {
  uint32_t m[8];
  msg_words(msg32, m);
  fp2 u0, u1;
  hash_to_field_g2(u0, u1, m);
  const g2j P = g2_add(map_to_curve_sswu_iso3_body(u0), map_to_curve_sswu_iso3_body(u1));  // k_cof_prep
  const g2a pa = g2_to_affine(P);
  const g2j ps = g2_psi(g2_from_affine(pa));
  g2j T[2], T2[2];
  host_lines_T(pa, g2a{ps.x, ps.y}, T);  // T0 = [|x|]P, T1 = [|x|]psi(P)
  const g2a t0a = g2_to_affine(T[0]);    // k_cof_mid
  host_lines_T(t0a, t0a, T2);            // T2 = [x^2]P
  g2j u = g2_add(T[0], g2_neg(P));       // k_cof_partial
  u = g2_add(u, g2_neg(T[1]));
  u = g2_add(u, g2_neg(g2_psi(P)));
  u = g2_add(u, g2_psi2(g2_dbl(P)));
  const g2j h = g2_add(T2[0], u);        // k_cof_final
  const bool inf = g2_is_inf(h);
  g2_compress(out96, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(h), inf);
}

// engine.cuh eng_kb_decompress_lz (lazy linear steps, what k_eng_kb_dec runs)
// == eng_kb_decompress (every step reduced) on n random CI inputs -- values
// up to the CI bound 2.01p, where the lazy bounds are tightest -- and on the
// all-maximal-limb input; returns the number of disagreements (outputs
// compared mod p and checked CI: normalized limbs, < 2.01p).
extern "C" int hs_kb_dec_lz_check(int n, uint64_t seed) {
  uint64_t s = seed | 1;
  auto rnd = [&]() {
    fp x;
    for (int i = 0; i < FP_LIMBS; ++i) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      x.l[i] = (uint32_t)s & FP_MASK;
    }
    x.l[FP_LIMBS - 1] &= 0x3FFFFFu;  // up to ~2.46p, reduced to CI (< 2.01p)
    return fp_reduce(x);
  };
  auto ci = [](const fp& v) {  // normalized, value < 2.01p (top limb below 2.01 x p's)
    for (int i = 0; i < FP_LIMBS - 1; ++i)
      if (v.l[i] > FP_MASK) return false;
    return v.l[FP_LIMBS - 1] <= (uint32_t)(2.01 * (double)FP_P[FP_LIMBS - 1]);
  };
  fp mx;
  for (int i = 0; i < FP_LIMBS; ++i) mx.l[i] = FP_MASK;
  mx.l[FP_LIMBS - 1] = 0x3FFFFFu;
  mx = fp_reduce(mx);
  int bad = 0;
  for (int t = 0; t <= n; ++t) {
    const bool edge = t == n;
    const fp2 f1 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()}, f2 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()};
    const fp2 f4 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()}, f5 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()};
    const fp ninv = edge ? mx : rnd();
    fp2 a0, a3, b0, b3;
    eng_kb_decompress(f1, f2, f4, f5, ninv, a0, a3);
    eng_kb_decompress_lz(f1, f2, f4, f5, ninv, b0, b3);
    if (!fp2_eq(a0, b0) || !fp2_eq(a3, b3) || !ci(b0.c0) || !ci(b0.c1) || !ci(b3.c0) || !ci(b3.c1)) ++bad;
  }
  return bad;
}

// kb_thread.cuh's two-lane compressed squaring (kb_pair_send on both halves,
// the (q, k) swap, kb_pair_recv: what k_kb_chain_pair runs) == kb_sqr_thr,
// limb for limb, over `reps` chained squarings from n random CI starts and
// the all-maximal-limb start; returns the number of disagreeing starts.
extern "C" int hs_kb_pair_check(int n, int reps, uint64_t seed) {
  uint64_t s = seed | 1;
  auto rnd = [&]() {
    fp x;
    for (int i = 0; i < FP_LIMBS; ++i) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      x.l[i] = (uint32_t)s & FP_MASK;
    }
    x.l[FP_LIMBS - 1] &= 0x3FFFFFu;
    return fp_reduce(x);
  };
  fp mx;
  for (int i = 0; i < FP_LIMBS; ++i) mx.l[i] = FP_MASK;
  mx.l[FP_LIMBS - 1] = 0x3FFFFFu;
  mx = fp_reduce(mx);
  auto same = [](const fp2& a, const fp2& b) { return !memcmp(&a, &b, sizeof(fp2)); };
  int bad = 0;
  for (int t = 0; t <= n; ++t) {
    const bool edge = t == n;
    fp2 f1 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()}, f2 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()};
    fp2 f4 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()}, f5 = edge ? fp2{mx, mx} : fp2{rnd(), rnd()};
    fp2 bx = f1, by = f4, cx = f2, cy = f5;  // the B lane's and the C lane's halves
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
      kb_sqr_thr(f1, f2, f4, f5);
      fp2 qb, kb, qc, kc;
      kb_pair_send(bx, by, false, qb, kb);
      kb_pair_send(cx, cy, true, qc, kc);
      kb_pair_recv(bx, by, false, qc, kc);
      kb_pair_recv(cx, cy, true, qb, kb);
      ok = ok && same(bx, f1) && same(by, f4) && same(cx, f2) && same(cy, f5);
    }
    if (!ok) ++bad;
  }
  return bad;
}

// curve.cuh g2_dbl_lz (the cofactor ladder's doubling: Y3's product and Z
// carried unreduced) == g2_dbl_body over `reps` chained doublings from n
// points H(msg_i) (Z reduced only at the end, as the ladder does before an
// addition); returns the number of starts whose chains disagree (compared as
// affine points).
extern "C" int hs_g2_dbl_lz_check(int n, int reps, uint64_t seed) {
  int bad = 0;
  for (int t = 0; t < n; ++t) {
    uint32_t m[8];
    for (int w = 0; w < 8; ++w) m[w] = (uint32_t)(seed * 0x9E3779B97F4A7C15ull >> 32) ^ (uint32_t)(t * 8 + w);
    fp2 u0, u1;
    hash_to_field_g2(u0, u1, m);
    g2j a = map_to_curve_sswu_iso3_body(u0), b = a;  // a point of E' with a large cofactor
    for (int r = 0; r < reps; ++r) {
      a = g2_dbl_body(a);
      b = g2_dbl_lz(b);
    }
    if (!g2_eq(a, g2_z_reduce(b))) ++bad;
  }
  return bad;
}

// curve.cuh g2_in_subgroup_ladder (the decode kernels' membership test: lazy
// doublings, fast mixed additions of the fetched point) == g2_in_subgroup on n
// points of E' outside G2 (SSWU outputs) and their images in G2 (h_eff);
// returns mismatches (an exceptional addition counts as one: none is expected
// on these inputs), -1 if the inputs were not what they should be.
struct hs_g2a_fetch {
  g2a p;
  fp2 x() const { return p.x; }
  fp2 y() const { return p.y; }
  g2a get() const { return p; }
};
extern "C" int hs_g2_subgroup_ladder_check(int n, uint64_t seed) {
  int bad = 0;
  for (int t = 0; t < n; ++t) {
    uint32_t m[8];
    for (int w = 0; w < 8; ++w) m[w] = (uint32_t)(seed * 0xD1B54A32D192ED03ull >> 32) ^ (uint32_t)(t * 8 + w);
    fp2 u0, u1;
    hash_to_field_g2(u0, u1, m);
    const g2j raw = map_to_curve_sswu_iso3_body(u0);
    for (int in_g2 = 0; in_g2 < 2; ++in_g2) {
      const g2a a = g2_to_affine(in_g2 ? g2_clear_cofactor(raw) : raw);
      const bool ref = g2_in_subgroup(g2_from_affine(a));
      if (ref != (in_g2 == 1)) return -1;
      bool exc = false;
      const bool got = g2_in_subgroup_ladder(a, hs_g2a_fetch{a}, exc);
      if (exc || got != ref) ++bad;
    }
  }
  return bad;
}
