// Signatures on G1 (schemes bls-unchained-on-g1 and bls-unchained-g1-rfc9380):
// hash to G1 (RFC 9380 section 8.8.1, suite BLS12381G1_XMD:SHA-256_SSWU_RO_,
// with the G2 suite's DST for the legacy scheme (R)), G1 signature decoding
// with the endomorphism membership test, and the fixed-Q line evaluation the
// pairing engine consumes (both G2 arguments of e(H, pk) e(-sig, g2) are fixed
// per key, so their Miller lines are computed once by dgpu_set_pubkey and each
// round only scales them by its G1 coordinates).
//
// Oracle: oracle/bls12381.py hash_to_g1 / verify_g1 / g1_decompress; model of
// the inversion-free map: tools/sswu_model.py sswu_iso11_jacobian.
#pragma once
#include "curve.cuh"
#include "h2c.cuh"
#ifndef DG_NO_KERNELS
#include "kernels.cuh"
#endif

namespace dgpu {

DG_FN fp fp_row(const uint32_t (*t)[FP_LIMBS], int i) {
  fp r;
#pragma unroll
  for (int l = 0; l < FP_LIMBS; ++l) r.l[l] = t[i][l];
  return r;
}

// RFC 9380 sgn0 for Fp: parity of the canonical value
DG_FN uint32_t fp_sgn0(const fp& a) { return fp_from_mont(a).l[0] & 1u; }

// sum_i c_i N^i D^(deg - i): a polynomial in x = N / D, homogenized (Horner)
DG_NOINL fp iso11_hom(const uint32_t (*c)[FP_LIMBS], int deg, const fp& N, const fp& D) {
  fp acc = fp_row(c, deg);
  fp dk = fp_one();
  for (int i = deg - 1; i >= 0; --i) {
    dk = fp_mul(dk, D);
    acc = fp_add(fp_mul(acc, N), fp_mul(fp_row(c, i), dk));
  }
  return acc;
}

// The four polynomials of the 11-isogeny (x numerator degree 11, denominator
// 10, y numerator and denominator 15), homogenized in x = N / D, in one Horner
// pass (round 6): at step s every polynomial of degree >= s takes
// acc = acc N + c_(deg - s) D^s, so D^s is formed once per step (15 products
// where four iso11_hom calls form 51), and the sums stay unreduced between
// steps -- two products < 1.01p each, the sum < 2.02p with limbs < 2^29, is
// the next product's operand -- reduced once at the end (51 reductions fewer).
DG_FN void iso11_hom4(const fp& N, const fp& D, fp& xn, fp& xd, fp& yn, fp& yd) {
  fp a0 = fp_row(ISO11_XNUM, 11), a1 = fp_row(ISO11_XDEN, 10), a2 = fp_row(ISO11_YNUM, 15),
     a3 = fp_row(ISO11_YDEN, 15);
  fp dk = fp_one();
#pragma unroll 1
  for (int st = 1; st <= 15; ++st) {
    dk = fp_mul(dk, D);
    if (st <= 11) a0 = fp_add_lz(fp_mul(a0, N), fp_mul(fp_row(ISO11_XNUM, 11 - st), dk));
    if (st <= 10) a1 = fp_add_lz(fp_mul(a1, N), fp_mul(fp_row(ISO11_XDEN, 10 - st), dk));
    a2 = fp_add_lz(fp_mul(a2, N), fp_mul(fp_row(ISO11_YNUM, 15 - st), dk));
    a3 = fp_add_lz(fp_mul(a3, N), fp_mul(fp_row(ISO11_YDEN, 15 - st), dk));
  }
  xn = fp_reduce(fp_norm(a0));
  xd = fp_reduce(fp_norm(a1));
  yn = fp_reduce(fp_norm(a2));
  yd = fp_reduce(fp_norm(a3));
}

// Simplified SWU on E1' (Z = 11) fused with the 11-isogeny to E1, inversion
// free: x1 = N/D, gx1 = U/V with V = D^3; t = (U V^3)^((p-3)/4) gives
// y1 = U V t with y1^2 = gx1 (if y1^2 V = U) or -gx1; in the latter case
// sqrt(gx2) = Z u^3 sqrt(-Z) y1 (gx2 = Z^3 u^6 gx1).  One exponentiation.
DG_FN g1j map_to_curve_sswu_iso11_body(const fp& u) {
  const fp zu2 = fp_mul(C_SSWU1_Z, fp_sqr(u));
  const fp den = fp_add(fp_sqr(zu2), zu2);
  const bool den0 = fp_is_zero(den);
  fp N = fp_cmov(fp_mul(C_SSWU1_MINUS_B_OVER_A, fp_add(den, fp_one())), C_SSWU1_B_OVER_ZA, den0);
  const fp D = fp_cmov(den, fp_one(), den0);
  const fp D2 = fp_sqr(D);
  const fp D3 = fp_mul(D2, D);
  const fp U = fp_add(fp_mul(N, fp_add(fp_sqr(N), fp_mul(C_SSWU1_A, D2))), fp_mul(C_SSWU1_B, D3));
  const fp t = DG_POW(fp_mul(U, fp_mul(fp_sqr(D3), D3)), EXP_P_MINUS_3_DIV_4);
  fp y = fp_mul(fp_mul(U, D3), t);
  if (!fp_eq(fp_mul(fp_sqr(y), D3), U)) {  // gx1 not square: x2 = Z u^2 x1
    y = fp_mul(fp_mul(C_SSWU1_Z_SQRT_MZ, fp_mul(fp_sqr(u), u)), y);
    N = fp_mul(zu2, N);
  }
  if (fp_sgn0(u) != fp_sgn0(y)) y = fp_neg(y);
#ifdef DG_ISO11_PLAIN  // A/B: rounds 2-5, four Horner passes, every sum reduced
  const fp xn = iso11_hom(ISO11_XNUM, 11, N, D);
  const fp xd = iso11_hom(ISO11_XDEN, 10, N, D);
  const fp yn = iso11_hom(ISO11_YNUM, 15, N, D);
  const fp yd = iso11_hom(ISO11_YDEN, 15, N, D);
#else
  fp xn, xd, yn, yd;
  iso11_hom4(N, D, xn, xd, yn, yd);
#endif
  // x_E1 = xn / (xd D), y_E1 = y yn / yd; Jacobian Z = xd D yd (0 for the exceptional inputs)
  const fp xdd = fp_mul(xd, D);
  const fp T = fp_mul(xdd, fp_sqr(yd));
  g1j r;
  r.z = fp_mul(xdd, yd);
  r.x = fp_mul(xn, T);
  r.y = fp_mul(fp_mul(y, yn), fp_mul(fp_sqr(xdd), T));
  return r;
}

DG_NOINL g1j map_to_curve_sswu_iso11(const fp& u) { return map_to_curve_sswu_iso11_body(u); }

// [|x|] p, |x| = 0xd201000000010000 (group law inlined: register-resident points)
DG_FN g1j g1_mul_absx(const g1j& p) {
  g1j r = p;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = g1_dbl_body(r);
    if ((BLS_X_ABS >> i) & 1ull) r = g1_add_body(r, p);
  }
  return r;
}

// map_to_curve of the two field elements in a 128-byte expand_message_xmd
// output, then cofactor clearing by h_eff = 1 - x = 1 + |x|.
template <bool INL>
DG_FN g1j hash_to_g1_from_uni(const uint32_t uni[32]) {
  const fp u0 = fp_from_be64_words(uni);
  const fp u1 = fp_from_be64_words(uni + 16);
  const g1j q = INL ? g1_add_body(map_to_curve_sswu_iso11_body(u0), map_to_curve_sswu_iso11_body(u1))
                   : g1_add(map_to_curve_sswu_iso11(u0), map_to_curve_sswu_iso11(u1));
  return g1_add_body(q, g1_mul_absx(q));
}

// hash_to_curve for G1 of a 32-byte digest; g1dst selects the G1 suite's DST
// (bls-unchained-g1-rfc9380) over the G2 suite's (bls-unchained-on-g1).
template <bool INL>
DG_FN g1j hash_to_g1_t(const uint32_t msg[8], bool g1dst) {
  uint32_t uni[32];
  if (g1dst)
    expand_xmd<true, 4>(uni, msg);
  else
    expand_xmd<false, 4>(uni, msg);
  return hash_to_g1_from_uni<INL>(uni);
}

DG_NOINL g1j hash_to_g1(const uint32_t msg[8], bool g1dst) { return hash_to_g1_t<false>(msg, g1dst); }

// G1 membership of an affine point on E1: (beta x, y) == -[x^2] P (Scott's
// endomorphism test; same verdict as [r] P == O, tests/test_oracle_g1.py).
DG_FN bool g1_in_subgroup_endo_body(const g1a& p) {
  const g1j t = g1_mul_absx(g1_mul_absx(g1j{p.x, p.y, fp_one()}));
  if (g1_is_inf(t)) return false;
  const fp z2 = fp_sqr(t.z);
  return fp_eq(fp_mul(fp_mul(C_G1_BETA, p.x), z2), t.x) && fp_is_zero(fp_add(fp_mul(p.y, fp_mul(z2, t.z)), t.y));
}
DG_NOINL bool g1_in_subgroup_endo(const g1a& p) { return g1_in_subgroup_endo_body(p); }

// 48-byte compressed G1 signature (kilic G1.FromCompressed semantics (R)).
// The _body form is force-inlined into k_decode_g1_sigs: an out-of-line
// callee's registers escape the kernel's launch bounds (249 VGPRs + 32 AGPRs,
// 1 wave/SIMD), inlined the kernel runs at 2 waves/SIMD -- 313.5 -> 229.0 ms
// per 10M (tools/engbench/dec_g1.hip, profiles/r04/r04c_dec_g1_variants.txt).
DG_FN int g1_decompress_sig_body(g1a* out, const uint8_t* in) {
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
  return g1_in_subgroup_endo_body(*out) ? DEC_OK : DEC_ERR_SUBGROUP;
}
DG_NOINL int g1_decompress_sig(g1a* out, const uint8_t* in) { return g1_decompress_sig_body(out, in); }

#ifndef DG_NO_KERNELS  // (the host-emulation test build takes the device functions only)
// ---------------------------------------------------------------- kernels
// H(m) in G1 of each item's message (msg_src: the unchained DigestMessage
// SHA-256(BE64(round)), chain/verify.go:24-32, or raw bytes): X, Y into h_out
// ([x, y][limb][n]), Z into z_out.
__global__ void __launch_bounds__(256, 2) k_hash_to_g1_beacons(size_t n, msg_src m, int g1dst,
                                                             uint32_t* __restrict__ h_out, uint32_t* __restrict__ z_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t uni[32];
  if (g1dst)
    msg_expand<true, 4>(m, i, uni);
  else
    msg_expand<false, 4>(m, i, uni);
  const g1j h = hash_to_g1_from_uni<true>(uni);
  st_fp(h_out, n, i, h.x);
  st_fp(h_out + FP_WORDS * n, n, i, h.y);
  st_fp(z_out, n, i, h.z);
}

// RLC mode (rlc_msm.cuh): the pre-cofactor hash point R = Q0 + Q1 on E1
// (Jacobian X, Y into r_out, Z into z_out): h_eff = 1 + |x| is applied once per
// checked node, by linearity, instead of a 64-step ladder per round.
__global__ void __launch_bounds__(256, 2) k_hash_to_g1_raw(size_t n, msg_src m, int g1dst,
                                                         uint32_t* __restrict__ r_out, uint32_t* __restrict__ z_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t uni[32];
  if (g1dst)
    msg_expand<true, 4>(m, i, uni);
  else
    msg_expand<false, 4>(m, i, uni);
  const g1j r = g1_add_body(map_to_curve_sswu_iso11_body(fp_from_be64_words(uni)),
                            map_to_curve_sswu_iso11_body(fp_from_be64_words(uni + 16)));
  st_fp(r_out, n, i, r.x);
  st_fp(r_out + FP_WORDS * n, n, i, r.y);
  st_fp(z_out, n, i, r.z);
}

// H(m) in G1 of raw messages of any length, compressed (parity surface:
// dgpu_hash_to_g1 / dgpu_hash_to_curve)
__global__ void __launch_bounds__(256) k_hash_to_g1_msgs(size_t n, msg_src m, int g1dst, uint8_t* __restrict__ out48) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t uni[32];
  if (g1dst)
    msg_expand<true, 4>(m, i, uni);
  else
    msg_expand<false, 4>(m, i, uni);
  const g1j h = hash_to_g1_from_uni<false>(uni);
  const bool inf = g1_is_inf(h);
  g1_compress(out48 + i * 48, inf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(h), inf);
}

// Jacobian -> affine in place for n G1 points (X, Y in pts, Z in z), one Fp
// inversion per thread by Montgomery's trick (as k_g2_batch_affine).
__global__ void __launch_bounds__(256) k_g1_batch_affine(size_t n, uint32_t* __restrict__ pts,
                                                         const uint32_t* __restrict__ z, uint32_t* __restrict__ pre) {
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  fp acc = fp_one();
  size_t last = t;
  for (size_t i = t; i < n; i += T) {
    const fp zi = ld_fp(z, n, i);
    acc = fp_mul(acc, fp_cmov(zi, fp_one(), fp_is_zero(zi)));
    st_fp(pre, n, i, acc);
    last = i;
  }
  fp inv = fp_inv(acc);
  for (size_t i = last;; i -= T) {
    const fp zi = ld_fp(z, n, i);
    const bool inf = fp_is_zero(zi);
    const fp zinv = i >= t + T ? fp_mul(inv, ld_fp(pre, n, i - T)) : inv;
    const fp zinv2 = fp_sqr(zinv);
    const fp x = fp_mul(ld_fp(pts, n, i), zinv2);
    const fp y = fp_mul(ld_fp(pts + FP_WORDS * n, n, i), fp_mul(zinv2, zinv));
    st_fp(pts, n, i, inf ? fp_zero() : x);
    st_fp(pts + FP_WORDS * n, n, i, inf ? fp_zero() : y);
    if (i < t + T) break;
    if (!inf) inv = fp_mul(inv, zi);
  }
}

// G1 signature decode + membership: affine [x, y][limb][n], status ST_*.
__global__ void __launch_bounds__(256, 2) k_decode_g1_sigs(size_t n, const uint8_t* __restrict__ sigs, size_t sig_stride,
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
    const int rc = g1_decompress_sig_body(&p, buf);
    st = rc == DEC_OK ? ST_OK : rc == DEC_INFINITY ? ST_INFINITY : rc == DEC_ERR_SUBGROUP ? ST_SUBGROUP : ST_DECODE;
  }
  st_fp(sig_out, n, i, p.x);
  st_fp(sig_out + FP_WORDS * n, n, i, p.y);
  status[i] = st;
}

// Public key (96-byte compressed G2, subgroup-checked) -> affine, one thread.
__global__ void k_decode_g2_pk(const uint8_t* __restrict__ in96, uint32_t* __restrict__ out, int* __restrict__ rc) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint8_t buf[96];
  for (int k = 0; k < 96; ++k) buf[k] = in96[k];
  g2a p{fp2_zero(), fp2_zero()};
  *rc = g2_decompress(&p, buf, true);
  st_g2a(out, 1, 0, p);
}

// pk = sk * g2 (96-byte compressed): synthetic-chain tool for the G1 schemes.
__global__ void k_derive_pubkey_g2(scalar256 sk, uint8_t* __restrict__ out96) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const g2j q = g2_mul_words(g2_from_affine(g2a{C_G2_X, C_G2_Y}), sk.w, 8);
  const bool inf = g2_is_inf(q);
  g2_compress(out96, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(q), inf);
}

// One step of S independent unchained segments signed on G1 (synthetic-chain
// tool, as k_sign_step): round first_round[s] + step, 48-byte signature.
__global__ void __launch_bounds__(256) k_sign_step_g1(size_t S, const uint64_t* __restrict__ first_round, uint64_t step,
                                                       int g1dst, scalar256 sk, uint8_t* __restrict__ sig_out,
                                                       size_t sig_stride) {
  const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  uint32_t msg[8];
  drand_digest(msg, nullptr, 0u, first_round[s] + step);
  const g1j sg = g1_mul_words(hash_to_g1(msg, g1dst != 0), sk.w, 8);
  const bool inf = g1_is_inf(sg);
  uint8_t out[48];
  g1_compress(out, inf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(sg), inf);
  for (int k = 0; k < 48; ++k) sig_out[s * sig_stride + k] = out[k];
}

// Sign n raw messages with one secret (test/tool surface of key.Scheme.Sign /
// AuthScheme.Sign, key/curve.go:36-39; key/curve_test.go:10-30 signs this
// way): sig = sk * H(msg), compressed.  on_g1: 48-byte G1 signatures under
// the DST g1dst selects; else 96-byte G2 signatures.
__global__ void __launch_bounds__(64) k_sign_msgs(size_t n, msg_src m, int on_g1, int g1dst, scalar256 sk,
                                                  uint8_t* __restrict__ out, size_t out_stride) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (on_g1) {
    uint32_t uni[32];
    if (g1dst)
      msg_expand<true, 4>(m, i, uni);
    else
      msg_expand<false, 4>(m, i, uni);
    const g1j sg = g1_mul_words(hash_to_g1_from_uni<false>(uni), sk.w, 8);
    const bool inf = g1_is_inf(sg);
    g1_compress(out + i * out_stride, inf ? g1a{fp_zero(), fp_zero()} : g1_to_affine(sg), inf);
  } else {
    uint32_t uni[64];
    msg_expand<false, 8>(m, i, uni);
    const fp2 u0{fp_from_be64_words(uni), fp_from_be64_words(uni + 16)};
    const fp2 u1{fp_from_be64_words(uni + 32), fp_from_be64_words(uni + 48)};
    const g2j h = g2_clear_cofactor(g2_add(map_to_curve_sswu_iso3(u0), map_to_curve_sswu_iso3(u1)));
    const g2j sg = g2_mul_words(h, sk.w, 8);
    const bool inf = g2_is_inf(sg);
    g2_compress(out + i * out_stride, inf ? g2a{fp2_zero(), fp2_zero()} : g2_to_affine(sg), inf);
  }
}

// Batch decode of compressed G1 points (48 bytes each, kilic G1.FromCompressed
// semantics (R) with the endomorphism membership test): public keys and
// commitments (chain/convert.go:20-23, deploy/*/group.toml).  rc[i] = DEC_*,
// out (optional) = canonical big-endian x || y (96 bytes) of decoded points.
__global__ void __launch_bounds__(64) k_decode_g1_points(size_t n, const uint8_t* __restrict__ in48,
                                                         int* __restrict__ rc, uint8_t* __restrict__ out96) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t buf[48];
  for (int k = 0; k < 48; ++k) buf[k] = in48[i * 48 + k];
  g1a p{fp_zero(), fp_zero()};
  const int r = g1_decompress_sig(&p, buf);
  rc[i] = r;
  if (out96) {
    fp_std_to_be48(fp_from_mont(p.x), out96 + i * 96);
    fp_std_to_be48(fp_from_mont(p.y), out96 + i * 96 + 48);
  }
}

#endif  // DG_NO_KERNELS

}  // namespace dgpu
