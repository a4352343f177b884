// SHA-256, drand's round digest, and RFC 9380 hash-to-curve
// (BLS12381G2_XMD:SHA-256_SSWU_RO_) on the 32-bit integer VALU.
//
// Reference: chain/verify.go:24-32 (DigestMessage), key/curve.go:36 (G2
// signatures hashed by kyber-bls12381 KyberG2.Hash -> kilic HashToCurve (R));
// pinned bit-exactly by key/curve_test.go:10-30 through the oracle.
#pragma once
#include "curve.cuh"

namespace dgpu {

// ================================================================ SHA-256
struct sha_state {
  uint32_t h[8];
};

#ifdef __HIP_DEVICE_COMPILE__
#define DG_ROTR(x, n) __builtin_amdgcn_alignbit((x), (x), (n))
#else
#define DG_ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
#endif

constexpr uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

DG_FN sha_state sha_init() {
  return sha_state{{0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19}};
}

// One compression of a 16-word big-endian block.
DG_NOINL void sha_compress(sha_state& s, const uint32_t* blk) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = DG_ROTR(w15, 7) ^ DG_ROTR(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = DG_ROTR(w2, 17) ^ DG_ROTR(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = DG_ROTR(e, 6) ^ DG_ROTR(e, 11) ^ DG_ROTR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA_K[i] + wi;
    uint32_t S0 = DG_ROTR(a, 2) ^ DG_ROTR(a, 13) ^ DG_ROTR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
  s.h[5] += f;
  s.h[6] += g;
  s.h[7] += h;
}

// drand DigestMessage: SHA-256(prev[0..prev_len) || BE64(round)), or
// SHA-256(BE64(round)) when prev_len == 0 (unchained / nil previous).
// Arbitrary prev_len: the padded message is streamed block by block.
DG_NOINL void drand_digest(uint32_t out[8], const uint8_t* prev, uint32_t prev_len, uint64_t round) {
  sha_state s = sha_init();
  uint32_t L = prev_len + 8;
  uint32_t nblk = (L + 9 + 63) / 64;
  uint64_t bitlen = (uint64_t)L * 8;
  for (uint32_t bidx = 0; bidx < nblk; ++bidx) {
    uint32_t blk[16];
    for (int wd = 0; wd < 16; ++wd) {
      uint32_t word = 0;
      for (int byte = 0; byte < 4; ++byte) {
        uint32_t pos = bidx * 64 + wd * 4 + byte;
        uint32_t v;
        if (pos < prev_len)
          v = prev[pos];
        else if (pos < L)
          v = (uint32_t)(round >> (8 * (7 - (pos - prev_len)))) & 0xff;
        else if (pos == L)
          v = 0x80;
        else if (pos >= nblk * 64 - 8)
          v = (uint32_t)(bitlen >> (8 * (nblk * 64 - 1 - pos))) & 0xff;
        else
          v = 0;
        word = (word << 8) | v;
      }
      blk[wd] = word;
    }
    sha_compress(s, blk);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = s.h[i];
}

// SHA-256 continued from state `s` (which has absorbed `pre_bytes` bytes, a
// multiple of 64) over L more bytes get(0) .. get(L - 1), with the padding
// of the whole (pre_bytes + L)-byte message.  Streams block by block, so any
// length works (raw VerifyRecovered messages, key/curve.go:36-39).
template <class Get>
DG_FN void sha_stream(sha_state& s, uint32_t L, uint64_t pre_bytes, Get&& get) {
  const uint32_t nblk = (L + 9 + 63) / 64;
  const uint64_t bitlen = (pre_bytes + L) * 8;
#pragma unroll 1
  for (uint32_t bidx = 0; bidx < nblk; ++bidx) {
    uint32_t blk[16];
#pragma unroll 1
    for (int wd = 0; wd < 16; ++wd) {
      uint32_t word = 0;
      for (int byte = 0; byte < 4; ++byte) {
        const uint32_t pos = bidx * 64 + wd * 4 + byte;
        uint32_t v;
        if (pos < L)
          v = get(pos);
        else if (pos == L)
          v = 0x80;
        else if (pos >= nblk * 64 - 8)
          v = (uint32_t)(bitlen >> (8 * (nblk * 64 - 1 - pos))) & 0xff;
        else
          v = 0;
        word = (word << 8) | v;
      }
      blk[wd] = word;
    }
    sha_compress(s, blk);
  }
}

// ================================================================ expand_message_xmd
// DST bytes as big-endian words: "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_" (43 bytes)
// followed by I2OSP(43, 1): DST_prime = 44 bytes = 11 words.
constexpr uint32_t DST_G2_PRIME[11] = {0x424c535f, 0x5349475f, 0x424c5331, 0x32333831,
                                                             0x47325f58, 0x4d443a53, 0x48412d32, 0x35365f53,
                                                             0x5357555f, 0x524f5f4e, 0x554c5f2b};

// DST' word i: the G2 suite's DST, or (G1DST) the G1 suite's
// "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_", which differs in word 4 only.
template <bool G1DST>
DG_FN uint32_t dst_word(int i) {
  return (G1DST && i == 4) ? 0x47315f58u : DST_G2_PRIME[i];
}

// b1 .. b_ELL of expand_message_xmd from b0:
//  bi: (b0 xor b_{i-1})(32) || i(1) || DST'(44) = 77 bytes, 2 blocks
template <bool G1DST, int ELL>
DG_FN void expand_xmd_tail(uint32_t out[8 * ELL], const uint32_t b0[8]) {
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) prev[i] = 0;
  for (int idx = 1; idx <= ELL; ++idx) {
    sha_state s = sha_init();
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) blk[i] = b0[i] ^ prev[i];
    blk[8] = ((uint32_t)idx << 24) | (dst_word<G1DST>(0) >> 8);
#pragma unroll
    for (int i = 1; i < 8; ++i) blk[8 + i] = (dst_word<G1DST>(i - 1) << 24) | (dst_word<G1DST>(i) >> 8);
    sha_compress(s, blk);
    // bytes 64..76: DST'[31..43] (13 bytes), 0x80, zeros, length 77*8 = 616
    uint32_t blk2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) blk2[i] = 0;
    blk2[0] = (dst_word<G1DST>(7) << 24) | (dst_word<G1DST>(8) >> 8);
    blk2[1] = (dst_word<G1DST>(8) << 24) | (dst_word<G1DST>(9) >> 8);
    blk2[2] = (dst_word<G1DST>(9) << 24) | (dst_word<G1DST>(10) >> 8);
    blk2[3] = (dst_word<G1DST>(10) << 24) | 0x00800000u;
    blk2[15] = 77 * 8;
    sha_compress(s, blk2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      prev[i] = s.h[i];
      out[(idx - 1) * 8 + i] = s.h[i];
    }
  }
}

// expand_message_xmd of an arbitrary-length message (len bytes at msg,
// device or host memory): b0 = H(Z_pad || msg || I2OSP(32 ELL, 2) || 0x00 ||
// DST'), streamed from the Z_pad midstate.
template <bool G1DST, int ELL>
DG_NOINL void expand_xmd_var(uint32_t out[8 * ELL], const uint8_t* msg, uint32_t len) {
  sha_state s0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s0.h[i] = SHA_ZPAD_MIDSTATE[i];
  sha_stream(s0, len + 47, 64, [&](uint32_t pos) -> uint32_t {
    if (pos < len) return msg[pos];
    const uint32_t k = pos - len;
    if (k == 0) return (32u * ELL) >> 8;
    if (k == 1) return (32u * ELL) & 0xffu;
    if (k == 2) return 0u;
    const uint32_t j = k - 3;  // DST' byte
    return (dst_word<G1DST>((int)(j >> 2)) >> (24 - 8 * (j & 3))) & 0xffu;
  });
  expand_xmd_tail<G1DST, ELL>(out, s0.h);
}

// expand_message_xmd(msg (32 bytes), DST, 32 ELL bytes) -> 8 ELL big-endian words
// (ELL = 8: hash to G2, 256 bytes; ELL = 4: hash to G1, 128 bytes).
// Message layouts (bytes):
//  b0: Z_pad(64) || msg(32) || I2OSP(32 ELL, 2) || 0x00 || DST'(44)  = 143 bytes, 3 blocks
//  bi: x(32) || i(1) || DST'(44)                                      =  77 bytes, 2 blocks
template <bool G1DST, int ELL>
DG_NOINL void expand_xmd(uint32_t out[8 * ELL], const uint32_t msg[8]) {
  // b0
  sha_state s0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s0.h[i] = SHA_ZPAD_MIDSTATE[i];  // after the all-zero Z_pad block
  {
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) blk[i] = msg[i];
    // bytes 96..: I2OSP(32 ELL, 2) 0x00 DST'[0]
    blk[8] = ((uint32_t)(32 * ELL) << 16) | (dst_word<G1DST>(0) >> 24);
#pragma unroll
    for (int i = 1; i < 8; ++i) blk[8 + i] = (dst_word<G1DST>(i - 1) << 8) | (dst_word<G1DST>(i) >> 24);
    sha_compress(s0, blk);
    // remaining DST' bytes: DST'[29..43] (15 bytes), then 0x80, zeros, length 143*8 = 1144
    uint32_t blk2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) blk2[i] = 0;
    blk2[0] = (dst_word<G1DST>(7) << 8) | (dst_word<G1DST>(8) >> 24);
    blk2[1] = (dst_word<G1DST>(8) << 8) | (dst_word<G1DST>(9) >> 24);
    blk2[2] = (dst_word<G1DST>(9) << 8) | (dst_word<G1DST>(10) >> 24);
    blk2[3] = (dst_word<G1DST>(10) << 8) | 0x80u;
    blk2[15] = 143 * 8;
    sha_compress(s0, blk2);
  }
  expand_xmd_tail<G1DST, ELL>(out, s0.h);
}

DG_NOINL void expand_xmd_g2(uint32_t out[64], const uint32_t msg[8]) { expand_xmd<false, 8>(out, msg); }

// 64 big-endian bytes (as 16 BE words) -> Fp (Montgomery): x = hi * 2^384 + lo
DG_NOINL fp fp_from_be64_words(const uint32_t* w) {
  uint8_t bytes[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    bytes[4 * i] = (uint8_t)(w[i] >> 24);
    bytes[4 * i + 1] = (uint8_t)(w[i] >> 16);
    bytes[4 * i + 2] = (uint8_t)(w[i] >> 8);
    bytes[4 * i + 3] = (uint8_t)w[i];
  }
  uint8_t hi48[48];
#pragma unroll
  for (int i = 0; i < 32; ++i) hi48[i] = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) hi48[32 + i] = bytes[i];
  fp lo = fp_std_from_be48(bytes + 16);
  fp hi = fp_std_from_be48(hi48);
  return fp_add(fp_mul(lo, FP_R2), fp_mul(hi, FP_2_384_R2));
}

DG_FN void hash_to_field_g2(fp2& u0, fp2& u1, const uint32_t msg[8]) {
  uint32_t uni[64];
  expand_xmd_g2(uni, msg);
  u0.c0 = fp_from_be64_words(uni + 0);
  u0.c1 = fp_from_be64_words(uni + 16);
  u1.c0 = fp_from_be64_words(uni + 32);
  u1.c1 = fp_from_be64_words(uni + 48);
}

// ================================================================ SSWU + 3-isogeny
// Simplified SWU on E2': y^2 = x^3 + A'x + B' (RFC 9380 section 6.6.2) fused
// with the 3-isogeny to E2, inversion-free: x1 = N/D, gx1 = U/D^3 and
// gx2 = (Z u^2)^3 gx1, so one norm-method square root of w = U D (or of
// (Z u^2)^3 U D) -- two Fp exponentiations in all, the square test of gx1
// included -- gives y = sqrt(w)/D^2 = fp2_sqrt_scaled(w, g, norm(D))
// conj(D)^2.  The isogeny is evaluated on x = N/D homogeneously.  Model and
// derivation: tools/sswu_model.py (tests/test_sswu_model.py).
// The body in stages (k_sswu_a / _b / _c run them as separate launches with
// the two exponentiations between them, k_fp_pow_planes):
//   sswu_pre   x1 = N/D and w = U D;  alpha = Norm(w) goes to the first exponentiation
//   sswu_mid   g = alpha^((p+1)/4): gx1 square or not (then x2, w scaled); returns
//              d (fp2_sqrt_scaled's real part) and dm4 = d Norm(D)^4 for the second
//   sswu_post  t = dm4^((p-3)/4): y, its sign, the 3-isogeny.
DG_FN fp2 sswu_zu2(const fp2& u) { return fp2_mul(C_SSWU_Z, fp2_sqr(u)); }
DG_FN void sswu_pre(const fp2& zu2, fp2& N, fp2& D, fp2& D2, fp2& D3, fp2& w) {
  const fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  const bool den0 = fp2_is_zero(den);
  N = fp2_cmov(fp2_mul(C_SSWU_MINUS_B_OVER_A, fp2_add(den, fp2_one())), C_SSWU_B_OVER_ZA, den0);
  D = fp2_cmov(den, fp2_one(), den0);
  D2 = fp2_sqr(D);
  D3 = fp2_mul(D2, D);
  w = fp2_mul(fp2_add(fp2_mul(N, fp2_add(fp2_sqr(N), fp2_mul(C_SSWU_A, D2))), fp2_mul(C_SSWU_B, D3)), D);
}
DG_FN void sswu_pre(const fp2& u, fp2& N, fp2& D, fp2& w) {
  fp2 D2, D3;
  sswu_pre(sswu_zu2(u), N, D, D2, D3, w);
}
// g: the candidate root of alpha = Norm(w); N, w updated to x2's when gx1 is
// not a square.  Returns d; dm4 = d Norm(D)^4 (fp2_sqrt_scaled's steps).
DG_FN fp sswu_mid(const fp2& u, const fp2& zu2, const fp& alpha, fp2& N, const fp2& D, fp2& w, fp g, fp& dm4) {
  if (!fp_eq(fp_sqr(g), alpha)) {  // gx1 not square: x2 = Z u^2 x1, gx2 = (Z u^2)^3 gx1
    const fp nu = fp2_norm(u);
    g = fp_mul(fp_mul(C_SQRT_M125, fp_mul(fp_sqr(nu), nu)), g);
    w = fp2_mul(fp2_mul(fp2_sqr(zu2), zu2), w);
    N = fp2_mul(zu2, N);
  }
  return fp2_sqrt_scaled_pre(w, g, fp2_norm(D), dm4);
}
DG_FN g2j sswu_post(const fp2& u, const fp2& N, const fp2& D, const fp2& D2, const fp2& D3, const fp2& w,
                    const fp& d, const fp& dm4, const fp& t) {
  fp2 y = fp2_mul(fp2_sqrt_scaled_post(w, d, dm4, t), fp2_sqr(fp2_conj(D)));
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  // 3-isogeny on x = N/D, numerators homogenized to degree 3 (x denominator 2)
  const fp2 N2 = fp2_sqr(N);
  const fp2 N3 = fp2_mul(N2, N);
  const fp2 N2D = fp2_mul(N2, D);
  const fp2 ND2 = fp2_mul(N, D2);
  const fp2 xn = fp2_add(fp2_add(fp2_mul(C_ISO3_XNUM_3, N3), fp2_mul(C_ISO3_XNUM_2, N2D)),
                         fp2_add(fp2_mul(C_ISO3_XNUM_1, ND2), fp2_mul(C_ISO3_XNUM_0, D3)));
  const fp2 xd = fp2_add(fp2_add(N2, fp2_mul(C_ISO3_XDEN_1, fp2_mul(N, D))), fp2_mul(C_ISO3_XDEN_0, D2));
  const fp2 yn = fp2_add(fp2_add(fp2_mul(C_ISO3_YNUM_3, N3), fp2_mul(C_ISO3_YNUM_2, N2D)),
                         fp2_add(fp2_mul(C_ISO3_YNUM_1, ND2), fp2_mul(C_ISO3_YNUM_0, D3)));
  const fp2 yd = fp2_add(fp2_add(N3, fp2_mul(C_ISO3_YDEN_2, N2D)),
                         fp2_add(fp2_mul(C_ISO3_YDEN_1, ND2), fp2_mul(C_ISO3_YDEN_0, D3)));
  // x_E2 = xn / (xd D), y_E2 = y yn / yd; Jacobian with Z = xd D yd
  const fp2 xdd = fp2_mul(xd, D);
  const fp2 tt = fp2_mul(xdd, fp2_sqr(yd));
  g2j r;
  r.z = fp2_mul(xdd, yd);
  r.x = fp2_mul(xn, tt);
  r.y = fp2_mul(fp2_mul(y, yn), fp2_mul(fp2_sqr(xdd), tt));
  // an exceptional input (xd or yd = 0) gives Z = 0: the identity (RFC 9380 section 6.6.3)
  return r;
}

DG_FN g2j sswu_post(const fp2& u, const fp2& N, const fp2& D, const fp2& w, const fp& d, const fp& dm4,
                    const fp& t) {
  const fp2 D2 = fp2_sqr(D);
  return sswu_post(u, N, D, D2, fp2_mul(D2, D), w, d, dm4, t);
}

DG_FN g2j map_to_curve_sswu_iso3_body(const fp2& u) {
  const fp2 zu2 = sswu_zu2(u);
  fp2 N, D, D2, D3, w;
  sswu_pre(zu2, N, D, D2, D3, w);
  const fp alpha = fp2_norm(w);
  fp dm4;
  const fp d = sswu_mid(u, zu2, alpha, N, D, w, fp_sqrt_cand(alpha), dm4);
  return sswu_post(u, N, D, D2, D3, w, d, dm4, DG_POW(dm4, EXP_P_MINUS_3_DIV_4));
}

DG_NOINL g2j map_to_curve_sswu_iso3(const fp2& u) { return map_to_curve_sswu_iso3_body(u); }

// hash_to_curve for G2 from the 32-byte drand digest; returns Jacobian H(m)
DG_NOINL g2j hash_to_g2(const uint32_t msg[8]) {
  fp2 u0, u1;
  hash_to_field_g2(u0, u1, msg);
  g2j q0 = map_to_curve_sswu_iso3(u0);
  g2j q1 = map_to_curve_sswu_iso3(u1);
  return g2_clear_cofactor(g2_add(q0, q1));
}

}  // namespace dgpu
