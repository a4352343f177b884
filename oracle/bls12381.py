"""Pure-Python CPU restatement of the BLS12-381 arithmetic drand's verify path uses.

TEST INFRASTRUCTURE ONLY (oracle).  Nothing in the product path (drand_amd/,
libdrand_gpu.so) imports, links or executes this file; only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only as
the checker.

What it restates (the reference's crypto lives in third-party Go modules that
are NOT present under /root/reference):

* kyber-bls12381 v0.2.1 / kilic bls12-381 (2020-08-20): field tower
  Fp/Fp2/Fp6/Fp12, G1/G2 group law, ZCash compressed (de)serialization with
  subgroup check, RFC 9380 hash-to-curve (expand_message_xmd SHA-256, SSWU,
  3-isogeny, h_eff cofactor clearing), optimal-ate pairing.  Called from the
  reference at chain/verify.go:44 (key.Scheme.VerifyRecovered) and
  key/curve.go:24-39 (suite roles: keys on G1, signatures on G2).
* Pinned by the reference's only curve known-answer test,
  key/curve_test.go:10-30 (TestBLS12381Compatv112): the signature bytes pin
  the G2 DST, hash-to-G2, scalar multiplication and G2 compression.
  tests/test_oracle.py::test_kat_bls12381_compat_v112 checks it bit-exactly.

This module is written for clarity and for small inputs (a pairing costs
~0.1 s); the C restatement in oracle/c/ is the fast CPU oracle/baseline.
"""

import hashlib

# ---------------------------------------------------------------- constants
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_X = -0xD201000000010000  # curve parameter x (negative)
BLS_X_ABS = 0xD201000000010000

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)

# G2 effective cofactor h_eff (RFC 9380 section 8.8.2)
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551
# G1 effective cofactor h_eff = 1 - x
H_EFF_G1 = 0xD201000000010001

DST_G2 = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"

# ---------------------------------------------------------------- Fp
def fp_inv(a):
    return pow(a, P - 2, P)


def fp_sqrt(a):
    """sqrt in Fp (p = 3 mod 4); None if a is a non-residue."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sgn0(a):
    return a % P & 1


# ---------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a0, a1=0):
    return (a0 % P, a1 % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return ((a[0] + a[1]) * (a[0] - a[1]) % P, 2 * a[0] * a[1] % P)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fp_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1] * t) % P)


def f2_mul_xi(a):
    """multiply by xi = 1 + u"""
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2_eq(a, b):
    return (a[0] - b[0]) % P == 0 and (a[1] - b[1]) % P == 0


def f2_is_square(a):
    # a is a square in Fp2 iff its norm is a square in Fp
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """A square root of a in Fp2, or None.  (Which root is returned does not
    matter to any caller: every caller fixes the sign afterwards.)"""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)
        return (0, s) if s is not None else None
    g = fp_sqrt(a0 * a0 + a1 * a1)
    if g is None:
        return None
    inv2 = (P + 1) // 2
    d = (a0 + g) * inv2 % P
    if not fp_is_square(d):
        d = (a0 - g) * inv2 % P
    x0 = fp_sqrt(d)
    if x0 is None or x0 == 0:
        return None
    x1 = a1 * fp_inv(2 * x0) % P
    r = (x0, x1)
    return r if f2_eq(f2_sqr(r), (a0, a1)) else None


def f2_sgn0(a):
    """RFC 9380 sgn0 for m = 2."""
    s0 = a[0] % P & 1
    z0 = a[0] % P == 0
    s1 = a[1] % P & 1
    return s0 | (z0 & s1)


def f2_frob(a):
    return f2_conj(a)


# ---------------------------------------------------------------- Fp6 = Fp2[v]/(v^3 - xi)
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), f2_add(t1, t2))))
    c1 = f2_add(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), f2_add(t0, t1)), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), f2_add(t0, t2)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    """multiply by v"""
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ---------------------------------------------------------------- Fp12 = Fp6[w]/(w^2 - v)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), f6_add(t0, t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


def f12_eq(a, b):
    return all(f2_eq(a[i][j], b[i][j]) for i in range(2) for j in range(3))


def f12_is_one(a):
    return f12_eq(a, F12_ONE)


def f12_to_ints(a):
    """Flatten to 12 Fp ints: order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... (Fp6 c0, then c1)."""
    out = []
    for i in range(2):
        for j in range(3):
            out.extend([a[i][j][0] % P, a[i][j][1] % P])
    return out


def f12_from_fp2_basis(coeffs):
    """Build Fp12 from Fp2 coefficients of 1, w, w^2, w^3, w^4, w^5.
    w^2 = v: 1->c0.c0, w->c1.c0, w^2->c0.c1, w^3->c1.c1, w^4->c0.c2, w^5->c1.c2"""
    c = coeffs
    return ((c[0], c[2], c[4]), (c[1], c[3], c[5]))


# ---------------------------------------------------------------- curve points (affine, None = infinity)
B1 = 4
B2 = (4, 4)  # 4 * (1 + u)


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * fp_inv(2 * y1) % P
    else:
        lam = (y2 - y1) * fp_inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_mul(pt, k):
    if k < 0:
        return g1_mul(g1_neg(pt), -k)
    r = None
    while k:
        if k & 1:
            r = g1_add(r, pt)
        pt = g1_add(pt, pt)
        k >>= 1
    return r


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2_is_zero(f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)))


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if f2_eq(x1, x2):
        if f2_is_zero(f2_add(y1, y2)):
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def g2_mul(pt, k):
    if k < 0:
        return g2_mul(g2_neg(pt), -k)
    r = None
    while k:
        if k & 1:
            r = g2_add(r, pt)
        pt = g2_add(pt, pt)
        k >>= 1
    return r


G1_GEN = (G1_X, G1_Y)
G2_GEN = (G2_X, G2_Y)

# psi endomorphism constants (untwist-Frobenius-twist), derived from definitions
XI = (1, 1)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    return (f2_mul(f2_frob(pt[0]), PSI_CX), f2_mul(f2_frob(pt[1]), PSI_CY))


def g1_in_subgroup(pt):
    return g1_mul(pt, R) is None


def g2_in_subgroup(pt):
    return g2_mul(pt, R) is None


# ---------------------------------------------------------------- serialization (ZCash format)
def fp_to_bytes(a):
    return (a % P).to_bytes(48, "big")


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    out = bytearray(fp_to_bytes(x))
    out[0] |= 0x80
    if y % P > (P - 1) // 2:
        out[0] |= 0x20
    return bytes(out)


def g2_lexi_largest(y):
    y0, y1 = y[0] % P, y[1] % P
    half = (P - 1) // 2
    return y1 > half or (y1 == 0 and y0 > half)


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    out = bytearray(fp_to_bytes(x[1]) + fp_to_bytes(x[0]))
    out[0] |= 0x80
    if g2_lexi_largest(y):
        out[0] |= 0x20
    return bytes(out)


class DecodeError(ValueError):
    pass


def g1_decompress(data, check_subgroup=True):
    """kilic G1.FromCompressed semantics (R): length 48, compression flag set,
    canonical infinity, x < p, on curve, in subgroup."""
    if len(data) != 48:
        raise DecodeError("length")
    b0 = data[0]
    if not b0 & 0x80:
        raise DecodeError("compression flag")
    if b0 & 0x40:
        if (b0 & 0x3F) or any(data[1:]):
            raise DecodeError("non-canonical infinity")
        return None
    sign = bool(b0 & 0x20)
    x = int.from_bytes(bytes([b0 & 0x1F]) + data[1:], "big")
    if x >= P:
        raise DecodeError("x >= p")
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise DecodeError("not on curve")
    if (y > (P - 1) // 2) != sign:
        y = (-y) % P
    pt = (x, y)
    if check_subgroup and not g1_in_subgroup(pt):
        raise DecodeError("not in subgroup")
    return pt


def g2_decompress(data, check_subgroup=True):
    """kilic G2.FromCompressed semantics (R): length 96, c1 || c0, flags as G1."""
    if len(data) != 96:
        raise DecodeError("length")
    b0 = data[0]
    if not b0 & 0x80:
        raise DecodeError("compression flag")
    if b0 & 0x40:
        if (b0 & 0x3F) or any(data[1:]):
            raise DecodeError("non-canonical infinity")
        return None
    sign = bool(b0 & 0x20)
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + data[1:48], "big")
    x0 = int.from_bytes(data[48:96], "big")
    if x0 >= P or x1 >= P:
        raise DecodeError("x >= p")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    if g2_lexi_largest(y) != sign:
        y = f2_neg(y)
    pt = (x, y)
    if check_subgroup and not g2_in_subgroup(pt):
        raise DecodeError("not in subgroup")
    return pt


# ---------------------------------------------------------------- hash to curve (RFC 9380)
def expand_message_xmd(msg, dst, length):
    assert len(dst) <= 255
    ell = (length + 31) // 32
    assert ell <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(64)
    l_i_b = length.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:length]


def hash_to_field_fp2(msg, count, dst):
    L = 64
    u = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = [int.from_bytes(u[L * (j + 2 * i): L * (j + 2 * i + 1)], "big") % P for j in range(2)]
        out.append((e[0], e[1]))
    return out


def hash_to_field_fp(msg, count, dst):
    L = 64
    u = expand_message_xmd(msg, dst, count * L)
    return [int.from_bytes(u[L * i: L * (i + 1)], "big") % P for i in range(count)]


# SSWU on E2': y^2 = x^3 + A'x + B'
SSWU2_A = (0, 240)
SSWU2_B = (1012, 1012)
SSWU2_Z = f2(-2, -1)


def map_to_curve_sswu_g2(u):
    A, B, Z = SSWU2_A, SSWU2_B, SSWU2_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        tv1 = f2_inv(den)
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


# 3-isogeny E2' -> E2 (RFC 9380 appendix E.3)
_I = lambda a, b=0: f2(a, b)  # noqa: E731
ISO3_XNUM = [
    _I(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
       0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    _I(0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    _I(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    _I(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO3_XDEN = [
    _I(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    _I(0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    _I(1, 0),
]
ISO3_YNUM = [
    _I(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
       0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    _I(0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    _I(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    _I(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO3_YDEN = [
    _I(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
       0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    _I(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    _I(0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    _I(1, 0),
]


def _f2_poly(coeffs, x):
    acc = coeffs[-1]
    for c in reversed(coeffs[:-1]):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    x, y = pt
    xn = _f2_poly(ISO3_XNUM, x)
    xd = _f2_poly(ISO3_XDEN, x)
    yn = _f2_poly(ISO3_YNUM, x)
    yd = _f2_poly(ISO3_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


def clear_cofactor_g2(pt):
    """h_eff * P via the psi decomposition (RFC 9380 G.3):
    h_eff P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)."""
    x = BLS_X
    t1 = g2_mul(pt, x * x - x - 1)
    t2 = g2_mul(g2_psi(pt), x - 1)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    return g2_add(g2_add(t1, t2), t3)


def hash_to_g2(msg, dst=DST_G2):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map_g2(map_to_curve_sswu_g2(u0))
    q1 = iso_map_g2(map_to_curve_sswu_g2(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ---------------------------------------------------------------- pairing
def _untwist(q):
    """E'(Fp2) -> E(Fp12): (x, y) -> (x / w^2, y / w^3)."""
    x, y = q
    # 1/w^2 = w^4 / xi, 1/w^3 = w^3 / xi ; w^4 -> c0.c2 , w^3 -> c1.c1
    xi_inv = f2_inv(XI)
    X = f12_from_fp2_basis([F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO, f2_mul(x, xi_inv), F2_ZERO])
    Y = f12_from_fp2_basis([F2_ZERO, F2_ZERO, F2_ZERO, f2_mul(y, xi_inv), F2_ZERO, F2_ZERO])
    return (X, Y)


def _f12_fp(a):
    return f12_from_fp2_basis([(a % P, 0), F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO])


def _f12_sub(a, b):
    return (f6_sub(a[0], b[0]), f6_sub(a[1], b[1]))


def _f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def _f12_smul(a, k):
    return f12_mul(a, _f12_fp(k))


def miller_loop(p, q):
    """f_{|x|,Q}(P) evaluated with generic affine line functions in E(Fp12),
    conjugated because x < 0.  Reference definition for the optimized code."""
    if p is None or q is None:
        return F12_ONE
    Qx, Qy = _untwist(q)
    Px, Py = _f12_fp(p[0]), _f12_fp(p[1])
    Tx, Ty = Qx, Qy
    f = F12_ONE
    bits = bin(BLS_X_ABS)[3:]
    for b in bits:
        # tangent at T
        lam = f12_mul(_f12_smul(f12_sqr(Tx), 3), f12_inv(_f12_smul(Ty, 2)))
        line = _f12_sub(_f12_sub(Py, Ty), f12_mul(lam, _f12_sub(Px, Tx)))
        f = f12_mul(f12_sqr(f), line)
        x3 = _f12_sub(_f12_sub(f12_sqr(lam), Tx), Tx)
        Ty = _f12_sub(f12_mul(lam, _f12_sub(Tx, x3)), Ty)
        Tx = x3
        if b == "1":
            lam = f12_mul(_f12_sub(Qy, Ty), f12_inv(_f12_sub(Qx, Tx)))
            line = _f12_sub(_f12_sub(Py, Ty), f12_mul(lam, _f12_sub(Px, Tx)))
            f = f12_mul(f, line)
            x3 = _f12_sub(_f12_sub(f12_sqr(lam), Tx), Qx)
            Ty = _f12_sub(f12_mul(lam, _f12_sub(Tx, x3)), Ty)
            Tx = x3
    return f12_conj(f)  # x < 0


FINAL_EXP_HARD_3 = 3 * (P ** 4 - P ** 2 + 1) // R


def final_exponentiation(f):
    """f^((p^12-1)/r * 3).  The factor 3 (coprime to r) matches the addition
    chain (x-1)^2 (x+p)(x^2+p^2-1)+3 used by the optimized implementations;
    f^(3k) == 1 iff f^k == 1."""
    # easy part: f^((p^6-1)(p^2+1))
    f1 = f12_mul(f12_conj(f), f12_inv(f))
    f2_ = f12_mul(f12_pow(f1, P * P), f1)  # generic pow for p^2 (clear, slow)
    return f12_pow(f2_, FINAL_EXP_HARD_3)


def pairing(p, q):
    return final_exponentiation(miller_loop(p, q))


def pairing_check(pairs):
    """prod e(P_i, Q_i) == 1 ; pairs with an infinity point are skipped (kilic AddPair (R))."""
    f = F12_ONE
    for p, q in pairs:
        if p is None or q is None:
            continue
        f = f12_mul(f, miller_loop(p, q))
    return f12_is_one(final_exponentiation(f))


# ---------------------------------------------------------------- BLS on G2 (kyber sign/bls, tbls)
def sk_to_pk(sk):
    return g1_compress(g1_mul(G1_GEN, sk))


def sign_g2(sk, msg, dst=DST_G2):
    return g2_compress(g2_mul(hash_to_g2(msg, dst), sk % R))


def verify_g2(pk_point, msg, sig_bytes, dst=DST_G2):
    """kyber sign/bls Verify (R): HM = Hash(msg); sig = UnmarshalBinary (error ->
    invalid); ValidatePairing(pk, HM, g1, sig) i.e. e(pk,HM) * e(-g1,sig) == 1."""
    try:
        sig = g2_decompress(sig_bytes)
    except DecodeError:
        return False
    hm = hash_to_g2(msg, dst)
    return pairing_check([(pk_point, hm), (g1_neg(G1_GEN), sig)])


# ---------------------------------------------------------------- hash to G1 (RFC 9380 section 8.8.1)
# Suite BLS12381G1_XMD:SHA-256_SSWU_RO_: expand_message_xmd (128 bytes), two
# Fp elements, simplified SWU on E1' (Z = 11), the 11-isogeny E1' -> E1
# (constants derived in tools/derive_iso11.py, pinned there by RFC 9380's
# published k_(1,0) and test vector J.9.1), h_eff = 1 - x.
from .iso11_consts import (ISO11_XDEN, ISO11_XNUM, ISO11_YDEN, ISO11_YNUM,  # noqa: E402
                           SSWU1_A, SSWU1_B, SSWU1_Z)

DST_G1 = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"


def map_to_curve_sswu_g1(u):
    A, Bc, Z = SSWU1_A, SSWU1_B, SSWU1_Z
    u %= P
    zu2 = Z * u * u % P
    den = (zu2 * zu2 + zu2) % P
    if den == 0:
        x1 = Bc * fp_inv(Z * A) % P
    else:
        x1 = (-Bc) * fp_inv(A) * (1 + fp_inv(den)) % P
    gx1 = (x1 * x1 * x1 + A * x1 + Bc) % P
    x2 = zu2 * x1 % P
    gx2 = (x2 * x2 * x2 + A * x2 + Bc) % P
    if fp_is_square(gx1):
        x, y = x1, fp_sqrt(gx1)
    else:
        x, y = x2, fp_sqrt(gx2)
    if fp_sgn0(u) != fp_sgn0(y):
        y = (-y) % P
    return (x, y)


def _fp_poly(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % P
    return acc


def iso_map_g1(pt):
    x, y = pt
    xd, yd = _fp_poly(ISO11_XDEN, x), _fp_poly(ISO11_YDEN, x)
    if xd == 0 or yd == 0:
        return None
    return (_fp_poly(ISO11_XNUM, x) * fp_inv(xd) % P, y * _fp_poly(ISO11_YNUM, x) * fp_inv(yd) % P)


def clear_cofactor_g1(pt):
    return g1_mul(pt, H_EFF_G1)


def hash_to_g1(msg, dst=DST_G1):
    u0, u1 = hash_to_field_fp(msg, 2, dst)
    return clear_cofactor_g1(g1_add(iso_map_g1(map_to_curve_sswu_g1(u0)), iso_map_g1(map_to_curve_sswu_g1(u1))))


# ---------------------------------------------------------------- BLS with signatures on G1 (kyber NewSchemeOnG1 (R))
def sk_to_pk_g2(sk):
    return g2_compress(g2_mul(G2_GEN, sk % R))


def sign_g1(sk, msg, dst=DST_G1):
    return g1_compress(g1_mul(hash_to_g1(msg, dst), sk % R))


def verify_g1(pk_point_g2, msg, sig_bytes, dst=DST_G1):
    """bls.Verify on G1 (R): HM = Hash(msg) in G1; sig = G1 UnmarshalBinary
    (error -> invalid); e(HM, pk) * e(-sig, g2) == 1."""
    try:
        sig = g1_decompress(sig_bytes)
    except DecodeError:
        return False
    if sig is None:
        return False
    return pairing_check([(hash_to_g1(msg, dst), pk_point_g2), (g1_neg(sig), G2_GEN)])
