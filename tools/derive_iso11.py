#!/usr/bin/env python3
"""Derive the 11-isogeny E1' -> E1 of RFC 9380's BLS12-381 G1 suite
(appendix E.2) from first principles and write oracle/iso11_consts.py.

E1': y^2 = x^3 + A'x + B' (RFC 9380 section 8.8.1, SSWU curve, Z = 11) is
11-isogenous to E1: y^2 = x^3 + 4.  Steps:
  1. #E1'(Fp) = #E1(Fp) = p + 1 - t, t = x + 1 (checked on random points:
     isogenous curves have equal order, Tate).
  2. The 11-division polynomial f11 (degree 60): its roots in Fp (11
     divides the G1 cofactor, so E1'(Fp) has a rational 11-subgroup) and its
     degree-5 irreducible factors (gcd with x^(p^5) - x, Cantor-Zassenhaus)
     give the kernel polynomials of the Fp-rational 11-isogenies.
  3. Kohel/Velu: codomain (A~, B~); keep the kernel with A~ = 0 (j = 0).
     x-map X = N / D^2 with N = x D^2 + D Tr(v(t) D/(x - t)) +
     Tr(u(t) (D/(x - t))^2), v = 6t^2 + 2a, u = 4(t^3 + a t + b), traces
     from Fp[t]/D(t) to Fp; y-map Y = y X'(x) (normalized isogeny).
  4. Isomorphism to y^2 = x^3 + 4: (s X, r Y) with s^3 = r^2 = 4 / B~.
     Three cube roots s x two signs r: the RFC's choice is fixed by its
     published constant k_(1,0) (x-map) and by the RFC 9380 J.9.1 test
     vector (y sign), both checked here.
Run: python tools/derive_iso11.py   (about a minute of pure Python)
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from oracle import bls12381 as B  # noqa: E402

P = B.P
A1 = 0x144698A3B8E9433D693A02C96D4982B0EA985383EE66A8D8E8981AEFD881AC98936F8DA0E0F97F5CF428082D584C1D
B1 = 0x12E2908D11688030018B12E8753EEE3B2016C1F0F24F4070A0B9C14FCEF35EF55A23215A316CEAA5D1CC48E98E172BE0
Z1 = 11
# RFC 9380 appendix E.2, first x_num coefficient, and test vector J.9.1 (msg = "")
K1_0 = 0x11A05F2B1E833340B809101DD99815856B303E88A2D7005FF2627B56CDB4E2C85610C2D5F2E62D6EAEAC1662734649B7
TV_DST = b"QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_"
TV_X = 0x052926ADD2207B76CA4FA57A8734416C8DC95E24501772C814278700EED6D1E4E8CF62D9C09DB0FAC349612B759E79A1
TV_Y = 0x08BA738453BFED09CB546DBB0783DBB3A5F1F566ED67BB6BE0E8C67E2E81A4CC68EE29813BB7994998F3EAE0C9C6A265


# ---------------------------------------------------------------- Fp[x] (coefficient lists, low degree first)
def trim(a):
    while a and a[-1] % P == 0:
        a.pop()
    return a


def padd(a, b):
    n = max(len(a), len(b))
    return trim([((a[i] if i < len(a) else 0) + (b[i] if i < len(b) else 0)) % P for i in range(n)])


def pneg(a):
    return [(-c) % P for c in a]


def psub(a, b):
    return padd(a, pneg(b))


def pscale(a, c):
    return trim([x * c % P for x in a])


def pmul(a, b):
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] += x * y
    return trim([c % P for c in out])


def pdivmod(a, b):
    a = list(a)
    inv = pow(b[-1], P - 2, P)
    q = [0] * max(1, len(a) - len(b) + 1)
    while len(trim(a)) >= len(b):
        d = len(a) - len(b)
        c = a[-1] * inv % P
        q[d] = c
        for i, y in enumerate(b):
            a[i + d] = (a[i + d] - c * y) % P
        trim(a)
    return trim(q), a


def pmod(a, m):
    return pdivmod(a, m)[1]


def pmonic(a):
    return pscale(a, pow(a[-1], P - 2, P)) if a else a


def pgcd(a, b):
    a, b = trim(list(a)), trim(list(b))
    while b:
        a, b = b, pmod(a, b)
    return pmonic(a)


def ppowmod(base, e, m):
    r, b = [1], pmod(base, m)
    while e:
        if e & 1:
            r = pmod(pmul(r, b), m)
        b = pmod(pmul(b, b), m)
        e >>= 1
    return r


def pderiv(a):
    return trim([i * a[i] % P for i in range(1, len(a))])


def peval(a, x):
    acc = 0
    for c in reversed(a):
        acc = (acc * x + c) % P
    return acc


# ---------------------------------------------------------------- curve helpers (affine, y^2 = x^3 + a x + b)
def ec_add(p1, p2, a):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + a) * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def ec_mul(pt, k, a):
    r = None
    while k:
        if k & 1:
            r = ec_add(r, pt, a)
        pt = ec_add(pt, pt, a)
        k >>= 1
    return r


def random_point(a, b, rng):
    while True:
        x = rng.randrange(P)
        y = B.fp_sqrt(x * x * x + a * x + b)
        if y is not None:
            return (x, y)


# ---------------------------------------------------------------- division polynomial f_n (f_n = psi_n / (2y) for even n)
def division_poly(a, b, n):
    y4 = pmul([b, a, 0, 1], [b, a, 0, 1])  # (x^3 + a x + b)^2
    c16y4 = pscale(y4, 16)
    f = {0: [], 1: [1], 2: [1],
         3: trim([(-a * a) % P, 12 * b % P, 6 * a % P, 0, 3]),
         4: pscale([(-8 * b * b - a ** 3) % P, (-4 * a * b) % P, (-5 * a * a) % P, 20 * b % P, 5 * a % P, 0, 1], 2)}

    def get(k):
        if k in f:
            return f[k]
        m = k // 2
        if k & 1:
            if m % 2 == 0:
                r = psub(pmul(c16y4, pmul(get(m + 2), pmul(get(m), pmul(get(m), get(m))))),
                         pmul(get(m - 1), pmul(get(m + 1), pmul(get(m + 1), get(m + 1)))))
            else:
                r = psub(pmul(get(m + 2), pmul(get(m), pmul(get(m), get(m)))),
                         pmul(c16y4, pmul(get(m - 1), pmul(get(m + 1), pmul(get(m + 1), get(m + 1))))))
        else:
            r = pmul(get(m), psub(pmul(get(m + 2), pmul(get(m - 1), get(m - 1))),
                                  pmul(get(m - 2), pmul(get(m + 1), get(m + 1)))))
        f[k] = r
        return r

    return get(n)


def split_equal_degree(f, d, rng):
    if len(f) - 1 == d:
        return [f]
    while True:
        a = [rng.randrange(P) for _ in range(len(f) - 1)]
        g = pgcd(f, psub(ppowmod(a, (P ** d - 1) // 2, f), [1]))
        if 0 < len(g) - 1 < len(f) - 1:
            return split_equal_degree(g, d, rng) + split_equal_degree(pdivmod(f, g)[0], d, rng)


# ---------------------------------------------------------------- Fp[t]/D(t) arithmetic for the traces
class Ext:
    def __init__(self, D):
        self.D = D
        self.d = len(D) - 1
        # traces of t^k, k < d, from the companion matrix
        self.tr = []
        M = [[0] * self.d for _ in range(self.d)]  # column j = t * t^j reduced
        for j in range(self.d):
            col = self.mulx([0] * j + [1])
            for i in range(self.d):
                M[i][j] = col[i]
        Mk = [[int(i == j) for j in range(self.d)] for i in range(self.d)]
        for k in range(self.d):
            self.tr.append(sum(Mk[i][i] for i in range(self.d)) % P)
            Mk = [[sum(Mk[i][l] * M[l][j] for l in range(self.d)) % P for j in range(self.d)] for i in range(self.d)]

    def red(self, a):
        r = pmod(trim(list(a)), self.D)
        return r + [0] * (self.d - len(r))

    def mulx(self, a):
        return self.red([0] + list(a))

    def mul(self, a, b):
        return self.red(pmul(trim(list(a)), trim(list(b))))

    def add(self, a, b):
        return [(x + y) % P for x, y in zip(a, b)]

    def trace(self, a):
        return sum(c * t for c, t in zip(a, self.tr)) % P


def kohel_maps(D, a, b):
    """Normalized isogeny with kernel polynomial D: (A~, B~, N, Dsq, ynum, yden)."""
    K = Ext(D)
    d = K.d
    # power sums p1..p3 from the traces
    p1, p2, p3 = K.trace(K.red([0, 1])), K.trace(K.red([0, 0, 1])), K.trace(K.red([0, 0, 0, 1]))
    v = (6 * p2 + 2 * a * d) % P
    w = (10 * p3 + 6 * a * p1 + 4 * b * d) % P
    At, Bt = (a - 5 * v) % P, (b - 7 * w) % P
    # Q(x) = D(x) / (x - t) with coefficients in K (synthetic division)
    Q = [None] * d
    Q[d - 1] = K.red([1])
    for i in range(d - 1, 0, -1):
        Q[i - 1] = K.add(K.red([D[i]]), K.mul(K.red([0, 1]), Q[i]))
    vt = K.red([2 * a % P, 0, 6])
    ut = K.red([4 * b % P, 4 * a % P, 0, 4])
    S1 = trim([K.trace(K.mul(vt, q)) for q in Q])
    QQ = [K.red([0])] * (2 * d - 1)
    for i in range(d):
        for j in range(d):
            QQ[i + j] = K.add(QQ[i + j], K.mul(Q[i], Q[j]))
    S2 = trim([K.trace(K.mul(ut, q)) for q in QQ])
    Dsq = pmul(D, D)
    N = padd(padd(pmul([0, 1], Dsq), pmul(D, S1)), S2)
    ynum = psub(pmul(pderiv(N), D), pscale(pmul(N, pderiv(D)), 2))
    yden = pmul(Dsq, D)
    return At, Bt, N, Dsq, ynum, yden


def fp_roots(poly, rng):
    """Roots in Fp of a small polynomial."""
    g = pgcd(poly, psub(ppowmod([0, 1], P, poly), [0, 1]))
    if len(g) <= 1:
        return []
    return [(-f[0]) * pow(f[1], P - 2, P) % P for f in split_equal_degree(g, 1, rng)]


def main():
    rng = random.Random(2024)
    a, b = A1, B1
    order = P + 1 - (B.BLS_X + 1)
    for _ in range(3):
        assert ec_mul(random_point(a, b, rng), order, a) is None, "E1' order != E1 order: wrong A', B'"
    print("E1' order check ok", flush=True)
    f11 = division_poly(a, b, 11)
    assert len(f11) == 61 and f11[-1] == 11
    xp = ppowmod([0, 1], P, f11)
    lin = pgcd(f11, psub(xp, [0, 1]))
    xpk = xp
    for _ in range(4):
        xpk = ppowmod(xpk, P, f11)
    g15 = pgcd(f11, psub(xpk, [0, 1]))
    g5 = pdivmod(g15, lin)[0] if len(lin) > 1 else g15
    print("degree-1 part", len(lin) - 1, "degree-5 part", len(g5) - 1, flush=True)
    # kernel polynomials: the rational 11-torsion (x-coordinates in Fp: 11
    # divides the G1 cofactor) and any irreducible degree-5 factor
    kernels = [lin] if len(lin) - 1 == 5 else []
    if len(g5) > 1:
        kernels += split_equal_degree(g5, 5, rng)
    assert kernels, "no degree-5 kernel polynomial"
    cands = []
    for D in kernels:
        At, Bt, N, Dsq, ynum, yden = kohel_maps(D, a, b)
        if At == 0:
            cands.append((D, Bt, N, Dsq, ynum, yden))
    print("kernels with j = 0 codomain:", len(cands), flush=True)
    assert cands, "no 11-isogeny to a j = 0 curve"
    for D, Bt, N, Dsq, ynum, yden in cands:
        c = 4 * pow(Bt, P - 2, P) % P
        r = B.fp_sqrt(c)
        assert r is not None
        for s in fp_roots([(-c) % P, 0, 0, 1], rng):
            xnum = pscale(N, s)
            print("candidate k_(1,0) =", hex(xnum[0]), flush=True)
            if xnum[0] != K1_0:
                continue
            for sign in (1, -1):
                maps = (xnum, Dsq, pscale(ynum, r * sign % P), yden)
                if hash_to_g1_with(maps, b"", TV_DST) == (TV_X, TV_Y):
                    write(maps)
                    print("11-isogeny derived; k_(1,0) and the RFC 9380 J.9.1 vector match")
                    return
    raise SystemExit("no candidate matched the RFC constants / test vector")


# ---------------------------------------------------------------- hash_to_G1 for the test-vector check
def sswu_g1(u):
    A, Bc, Z = A1, B1, Z1
    tv1 = (Z * Z * pow(u, 4, P) + Z * u * u) % P
    if tv1 == 0:
        x1 = Bc * pow(Z * A, P - 2, P) % P
    else:
        x1 = (-Bc) * pow(A, P - 2, P) * (1 + pow(tv1, P - 2, P)) % P
    gx1 = (x1 ** 3 + A * x1 + Bc) % P
    x2 = Z * u * u * x1 % P
    gx2 = (x2 ** 3 + A * x2 + Bc) % P
    if B.fp_is_square(gx1):
        x, y = x1, B.fp_sqrt(gx1)
    else:
        x, y = x2, B.fp_sqrt(gx2)
    if (u % 2) != (y % 2):
        y = (-y) % P
    return (x, y)


def iso_with(maps, pt):
    xnum, xden, ynum, yden = maps
    x, y = pt
    xd, yd = peval(xden, x), peval(yden, x)
    if xd == 0 or yd == 0:
        return None
    return (peval(xnum, x) * pow(xd, P - 2, P) % P, y * peval(ynum, x) * pow(yd, P - 2, P) % P)


def hash_to_g1_with(maps, msg, dst):
    u0, u1 = B.hash_to_field_fp(msg, 2, dst)
    q = B.g1_add(iso_with(maps, sswu_g1(u0)), iso_with(maps, sswu_g1(u1)))
    return B.g1_mul(q, 1 - B.BLS_X)


def write(maps):
    xnum, xden, ynum, yden = maps
    path = os.path.join(HERE, "..", "oracle", "iso11_consts.py")
    with open(path, "w") as f:
        f.write('"""GENERATED by tools/derive_iso11.py: RFC 9380 BLS12-381 G1 SSWU curve E1\' and\n'
                'the 11-isogeny E1\' -> E1 (coefficients low degree first; x = xnum/xden,\n'
                'y = y\' * ynum/yden).  Derived, not copied: see the generator."""\n')
        f.write(f"SSWU1_A = {hex(A1)}\nSSWU1_B = {hex(B1)}\nSSWU1_Z = {Z1}\n")
        for name, poly in (("ISO11_XNUM", xnum), ("ISO11_XDEN", xden), ("ISO11_YNUM", ynum), ("ISO11_YDEN", yden)):
            f.write(f"{name} = [\n" + "".join(f"    {hex(c)},\n" for c in poly) + "]\n")


if __name__ == "__main__":
    main()
