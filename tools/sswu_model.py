"""Reference model of the kernels' inversion-free SSWU + 3-isogeny
(drand_amd/csrc/h2c.cuh map_to_curve_sswu_iso3), written with the oracle's
field helpers so tests can check it against oracle.bls12381's
RFC 9380 map_to_curve_simple_swu + iso_map on many inputs.

Per field element u it costs two Fp exponentiations and no inversion:

  zu2 = Z u^2, den = zu2^2 + zu2;  x1 = N / D with
      N = (-B/A)(den + 1), D = den      (den = 0: N = B/(Z A), D = 1)
  gx1 = U / D^3, U = N (N^2 + A D^2) + B D^3;   w1 = U D  (square iff gx1 is)
  gx2 = zu2^3 gx1 (RFC 9380 6.6.2), so w2 = zu2^3 w1 and x2 = zu2 x1.
  Norm method (p = 3 mod 4):
      alpha1 = norm(w1), g = alpha1^((p+1)/4)                   [exp 1]
      gx1 square iff g^2 = alpha1; otherwise g^2 = -alpha1 and
      sqrt(norm(w2)) = sqrt(-125) norm(u)^3 g   (norm(Z) = 5, a non-square)
      d = (w0 + g) / 2 (or (w0 - g) / 2 if that is 0, i.e. w1 = 0),
      m = norm(D), t = (d m^4)^((p-3)/4)                        [exp 2]
      d m^4 square:     y' = d t + (w1 t / 2) u
      otherwise:        y' = (w1 t / 2) - d t u
      y = y' conj(D)^2  (= sqrt(w) / D^2 = sqrt(gx)),  then the sgn0 fix.
  The isogeny is evaluated on x = N / D homogeneously; the result is a
  Jacobian point (X, Y, Z) with Z = 0 for the exceptional inputs.
"""
from oracle import bls12381 as B

P = B.P
SQRT_M125 = pow((-125) % P, (P + 1) // 4, P)
assert SQRT_M125 * SQRT_M125 % P == (-125) % P
HALF = pow(2, P - 2, P)


def _norm(a):
    return (a[0] * a[0] + a[1] * a[1]) % P


def _poly_h(coeffs, N, D):
    """sum_i c_i N^i D^(deg - i) for coefficients c_0..c_deg."""
    deg = len(coeffs) - 1
    acc = B.F2_ZERO
    for i, c in enumerate(coeffs):
        term = c
        for _ in range(i):
            term = B.f2_mul(term, N)
        for _ in range(deg - i):
            term = B.f2_mul(term, D)
        acc = B.f2_add(acc, term)
    return acc


def sqrt_scaled(w, g, m):
    """sqrt(w) / m^2 for w in Fp2 with norm(w) = g^2, m in Fp nonzero."""
    d = (w[0] + g) * HALF % P
    if d == 0:
        d = (w[0] - g) * HALF % P
    dm4 = d * pow(m, 4, P) % P
    t = pow(dm4, (P - 3) // 4, P)
    if dm4 * t * t % P == 1:
        return (d * t % P, w[1] * t * HALF % P)
    return (w[1] * t * HALF % P, (-d * t) % P)


def fp2_sqrt(a):
    """The kernels' fp2_sqrt: None if a is not a square."""
    alpha = _norm(a)
    g = pow(alpha, (P + 1) // 4, P)
    if g * g % P != alpha:
        return None
    return sqrt_scaled(a, g, 1)


def sswu_iso3_jacobian(u):
    A, Bc, Z = B.SSWU2_A, B.SSWU2_B, B.SSWU2_Z
    zu2 = B.f2_mul(Z, B.f2_sqr(u))
    den = B.f2_add(B.f2_sqr(zu2), zu2)
    if B.f2_is_zero(den):
        N, D = B.f2_mul(Bc, B.f2_inv(B.f2_mul(Z, A))), B.F2_ONE
    else:
        N = B.f2_mul(B.f2_mul(B.f2_neg(Bc), B.f2_inv(A)), B.f2_add(den, B.F2_ONE))
        D = den
    D2 = B.f2_sqr(D)
    U = B.f2_add(B.f2_mul(N, B.f2_add(B.f2_sqr(N), B.f2_mul(A, D2))), B.f2_mul(Bc, B.f2_mul(D2, D)))
    w = B.f2_mul(U, D)
    alpha = _norm(w)
    g = pow(alpha, (P + 1) // 4, P)
    if g * g % P != alpha:  # gx1 non-square: take x2, w2
        g = SQRT_M125 * pow(_norm(u), 3, P) * g % P
        w = B.f2_mul(B.f2_mul(B.f2_sqr(zu2), zu2), w)
        N = B.f2_mul(zu2, N)
    y = B.f2_mul(sqrt_scaled(w, g, _norm(D)), B.f2_sqr(B.f2_conj(D)))
    if B.f2_sgn0(u) != B.f2_sgn0(y):
        y = B.f2_neg(y)
    XN = _poly_h(B.ISO3_XNUM, N, D)
    XD = _poly_h(B.ISO3_XDEN, N, D)
    YN = _poly_h(B.ISO3_YNUM, N, D)
    YD = _poly_h(B.ISO3_YDEN, N, D)
    XDD = B.f2_mul(XD, D)
    T = B.f2_mul(XDD, B.f2_sqr(YD))
    X = B.f2_mul(XN, T)
    Y = B.f2_mul(B.f2_mul(y, YN), B.f2_mul(B.f2_sqr(XDD), T))
    Zj = B.f2_mul(XDD, YD)
    return X, Y, Zj


def to_affine(J):
    X, Y, Zj = J
    if B.f2_is_zero(Zj):
        return None
    zi = B.f2_inv(Zj)
    zi2 = B.f2_sqr(zi)
    return (B.f2_mul(X, zi2), B.f2_mul(Y, B.f2_mul(zi2, zi)))


# ---------------------------------------------------------------- G1: SSWU on E1' + 11-isogeny, inversion-free
def sswu_iso11_jacobian(u):
    """Kernel model (h2c_g1.cuh map_to_curve_sswu_iso11): x1 = N/D, gx1 = U/D^3;
    t = (U V^3)^((p-3)/4) with V = D^3 gives y1 = U V t, a square root of
    gx1 when y1^2 V = U, else of -gx1; then sqrt(gx2) = Z u^3 sqrt(-Z) y1
    (gx2 = Z^3 u^6 gx1, -Z a square).  One exponentiation, no inversion."""
    from oracle import iso11_consts as I
    A, Bc, Z = I.SSWU1_A, I.SSWU1_B, I.SSWU1_Z
    sqrt_mz = pow((-Z) % P, (P + 1) // 4, P)
    assert sqrt_mz * sqrt_mz % P == (-Z) % P
    u %= P
    zu2 = Z * u * u % P
    den = (zu2 * zu2 + zu2) % P
    if den == 0:
        N, D = Bc * pow(Z * A, P - 2, P) % P, 1
    else:
        N, D = (-Bc) * pow(A, P - 2, P) * (den + 1) % P, den
    D3 = pow(D, 3, P)
    U = (N * (N * N + A * D * D) + Bc * D3) % P
    t = pow(U * pow(D3, 3, P) % P, (P - 3) // 4, P)
    y = U * D3 * t % P
    if y * y * D3 % P != U:
        y = Z * pow(u, 3, P) * sqrt_mz * y % P
        N = zu2 * N % P
    if (u & 1) != (y & 1):
        y = (-y) % P

    def hom(coeffs, deg):
        return sum(c * pow(N, i, P) * pow(D, deg - i, P) for i, c in enumerate(coeffs)) % P
    xn, xd = hom(I.ISO11_XNUM, 11), hom(I.ISO11_XDEN, 10)
    yn, yd = hom(I.ISO11_YNUM, 15), hom(I.ISO11_YDEN, 15)
    xdd = xd * D % P
    T = xdd * yd * yd % P
    return xn * T % P, y * yn * xdd * xdd % P * T % P, xdd * yd % P


def g1_to_affine(J):
    X, Y, Zj = J
    if Zj % P == 0:
        return None
    zi = pow(Zj, P - 2, P)
    return (X * zi * zi % P, Y * zi * zi * zi % P)
