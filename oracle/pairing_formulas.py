"""Python mirror of the optimized pairing formulas the HIP kernels use
(TEST INFRASTRUCTURE: lets tests compare kernel intermediates element by
element).  Correctness of these formulas is established against the generic
definition in bls12381.py (tests/test_oracle.py::test_projective_miller_matches_generic).

Doubling (homogeneous projective T = (X, Y, Z) on E': y^2 = x^3 + b'), line
evaluated at P = (xP, yP) after untwisting (x, y) -> (x/w^2, y/w^3) and
scaling by w^3 * 2y'Z^2 (subfield factors, killed by the final exponentiation):
    l = (Y^2 - 3b'Z^2) + (-3 X^2 xP) w^2 + (2 Y Z yP) w^3
Mixed addition with affine Q = (xQ, yQ), theta = Y - yQ Z, lam = X - xQ Z:
    l = (theta xQ - lam yQ) + (-theta xP) w^2 + (lam yP) w^3
"""
from . import bls12381 as B

f2_add, f2_sub, f2_mul, f2_sqr, f2_neg = B.f2_add, B.f2_sub, B.f2_mul, B.f2_sqr, B.f2_neg
B2_3 = (12, 12)  # 3 b'


def f2_half(a):
    inv2 = (B.P + 1) // 2
    return (a[0] * inv2 % B.P, a[1] * inv2 % B.P)


def dbl_step(T, xP, yP):
    X, Y, Z = T
    t0 = f2_sqr(Y)
    t1 = f2_sqr(Z)
    t2 = f2_mul(B2_3, t1)
    t3 = f2_add(f2_add(t2, t2), t2)
    XY = f2_mul(X, Y)
    X3 = f2_mul(f2_half(XY), f2_sub(t0, t3))
    Y3 = f2_sub(f2_sqr(f2_half(f2_add(t0, t3))), f2_mul((3, 0), f2_sqr(t2)))
    yz2 = f2_sub(f2_sqr(f2_add(Y, Z)), f2_add(t0, t1))
    Z3 = f2_mul(t0, yz2)
    c0 = f2_sub(t0, t2)
    c2 = B.f2_muls(f2_mul((3, 0), f2_sqr(X)), (-xP) % B.P)
    c3 = B.f2_muls(yz2, yP)
    return (X3, Y3, Z3), (c0, c2, c3)


def add_step(T, Q, xP, yP):
    X, Y, Z = T
    xQ, yQ = Q
    theta = f2_sub(Y, f2_mul(yQ, Z))
    lam = f2_sub(X, f2_mul(xQ, Z))
    C = f2_sqr(theta)
    D = f2_sqr(lam)
    E = f2_mul(lam, D)
    F = f2_mul(Z, C)
    G = f2_mul(X, D)
    H = f2_sub(f2_add(E, F), f2_add(G, G))
    X3 = f2_mul(lam, H)
    Y3 = f2_sub(f2_mul(theta, f2_sub(G, H)), f2_mul(Y, E))
    Z3 = f2_mul(Z, E)
    c0 = f2_sub(f2_mul(theta, xQ), f2_mul(lam, yQ))
    c2 = B.f2_muls(theta, (-xP) % B.P)
    c3 = B.f2_muls(lam, yP)
    return (X3, Y3, Z3), (c0, c2, c3)


def line_to_f12(c):
    c0, c2, c3 = c
    z = B.F2_ZERO
    return B.f12_from_fp2_basis([c0, z, c2, c3, z, z])


def miller_loop_multi(pairs):
    """Shared-squaring multi Miller loop over (P affine G1, Q affine G2) pairs,
    conjugated at the end (x < 0).  Pairs with an infinity point are skipped."""
    pairs = [(p, q) for p, q in pairs if p is not None and q is not None]
    Ts = [(q[0], q[1], B.F2_ONE) for _, q in pairs]
    f = B.F12_ONE
    bits = bin(B.BLS_X_ABS)[3:]
    for b in bits:
        f = B.f12_sqr(f)
        for k, (p, q) in enumerate(pairs):
            Ts[k], line = dbl_step(Ts[k], p[0], p[1])
            f = B.f12_mul(f, line_to_f12(line))
        if b == "1":
            for k, (p, q) in enumerate(pairs):
                Ts[k], line = add_step(Ts[k], q, p[0], p[1])
                f = B.f12_mul(f, line_to_f12(line))
    return B.f12_conj(f)


def f12_frob(a, k):
    """a^(p^k) via the generic power (slow; tests only)."""
    return B.f12_pow(a, B.P ** k)


def exp_by_x(a):
    """a^x for x < 0 on the cyclotomic subgroup: conj(a^|x|)."""
    return B.f12_conj(B.f12_pow(a, B.BLS_X_ABS))


def final_exp_chain(f):
    """Easy part then the hard-part chain
    3*(p^4-p^2+1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3."""
    f1 = B.f12_mul(B.f12_conj(f), B.f12_inv(f))
    f = B.f12_mul(f12_frob(f1, 2), f1)
    t0 = B.f12_mul(exp_by_x(f), B.f12_conj(f))
    t1 = B.f12_mul(exp_by_x(t0), B.f12_conj(t0))
    t2 = B.f12_mul(exp_by_x(t1), f12_frob(t1, 1))
    t3 = B.f12_mul(B.f12_mul(exp_by_x(exp_by_x(t2)), f12_frob(t2, 2)), B.f12_conj(t2))
    return B.f12_mul(t3, B.f12_mul(B.f12_sqr(f), f))
