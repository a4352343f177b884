#!/usr/bin/env python3
"""Generator (and executable model) of the lane-cooperative pairing engine.

Design: a pairing is worked on by a GROUP of 12 lanes
of one wavefront (5 groups per wave64).  Every Fp12 / G2 value of the group
lives in LDS "slots" (one slot = one Fp element, 14 x 28-bit limbs,
Montgomery form).  An OP is a list of SUB-OPS; in a sub-op every lane k of
the group computes ONE Fp output

    out = reduce( cm * redc( sum_t coef_t * a_t * b'_t )  +  sum_u d_u * s_u )

where a_t, b_t, s_u are slots, b'_t is b_t or (8p - b_t) (negated), coef_t is
1 or 2, cm and d_u are small signed integers; the product sum is
accumulated double-width (28 limbs, no intermediate reduction: lazy
reduction) and Montgomery-reduced once.  The output is written to a slot
and/or exported (to HBM by the kernel).  All lanes of a sub-op read before
any lane writes, so ops may update in place.

This file
  * builds the op tables for the three kernels (k_lines, k_miller, k_fe),
  * emits drand_amd/csrc/engine_tables.h,
  * provides `Model`, a Python interpreter with exactly the device
    semantics (mod p), which tests/test_engine_model.py runs against the
    oracle's tower arithmetic (TEST INFRASTRUCTURE only).

Fp12 layout: Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u; an Fp12 value occupies 12
consecutive slots, w^k coefficient k at slots (2k, 2k+1) = (re, im).  (The
tower basis of tower.cuh is the same basis: c0.cj = w^(2j), c1.cj = w^(2j+1).)
"""
import os
import sys

LANES = 12
MAX_GROUP_SLOTS = 64
MAX_TERMS = 12        # engine.cuh prefetches a lane's term words into a 12-entry FIFO
SLOT_WORDS = 14       # 14 limbs of 28 bits, one 32-bit word each

# ---------------------------------------------------------------- block constant slots (>= 64)
C_ONE = 64
C_NXP0, C_YP0, C_NXP1, C_YP1 = 65, 66, 67, 68      # pairing points (-x, y): pair 0 = pk, pair 1 = -g1
C_G1 = 69                                         # gamma1_k, k = 1..5: (re, im) at 69 + 2(k-1)
C_G2 = 79                                         # gamma2_k (Fp), k = 1..5 at 79 + (k-1)
C_PSI = 84                                        # psi constants cx (re, im) at 84, 85; cy at 86, 87
N_CONST = 24

# export ids (k_lines): pair p line component e (l0.re, l0.im, l2.re, l2.im, l3.re, l3.im) -> 6p + e
# export ids (k_miller): 0..11 = f components, 12 = N1 (the Fp norm of f)
EXP_N1 = 12


class Rec:
    __slots__ = ("dst", "exp", "cm", "terms", "post")

    def __init__(self, dst=None, exp=None, cm=1, terms=(), post=()):
        self.dst, self.exp, self.cm = dst, exp, cm
        self.terms = list(terms)   # (a, b, sign, coef)   sign in {+1,-1}, coef in {1,2}
        self.post = list(post)     # (slot, d)
        if not self.terms:
            self.cm = 0


def T(a, b, sign=1, coef=1):
    return (a, b, sign, coef)


# ---------------------------------------------------------------- Fp2 helpers (slot pairs)
def fp2(base):
    return (base, base + 1)


def mul_terms(x, y, sign=1, coef=1):
    """(x*y).re and (x*y).im as term lists; x, y slot pairs."""
    re = [T(x[0], y[0], sign, coef), T(x[1], y[1], -sign, coef)]
    im = [T(x[0], y[1], sign, coef), T(x[1], y[0], sign, coef)]
    return re, im


def sqr_terms(x, sign=1, coef=1):
    """(x^2).re = x0^2 - x1^2, (x^2).im = 2 x0 x1"""
    re = [T(x[0], x[0], sign, coef), T(x[1], x[1], -sign, coef)]
    if coef == 1:
        im = [T(x[0], x[1], sign, 2)]
    else:
        im = [T(x[0], x[1], sign, 2), T(x[0], x[1], sign, 2)]
    return re, im


def fp12(base):
    return [fp2(base + 2 * k) for k in range(6)]


# ---------------------------------------------------------------- op builders
# Fused epilogue of a sub-op (FUSE_SUM / FUSE_DIFF per lane): after the
# sub-op's outputs are stored, lane k forms from its own output and its DPP
# partner's (lane k ^ 1, the other half of the same Fp2 value) own + partner
# (SUM, the re lane: re + im) or partner - own + 8p (DIFF, the im lane:
# re - im), normalized and NOT reduced (< 4.02p / < 10.02p), into slot dst --
# the a +- b sums a later squaring's one-product real part (a+b)(a-b) needs.
FUSE_SUM, FUSE_DIFF = 1, 2
FUSE_BOUND = {FUSE_SUM: 4.02, FUSE_DIFF: 10.02}


class Op:
    def __init__(self, name, subs, fuse=None):
        self.name = name
        self.subs = subs  # list of list[Rec] (<= 12 each)
        for s in subs:
            assert len(s) <= LANES, (name, len(s))
        # {sub index: [(dst slot, FUSE_*) or None per lane]}
        self.fuse = fuse or {}
        for si, lanes in self.fuse.items():
            sub = subs[si]
            for k, f in enumerate(lanes):
                if f is None:
                    continue
                # the partner lane holds the other half of the same Fp2 output
                assert sub[k].dst is not None and sub[k ^ 1].dst == sub[k].dst ^ 1, (name, si, k)
                assert f[1] == (FUSE_SUM if sub[k].dst % 2 == 0 else FUSE_DIFF), (name, si, k)


def pack(name, recs):
    """Split a flat list of records into sub-ops of <= 12 lanes."""
    return Op(name, [recs[i:i + LANES] for i in range(0, len(recs), LANES)])


def op_xi_copy(name, src_base, dst_base, ks):
    """dst[j] = xi * src[k] for k in ks (j-th copy), LIN."""
    recs = []
    for j, k in enumerate(ks):
        s = fp2(src_base + 2 * k)
        d = fp2(dst_base + 2 * j)
        recs.append(Rec(dst=d[0], post=[(s[0], 1), (s[1], -1)]))
        recs.append(Rec(dst=d[1], post=[(s[0], 1), (s[1], 1)]))
    return pack(name, recs)


def op_sqr12(name, F, XF, conj=False, XF0=None):
    """F <- F^2 (conj: F <- conj(F)^2 = conj(F^2)), in place; XF = xi*F[1..5],
    XF0 (optional) = xi*F[0].  The xi-copy of a coefficient a + bu is
    (a - b) + (a + b)u, so a square's real part a^2 - b^2 is ONE product of its
    xi-copy's halves: the squares f_i^2 (i = 0, 1, 2, no wrap) take 1 term
    instead of 2, and no output needs more than 7 (8 before)."""
    f = fp12(F)
    xf = {k: fp2(XF + 2 * (k - 1)) for k in range(1, 6)}
    if XF0 is not None:
        xf[0] = fp2(XF0)
    recs = []
    for k in range(6):
        re, im = [], []
        for i in range(6):
            for j in range(i, 6):
                if (i + j) % 6 != k:
                    continue
                wrap = i + j >= 6
                y = xf[j] if wrap else f[j]
                if i == j and not wrap and i in xf:
                    r = [T(xf[i][0], xf[i][1])]       # (a - b)(a + b)
                    m = [T(f[i][0], f[i][1], 1, 2)]   # 2ab
                elif i == j and not wrap:
                    r, m = sqr_terms(f[i])
                elif i == j:
                    r, m = mul_terms(f[i], y)
                else:
                    r, m = mul_terms(f[i], y, coef=2)
                re += r
                im += m
        sgn = -1 if (conj and k % 2) else 1
        recs.append(Rec(dst=f[k][0], cm=sgn, terms=re))
        recs.append(Rec(dst=f[k][1], cm=sgn, terms=im))
    return pack(name, recs)


def op_line_mul(name, F, L, XL=None, XF=None):
    """F <- F * (l0 + l2 w^2 + l3 w^3); L = (l0, l2, l3) at L..L+5.  The
    terms that wrap past w^6 carry a factor xi: with XL = (xi l2, xi l3) they
    read the line's xi-copies, with XF = {k: xi f_k} (k = 3, 4, 5) the
    coefficient's (round 3: from the previous op's fused epilogue, no per-line
    xi pass)."""
    f = fp12(F)
    l0, l2, l3 = fp2(L), fp2(L + 2), fp2(L + 4)
    xl = {2: fp2(XL), 3: fp2(XL + 2)} if XL is not None else None
    recs = []
    for k in range(6):
        re, im = [], []
        for src, coeff, sh in ((k, l0, 0), ((k - 2) % 6, l2, 2), ((k - 3) % 6, l3, 3)):
            if k >= sh:
                r, m = mul_terms(f[src], coeff)
            elif xl is not None:
                r, m = mul_terms(f[src], xl[sh])
            else:
                r, m = mul_terms(fp2(XF[src]), coeff)
            re += r
            im += m
        recs.append(Rec(dst=f[k][0], terms=re))
        recs.append(Rec(dst=f[k][1], terms=im))
    return pack(name, recs)


def op_mul12(name, R, A, XA, conj_a=False):
    """R <- R * A (conj_a: R * conj(A)); XA = xi*A[1..5]."""
    r, a = fp12(R), fp12(A)
    xa = {k: fp2(XA + 2 * (k - 1)) for k in range(1, 6)}
    recs = []
    for k in range(6):
        re, im = [], []
        for i in range(6):
            j = (k - i) % 6
            y = a[j] if i <= k else xa[j]
            s = -1 if (conj_a and j % 2) else 1
            rr, mm = mul_terms(r[i], y, sign=s)
            re += rr
            im += mm
        recs.append(Rec(dst=r[k][0], terms=re))
        recs.append(Rec(dst=r[k][1], terms=im))
    return pack(name, recs)


def op_mul_fp6(name, R, N, XN, out=None):
    """out <- R * n, n = n0 + n1 w^2 + n2 w^4 (slots N: n0, n1, n2), XN = (xi n1, xi n2)."""
    r = fp12(R)
    o = fp12(out if out is not None else R)
    n = [fp2(N + 2 * j) for j in range(3)]
    xn = {1: fp2(XN), 2: fp2(XN + 2)}
    recs = []
    for k in range(6):
        re, im = [], []
        for j in range(3):
            i = (k - 2 * j) % 6
            y = xn[j] if 2 * j > k else n[j]
            rr, mm = mul_terms(r[i], y)
            re += rr
            im += mm
        recs.append(Rec(dst=o[k][0], terms=re))
        recs.append(Rec(dst=o[k][1], terms=im))
    return pack(name, recs)


def op_norm6(name, F, XF, N):
    """N <- f * conj(f) (in Fp6: coefficients of w^0, w^2, w^4)."""
    f = fp12(F)
    xf = {k: fp2(XF + 2 * (k - 1)) for k in range(1, 6)}
    recs = []
    for jj, k in enumerate((0, 2, 4)):
        re, im = [], []
        for i in range(6):
            for m in range(i, 6):
                if (i + m) % 6 != k:
                    continue
                wrap = i + m >= 6
                y = xf[m] if wrap else f[m]
                s = -1 if m % 2 else 1
                if i == m:
                    rr, mm = (sqr_terms(f[i], sign=s) if not wrap else mul_terms(f[i], y, sign=s))
                else:
                    rr, mm = mul_terms(f[i], y, sign=s, coef=2)
                re += rr
                im += mm
        d = fp2(N + 2 * jj)
        recs.append(Rec(dst=d[0], terms=re))
        recs.append(Rec(dst=d[1], terms=im))
    return pack(name, recs)


def fp2_out(recs, dst, re, im, exp=None, cm=1):
    recs.append(Rec(dst=dst[0] if dst else None, exp=None if exp is None else exp, cm=cm, terms=re))
    recs.append(Rec(dst=dst[1] if dst else None, exp=None if exp is None else exp + 1, cm=cm, terms=im))


def op_fp6_inv_t(name, N, XN2, Tt):
    """t0 = n0^2 - n1 (xi n2), t1 = n2 (xi n2) - n0 n1, t2 = n1^2 - n0 n2  ->  Tt (6 slots)"""
    n0, n1, n2 = fp2(N), fp2(N + 2), fp2(N + 4)
    xn2 = fp2(XN2)
    recs = []
    a, b = sqr_terms(n0)
    c, d = mul_terms(n1, xn2, sign=-1)
    fp2_out(recs, fp2(Tt), a + c, b + d)
    a, b = mul_terms(n2, xn2)
    c, d = mul_terms(n0, n1, sign=-1)
    fp2_out(recs, fp2(Tt + 2), a + c, b + d)
    a, b = sqr_terms(n1)
    c, d = mul_terms(n0, n2, sign=-1)
    fp2_out(recs, fp2(Tt + 4), a + c, b + d)
    return pack(name, recs)


def op_fp6_inv_d(name, N, Tt, XT, D):
    """d = n0 t0 + n2 (xi t1) + n1 (xi t2)"""
    n0, n1, n2 = fp2(N), fp2(N + 2), fp2(N + 4)
    t0 = fp2(Tt)
    xt1, xt2 = fp2(XT), fp2(XT + 2)
    recs = []
    a, b = mul_terms(n0, t0)
    c, d = mul_terms(n2, xt1)
    e, f = mul_terms(n1, xt2)
    fp2_out(recs, fp2(D), a + c + e, b + d + f)
    return pack(name, recs)


def op_n1(name, D, N1, exp=None):
    d = fp2(D)
    return pack(name, [Rec(dst=N1, exp=exp, terms=[T(d[0], d[0]), T(d[1], d[1])])])


def op_ninv(name, D, N1I, Tt, DI, NI):
    """dinv = conj(d) * n1inv, then Ninv_j = t_j * dinv (two ops)"""
    d = fp2(D)
    op1 = pack(name + "_d", [Rec(dst=DI, terms=[T(d[0], N1I)]), Rec(dst=DI + 1, terms=[T(d[1], N1I, -1)])])
    recs = []
    for j in range(3):
        a, b = mul_terms(fp2(Tt + 2 * j), fp2(DI))
        fp2_out(recs, fp2(NI + 2 * j), a, b)
    return op1, pack(name, recs)


def op_frob(name, A, power, out=None):
    """out <- A^(p^power), power in (1, 2)."""
    a = fp12(A)
    o = fp12(out if out is not None else A)
    recs = []
    for k in range(6):
        x = a[k]
        if k == 0:
            if power == 1:
                recs.append(Rec(dst=o[0][0], post=[(x[0], 1)]))
                recs.append(Rec(dst=o[0][1], post=[(x[1], -1)]))
            else:
                recs.append(Rec(dst=o[0][0], post=[(x[0], 1)]))
                recs.append(Rec(dst=o[0][1], post=[(x[1], 1)]))
            continue
        if power == 1:
            g = fp2(C_G1 + 2 * (k - 1))
            # conj(x) * g: re = x0 g0 + x1 g1, im = x0 g1 - x1 g0
            recs.append(Rec(dst=o[k][0], terms=[T(x[0], g[0]), T(x[1], g[1])]))
            recs.append(Rec(dst=o[k][1], terms=[T(x[0], g[1]), T(x[1], g[0], -1)]))
        else:
            g = C_G2 + (k - 1)
            recs.append(Rec(dst=o[k][0], terms=[T(x[0], g)]))
            recs.append(Rec(dst=o[k][1], terms=[T(x[1], g)]))
    return pack(name, recs)


def op_copy(name, A, B, conj=False):
    recs = []
    for k in range(6):
        s = -1 if (conj and k % 2) else 1
        for c in range(2):
            recs.append(Rec(dst=B + 2 * k + c, post=[(A + 2 * k + c, s)]))
    return pack(name, recs)


def op_conj(name, R):
    recs = []
    for k in (1, 3, 5):
        for c in range(2):
            recs.append(Rec(dst=R + 2 * k + c, post=[(R + 2 * k + c, -1)]))
    return pack(name, recs)


def op_cyclo_sqr(name, R, TMP):
    """Granger-Scott squaring in the cyclotomic subgroup, in place.
    Fp4 pairs A = (f0, f3), B = (f1, f4), C = (f2, f5):
      f0' = 3(f0^2 + xi f3^2) - 2 f0     f3' = 6 f0 f3 + 2 f3
      f1' = 6 xi f2 f5 + 2 f1            f4' = 3(f2^2 + xi f5^2) - 2 f4
      f2' = 3(f1^2 + xi f4^2) - 2 f2     f5' = 6 f1 f4 + 2 f5
    Two sub-ops: a LIN pass writes a+b, a-b, c+d, c-d for each pair
    (x0 = a + bu, x1 = c + du) to TMP, so that every output needs at most 3
    products:  (x0^2 + xi x1^2).re = (a+b)(a-b) + (c+d)(c-d) - 2cd,
               (x0^2 + xi x1^2).im = 2ab + (c+d)(c-d) + 2cd,
               (2 x0 x1).re = 2ac - 2bd,  (2 x0 x1).im = 2ad + 2bc."""
    f = fp12(R)
    pairs = {0: (0, 3), 1: (1, 4), 2: (2, 5)}   # Fp4 pair j = (f_j, f_{j+3})
    lin = []
    tmp = {}
    for j, (i0, i1) in pairs.items():
        a, b = f[i0]
        c_, d = f[i1]
        base = TMP + 4 * j
        tmp[j] = (base, base + 1, base + 2, base + 3)  # a+b, a-b, c+d, c-d
        lin.append(Rec(dst=base, post=[(a, 1), (b, 1)]))
        lin.append(Rec(dst=base + 1, post=[(a, 1), (b, -1)]))
        lin.append(Rec(dst=base + 2, post=[(c_, 1), (d, 1)]))
        lin.append(Rec(dst=base + 3, post=[(c_, 1), (d, -1)]))

    def s_terms(j, xi_outer=False):
        (i0, i1) = pairs[j]
        a, b = f[i0]
        c_, d = f[i1]
        apb, amb, cpd, cmd = tmp[j]
        re = [T(apb, amb), T(cpd, cmd), T(c_, d, -1, 2)]
        im = [T(a, b, 1, 2), T(cpd, cmd), T(c_, d, 1, 2)]
        return re, im

    def t_terms(j):
        (i0, i1) = pairs[j]
        a, b = f[i0]
        c_, d = f[i1]
        re = [T(a, c_, 1, 2), T(b, d, -1, 2)]
        im = [T(a, d, 1, 2), T(b, c_, 1, 2)]
        return re, im

    recs = []
    # f0' = 3 S(A) - 2 f0 ; f3' = 3 T(A) + 2 f3
    for k, (re, im), cm, dd in ((0, s_terms(0), 3, -2), (3, t_terms(0), 3, 2),
                                (4, s_terms(2), 3, -2), (2, s_terms(1), 3, -2), (5, t_terms(1), 3, 2)):
        recs.append(Rec(dst=f[k][0], cm=cm, terms=re, post=[(f[k][0], dd)]))
        recs.append(Rec(dst=f[k][1], cm=cm, terms=im, post=[(f[k][1], dd)]))
    # f1' = 3 xi T(C) + 2 f1: xi (r + s u) = (r - s) + (r + s) u with T(C) = 2 x0 x1
    # (x0 = f2 = a + bu, x1 = f5 = c + du): r - s = 2a(c - d) - 2b(c + d),
    # r + s = 2a(c + d) + 2b(c - d) -- two terms each over the LIN pass's c +- d,
    # so no lane of this sub-op needs more than three products
    (i0, i1) = pairs[2]
    a, b = f[i0]
    _, _, cpd, cmd = tmp[2]
    recs.append(Rec(dst=f[1][0], cm=3, terms=[T(a, cmd, 1, 2), T(b, cpd, -1, 2)], post=[(f[1][0], 2)]))
    recs.append(Rec(dst=f[1][1], cm=3, terms=[T(a, cpd, 1, 2), T(b, cmd, 1, 2)], post=[(f[1][1], 2)]))
    return Op(name, [lin, recs])


# ---------------------------------------------------------------- k_lines: T steps for two pairs
# per pair p (slot base 24 p): X 0,1  Y 2,3  Z 4,5  xQ 6,7  yQ 8,9  temporaries 10..23;
# pair 0's G1 point (-x, y) per item at 48, 49 (the group key, or a share's key
# PubPoly.Eval(i) in threshold recovery); pair 1's (-g1) is a block constant.
LINE_PAIR_SLOTS = 24
L_NXP0, L_YP0 = 48, 49
L_YS = 16      # per pair: YS, YD, ZS, ZD = Y.re +- Y.im, Z.re +- Z.im (live from a step's last sub-op to the next S2)


def _pb(p, off):
    return LINE_PAIR_SLOTS * p + off


def lines_dbl_op():
    """Doubling step on T = (X, Y, Z) (homogeneous projective, T scaled by 4
    relative to oracle/pairing_formulas.dbl_step: a subfield factor), with
    line l = (Y^2 - 3b'Z^2) + (-3X^2 xP) w^2 + (2YZ yP) w^3:
      t0 = Y^2, t1 = Z^2, w = 12 xi t1 (= 3b' Z^2), u = t0 - 3w, v = t0 + 3w
      X4 = 2 XY u,  Y4 = v^2 - 12 w^2,  Z4 = 8 t0 YZ
      l0 = t0 - w,  l2 = 3 X^2 (-xP),  l3 = 2 YZ yP
    Y4 = (v0 + v1)(v0 - v1) - (w0 + w1)(12w0 - 12w1) + (2 v0 v1 - 2 w0 12w1) u
    over sums that S3's and S4's fused epilogues form (round 2 ran a LIN
    sub-op, S4b, for them), so no lane of S5 needs more than two products
    (the sub-op costs its busiest lane); likewise S2's squares take one
    product each over the sums of Y and Z that S5's epilogue (or LADD's, or
    LINIT) leaves in YS, YD, ZS, ZD.  Five sub-ops."""
    S1, S2, S3, S4, S5 = [], [], [], [], []
    for p in range(2):
        X, Y, Z = fp2(_pb(p, 0)), fp2(_pb(p, 2)), fp2(_pb(p, 4))
        X2, XY, YZ = fp2(_pb(p, 10)), fp2(_pb(p, 12)), fp2(_pb(p, 14))
        W, U, V = fp2(_pb(p, 16)), fp2(_pb(p, 18)), fp2(_pb(p, 20))
        nxp, yp = (L_NXP0, L_YP0) if p == 0 else (C_NXP1, C_YP1)
        # S1: X2 = X^2, XY = X Y, YZ = Y Z
        fp2_out(S1, X2, *sqr_terms(X))
        fp2_out(S1, XY, *mul_terms(X, Y))
        fp2_out(S1, YZ, *mul_terms(Y, Z))
        # S2: t0 = Y^2 -> X slot, t1 = Z^2 -> Y slot; l2 = 3 X2 (-xP) (export).
        # The squares' real parts are one product (a+b)(a-b) of the sums the
        # previous step's last sub-op (or LINIT) left in YS, YD, ZS, ZD
        YS, YD, ZS, ZD = _pb(p, L_YS), _pb(p, L_YS + 1), _pb(p, L_YS + 2), _pb(p, L_YS + 3)
        fp2_out(S2, X, [T(YS, YD)], [T(Y[0], Y[1], 1, 2)])
        fp2_out(S2, Y, [T(ZS, ZD)], [T(Z[0], Z[1], 1, 2)])
        S2.append(Rec(exp=6 * p + 2, cm=3, terms=[T(X2[0], nxp)]))
        S2.append(Rec(exp=6 * p + 3, cm=3, terms=[T(X2[1], nxp)]))
        t0, t1 = X, Y
        # S3 (LIN): w = 12 xi t1, u = t0 - 36 xi t1, v = t0 + 36 xi t1
        S3.append(Rec(dst=W[0], post=[(t1[0], 12), (t1[1], -12)]))
        S3.append(Rec(dst=W[1], post=[(t1[0], 12), (t1[1], 12)]))
        S3.append(Rec(dst=U[0], post=[(t0[0], 1), (t1[0], -36), (t1[1], 36)]))
        S3.append(Rec(dst=U[1], post=[(t0[1], 1), (t1[0], -36), (t1[1], -36)]))
        S3.append(Rec(dst=V[0], post=[(t0[0], 1), (t1[0], 36), (t1[1], -36)]))
        S3.append(Rec(dst=V[1], post=[(t0[1], 1), (t1[0], 36), (t1[1], 36)]))
        # S4: l0 = t0 - w (export), w12 = 12 w -> Y slot (t1 dead), l3 = 2 YZ yP (export)
        S4.append(Rec(exp=6 * p + 0, post=[(t0[0], 1), (W[0], -1)]))
        S4.append(Rec(exp=6 * p + 1, post=[(t0[1], 1), (W[1], -1)]))
        S4.append(Rec(dst=Y[0], post=[(W[0], 12)]))
        S4.append(Rec(dst=Y[1], post=[(W[1], 12)]))
        S4.append(Rec(exp=6 * p + 4, cm=2, terms=[T(YZ[0], yp)]))
        S4.append(Rec(exp=6 * p + 5, cm=2, terms=[T(YZ[1], yp)]))
        W12 = Y
        # the sums vp = v0 + v1, vm = v0 - v1 (X2's slots, dead after S2) and
        # wp = w0 + w1 (22) come from S3's fused epilogue, w12m = 12 w0 - 12 w1
        # (23) from S4's (unreduced: w12m is S5's a operand, wp the negated b)
        VP, VM, WP, W12M = _pb(p, 10), _pb(p, 11), _pb(p, 22), _pb(p, 23)
        # S5: X4 = 2 XY u -> X, Y4 = v^2 - w w12 -> Y, Z4 = 8 t0 YZ -> Z
        fp2_out(S5, X, *mul_terms(XY, U, coef=2))
        fp2_out(S5, Y, [T(VP, VM), T(W12M, WP, -1)], [T(V[0], V[1], 1, 2), T(W[0], W12[1], -1, 2)])
        fp2_out(S5, Z, *mul_terms(t0, YZ), cm=8)
    # S3 lanes 6p + (0..5) = W, U, V (re, im); S4 lanes 6p + (2, 3) = w12
    f3, f4 = [None] * LANES, [None] * LANES
    for p in range(2):
        f3[6 * p + 0] = (_pb(p, 22), FUSE_SUM)      # wp
        f3[6 * p + 4] = (_pb(p, 10), FUSE_SUM)      # vp
        f3[6 * p + 5] = (_pb(p, 11), FUSE_DIFF)     # vm
        f4[6 * p + 3] = (_pb(p, 23), FUSE_DIFF)     # w12m
    return Op("LDBL", [S1, S2, S3, S4, S5], fuse={2: f3, 3: f4, 4: _yz_fuse()})


def lines_add_op():
    """Mixed addition T + Q (Q affine at xQ, yQ):
      theta = Y - yQ Z, lam = X - xQ Z, C = theta^2, D = lam^2, E = lam D,
      F = Z C, G = X D, H = E + F - 2G,
      X' = lam H, Y' = theta (G - H) - Y E, Z' = Z E,
      l0 = theta xQ - lam yQ, l2 = theta (-xP), l3 = lam yP"""
    S1, S2, S3, S4, S5, S6 = [], [], [], [], [], []
    for p in range(2):
        X, Y, Z = fp2(_pb(p, 0)), fp2(_pb(p, 2)), fp2(_pb(p, 4))
        xQ, yQ = fp2(_pb(p, 6)), fp2(_pb(p, 8))
        TH, LA, C, D = fp2(_pb(p, 10)), fp2(_pb(p, 12)), fp2(_pb(p, 14)), fp2(_pb(p, 16))
        E, F, G = fp2(_pb(p, 18)), fp2(_pb(p, 20)), fp2(_pb(p, 22))
        H, GH = C, D
        nxp, yp = (L_NXP0, L_YP0) if p == 0 else (C_NXP1, C_YP1)
        # S1: theta = Y - yQ Z, lam = X - xQ Z
        a, b = mul_terms(yQ, Z)
        S1.append(Rec(dst=TH[0], cm=-1, terms=a, post=[(Y[0], 1)]))
        S1.append(Rec(dst=TH[1], cm=-1, terms=b, post=[(Y[1], 1)]))
        a, b = mul_terms(xQ, Z)
        S1.append(Rec(dst=LA[0], cm=-1, terms=a, post=[(X[0], 1)]))
        S1.append(Rec(dst=LA[1], cm=-1, terms=b, post=[(X[1], 1)]))
        # S2: C = theta^2, D = lam^2, l2 = theta (-xP)
        fp2_out(S2, C, *sqr_terms(TH))
        fp2_out(S2, D, *sqr_terms(LA))
        S2.append(Rec(exp=6 * p + 2, terms=[T(TH[0], nxp)]))
        S2.append(Rec(exp=6 * p + 3, terms=[T(TH[1], nxp)]))
        # S3: l0 = theta xQ - lam yQ, l3 = lam yP
        a, b = mul_terms(TH, xQ)
        c, d = mul_terms(LA, yQ, sign=-1)
        S3.append(Rec(exp=6 * p + 0, terms=a + c))
        S3.append(Rec(exp=6 * p + 1, terms=b + d))
        S3.append(Rec(exp=6 * p + 4, terms=[T(LA[0], yp)]))
        S3.append(Rec(exp=6 * p + 5, terms=[T(LA[1], yp)]))
        # S4: E = lam D, F = Z C, G = X D
        fp2_out(S4, E, *mul_terms(LA, D))
        fp2_out(S4, F, *mul_terms(Z, C))
        fp2_out(S4, G, *mul_terms(X, D))
        # S5 (LIN): H = E + F - 2G -> C slot, GH = G - H = 3G - E - F -> D slot
        for c_ in range(2):
            S5.append(Rec(dst=H[c_], post=[(E[c_], 1), (F[c_], 1), (G[c_], -2)]))
        for c_ in range(2):
            S5.append(Rec(dst=GH[c_], post=[(G[c_], 3), (E[c_], -1), (F[c_], -1)]))
        # S6: X' = lam H, Y' = theta GH - Y E, Z' = Z E
        fp2_out(S6, X, *mul_terms(LA, H))
        a, b = mul_terms(TH, GH)
        c, d = mul_terms(Y, E, sign=-1)
        fp2_out(S6, Y, a + c, b + d)
        fp2_out(S6, Z, *mul_terms(Z, E))
    return Op("LADD", [S1, S2, S3, S4, S5, S6], fuse={5: _yz_fuse()})


def _yz_fuse():
    """The fused epilogue of the sub-op that writes (X, Y, Z) of both pairs
    (lanes 6p + 0..5 = X, Y, Z re/im): Y and Z's a+-b sums for the next
    doubling's S2."""
    lanes = [None] * LANES
    for p in range(2):
        for c, base in ((1, L_YS), (2, L_YS + 2)):   # Y, Z
            lanes[6 * p + 2 * c] = (_pb(p, base), FUSE_SUM)
            lanes[6 * p + 2 * c + 1] = (_pb(p, base + 1), FUSE_DIFF)
    return lanes


def lines_init_op():
    """LINIT: the sums YS, YD, ZS, ZD of the initial T = (xQ, yQ, 1) for both
    pairs (afterwards each step's last sub-op forms them, _yz_fuse)."""
    recs = []
    for p in range(2):
        Y, Z = fp2(_pb(p, 2)), fp2(_pb(p, 4))
        for src, base in ((Y, L_YS), (Z, L_YS + 2)):
            recs.append(Rec(dst=_pb(p, base), post=[(src[0], 1), (src[1], 1)]))
            recs.append(Rec(dst=_pb(p, base + 1), post=[(src[0], 1), (src[1], -1)]))
    return pack("LINIT", recs)


# After the loop T of pair 1 is [|x|] sigma (the ladder of |x| = 0xd201000000010000,
# mixed additions of the affine sigma; doubling / addition steps only scale T
# projectively).  sigma is in G2 iff psi(sigma) == [x] sigma = -T (Scott's
# test, as curve.cuh g2_in_subgroup), so the Miller loop's own ladder replaces
# the decoder's 63-doubling subgroup check.  An exceptional step (a 2-torsion
# doubling, T = +-sigma in an addition) implies sigma has order dividing a
# number below 2^64 + 1, so sigma is not in G2 -- and those steps zero Z,
# which stays zero, so the test (Z != 0) rejects them too.
L_SUB_XP, L_SUB_YP, L_SUB_D1, L_SUB_D2 = 34, 36, 38, 40   # pair 1's temporaries, free after the loop
L_SUB_Z = LINE_PAIR_SLOTS + 4


def lines_subgroup_op():
    """D1 = X - x_psi Z, D2 = Y + y_psi Z for pair 1, with x_psi = conj(xQ) cx,
    y_psi = conj(yQ) cy: sigma in G2 iff D1 = D2 = 0 and Z != 0."""
    X, Y, Z = fp2(_pb(1, 0)), fp2(_pb(1, 2)), fp2(_pb(1, 4))
    xQ, yQ = fp2(_pb(1, 6)), fp2(_pb(1, 8))
    XP, YP, D1, D2 = fp2(L_SUB_XP), fp2(L_SUB_YP), fp2(L_SUB_D1), fp2(L_SUB_D2)
    S1 = []
    for src, c, dst in ((xQ, fp2(C_PSI), XP), (yQ, fp2(C_PSI + 2), YP)):
        # conj(s) c: re = s0 c0 + s1 c1, im = s0 c1 - s1 c0
        S1.append(Rec(dst=dst[0], terms=[T(src[0], c[0]), T(src[1], c[1])]))
        S1.append(Rec(dst=dst[1], terms=[T(src[0], c[1]), T(src[1], c[0], -1)]))
    S2 = []
    a, b = mul_terms(XP, Z)
    S2.append(Rec(dst=D1[0], cm=-1, terms=a, post=[(X[0], 1)]))
    S2.append(Rec(dst=D1[1], cm=-1, terms=b, post=[(X[1], 1)]))
    a, b = mul_terms(YP, Z)
    S2.append(Rec(dst=D2[0], terms=a, post=[(Y[0], 1)]))
    S2.append(Rec(dst=D2[1], terms=b, post=[(Y[1], 1)]))
    return Op("LSUB", [S1, S2])


# ---------------------------------------------------------------- k_miller slots
M_F, M_X, M_L1, M_L2 = 0, 12, 22, 28      # F (12), xi-copies (10), line 1 (6), line 2 (6)
M_XF0 = 34                                # xi-copy of F's w^0 coefficient (the squaring's f0^2)
M_N, M_XN2, M_T, M_XT, M_D, M_N1 = 22, 12, 14, 28, 20, 12  # norm epilogue (after the loop)

# ---------------------------------------------------------------- k_fe slots
E_F, E_X, E_N, E_XN2, E_T, E_XT, E_D, E_N1I, E_DI = 0, 12, 22, 28, 30, 36, 40, 42, 43
E_NI, E_XNI = 22, 28          # Ninv (6, over N), xi Ninv1, xi Ninv2 (4, over XN2 and t0)
E_R, E_A, E_XA, E_CT = 0, 12, 24, 34   # hard part: R (12), A (12), xi A (10), cyclotomic-squaring temps (12)


def build_ops():
    ops = []
    # k_lines
    ops.append(lines_dbl_op())
    ops.append(lines_add_op())
    ops.append(lines_subgroup_op())
    ops.append(lines_init_op())
    # k_miller
    ops.append(pack("M_XIF", op_xi_copy("_a", M_F, M_X, [1, 2, 3, 4, 5]).subs[0] +
                    op_xi_copy("_b", M_F, M_XF0, [0]).subs[0]))
    # Fused epilogues leave xi f = (re - im, re + im) of coefficients for the
    # next op (the re lane's re + im is the copy's im half, the im lane's
    # re - im its re half): M_LM2 -> all six, for the next step's M_SQR (the
    # loop's M_XIF pass of round 2 is gone); M_SQR and M_LM1 -> f3, f4, f5,
    # the factors of the line products' wrapped terms (xi f_k) l_j, so no
    # per-line xi-copy pass (M_XIL, to r03aa) either.
    def xi_lanes(ks):
        lanes = [None] * LANES
        for k in ks:
            xr = M_XF0 if k == 0 else M_X + 2 * (k - 1)
            lanes[2 * k] = (xr + 1, FUSE_SUM)
            lanes[2 * k + 1] = (xr, FUSE_DIFF)
        return lanes
    xf_wrap = {k: M_X + 2 * (k - 1) for k in (3, 4, 5)}
    ops.append(Op("M_SQR", op_sqr12("M_SQR", M_F, M_X, XF0=M_XF0).subs, fuse={0: xi_lanes((3, 4, 5))}))
    ops.append(Op("M_LM1", op_line_mul("M_LM1", M_F, M_L1, XF=xf_wrap).subs, fuse={0: xi_lanes((3, 4, 5))}))
    ops.append(Op("M_LM2", op_line_mul("M_LM2", M_F, M_L2, XF=xf_wrap).subs, fuse={0: xi_lanes(range(6))}))
    ops.append(op_norm6("M_NRM", M_F, M_X, M_N))
    ops.append(op_xi_copy("M_XIN2", M_N, M_XN2, [2]))
    ops.append(op_fp6_inv_t("M_T012", M_N, M_XN2, M_T))
    ops.append(op_xi_copy("M_XIT", M_T, M_XT, [1, 2]))
    ops.append(op_fp6_inv_d("M_D", M_N, M_T, M_XT, M_D))
    ops.append(op_n1("M_N1", M_D, M_N1, exp=EXP_N1))
    # k_fe: easy part
    ops.append(op_xi_copy("E_XIF", E_F, E_X, [1, 2, 3, 4, 5]))
    ops.append(op_norm6("E_NRM", E_F, E_X, E_N))
    ops.append(op_xi_copy("E_XIN2", E_N, E_XN2, [2]))
    ops.append(op_fp6_inv_t("E_T012", E_N, E_XN2, E_T))
    ops.append(op_xi_copy("E_XIT", E_T, E_XT, [1, 2]))
    ops.append(op_fp6_inv_d("E_D", E_N, E_T, E_XT, E_D))
    o1, o2 = op_ninv("E_NINV", E_D, E_N1I, E_T, E_DI, E_NI)
    ops.append(o1)
    ops.append(o2)
    ops.append(op_xi_copy("E_XINI", E_NI, E_XNI, [1, 2]))
    ops.append(op_sqr12("E_SQRC", E_F, E_X, conj=True))          # F <- conj(f)^2
    ops.append(op_mul_fp6("E_MULN", E_F, E_NI, E_XNI))           # F <- F * Ninv  (= f^(p^6-1))
    # (F = R from here on: E_R == E_F == 0)
    ops.append(op_frob("E_FROB2A", E_R, 2, out=E_A))             # A <- frob2(R)
    ops.append(op_xi_copy("E_XIA", E_A, E_XA, [1, 2, 3, 4, 5]))
    ops.append(op_mul12("E_MUL", E_R, E_A, E_XA))                # R <- R * A
    ops.append(op_mul12("E_MULCJ", E_R, E_A, E_XA, conj_a=True)) # R <- R * conj(A)
    ops.append(op_copy("E_COPYRA", E_R, E_A))                    # A <- R
    ops.append(op_conj("E_CONJ", E_R))                           # R <- conj(R)
    ops.append(op_cyclo_sqr("E_CYC", E_R, E_CT))                 # R <- R^2 (cyclotomic)
    ops.append(op_cyclo_sqr("E_CYCA", E_A, E_CT))                # A <- A^2 (cyclotomic)
    ops.append(op_frob("E_FROB1", E_A, 1))                       # A <- frob1(A)
    ops.append(op_frob("E_FROB2", E_A, 2))                       # A <- frob2(A)
    return ops


# ---------------------------------------------------------------- kernel programs
# Each engine kernel executes one linear program (a single interpreter loop on
# the device, so the interpreter is inlined once).  Instructions:
#   ("run", op)           run op; its exports go to lines[step][e] (e < 12) or n1 (e == 12)
#   ("step",)             step += 1 (line index of exports and ldline)
#   ("ldline", slot)      lane k: slot + k <- lines[step][k]; step += 1
#   ("ld12", slot, comp)  lane k: slot + k <- fbuf[comp + k]
#   ("st12", slot, comp)  lane k: fbuf[comp + k] <- slot + k
OPC = {"run": 0, "step": 1, "ldline": 2, "ld12": 3, "st12": 4}
BITS = [(0xD201000000010000 >> i) & 1 for i in range(62, -1, -1)]


def prog_lines():
    prog = [("run", "LINIT")]
    for b in BITS:
        prog += [("run", "LDBL"), ("step",)]
        if b:
            prog += [("run", "LADD"), ("step",)]
    return prog + [("run", "LSUB")]


def prog_miller():
    # M_XIF once: xi-copies of f = 1 for the first step's line products
    prog = [("run", "M_XIF")]
    line = [("ldline", M_L1), ("run", "M_LM1"), ("run", "M_LM2")]
    for j, b in enumerate(BITS):
        if j:   # M_SQR's xi-copies of f: the previous M_LM2's fused epilogue
            prog += [("run", "M_SQR")]
        prog += line
        if b:
            prog += line
    prog += [("run", n) for n in ("M_XIF", "M_NRM", "M_XIN2", "M_T012", "M_XIT", "M_D", "M_N1")]
    return prog


def prog_fe():
    """Final exponentiation; on entry F = f (slots 0..11), slot E_N1I = 1/N1.
    On exit R = FE(f).  fbuf components 0..11 hold t, 12..23 t2."""
    run = lambda *names: [("run", n) for n in names]  # noqa: E731
    prog = run("E_XIF", "E_NRM", "E_XIN2", "E_T012", "E_XIT", "E_D", "E_NINV_d", "E_NINV", "E_XINI",
               "E_SQRC", "E_MULN", "E_FROB2A", "E_XIA", "E_MUL")
    prog += [("st12", E_R, 0)]

    def exp_x():  # A <- R, R <- conj(R^|x|)
        p = run("E_COPYRA", "E_XIA")
        for b in BITS:
            p += run("E_CYC")
            if b:
                p += run("E_MUL")
        return p + run("E_CONJ")

    prog += exp_x() + run("E_MULCJ")                      # t0 = t^x conj(t)
    prog += exp_x() + run("E_MULCJ")                      # t1 = t0^x conj(t0)
    prog += exp_x() + run("E_FROB1", "E_XIA", "E_MUL")    # t2 = t1^x t1^p
    prog += [("st12", E_R, 12)]
    prog += exp_x() + exp_x()
    prog += [("ld12", E_A, 12)] + run("E_FROB2", "E_XIA", "E_MUL")
    prog += [("ld12", E_A, 12)] + run("E_XIA", "E_MULCJ")  # t3 = t2^(x^2) t2^(p^2) conj(t2)
    prog += [("ld12", E_A, 0)] + run("E_XIA", "E_MUL", "E_CYCA", "E_XIA", "E_MUL")  # t3 t^3
    return prog


def encode_prog(prog, op_index):
    out = []
    for ins in prog:
        opc = OPC[ins[0]]
        a = op_index[ins[1]] if ins[0] == "run" else (ins[1] if len(ins) > 1 else 0)
        b = ins[2] if len(ins) > 2 else 0
        out.append((opc << 24) | (b << 8) | a)
    return out


class ProgramRunner:
    """Executes a kernel program on a Model (one group) with simulated HBM."""

    def __init__(self, model):
        self.m = model
        self.step = 0
        self.lines = {}   # (step, e) -> value
        self.fbuf = {}
        self.n1 = None

    def run(self, prog):
        m = self.m
        for ins in prog:
            kind = ins[0]
            if kind == "run":
                m.exports = {}
                m.run(ins[1])
                for e, v in m.exports.items():
                    if e < 12:
                        self.lines[(self.step, e)] = v
                    else:
                        self.n1 = v
            elif kind == "step":
                self.step += 1
            elif kind == "ldline":
                for k in range(LANES):
                    m.s[ins[1] + k] = self.lines[(self.step, k)]
                self.step += 1
            elif kind == "ld12":
                for k in range(LANES):
                    m.s[ins[1] + k] = self.fbuf[ins[2] + k]
            elif kind == "st12":
                for k in range(LANES):
                    self.fbuf[ins[2] + k] = m.s[ins[1] + k]


# ---------------------------------------------------------------- table emission
# ---------------------------------------------------------------- column normalization schedule
# engine.cuh accumulates each lane's products in 27 64-bit columns and carries
# them (normalizes) only where this schedule says: a greedy pass over the
# sub-op's terms (in encoded order) with exact per-column bounds of every lane,
# normalizing before a term whenever some lane's column could reach 2^64, and
# after the last term when the reduction's headroom (2^64 - 2^60: it adds up to
# 14 (2^28)^2 and a carry) would be exceeded.
def _p_limbs():
    from fractions import Fraction  # noqa: F401  (exact integers only)
    p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
    return p


_P = _p_limbs()
_SUBK = [(8 * _P >> (28 * i)) & 0xFFFFFFF for i in range(14)]


def _subk_limbs():
    # FP_SUBK (constants.h): 8p with every non-top limb raised by 2^28 (borrowed from the next)
    v = 8 * _P
    limbs = [(v >> (28 * i)) & 0xFFFFFFF for i in range(14)]
    limbs[13] = v >> (28 * 13)
    out = []
    for i in range(14):
        x = limbs[i] + ((1 << 28) if i < 13 else 0) - (1 if i > 0 else 0)
        out.append(x)
    return out


def _slot_limb_max(bound_p=2.01):
    top = int(bound_p * _P) >> (28 * 13)
    return [(1 << 28) - 1] * 13 + [top]


def norm_schedule(sub, wide=None):
    """Bit t set: normalize after term t (encoded term order).  wide: {slot:
    bound in p} of operands above the slot bound (fused_reads)."""
    amax0 = _slot_limb_max()
    wide = wide or {}
    amax_of = lambda s: _slot_limb_max(wide[s]) if s in wide else amax0  # noqa: E731
    subk = _subk_limbs()
    LIM, LIM_REDC = (1 << 64) - 1, (1 << 64) - (1 << 60)
    lanes = [sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2)) for r in sub]
    nt = max([len(t) for t in lanes] + [0])
    after_norm = [(1 << 28) - 1] * 27 + [1 << 40]
    cur = [[0] * 28 for _ in lanes]
    mask = 0
    for t in range(nt):
        grow = []
        for terms in lanes:
            g = [0] * 28
            if t < len(terms):
                a, b, sg, cf = terms[t]
                amax, bm = amax_of(a), amax_of(b)
                bmax = [(subk[j] if sg < 0 else bm[j]) << (cf - 1) for j in range(14)]
                for i in range(14):
                    for j in range(14):
                        g[i + j] += amax[i] * bmax[j]
            grow.append(g)
        if t and any(c[k] + g[k] > LIM for c, g in zip(cur, grow) for k in range(28)):
            mask |= 1 << (t - 1)
            cur = [list(after_norm) for _ in lanes]
        cur = [[c[k] + g[k] for k in range(28)] for c, g in zip(cur, grow)]
        assert all(max(c) <= LIM for c in cur)
    if nt and any(max(c) > LIM_REDC for c in cur):
        mask |= 1 << (nt - 1)
    return mask


def slot_ref(s):
    """An operand in a term or post word: its word offset (bits 0..9) from the
    group's slots, or (bit 10 set) from the block constant region."""
    return (s * SLOT_WORDS) if s < 64 else (((s - 64) * SLOT_WORDS) | 0x400)


def fuse_tables(ops):
    """Per fused sub-op (in op order): 12 lane words dst | FUSE_* << 16
    (0xFFFF: no epilogue on that lane).  Returns (tables, {(op, sub): 1-based index})."""
    tabs, idx = [], {}
    for op in ops:
        for si in sorted(op.fuse):
            lanes = op.fuse[si] + [None] * (LANES - len(op.fuse[si]))
            tabs.append([0xFFFF if f is None else f[0] | f[1] << 16 for f in lanes])
            idx[(op.name, si)] = len(tabs)
    return tabs, idx


def encode(ops):
    words = []
    op_tab = []
    sub_tab = []
    _, fidx = fuse_tables(ops)
    assert len(fidx) < 256
    for op in ops:
        op_tab.append((len(sub_tab), len(op.subs)))
        for si, sub in enumerate(op.subs):
            nt = max([len(r.terms) for r in sub] + [0])
            assert nt <= MAX_TERMS, (op.name, nt)
            ntp = (nt + 3) & ~3   # records are 16-byte aligned: header + terms padded to 4 words
            uses_c = any(x >= 64 for r in sub for t in r.terms for x in t[:2]) or any(x >= 64 for r in sub for x, _ in r.post)
            fz = fidx.get((op.name, si), 0)
            ns = norm_schedule(sub, fused_reads(op).get(si))
            sub_tab.append((len(words), nt | ns << 8 | uses_c << 20 | fz << 21))
            for k in range(LANES):
                r = sub[k] if k < len(sub) else None
                if r is None:
                    words += [0xFFFF, 0, 0, 0] + [0] * ntp
                    continue
                assert len(r.post) <= 3 and -16 < r.cm < 16
                dst = 0xFF if r.dst is None else r.dst
                exp = 0xFF if r.exp is None else r.exp
                h0 = dst | (exp << 8) | ((r.cm & 0xFF) << 16) | (len(r.post) << 24)
                posts = [(slot_ref(s) | ((d & 0xFFFF) << 16)) for s, d in r.post] + [0] * (3 - len(r.post))
                words += [h0] + posts
                # plain products first: for the leading term positions no lane
                # of a sub-op negates or doubles its operand (engine.cuh skips
                # that transform wave-uniformly)
                terms = sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2))
                for t in range(nt):
                    if t < len(terms):
                        a, b, sg, cf = terms[t]
                        assert cf in (1, 2) and sg in (1, -1)
                        words.append(slot_ref(a) | (slot_ref(b) << 11) | ((sg < 0) << 22) | ((cf == 2) << 23) | (1 << 31))
                    else:
                        words.append(0)
                words += [0] * (ntp - nt)
    assert len(words) % 4 == 0
    return op_tab, sub_tab, words


def cyc_fast_params(ops, name="E_CYC"):
    """Per-lane parameters of the straight-line cyclotomic squaring
    (engine.cuh eng_cyc_fast): the op's two sub-ops, decoded once here.
    Sub-op 0 (LIN): out = x + y or x - y; sub-op 1: out = cm * redc(sum of <= 3
    products) + d * post, with cm = ENG_CYC_CM and |d| = ENG_CYC_ABSD the same
    for every lane.  Offsets are group-relative word offsets (slot * 14).
    Word layout per lane (8 words):
      0: lin dst | lin x << 16      1: lin y | (lin y negated) << 16
      2..4: term t operands a | b << 16 (unused terms: 0, 0)
      5: post | dst << 16
      6: flags: bit 2t = term t negated, bit 2t+1 = term t doubled,
         bits 8..9 = term count, bits 16..23 = cm (int8), 24..31 = d (int8)
      7: fused LIN destination: the next E_CYC's sub-op 0 output that this
         lane forms from its own output and its partner lane's (k ^ 1: the
         other half of the same Fp2 coefficient): re + im on the re lane,
         re - im on the im lane.
    The LIN outputs are left unreduced (normalized limbs, value < 10.02p):
    their only readers are this op's product terms, bounded below."""
    op = {o.name: o for o in ops}[name]
    assert len(op.subs) == 2
    lin, prod = op.subs
    assert len(lin) == LANES and len(prod) == LANES
    return _cyc_rows(lin, prod, lin, prod, {})


def _cyc_rows(lin, prod, lin_all, prod_all, remap):
    """Rows of eng_cyc_fast for the lanes `prod` (lane k computes prod[k] and
    the LIN record lin[k]); slots are renumbered by `remap` (identity where
    absent); lin_all / prod_all: the op's full sub-ops (partner and fused-LIN
    lookups)."""
    slot = SLOT_WORDS
    rows = []
    nl = len(prod)
    assert len(lin) == nl
    assert len({r.cm for r in prod}) == 1 and len({abs(r.post[0][1]) for r in prod}) == 1
    for k in range(nl):
        lr, pr = lin[k], prod[k]
        assert not lr.terms and len(lr.post) == 2 and lr.post[0][1] == 1 and abs(lr.post[1][1]) == 1
        assert lr.dst is not None and lr.exp is None and pr.dst is not None and pr.exp is None
        assert 2 <= len(pr.terms) <= 3 and len(pr.post) == 1 and -128 <= pr.cm < 128
        (x, _), (y, dy) = lr.post
        sl = lambda s: remap.get(s, s)  # noqa: E731
        terms = sorted(pr.terms, key=lambda t: (t[2] < 0) + (t[3] == 2))
        w = [sl(lr.dst) * slot | (sl(x) * slot) << 16, sl(y) * slot | (1 if dy < 0 else 0) << 16]
        flags = 0
        for t in range(3):
            if t < len(terms):
                a, b, sg, cf = terms[t]
                assert a < 64 and b < 64
                w.append(sl(a) * slot | (sl(b) * slot) << 16)
                flags |= (sg < 0) << (2 * t) | (cf == 2) << (2 * t + 1)
            else:
                w.append(0)
        (ps, d), = pr.post
        assert ps < 64 and -128 <= d < 128
        assert ps == pr.dst   # the post operand is the lane's own slot (engine.cuh eng_cyc_chain keeps it in registers)
        w.append(sl(ps) * slot | (sl(pr.dst) * slot) << 16)
        flags |= len(terms) << 8 | (pr.cm & 0xFF) << 16 | (d & 0xFF) << 24
        # fused LIN: this lane holds coefficient half pr.dst; partner k ^ 1 the other half
        assert prod[k ^ 1].dst == pr.dst ^ 1
        re, im = pr.dst & ~1, pr.dst | 1
        want = [(re, 1), (im, 1 if pr.dst == re else -1)]
        fused = [r.dst for r in lin_all if r.post == want]
        assert len(fused) == 1, (k, want)
        w += [flags, sl(fused[0]) * slot]
        rows.append(w)
    # bounds: LIN outputs x + y < 4.02p, x - y + 8p < 10.02p (normalized, unreduced);
    # every product sum < 2048 p^2 (redc output < 1.06p), <= 4 terms (no column normalization)
    tmp = {}
    for r in lin_all:
        tmp[r.dst] = 4.02 if r.post[1][1] > 0 else 10.02
    for r in prod:
        tot = 0.0
        for a, b, sg, cf in r.terms:
            ba, bb = tmp.get(a, 2.01), tmp.get(b, 2.01)
            assert not (sg < 0 and bb >= 7.99)   # 8p - b needs b < 7.99p
            tot += cf * ba * (8.0 if sg < 0 else bb)
        assert tot < 2048 and len(r.terms) <= 4, (r.dst, tot)
    return rows


# ---------------------------------------------------------------- Karabina final exponentiation
# The hard part's five exponentiations by |x| (315 of the FE's cyclotomic
# squarings) run on COMPRESSED elements (Karabina 2010): of the Granger-Scott
# formulas (op_cyclo_sqr) the outputs f1, f2, f4, f5 depend only on f1, f2,
# f4, f5 -- eight Fp instead of twelve.  The compressed chain runs in its own
# kernel with 8 lanes per item (8 items per wave64, no idle lane; the 12-lane
# groups run 5 items on 60 lanes), squaring m itself 63 times and storing
# m^(2^s) for the six set bits s of |x|; decompression
#   f3 = (xi f5^2 + 3 f2^2 - 2 f4) / (4 f1),  f0 = xi (2 f3^2 + f1 f5 - 3 f4 f2) + 1
# needs one inversion per stored value, batched over the chunk (Montgomery's
# trick, k_eng_kb_inv); the 12-lane program segments multiply the six values
# (m^|x|) and run the glue between exponentiations.  An item with f1 = 0 at a
# stored value (probability ~2^-762, or m = 1) is flagged and re-run through
# the Granger-Scott program (prog_fe).
KB_SNAP = (16, 48, 57, 60, 62, 63)     # m^(2^s) stored after s squarings: sum of 2^s = |x|
KB_COMP = (2, 3, 4, 5, 8, 9, 10, 11)   # compressed coordinates (f1, f2, f4, f5) as w-basis components (re, im)
KB_SLOTS = 16                          # chain kernel slots per item: 8 state + 8 LIN sums (pairs B, C)
PL_T, PL_T2, PL_M, PL_X0 = 0, 1, 2, 3  # planes of the Karabina FE state: t, t2, exponentiation input, stored values
KB_PLANES = PL_X0 + len(KB_SNAP)
assert sum(1 << s for s in KB_SNAP) == 0xD201000000010000


def cyc8_params(ops, name="E_CYC"):
    """eng_cyc_fast rows of the 8-lane compressed squaring: E_CYC's records
    for the outputs f1, f2, f4, f5 (lane k computes component KB_COMP[k]) and
    the LIN sums of the Fp4 pairs B = (f1, f4), C = (f2, f5), renumbered into
    the chain kernel's 16 slots (state k at slot k, sums at 8..15).  Lane k's
    LIN record is the one it forms in the fused epilogue."""
    op = {o.name: o for o in ops}[name]
    lin, prod = op.subs
    remap = {E_R + c: i for i, c in enumerate(KB_COMP)}
    remap.update({E_CT + 4 + t: 8 + t for t in range(8)})
    by_dst = {r.dst: r for r in prod}
    prod8 = [by_dst[E_R + c] for c in KB_COMP]
    lin8 = []
    for r in prod8:
        re, im = r.dst & ~1, r.dst | 1
        want = [(re, 1), (im, 1 if r.dst == re else -1)]
        lr = [x for x in lin if x.post == want]
        assert len(lr) == 1
        lin8.append(lr[0])
    # closed: the eight outputs read only the eight state slots and the pairs B, C sums
    for r in prod8 + lin8:
        refs = [r.dst] + [t[0] for t in r.terms] + [t[1] for t in r.terms] + [s for s, _ in r.post]
        assert all(s in remap for s in refs), r.dst
    rows = _cyc_rows(lin8, prod8, lin, prod, remap)
    xf = 0
    for r in prod8:
        for t, (_, _, sg, cf) in enumerate(sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2))):
            xf |= (sg < 0) << t | (cf == 2) << (16 + t)
    return rows, xf


def prog_fe_kb():
    """The Karabina FE as seven 12-lane program segments (k_eng_fe_seg):
    segment 0 is prog_fe's easy part and stores t = m (planes T and M);
    segment e = 1..5 follows exponentiation e's compressed chain: the product
    of its six decompressed values (planes X0..X5) is m^|x|, conjugated m^x,
    then the glue of prog_fe up to the next exponentiation's input (plane M).
    Segment 5 ends with R = FE(f)."""
    run = lambda *names: [("run", n) for n in names]  # noqa: E731
    seg0 = run("E_XIF", "E_NRM", "E_XIN2", "E_T012", "E_XIT", "E_D", "E_NINV_d", "E_NINV", "E_XINI",
               "E_SQRC", "E_MULN", "E_FROB2A", "E_XIA", "E_MUL")
    seg0 += [("st12", E_R, 12 * PL_T), ("st12", E_R, 12 * PL_M)]
    segs = [seg0]
    for e in range(1, 6):
        p = [("ld12", E_R, 12 * PL_X0)]
        for j in range(1, len(KB_SNAP)):
            p += [("ld12", E_A, 12 * (PL_X0 + j))] + run("E_XIA", "E_MUL")
        p += run("E_CONJ")                                          # R = m^x
        if e in (1, 2):                                             # t0 = t^x conj(t), t1 = t0^x conj(t0)
            p += [("ld12", E_A, 12 * PL_M)] + run("E_XIA", "E_MULCJ") + [("st12", E_R, 12 * PL_M)]
        elif e == 3:                                                # t2 = t1^x t1^p
            p += [("ld12", E_A, 12 * PL_M)] + run("E_FROB1", "E_XIA", "E_MUL")
            p += [("st12", E_R, 12 * PL_M), ("st12", E_R, 12 * PL_T2)]
        elif e == 4:                                                # t2^x
            p += [("st12", E_R, 12 * PL_M)]
        else:                                                       # t3 = t2^(x^2) t2^(p^2) conj(t2), times t^3
            p += [("ld12", E_A, 12 * PL_T2)] + run("E_FROB2", "E_XIA", "E_MUL")
            p += [("ld12", E_A, 12 * PL_T2)] + run("E_XIA", "E_MULCJ")
            p += [("ld12", E_A, 12 * PL_T)] + run("E_XIA", "E_MUL", "E_CYCA", "E_XIA", "E_MUL")
        segs.append(p)
    return segs


class KbChainModel:
    """The 8-lane compressed squaring (engine.cuh eng_cyc_fast over
    ENG_CYC8_PAR) over Python ints mod p: the rows' semantics, TEST
    INFRASTRUCTURE (tests/test_engine_model.py)."""

    def __init__(self, rows, p):
        self.rows, self.p = rows, p
        self.s = [0] * KB_SLOTS

    def _get(self, w):
        return self.s[w // SLOT_WORDS]

    def square(self, lin):
        p, rows = self.p, self.rows
        if lin:
            outs = []
            for w in rows:
                x, y = self._get(w[0] >> 16), self._get(w[1] & 0xFFFF)
                outs.append((w[0] & 0xFFFF, (x - y) if (w[1] >> 16) else (x + y)))
            for d, v in outs:
                self.s[d // SLOT_WORDS] = v % p
        outs = []
        for w in rows:
            fl = w[6]
            acc = 0
            for t in range((fl >> 8) & 3):
                a, b = self._get(w[2 + t] & 0xFFFF), self._get(w[2 + t] >> 16)
                sg = -1 if (fl >> (2 * t)) & 1 else 1
                cf = 2 if (fl >> (2 * t + 1)) & 1 else 1
                acc += sg * cf * a * b
            cm = ((fl >> 16) & 0xFF) - (256 if (fl >> 23) & 1 else 0)
            d = ((fl >> 24) & 0xFF) - (256 if (fl >> 31) & 1 else 0)
            outs.append((w[5] >> 16, (cm * acc + d * self._get(w[5] & 0xFFFF)) % p))
        for dd, v in outs:
            self.s[dd // SLOT_WORDS] = v
        # fused LIN epilogue: lane k forms own + partner (re lane) / partner - own... (im lane)
        for k, w in enumerate(rows):
            own, par = outs[k][1], outs[k ^ 1][1]
            self.s[w[7] // SLOT_WORDS] = ((par - own) if (k & 1) else (own + par)) % p


def kb_decompress(v, p):
    """(f1, f2, f4, f5) (8 ints, KB_COMP order) -> the 12 w-basis components;
    None when f1 = 0 (the flagged case)."""
    f1, f2, f4, f5 = (v[0], v[1]), (v[2], v[3]), (v[4], v[5]), (v[6], v[7])
    mul = lambda a, b: ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)  # noqa: E731
    xi = lambda a: ((a[0] - a[1]) % p, (a[0] + a[1]) % p)  # noqa: E731
    lin = lambda *ts: (sum(c * a[0] for c, a in ts) % p, sum(c * a[1] for c, a in ts) % p)  # noqa: E731
    d = lin((4, f1))
    nd = (d[0] * d[0] + d[1] * d[1]) % p
    if nd == 0:
        return None
    ninv = pow(nd, p - 2, p)
    dinv = (d[0] * ninv % p, (-d[1]) * ninv % p)
    n = lin((1, xi(mul(f5, f5))), (3, mul(f2, f2)), (-2, f4))
    f3 = mul(n, dinv)
    f0 = lin((1, xi(lin((2, mul(f3, f3)), (1, mul(f1, f5)), (-3, mul(f4, f2))))), (1, (1, 0)))
    return [f0, f1, f2, f3, f4, f5]


# ---------------------------------------------------------------- compiled ops (engine_compiled.h)
# Hot ops run as straight-line code (engine.cuh eng_sub_c): the generator
# fixes each sub-op's shape at compile time.  Families: the kernel whose
# eng_exec includes the op (0 lines, 1 miller, 2 fe).
# (M_LM1 / M_LM2 compile without spills since eng_sub_c fences each term's
# products; without the fence k_eng_miller spilled 179 VGPRs)
COMPILED = {"LDBL": 0, "LADD": 0, "M_XIF": 1, "M_SQR": 1, "M_LM1": 1, "M_LM2": 1,
            "E_MUL": 2, "E_MULCJ": 2, "E_XIA": 2}


def sub_shape(sub):
    lanes = [sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2)) for r in sub] + [[]] * (LANES - len(sub))
    nt = max(len(t) for t in lanes)
    ntmin = min(len(t) for t in lanes)
    xf = 0   # bit t: some lane negates term t's b operand; bit 16 + t: some lane doubles it
    for t in range(nt):
        if any(t < len(ts) and ts[t][2] < 0 for ts in lanes):
            xf |= 1 << t
        if any(t < len(ts) and ts[t][3] == 2 for ts in lanes):
            xf |= 1 << (16 + t)
    np_ = max(len(r.post) for r in sub)
    plain = all(r.cm == 1 and not r.post for r in sub) and len(sub) == LANES
    kind = "ENG_K_PLAIN" if plain else ("ENG_K_LIN" if nt == 0 else "ENG_K_MIXED")
    lin32 = all(abs(r.cm) * (1 << (29 if r.cm < 0 else 28)) + sum(abs(d) * (1 << (29 if d < 0 else 28)) for _, d in r.post)
                <= (1 << 31) for r in sub)
    consts = any(x >= 64 for r in sub for t in r.terms for x in t[:2]) or any(x >= 64 for r in sub for x, _ in r.post)
    has_dst = any(r.dst is not None for r in sub)
    has_exp = any(r.exp is not None for r in sub)
    return nt, ntmin, xf, np_, kind, lin32, consts, has_dst, has_exp


def sub_in_place(op, si):
    """Sub-op si writes a slot (output or fused-epilogue sum) that some lane
    of the same sub-op reads.  Within one wave all lanes read before any
    writes; when a group spans waves (XW kernels, engine.cuh eng_sync) such a
    sub-op needs a barrier between its reads and its writes."""
    sub = op.subs[si]
    reads = set()
    for r in sub:
        for a, b, _, _ in r.terms:
            reads |= {a, b}
        for sl, _ in r.post:
            reads.add(sl)
    writes = {r.dst for r in sub if r.dst is not None}
    writes |= {f[0] for f in op.fuse.get(si, []) if f is not None}
    return bool(reads & writes)


def emit_compiled(ops, sub_tab, path):
    idx = {op.name: i for i, op in enumerate(ops)}
    out = ["// GENERATED by tools/gen_engine.py -- do not edit.",
           "// Straight-line forms of the hot engine ops (engine.cuh eng_sub_c): each",
           "// sub-op's shape fixed at compile time, the records and sums the interpreter's.",
           "// XW: the group's lanes span waves (engine.cuh eng_sync: a barrier between an",
           "// in-place sub-op's reads and its writes, and after every sub-op's writes).",
           "// Included by engine.cuh inside namespace dgpu.",
           "#pragma once", ""]
    s_index = 0
    first_sub = {}
    for op in ops:
        first_sub[op.name] = s_index
        s_index += len(op.subs)
    for name, fam in COMPILED.items():
        op = ops[idx[name]]
        out.append("template <bool XW, class Sink>")
        out.append(f"__device__ __forceinline__ void eng_op_c_{name}(uint32_t* g, const uint32_t* c, int k, Sink&& sink) {{")
        for si, sub in enumerate(op.subs):
            nt, ntmin, xf, np_, kind, lin32, consts, has_dst, has_exp = sub_shape(sub)
            off, ntw = sub_tab[first_sub[name] + si]
            recw = 4 + ((nt + 3) & ~3)
            out.append("  {")
            out.append(f"    const uint32_t* rec = ENG_WORDS + {off}u + (uint32_t)k * {recw}u;")
            out.append(f"    const fp o = eng_sub_c<{nt}, {ntmin}, 0x{xf:x}u, {np_}, {kind}, {str(lin32).lower()}, "
                       f"{str(consts).lower()}>(g, c, rec);")
            out.append("    const uint32_t h0 = rec[0];")
            out.append(f"    eng_sync<XW && {str(sub_in_place(op, si)).lower()}>();")
            if has_dst:
                out.append("    if ((h0 & 0xFFu) != 0xFFu) eng_st(g + (h0 & 0xFFu) * ENG_SLOT_WORDS, o);")
            if has_exp:
                out.append("    if (((h0 >> 8) & 0xFFu) != 0xFFu) sink((h0 >> 8) & 0xFFu, o);")
            fz = (ntw >> 21) & 0xFF
            if fz:
                out.append(f"    eng_fuse_epilogue(g, o, ENG_FUSE_TAB[{fz - 1}][k], k);")
            out.append("    eng_sync<XW>();")
            out.append("  }")
        out.append("}")
        out.append("")
    for fam in range(3):
        out.append("template <bool XW, class Sink>")
        out.append(f"__device__ __forceinline__ bool eng_run_c{fam}(int op, uint32_t* g, const uint32_t* c, int k, Sink&& sink) {{")
        out.append("  switch (op) {")
        for name, f in COMPILED.items():
            if f == fam:
                out.append(f"    case OP_{name}: eng_op_c_{name}<XW>(g, c, k, sink); return true;")
        out.append("    default: return false;")
        out.append("  }")
        out.append("}")
        out.append("")
    # host emulation: one sub-op for one lane
    out.append("// host emulation (tests/hostsim): sub-op si of compiled op `op` for the lane")
    out.append("// whose record is `rec`; false if the op is not compiled")
    out.append("DG_FN bool eng_sub_c_host(int op, int si, const uint32_t* g, const uint32_t* c, const uint32_t* rec, fp& o) {")
    out.append("  switch (op * 16 + si) {")
    for name in COMPILED:
        op = ops[idx[name]]
        for si, sub in enumerate(op.subs):
            nt, ntmin, xf, np_, kind, lin32, consts, _, _ = sub_shape(sub)
            out.append(f"    case OP_{name} * 16 + {si}: o = eng_sub_c<{nt}, {ntmin}, 0x{xf:x}u, {np_}, {kind}, "
                       f"{str(lin32).lower()}, {str(consts).lower()}>(g, c, rec); return true;")
    out.append("    default: return false;")
    out.append("  }")
    out.append("}")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def fused_reads(op):
    """{sub index: {slot: bound in p}}: the sub-ops that read a fused
    epilogue's unreduced sums (LDBL's S2 reads the a+-b sums of Y and Z)."""
    wide = {}
    if op.name == "LDBL":
        wide[1] = {}
        for p in range(2):
            for j in range(4):
                wide[1][_pb(p, L_YS + j)] = FUSE_BOUND[FUSE_SUM if j % 2 == 0 else FUSE_DIFF]
        wide[4] = {}
        for p in range(2):
            for off, mode in ((10, FUSE_SUM), (11, FUSE_DIFF), (22, FUSE_SUM), (23, FUSE_DIFF)):
                wide[4][_pb(p, off)] = FUSE_BOUND[mode]
    if op.name in ("M_SQR", "M_LM1", "M_LM2"):   # xi-copies (re - im, re + im) of f from fused epilogues
        wide[0] = {}
        for k in (range(6) if op.name == "M_SQR" else (3, 4, 5)):
            xr = M_XF0 if k == 0 else M_X + 2 * (k - 1)
            wide[0][xr] = FUSE_BOUND[FUSE_DIFF]
            wide[0][xr + 1] = FUSE_BOUND[FUSE_SUM]
    return wide


def check_bounds(ops):
    """Static bounds the device arithmetic relies on (see engine.cuh):
    slot values < 2.01p (fused-epilogue sums: fused_reads); product sum
    < 2048 p^2 so redc < 1.8p; the post linear combination stays < 2^392."""
    for op in ops:
        wide = fused_reads(op)
        for si, sub in enumerate(op.subs):
            bnd = lambda s: wide.get(si, {}).get(s, 2.01)  # noqa: E731
            for r in sub:
                # negated operands are 8p - b (FP_SUBK), < 8p: b < 7.99p
                assert all(not (sg < 0 and bnd(b) >= 7.99) for _, b, sg, _ in r.terms), op.name
                prod = sum(cf * bnd(a) * (8.0 if sg < 0 else bnd(b)) for a, b, sg, cf in r.terms)
                assert prod < 2048, (op.name, prod)
                # redc output < 1.8p; negative multipliers act on 8p - x
                lin = abs(r.cm) * (8.0 if r.cm < 0 else 1.8) + sum(abs(d) * (8.0 if d < 0 else 2.01) for _, d in r.post)
                assert lin < 2500, (op.name, lin)
                for a, b, _, _ in r.terms:
                    assert a < 64 + N_CONST and b < 64 + N_CONST
                for s, _ in r.post:
                    assert s < 64 + N_CONST


# Group bases in LDS (slots from the start of the block's LDS; the constant
# region takes slots 0 .. N_CONST-1): consecutive groups, no padding.  The
# bank model (tools/lds_banks.py search_bases) predicted 10-45% fewer
# operand-load LDS cycles for padded bases (lines 24 + 51 g, Miller
# [24, 65, 113, 161, 202], FE [24, 71, 117, 164, 210] with the hard part's
# blocks reordered), but those measured slower (profiles/r02/r02s_group_bases_ab.json:
# lines +3%, Miller +2%), so the layout stays packed.
GROUP_BASES = {k: [N_CONST + g * n for g in range(5)] for k, n in (("LINES", 50), ("MILLER", 36), ("FE", 46))}


def emit(path):
    ops = build_ops()
    check_bounds(ops)
    op_tab, sub_tab, words = encode(ops)
    nslots = {}
    for op in ops:
        m = 0
        for sub in op.subs:
            for r in sub:
                for s in [r.dst] + [t[0] for t in r.terms] + [t[1] for t in r.terms] + [p[0] for p in r.post]:
                    if s is not None and s < 64:
                        m = max(m, s + 1)
        nslots[op.name] = m
    lines = [
        "// GENERATED by tools/gen_engine.py -- do not edit.",
        "// Micro-op tables of the lane-cooperative pairing engine (engine.cuh).",
        "#pragma once",
        "#include <cstdint>",
        "",
        "namespace dgpu {",
        "",
        f"constexpr int ENG_LANES = {LANES};",
        f"constexpr int ENG_MAX_TERMS = {MAX_TERMS};",
        f"constexpr int ENG_NCONST = {N_CONST};",
        f"constexpr int ENG_C_ONE = {C_ONE}, ENG_C_NXP0 = {C_NXP0}, ENG_C_YP0 = {C_YP0}, ENG_C_NXP1 = {C_NXP1}, ENG_C_YP1 = {C_YP1};",
        f"constexpr int ENG_C_G1 = {C_G1}, ENG_C_G2 = {C_G2}, ENG_C_PSI = {C_PSI};",
        f"constexpr int ENG_L_SUB_D1 = {L_SUB_D1}, ENG_L_SUB_D2 = {L_SUB_D2}, ENG_L_SUB_Z = {L_SUB_Z};",
        f"constexpr int ENG_LINE_PAIR_SLOTS = {LINE_PAIR_SLOTS}, ENG_L_NXP0 = {L_NXP0}, ENG_L_YP0 = {L_YP0};",
        f"constexpr int ENG_M_F = {M_F}, ENG_M_L1 = {M_L1}, ENG_M_L2 = {M_L2}, ENG_EXP_N1 = {EXP_N1};",
        f"constexpr int ENG_E_F = {E_F}, ENG_E_N1I = {E_N1I}, ENG_E_R = {E_R}, ENG_E_A = {E_A};",
        "",
        "enum EngOp : int {",
    ]
    for i, op in enumerate(ops):
        lines.append(f"  OP_{op.name} = {i},  // {len(op.subs)} sub-op(s), slots < {nslots[op.name]}")
    lines.append("};")
    nsl = {
        "LINES": max(nslots["LDBL"], nslots["LADD"], nslots["LSUB"]),
        "MILLER": max(v for k, v in nslots.items() if k.startswith("M_")),
        "FE": max(v for k, v in nslots.items() if k.startswith("E_")),
    }
    for k, v in nsl.items():
        b = GROUP_BASES[k]
        assert b[0] >= N_CONST and all(b[g + 1] - b[g] >= v for g in range(4)), (k, v, b)
        lines.append(f"constexpr int ENG_SLOTS_{k} = {v};")
        # group g's slots start at LDS slot ENG_GBASE_k[g]; the block's LDS is ENG_LDS_SLOTS_k slots
        lines.append(f"constexpr int ENG_GBASE_{k}[5] = {{{', '.join(map(str, b))}}};")
        lines.append(f"constexpr int ENG_LDS_SLOTS_{k} = {b[4] + v};")
    lines.append("")
    lines.append("#ifndef ENG_TABLE_QUAL")
    lines.append("#define ENG_TABLE_QUAL static const")
    lines.append("#endif")
    lines.append(f"ENG_TABLE_QUAL uint32_t ENG_OP_TAB[{len(op_tab)}][2] = {{")
    lines.append("  " + ", ".join(f"{{{a}, {b}}}" for a, b in op_tab))
    lines.append("};")
    lines.append(f"ENG_TABLE_QUAL uint32_t ENG_SUB_TAB[{len(sub_tab)}][2] = {{")
    lines.append("  " + ", ".join(f"{{{a}, {b}}}" for a, b in sub_tab))
    lines.append("};")
    lines.append(f"alignas(16) ENG_TABLE_QUAL uint32_t ENG_WORDS[{len(words)}] = {{")
    for i in range(0, len(words), 12):
        lines.append("  " + ", ".join(f"0x{w:08x}u" for w in words[i:i + 12]) + ",")
    lines.append("};")
    rows = cyc_fast_params(ops)
    cyc = {o.name: o for o in ops}["E_CYC"].subs[1]
    lines.append("// eng_cyc_fast: per-lane parameters of E_CYC (tools/gen_engine.py cyc_fast_params)")
    lines.append(f"constexpr int ENG_CYC_CM = {cyc[0].cm}, ENG_CYC_ABSD = {abs(cyc[0].post[0][1])};")
    xf = 0   # product term t: bit t some lane negates, bit 16 + t some lane doubles (eng_cyc_term)
    for r in cyc:
        for t, (_, _, sg, cf) in enumerate(sorted(r.terms, key=lambda x: (x[2] < 0) + (x[3] == 2))):
            xf |= (sg < 0) << t | (cf == 2) << (16 + t)
    lines.append(f"constexpr uint32_t ENG_CYC_XF = 0x{xf:x}u;")
    ftabs, _ = fuse_tables(ops)
    lines.append("// fused epilogues (tools/gen_engine.py fuse_tables): per fused sub-op, lane word dst | mode << 16")
    lines.append(f"constexpr int ENG_NFUSE = {len(ftabs)};")
    lines.append(f"ENG_TABLE_QUAL uint32_t ENG_FUSE_TAB[{max(1, len(ftabs))}][{LANES}] = {{")
    for t in ftabs:
        lines.append("  {" + ", ".join(f"0x{x:08x}u" for x in t) + "},")
    lines.append("};")
    lines.append(f"alignas(16) ENG_TABLE_QUAL uint32_t ENG_CYC_PAR[{LANES}][8] = {{")
    for w in rows:
        lines.append("  {" + ", ".join(f"0x{x:08x}u" for x in w) + "},")
    lines.append("};")
    rows8, xf8 = cyc8_params(ops)
    lines.append("// Karabina FE (tools/gen_engine.py cyc8_params, prog_fe_kb): the 8-lane compressed squaring")
    lines.append(f"constexpr int ENG_KB_SLOTS = {KB_SLOTS}, ENG_KB_NSNAP = {len(KB_SNAP)}, ENG_KB_PLANES = {KB_PLANES};")
    lines.append(f"constexpr int ENG_KB_PL_T = {PL_T}, ENG_KB_PL_T2 = {PL_T2}, ENG_KB_PL_M = {PL_M}, ENG_KB_PL_X0 = {PL_X0};")
    lines.append(f"constexpr int ENG_KB_SNAP[{len(KB_SNAP)}] = {{{', '.join(map(str, KB_SNAP))}}};")
    lines.append(f"constexpr int ENG_KB_COMP[8] = {{{', '.join(map(str, KB_COMP))}}};")
    lines.append(f"constexpr uint32_t ENG_CYC8_XF = 0x{xf8:x}u;")
    lines.append(f"alignas(16) ENG_TABLE_QUAL uint32_t ENG_CYC8_PAR[8][8] = {{")
    for w in rows8:
        lines.append("  {" + ", ".join(f"0x{x:08x}u" for x in w) + "},")
    lines.append("};")
    op_index = {op.name: i for i, op in enumerate(ops)}
    segs = [encode_prog(s, op_index) for s in prog_fe_kb()]
    offs = [0]
    for s in segs:
        offs.append(offs[-1] + len(s))
    lines.append(f"constexpr int ENG_PROG_FEK_OFF[{len(offs)}] = {{{', '.join(map(str, offs))}}};")
    # group slots each segment touches (ops' records and fused-epilogue sums,
    # LD12 / ST12 planes): the segments between the chains need fewer than the
    # FE's maximum, so their XW kernel fits more blocks per CU
    def op_slots(op):
        m = nslots[op.name]
        for lanes in op.fuse.values():
            m = max([m] + [f[0] + 1 for f in lanes if f is not None])
        return m
    seg_slots = []
    for seg in prog_fe_kb():
        m = 0
        for ins in seg:
            m = max(m, op_slots(ops[op_index[ins[1]]]) if ins[0] == "run" else ins[1] + LANES)
        seg_slots.append(m)
    assert max(seg_slots) <= nsl["FE"], (seg_slots, nsl["FE"])
    lines.append(f"constexpr int ENG_FEK_MID_SLOTS = {max(seg_slots[1:-1])};  // segments 1 .. 4 (per segment: "
                 f"{', '.join(map(str, seg_slots))})")
    allk = [w for s in segs for w in s]
    lines.append(f"ENG_TABLE_QUAL uint32_t ENG_PROG_FEK[{len(allk)}] = {{")
    for i in range(0, len(allk), 12):
        lines.append("  " + ", ".join(f"0x{w:08x}u" for w in allk[i:i + 12]) + ",")
    lines.append("};")
    lines.append(f"constexpr uint32_t ENG_OPC_RUN = {OPC['run']}, ENG_OPC_STEP = {OPC['step']}, ENG_OPC_LDLINE = {OPC['ldline']}, "
                 f"ENG_OPC_LD12 = {OPC['ld12']}, ENG_OPC_ST12 = {OPC['st12']};")
    for pname, prog in (("LINES", prog_lines()), ("MILLER", prog_miller()), ("FE", prog_fe())):
        code = encode_prog(prog, op_index)
        lines.append(f"constexpr int ENG_PROG_{pname}_LEN = {len(code)};")
        lines.append(f"ENG_TABLE_QUAL uint32_t ENG_PROG_{pname}[{len(code)}] = {{")
        for i in range(0, len(code), 12):
            lines.append("  " + ", ".join(f"0x{w:08x}u" for w in code[i:i + 12]) + ",")
        lines.append("};")
    lines.append("")
    lines.append("}  // namespace dgpu")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    emit_compiled(ops, sub_tab, os.path.join(os.path.dirname(path), "engine_compiled.h"))
    return ops, nsl


# ---------------------------------------------------------------- executable model (mod p)
class Model:
    """Device semantics over Python ints mod p (slot values as plain field
    elements; the device keeps them in Montgomery form, which commutes with
    every operation here).  One instance models one group."""

    def __init__(self, ops, p, const):
        self.ops = {op.name: op for op in ops}
        self.p = p
        self.s = [0] * 64
        self.const = const            # dict slot -> value
        self.exports = {}

    def get(self, s):
        return self.s[s] if s < 64 else self.const[s]

    def run(self, name):
        p = self.p
        for sub in self.ops[name].subs:
            outs = []
            for r in sub:
                acc = 0
                for a, b, sg, cf in r.terms:
                    acc += cf * sg * self.get(a) * self.get(b)
                v = r.cm * acc + sum(d * self.get(s) for s, d in r.post)
                outs.append((r, v % p))
            for r, v in outs:
                if r.dst is not None:
                    self.s[r.dst] = v
                if r.exp is not None:
                    self.exports[r.exp] = v
            for k, f in enumerate(self.ops[name].fuse.get(self.ops[name].subs.index(sub), [])):
                if f is not None:
                    own, par = outs[k][1], outs[k ^ 1][1]
                    self.s[f[0]] = (own + par) % p if f[1] == FUSE_SUM else (par - own) % p


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "drand_amd", "csrc", "engine_tables.h")
    ops, nsl = emit(out)
    print("wrote", out, "ops:", len(ops), "slots:", nsl, file=sys.stderr)
