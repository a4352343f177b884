"""The pairing engine's micro-op programs (tools/gen_engine.py), executed by
the Python model with the device semantics, against the oracle's tower
arithmetic and pairing: every op on random operands, then the full
k_lines -> k_miller -> k_inv -> k_fe flow on valid and invalid signatures.
CPU only (the device interpreter itself is checked by tests/test_hostsim.py
and the GPU parity suite)."""
import os
import random
import sys

import pytest

from oracle import bls12381 as B
from oracle import drand_ref as D

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gen_engine as G  # noqa: E402

P = B.P
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _consts(pk=None):
    c = {G.C_ONE: 1}
    xi = (1, 1)
    for k in range(1, 6):
        g1 = B.f2_pow(xi, k * (P - 1) // 6)
        c[G.C_G1 + 2 * (k - 1)] = g1[0]
        c[G.C_G1 + 2 * (k - 1) + 1] = g1[1]
        g2 = B.f2_pow(xi, k * (P * P - 1) // 6)
        assert g2[1] == 0
        c[G.C_G2 + (k - 1)] = g2[0]
    c[G.C_PSI], c[G.C_PSI + 1] = B.PSI_CX
    c[G.C_PSI + 2], c[G.C_PSI + 3] = B.PSI_CY
    if pk is not None:
        ng1 = B.g1_neg(B.G1_GEN)
        c[G.C_NXP0], c[G.C_YP0] = (-pk[0]) % P, pk[1]
        c[G.C_NXP1], c[G.C_YP1] = (-ng1[0]) % P, ng1[1]
    return c


@pytest.fixture(scope="module")
def ops():
    return G.build_ops()


def _rand_f12(rng):
    return [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]


def _to_tower(w):
    return B.f12_from_fp2_basis(w)


def _from_tower(t):
    return [t[0][0], t[1][0], t[0][1], t[1][1], t[0][2], t[1][2]]


def _load(m, base, w):
    for k, (a, b) in enumerate(w):
        m.s[base + 2 * k] = a % P
        m.s[base + 2 * k + 1] = b % P


def _read(m, base):
    return [(m.s[base + 2 * k], m.s[base + 2 * k + 1]) for k in range(6)]


def test_tables_emit_and_bounds(ops, tmp_path):
    G.check_bounds(ops)
    out, nsl = G.emit(str(tmp_path / "t.h"))
    assert nsl["MILLER"] <= 36 and nsl["FE"] <= 48 and nsl["LINES"] <= 52
    # the committed header is what the generator produces
    with open(os.path.join(ROOT, "drand_amd", "csrc", "engine_tables.h")) as f:
        assert f.read() == open(tmp_path / "t.h").read()


def test_sqr_and_line_mul(ops):
    rng = random.Random(1)
    m = G.Model(ops, P, _consts())
    f = _rand_f12(rng)
    _load(m, G.M_F, f)
    m.run("M_XIF")
    m.run("M_SQR")
    assert _read(m, G.M_F) == _from_tower(B.f12_sqr(_to_tower(f)))
    # line mult
    l0, l2, l3 = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
    _load(m, G.M_F, f)
    for j, v in enumerate((l0, l2, l3)):
        m.s[G.M_L1 + 2 * j], m.s[G.M_L1 + 2 * j + 1] = v
        m.s[G.M_L2 + 2 * j], m.s[G.M_L2 + 2 * j + 1] = v
    m.run("M_XIF")   # xi-copies of f; M_LM1's epilogue leaves those of f l for M_LM2
    m.run("M_LM1")
    line = _to_tower([l0, (0, 0), l2, l3, (0, 0), (0, 0)])
    exp = B.f12_mul(_to_tower(f), line)
    assert _read(m, G.M_F) == _from_tower(exp)
    m.run("M_LM2")
    assert _read(m, G.M_F) == _from_tower(B.f12_mul(exp, line))


def test_mul_conj_frob_cyclo(ops):
    rng = random.Random(2)
    m = G.Model(ops, P, _consts())
    r, a = _rand_f12(rng), _rand_f12(rng)
    _load(m, G.E_R, r)
    _load(m, G.E_A, a)
    m.run("E_XIA")
    m.run("E_MUL")
    assert _read(m, G.E_R) == _from_tower(B.f12_mul(_to_tower(r), _to_tower(a)))
    _load(m, G.E_R, r)
    m.run("E_MULCJ")
    assert _read(m, G.E_R) == _from_tower(B.f12_mul(_to_tower(r), B.f12_conj(_to_tower(a))))
    _load(m, G.E_R, r)
    m.run("E_CONJ")
    assert _read(m, G.E_R) == _from_tower(B.f12_conj(_to_tower(r)))
    _load(m, G.E_A, a)
    m.run("E_FROB1")
    assert _read(m, G.E_A) == _from_tower(B.f12_pow(_to_tower(a), P))
    _load(m, G.E_A, a)
    m.run("E_FROB2")
    assert _read(m, G.E_A) == _from_tower(B.f12_pow(_to_tower(a), P * P))
    # cyclotomic element: g = a^((p^6-1)(p^2+1))
    ta = _to_tower(a)
    g = B.f12_mul(B.f12_conj(ta), B.f12_inv(ta))
    g = B.f12_mul(B.f12_pow(g, P * P), g)
    _load(m, G.E_R, _from_tower(g))
    m.run("E_CYC")
    assert _read(m, G.E_R) == _from_tower(B.f12_sqr(g))


def run_pairing_model(ops, pk, q1, q2):
    """The kernel flow of the per-round pairing check: the generated kernel
    programs (gen_engine.prog_*) on the model, with the setup and epilogue
    the kernels do (pairing_engine.cuh).  q1 = H(m), q2 = sig (affine G2),
    pairs (pk, q1), (-g1, q2).  Returns (FE(f) in w-basis, f, verdict)."""
    c = _consts(pk)
    # ---- k_eng_lines: lanes load Q into X, Y and (xQ, yQ); Z = 1
    m = G.Model(ops, P, c)
    for p, q in enumerate((q1, q2)):
        b = G.LINE_PAIR_SLOTS * p
        (x0, x1), (y0, y1) = q
        m.s[b + 0], m.s[b + 1], m.s[b + 2], m.s[b + 3], m.s[b + 4], m.s[b + 5] = x0, x1, y0, y1, 1, 0
        m.s[b + 6], m.s[b + 7], m.s[b + 8], m.s[b + 9] = x0, x1, y0, y1
    m.s[G.L_NXP0], m.s[G.L_YP0] = c[G.C_NXP0], c[G.C_YP0]
    lines = G.ProgramRunner(m)
    lines.run(G.prog_lines())
    assert lines.step == 68
    # ---- k_eng_miller: F = 1, program, then f and N1 out
    m = G.Model(ops, P, c)
    _load(m, G.M_F, [(1, 0)] + [(0, 0)] * 5)
    mil = G.ProgramRunner(m)
    mil.lines = lines.lines
    mil.run(G.prog_miller())
    f = _read(m, G.M_F)
    n1 = mil.n1
    # ---- k_eng_inv
    n1inv = pow(n1, P - 2, P)
    # ---- k_eng_fe
    m = G.Model(ops, P, c)
    _load(m, G.E_F, f)
    m.s[G.E_N1I] = n1inv
    fe = G.ProgramRunner(m)
    fe.run(G.prog_fe())
    res = _read(m, G.E_R)
    run_pairing_model.n1inv = n1inv
    return res, f, res == [(1, 0)] + [(0, 0)] * 5


@pytest.mark.parametrize("kind", ["valid", "wrong_msg"])
def test_full_pairing_flow(ops, kind):
    sk = D.derive_secret(7)
    pk = B.g1_mul(B.G1_GEN, sk)
    msg = b"\x01" * 32
    h = B.hash_to_g2(msg)
    sig = B.g2_mul(h, sk)
    if kind == "wrong_msg":
        h = B.hash_to_g2(b"\x02" * 32)
    res, f, ok = run_pairing_model(ops, pk, h, sig)
    assert ok == (kind == "valid")
    # exact GT value: FE(f_model) = FE(oracle product)^-1 (the model skips the conjugation)
    fo = B.f12_mul(B.miller_loop(pk, h), B.miller_loop(B.g1_neg(B.G1_GEN), sig))
    assert _to_tower(res) == B.f12_conj(B.final_exponentiation(fo))


def run_fe_kb_model(ops, c, f, n1inv):
    """The Karabina FE flow (gen_engine.prog_fe_kb, KbChainModel,
    kb_decompress): segment 0, then per exponentiation the 8-lane compressed
    chain from plane M storing m^(2^s) at KB_SNAP, their decompression, and
    the next segment.  Every segment starts from a fresh group (a new kernel);
    only the HBM planes carry state.  Returns R in w-basis, or None if an
    item would be flagged (f1 = 0 at a stored value)."""
    rows, _ = G.cyc8_params(ops)
    segs = G.prog_fe_kb()
    fbuf = {}

    def segment(prog, setup=None):
        m = G.Model(ops, P, c)
        if setup:
            setup(m)
        r = G.ProgramRunner(m)
        r.fbuf = fbuf
        r.run(prog)
        return m

    def setup0(m):
        _load(m, G.E_F, f)
        m.s[G.E_N1I] = n1inv

    m = segment(segs[0], setup0)
    for e in range(1, 6):
        ch = G.KbChainModel(rows, P)
        for i, comp in enumerate(G.KB_COMP):
            ch.s[i] = fbuf[12 * G.PL_M + comp]
        snaps = {}
        for s in range(1, 64):
            ch.square(lin=(s == 1))
            if s in G.KB_SNAP:
                snaps[s] = list(ch.s[:8])
        for j, s in enumerate(G.KB_SNAP):
            x = G.kb_decompress(snaps[s], P)
            if x is None:
                return None
            for k, (a, b) in enumerate(x):
                fbuf[12 * (G.PL_X0 + j) + 2 * k], fbuf[12 * (G.PL_X0 + j) + 2 * k + 1] = a, b
        m = segment(segs[e])
    return _read(m, G.E_R)


@pytest.mark.parametrize("kind", ["valid", "wrong_msg"])
def test_fe_karabina_flow(ops, kind):
    """The Karabina FE gives exactly the Granger-Scott program's FE(f), on a
    valid and an invalid pairing check; the chain's compressed coordinates
    equal the oracle's powers m^(2^s)."""
    sk = D.derive_secret(9)
    pk = B.g1_mul(B.G1_GEN, sk)
    msg = b"\x03" * 32
    h = B.hash_to_g2(msg)
    sig = B.g2_mul(h, sk)
    if kind == "wrong_msg":
        h = B.hash_to_g2(b"\x04" * 32)
    res, f, ok = run_pairing_model(ops, pk, h, sig)
    kb = run_fe_kb_model(ops, _consts(pk), f, run_pairing_model.n1inv)
    assert kb is not None
    assert kb == res
    assert (kb == [(1, 0)] + [(0, 0)] * 5) == (kind == "valid")


def test_karabina_chain_rows_and_decompression(ops):
    """KbChainModel over cyc8_params equals the oracle's squarings of a
    cyclotomic element on the compressed coordinates, and kb_decompress
    recovers the full element."""
    rng = random.Random(4)
    a = _to_tower(_rand_f12(rng))
    g = B.f12_mul(B.f12_conj(a), B.f12_inv(a))
    g = B.f12_mul(B.f12_pow(g, P * P), g)
    rows, _ = G.cyc8_params(ops)
    ch = G.KbChainModel(rows, P)
    w = _from_tower(g)
    flat = [c for pair in w for c in pair]
    for i, comp in enumerate(G.KB_COMP):
        ch.s[i] = flat[comp]
    cur = g
    for s in range(1, 20):
        ch.square(lin=(s == 1))
        cur = B.f12_sqr(cur)
        wf = [c for pair in _from_tower(cur) for c in pair]
        assert ch.s[:8] == [wf[comp] for comp in G.KB_COMP]
    assert G.kb_decompress(ch.s[:8], P) == _from_tower(cur)


@pytest.mark.parametrize("in_g2", [True, False])
def test_lines_fused_subgroup_op(ops, in_g2):
    """k_lines ends with LSUB: D1 = X - x_psi Z and D2 = Y + y_psi Z of pair 1
    vanish (with Z != 0) iff psi(sig) == [x] sig, i.e. sig in G2."""
    rng = random.Random(5 if in_g2 else 6)
    if in_g2:
        q = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
    else:
        q = B.iso_map_g2(B.map_to_curve_sswu_g2((rng.randrange(P), rng.randrange(P))))
        assert not B.g2_in_subgroup(q)
    pk = B.g1_mul(B.G1_GEN, 7)
    m = G.Model(ops, P, _consts(pk))
    for p in range(2):
        base = G.LINE_PAIR_SLOTS * p
        for off, v in ((0, q[0]), (2, q[1]), (6, q[0]), (8, q[1])):
            m.s[base + off], m.s[base + off + 1] = v[0] % P, v[1] % P
        m.s[base + 4], m.s[base + 5] = 1, 0
    m.s[G.L_NXP0], m.s[G.L_YP0] = (-pk[0]) % P, pk[1]
    G.ProgramRunner(m).run(G.prog_lines())
    d = [m.s[G.L_SUB_D1], m.s[G.L_SUB_D1 + 1], m.s[G.L_SUB_D2], m.s[G.L_SUB_D2 + 1]]
    z = (m.s[G.L_SUB_Z], m.s[G.L_SUB_Z + 1])
    assert z != (0, 0)
    assert (d == [0, 0, 0, 0]) == in_g2
