"""The kernels' arithmetic (drand_amd/csrc/*.cuh), compiled for the host by
the test-only tests/hostsim build, against the oracle (CPU)."""
import ctypes
import hashlib
import random

import pytest

from conftest import load_golden
from oracle import bls12381 as B
from oracle import drand_ref as D

P = B.P


def be(x):
    return (x % P).to_bytes(48, "big")


def ib(b):
    return int.from_bytes(b, "big")


def buf(n):
    return ctypes.create_string_buffer(n)


def test_fp_ops(hostsim):
    rnd = random.Random(1)
    vals = [(rnd.randrange(P), rnd.randrange(P)) for _ in range(30)] + [(0, 0), (P - 1, P - 1), (1, P - 1), (P - 1, 0)]
    for a, b in vals:
        mul, add, sub, sqr, inv = buf(48), buf(48), buf(48), buf(48), buf(48)
        hostsim.hs_fp_ops(be(a), be(b), mul, add, sub, sqr, inv)
        assert ib(mul.raw) == a * b % P
        assert ib(add.raw) == (a + b) % P
        assert ib(sub.raw) == (a - b) % P
        assert ib(sqr.raw) == a * a % P
        if a:
            assert ib(inv.raw) == pow(a, P - 2, P)


def test_fp_inv_divsteps_matches_fermat(hostsim):
    # fp_inv (Bernstein-Yang divsteps, fp.cuh) == fp_inv_pow (a^(p-2)) on
    # random non-reduced inputs, 0, p, 2p, 1, p - 1 and powers of two
    hostsim.hs_fp_inv_check.restype = ctypes.c_int
    hostsim.hs_fp_inv_check.argtypes = [ctypes.c_int, ctypes.c_uint64]
    assert hostsim.hs_fp_inv_check(20000, 12345) == 0


def test_fp2_ops_and_sqrt(hostsim):
    rnd = random.Random(2)
    for t in range(12):
        a = (rnd.randrange(P), rnd.randrange(P))
        b = (rnd.randrange(P), rnd.randrange(P))
        if t % 2 == 0:
            a = B.f2_sqr(a)
        mul, sqr, inv, sq = buf(96), buf(96), buf(96), buf(96)
        ok = ctypes.c_int()
        hostsim.hs_fp2_ops(be(a[0]) + be(a[1]), be(b[0]) + be(b[1]), mul, sqr, inv, sq, ctypes.byref(ok))
        g = lambda x: (ib(x.raw[:48]), ib(x.raw[48:]))  # noqa: E731
        assert g(mul) == B.f2_mul(a, b)
        assert g(sqr) == B.f2_sqr(a)
        assert g(inv) == B.f2_inv(a)
        assert bool(ok.value) == B.f2_is_square(a)
        if ok.value:
            assert B.f2_sqr(g(sq)) == (a[0] % P, a[1] % P)


def test_digest_any_prev_length(hostsim):
    rnd = random.Random(3)
    for plen in [0, 8, 32, 47, 48, 55, 56, 63, 64, 96, 119, 120, 200]:
        prev = bytes(rnd.randrange(256) for _ in range(plen))
        r = rnd.randrange(1 << 64)
        out = buf(32)
        hostsim.hs_digest(prev, plen, ctypes.c_uint64(r), out)
        assert out.raw == hashlib.sha256(prev + r.to_bytes(8, "big")).digest()


def test_expand_hash_to_field_sswu(hostsim):
    msg = hashlib.sha256(b"hello").digest()
    out = buf(256)
    hostsim.hs_expand_xmd(msg, out)
    assert out.raw == B.expand_message_xmd(msg, B.DST_G2, 256)
    out = buf(192)
    hostsim.hs_hash_to_field(msg, out)
    u = B.hash_to_field_fp2(msg, 2, B.DST_G2)
    assert [ib(out.raw[i * 48:(i + 1) * 48]) for i in range(4)] == [u[0][0], u[0][1], u[1][0], u[1][1]]
    for uu in u:
        o = buf(192)
        hostsim.hs_sswu(be(uu[0]) + be(uu[1]), o)
        q = B.iso_map_g2(B.map_to_curve_sswu_g2(uu))
        assert [ib(o.raw[i * 48:(i + 1) * 48]) for i in range(4)] == [q[0][0], q[0][1], q[1][0], q[1][1]]


def test_hash_to_g2_golden(hostsim):
    for c in load_golden("hash_to_g2.json")["cases"]:
        o = buf(96)
        hostsim.hs_hash_to_g2(bytes.fromhex(c["msg"]), o)
        assert o.raw.hex() == c["h"]


def test_h2c_finish_ladder_matches_generic(hostsim):
    """k_h2c_finish's sequence (cold points parked in slots, fast additions
    flagging the exceptional cases, the generic cofactor clearing as the
    fallback) equals hash_to_g2 on the golden messages and on 32 random ones,
    and on Q1 = Q0 (P = 2 Q0 via the generic first addition) and Q1 = -Q0
    (P = O: every later addition is exceptional -> fallback, H = O)."""
    import random
    rng = random.Random(5)
    msgs = [bytes.fromhex(c["msg"]) for c in load_golden("hash_to_g2.json")["cases"]]
    msgs += [rng.randbytes(32) for _ in range(32)]
    for msg in msgs:
        for mode in (0, 1, 2):
            o, g = buf(96), buf(96)
            exc = hostsim.hs_h2c_finish_check(msg, mode, o, g)
            assert o.raw == g.raw
            assert exc == (1 if mode == 2 else 0)
            if mode == 0:
                h = buf(96)
                hostsim.hs_hash_to_g2(msg, h)
                assert o.raw == h.raw
            if mode == 2:
                assert o.raw[0] & 0x40  # the infinity flag


def test_ladder_doubling_lazy_matches(hostsim):
    # the cofactor ladder's doubling with Y3's product and Z unreduced
    # (g2_dbl_lz) == the fully reduced doubling over 200 chained doublings
    # from 20 SSWU points
    hostsim.hs_g2_dbl_lz_check.restype = ctypes.c_int
    hostsim.hs_g2_dbl_lz_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
    assert hostsim.hs_g2_dbl_lz_check(20, 200, 3) == 0


def test_subgroup_ladder_matches_generic(hostsim):
    # the decode kernels' G2 membership test on the ladder (lazy doublings,
    # fast mixed additions, P fetched where used) == g2_in_subgroup, on 24
    # points outside G2 (SSWU outputs) and their cofactor-cleared images
    hostsim.hs_g2_subgroup_ladder_check.restype = ctypes.c_int
    hostsim.hs_g2_subgroup_ladder_check.argtypes = [ctypes.c_int, ctypes.c_uint64]
    assert hostsim.hs_g2_subgroup_ladder_check(24, 11) == 0


def test_decompress_kat(hostsim):
    k = load_golden("kat_bls12381_compat_v112.json")
    o = buf(96)
    assert hostsim.hs_decompress_g2(bytes.fromhex(k["sig"]), o) == 0
    assert o.raw.hex() == k["sig"]


def test_verify_golden_chains(hostsim):
    for name in ["chain_chained_s1.json", "chain_unchained_s1.json"]:
        g = load_golden(name)
        pk = bytes.fromhex(g["pk"])
        for r in g["rounds"][:6]:
            msg = D.digest_message(g["scheme"], r["round"], bytes.fromhex(r["prev"]))
            assert hostsim.hs_verify(pk, msg, bytes.fromhex(r["sig"])) == 0
        for c in g["corrupted"]:
            sig = bytes.fromhex(c["sig"])
            if len(sig) != 96:
                continue  # length rule is applied by the batch kernel before decode
            msg = D.digest_message(g["scheme"], c["round"], bytes.fromhex(c["prev"]))
            assert (hostsim.hs_verify(pk, msg, sig) == 0) == c["valid"], c["kind"]


def test_non_subgroup_rejected(hostsim):
    rnd = random.Random(4)
    q = B.iso_map_g2(B.map_to_curve_sswu_g2((rnd.randrange(P), rnd.randrange(P))))
    k = load_golden("kat_bls12381_compat_v112.json")
    assert hostsim.hs_verify(bytes.fromhex(k["pk"]), bytes(32), B.g2_compress(q)) == 2


def test_cyclotomic_squaring(hostsim):
    k = load_golden("kat_bls12381_compat_v112.json")
    assert hostsim.hs_cyclo_sqr_check(bytes.fromhex(k["pk"]), bytes.fromhex(k["sig"])) == 0


def test_pairing_value_matches_generic(hostsim):
    """Full reduced pairing value e(P,Q)^2 (both pairs = (P,Q)) equals the
    generic definition's, element by element."""
    sk = 0x1234567
    P1 = B.g1_mul(B.G1_GEN, sk)
    Q1 = B.g2_mul(B.G2_GEN, 77)
    out = buf(576)
    hostsim.hs_pairing(B.g1_compress(P1), B.g2_compress(Q1), out)
    e = B.f12_pow(B.pairing(P1, Q1), 2)
    assert [ib(out.raw[48 * i:48 * (i + 1)]) for i in range(12)] == B.f12_to_ints(e)


def test_rlc_collapse_algebra(hostsim):
    """sum r_i R_i with h_eff applied once == sum r_i H_i, with the leaves
    computed as the device does ([a] R + [b] psi(R), r = a + b x, joint NAF
    ladder; each leaf checked against plain double-and-add): a valid batch
    passes, one altered round (valid point, wrong message) fails."""
    g = load_golden("chain_chained_s1.json")
    pk = bytes.fromhex(g["pk"])
    rs = g["rounds"][:5]
    msgs = b"".join(D.digest_message(g["scheme"], r["round"], bytes.fromhex(r["prev"])) for r in rs)
    sigs = b"".join(bytes.fromhex(r["sig"]) for r in rs)
    rounds = (ctypes.c_uint64 * 5)(*[r["round"] for r in rs])
    assert hostsim.hs_rlc_batch_check(pk, msgs, sigs, 5, ctypes.c_uint64(99), rounds) == 0
    bad = sigs[:96] + sigs[192:288] + sigs[96:192] + sigs[288:]  # swap rounds 1 and 2
    assert hostsim.hs_rlc_batch_check(pk, msgs, bad, 5, ctypes.c_uint64(99), rounds) == 1


def test_rlc_window_ladder_edge_scalars(hostsim):
    """k_rlc_leaves' uniform ladder [a] q + [b] psi(q) (signed radix-16
    windows, zero digits computed and discarded) equals plain double-and-add
    on a point outside G2, for scalar halves at the recoding's edges: zero
    halves, digits 7 / 8 / 9 (sign flips and carries), carry chains into the
    top digit, and random pairs."""
    import random
    rnd = random.Random(7)
    edge = [0, 1, 7, 8, 9, 15, 16, 0x88888888, 0x77777777, 0xFFFFFFFF, 0x80000000, 0x7FFFFFFF, 0xF8F8F8F8]
    pairs = [(a, b) for a in edge[:7] for b in (0, 8, 0xFFFFFFFF)] + [(a, a ^ 0x5A5A5A5A) for a in edge]
    pairs += [(rnd.getrandbits(32), rnd.getrandbits(32)) for _ in range(8)]
    ab = (ctypes.c_uint32 * (2 * len(pairs)))(*[v for p in pairs for v in p])
    assert hostsim.hs_g2_mul2_win4_check(bytes(range(32)), ab, len(pairs)) == 0


def test_g1_rlc_window_ladder_and_endomorphism(hostsim):
    """G1-signature RLC leaves (rlc_msm.cuh k_rlc_leaves<G1Ops>): the
    group-generic ladder [a] R + [b] phi(R) equals plain double-and-add on a
    pre-cofactor hash point R outside G1; phi(x, y) = (beta x, y) acts on
    H = h_eff R as [-x^2] (and not on R); h_eff commutes with the ladder."""
    import random
    rnd = random.Random(9)
    edge = [0, 1, 7, 8, 9, 15, 16, 0x88888888, 0xFFFFFFFF, 0x80000000]
    pairs = [(a, b) for a in edge for b in (0, 9, 0xFFFFFFFF)] + [(rnd.getrandbits(32), rnd.getrandbits(32)) for _ in range(6)]
    ab = (ctypes.c_uint32 * (2 * len(pairs)))(*[v for p in pairs for v in p])
    assert hostsim.hs_g1_mul2_win4_check(bytes(range(32)), ab, len(pairs)) == 0


@pytest.mark.parametrize("g1dst", [0, 1])
def test_g1_rlc_collapse_algebra(hostsim, g1dst):
    """e(h_eff sum r_i R_i, pk) e(-sum r_i sig_i, g2) == 1 for a valid batch of
    G1 signatures (both DSTs), with r_i = a_i + b_i lambda as the device draws
    them; one signature over another round's message makes it fail."""
    msgs = b"".join(bytes([i]) * 32 for i in range(4))
    assert hostsim.hs_g1_rlc_batch_check(msgs, 4, ctypes.c_uint64(0x1234567), ctypes.c_uint64(5), -1, g1dst) == 0
    assert hostsim.hs_g1_rlc_batch_check(msgs, 4, ctypes.c_uint64(0x1234567), ctypes.c_uint64(5), 2, g1dst) == 1


def test_engine_pairing_host_emulation(hostsim):
    """The device engine's per-lane arithmetic (engine.cuh) run by the host
    emulation over the generated programs: verdict and the exact GT value
    against the oracle, valid and invalid."""
    sk = D.derive_secret(11)
    pk = B.g1_mul(B.G1_GEN, sk)
    pk48 = B.g1_compress(pk)
    for msg, other in ((b"\x05" * 32, None), (b"\x06" * 32, b"\x07" * 32)):
        sig_pt = B.g2_mul(B.hash_to_g2(other or msg), sk)
        out = buf(576)
        rc = hostsim.hs_eng_pairing(pk48, msg, B.g2_compress(sig_pt), out)
        assert rc == (1 if other is None else 0)
        fo = B.f12_mul(B.miller_loop(pk, B.hash_to_g2(msg)), B.miller_loop(B.g1_neg(B.G1_GEN), sig_pt))
        exp = B.f12_conj(B.final_exponentiation(fo))
        w = [exp[0][0], exp[1][0], exp[0][1], exp[1][1], exp[0][2], exp[1][2]]
        got = [ib(out.raw[48 * k:48 * k + 48]) for k in range(12)]
        assert got == [c % P for pair in w for c in pair]


def test_engine_fast_cyc_matches_interpreter(hostsim):
    """The straight-line cyclotomic squaring (engine.cuh eng_cyc_fast, with
    the fused LIN epilogue) leaves every state and LIN slot with the same
    residue as the interpreted E_CYC op, over chains of squarings from random
    slot contents, and the full pairing check through the FE program gives
    the same GT value with it."""
    for seed in (1, 2, 3, 0xDEADBEEF):
        assert hostsim.hs_eng_cyc_compare(ctypes.c_uint64(seed), 40) == 0
    sk = D.derive_secret(12)
    pk48 = B.g1_compress(B.g1_mul(B.G1_GEN, sk))
    msg = b"\x09" * 32
    sig = B.g2_compress(B.g2_mul(B.hash_to_g2(msg), sk))
    outs = []
    for fast in (0, 1):
        hostsim.hs_eng_set_cyc_fast(fast)
        out = buf(576)
        assert hostsim.hs_eng_pairing(pk48, msg, sig, out) == 1
        outs.append(out.raw)
    hostsim.hs_eng_set_cyc_fast(0)
    assert outs[0] == outs[1]


def test_engine_karabina_fe_matches_granger_scott(hostsim):
    """The Karabina FE as the device runs it (8-lane compressed chain over
    ENG_CYC8_PAR, eng_kb_norm / eng_kb_decompress, the ENG_PROG_FEK segments,
    each segment starting from scrambled slots) gives the same GT value words
    as the Granger-Scott program, on valid and invalid pairing checks."""
    sk = D.derive_secret(14)
    pk = B.g1_mul(B.G1_GEN, sk)
    pk48 = B.g1_compress(pk)
    for msg, other in ((b"\x0b" * 32, None), (b"\x0c" * 32, b"\x0d" * 32), (b"\x0e" * 32, None)):
        sig = B.g2_compress(B.g2_mul(B.hash_to_g2(other or msg), sk))
        outs = []
        for kb in (0, 1):
            hostsim.hs_eng_set_fe_kb(kb)
            out = buf(576)
            rc = hostsim.hs_eng_pairing(pk48, msg, sig, out)
            assert rc == (1 if other is None else 0)
            outs.append(out.raw)
        hostsim.hs_eng_set_fe_kb(0)
        assert outs[0] == outs[1]


def test_engine_compiled_ops_match_interpreter(hostsim):
    """The compiled (straight-line) hot ops (engine_compiled.h) give the same
    output words as the interpreter on random slots, and the full pairing
    check through all three programs gives the same GT value with them."""
    for seed in (1, 7, 99):
        assert hostsim.hs_eng_compiled_compare(ctypes.c_uint64(seed)) == 0
    sk = D.derive_secret(13)
    pk48 = B.g1_compress(B.g1_mul(B.G1_GEN, sk))
    msg = b"\x0a" * 32
    sig = B.g2_compress(B.g2_mul(B.hash_to_g2(msg), sk))
    outs = []
    for on in (0, 1):
        hostsim.hs_eng_set_compiled(on)
        out = buf(576)
        assert hostsim.hs_eng_pairing(pk48, msg, sig, out) == 1
        outs.append(out.raw)
    hostsim.hs_eng_set_compiled(0)
    assert outs[0] == outs[1]


def test_hash_to_g1_golden(hostsim):
    """Kernel hash-to-G1 (inversion-free SSWU + 11-isogeny, both DSTs) vs the
    oracle's fixture, including drand digests under the legacy and RFC DSTs."""
    for c in load_golden("hash_to_g1.json")["cases"]:
        if c["msg"] == "":
            continue  # the RFC vector's empty message is not a 32-byte digest
        o = buf(48)
        hostsim.hs_hash_to_g1(bytes.fromhex(c["msg"]), 1 if "G1" in c["dst"] else 0, o)
        assert o.raw.hex() == c["h"], c


def test_decompress_g1_catalog(hostsim):
    """G1 signature decode verdicts (incl. the endomorphism subgroup test) on
    the on-G1 chain fixtures' catalog and valid rounds."""
    codes = {0: D.REASON_OK, 4: D.REASON_INFINITY, 7: D.REASON_SUBGROUP}
    for name in ("chain_on_g1_s1.json", "chain_g1_rfc9380_s2.json"):
        g = load_golden(name)
        for r in g["rounds"][:4]:
            o = buf(48)
            assert hostsim.hs_decompress_g1(bytes.fromhex(r["sig"]), o) == 0
            assert o.raw.hex() == r["sig"]
        for c in g["corrupted"]:
            sig = bytes.fromhex(c["sig"])
            if len(sig) != 48:
                continue
            rc = hostsim.hs_decompress_g1(sig, buf(48))
            want = c["reason"] if c["reason"] != D.REASON_PAIRING else D.REASON_OK
            assert codes.get(rc, D.REASON_DECODE) == want, (c["kind"], rc)


def test_engine_fused_subgroup_check(hostsim):
    """The lines program's LSUB op (psi(sig) == -[|x|] sig from the Miller
    loop's own ladder, k_eng_lines status) on the device arithmetic: G2
    points pass, random curve points outside G2 fail -- same verdict as the
    oracle's [r]Q test."""
    k = load_golden("kat_bls12381_compat_v112.json")
    assert hostsim.hs_eng_subgroup(bytes.fromhex(k["sig"])) == 1
    g = load_golden("chain_chained_s1.json")
    for r in g["rounds"][:3]:
        assert hostsim.hs_eng_subgroup(bytes.fromhex(r["sig"])) == 1
    rnd = random.Random(9)
    for _ in range(3):
        q = B.iso_map_g2(B.map_to_curve_sswu_g2((rnd.randrange(P), rnd.randrange(P))))
        assert not B.g2_in_subgroup(q)
        assert hostsim.hs_eng_subgroup(B.g2_compress(q)) == 0


def test_thread_lines_match_oracle_and_engine(hostsim):
    """The per-thread T-steps (lines_thread.cuh lt_pair, k_lines_thr) feeding
    the engine's Miller and FE programs give the oracle's exact GT value on
    valid and invalid checks (each line may differ from the engine's by an Fp2
    scale, which the final exponentiation removes), and their fused membership
    test gives the oracle's verdicts."""
    sk = D.derive_secret(15)
    pk = B.g1_mul(B.G1_GEN, sk)
    pk48 = B.g1_compress(pk)
    try:
        for msg, other in ((b"\x21" * 32, None), (b"\x22" * 32, b"\x23" * 32)):
            sig_pt = B.g2_mul(B.hash_to_g2(other or msg), sk)
            outs = []
            for on in (0, 1):
                hostsim.hs_eng_set_lines_thread(on)
                out = buf(576)
                assert hostsim.hs_eng_pairing(pk48, msg, B.g2_compress(sig_pt), out) == (1 if other is None else 0)
                outs.append(out.raw)
            assert outs[0] == outs[1]
            fo = B.f12_mul(B.miller_loop(pk, B.hash_to_g2(msg)), B.miller_loop(B.g1_neg(B.G1_GEN), sig_pt))
            exp = B.f12_conj(B.final_exponentiation(fo))
            w = [exp[0][0], exp[1][0], exp[0][1], exp[1][1], exp[0][2], exp[1][2]]
            assert [ib(outs[1][48 * k:48 * k + 48]) for k in range(12)] == [c % P for pair in w for c in pair]
        hostsim.hs_eng_set_lines_thread(1)
        g = load_golden("chain_chained_s1.json")
        for r in g["rounds"][:2]:
            assert hostsim.hs_eng_subgroup(bytes.fromhex(r["sig"])) == 1
        rnd = random.Random(10)
        for _ in range(2):
            q = B.iso_map_g2(B.map_to_curve_sswu_g2((rnd.randrange(P), rnd.randrange(P))))
            assert hostsim.hs_eng_subgroup(B.g2_compress(q)) == 0
    finally:
        hostsim.hs_eng_set_lines_thread(0)


def test_kb_chain_two_lane_squaring_matches(hostsim):
    # k_kb_chain_pair's squaring (each lane squares its Fp4 half, the lanes
    # swap (q, k), each forms its new half) == the one-thread kb_sqr_thr, limb
    # for limb, over 20 chained squarings from 300 random CI starts and the
    # all-maximal-limb start
    hostsim.hs_kb_pair_check.restype = ctypes.c_int
    hostsim.hs_kb_pair_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
    assert hostsim.hs_kb_pair_check(300, 20, 91) == 0


def test_kb_decompress_lazy_matches(hostsim):
    # the decompression with lazy linear steps (what k_eng_kb_dec runs) ==
    # the every-step-reduced form, outputs CI, on 2,000 random inputs up to the
    # CI bound and the all-maximal-limb input
    hostsim.hs_kb_dec_lz_check.restype = ctypes.c_int
    hostsim.hs_kb_dec_lz_check.argtypes = [ctypes.c_int, ctypes.c_uint64]
    assert hostsim.hs_kb_dec_lz_check(2000, 77) == 0


def test_thread_kb_chain_matches_lane_chain(hostsim):
    """The per-thread compressed chain (kb_thread.cuh kb_chain_thr,
    k_kb_chain_thr) in the Karabina FE gives the same GT value words as the
    8-lane chain rows, and the oracle's, on valid and invalid checks."""
    sk = D.derive_secret(16)
    pk = B.g1_mul(B.G1_GEN, sk)
    pk48 = B.g1_compress(pk)
    hostsim.hs_eng_set_fe_kb(1)
    try:
        for msg, other in ((b"\x31" * 32, None), (b"\x32" * 32, b"\x33" * 32)):
            sig_pt = B.g2_mul(B.hash_to_g2(other or msg), sk)
            outs = []
            for on in (0, 1):
                hostsim.hs_eng_set_kb_thread(on)
                out = buf(576)
                assert hostsim.hs_eng_pairing(pk48, msg, B.g2_compress(sig_pt), out) == (1 if other is None else 0)
                outs.append(out.raw)
            assert outs[0] == outs[1]
            fo = B.f12_mul(B.miller_loop(pk, B.hash_to_g2(msg)), B.miller_loop(B.g1_neg(B.G1_GEN), sig_pt))
            exp = B.f12_conj(B.final_exponentiation(fo))
            w = [exp[0][0], exp[1][0], exp[0][1], exp[1][1], exp[0][2], exp[1][2]]
            assert [ib(outs[1][48 * k:48 * k + 48]) for k in range(12)] == [c % P for pair in w for c in pair]
    finally:
        hostsim.hs_eng_set_kb_thread(0)
        hostsim.hs_eng_set_fe_kb(0)


def test_engine_cofactor_ladder_matches_golden_hash(hostsim):
    """The small-call cofactor clearing (two passes of the LINES program,
    whose T after the loop is [|x|]Q, composed as k_cof_partial / k_cof_final
    compose it) gives the golden H(m) -- the vectors k_h2c_finish's
    per-thread ladders are pinned to (hash_to_g2.json, from the oracle
    pinned by key/curve_test.go:10-30)."""
    cases = load_golden("hash_to_g2.json")["cases"]
    for c in cases:
        o = buf(96)
        hostsim.hs_eng_cof_hash_to_g2(bytes.fromhex(c["msg"]), o)
        assert o.raw.hex() == c["h"]
