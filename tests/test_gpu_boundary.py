"""GPU tests of the C-ABI boundary (include/drand_gpu.h, ABI 3) beyond the
per-round verdicts of test_gpu_parity.py:

  * raw-message surface (key.Scheme.VerifyRecovered / AuthScheme with any msg,
    key/curve.go:36-39): hash-to-curve of many message lengths vs the oracle's
    fixture, sign + verify on G2 and G1;
  * decode of every deploy/latest/group.toml key on the GPU;
  * the public key per call (VerifyBeacon(b, pubkey), chain/verify.go:38): two
    chains with different keys and schemes interleaved on one context;
  * RLC soundness with duplicated Round fields (+D / -D corruptions) and the
    root-first check;
  * records whose length exceeds their stride on the device entry point;
  * the multi-GPU handle (dgpu_verify_multi) with one device equals the
    single-context verdicts (RCCL all-gathers over one rank).
Marked gpu."""
import numpy as np
import pytest

from conftest import load_golden, open_ctx
from oracle import bls12381 as B

pytestmark = pytest.mark.gpu


def _sch(name):
    from drand_amd.scheme import get_scheme_by_id_with_default
    return get_scheme_by_id_with_default(name)


def test_hash_to_curve_any_length(gpu_ctx):
    from drand_amd.chain import hash_to_curve
    g = load_golden("hash_var_len.json")
    msgs = [bytes.fromhex(c["msg"]) for c in g["cases"]]
    assert [h.hex() for h in hash_to_curve(msgs, _sch("pedersen-bls-chained"))] == [c["g2"] for c in g["cases"]]
    for name in ("bls-unchained-on-g1", "bls-unchained-g1-rfc9380"):
        assert [h.hex() for h in hash_to_curve(msgs, _sch(name))] == [c["g1/" + name] for c in g["cases"]]


@pytest.mark.parametrize("name", ["pedersen-bls-chained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"])
def test_sign_and_verify_recovered_any_length(name, gpu_ctx):
    """AuthScheme.Sign -> VerifyRecovered round trip over raw messages of many
    lengths; a signature of another message, a wrong key and an empty
    signature fail; signatures equal the oracle's sk * H(msg)."""
    from drand_amd import _lib
    from drand_amd.chain import sign, verify_recovered
    from drand_amd.synth import derive_secret
    sch = _sch(name)
    on_g1 = name != "pedersen-bls-chained"
    sk = derive_secret(21)
    msgs = [bytes.fromhex(c["msg"]) for c in load_golden("hash_var_len.json")["cases"]]
    sigs = sign(sk, msgs, sch)
    code = _lib.SCHEME_UNCHAINED_G1 if name == "bls-unchained-on-g1" else (
        _lib.SCHEME_G1_RFC9380 if on_g1 else _lib.SCHEME_CHAINED)
    pk = np.zeros(96 if on_g1 else 48, dtype=np.uint8)
    skb = np.frombuffer(sk.to_bytes(32, "big"), dtype=np.uint8).copy()
    _lib.check(gpu_ctx.lib.dgpu_derive_pubkey(gpu_ctx.handle, code, _lib.ptr(skb), _lib.ptr(pk), pk.size))
    pk = bytes(pk)
    assert verify_recovered(sch, pk, msgs, sigs).tolist() == [0] * len(msgs)
    swapped = sigs[1:] + sigs[:1]
    assert verify_recovered(sch, pk, msgs, swapped).tolist() == [3] * len(msgs)
    assert verify_recovered(sch, pk, msgs[:2], [b"", sigs[1][:10]]).tolist() == [1, 1]
    other = sign(derive_secret(22), msgs[:1], sch)
    assert verify_recovered(sch, pk, msgs[:1], other).tolist() == [3]
    # the oracle's signature for two lengths
    from oracle import drand_ref as D
    for i in (0, 2):
        if on_g1:
            exp = B.sign_g1(sk, msgs[i], D.SIG_ON_G1_DST[name])
        else:
            exp = B.sign_g2(sk, msgs[i])
        assert sigs[i] == exp


def test_group_toml_keys_decode_on_gpu(gpu_ctx):
    """Every key of deploy/latest/group.toml decodes on the GPU to the
    oracle's point; malformed encodings are rejected with kilic's classes."""
    from drand_amd.chain import decode_g1_points
    keys = load_golden("group_toml_keys.json")["keys"]
    rc, pts = decode_g1_points([bytes.fromhex(k["pk"]) for k in keys])
    assert rc == [0 if k["decodes"] else rc[i] for i, k in enumerate(keys)]
    for k, pt in zip(keys, pts):
        if k["decodes"]:
            assert pt == B.g1_decompress(bytes.fromhex(k["pk"]))
    good = bytes.fromhex(keys[0]["pk"])
    bad = [bytes([good[0] & 0x7F]) + good[1:],             # compression flag clear
           bytes([0xC0]) + bytes(47),                       # canonical infinity
           bytes([0xC0]) + bytes(46) + b"\x01",             # non-canonical infinity
           bytes([0x9F]) + b"\xff" * 47]                    # x >= p
    x = 5
    while B.fp_sqrt(x ** 3 + 4) is not None:
        x += 1
    bad.append(bytes([0x80]) + x.to_bytes(48, "big")[1:])  # not on the curve
    rc, _ = decode_g1_points(bad)
    assert rc[1] == 4 and all(r not in (0, 4) for i, r in enumerate(rc) if i != 1)


def test_reference_legacy_encodings_decode_on_gpu(gpu_ctx):
    """The reference's decode-only encodings for the G1-signature layout
    (SURVEY.md 8(c)4): test/test-integration/test.json's 48-byte G1 Signature
    and Previous and 96-byte G2 Public, and demo/docker/data's five G1 node
    keys, each as stored and mutated.  G1 encodings go through the on-G1
    schemes' signature decoder (k_decode_g1_sigs) and the G2-signature
    schemes' key decoder; G2 encodings through the on-G1 schemes' key decoder
    and the G2 signature decoder (k_decode_g2_sigs_sub).  Reasons and
    coordinates equal the oracle's (tests/golden/reference_legacy_encodings.json).
    Decode only: test.json's message and hash predate RFC 9380 (its signature
    verifies under none of SHA-256(prev||round), SHA-256(round) with either
    RFC 9380 DST), so no verdict is asserted."""
    from drand_amd import _lib
    from drand_amd.chain import decode_pubkey, decode_signatures
    cases = load_golden("reference_legacy_encodings.json")["cases"]
    for grp, sig_schemes, key_schemes in (
            ("g1", ("bls-unchained-on-g1", "bls-unchained-g1-rfc9380"), ("pedersen-bls-chained",)),
            ("g2", ("pedersen-bls-chained", "pedersen-bls-unchained"), ("bls-unchained-on-g1",))):
        cs = [c for c in cases if c["group"] == grp]
        raw = [bytes.fromhex(c["hex"]) for c in cs]

        def expect(c):
            if not c["decodes"]:
                return None
            v = [int(c["xy"][96 * j:96 * j + 96], 16) for j in range(len(c["xy"]) // 96)]
            return tuple(v) if grp == "g1" else ((v[0], v[1]), (v[2], v[3]))

        for name in sig_schemes:
            reasons, pts = decode_signatures(_sch(name), raw)
            assert reasons == [c["reason"] for c in cs], name
            assert pts == [expect(c) for c in cs], name
        for name in key_schemes:
            for c, r in zip(cs, raw):
                if c["decodes"]:
                    assert decode_pubkey(_sch(name), r) == expect(c)
                else:
                    with pytest.raises(_lib.DrandGPUError):
                        decode_pubkey(_sch(name), r)
    # the stored test.json key installs as an on-G1 scheme's key (line table built)
    pub = next(c for c in cases if c["kind"] == "as_stored" and c["group"] == "g2")
    pkb = np.frombuffer(bytes.fromhex(pub["hex"]), dtype=np.uint8).copy()
    _lib.check(gpu_ctx.lib.dgpu_set_pubkey(gpu_ctx.handle, _lib.SCHEME_UNCHAINED_G1, _lib.ptr(pkb), 96))


def test_two_chains_two_keys_one_context(gpu_ctx):
    """Verifiers of different chains (different keys, chained / unchained /
    on-G1) share one GPU context; calls alternate and each verdict uses the
    key passed with it (no stale per-verifier key)."""
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.synth import make_chain
    ca = make_chain(31, 40, _lib.SCHEME_CHAINED, seg_len=8)
    cb = make_chain(32, 40, _lib.SCHEME_UNCHAINED, seg_len=8)
    cg = make_chain(33, 40, _lib.SCHEME_UNCHAINED_G1, seg_len=8)
    va, vb, vg = (Verifier(_sch(n)) for n in ("pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1"))
    ba = [ca.beacon(i) for i in range(len(ca))]
    bb = [cb.beacon(i) for i in range(len(cb))]
    bg = [cg.beacon(i) for i in range(len(cg))]
    for _ in range(2):
        assert va.verify_reasons(ba, ca.pk).tolist() == [0] * 40
        assert vb.verify_reasons(bb, cb.pk).tolist() == [0] * 40
        assert vg.verify_reasons(bg, cg.pk).tolist() == [0] * 40
        assert va.verify_reasons(ba, cb.pk).tolist() == [3] * 40   # the other chain's key
        assert vb.verify_reasons(bb, ca.pk, _lib.MODE_RLC).tolist() == [3] * 40
    with pytest.raises(_lib.DrandGPUError):
        vg.verify_reasons(bg, ca.pk)                                # a G1 key for a G2-key scheme


def test_rlc_duplicate_rounds_cannot_cancel(gpu_ctx):
    """Two records with the same Round (and PreviousSig) whose signatures are
    sig + D and sig - D: with coefficients keyed on the Round field they
    would cancel in every RLC node; keyed on the batch position both fail,
    as per-round mode says."""
    from drand_amd import _lib
    from drand_amd.chain import Beacon, Verifier
    from drand_amd.synth import make_chain
    c = make_chain(41, 300, _lib.SCHEME_CHAINED, seg_len=64)
    beacons = [c.beacon(i) for i in range(len(c))]
    i = 137
    s = B.g2_decompress(beacons[i].signature)
    d = B.G2_GEN
    plus = B.g2_compress(B.g2_add(s, d))
    minus = B.g2_compress(B.g2_add(s, B.g2_neg(d)))
    b = beacons[i]
    beacons[i] = Beacon(b.previous_sig, b.round, plus)
    beacons.insert(i + 1, Beacon(b.previous_sig, b.round, minus))
    v = Verifier(_sch("pedersen-bls-chained"))
    per = v.verify_reasons(beacons, c.pk)
    expect = [0] * len(beacons)
    expect[i] = expect[i + 1] = 3
    assert per.tolist() == expect
    for seed in (1, 2, 0xFFFFFFFFFFFFFFFF):
        assert v.verify_reasons(beacons, c.pk, _lib.MODE_RLC, seed).tolist() == expect


def test_rlc_localize_then_confirm_and_fallback(gpu_ctx):
    """A failing RLC root is resolved on the tree of plain sums (leaf checks
    are the rounds' own pairings), then the rest is confirmed with a fresh
    random combination (capi.hip rlc_resolve_locked).  Ordinary corruption:
    the confirmation passes and the random-coefficient leaves are never
    built.  Errors crafted to cancel in a plain sum (sig + D, sig - D under
    one node) slip past the localization: the confirmation fails and the
    random-coefficient tree finds them -- verdicts equal per-round mode either
    way."""
    from drand_amd import _lib
    from drand_amd.chain import Beacon, Verifier
    from drand_amd.synth import corrupt, make_chain
    v = Verifier(_sch("pedersen-bls-chained"))
    lib = v.ctx.lib

    def rlc_stages(beacons, pk):
        _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 1))
        try:
            got = v.verify_reasons(beacons, pk, _lib.MODE_RLC)
            return got, set(_lib.stage_times(v.ctx))
        finally:
            _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 0))

    c = make_chain(45, 4000, _lib.SCHEME_CHAINED, seg_len=64)
    corrupt(c, 45, rate=3e-3)
    beacons = [c.beacon(i) for i in range(len(c))]
    per = v.verify_reasons(beacons, c.pk)
    got, st = rlc_stages(beacons, c.pk)
    assert got.tolist() == per.tolist()
    assert {"rlc_plain_tree", "rlc_confirm"} <= st and "rlc_leaves_tree" not in st, st
    # +D / -D in rounds 137 and 138: one level-3 node (rounds 136..143) of
    # the plain tree, the first level the descent checks for a batch above
    # 64Ki rounds (descent step 3: 70,000 -> 8,750 nodes)
    c2 = make_chain(46, 70000, _lib.SCHEME_CHAINED, seg_len=64)
    b2 = [c2.beacon(i) for i in range(len(c2))]
    s = B.g2_decompress(b2[137].signature)
    s2 = B.g2_decompress(b2[138].signature)
    b2[137] = Beacon(b2[137].previous_sig, b2[137].round, B.g2_compress(B.g2_add(s, B.G2_GEN)))
    b2[138] = Beacon(b2[138].previous_sig, b2[138].round, B.g2_compress(B.g2_add(s2, B.g2_neg(B.G2_GEN))))
    per2 = v.verify_reasons(b2, c2.pk)
    assert per2[137] == per2[138] == _lib.REASON_PAIRING
    got2, st2 = rlc_stages(b2, c2.pk)
    assert got2.tolist() == per2.tolist()
    assert {"rlc_plain_tree", "rlc_confirm", "rlc_leaves_tree"} <= st2, st2


def test_rlc_root_first_clean_and_single_bad(gpu_ctx):
    """A clean batch passes with the root check alone; one bad round among
    70k is found (descent from the root) -- verdicts equal per-round mode."""
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.synth import corrupt, make_chain
    import ctypes
    v = Verifier(_sch("pedersen-bls-chained"))
    c = make_chain(43, 70000, _lib.SCHEME_CHAINED, seg_len=64)
    beacons = [c.beacon(i) for i in range(len(c))]
    lib = v.ctx.lib
    _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 1))
    try:
        assert not v.verify_reasons(beacons, c.pk, _lib.MODE_RLC).any()
        stages = set(_lib.stage_times(v.ctx))
    finally:
        _lib.check(lib.dgpu_set_profiling(v.ctx.handle, 0))
    # the bucket-MSM root (rlc_msm.cuh) equals the tree's: a clean batch
    # passes on it alone, without building the leaves
    assert "rlc_root_msm" in stages and "rlc_leaves_tree" not in stages, stages
    bad = corrupt(c, 43, rate=1e-5, kinds=(3,))  # one signature of another round
    (k,) = bad.keys()
    beacons[k] = c.beacon(k)
    rlc = v.verify_reasons(beacons, c.pk, _lib.MODE_RLC)
    assert np.nonzero(rlc)[0].tolist() == [k] and rlc[k] == 3


def test_device_record_over_stride_fails_without_overrun(gpu_ctx):
    """dgpu_verify_beacons_device with prev_len[i] > prev_stride: round i is
    not read past its stride and fails (DGPU_REASON_DECODE); the others keep
    their verdicts."""
    import ctypes
    import torch
    from drand_amd import _lib
    from drand_amd.synth import make_chain
    c = make_chain(51, 64, _lib.SCHEME_CHAINED, seg_len=64)
    n = len(c)
    dev = torch.device("cuda", 0)
    prev_len = c.prev_len.copy()
    prev_len[5] = 97        # stride is 96
    prev_len[9] = 1 << 30   # far past the buffer
    t = {k: torch.from_numpy(a).to(dev) for k, a in (("r", c.rounds.view(np.int64)), ("s", c.sigs),
                                                      ("sl", c.sig_len.view(np.int32)), ("p", c.prev),
                                                      ("pl", prev_len.view(np.int32)))}
    bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
    reason = torch.zeros(n, dtype=torch.uint8, device=dev)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    stream = torch.cuda.current_stream(dev)
    _lib.check(gpu_ctx.lib.dgpu_verify_beacons_device(
        gpu_ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(pk), pk.size, n, t["r"].data_ptr(), t["s"].data_ptr(), 96,
        t["sl"].data_ptr(), t["p"].data_ptr(), 96, t["pl"].data_ptr(), _lib.MODE_PER_ROUND, 0, bits.data_ptr(),
        reason.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
    r = reason.cpu().numpy()
    expect = np.zeros(n, dtype=np.uint8)
    expect[[5, 9]] = 1
    assert r.tolist() == expect.tolist()
    assert np.array_equal(np.unpackbits(bits.cpu().numpy(), bitorder="little")[:n].astype(bool), r == 0)


def test_unpinned_x_ge_p_rejected(gpu_ctx):
    """kilic's x >= p rejection is recalled, not pinned by a reference test
    (SURVEY.md 8(c)); the GPU rejects like the oracle (reason 1).  Listed
    apart from the verdict corpus."""
    from drand_amd.chain import Beacon, Verifier
    for name in ("chain_chained_s1.json", "chain_unchained_s1.json"):
        g = load_golden(name)
        v = Verifier(_sch(g["scheme"]))
        cases = g["unpinned"]
        got = v.verify_reasons([Beacon(bytes.fromhex(c["prev"]), c["round"], bytes.fromhex(c["sig"])) for c in cases],
                               bytes.fromhex(g["pk"]))
        assert got.tolist() == [c["reason"] for c in cases]


@pytest.mark.parametrize("mode", [0, 1])
def test_verify_multi_one_device_equals_single_context(mode, gpu_ctx):
    """dgpu_verify_multi over one device (RCCL communicator of one rank:
    all-gather of the bitmap, and in RLC mode of the root) == the single
    context's verdicts and reasons == construction."""
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.multi import MultiVerifier
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(61, 5003, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 61, rate=2e-3)
    beacons = [c.beacon(i) for i in range(len(c))]
    single = Verifier(_sch("pedersen-bls-chained")).verify_reasons(beacons, c.pk)
    mv = MultiVerifier(_sch("pedersen-bls-chained"), [0])
    try:
        got = mv.verify_reasons(beacons, c.pk, mode)
        clean = mv.verify_reasons([b for i, b in enumerate(beacons[:1000]) if i not in bad], c.pk, mode)
    finally:
        mv.close()
    assert got.tolist() == single.tolist()
    expect = np.ones(len(c), dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(got == 0, expect)
    assert not clean.any()


def test_async_calls_on_two_streams_are_ordered(gpu_ctx):
    """Two dgpu_verify_beacons_device calls on different streams share the
    context's scratch; the second is ordered after the first on the device
    (ADVICE r01), so both verdict sets are right."""
    import ctypes
    import torch
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    dev = torch.device("cuda", 0)
    chains = [make_chain(71 + k, 40000, _lib.SCHEME_CHAINED, seg_len=64) for k in range(2)]
    bads = [corrupt(c, 71 + k, rate=1e-3) for k, c in enumerate(chains)]
    from drand_amd.chain import Verifier
    v = Verifier(_sch("pedersen-bls-chained"))
    for c in chains:  # both keys cached first: the async calls below never synchronize on a key decode
        v.verify_reasons([c.beacon(0)], c.pk)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = []
    keep = []
    for c, st in zip(chains, streams):
        t = [torch.from_numpy(a).to(dev) for a in (c.rounds.view(np.int64), c.sigs, c.sig_len.view(np.int32), c.prev,
                                                  c.prev_len.view(np.int32))]
        torch.cuda.synchronize()
        with torch.cuda.stream(st):  # zero-filled in the order of the stream the library runs on
            bits = torch.zeros((len(c) + 7) // 8, dtype=torch.uint8, device=dev)
        pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
        keep.append((t, pk))
        _lib.check(gpu_ctx.lib.dgpu_verify_beacons_device(
            gpu_ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(pk), pk.size, len(c), t[0].data_ptr(), t[1].data_ptr(), 96,
            t[2].data_ptr(), t[3].data_ptr(), 96, t[4].data_ptr(), _lib.MODE_PER_ROUND, 0, bits.data_ptr(), None,
            ctypes.c_void_p(st.cuda_stream)))
        outs.append(bits)
    torch.cuda.synchronize()
    for c, bad, bits in zip(chains, bads, outs):
        got = np.unpackbits(bits.cpu().numpy(), bitorder="little")[: len(c)].astype(bool)
        expect = np.ones(len(c), dtype=bool)
        expect[list(bad.keys())] = False
        assert np.array_equal(got, expect)


@pytest.mark.parametrize("mode", [0, 1])
def test_null_stream_is_the_default_stream(mode, gpu_ctx):
    """ABI 3 stream contract: a NULL stream is the legacy
    default stream, so outputs torch fills on its default stream before the
    call and reads after it are ordered with the library's work -- no
    synchronize anywhere.  Outputs are pre-filled with a pattern the verdict
    packing never leaves (0xA5), inputs are copied with non_blocking H2D on
    the default stream; per-round and RLC mode (a 70k batch, above the RLC
    threshold), verdicts and reasons equal construction."""
    import ctypes
    import torch
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    dev = torch.device("cuda", 0)
    assert torch.cuda.current_stream(dev).cuda_stream == 0
    c = make_chain(81, 70001, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 81, rate=1e-3)
    n = len(c)
    t = [torch.from_numpy(a).pin_memory().to(dev, non_blocking=True)
         for a in (c.rounds.view(np.int64), c.sigs, c.sig_len.view(np.int32), c.prev, c.prev_len.view(np.int32))]
    bits = torch.full(((n + 7) // 8,), 0xA5, dtype=torch.uint8, device=dev)
    reason = torch.full((n,), 0xA5, dtype=torch.uint8, device=dev)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    _lib.check(gpu_ctx.lib.dgpu_verify_beacons_device(
        gpu_ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(pk), pk.size, n, t[0].data_ptr(), t[1].data_ptr(), 96,
        t[2].data_ptr(), t[3].data_ptr(), 96, t[4].data_ptr(), mode, 12345, bits.data_ptr(), reason.data_ptr(),
        ctypes.c_void_p(None)))
    got = np.unpackbits(bits.cpu().numpy(), bitorder="little")[:n].astype(bool)
    r = reason.cpu().numpy()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(got, expect)
    assert np.array_equal(r == 0, expect) and set(np.unique(r)) <= {0, 1, 2, 3, 4}
    # dgpu_synchronize: the host-side wait a caller without HIP (cgo) uses
    _lib.check(gpu_ctx.lib.dgpu_synchronize(gpu_ctx.handle))


def test_engine_chunk_retry_after_out_of_memory(gpu_ctx):
    """The engine chunk halves and retries when its buffers do not fit
    (eng_pairing_locked): the A/B build's DGPU_TEST_ALLOC_CAP=1 GB
    fails the 40,000-round chunk's 1.8 GB line buffer until the chunk is
    20,000 rounds.  The call succeeds with the verdicts of an unconstrained
    context and leaves no stale error message; a later call on the context
    still works."""
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    n = 40000
    c = make_chain(71, n, _lib.SCHEME_CHAINED, seg_len=64)
    bad = corrupt(c, 71, rate=1e-3)
    ctx = open_ctx({"DGPU_TEST_ALLOC_CAP": str(1 << 30)})
    try:
        got = []
        for _ in range(2):
            bits = np.zeros((n + 7) // 8, dtype=np.uint8)
            reason = np.zeros(n, dtype=np.uint8)
            pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
            _lib.check(ctx.lib.dgpu_verify_beacons(ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(pk), pk.size, n,
                                                   _lib.ptr(c.rounds), _lib.ptr(c.sigs), c.sigs.shape[1],
                                                   _lib.ptr(c.sig_len), _lib.ptr(c.prev), c.prev.shape[1],
                                                   _lib.ptr(c.prev_len), _lib.MODE_PER_ROUND, 0, _lib.ptr(bits),
                                                   _lib.ptr(reason)), ctx.lib)
            assert ctx.lib.dgpu_last_error() == b""
            got.append(reason)
    finally:
        ctx.close()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(got[0] == 0, expect) and got[0].tolist() == got[1].tolist()


@pytest.mark.parametrize("n,scheme", [(300001, "SCHEME_CHAINED"), (70001, "SCHEME_UNCHAINED"),
                                      (50001, "SCHEME_UNCHAINED_G1")])
def test_host_records_staged_through_the_ring(n, scheme, gpu_ctx):
    """Host records reach the device through the pinned ring (two 16 MiB
    slots, so every array here takes several pieces), in two slices beside
    the two lanes for the large chained batch and in one slice otherwise:
    dgpu_staging_stats reports exactly the record bytes, the verdicts equal
    the device-resident entry point's on the same records (and the
    construction), and the caller's buffers are free to reuse after the
    call (they are overwritten and verified again)."""
    import torch
    from drand_amd import _lib
    from drand_amd.synth import corrupt, make_chain
    code = getattr(_lib, scheme)
    c = make_chain(73, n, code, seg_len=64)
    bad = corrupt(c, 73, rate=1e-3)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    lib, h = gpu_ctx.lib, gpu_ctx.handle

    def host_call():
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        _lib.check(lib.dgpu_verify_beacons(h, code, _lib.ptr(pk), pk.size, n, _lib.ptr(c.rounds), _lib.ptr(c.sigs),
                                           c.sigs.shape[1], _lib.ptr(c.sig_len), _lib.ptr(c.prev), c.prev.shape[1],
                                           _lib.ptr(c.prev_len), _lib.MODE_PER_ROUND, 0, _lib.ptr(bits),
                                           _lib.ptr(reason)))
        return reason

    got = host_call()
    ms, host_ms, nbytes = _lib.staging_stats(gpu_ctx)
    per = c.sigs.shape[1] + 4 + 8 + ((c.prev.shape[1] + 4) if code == _lib.SCHEME_CHAINED else 0)
    assert nbytes == n * per and ms > 0 and host_ms > 0
    dev = {k: torch.from_numpy(np.ascontiguousarray(getattr(c, k))).cuda()
           for k in ("rounds", "sigs", "sig_len", "prev", "prev_len")}
    dbits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device="cuda")
    dreason = torch.zeros(n, dtype=torch.uint8, device="cuda")
    _lib.check(lib.dgpu_verify_beacons_device(h, code, _lib.ptr(pk), pk.size, n, _lib.ptr(dev["rounds"]),
                                              _lib.ptr(dev["sigs"]), c.sigs.shape[1], _lib.ptr(dev["sig_len"]),
                                              _lib.ptr(dev["prev"]), c.prev.shape[1], _lib.ptr(dev["prev_len"]),
                                              _lib.MODE_PER_ROUND, 0, _lib.ptr(dbits), _lib.ptr(dreason), None))
    torch.cuda.synchronize()
    assert dreason.cpu().numpy().tolist() == got.tolist()
    expect = np.ones(n, dtype=bool)
    expect[list(bad.keys())] = False
    assert np.array_equal(got == 0, expect)
    # the caller reuses its buffers: every signature moved to the next round
    # (only an "other round's signature" corruption can turn valid again)
    keep = c.sigs.copy()
    c.sigs[:] = np.roll(keep, 1, axis=0)
    try:
        again = host_call()
        dev["sigs"].copy_(torch.from_numpy(c.sigs))
        _lib.check(lib.dgpu_verify_beacons_device(h, code, _lib.ptr(pk), pk.size, n, _lib.ptr(dev["rounds"]),
                                                  _lib.ptr(dev["sigs"]), c.sigs.shape[1], _lib.ptr(dev["sig_len"]),
                                                  _lib.ptr(dev["prev"]), c.prev.shape[1], _lib.ptr(dev["prev_len"]),
                                                  _lib.MODE_PER_ROUND, 0, _lib.ptr(dbits), _lib.ptr(dreason), None))
        torch.cuda.synchronize()
    finally:
        c.sigs[:] = keep
    assert dreason.cpu().numpy().tolist() == again.tolist()
    assert (again != 0).sum() >= n - len(bad)
    if code == _lib.SCHEME_CHAINED:
        # a record longer than its stride, in the first and in the last slice:
        # the staging thread finds it and the call fails with DGPU_EINVAL; the
        # context serves the next call
        for i in (2, n - 3):
            old = int(c.prev_len[i])
            c.prev_len[i] = c.prev.shape[1] + 1
            try:
                with pytest.raises(_lib.DrandGPUError) as e:
                    host_call()
                assert e.value.code == _lib.DGPU_EINVAL and f"prev_len[{i}]" in str(e.value)
            finally:
                c.prev_len[i] = old
        assert host_call().tolist() == got.tolist()


def test_empty_batches_are_no_ops(gpu_ctx):
    """n = 0 on the batch entry points (CheckPastBeacons over an empty range,
    an empty tryNode window): DGPU_OK, nothing written, NULL record arrays
    accepted.  G2 and G1 schemes, per-round and RLC, host and device entry
    points, raw-message verify and recovery with zero rounds."""
    from drand_amd import _lib
    from drand_amd.synth import make_chain
    lib, h = gpu_ctx.lib, gpu_ctx.handle
    bits = np.full(2, 0xAB, dtype=np.uint8)
    reason = np.full(2, 0xCD, dtype=np.uint8)
    for code in (_lib.SCHEME_CHAINED, _lib.SCHEME_UNCHAINED_G1):
        pk = np.frombuffer(make_chain(72, 2, code, seg_len=2).pk, dtype=np.uint8).copy()
        for mode in (_lib.MODE_PER_ROUND, _lib.MODE_RLC):
            _lib.check(lib.dgpu_verify_beacons(h, code, _lib.ptr(pk), pk.size, 0, None, None, 96, None, None, 96, None,
                                               mode, 7, _lib.ptr(bits), _lib.ptr(reason)))
            _lib.check(lib.dgpu_verify_beacons_device(h, code, _lib.ptr(pk), pk.size, 0, None, None, 96, None, None, 96,
                                                      None, mode, 7, None, None, None))
            _lib.check(lib.dgpu_verify_recovered(h, code, _lib.ptr(pk), pk.size, 0, None, 32, None, None, 96, None,
                                                 mode, 7, _lib.ptr(bits), _lib.ptr(reason)))
    g = load_golden("recover_t3_n8.json")
    commits = np.frombuffer(b"".join(bytes.fromhex(x) for x in g["commits"]), dtype=np.uint8).copy()
    _lib.check(lib.dgpu_set_group(h, len(g["commits"]), g["n"], _lib.ptr(commits)))
    _lib.check(lib.dgpu_recover_batch(h, 0, None, 8, None, 96, None, None, _lib.ptr(bits), None))
    assert bits.tolist() == [0xAB, 0xAB] and reason.tolist() == [0xCD, 0xCD]
