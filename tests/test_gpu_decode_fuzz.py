"""Randomized signature encodings through the whole verify path: per-round
reasons from the GPU equal the C restatement's (oracle/c, test
infrastructure) record by record.  Signatures of a generated chain are
replaced by
  * uniformly random bytes (flag combinations, lengths 0..97),
  * compressed points with the compression flag, a random sign bit and a
    random x < p (about half on the curve, then almost surely outside the
    subgroup),
  * infinity encodings, clean and with stray bits,
  * single bit flips of the valid signature,
for G2 signatures (chained) and G1 signatures (bls-unchained-on-g1), in
per-round and RLC mode.  x >= p is left out: kilic's rule for it is
unpinned.  Marked gpu."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def _mutate(c, rng, width):
    """Overwrite 90% of the signatures (stride `width`) with random encodings; returns the kind per row."""
    n = len(c)
    kinds = rng.integers(0, 5, size=n)
    kinds[rng.random(n) < 0.1] = 5  # kept valid
    for i in range(n):
        k = int(kinds[i])
        if k == 0:  # random bytes, random length
            ln = int(rng.integers(0, width + 2))
            c.sigs[i] = 0
            c.sigs[i, :min(ln, width)] = rng.integers(0, 256, size=min(ln, width), dtype=np.uint8)
            c.sig_len[i] = ln
        elif k in (1, 2):  # compressed, random x < p
            xs = [int.from_bytes(rng.bytes(48), "big") % P for _ in range(width // 48)]
            b = bytearray(b"".join(x.to_bytes(48, "big") for x in xs))
            b[0] |= 0x80 | (0x20 if k == 2 else 0)
            c.sigs[i] = np.frombuffer(bytes(b), dtype=np.uint8)
            c.sig_len[i] = width
        elif k == 3:  # infinity, clean or with a stray bit
            b = bytearray(width)
            b[0] = 0xC0
            if rng.random() < 0.5:
                b[int(rng.integers(0, width))] |= 1 << int(rng.integers(0, 8))
            c.sigs[i] = np.frombuffer(bytes(b), dtype=np.uint8)
            c.sig_len[i] = width
        elif k == 4:  # one bit flipped in the valid signature
            j = int(rng.integers(0, width * 8))
            c.sigs[i, j // 8] ^= np.uint8(1 << (j % 8))
    return kinds


def _gpu_reasons(code, c, mode):
    from drand_amd import _lib
    from drand_amd.chain import get_context
    ctx = get_context(0)
    n = len(c)
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    reason = np.zeros(n, dtype=np.uint8)
    pk = np.frombuffer(c.pk, dtype=np.uint8).copy()
    _lib.check(ctx.lib.dgpu_verify_beacons(ctx.handle, code, _lib.ptr(pk), pk.size, n, _lib.ptr(c.rounds),
                                           _lib.ptr(c.sigs), c.sigs.shape[1], _lib.ptr(c.sig_len), _lib.ptr(c.prev),
                                           c.prev.shape[1], _lib.ptr(c.prev_len), mode, 0xFACE, _lib.ptr(bits),
                                           _lib.ptr(reason)))
    assert np.array_equal(np.unpackbits(bits, bitorder="little")[:n].astype(bool), reason == 0)
    return reason


@pytest.mark.parametrize("code_name", ["SCHEME_CHAINED", "SCHEME_UNCHAINED_G1"])
def test_random_encodings_reasons_equal_c_restatement(code_name):
    from drand_amd import _lib
    from drand_amd.synth import make_chain
    from oracle import c_ref
    code = getattr(_lib, code_name)
    c = make_chain(5150, 3000, code, seg_len=64)
    width = c.sigs.shape[1]
    kinds = _mutate(c, np.random.default_rng(5150 + code), width)
    threads = min(16, os.cpu_count() or 1)
    if code == _lib.SCHEME_CHAINED:
        ref = c_ref.verify_batch(True, c.pk, c.rounds, c.sigs, c.sig_len, c.prev, c.prev_len, threads)
    else:
        ref = c_ref.verify_batch_g1(False, c.pk, c.rounds, c.sigs, c.sig_len, threads)
    per = _gpu_reasons(code, c, _lib.MODE_PER_ROUND)
    bad = np.nonzero(per != ref)[0]
    assert bad.size == 0, [(int(i), int(kinds[i]), int(per[i]), int(ref[i]), bytes(c.sigs[i]).hex()) for i in bad[:5]]
    # every class occurs (the identity: REASON_INFINITY for G2 signatures; a
    # G1 signature at infinity fails its pairing, as in the restatement), the
    # valid rows stay valid and no infinity encoding passes
    classes = {0, _lib.REASON_DECODE, _lib.REASON_SUBGROUP}
    classes |= {_lib.REASON_INFINITY} if code == _lib.SCHEME_CHAINED else {_lib.REASON_PAIRING}
    assert set(np.unique(ref).tolist()) >= classes
    assert (per[kinds == 5] == 0).all() and (per[kinds == 3] != 0).all()
    rlc = _gpu_reasons(code, c, _lib.MODE_RLC)
    assert rlc.tolist() == per.tolist()
