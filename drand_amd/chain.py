"""Host-side mirror of drand's chain verification surface, backed by the
MI355X kernels through the C-ABI (include/drand_gpu.h).

Mirrors (same names, argument meaning and error behaviour):
  chain.Beacon                      chain/beacon.go:13-20  (+ Randomness :51-54)
  chain.RoundToBytes                chain/store.go:42-46
  chain.NewVerifier / Verifier      chain/verify.go:13-49
      DigestMessage(round, prevSig) chain/verify.go:24-32
      VerifyBeacon(b, pubkey) error chain/verify.go:38-45
      IsPrevSigMeaningful()         chain/verify.go:47-49
and adds the batch form every bulk caller needs (sync_manager.go:188-222,
client/verify.go:149-169): Verifier.verify_beacons(beacons, pubkey).

There is no CPU fallback: every digest and every verification runs on the
GPU; constructing a Verifier without the HIP library or a gfx950 device
raises DrandGPUError.
"""
import hashlib
import secrets
import struct
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib
from .scheme import Scheme, scheme_code


class VerifyError(Exception):
    """Non-nil error of VerifyBeacon; `reason` is the DGPU_REASON_* code."""

    MESSAGES = {
        _lib.REASON_DECODE: "bls: invalid signature encoding",
        _lib.REASON_SUBGROUP: "bls: signature point is not on correct subgroup",
        _lib.REASON_PAIRING: "bls: invalid signature",
        _lib.REASON_INFINITY: "bls: invalid signature",
    }

    def __init__(self, round_, reason):
        super().__init__(f"round {round_}: {self.MESSAGES.get(reason, 'invalid beacon')}")
        self.round = round_
        self.reason = reason


@dataclass
class Beacon:
    """chain/beacon.go:13-20"""
    previous_sig: bytes
    round: int
    signature: bytes

    def randomness(self):
        """chain/beacon.go:43-45 (host bookkeeping, SHA-256 of the signature)."""
        return randomness_from_signature(self.signature)

    def get_round(self):
        return self.round


def round_to_bytes(r):
    """chain/store.go:42-46: 8-byte big-endian."""
    return struct.pack(">Q", r)


def randomness_from_signature(sig):
    """chain/beacon.go:51-54 (not part of the verify hot path)."""
    return hashlib.sha256(sig).digest()


_contexts = {}
_ctx_lock = threading.Lock()


def get_context(device=0):
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = _lib.Context(device)
            _contexts[device] = ctx
        return ctx


def pack_beacons(beacons, sig_stride=96, prev_stride=None):
    """Fixed-stride records for dgpu_verify_batch (numpy arrays)."""
    n = len(beacons)
    if prev_stride is None:
        prev_stride = max([96] + [len(b.previous_sig or b"") for b in beacons])
    rounds = np.fromiter((b.round for b in beacons), dtype=np.uint64, count=n)
    sig_len = np.fromiter((len(b.signature or b"") for b in beacons), dtype=np.uint32, count=n)
    prev_len = np.fromiter((len(b.previous_sig or b"") for b in beacons), dtype=np.uint32, count=n)
    stride = max(sig_stride, 96)
    sigs = np.zeros((n, stride), dtype=np.uint8)
    prev = np.zeros((n, prev_stride), dtype=np.uint8)
    for i, b in enumerate(beacons):
        s = b.signature or b""
        if 0 < len(s) <= stride:
            sigs[i, : len(s)] = np.frombuffer(s, dtype=np.uint8)
        elif len(s) > stride:
            sig_len[i] = 0xFFFFFFFF  # any length != 96 fails decode, like kilic (R)
        p = b.previous_sig or b""
        if p:
            prev[i, : len(p)] = np.frombuffer(p, dtype=np.uint8)
    return rounds, sigs, sig_len, prev, prev_len


def rlc_seed_for(mode, rlc_seed):
    """RLC coefficients must be unpredictable to whoever produced the
    beacons: without an explicit seed, RLC mode draws a fresh 64-bit one per
    call (a known seed lets an attacker choose corruptions that cancel)."""
    if mode == _lib.MODE_RLC and rlc_seed is None:
        return secrets.randbits(64)
    return 0 if rlc_seed is None else int(rlc_seed)


class Verifier:
    """chain.Verifier (chain/verify.go:13-20): stateless apart from the scheme;
    safe for concurrent use (the GPU context serializes).  The public key is
    passed per call, like VerifyBeacon(b, pubkey) (chain/verify.go:38); the
    context caches decoded keys, so verifiers of different chains and schemes
    can share one GPU context."""

    def __init__(self, scheme: Scheme, device=0):
        self.scheme = scheme
        self.ctx = get_context(device)
        self._code = scheme_code(scheme)

    def is_prev_sig_meaningful(self):
        """chain/verify.go:47-49"""
        return not self.scheme.decouple_prev_sig

    def digest_message(self, round_, prev_sig):
        """chain/verify.go:24-32 (computed on the GPU)."""
        return self.digest_messages([round_], [prev_sig])[0]

    def digest_messages(self, rounds, prev_sigs):
        n = len(rounds)
        r = np.asarray(rounds, dtype=np.uint64)
        stride = max([1] + [len(p or b"") for p in prev_sigs])
        prev = np.zeros((n, stride), dtype=np.uint8)
        plen = np.zeros(n, dtype=np.uint32)
        for i, p in enumerate(prev_sigs):
            if p:
                prev[i, : len(p)] = np.frombuffer(p, dtype=np.uint8)
                plen[i] = len(p)
        out = np.zeros((n, 32), dtype=np.uint8)
        lib = self.ctx.lib
        _lib.check(lib.dgpu_digest_batch(self.ctx.handle, self._code, n, _lib.ptr(r), _lib.ptr(prev), stride,
                                         _lib.ptr(plen), _lib.ptr(out)))
        return [bytes(row) for row in out]

    def verify_beacons(self, beacons, pubkey, mode=_lib.MODE_PER_ROUND, rlc_seed=None):
        """Batch VerifyBeacon: returns a list of (None | VerifyError), one per beacon."""
        reasons = self.verify_reasons(beacons, pubkey, mode, rlc_seed)
        return [None if r == _lib.REASON_OK else VerifyError(b.round, int(r)) for b, r in zip(beacons, reasons)]

    def verify_reasons(self, beacons, pubkey, mode=_lib.MODE_PER_ROUND, rlc_seed=None):
        n = len(beacons)
        if n == 0:
            return np.zeros(0, dtype=np.uint8)
        rounds, sigs, sig_len, prev, prev_len = pack_beacons(beacons)
        return self.verify_records(pubkey, rounds, sigs, sig_len, prev, prev_len, mode, rlc_seed)

    def verify_records(self, pubkey, rounds, sigs, sig_len, prev, prev_len, mode=_lib.MODE_PER_ROUND, rlc_seed=None):
        """Fixed-stride host records (numpy, as pack_beacons builds them or
        the native bolt ingest decodes them): DGPU_REASON_* per record."""
        n = len(rounds)
        if n == 0:
            return np.zeros(0, dtype=np.uint8)
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        pk = np.frombuffer(bytes(pubkey), dtype=np.uint8).copy()
        lib = self.ctx.lib
        _lib.check(lib.dgpu_verify_beacons(self.ctx.handle, self._code, _lib.ptr(pk), pk.size, n, _lib.ptr(rounds),
                                           _lib.ptr(sigs), sigs.shape[1], _lib.ptr(sig_len), _lib.ptr(prev),
                                           prev.shape[1], _lib.ptr(prev_len), mode, rlc_seed_for(mode, rlc_seed),
                                           _lib.ptr(bits), _lib.ptr(reason)))
        valid = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
        if not np.array_equal(valid, reason == _lib.REASON_OK):
            raise _lib.DrandGPUError(_lib.DGPU_EINVAL, "verdict bitmap and reasons disagree")
        return reason

    def verify_beacon(self, b: Beacon, pubkey: bytes):
        """chain/verify.go:38-45: raises VerifyError (the reference's non-nil
        error) or returns None."""
        err = self.verify_beacons([b], pubkey)[0]
        if err is not None:
            raise err


def new_verifier(scheme: Scheme, device=0):
    """chain.NewVerifier (chain/verify.go:18-20)."""
    return Verifier(scheme, device)


def _pack_msgs(msgs):
    n = len(msgs)
    stride = max([1] + [len(m) for m in msgs])
    buf = np.zeros((n, stride), dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    for i, m in enumerate(msgs):
        if m:
            buf[i, : len(m)] = np.frombuffer(bytes(m), dtype=np.uint8)
        lens[i] = len(m)
    return buf, lens


def verify_recovered(scheme: Scheme, pubkey, msgs, sigs, mode=_lib.MODE_PER_ROUND, rlc_seed=None, device=0):
    """Batch key.Scheme.VerifyRecovered(pk, msg, sig) (chain/verify.go:44,
    chain/beacon/chain.go:165; kyber bls.Verify (R)) over raw messages of any
    length.  Returns the DGPU_REASON_* code per message (0 = valid)."""
    ctx = get_context(device)
    n = len(msgs)
    if n == 0:
        return np.zeros(0, dtype=np.uint8)
    mb, ml = _pack_msgs(msgs)
    sb, sl = _pack_msgs(sigs)
    width = 48 if scheme_code(scheme) in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380) else 96
    if sb.shape[1] < width:
        sb = np.pad(sb, ((0, 0), (0, width - sb.shape[1])))
    pk = np.frombuffer(bytes(pubkey), dtype=np.uint8).copy()
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    reason = np.zeros(n, dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_verify_recovered(ctx.handle, scheme_code(scheme), _lib.ptr(pk), pk.size, n, _lib.ptr(mb),
                                             mb.shape[1], _lib.ptr(ml), _lib.ptr(sb), sb.shape[1], _lib.ptr(sl), mode,
                                             rlc_seed_for(mode, rlc_seed), _lib.ptr(bits), _lib.ptr(reason)))
    return reason


def hash_to_curve(msgs, scheme: Scheme = None, device=0):
    """Hash raw messages of any length to the scheme's signature group
    (compressed: 96-byte G2 under drand's DST, 48-byte G1 for the G1 schemes)."""
    from .scheme import get_scheme_by_id_with_default
    code = scheme_code(scheme or get_scheme_by_id_with_default(""))
    ctx = get_context(device)
    n = len(msgs)
    mb, ml = _pack_msgs(msgs)
    width = 48 if code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380) else 96
    out = np.zeros(n * width, dtype=np.uint8)
    if n:
        _lib.check(ctx.lib.dgpu_hash_to_curve(ctx.handle, code, n, _lib.ptr(mb), mb.shape[1], _lib.ptr(ml),
                                              _lib.ptr(out)))
    return [bytes(out[i * width:(i + 1) * width]) for i in range(n)]


def sign(secret, msgs, scheme: Scheme = None, device=0):
    """key.Scheme.Sign / AuthScheme.Sign (key/curve.go:36-39) of raw messages
    with a secret scalar (int or 32 big-endian bytes): test/tool surface."""
    from .scheme import get_scheme_by_id_with_default
    code = scheme_code(scheme or get_scheme_by_id_with_default(""))
    ctx = get_context(device)
    sk = secret.to_bytes(32, "big") if isinstance(secret, int) else bytes(secret)
    skb = np.frombuffer(sk, dtype=np.uint8).copy()
    n = len(msgs)
    mb, ml = _pack_msgs(msgs)
    width = 48 if code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380) else 96
    out = np.zeros(n * width, dtype=np.uint8)
    if n:
        _lib.check(ctx.lib.dgpu_sign(ctx.handle, code, _lib.ptr(skb), n, _lib.ptr(mb), mb.shape[1], _lib.ptr(ml),
                                     _lib.ptr(out)))
    return [bytes(out[i * width:(i + 1) * width]) for i in range(n)]


def decode_g1_points(points, device=0):
    """Batch G1 decode (KeyGroup.Point().UnmarshalBinary, chain/convert.go:20-23):
    returns (rc list, [(x, y) ints or None])."""
    ctx = get_context(device)
    n = len(points)
    buf = np.frombuffer(b"".join(bytes(p) for p in points), dtype=np.uint8).copy()
    rc = np.zeros(n, dtype=np.int32)
    xy = np.zeros(n * 96, dtype=np.uint8)
    if n:
        _lib.check(ctx.lib.dgpu_decode_g1_points(ctx.handle, n, _lib.ptr(buf), _lib.ptr(rc), _lib.ptr(xy)))
    coords = [(int.from_bytes(bytes(xy[i * 96:i * 96 + 48]), "big"), int.from_bytes(bytes(xy[i * 96 + 48:i * 96 + 96]), "big"))
              if rc[i] == 0 else None for i in range(n)]
    return rc.tolist(), coords


def _be_coords(xy, k):
    return tuple(int.from_bytes(bytes(xy[48 * j:48 * j + 48]), "big") for j in range(k))


def decode_signatures(scheme, sigs, device=0):
    """The scheme's signature decoder (the UnmarshalBinary inside bls.Verify,
    chain/verify.go:44): returns (reasons, points) with points[i] = (x, y)
    ints on G1 or ((x0, x1), (y0, y1)) on G2 for decoded records, else None."""
    ctx = get_context(device)
    code = scheme_code(scheme)
    n = len(sigs)
    g1 = code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)
    stride = max([96] + [len(s) for s in sigs])
    buf = np.zeros((max(n, 1), stride), dtype=np.uint8)
    ln = np.zeros(max(n, 1), dtype=np.uint32)
    for i, s in enumerate(sigs):
        buf[i, :len(s)] = np.frombuffer(bytes(s), dtype=np.uint8)
        ln[i] = len(s)
    w = 96 if g1 else 192
    reason = np.zeros(max(n, 1), dtype=np.uint8)
    xy = np.zeros(max(n, 1) * w, dtype=np.uint8)
    if n:
        _lib.check(ctx.lib.dgpu_decode_signatures(ctx.handle, code, n, _lib.ptr(buf), stride, _lib.ptr(ln),
                                                  _lib.ptr(reason), _lib.ptr(xy)))
    pts = []
    for i in range(n):
        if reason[i] != _lib.REASON_OK:
            pts.append(None)
            continue
        c = _be_coords(xy[i * w:(i + 1) * w], w // 48)
        pts.append(c if g1 else ((c[0], c[1]), (c[2], c[3])))
    return reason[:n].tolist(), pts


def decode_pubkey(scheme, pk, device=0):
    """The scheme's public-key decoder (chain/convert.go:20-23): the affine key
    point ((x, y) on G1, ((x0, x1), (y0, y1)) on G2); raises DrandGPUError
    (DGPU_EINVAL) when the key is rejected."""
    ctx = get_context(device)
    code = scheme_code(scheme)
    b = np.frombuffer(bytes(pk), dtype=np.uint8).copy()
    g2 = code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)
    xy = np.zeros(192, dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_decode_pubkey(ctx.handle, code, _lib.ptr(b), len(pk), _lib.ptr(xy)))
    c = _be_coords(xy, 4 if g2 else 2)
    return ((c[0], c[1]), (c[2], c[3])) if g2 else c


def hash_to_g2(msgs, device=0):
    """kyber G2 Hash (R) of 32-byte messages -> 96-byte compressed points (parity surface)."""
    ctx = get_context(device)
    n = len(msgs)
    m = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    out = np.zeros(n * 96, dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_hash_to_g2(ctx.handle, n, _lib.ptr(m), _lib.ptr(out)))
    return [bytes(out[i * 96:(i + 1) * 96]) for i in range(n)]


def hash_to_g1(msgs, scheme_code_=None, device=0):
    """Hash to G1 (RFC 9380 G1 suite) of 32-byte messages under a G1-signature
    scheme's DST -> 48-byte compressed points (parity surface)."""
    ctx = get_context(device)
    n = len(msgs)
    m = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    out = np.zeros(n * 48, dtype=np.uint8)
    code = _lib.SCHEME_UNCHAINED_G1 if scheme_code_ is None else scheme_code_
    _lib.check(ctx.lib.dgpu_hash_to_g1(ctx.handle, code, n, _lib.ptr(m), _lib.ptr(out)))
    return [bytes(out[i * 48:(i + 1) * 48]) for i in range(n)]
