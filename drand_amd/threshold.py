"""Threshold recovery (drand's aggregator path) on the GPU through the C-ABI.

Mirrors (names, argument meaning, error behaviour):
  key.Scheme.IndexOf(partial)                    kyber tbls.SigShare.Index (R); node.go:119
  key.Scheme.Recover(pub, msg, sigs, t, n)       kyber tbls.Recover (R); chain/beacon/chain.go:160
and the batch form an aggregator or a catch-up recomputation needs:
  ThresholdGroup.recover_batch(msgs, partials)   one GPU call for many rounds

A share.PubPoly is represented by its t compressed G1 commitments (48 bytes
each, key/keys.go DistPublic.Coefficients).  No CPU fallback: the work runs
in libdrand_gpu.so (dgpu_set_group / dgpu_recover_batch).
"""
import struct
import threading

import numpy as np

from . import _lib
from .chain import get_context


class RecoverError(Exception):
    """The reference's Recover error ("not enough good public shares to
    reconstruct secret commitment")."""


def index_of(partial):
    """key.Scheme.IndexOf: BE16 of the first two bytes; error (-1) if shorter."""
    if len(partial) < 2:
        return -1
    return struct.unpack(">H", partial[:2])[0]


def pack_partials(msgs, partials):
    """Fixed-stride partial records of the C-ABI: (msgs (nr*32,), partials
    (nr, m, stride), partial_len (nr, m), m, stride); empty slots have length 0."""
    nr = len(msgs)
    m = max(1, max(len(p) for p in partials))
    stride = max([98] + [len(s) for p in partials for s in p])
    buf = np.zeros((nr, m, stride), dtype=np.uint8)
    plen = np.zeros((nr, m), dtype=np.uint32)
    for r, plist in enumerate(partials):
        for j, s in enumerate(plist):
            plen[r, j] = len(s)
            if s:
                buf[r, j, :len(s)] = np.frombuffer(s, dtype=np.uint8)
    mb = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    if mb.size != 32 * nr:
        raise ValueError("messages must be 32 bytes (DigestMessage output)")
    return mb, buf, plen, m, stride


def unpack_recovered(out, ok, pv, partials, m):
    nr = len(partials)
    okb = np.unpackbits(ok, bitorder="little")[:nr]
    sigs = [bytes(out[96 * r:96 * (r + 1)]) if okb[r] else None for r in range(nr)]
    if pv is None:
        return sigs, None
    valid = [[bool(pv[r * m + j]) for j in range(len(partials[r]))] for r in range(nr)]
    return sigs, valid


class ThresholdGroup:
    """A group's share.PubPoly installed on one GPU context."""

    _lock = threading.Lock()

    def __init__(self, commits, n, device=0):
        self.commits = [bytes(c) for c in commits]
        self.t = len(self.commits)
        self.n = n
        self.ctx = get_context(device)
        buf = np.frombuffer(b"".join(self.commits), dtype=np.uint8).copy()
        with ThresholdGroup._lock:
            _lib.check(self.ctx.lib.dgpu_set_group(self.ctx.handle, self.t, n, _lib.ptr(buf)))
            ThresholdGroup._active = (id(self.ctx), tuple(self.commits), n)

    def _install(self):
        key = (id(self.ctx), tuple(self.commits), self.n)
        if getattr(ThresholdGroup, "_active", None) != key:
            buf = np.frombuffer(b"".join(self.commits), dtype=np.uint8).copy()
            _lib.check(self.ctx.lib.dgpu_set_group(self.ctx.handle, self.t, self.n, _lib.ptr(buf)))
            ThresholdGroup._active = key

    def recover_batch(self, msgs, partials, statuses=True):
        """msgs: list of 32-byte messages (DigestMessage of each round);
        partials: list (per round) of lists of partial signatures (bytes).
        Returns (sigs, valid): sigs[r] = 96-byte recovered signature or None
        (the reference's error), valid[r][j] = partial j verified.  With
        statuses=False valid is None and the library verifies each round's
        candidates with one batched pairing (recover.cuh)."""
        nr = len(msgs)
        if nr == 0:
            return [], []
        mb, buf, plen, m, stride = pack_partials(msgs, partials)
        out = np.zeros(nr * 96, dtype=np.uint8)
        ok = np.zeros((nr + 7) // 8, dtype=np.uint8)
        pv = np.zeros(nr * m, dtype=np.uint8) if statuses else None
        with ThresholdGroup._lock:
            self._install()
            _lib.check(self.ctx.lib.dgpu_recover_batch(self.ctx.handle, nr, _lib.ptr(mb), m, _lib.ptr(buf), stride,
                                                       _lib.ptr(plen), _lib.ptr(out), _lib.ptr(ok), _lib.ptr(pv)))
        return unpack_recovered(out, ok, pv, partials, m)

    def recover(self, msg, sigs):
        """key.Scheme.Recover(pub, msg, sigs, t, n): the recovered 96-byte
        signature, or RecoverError."""
        out, _ = self.recover_batch([msg], [list(sigs)], statuses=False)
        if out[0] is None:
            raise RecoverError("share: not enough good public shares to reconstruct secret commitment")
        return out[0]
