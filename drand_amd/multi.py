"""Multi-GPU verification through the C ABI (dgpu_multi_open /
dgpu_verify_multi, include/drand_gpu.h): one process drives every GPU of a
node, as a Go caller of the crypto/gpu package would.
Rounds shard contiguously across the devices; RCCL over xGMI gathers only
the per-device verdict bitmaps (and, in RLC mode, the per-device RLC roots,
checked once).  Verdicts equal chain.Verifier's on the same beacons.

The one-process-per-GPU form (torch.distributed ranks, bench.py) lives in
drand_amd/dist.py; both shard with the same contiguous rule."""
import numpy as np

from . import _lib
from .chain import pack_beacons, rlc_seed_for
from .scheme import Scheme, scheme_code
from .threshold import pack_partials, unpack_recovered


class MultiVerifier:
    """chain.Verifier's batch surface over several GPUs (one dgpu_multi handle)."""

    def __init__(self, scheme: Scheme, devices=None, mctx=None):
        self.scheme = scheme
        self._code = scheme_code(scheme)
        self.mctx = mctx if mctx is not None else _lib.MultiContext(devices)

    def close(self):
        self.mctx.close()

    def verify_reasons(self, beacons, pubkey, mode=_lib.MODE_PER_ROUND, rlc_seed=None):
        n = len(beacons)
        if n == 0:
            return np.zeros(0, dtype=np.uint8)
        rounds, sigs, sig_len, prev, prev_len = pack_beacons(beacons)
        return self.verify_records(pubkey, rounds, sigs, sig_len, prev, prev_len, mode, rlc_seed)

    def verify_records(self, pubkey, rounds, sigs, sig_len, prev, prev_len, mode=_lib.MODE_PER_ROUND, rlc_seed=None):
        """Fixed-stride host records (numpy, as chain.pack_beacons builds)."""
        n = len(rounds)
        bits = np.zeros((n + 7) // 8, dtype=np.uint8)
        reason = np.zeros(n, dtype=np.uint8)
        pk = np.frombuffer(bytes(pubkey), dtype=np.uint8).copy()
        lib = self.mctx.lib
        _lib.check(lib.dgpu_verify_multi(self.mctx.handle, self._code, _lib.ptr(pk), pk.size, n, _lib.ptr(rounds),
                                         _lib.ptr(sigs), sigs.shape[1], _lib.ptr(sig_len), _lib.ptr(prev),
                                         prev.shape[1], _lib.ptr(prev_len), mode, rlc_seed_for(mode, rlc_seed),
                                         _lib.ptr(bits), _lib.ptr(reason)))
        valid = np.unpackbits(bits, bitorder="little")[:n].astype(bool)
        if not np.array_equal(valid, reason == _lib.REASON_OK):
            raise _lib.DrandGPUError(_lib.DGPU_EINVAL, "verdict bitmap and reasons disagree")
        return reason


class MultiThresholdGroup:
    """ThresholdGroup's batch recovery over several GPUs (dgpu_multi_set_group
    + dgpu_recover_multi): rounds shard contiguously across the devices."""

    def __init__(self, commits, n, devices=None, mctx=None):
        self.commits = [bytes(c) for c in commits]
        self.t, self.n = len(self.commits), n
        self.mctx = mctx if mctx is not None else _lib.MultiContext(devices)
        buf = np.frombuffer(b"".join(self.commits), dtype=np.uint8).copy()
        _lib.check(self.mctx.lib.dgpu_multi_set_group(self.mctx.handle, self.t, n, _lib.ptr(buf)))

    def close(self):
        self.mctx.close()

    def recover_batch(self, msgs, partials, statuses=True):
        """As ThresholdGroup.recover_batch: (sigs or None per round, per-partial validity or None)."""
        nr = len(msgs)
        if nr == 0:
            return [], []
        mb, buf, plen, m, stride = pack_partials(msgs, partials)
        return self.recover_records(mb, buf, plen, partials, statuses)

    def recover_records(self, mb, buf, plen, partials=None, statuses=False):
        nr, m, stride = buf.shape
        out = np.zeros(nr * 96, dtype=np.uint8)
        ok = np.zeros((nr + 7) // 8, dtype=np.uint8)
        pv = np.zeros(nr * m, dtype=np.uint8) if statuses else None
        _lib.check(self.mctx.lib.dgpu_recover_multi(self.mctx.handle, nr, _lib.ptr(mb), m, _lib.ptr(buf), stride,
                                                    _lib.ptr(plen), _lib.ptr(out), _lib.ptr(ok), _lib.ptr(pv)))
        if partials is None:
            partials = [[b"x"] * m for _ in range(nr)]
        return unpack_recovered(out, ok, pv, partials, m)
