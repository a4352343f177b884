"""ctypes wrapper of the C restatement (oracle/c -> oracle/build/liboracle_ref.so).
TEST INFRASTRUCTURE: tests/ and bench.py's cpu_baseline leg only."""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "build", "liboracle_ref.so")
_lib = None


def load(build=True):
    global _lib
    if _lib is None:
        if not os.path.exists(SO) and build:
            subprocess.check_call(["make", "-C", os.path.join(_HERE, "c")])
        L = ctypes.CDLL(SO)
        c = ctypes
        L.ref_verify_msg.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t]
        L.ref_verify_beacon.argtypes = [c.c_int, c.c_char_p, c.c_uint64, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t]
        L.ref_hash_to_g2.argtypes = [c.c_char_p, c.c_char_p]
        L.ref_digest.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_uint64, c.c_char_p]
        L.ref_verify_batch.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                       c.c_void_p, c.c_size_t, c.c_void_p, c.c_int, c.c_void_p]
        L.ref_verify_beacon_g1.argtypes = [c.c_int, c.c_char_p, c.c_uint64, c.c_char_p, c.c_size_t]
        L.ref_hash_to_g1.argtypes = [c.c_int, c.c_char_p, c.c_char_p]
        L.ref_verify_batch_g1.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_void_p, c.c_void_p, c.c_size_t,
                                          c.c_void_p, c.c_int, c.c_void_p]
        L.ref_recover.argtypes = [c.c_char_p, c.c_int, c.c_char_p, c.c_char_p, c.c_size_t, c.c_void_p, c.c_int,
                                  c.c_char_p]
        L.ref_recover_batch.argtypes = [c.c_char_p, c.c_int, c.c_size_t, c.c_void_p, c.c_void_p, c.c_size_t,
                                        c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p]
        _lib = L
    return _lib


def verify_beacon(chained, pk48, round_, prev, sig):
    """reason code (0 valid, 1 decode, 2 subgroup, 3 pairing, 4 infinity)"""
    return load().ref_verify_beacon(1 if chained else 0, pk48, round_, prev or b"", len(prev or b""), sig or b"",
                                    len(sig or b""))


def hash_to_g2(msg32):
    out = ctypes.create_string_buffer(96)
    load().ref_hash_to_g2(msg32, out)
    return out.raw


def verify_batch(chained, pk48, rounds, sigs, sig_len, prev, prev_len, threads):
    """numpy arrays (rounds u64 (n,), sigs u8 (n, stride), sig_len u32, prev u8 (n, pstride), prev_len u32)."""
    import numpy as np
    n = len(rounds)
    reason = np.zeros(n, dtype=np.uint8)
    load().ref_verify_batch(1 if chained else 0, pk48, n, rounds.ctypes.data, sigs.ctypes.data, sigs.shape[1],
                            sig_len.ctypes.data, prev.ctypes.data, prev.shape[1], prev_len.ctypes.data, threads,
                            reason.ctypes.data)
    return reason


def verify_beacon_g1(rfc_dst, pk96, round_, sig):
    """G1-signature schemes (unchained): reason code as verify_beacon."""
    return load().ref_verify_beacon_g1(1 if rfc_dst else 0, pk96, round_, sig or b"", len(sig or b""))


def hash_to_g1(rfc_dst, msg32):
    out = ctypes.create_string_buffer(48)
    load().ref_hash_to_g1(1 if rfc_dst else 0, msg32, out)
    return out.raw


def verify_batch_g1(rfc_dst, pk96, rounds, sigs, sig_len, threads):
    import numpy as np
    n = len(rounds)
    reason = np.zeros(n, dtype=np.uint8)
    load().ref_verify_batch_g1(1 if rfc_dst else 0, pk96, n, rounds.ctypes.data, sigs.ctypes.data, sigs.shape[1],
                               sig_len.ctypes.data, threads, reason.ctypes.data)
    return reason


def recover(commits, t, msg32, partials):
    """kyber tbls.Recover + VerifyRecovered (C restatement): 96-byte signature or None."""
    import numpy as np
    m = len(partials)
    stride = max([2] + [len(p) for p in partials])
    buf = np.zeros((max(m, 1), stride), dtype=np.uint8)
    plen = np.zeros(max(m, 1), dtype=np.uint32)
    for i, p in enumerate(partials):
        buf[i, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        plen[i] = len(p)
    out = ctypes.create_string_buffer(96)
    ok = load().ref_recover(b"".join(commits), t, msg32, buf.tobytes(), stride, plen.ctypes.data, m, out)
    return out.raw if ok else None


def recover_batch(commits, t, msgs, partials, threads):
    """msgs (n, 32) u8, partials (n, m, stride) u8 with every slot full; returns (sigs (n, 96), ok (n,))."""
    import numpy as np
    n, m, stride = partials.shape
    parts = np.ascontiguousarray(partials)
    plen = np.full(n * m, stride, dtype=np.uint32)
    out = np.zeros((n, 96), dtype=np.uint8)
    ok = np.zeros(n, dtype=np.uint8)
    load().ref_recover_batch(b"".join(commits), t, n, np.ascontiguousarray(msgs).ctypes.data, parts.ctypes.data, stride,
                             plen.ctypes.data, m, threads, out.ctypes.data, ok.ctypes.data)
    return out, ok.astype(bool)
