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
