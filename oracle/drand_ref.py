"""CPU restatement of drand's beacon-verification semantics (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  Each function cites the reference line
it restates (paths relative to the reference repo root).
"""

import hashlib
import struct

from . import bls12381 as B

# common/scheme/scheme.go:9,12 (+ the scheme this build adds)
SCHEME_CHAINED = "pedersen-bls-chained"
SCHEME_UNCHAINED = "pedersen-bls-unchained"
SCHEME_UNCHAINED_G1 = "bls-unchained-on-g1"
DECOUPLE_PREV_SIG = {SCHEME_CHAINED: False, SCHEME_UNCHAINED: True, SCHEME_UNCHAINED_G1: True}


def round_to_bytes(r):
    """chain/store.go:42-46: 8-byte big-endian round."""
    return struct.pack(">Q", r)


def digest_message(scheme_id, round_, prev_sig):
    """chain/verify.go:24-32: SHA-256(prevSig || BE64(round)) for chained,
    SHA-256(BE64(round)) when the scheme decouples the previous signature."""
    h = hashlib.sha256()
    if not DECOUPLE_PREV_SIG[scheme_id]:
        h.update(prev_sig or b"")
    h.update(round_to_bytes(round_))
    return h.digest()


def randomness_from_signature(sig):
    """chain/beacon.go:51-54"""
    return hashlib.sha256(sig).digest()


def verify_beacon(scheme_id, pk_point, round_, prev_sig, sig):
    """chain/verify.go:38-45 -> key.Scheme.VerifyRecovered (kyber tbls ->
    bls.Verify (R)).  Returns True iff the reference would return nil."""
    if scheme_id == SCHEME_UNCHAINED_G1:
        raise NotImplementedError("bls-unchained-on-g1 oracle not built yet")
    msg = digest_message(scheme_id, round_, prev_sig)
    return B.verify_g2(pk_point, msg, sig)


# reason codes shared with include/drand_gpu.h (DGPU_REASON_*)
REASON_OK, REASON_DECODE, REASON_SUBGROUP, REASON_PAIRING, REASON_INFINITY = 0, 1, 2, 3, 4


def verify_reason(scheme_id, pk_point, round_, prev_sig, sig):
    """Like verify_beacon, but says why: the kyber error class (R)."""
    msg = digest_message(scheme_id, round_, prev_sig)
    try:
        s = B.g2_decompress(sig)
    except B.DecodeError as e:
        return REASON_SUBGROUP if "subgroup" in str(e) else REASON_DECODE
    if s is None:
        return REASON_INFINITY
    hm = B.hash_to_g2(msg)
    ok = B.pairing_check([(pk_point, hm), (B.g1_neg(B.G1_GEN), s)])
    return REASON_OK if ok else REASON_PAIRING


# ------------------------------------------------------------- synthetic chains
def derive_secret(seed):
    """sk = OS2IP(SHA-256("drand-mi355x/sk/" || LE64(s0))) mod r."""
    d = hashlib.sha256(b"drand-mi355x/sk/" + struct.pack("<Q", seed)).digest()
    return int.from_bytes(d, "big") % B.R


def derive_genesis(seed):
    """genesis seed = SHA-256("drand-mi355x/genesis/" || LE64(s0))."""
    return hashlib.sha256(b"drand-mi355x/genesis/" + struct.pack("<Q", seed)).digest()


def make_chain(seed, n, scheme_id=SCHEME_CHAINED, start_round=1, prev=None):
    """Synthetic chain following client/test/result/mock/result.go:86-130
    (msg per DigestMessage, sig = sk * H(msg), previous = sig).  Returns
    (pk_bytes, [(round, prev_sig, sig)]).  For unchained schemes the stored
    PreviousSig is nil (chain/beacon/store.go:82-83)."""
    sk = derive_secret(seed)
    pk = B.sk_to_pk(sk)
    prev = derive_genesis(seed) if prev is None else prev
    out = []
    for i in range(n):
        rnd = start_round + i
        msg = digest_message(scheme_id, rnd, prev)
        sig = B.sign_g2(sk, msg)
        stored_prev = prev if not DECOUPLE_PREV_SIG[scheme_id] else b""
        out.append((rnd, stored_prev, sig))
        prev = sig
    return pk, out


def check_past_beacons(store, up_to, verify):
    """chain/beacon/sync_manager.go:171-232 restated.  `store` maps round ->
    (round, prev, sig) and includes round 0 (genesis) in its length; `verify`
    is a callable on one stored beacon.  Returns (faulty_rounds or None,
    progress_calls)."""
    if not store:
        raise ValueError("empty store")
    last = store[max(store)][0]  # store.Last() (bolt: value under the largest key), its Round field
    if last < up_to:  # :180-184
        up_to = last
    faulty = []
    progress = []
    length = len(store)
    i = 1
    while i < length:  # :188
        progress.append((i, up_to))  # :198-200
        b = store.get(i)
        if b is None:  # :202-210
            faulty.append(i)
            if i >= up_to:
                break
            i += 1
            continue
        if not verify(b):  # :212-214
            faulty.append(b[0])
        if i >= up_to:  # :219-221
            break
        i += 1
    return (faulty if faulty else None), progress
