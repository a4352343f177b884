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
SCHEME_G1_RFC9380 = "bls-unchained-g1-rfc9380"
DECOUPLE_PREV_SIG = {SCHEME_CHAINED: False, SCHEME_UNCHAINED: True, SCHEME_UNCHAINED_G1: True,
                     SCHEME_G1_RFC9380: True}
# Signatures on G1 (public key on G2): the hash-to-G1 domain separation tag.
# bls-unchained-on-g1 hashes to G1 under the G2 suite's DST (upstream drand's
# historical choice (R); the scheme is absent from this snapshot, SURVEY.md
# section 8c: unpinned); bls-unchained-g1-rfc9380 uses the RFC 9380 G1 DST.
SIG_ON_G1_DST = {SCHEME_UNCHAINED_G1: B.DST_G2, SCHEME_G1_RFC9380: B.DST_G1}


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
    msg = digest_message(scheme_id, round_, prev_sig)
    if scheme_id in SIG_ON_G1_DST:  # pk_point on G2, sig on G1
        return B.verify_g1(pk_point, msg, sig, SIG_ON_G1_DST[scheme_id])
    return B.verify_g2(pk_point, msg, sig)


# reason codes shared with include/drand_gpu.h (DGPU_REASON_*)
REASON_OK, REASON_DECODE, REASON_SUBGROUP, REASON_PAIRING, REASON_INFINITY = 0, 1, 2, 3, 4


def verify_reason(scheme_id, pk_point, round_, prev_sig, sig):
    """Like verify_beacon, but says why: the kyber error class (R)."""
    msg = digest_message(scheme_id, round_, prev_sig)
    on_g1 = scheme_id in SIG_ON_G1_DST
    try:
        s = B.g1_decompress(sig) if on_g1 else B.g2_decompress(sig)
    except B.DecodeError as e:
        return REASON_SUBGROUP if "subgroup" in str(e) else REASON_DECODE
    if s is None:
        return REASON_INFINITY
    if on_g1:
        hm = B.hash_to_g1(msg, SIG_ON_G1_DST[scheme_id])
        ok = B.pairing_check([(hm, pk_point), (B.g1_neg(s), B.G2_GEN)])
    else:
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
    on_g1 = scheme_id in SIG_ON_G1_DST
    pk = B.sk_to_pk_g2(sk) if on_g1 else B.sk_to_pk(sk)
    prev = derive_genesis(seed) if prev is None else prev
    out = []
    for i in range(n):
        rnd = start_round + i
        msg = digest_message(scheme_id, rnd, prev)
        sig = B.sign_g1(sk, msg, SIG_ON_G1_DST[scheme_id]) if on_g1 else B.sign_g2(sk, msg)
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


# ------------------------------------------------------------- threshold BLS (kyber share / sign/tbls (R))
# The reference's threshold path lives in kyber v1.1.10 (go.mod:9), absent
# from /root/reference; restated from its published algorithm and pinned by
# the reference's own round trip chain/beacon/node_test.go:88-105 (sign with
# shares, Recover, VerifyRecovered against the group key): the recovered
# signature equals sk * H(msg), the signature of the group secret.

def share_poly(seed, t):
    """Degree t-1 polynomial over Fr: a_0 = sk (derive_secret), a_j from seed
    (coefficients from s0)."""
    coeffs = [derive_secret(seed)]
    for j in range(1, t):
        d = hashlib.sha256(b"drand-mi355x/poly/" + struct.pack("<QQ", seed, j)).digest()
        coeffs.append(int.from_bytes(d, "big") % B.R)
    return coeffs


def poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % B.R
    return acc


def pub_poly_commits(coeffs):
    """share.PubPoly commitments: C_j = a_j * g1 (48-byte compressed each)."""
    return [B.g1_compress(B.g1_mul(B.G1_GEN, a)) for a in coeffs]


def pub_poly_eval(commit_points, i):
    """PubPoly.Eval(i): sum_j C_j (i+1)^j (x_i = i + 1, kyber share/poly.go (R))."""
    x = i + 1
    acc = None
    for c in reversed(commit_points):
        acc = B.g1_add(B.g1_mul(acc, x) if acc is not None else None, c)
    return acc


def partial_sign(share_index, share_value, msg):
    """tbls.Sign (R): BE16(index) || bls.Sign(share, msg)."""
    return struct.pack(">H", share_index) + B.sign_g2(share_value, msg)


def lagrange_at_zero(xs):
    """Lagrange basis at 0 over Fr for distinct points xs."""
    out = []
    for j, xj in enumerate(xs):
        num, den = 1, 1
        for m, xm in enumerate(xs):
            if m == j:
                continue
            num = num * xm % B.R
            den = den * (xm - xj) % B.R
        out.append(num * pow(den, B.R - 2, B.R) % B.R)
    return out


def recover(commit_points, msg, partials, t, n, verify=None):
    """kyber tbls.Recover (R), sign/tbls/tbls.go: walk the partials in order,
    skip those whose index cannot be read or that fail Verify against
    PubPoly.Eval(index) (which decodes the signature), stop after t good
    ones; then share.RecoverCommit: sort by index, keep the first of each
    index up to t distinct (xyCommit), fail with fewer than t, Lagrange
    interpolation at 0 with x_i = i + 1.  Returns the 96-byte recovered
    signature or None (the reference's error).  `verify(i, sig)` may replace
    the pairing check (tests that already know the verdicts)."""
    good = []
    for s in partials:
        if len(s) < 2:
            continue
        idx = struct.unpack(">H", s[:2])[0]
        sig = s[2:]
        if verify is not None:
            ok = verify(idx, sig)
        else:
            ok = B.verify_g2(pub_poly_eval(commit_points, idx), msg, sig)
        if not ok:
            continue
        good.append((idx, B.g2_decompress(sig)))
        if len(good) >= t:
            break
    good.sort(key=lambda p: p[0])
    xs, ys = {}, {}
    for idx, pt in good:
        xs[idx] = idx + 1
        ys[idx] = pt
        if len(xs) == t:
            break
    if len(xs) < t:
        return None
    order = sorted(xs)
    lam = lagrange_at_zero([xs[i] for i in order])
    acc = None
    for i, l in zip(order, lam):
        acc = B.g2_add(acc, B.g2_mul(ys[i], l))
    return B.g2_compress(acc)


# ------------------------------------------------------------- streaming sync / client walk (sequential)
def try_node(packets, verify, put, up_to, beacon_id=None):
    """chain/beacon/sync_manager.go:370-424 restated: one packet at a time.
    packets: iterable of (beacon, beacon_id | None); verify(beacon) -> bool;
    put(beacon) may raise.  Returns (ok, last_stored)."""
    last = None
    for b, bid in packets:
        if bid is not None and beacon_id is not None and bid != beacon_id:  # :378-381
            return False, last
        if not verify(b):  # :394-397
            return False, last
        try:
            put(b)  # :399-410
        except Exception:
            return False, last
        last = b
        if last[0] == up_to:  # :417-420
            return True, last
    return False, last  # :372-375 channel closed


def trusted_previous_signature(verify, get_signature, genesis_seed, round_, point_of_trust=None):
    """client/verify.go:118-178 restated: returns (prev_sig, point_of_trust)
    or raises ValueError("verifying beacon") at the first invalid beacon.
    verify(round, prev, sig) -> bool."""
    if round_ == 1:
        return genesis_seed, point_of_trust
    if point_of_trust is None or point_of_trust[0] > round_:
        trust_round, trust_sig = 1, genesis_seed
    else:
        trust_round, trust_sig = point_of_trust
    initial = trust_round
    nxt = None
    while trust_round < round_ - 1:
        trust_round += 1
        sig = get_signature(trust_round)
        if not verify(trust_round, trust_sig, sig):
            raise ValueError(f"verifying beacon {trust_round}")
        trust_sig = sig
        nxt = (trust_round, sig)
    if trust_round == round_ - 1 and trust_round > initial:
        point_of_trust = nxt
    return trust_sig, point_of_trust
