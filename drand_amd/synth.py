"""Deterministic synthetic drand chains, generated on
the GPU through the C-ABI (dgpu_derive_pubkey / dgpu_make_chain), following the
reference's fixture generator client/test/result/mock/result.go:86-130.

A chain of n rounds is built as `n_seg` independently signed segments of
`seg_len` rounds: inside a segment PreviousSig is the previous round's
signature (real linkage); the first round of segment 0 links to the genesis
seed and the first round of every other segment links to a 32-byte
seed-derived value instead of the previous segment's last signature (the
chain is serial, so a single segment of 1M rounds would take ~1M dependent
signing steps).  VerifyBeacon hashes PreviousSig as opaque bytes
(chain/verify.go:24-32), so every round costs the verifier exactly what a
fully linked chain's round costs.
"""
import hashlib
import struct

import numpy as np

from . import _lib
from .chain import get_context

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def derive_secret(seed):
    """sk = OS2IP(SHA-256("drand-mi355x/sk/" || LE64(s0))) mod r."""
    d = hashlib.sha256(b"drand-mi355x/sk/" + struct.pack("<Q", seed)).digest()
    return int.from_bytes(d, "big") % R_ORDER


def derive_genesis(seed):
    """genesis = SHA-256("drand-mi355x/genesis/" || LE64(s0))."""
    return hashlib.sha256(b"drand-mi355x/genesis/" + struct.pack("<Q", seed)).digest()


def segment_seed(seed, s):
    if s == 0:
        return derive_genesis(seed)
    return hashlib.sha256(b"drand-mi355x/segment/" + struct.pack("<QQ", seed, s)).digest()


class Chain:
    """Structure-of-arrays chain: rounds (n,), sigs (n, 96), prev (n, 96), prev_len (n,)."""

    def __init__(self, scheme_code, pk, rounds, sigs, sig_len, prev, prev_len, genesis):
        self.scheme_code = scheme_code
        self.pk = pk
        self.rounds = rounds
        self.sigs = sigs
        self.sig_len = sig_len
        self.prev = prev
        self.prev_len = prev_len
        self.genesis = genesis

    def __len__(self):
        return len(self.rounds)

    def beacon(self, i):
        from .chain import Beacon
        return Beacon(bytes(self.prev[i, : self.prev_len[i]]), int(self.rounds[i]),
                      bytes(self.sigs[i, : self.sig_len[i]]))


def make_chain(seed, n, scheme_code=_lib.SCHEME_CHAINED, seg_len=64, device=0, start_round=1, sk=None):
    """n rounds starting at `start_round`, in segments of `seg_len` rounds;
    signed with derive_secret(seed), or with the secret `sk` when given."""
    ctx = get_context(device)
    lib = ctx.lib
    sk = (derive_secret(seed) if sk is None else sk).to_bytes(32, "big")
    on_g1 = scheme_code in (_lib.SCHEME_UNCHAINED_G1, _lib.SCHEME_G1_RFC9380)
    pk = np.zeros(96 if on_g1 else 48, dtype=np.uint8)
    skb = np.frombuffer(sk, dtype=np.uint8).copy()
    _lib.check(lib.dgpu_derive_pubkey(ctx.handle, scheme_code, _lib.ptr(skb), _lib.ptr(pk), pk.size))
    seg_len = max(1, min(seg_len, n))
    n_seg = (n + seg_len - 1) // seg_len
    first = (start_round + np.arange(n_seg, dtype=np.uint64) * seg_len).astype(np.uint64)
    seeds = np.zeros((n_seg, 96), dtype=np.uint8)
    seed_len = np.full(n_seg, 32, dtype=np.uint32)
    for s in range(n_seg):
        seeds[s, :32] = np.frombuffer(segment_seed(seed, s + (start_round - 1) // seg_len), dtype=np.uint8)
    out = np.zeros((n_seg * seg_len, 96), dtype=np.uint8)
    _lib.check(lib.dgpu_make_chain(ctx.handle, scheme_code, _lib.ptr(skb), n_seg, seg_len, _lib.ptr(first),
                                   _lib.ptr(seeds), _lib.ptr(seed_len), _lib.ptr(out)))
    out = out[:n]
    rounds = (start_round + np.arange(n, dtype=np.uint64)).astype(np.uint64)
    prev = np.zeros((n, 96), dtype=np.uint8)
    prev_len = np.zeros(n, dtype=np.uint32)
    if scheme_code == _lib.SCHEME_CHAINED:
        prev[1:] = out[:-1]
        prev_len[:] = 96
        starts = np.arange(0, n, seg_len)
        prev[starts] = seeds[: len(starts)]
        prev_len[starts] = 32
    sig_len = np.full(n, 48 if on_g1 else 96, dtype=np.uint32)
    return Chain(scheme_code, bytes(pk), rounds, out.copy(), sig_len, prev, prev_len, derive_genesis(seed))


# ---------------------------------------------------------------- corruption catalog
CORRUPT_X_BIT = 1        # (i) bit flip in x -> off curve / off subgroup -> decode failure
CORRUPT_Y_SIGN = 2       # (ii) y-sign flipped (valid point -sigma) -> pairing failure
CORRUPT_OTHER_ROUND = 3  # (iii) signature of another round -> pairing failure
CORRUPT_PREV = 4         # (iv) PreviousSig altered (chained) -> pairing failure
CORRUPT_INFINITY = 5     # (v) canonical infinity -> failure
CORRUPT_TRUNCATED = 6    # (vi) empty / truncated signature -> decode failure
ALL_CORRUPTIONS = (CORRUPT_X_BIT, CORRUPT_Y_SIGN, CORRUPT_OTHER_ROUND, CORRUPT_PREV, CORRUPT_INFINITY,
                   CORRUPT_TRUNCATED)


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x, z ^ (z >> 31)


def corrupt(chain, seed, rate=1e-3, kinds=ALL_CORRUPTIONS):
    """Corrupt ~rate*n rounds in place (at least one of each kind).  Returns
    {index: kind}; every other round is valid by construction."""
    n = len(chain)
    count = max(len(kinds), int(round(n * rate)))
    state = (seed ^ 0xC0FFEE) & 0xFFFFFFFFFFFFFFFF
    chosen = {}
    chained = chain.scheme_code == _lib.SCHEME_CHAINED
    k = 0
    while len(chosen) < min(count, n):
        state, r = splitmix64(state)
        i = r % n
        if i in chosen:
            continue
        kind = kinds[k % len(kinds)]
        k += 1
        if kind == CORRUPT_PREV and not chained:
            kind = CORRUPT_Y_SIGN
        if kind == CORRUPT_OTHER_ROUND and n < 2:
            kind = CORRUPT_Y_SIGN
        chosen[int(i)] = kind
    for i, kind in chosen.items():
        if kind == CORRUPT_X_BIT:
            chain.sigs[i, 47] ^= 0x01
        elif kind == CORRUPT_Y_SIGN:
            chain.sigs[i, 0] ^= 0x20
        elif kind == CORRUPT_OTHER_ROUND:
            j = (i + 1) % n
            chain.sigs[i] = chain.sigs[j].copy()
            if j in chosen:  # keep the donor's original bytes irrelevant: any non-matching valid point fails
                pass
        elif kind == CORRUPT_PREV:
            chain.prev[i, 0] ^= 0x01
        elif kind == CORRUPT_INFINITY:
            chain.sigs[i] = 0
            chain.sigs[i, 0] = 0xC0
        elif kind == CORRUPT_TRUNCATED:
            chain.sig_len[i] = (chain.sig_len[i] // 2) if (i & 1) else 0
    return chosen


def corrupt_global(shard, seed, n_total, lo, rate=1e-3, kinds=ALL_CORRUPTIONS):
    """The corruption catalog of a whole n_total-round chain (chosen from the
    seed alone, like `corrupt`), applied to the shard holding global items
    [lo, lo + len(shard)).  Returns {global index: kind} for the whole chain,
    so every rank knows the expected verdict of every round whatever the
    number of shards; a signature-of-another-round corruption takes its donor
    from the shard (the next round, or the previous one at the shard's end)."""
    n = len(shard)
    count = max(len(kinds), int(round(n_total * rate))) if rate > 0 else 0
    state = (seed ^ 0xC0FFEE) & 0xFFFFFFFFFFFFFFFF
    chosen = {}
    chained = shard.scheme_code == _lib.SCHEME_CHAINED
    k = 0
    while len(chosen) < min(count, n_total):
        state, r = splitmix64(state)
        i = r % n_total
        if i in chosen:
            continue
        kind = kinds[k % len(kinds)]
        k += 1
        if kind == CORRUPT_PREV and not chained:
            kind = CORRUPT_Y_SIGN
        if kind == CORRUPT_OTHER_ROUND and n_total < 2:
            kind = CORRUPT_Y_SIGN
        chosen[int(i)] = kind
    for gi, kind in chosen.items():
        i = gi - lo
        if not 0 <= i < n:
            continue
        if kind == CORRUPT_X_BIT:
            shard.sigs[i, 47] ^= 0x01
        elif kind == CORRUPT_Y_SIGN:
            shard.sigs[i, 0] ^= 0x20
        elif kind == CORRUPT_OTHER_ROUND:
            j = i + 1 if i + 1 < n else i - 1
            if j < 0:  # one-round shard: any other valid point fails too
                shard.sigs[i, 0] ^= 0x20
            else:
                shard.sigs[i] = shard.sigs[j].copy()
        elif kind == CORRUPT_PREV:
            shard.prev[i, 0] ^= 0x01
        elif kind == CORRUPT_INFINITY:
            shard.sigs[i] = 0
            shard.sigs[i, 0] = 0xC0
        elif kind == CORRUPT_TRUNCATED:
            shard.sig_len[i] = (shard.sig_len[i] // 2) if (gi & 1) else 0
    return chosen


# ---------------------------------------------------------------- threshold groups
class Group:
    """A t-of-n threshold group: polynomial coefficients a_0..a_{t-1} over Fr
    (a_0 = derive_secret(seed), the group secret), the public commitments
    C_j = a_j * g1 (48-byte compressed) and the shares s_i = f(i + 1)."""

    def __init__(self, seed, t, n, coeffs, commits):
        self.seed, self.t, self.n = seed, t, n
        self.coeffs = coeffs
        self.commits = commits
        self.shares = [poly_eval(coeffs, i + 1) for i in range(n)]


def share_coeffs(seed, t):
    """a_0 = derive_secret(seed); a_j = OS2IP(SHA-256("drand-mi355x/poly/" ||
    LE64(seed) || LE64(j))) mod r."""
    out = [derive_secret(seed)]
    for j in range(1, t):
        d = hashlib.sha256(b"drand-mi355x/poly/" + struct.pack("<QQ", seed, j)).digest()
        out.append(int.from_bytes(d, "big") % R_ORDER)
    return out


def poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R_ORDER
    return acc


def make_group(seed, t, n, device=0):
    """Commitments derived on the GPU (dgpu_derive_pubkey per coefficient)."""
    ctx = get_context(device)
    coeffs = share_coeffs(seed, t)
    commits = []
    for a in coeffs:
        pk = np.zeros(48, dtype=np.uint8)
        skb = np.frombuffer(a.to_bytes(32, "big"), dtype=np.uint8).copy()
        _lib.check(ctx.lib.dgpu_derive_pubkey(ctx.handle, _lib.SCHEME_CHAINED, _lib.ptr(skb), _lib.ptr(pk), 48))
        commits.append(bytes(pk))
    return Group(seed, t, n, coeffs, commits)


def sign_partials(group, msgs, sign_idx, labels=None, device=0):
    """tbls.Sign of every (round, slot): msgs (n_rounds, 32) uint8, sign_idx
    (n_rounds, m) share indices; labels (default = sign_idx) the BE16 index
    written in front (a label that differs from the signer makes an invalid
    partial).  Returns (n_rounds, m, 98) uint8.  Runs on the GPU
    (dgpu_make_partials)."""
    ctx = get_context(device)
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    sign_idx = np.ascontiguousarray(sign_idx, dtype=np.uint32)
    labels = sign_idx if labels is None else np.ascontiguousarray(labels, dtype=np.uint32)
    nr, m = sign_idx.shape
    shares = np.frombuffer(b"".join(s.to_bytes(32, "big") for s in group.shares), dtype=np.uint8).copy()
    out = np.zeros((nr, m, 98), dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_make_partials(ctx.handle, nr, _lib.ptr(msgs), m, _lib.ptr(sign_idx), _lib.ptr(labels),
                                          _lib.ptr(shares), len(group.shares), _lib.ptr(out)))
    return out


def group_signatures(group, msgs, device=0):
    """sk * H(msg) for every message (the expected recovered signatures),
    through dgpu_make_partials with the group secret as the only share."""
    ctx = get_context(device)
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    nr = msgs.shape[0]
    zeros = np.zeros(nr, dtype=np.uint32)
    sk = np.frombuffer(group.coeffs[0].to_bytes(32, "big"), dtype=np.uint8).copy()
    out = np.zeros((nr, 98), dtype=np.uint8)
    _lib.check(ctx.lib.dgpu_make_partials(ctx.handle, nr, _lib.ptr(msgs), 1, _lib.ptr(zeros), _lib.ptr(zeros),
                                          _lib.ptr(sk), 1, _lib.ptr(out)))
    return out[:, 2:].copy()


def make_recovery_batch(group, n_rounds, seed, bad_rate=0.1, first_round=1, device=0):
    """configs[4] workload: per round the DigestMessage of an unchained round
    (SHA-256(BE64 round)) and t partials from distinct random signers; in a
    `bad_rate` fraction of rounds one partial carries a wrong index (fails
    VerifyPartial), so that round cannot be recovered (t - 1 good).
    Returns (msgs (n, 32), partials (n, t, 98), expect_ok (n,) bool)."""
    rng = np.random.default_rng(seed)
    msgs = np.zeros((n_rounds, 32), dtype=np.uint8)
    for r in range(n_rounds):
        msgs[r] = np.frombuffer(hashlib.sha256(struct.pack(">Q", first_round + r)).digest(), dtype=np.uint8)
    t, n = group.t, group.n
    sign_idx = np.argsort(rng.random((n_rounds, n)), axis=1)[:, :t].astype(np.uint32)
    labels = sign_idx.copy()
    bad = rng.random(n_rounds) < bad_rate
    rows = np.nonzero(bad)[0]
    cols = rng.integers(0, t, size=len(rows))
    labels[rows, cols] = (labels[rows, cols] + 1 + rng.integers(0, n - 1, size=len(rows))) % n
    parts = sign_partials(group, msgs, sign_idx, labels, device=device)
    return msgs, parts, ~bad
