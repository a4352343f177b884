"""Bulk chain check (the historical-chain caller of the verify path), batched
onto the GPU with the reference's exact verdict semantics.

Mirrors:
  SyncManager.CheckPastBeacons    chain/beacon/sync_manager.go:171-232
  chain.Store (Len/Last/Get)      chain/store.go:16-27, chain/boltdb/store.go:70-130
  Beacon.Marshal/Unmarshal        chain/beacon.go:29-37 (hexjson: []byte fields as hex strings)

The reference walks rounds 1 .. store.Len()-1 one at a time: Get, then
VerifyBeacon, then a progress callback.  Here the walk is split into windows:
each window's stored beacons are fetched, verified in ONE batch call on the
GPU, and then replayed in round order so that the faulty list, the progress
callbacks and the stopping rule are the reference's, element for element:
  * upTo is clamped to the last stored round (:180-184);
  * cb(i, upTo) fires for every visited i before its beacon is examined (:198-200);
  * a missing row makes round i faulty (:202-210); a failed verification
    records the *stored* beacon's Round field (:212-214);
  * the walk stops after i >= upTo (:207-209, :219-221) or at store.Len()-1;
  * the result is the ascending faulty list, or None when there is none (:225-231).
Context cancellation (:189-194) maps to the optional `cancelled()` predicate,
checked at the same point of every iteration.
"""
import json
import struct

from .chain import Beacon


class ErrNoBeaconSaved(KeyError):
    """chain/store.go ErrNoBeaconSaved: no beacon stored for that round."""


class Cancelled(Exception):
    """ctx.Err() of CheckPastBeacons (context cancelled)."""


def beacon_marshal(b: Beacon) -> bytes:
    """Beacon.Marshal (chain/beacon.go:29-32): hexjson, byte slices as hex."""
    return json.dumps({
        "PreviousSig": (b.previous_sig or b"").hex(),
        "Round": b.round,
        "Signature": (b.signature or b"").hex(),
    }, separators=(",", ":")).encode()


_HEX_DIGITS = frozenset("0123456789abcdefABCDEF")


def hex_decode_strict(s: str, name="field") -> bytes:
    """Go's hex.DecodeString, which hexjson uses for []byte fields: an
    even-length string of hex digits only.  Python's bytes.fromhex would
    also accept whitespace between byte pairs ('ab cd'); Go rejects it
    (InvalidByteError), so the round must come out faulty here too."""
    if len(s) & 1 or not _HEX_DIGITS.issuperset(s):
        raise ValueError(f"beacon: {name} is not valid hex")
    return bytes.fromhex(s)


def _json_field(d, name):
    """encoding/json field lookup: exact key first, then case-insensitive."""
    if name in d:
        return d[name]
    low = name.lower()
    for k, v in d.items():
        if isinstance(k, str) and k.lower() == low:
            return v
    return None


def beacon_unmarshal(buf: bytes) -> Beacon:
    """Beacon.Unmarshal (chain/beacon.go:34-37, hexjson).  Missing or null
    fields decode to their zero values, like Go's encoding/json; anything Go
    would refuse (not a JSON object, a non-hex byte field, a Round that is not
    a non-negative integer below 2^64) raises ValueError -- Get's unmarshal
    error, which CheckPastBeacons counts as a faulty round."""
    try:
        d = json.loads(buf)
    except (ValueError, UnicodeDecodeError, TypeError) as e:
        raise ValueError(f"beacon: invalid JSON: {e}") from None
    if not isinstance(d, dict):
        raise ValueError("beacon: not a JSON object")

    def hexbytes(name):
        v = _json_field(d, name)
        if v is None:
            return b""
        if not isinstance(v, str):
            raise ValueError(f"beacon: {name} is not a hex string")
        return hex_decode_strict(v, name)

    r = _json_field(d, "Round")
    if r is None:
        r = 0
    if isinstance(r, bool) or not isinstance(r, int) or not 0 <= r < 1 << 64:
        raise ValueError("beacon: Round is not a uint64")
    return Beacon(hexbytes("PreviousSig"), r, hexbytes("Signature"))


class MemoryStore:
    """A chain.Store with boltdb's key/value shape (key = BE64(round), value =
    marshalled beacon; chain/boltdb/store.go:70-130), held in memory.  Len()
    counts stored keys, round 0 (the genesis) included, like the bolt
    bucket's KeyN."""

    def __init__(self):
        self._kv = {}

    def put(self, b: Beacon):
        self._kv[struct.pack(">Q", b.round)] = beacon_marshal(b)

    def put_raw(self, round_, value: bytes):
        self._kv[struct.pack(">Q", round_)] = value

    def delete(self, round_):
        self._kv.pop(struct.pack(">Q", round_), None)

    def len(self):
        return len(self._kv)

    def last(self) -> Beacon:
        if not self._kv:
            raise ErrNoBeaconSaved("no beacon saved")
        return beacon_unmarshal(self._kv[max(self._kv)])

    def get(self, round_) -> Beacon:
        v = self._kv.get(struct.pack(">Q", round_))
        if v is None:
            raise ErrNoBeaconSaved(round_)
        return beacon_unmarshal(v)


def check_past_beacons(store, verifier, pubkey, up_to, cb=None, window=1 << 16, cancelled=None, mode=0):
    """SyncManager.CheckPastBeacons (chain/beacon/sync_manager.go:171-232).

    `verifier` is a drand_amd.chain.Verifier (GPU); `pubkey` the group key
    bytes.  Returns the ascending list of faulty rounds, or None."""
    last = store.last()
    if last.round < up_to:
        up_to = last.round
    n = store.len()
    if hasattr(store, "scan_offsets") and hasattr(verifier, "verify_records"):
        return _check_past_records(store, verifier, pubkey, up_to, n, cb, window, cancelled, mode)
    faulty = []
    i = 1
    while i < n:
        # fetch one window of rows, then verify every present beacon in one batch
        hi = min(n, i + window)
        rows = []
        if hasattr(store, "scan"):  # one ordered pass over the window's rows (drand_amd/boltstore.py)
            got = dict(store.scan(i, hi))
            for r in range(i, hi):
                v = got.get(r)
                try:
                    rows.append(None if v is None else beacon_unmarshal(v))
                except ValueError:  # Unmarshal error: the round is faulty
                    rows.append(None)
        else:
            for r in range(i, hi):
                try:
                    rows.append(store.get(r))
                except (ErrNoBeaconSaved, ValueError):  # no row, or Unmarshal error: the round is faulty
                    rows.append(None)
        present = [b for b in rows if b is not None]
        reasons = verifier.verify_reasons(present, pubkey, mode) if present else []
        ok = iter(r == 0 for r in reasons)
        # replay in order: identical callbacks, faulty list and stopping rule
        for k, b in enumerate(rows):
            r = i + k
            if cancelled is not None and cancelled():
                raise Cancelled()
            if cb is not None:
                cb(r, up_to)
            if b is None:
                faulty.append(r)
                if r >= up_to:
                    return faulty or None
                continue
            if not next(ok):
                faulty.append(b.round)
            if r >= up_to:
                return faulty or None
        i = hi
    return faulty or None


def _check_past_records(store, verifier, pubkey, up_to, n, cb, window, cancelled, mode):
    """CheckPastBeacons over a BoltStore with the native ingest
    (drand_amd/ingest.py): each window's rows are walked and decoded into
    fixed-stride records off the Python heap -- the next window's while the
    GPU verifies the current one (the ctypes call releases the GIL) -- and
    replayed with the loop's exact rules: rounds visited 1 .. min(Len-1,
    upTo); a missing or undecodable row faults its round i, a failed
    verification the stored beacon's Round; callbacks and cancellation per
    visited round when given."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from .ingest import window_records
    # visited rounds: [1, end) -- round 1 always (the loop tests i >= upTo only
    # after checking round i, sync_manager.go:188-221), so up_to = 0 checks it too
    end = min(n, max(up_to, 1) + 1)
    if end <= 1:
        return None
    bounds = [(lo, min(end, lo + window)) for lo in range(1, end, window)]
    faulty = []
    with ThreadPoolExecutor(1) as ex:
        nxt = ex.submit(window_records, store, *bounds[0])
        for k in range(len(bounds)):
            rec = nxt.result()
            if k + 1 < len(bounds):
                nxt = ex.submit(window_records, store, *bounds[k + 1])
            reasons = verifier.verify_records(pubkey, rec.rounds, rec.sigs, rec.sig_len, rec.prev, rec.prev_len,
                                              mode) if len(rec.rounds) else np.zeros(0, dtype=np.uint8)
            # the faulty value of every visited round of the window, in order
            size = rec.hi - rec.lo
            val = np.zeros(size, dtype=np.uint64)
            hit = np.zeros(size, dtype=bool)
            hit[rec.bad] = True
            val[rec.bad] = rec.lo + rec.bad.astype(np.uint64)
            fail = reasons != 0
            hit[rec.index[fail]] = True
            val[rec.index[fail]] = rec.rounds[fail]
            if cb is None and cancelled is None:
                faulty.extend(val[hit].tolist())
                continue
            for j in range(size):
                if cancelled is not None and cancelled():
                    raise Cancelled()
                if cb is not None:
                    cb(rec.lo + j, up_to)
                if hit[j]:
                    faulty.append(int(val[j]))
    return faulty or None


# ---------------------------------------------------------------- streaming sync
class SchemeStore:
    """chain/beacon/store.go:56-95 schemeStore.Put: unchained schemes store
    PreviousSig as nil; chained ones require PreviousSig to equal the last
    stored signature or the stored signature of round - 1."""

    def __init__(self, store, decouple_prev_sig):
        self.store = store
        self.decouple = decouple_prev_sig
        try:
            self._last = store.last()
        except ErrNoBeaconSaved:
            self._last = None

    def put(self, b: Beacon):
        if self.decouple:
            b = Beacon(b"", b.round, b.signature)
        elif self._last is None or self._last.signature != b.previous_sig:
            try:
                pb = self.store.get(b.round - 1)
            except ErrNoBeaconSaved as e:
                raise ValueError(f"invalid previous signature for {b.round} or previous beacon not found "
                                 f"in database. Err: {e}") from None
            if pb.signature != b.previous_sig:
                raise ValueError(f"invalid previous signature for {b.round} or previous beacon not found "
                                 f"in database. Err: <nil>")
        self.store.put(b)
        self._last = b

    def last(self):
        return self.store.last()

    def get(self, round_):
        return self.store.get(round_)


def try_node(packets, verifier, pubkey, store, up_to, beacon_id=None, window=500, mode=0):
    """Batch mirror of SyncManager.tryNode's receive loop
    (chain/beacon/sync_manager.go:370-424).  `packets` yields (Beacon,
    beacon_id or None) in stream order (the peer's channel; exhaustion = the
    channel closed).  Up to `window` buffered packets (the peer buffer,
    MaxSyncBuffer = 500, net/client_grpc.go:220) are verified in one GPU call;
    then, per packet in order, exactly the reference's rules: a wrong beacon
    ID -> False; an invalid beacon -> False (earlier ones stay stored);
    store.put failure -> False; the beacon reaching up_to -> True.  Returns
    (ok, last_stored_beacon or None)."""
    it = iter(packets)
    last = None
    while True:
        buf = []
        for pkt in it:
            buf.append(pkt)
            if len(buf) >= window:
                break
        if not buf:
            return False, last  # channel closed
        # verify only the prefix the loop can reach: up to the first wrong ID
        stop = next((k for k, (_, bid) in enumerate(buf) if bid is not None and beacon_id is not None
                     and bid != beacon_id), len(buf))
        reasons = verifier.verify_reasons([b for b, _ in buf[:stop]], pubkey, mode) if stop else []
        for k, (b, _) in enumerate(buf):
            if k == stop:
                return False, last  # sync_manager.go:378-381
            if int(reasons[k]) != 0:
                return False, last  # :394-397
            try:
                store.put(b)
            except Exception:
                return False, last  # :406-410
            last = b
            if last.round == up_to:
                return True, last  # :417-420


def trusted_previous_signature(verifier, pubkey, get_signature, genesis_seed, round_, point_of_trust=None,
                               window=1 << 14, mode=0):
    """Batch mirror of verifyingClient.getTrustedPreviousSignature
    (client/verify.go:118-178): walk from the point of trust (or round 1,
    whose previous signature is the genesis seed) to round - 1, verifying each
    fetched beacon with PreviousSig = the previous signature; here the walk's
    beacons are verified `window` at a time.  `get_signature(r)` fetches round
    r's signature (raise to signal a fetch error).  Returns (prev_sig,
    new_point_of_trust) where the point of trust is (round, signature) or the
    old one; raises VerifyError at the first invalid beacon, as the reference
    returns "verifying beacon: ..."."""
    from .chain import VerifyError
    if round_ == 1:
        return genesis_seed, point_of_trust
    if point_of_trust is None or point_of_trust[0] > round_:
        trust_round, trust_sig = 1, genesis_seed  # slow path: from round 1
    else:
        trust_round, trust_sig = point_of_trust
    initial = trust_round
    new_pot = point_of_trust
    while trust_round < round_ - 1:
        hi = min(round_ - 1, trust_round + window)
        rounds = list(range(trust_round + 1, hi + 1))
        sigs = [get_signature(r) for r in rounds]
        prevs = [trust_sig] + sigs[:-1]
        beacons = [Beacon(p, r, s) for p, r, s in zip(prevs, rounds, sigs)]
        reasons = verifier.verify_reasons(beacons, pubkey, mode)
        for b, rs in zip(beacons, reasons):
            if int(rs) != 0:
                raise VerifyError(b.round, int(rs))
        trust_round, trust_sig = hi, sigs[-1]
    if trust_round == round_ - 1 and trust_round > initial:
        new_pot = (trust_round, trust_sig)
    return trust_sig, new_pot
