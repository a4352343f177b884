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


def beacon_unmarshal(buf: bytes) -> Beacon:
    """Beacon.Unmarshal (chain/beacon.go:34-37).  Missing fields decode to
    their zero values, like Go's encoding/json."""
    d = json.loads(buf)
    return Beacon(bytes.fromhex(d.get("PreviousSig") or ""), int(d.get("Round") or 0),
                  bytes.fromhex(d.get("Signature") or ""))


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
    faulty = []
    i = 1
    while i < n:
        # fetch one window of rows, then verify every present beacon in one batch
        hi = min(n, i + window)
        rows = []
        for r in range(i, hi):
            try:
                rows.append(store.get(r))
            except ErrNoBeaconSaved:
                rows.append(None)
            except ValueError:  # Unmarshal error: Get returns err, the round is faulty
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
