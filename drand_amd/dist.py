"""Multi-GPU sharding for bulk verification.

Rounds shard contiguously across ranks: every stored beacon carries its own
PreviousSig (chain/beacon.go:15), so round verdicts are independent and the
data path needs no collective.  The one exchange step is the result: each
rank's verdict bitmap (and its count of failures) is gathered so the caller
(CheckPastBeacons-style, chain/beacon/sync_manager.go:171-232) can rebuild the
global ascending faulty-round list.  Over RCCL ("nccl" backend) on GPUs, gloo
on CPU tensors in tests.
"""
import numpy as np


def shard_range(n_total, world, rank):
    """Contiguous shard [lo, hi) of n_total items for `rank`: the C ABI's rule
    (dgpu_shard_range, used by dgpu_verify_multi) -- shards of
    ceil(n_total / world) items rounded up to a multiple of 8 (whole bitmap
    bytes), the last one takes the remainder (possibly empty)."""
    world = max(1, world)
    per = -(-n_total // world)
    per = (per + 7) & ~7
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def gather_verdict_bits(local_bits, n_local, n_total, world, rank, device=None):
    """All-gather per-rank verdict bitmaps (uint8 tensors, ceil(n_local/8) bytes)
    and return the global boolean verdict vector (numpy) on every rank."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return np.unpackbits(local_bits.cpu().numpy(), bitorder="little")[:n_local].astype(bool)
    sizes = [shard_range(n_total, world, r) for r in range(world)]
    max_bytes = max((hi - lo + 7) // 8 for lo, hi in sizes)
    dev = local_bits.device if device is None else device
    buf = torch.zeros(max_bytes, dtype=torch.uint8, device=dev)
    buf[: local_bits.numel()] = local_bits
    out = [torch.zeros(max_bytes, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(out, buf)
    parts = []
    for (lo, hi), t in zip(sizes, out):
        parts.append(np.unpackbits(t.cpu().numpy(), bitorder="little")[: hi - lo].astype(bool))
    return np.concatenate(parts)


def faulty_rounds(verdicts, first_round):
    """Ascending list of invalid rounds (None if none), like CheckPastBeacons."""
    bad = np.nonzero(~verdicts)[0]
    return [int(first_round + i) for i in bad] or None
