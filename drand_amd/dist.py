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
    if dist.get_backend() == "gloo":  # CPU collectives (tests, one-GPU rehearsals)
        dev = torch.device("cpu")
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


def rank_seed(seed, rank, world):
    """The RLC seed rank `rank` uses: SplitMix64(seed ^ 0x5EED * (rank + 1)),
    the per-device derivation of dgpu_verify_multi (multi_gpu.h), so every
    rank draws independent coefficients from one caller seed.  Coefficients
    are keyed on the position inside the shard; with one seed shared by two
    ranks, round i of shard A and round i of shard B would get the same
    coefficient and errors +D / -D there would cancel in the summed node
    (ADVICE r04).  world == 1 keeps the seed."""
    if world <= 1:
        return seed & 0xFFFFFFFFFFFFFFFF
    m = 0xFFFFFFFFFFFFFFFF
    z = ((seed ^ (0x5EED * (rank + 1))) + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def verify_rlc_sharded(ctx, code, pk, n, d_rounds, d_sigs, d_sig_len, d_prev, d_prev_len, seed, d_bits, stream,
                       world, rank, d_reason=None, sig_stride=96, prev_stride=96):
    """RLC mode across ranks through the library's per-rank protocol
    (include/drand_gpu.h dgpu_rlc_root_device / dgpu_rlc_finish_device, the
    multi-process form of dgpu_verify_multi's RLC mode): this rank's shard
    root by bucket MSM, the roots all-gathered over torch.distributed (RCCL
    on GPUs), the node (sum of every rank's root) checked with one pairing on
    every rank, this shard's tree descended only when the node fails.  d_* are
    device tensors of this rank's shard.  `seed` may be the same on every
    rank: each rank derives its own (rank_seed).  `stream`: a torch stream or
    None (the legacy default stream, NULL at the C ABI).  The library's work
    is enqueued on it; the exchange is ordered after it by stream waits
    (torch's current stream waits on `stream` before the collective and
    `stream` waits on the collective's result), never by a device-wide
    synchronize.  Returns nothing: the verdict bits land in d_bits (and
    reasons in d_reason) in `stream` order."""
    import ctypes
    import torch
    import torch.distributed as dist
    from . import _lib
    lib = ctx.lib
    rb = lib.dgpu_rlc_root_bytes(code)
    _lib.check(min(rb, 0))
    dev = d_bits.device
    s = ctypes.c_void_p(None if stream is None else stream.cuda_stream)
    lib_stream = torch.cuda.default_stream(dev) if stream is None else stream
    cur = torch.cuda.current_stream(dev)
    with torch.cuda.stream(lib_stream):  # root allocated in the library's stream order
        root = torch.empty(rb, dtype=torch.uint8, device=dev)
    pkb = pk if hasattr(pk, "ctypes") else np.frombuffer(bytes(pk), dtype=np.uint8).copy()
    _lib.check(lib.dgpu_rlc_root_device(ctx.handle, code, _lib.ptr(pkb), pkb.size, n, d_rounds.data_ptr(),
                                        d_sigs.data_ptr(), sig_stride, d_sig_len.data_ptr(), d_prev.data_ptr(),
                                        prev_stride, d_prev_len.data_ptr(), rank_seed(seed, rank, world),
                                        root.data_ptr(), s))
    if world > 1:
        cur.wait_stream(lib_stream)  # the root is written before the collective reads it
        root.record_stream(cur)
        roots = torch.empty(world * rb, dtype=torch.uint8, device=dev)
        if dist.get_backend() == "gloo":  # CPU collectives (tests): .cpu() waits on the current stream
            out = [torch.empty(rb, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(out, root.cpu())
            roots.copy_(torch.cat(out))
        else:
            dist.all_gather_into_tensor(roots, root)
        lib_stream.wait_stream(cur)  # the gathered roots are complete before the finish step reads them
        roots.record_stream(lib_stream)
    else:
        roots = root
    _lib.check(lib.dgpu_rlc_finish_device(ctx.handle, world, roots.data_ptr(), d_bits.data_ptr(),
                                          None if d_reason is None else d_reason.data_ptr(), s))
