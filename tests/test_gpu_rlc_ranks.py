"""The per-rank RLC protocol (include/drand_gpu.h dgpu_rlc_root_device ->
caller's all-gather of roots -> dgpu_rlc_finish_device; drand_amd/dist.py
verify_rlc_sharded, the path bench.py --gpus N takes in RLC mode) with two
rank processes over gloo sharing the one GPU of the box: every rank's shard
verdicts, gathered, equal the single-context per-round reasons and the
construction -- for a corrupted chain (the node fails, each shard descends),
a clean one (the node passes on the summed roots alone), G2 and G1
signatures.

Stream contract: every rank passes the NULL stream
(the legacy default stream, ABI 3), zero-fills its outputs with torch on the
default stream and reads them back with no device-wide synchronize anywhere
in the protocol (drand_amd/dist.py orders the exchange by stream waits).
Under ABI 2 NULL meant the context's non-blocking stream and this exact
sequence accepted a corrupted round (gpurun_out/r04c).

Seeds: both ranks pass the same seed; dist.rank_seed derives
per-rank coefficients, so errors +D / -D planted at the same position of the
two shards cannot cancel in the summed node.  Marked gpu."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 3001


CRAFT_POS = 100  # local position of the +D / -D pair in both shards


def _chain(code, seed, rate, crafted=False):
    from drand_amd.dist import shard_range
    from drand_amd.synth import corrupt, make_chain
    c = make_chain(seed, N, code, seg_len=64)
    bad = corrupt(c, seed, rate=rate) if rate else {}
    if crafted:  # sig + g2 in shard 0, sig - g2 in shard 1, same local position
        from oracle import bls12381 as B
        lo1, _ = shard_range(N, 2, 1)
        for i, sign in ((CRAFT_POS, 1), (lo1 + CRAFT_POS, -1)):
            s = B.g2_decompress(bytes(c.sigs[i]))
            d = B.G2_GEN if sign > 0 else B.g2_neg(B.G2_GEN)
            c.sigs[i] = np.frombuffer(B.g2_compress(B.g2_add(s, d)), dtype=np.uint8)
            bad[i] = "crafted"
    return c, bad


def _rank(rank, world, port, code, seed, rate, crafted, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from drand_amd.chain import get_context
        from drand_amd.dist import gather_verdict_bits, shard_range, verify_rlc_sharded
        torch.cuda.set_device(0)
        c, _ = _chain(code, seed, rate, crafted)
        lo, hi = shard_range(N, world, rank)
        dev = torch.device("cuda", 0)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a[lo:hi])).to(dev)  # noqa: E731
        d_rounds, d_sigs = t(c.rounds.view(np.int64)), t(c.sigs)
        d_sig_len, d_prev, d_prev_len = t(c.sig_len.view(np.int32)), t(c.prev), t(c.prev_len.view(np.int32))
        n = hi - lo
        d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
        d_reason = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        ctx = get_context(0)
        # NULL stream, one seed for both ranks, no synchronize: .cpu() below
        # is ordered after the library's work by the default stream alone
        verify_rlc_sharded(ctx, code, np.frombuffer(c.pk, dtype=np.uint8).copy(), n, d_rounds, d_sigs, d_sig_len,
                           d_prev, d_prev_len, 1000, d_bits, None, world, rank, d_reason=d_reason)
        bits = gather_verdict_bits(d_bits.cpu(), n, N, world, rank)
        reasons = [None] * world
        dist.all_gather_object(reasons, d_reason.cpu().numpy()[:n].tolist())
        if rank == 0:
            q.put((bits.tolist(), sum(reasons, [])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("code_name,rate,crafted", [("SCHEME_CHAINED", 2e-3, False), ("SCHEME_CHAINED", 0, False),
                                                    ("SCHEME_UNCHAINED_G1", 2e-3, False),
                                                    ("SCHEME_CHAINED", 0, True)])
def test_rlc_rank_protocol_world2_equals_single(code_name, rate, crafted):
    import torch.multiprocessing as mp
    from drand_amd import _lib
    from drand_amd.chain import Verifier
    from drand_amd.scheme import get_scheme_by_id_with_default
    code = getattr(_lib, code_name)
    name = {_lib.SCHEME_CHAINED: "pedersen-bls-chained", _lib.SCHEME_UNCHAINED_G1: "bls-unchained-on-g1"}[code]
    c, bad = _chain(code, 71, rate, crafted)
    single = Verifier(get_scheme_by_id_with_default(name)).verify_reasons([c.beacon(i) for i in range(N)], c.pk)
    expect = np.ones(N, dtype=bool)
    expect[list(bad)] = False
    assert np.array_equal(single == 0, expect)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, code, 71, rate, crafted, q)) for r in range(2)]
    for p in procs:
        p.start()
    bits, reasons = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert bits == expect.tolist()
    assert reasons == single.tolist()
