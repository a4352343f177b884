"""World-size-2 gloo test of the sharded verification path (CPU): each rank
verifies its contiguous shard of a golden chain with the kernels' host build
(test-only tests/hostsim), the verdict bitmaps are all-gathered, and every
rank rebuilds the same global faulty list as a single-rank oracle pass."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import HOSTSIM, load_golden
from oracle import drand_ref as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drand_amd.dist import faulty_rounds, gather_verdict_bits, shard_range
    g = load_golden("chain_chained_s1.json")
    items = [(r["round"], bytes.fromhex(r["prev"]), bytes.fromhex(r["sig"])) for r in g["rounds"][:10]]
    # corrupt two rounds (one per shard)
    items[3] = (items[3][0], items[3][1], bytes([items[3][2][0] ^ 0x20]) + items[3][2][1:])
    items[8] = (items[8][0], items[8][1], b"")
    lo, hi = shard_range(len(items), world, rank)
    hs = ctypes.CDLL(HOSTSIM)
    pk = bytes.fromhex(g["pk"])
    local = []
    for r, prev, sig in items[lo:hi]:
        ok = len(sig) == 96 and hs.hs_verify(pk, D.digest_message(D.SCHEME_CHAINED, r, prev), sig) == 0
        local.append(ok)
    bits = torch.from_numpy(np.packbits(np.array(local, dtype=bool), bitorder="little"))
    verdicts = gather_verdict_bits(bits, hi - lo, len(items), world, rank)
    with open(os.path.join(result_dir, f"rank{rank}.txt"), "w") as f:
        f.write(repr(faulty_rounds(verdicts, items[0][0])))
    dist.destroy_process_group()


def test_sharded_verify_gather_world2(tmp_path, hostsim):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [open(tmp_path / f"rank{r}.txt").read() for r in range(world)]
    assert res[0] == res[1] == repr([4, 9])


def test_shard_range_covers():
    """Contiguous cover; every shard but the last a multiple of 8 rounds (whole
    bitmap bytes); the Python rule equals the C ABI's dgpu_shard_range, which
    dgpu_verify_multi uses (the library loads without a GPU)."""
    from drand_amd import _lib
    from drand_amd.dist import shard_range
    for n in (0, 1, 7, 10, 1000001, 10_000_000):
        for w in (1, 2, 3, 4, 7, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert all((h - l) % 8 == 0 or h == n for l, h in spans[:-1])
            assert all(h - l == spans[0][1] - spans[0][0] for l, h in spans[:-1] if h < n)
            assert spans == [_lib.shard_range(n, w, r) for r in range(w)]


def test_bench_launches_ranks():
    """bench.py --gpus 2 starts two rank processes itself (no torchrun): the
    DRAND_BENCH_DRYRUN stub runs the rank plumbing over gloo without a GPU."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, DRAND_BENCH_DRYRUN="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rounds", "1000"],
                         env=env, capture_output=True, text=True, timeout=300, check=True).stdout
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert sorted(r["rank"] for r in line["ranks"]) == [0, 1]
    assert [tuple(r["shard"]) for r in sorted(line["ranks"], key=lambda r: r["rank"])] == [(0, 504), (504, 1000)]


@pytest.mark.parametrize("driver", ["dist", "abi"])
def test_bench_dry_run_reports_driver_and_ranks(driver):
    """bench.py --gpus 2 --dry-run prints the chosen driver and the rank (or
    device) count with each shard; both drivers shard the chain the same way
    (dgpu_shard_range's rule), so their gathered verdict bitmaps cover the
    same round ranges."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rounds", "1000",
                          "--dry-run", "--driver", driver], env=env, capture_output=True, text=True, timeout=300,
                         check=True).stdout
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["driver"] == driver and line["n_gpus"] == 2
    shards = [tuple(r["shard"]) for r in sorted(line["ranks"], key=lambda r: r.get("rank", r.get("device")))]
    assert shards == [(0, 504), (504, 1000)]
