"""bench.py --gpus 2 end to end on the one GPU of a test box: the rank
launcher, the per-rank C-ABI calls (dgpu_verify_beacons_device per shard),
the exchange of verdict bitmaps and, in RLC mode, the per-rank protocol
(dgpu_rlc_root_device -> all-gather of roots -> dgpu_rlc_finish_device),
the barrier + max-over-ranks timing, and the rank-0 JSON line -- with the
process group over gloo (DRAND_BENCH_BACKEND=gloo: both ranks share GPU 0)
instead of RCCL, which refuses two ranks on one device.  This is the path
the driver's multi-GPU scaling run takes with one rank per GPU over RCCL.
Marked gpu."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_share_one_gpu_over_gloo():
    env = dict(os.environ, DRAND_BENCH_BACKEND="gloo")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rounds", "40000", "--steps", "1",
           "--warmup", "1", "--no-legs", "--no-e2e", "--no-cpu-baseline", "--no-ingest", "--no-small-batch"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["driver"]["ranks"] == 2 and line["driver"].get("backend") == "gloo"
    assert line["config"]["rounds_total"] == 40000 and line["config"]["rounds_per_gpu"] == 20000
    assert line["verdict_mismatches"] == 0 and line["corrupted_rounds_total"] > 0
    assert line["rlc"]["verdict_mismatches"] == 0
