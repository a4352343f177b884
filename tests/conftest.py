import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
# The library runs DGPU_MODE_RLC batches under 131,072 rounds on the per-round
# path (DGPU_RLC_MIN); the tests' RLC batches are smaller, so they lower the
# threshold to exercise the RLC path itself (read at every dgpu_open).
# tests/test_gpu_parity.py::test_rlc_small_batches_take_per_round_path
# checks the default.
os.environ.setdefault("DGPU_RLC_MIN", "0")
# Likewise pairing batches under DGPU_THR_MIN (65,536) items run the 12-lane
# lines and 8-lane chain; the suite lowers it so its batches run the
# per-thread kernels the bulk path uses.  Tests that compare the two kernel
# families set it (or DGPU_LINES / DGPU_KB_CHAIN) on their own contexts.
os.environ.setdefault("DGPU_THR_MIN", "0")
# Likewise calls up to 16Ki rounds clear the hash cofactor on the engine
# ladder (DGPU_COF_ENGINE_MAX) and take the Granger-Scott final
# exponentiation (DGPU_FE_GS_MAX); the suite turns both latency paths off so
# its small batches run k_h2c_finish and the Karabina FE of the bulk path.
# tests/test_gpu_defaults.py runs the library defaults (both paths on).
os.environ.setdefault("DGPU_COF_ENGINE_MAX", "0")
os.environ.setdefault("DGPU_FE_GS_MAX", "0")
HOSTSIM = os.path.join(ROOT, "tests", "hostsim", "libdrand_hostsim.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def hostsim():
    """Test-only host build of the kernel arithmetic (tests/hostsim)."""
    import ctypes
    src = os.path.join(ROOT, "tests", "hostsim", "hostsim.hip")
    deps = [src] + [os.path.join(ROOT, "drand_amd", "csrc", f) for f in os.listdir(os.path.join(ROOT, "drand_amd", "csrc"))]
    if not os.path.exists(HOSTSIM) or os.path.getmtime(HOSTSIM) < max(os.path.getmtime(d) for d in deps):
        subprocess.check_call(["hipcc", "-O2", "-std=c++17", "--cuda-host-only", "-fPIC", "-shared", "-o", HOSTSIM, src])
    return ctypes.CDLL(HOSTSIM)


@pytest.fixture(scope="session", autouse=True)
def _torch_before_library(request):
    """GPU sessions: initialise torch's HIP state before any library context.
    torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's): when
    torch loads first, the library binds to torch's runtime; when the library
    initialises HIP first, torch later runs on the system runtime and
    torch._C._cuda_init() fails with "No HIP GPUs are available"
    (gpurun_out/r05n, r05u).  Session-scoped and autouse, so it runs before
    the session's gpu_ctx whatever test comes first; a session without GPU
    tests never touches torch here."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        torch.cuda.init()
    yield


def open_ctx(env, device=0):
    """A fresh library context opened under the environment `env` (the
    library reads its knobs at dgpu_open).  Knobs of variants not shipped and
    test hooks (_lib.AB_KNOBS) are read only by the A/B build
    (drand_amd/libdrand_gpu_ab.so), so such an env opens that build."""
    from drand_amd import _lib
    ab = any(k in _lib.AB_KNOBS for k in env)
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return _lib.Context(device, lib_path=_lib.AB_LIB_PATH if ab else None)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="session")
def gpu_ctx():
    from drand_amd.chain import get_context
    return get_context(0)
