"""The generated kernel tables in drand_amd/csrc are what their generators
produce: engine_tables.h + engine_compiled.h from tools/gen_engine.py (the
pairing engine's programs, compiled ops and LDS layout) and constants.h from
tools/gen_constants.py (curve constants, exponent schedules).  A stale
header would make the device run programs the Model tests never checked."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "drand_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_engine_tables_up_to_date(tmp_path):
    import gen_engine as ge
    out = tmp_path / "engine_tables.h"
    ge.emit(str(out))
    for name in ("engine_tables.h", "engine_compiled.h"):
        with open(os.path.join(CSRC, name)) as f:
            committed = f.read()
        assert (tmp_path / name).read_text() == committed, f"{name} is stale: run python tools/gen_engine.py"


def test_constants_up_to_date(tmp_path):
    # gen_constants.py writes next to itself; run a copy of the tree's script
    # with its output redirected by reading the generated text from stdout-free
    # execution in a scratch directory
    src = os.path.join(ROOT, "tools", "gen_constants.py")
    code = open(src).read()
    dst = tmp_path / "constants.h"
    code = code.replace('dst = os.path.join(os.path.dirname(__file__), "..", "drand_amd", "csrc", "constants.h")',
                        f"dst = {str(dst)!r}")
    assert str(dst) in code
    script = tmp_path / "gen_constants.py"
    script.write_text(code)
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.check_call([sys.executable, str(script)], cwd=os.path.join(ROOT, "tools"), env=env,
                          stdout=subprocess.DEVNULL)
    with open(os.path.join(CSRC, "constants.h")) as f:
        assert dst.read_text() == f.read(), "constants.h is stale: run python tools/gen_constants.py"
