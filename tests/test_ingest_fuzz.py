"""Mutation fuzzing of the native bolt-store parsers (libdrand_ingest's
dgpu_ingest_count / dgpu_ingest_scan / dgpu_ingest_decode,
drand_amd/csrc/ingest.cpp) under AddressSanitizer and UBSan: the parsers read
files that arrive from disk (a drand.db copied from another node), so a
malformed page, element or row must give -1 / ok = 0, never a read outside
the mapped file.  tests/fuzz_ingest.cpp is built here together with
ingest.cpp (host code only) and run on multi-level and inline-bucket files
written by tests/bolt_writer.py.  CPU test; skipped when the sanitizer
runtime cannot be built."""
import os
import random
import subprocess

import pytest

from bolt_writer import write_bolt
from drand_amd.boltstore import BoltStore
from test_boltstore import _kv, _random_store

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    exe = tmp_path_factory.mktemp("fuzz") / "fuzz_ingest"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-o", str(exe), os.path.join(ROOT, "tests", "fuzz_ingest.cpp"),
           os.path.join(ROOT, "drand_amd", "csrc", "ingest.cpp")]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode:
        pytest.skip("sanitizer build unavailable: " + p.stderr[-300:])
    return str(exe)


@pytest.mark.parametrize("n,page_size,inline", [(3000, 4096, False), (900, 1024, False), (20, 4096, True)])
def test_ingest_parsers_survive_mutated_files(tmp_path, fuzzer, n, page_size, inline):
    st, _ = _random_store(random.Random(n), n, big=400)
    path = tmp_path / "drand.db"
    write_bolt(path, _kv(st), page_size=page_size, inline=inline)
    bs = BoltStore(path)
    root = bs._b.root
    bs.close()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([fuzzer, str(path), str(page_size), str(root), "1500", str(n)], capture_output=True, text=True,
                       env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "scans=1500" in p.stdout, p.stdout
