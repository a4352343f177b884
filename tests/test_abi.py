"""The C-ABI library builds, loads and exports every symbol include/drand_gpu.h
declares; without a GPU it fails loudly (no CPU fallback).  CPU-only."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "drand_gpu.h")).read()
    return sorted(set(re.findall(r"\b(dgpu_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    from drand_amd import _lib
    assert sorted(n for n, _, _ in _lib.SYMBOLS) == declared_symbols()


def test_library_exports_all_symbols():
    from drand_amd import _lib
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.dgpu_abi_version() == _lib.ABI_VERSION == 3
    assert lib.dgpu_scheme_from_name(b"") == _lib.SCHEME_CHAINED
    assert lib.dgpu_scheme_from_name(b"pedersen-bls-unchained") == _lib.SCHEME_UNCHAINED
    assert lib.dgpu_scheme_from_name(b"bls-unchained-on-g1") == _lib.SCHEME_UNCHAINED_G1
    assert lib.dgpu_scheme_from_name(b"nope") == _lib.DGPU_EINVAL
    assert b"not valid" in lib.dgpu_last_error()


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from drand_amd import _lib
    with pytest.raises(_lib.DrandGPUError):
        _lib.Context(0)


def test_ingest_library_exports_its_header():
    """libdrand_ingest.so (host-only ingest helpers) exports every symbol
    include/drand_ingest.h declares, and drand_amd/ingest.py binds them."""
    from drand_amd import ingest
    txt = open(os.path.join(ROOT, "include", "drand_ingest.h")).read()
    names = sorted(set(re.findall(r"\b(dgpu_[a-z0-9_]+)\s*\(", txt)))
    assert names == ["dgpu_ingest_count", "dgpu_ingest_decode", "dgpu_ingest_scan"]
    lib = ingest.load()
    assert lib is not None, "libdrand_ingest.so not built (__graft_entry__.build())"
    for n in names:
        assert hasattr(lib, n), n


def test_max_stages_macro_matches_binding():
    """DGPU_MAX_STAGES (include/drand_gpu.h) is what the Python binding sizes
    dgpu_stage_times' arrays by; the GPU tests assert every pipeline's stage
    count (the call returns the count needed) stays within it."""
    from drand_amd import _lib
    txt = open(os.path.join(ROOT, "include", "drand_gpu.h")).read()
    (val,) = re.findall(r"#define DGPU_MAX_STAGES (\d+)", txt)
    assert int(val) == _lib.MAX_STAGES >= 16
