"""drand_amd: MI355X-native batch verifier for drand beacon chains.

Product path: drand_amd.chain.Verifier -> libdrand_gpu.so (C-ABI,
include/drand_gpu.h) -> gfx950 HIP kernels.  No CPU fallback.
"""
from . import _lib, scheme  # noqa: F401
from .scheme import Scheme, get_scheme_by_id, get_scheme_by_id_with_default, list_schemes  # noqa: F401

__all__ = ["Scheme", "get_scheme_by_id", "get_scheme_by_id_with_default", "list_schemes"]
