"""Scheme registry: mirrors common/scheme/scheme.go (same IDs, same lookup
and error behaviour), plus the `bls-unchained-on-g1` scheme this build adds
(absent from the reference snapshot) and its RFC 9380
DST variant `bls-unchained-g1-rfc9380`."""
import os
from dataclasses import dataclass

DEFAULT_SCHEME_ID = "pedersen-bls-chained"       # scheme.go:9
UNCHAINED_SCHEME_ID = "pedersen-bls-unchained"   # scheme.go:12
UNCHAINED_ON_G1_SCHEME_ID = "bls-unchained-on-g1"  # added (G1 signatures, G2 public key)
G1_RFC9380_SCHEME_ID = "bls-unchained-g1-rfc9380"  # added: as on-g1 with the RFC 9380 G1 DST


@dataclass(frozen=True)
class Scheme:
    """scheme.go:15-18"""
    id: str
    decouple_prev_sig: bool
    sigs_on_g1: bool = False


_SCHEMES = [
    Scheme(DEFAULT_SCHEME_ID, False),
    Scheme(UNCHAINED_SCHEME_ID, True),
    Scheme(UNCHAINED_ON_G1_SCHEME_ID, True, sigs_on_g1=True),
    Scheme(G1_RFC9380_SCHEME_ID, True, sigs_on_g1=True),
]


def get_scheme_by_id(scheme_id):
    """scheme.go:22-31: (scheme, found)."""
    for s in _SCHEMES:
        if s.id == scheme_id:
            return s, True
    return Scheme("", False), False


def get_scheme_by_id_with_default(scheme_id):
    """scheme.go:33-48: "" -> default; unknown -> error."""
    if scheme_id == "":
        scheme_id = DEFAULT_SCHEME_ID
    s, ok = get_scheme_by_id(scheme_id)
    if not ok:
        raise ValueError(f"scheme [{scheme_id}] is not valid")
    return s


def list_schemes():
    """scheme.go:50-57"""
    return [s.id for s in _SCHEMES]


def read_scheme_by_env():
    """scheme.go:59-71 (env SCHEME_ID, default chained)."""
    return get_scheme_by_id(os.environ.get("SCHEME_ID", "") or DEFAULT_SCHEME_ID)


def get_scheme_from_env():
    """scheme.go:73-80: panics (raises) on an invalid id."""
    s, ok = read_scheme_by_env()
    if not ok:
        raise ValueError("scheme is not valid")
    return s


def scheme_code(s):
    from . import _lib
    return {DEFAULT_SCHEME_ID: _lib.SCHEME_CHAINED, UNCHAINED_SCHEME_ID: _lib.SCHEME_UNCHAINED,
            UNCHAINED_ON_G1_SCHEME_ID: _lib.SCHEME_UNCHAINED_G1, G1_RFC9380_SCHEME_ID: _lib.SCHEME_G1_RFC9380}[s.id]
