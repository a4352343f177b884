"""drand_amd.scheme mirrors common/scheme/scheme.go (CPU)."""
import pytest

from drand_amd import scheme as S


def test_lookup():
    s, ok = S.get_scheme_by_id("pedersen-bls-chained")
    assert ok and not s.decouple_prev_sig
    s, ok = S.get_scheme_by_id("pedersen-bls-unchained")
    assert ok and s.decouple_prev_sig
    s, ok = S.get_scheme_by_id("bls-unchained-on-g1")
    assert ok and s.decouple_prev_sig and s.sigs_on_g1
    assert not S.get_scheme_by_id("x")[1]


def test_default_and_errors(monkeypatch):
    assert S.get_scheme_by_id_with_default("").id == S.DEFAULT_SCHEME_ID
    with pytest.raises(ValueError, match=r"scheme \[bogus\] is not valid"):
        S.get_scheme_by_id_with_default("bogus")
    monkeypatch.setenv("SCHEME_ID", "pedersen-bls-unchained")
    assert S.get_scheme_from_env().id == S.UNCHAINED_SCHEME_ID
    monkeypatch.setenv("SCHEME_ID", "bogus")
    with pytest.raises(ValueError):
        S.get_scheme_from_env()
    assert S.list_schemes()[:2] == ["pedersen-bls-chained", "pedersen-bls-unchained"]
