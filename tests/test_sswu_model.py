"""The inversion-free SSWU + isogeny and the two-exponentiation Fp2 square
root the kernels implement (model: tools/sswu_model.py) agree with the
oracle's RFC 9380 map_to_curve_simple_swu + iso_map and with the oracle's
square test, including the w1 = 0 and zero cases an adversarial signature
encoding can reach."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))

import sswu_model as S  # noqa: E402
from oracle import bls12381 as B  # noqa: E402

P = B.P


def test_sswu_iso3_matches_oracle():
    rng = random.Random(1)
    for _ in range(120):
        u = (rng.randrange(P), rng.randrange(P))
        assert S.to_affine(S.sswu_iso3_jacobian(u)) == B.iso_map_g2(B.map_to_curve_sswu_g2(u))


def test_sswu_special_inputs():
    # u = 0 (den = 0 branch) and small values
    for u in [(0, 0), (1, 0), (0, 1), (P - 1, 0), (2, 3)]:
        assert S.to_affine(S.sswu_iso3_jacobian(u)) == B.iso_map_g2(B.map_to_curve_sswu_g2(u))


def test_fp2_sqrt_two_exponentiations():
    rng = random.Random(2)
    cases = [(rng.randrange(P), rng.randrange(P)) for _ in range(150)]
    cases += [(rng.randrange(P), 0) for _ in range(40)] + [(0, rng.randrange(P)) for _ in range(20)]
    cases += [(0, 0), (1, 0), (P - 1, 0), (4, 0)]
    for a in cases:
        r = S.fp2_sqrt(a)
        assert (r is not None) == B.f2_is_square(a), a
        if r is not None:
            assert B.f2_sqr(r) == (a[0] % P, a[1] % P)


def test_sswu_iso11_g1_matches_oracle():
    rng = random.Random(3)
    for u in [0, 1, P - 1] + [rng.randrange(P) for _ in range(150)]:
        assert S.g1_to_affine(S.sswu_iso11_jacobian(u)) == B.iso_map_g1(B.map_to_curve_sswu_g1(u))
