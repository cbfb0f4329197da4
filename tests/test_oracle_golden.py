"""Pin the C restatement oracle (oracle/c) against the golden fixtures made by
the independent Python big-int oracle (tests/golden/gen_golden.py) and against
public BN254 known answers.  CPU only."""
import os
import sys

import numpy as np
import pytest

import _oracle as O

sys.path.insert(0, os.path.join(O.REPO, "oracle", "py"))
import bn254_ref as B  # noqa: E402


def test_public_bn254_constants():
    # 2G for the BN254 G1 generator (1, 2): public known-answer value
    two_g = B.g1_add(B.G1_GEN, B.G1_GEN)
    assert two_g == (0x030644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD3,
                     0x15ED738C0E0A7C92E7845F96B2AE9C0A68A6A449E3538FC7FF3EBF7A5A18A2C4)
    assert B.ROOT_OF_UNITY == 0x03DDB9F5166D18B798865EA93DD31F743215CF6DD39329C8D34F1ED960C37C9C
    assert B.DELTA == 0x09226B6E22C6F0CA64EC26AAD4C86E715B5F898E5E963F25870E56BBE533E9A2
    assert pow(B.ROOT_OF_UNITY, 1 << 28, B.R) == 1 and pow(B.ROOT_OF_UNITY, 1 << 27, B.R) != 1
    assert pow(B.ZETA, 3, B.R) == 1 and B.ZETA != 1
    assert B.g1_mul(B.G1_GEN, B.R) is None  # r is the group order


def test_oracle_point_ops():
    g = np.array(B.g1_affine_mont_limbs(B.G1_GEN), dtype=np.uint64)
    assert O.lib().or_g1_is_on_curve(O._p(g)) == 1
    two = O.g1_add(g, g)
    assert list(two) == B.g1_affine_mont_limbs(B.g1_add(B.G1_GEN, B.G1_GEN))
    s = np.array(B.fr_mont_limbs(123456789), dtype=np.uint64)
    assert list(O.g1_mul(g, s)) == B.g1_affine_mont_limbs(B.g1_mul(B.G1_GEN, 123456789))


@pytest.mark.parametrize("algo", ["naive", "best1", "best4"])
def test_oracle_msm_golden(golden, algo):
    g = golden["msm"]
    for name in g["__names"]:
        sc, bs = g[f"{name}__scalars"], g[f"{name}__bases"]
        if algo == "naive" and len(sc) > 256:
            continue
        got = {"naive": lambda: O.msm_naive(sc, bs),
               "best1": lambda: O.msm_best(sc, bs, 1),
               "best4": lambda: O.msm_best(sc, bs, 4)}[algo]()
        assert np.array_equal(got, g[f"{name}__result"]), name


def test_oracle_srs_matches_golden(golden):
    g = golden["msm"]
    bs = g["srs_random_k5__bases"]
    assert np.array_equal(O.srs_powers(g["srs_s"], len(bs)), bs)


@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_fft_golden(golden, threads):
    g = golden["ntt"]
    for name in g["__names"]:
        got = O.fft(g[f"{name}__input"], g[f"{name}__omega"], threads)
        assert np.array_equal(got, g[f"{name}__fft"]), name


def test_oracle_domain_golden(golden):
    g = golden["ntt"]
    for name in g["__domains"]:
        j, k, ek = (int(v) for v in g[f"{name}__meta"])
        ek2, consts, t = O.domain_constants(j, k)
        assert ek2 == ek
        assert np.array_equal(consts, g[f"{name}__consts"]), name
        assert np.array_equal(t, g[f"{name}__t_evaluations"]), name
        assert np.array_equal(O.lagrange_to_coeff(g[f"{name}__lagrange"], j, k), g[f"{name}__coeff"]), name
        assert np.array_equal(O.coeff_to_extended(g[f"{name}__coeff"], j, k), g[f"{name}__extended"]), name
        assert np.array_equal(O.divide_by_vanishing_poly(g[f"{name}__ext_in"], j, k), g[f"{name}__divided"]), name
        assert np.array_equal(O.extended_to_coeff(g[f"{name}__ext_in"], j, k), g[f"{name}__ext_to_coeff"]), name
        rt = O.extended_to_coeff(g[f"{name}__extended"], j, k)
        assert np.array_equal(rt, g[f"{name}__roundtrip"]), name
        n = 1 << k
        assert np.array_equal(rt[:n], g[f"{name}__coeff"]) and not rt[n:].any()


def test_oracle_poly_golden(golden):
    g = golden["poly"]
    for name in g["__names"]:
        a, b, x = g[f"{name}__a"], g[f"{name}__b"], g[f"{name}__x"]
        assert np.array_equal(O.binop("or_fr_add", a, b), g[f"{name}__add"])
        assert np.array_equal(O.binop("or_fr_sub", a, b), g[f"{name}__sub"])
        assert np.array_equal(O.binop("or_fr_mul", a, b), g[f"{name}__mul"])
        assert np.array_equal(O.scale(a, x), g[f"{name}__scale"])
        assert np.array_equal(O.eval_poly(a, x), g[f"{name}__eval"])
        assert np.array_equal(O.batch_invert(a), g[f"{name}__inv"])
        assert np.array_equal(O.prefix_product(a), g[f"{name}__prefix_product"])
        if f"{name}__kate_in" in g:
            assert np.array_equal(O.kate_division(g[f"{name}__kate_in"], x), g[f"{name}__kate_q"])
