"""A rank's slab of the params and the prefix-summed Lagrange basis (csrc/prover.cpp
params_prefix): the windows of the basis P_i = L_0 + ... + L_i that the lookup
commitments use are built for the slab on the first set-2 MSM inside it -- what a shard
mode peer's serve loop runs (h2g_comm_serve) -- and never as the full-size table there
(ADVICE r05); h2g_params_set_slab itself builds no prefix windows.  The results are
checked against the oracle: sum_i s_i P_i = sum_j L_j (sum_{i >= j} s_i)."""
import numpy as np
import pytest

import _oracle as O
import h2g
import h2g_circuit as hc

pytestmark = pytest.mark.gpu

K = 14


@pytest.fixture(scope="module", autouse=True)
def engine():
    h2g.init()
    yield
    h2g.shutdown()


def _prefix_msm_ref(sc, gl, lo, hi):
    """sum_{i in [lo, hi)} s_i P_i over the Lagrange basis gl, through suffix sums"""
    n = hi - lo
    suf = np.zeros((hi, 4), dtype=np.uint64)
    acc = np.zeros((1, 4), dtype=np.uint64)
    for i in range(hi - 1, -1, -1):
        if i >= lo:
            acc = O.binop("or_fr_add", acc, sc[i - lo].reshape(1, 4))
        suf[i] = acc[0]
    assert n == len(sc)
    return O.msm_best(suf, gl[:hi], 8)


def test_slab_prefix_windows_are_built_lazily_for_the_slab_only():
    n = 1 << K
    params = h2g.Params(K, s=np.asarray(hc.fr_to_limbs(0xabcdef + K), dtype=np.uint64))
    try:
        g, gl = params.export()
        full0, slab0, fgp0, sgp0 = h2g.params_table_bytes(params)
        assert full0 > 0 and slab0 == 0 and fgp0 == 0 and sgp0 == 0
        lo, hi = n // 4, n // 2
        params.set_slab(lo, hi)
        full1, slab1, fgp1, sgp1 = h2g.params_table_bytes(params)
        assert slab1 > 0 and fgp1 == 0 and sgp1 == 0  # set_slab builds no prefix windows
        r = np.random.default_rng(5)
        sc = O.random_fr(r, hi - lo)
        d = h2g.DevBuf.from_array(sc)
        try:
            got, _ = h2g.params_msm_dev(params, 2, lo, hi - lo, d.ptr)  # a peer's set-2 request
        finally:
            d.close()
        full2, slab2, fgp2, sgp2 = h2g.params_table_bytes(params)
        assert sgp2 > 0 and fgp2 == 0, (sgp2, fgp2)  # the slab's windows, not the full table
        assert sgp2 < full0  # a quarter of the points
        assert np.array_equal(got, _prefix_msm_ref(sc, gl, lo, hi))
        # a set-2 MSM outside the slab needs the full windows (built then)
        sc2 = O.random_fr(r, n)
        d2 = h2g.DevBuf.from_array(sc2)
        try:
            got2, _ = h2g.params_msm_dev(params, 2, 0, n, d2.ptr)
        finally:
            d2.close()
        full3, slab3, fgp3, sgp3 = h2g.params_table_bytes(params)
        assert fgp3 > 0 and sgp3 == sgp2
        assert np.array_equal(got2, _prefix_msm_ref(sc2, gl, 0, n))
        params.set_slab(0, 0)  # no slab: its windows are released
        _, slab4, fgp4, sgp4 = h2g.params_table_bytes(params)
        assert slab4 == 0 and sgp4 == 0 and fgp4 == fgp3
    finally:
        params.close()
