"""CPU-side checks of the C ABI library: it loads, exports every symbol that
include/h2g.h declares, and fails loudly (no CPU fallback) without a device."""
import ctypes

import numpy as np
import pytest

import h2g


def test_library_exports_every_header_symbol():
    L = h2g.lib()
    syms = h2g.header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # and the Python binding covers all of them
    assert set(syms) == set(h2g._SIGS), set(syms) ^ set(h2g._SIGS)


def test_abi_version():
    assert h2g.lib().h2g_abi_version() == 1


def test_calls_before_init_fail_loudly():
    a = np.zeros((4, 4), dtype=np.uint64)
    rc = h2g.lib().h2g_fr_batch_invert(h2g.p64(a), 4)
    assert rc == 4  # H2G_ERR_STATE
    assert b"h2g_init" in h2g.lib().h2g_last_error()


def test_host_point_add_matches_oracle(golden):
    import _oracle as O
    g = golden["msm"]
    pts = g["srs_random_k3__bases"]
    for i in range(len(pts) - 1):
        assert np.array_equal(h2g.g1_add_affine(pts[i], pts[i + 1]), O.g1_add(pts[i], pts[i + 1]))
    # doubling and identity handling
    assert np.array_equal(h2g.g1_add_affine(pts[1], pts[1]), O.g1_add(pts[1], pts[1]))
    z = np.zeros(8, dtype=np.uint64)
    assert np.array_equal(h2g.g1_add_affine(pts[2], z), pts[2])
