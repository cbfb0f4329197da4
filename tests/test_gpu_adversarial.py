"""GPU parity on adversarial values: the F29 NTT passes and the F29 MSM accumulation on
the inputs whose limbs sit at the top of their range, against the C oracle, bit-exact.

Random inputs rarely push the lazily reduced F29 values (csrc/f29.h, bounds in
tools/f29_bounds.py) toward their worst cases.  These vectors do:
  * Fr data whose storage integers are all r - 1 (the largest value a stored element
    takes), canonical r - 1, alternating 0 / r - 1, and single spikes at the first, a
    middle and the last position -- through the FFT, lagrange_to_coeff, the coset
    extension (sparse first pass), extended_to_coeff and divide_by_vanishing_poly
    (reference: best_fft via poly/domain.rs:238,344; domain.rs:216-316);
  * MSM bases whose x (canonical, and the stored Montgomery integer) is within a few
    hundred of p, with r - 1 scalars, repeated points (every bucket's doubling branch)
    and P / -P pairs (the identity branch) -- generic and fixed-base paths
    (reference: best_multiexp via zal.rs:136-138).
The host-side worst-case test of the same arithmetic is tests/test_f29_host_cpu.py.
"""
import os
import sys

import numpy as np
import pytest

import _oracle as O
import h2g

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "py"))
import bn254_ref as B  # noqa: E402

pytestmark = pytest.mark.gpu

RM1 = B.R - 1


def _u64(v, n=4):
    return np.array([(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)], dtype=np.uint64)


def _storage(v):  # an element given by its stored (Montgomery) integer
    return _u64(v)


@pytest.fixture(scope="module", autouse=True)
def engine():
    h2g.init()
    yield
    h2g.shutdown()


def _vector(kind, n):
    out = np.zeros((n, 4), dtype=np.uint64)
    st_rm1 = _storage(RM1)                                # stored integer r - 1
    can_rm1 = O.fr_from_canonical(_u64(RM1))[0]           # the element r - 1
    if kind == "storage_rm1":
        out[:] = st_rm1
    elif kind == "canonical_rm1":
        out[:] = can_rm1
    elif kind == "alternating":
        out[1::2] = st_rm1
    elif kind == "alternating_canonical":
        out[::2] = can_rm1
    elif kind == "spikes":
        out[0] = st_rm1
        out[n // 2 + 1] = st_rm1
        out[n - 1] = st_rm1
    elif kind == "spike_last":
        out[n - 1] = can_rm1
    else:
        raise ValueError(kind)
    return out


KINDS = ["storage_rm1", "canonical_rm1", "alternating", "alternating_canonical", "spikes", "spike_last"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("k", [11, 13, 16, 19])
def test_fft_adversarial_vs_oracle(kind, k):
    """pass layouts of 3..6 stages and the last-pass variants, forward and inverse root"""
    a = _vector(kind, 1 << k)
    _, consts, _ = O.domain_constants(2, k)
    for w in (consts[0], consts[1]):
        assert np.array_equal(h2g.fft(a, w), O.fft(a, w, 8)), (kind, k)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("j,k", [(3, 11), (3, 14), (5, 12), (3, 17)])
def test_domain_maps_adversarial_vs_oracle(kind, j, k):
    d = h2g.Domain(j, k)
    try:
        a = _vector(kind, 1 << k)
        coeff = d.lagrange_to_coeff(a)
        assert np.array_equal(coeff, O.lagrange_to_coeff(a, j, k, 8)), kind
        # the coset extension of the adversarial vector itself (sparse first pass)
        assert np.array_equal(d.coeff_to_extended(a), O.coeff_to_extended(a, j, k, 8)), kind
        h = _vector(kind, d.extended_len)
        assert np.array_equal(d.extended_to_coeff(h), O.extended_to_coeff(h, j, k, 8)), kind
        assert np.array_equal(d.divide_by_vanishing_poly(h), O.divide_by_vanishing_poly(h, j, k)), kind
    finally:
        d.close()


def _points_near_p(count, stored):
    """affine points whose x is p - 1, p - 2, ... (canonical x, or the stored Montgomery
    integer when `stored`), the larger square root as y; G1 has cofactor 1, so every curve
    point is in the group"""
    pts, d = [], 1
    rinv = pow(1 << 256, -1, B.P)
    while len(pts) < count:
        xs = B.P - d
        x = xs * rinv % B.P if stored else xs
        d += 1
        rhs = (x * x * x + B.G1_B) % B.P
        if pow(rhs, (B.P - 1) // 2, B.P) != 1:
            continue
        y = B.fq_sqrt(rhs)
        y = max(y, B.P - y)
        assert B.g1_on_curve((x, y))
        pts.append((x, y))
    return pts


def _bases(pts):
    return np.array([B.g1_affine_mont_limbs(p) for p in pts], dtype=np.uint64)


@pytest.mark.parametrize("stored", [False, True], ids=["x_canonical_near_p", "x_stored_near_p"])
@pytest.mark.parametrize("scal", ["rminus1", "random", "alternating"])
def test_msm_points_near_p_vs_oracle(stored, scal):
    pts = _points_near_p(64, stored)
    # 64 distinct points, each repeated, and each followed somewhere by its negation: equal
    # points meet in a bucket (the doubling branch of the mixed addition), P and -P cancel
    neg = [B.g1_neg(p) for p in pts]
    base_pts = (pts * 40 + neg * 8)[:2048 + 512]
    bases = _bases(base_pts)
    n = len(bases)
    r = np.random.default_rng(31 + stored)
    if scal == "rminus1":
        sc = np.tile(O.fr_from_canonical(_u64(RM1)), (n, 1))
    elif scal == "random":
        sc = O.random_fr(r, n)
    else:
        sc = np.zeros((n, 4), dtype=np.uint64)
        sc[::2] = O.fr_from_canonical(_u64(RM1))[0]
        sc[1::2] = _storage(RM1)
    want = O.msm_best(sc, bases, 8)
    assert np.array_equal(h2g.msm(sc, bases), want)
    hb = h2g.base_descriptor(bases)  # the fixed-base windows (one shared bucket set)
    try:
        assert np.array_equal(h2g.msm_with_cached_base(sc, hb), want)
    finally:
        h2g.descriptor_free(hb)
    for wb in (4, 13):
        dsc, dbs, dout = h2g.DevBuf.from_array(sc), h2g.DevBuf.from_array(bases), h2g.DevBuf(64)
        try:
            h2g.msm_dev(dsc.ptr, dbs.ptr, n, dout.ptr, window_bits=wb)
            assert np.array_equal(dout.download(8), want), wb
        finally:
            for b in (dsc, dbs, dout):
                b.close()


def test_msm_single_point_all_buckets_near_p():
    """one point near p with every scalar r - 1: every window's top bucket holds all n
    copies (the big-bucket combine on repeated doublings)"""
    p = _points_near_p(1, True)[0]
    n = 4096
    bases = np.tile(_bases([p]), (n, 1))
    sc = np.tile(O.fr_from_canonical(_u64(RM1)), (n, 1))
    want = O.msm_best(sc, bases, 8)
    assert np.array_equal(want, O.g1_mul(_bases([p])[0], O.fr_from_canonical(_u64((n * RM1) % B.R))[0]))
    assert np.array_equal(h2g.msm(sc, bases), want)


def test_msm_repeated_point_beyond_the_repair_list():
    """2^17 copies of one point with one scalar: every chunk of the accumulation meets
    p == q, more chunks than the repair list holds (msm_acc.hip MSM_REPAIR_CAP), so the
    repair launch redoes every chunk -- generic and fixed-base paths, against the oracle"""
    p = _points_near_p(1, False)[0]
    n = 1 << 17
    bases = np.tile(_bases([p]), (n, 1))
    r = np.random.default_rng(77)
    sc = np.tile(O.random_fr(r, 1), (n, 1))
    want = O.msm_best(sc, bases, 8)
    assert np.array_equal(h2g.msm(sc, bases), want)
    hb = h2g.base_descriptor(bases)
    try:
        assert np.array_equal(h2g.msm_with_cached_base(sc, hb), want)
    finally:
        h2g.descriptor_free(hb)


@pytest.mark.parametrize("kind", ["nibbles", "sparse", "one_window_dense"])
@pytest.mark.parametrize("lg", [14, 17])
def test_msm_few_entries_device_chunk_length(kind, lg):
    """scalars that fill a fraction of the entry bound n W: 4-bit values (one window of
    W), 1 % nonzero, and 2^16-bounded values -- the partition's last scan then picks a
    shorter chunk length on the device (msm_part.h msm_chunk_len_dev) and every later
    kernel reads it; generic and fixed-base paths, against the oracle"""
    n = 1 << lg
    r = np.random.default_rng(90 + lg)
    bases = h2g.DevBuf(n * 64)
    try:
        h2g.srs_setup_dev(O.random_fr(r, 1)[0], n, bases.ptr)
        bs = bases.download((n, 8))
    finally:
        bases.close()
    if kind == "nibbles":
        vals = r.integers(0, 16, size=n)
    elif kind == "sparse":
        vals = np.where(r.random(n) < 0.01, r.integers(1, 1 << 62, size=n), 0)
    else:
        vals = r.integers(1, 1 << 16, size=n)
    can = np.zeros((n, 4), dtype=np.uint64)
    can[:, 0] = vals.astype(np.uint64)
    sc = O.fr_from_canonical(can)
    want = O.msm_best(sc, bs, 8)
    assert np.array_equal(h2g.msm(sc, bs), want), kind
    hb = h2g.base_descriptor(bs)
    try:
        assert np.array_equal(h2g.msm_with_cached_base(sc, hb), want), kind
    finally:
        h2g.descriptor_free(hb)


@pytest.mark.parametrize("kind", ["nibbles", "mixed", "random"])
def test_msm_large_skewed_two_partition_paths(kind):
    """large MSMs with skewed scalars, two partition paths on one workspace: 4-bit scalars
    put every entry into one coarse bin, half 4-bit / half random skews some bins, random
    scalars none -- fixed-base at 2^22 points (13 windows, the unstaged fine pass)
    interleaved with generic MSMs at 2^21 points (15 windows, the staged one), against the
    oracle.  (Written for a one-pass partition into capacity bins, measured slower and
    removed: profiles/r06/cap/.)"""
    r = np.random.default_rng({"nibbles": 11, "mixed": 12, "random": 13}[kind])
    for lg, fixed in ((21, False), (22, True)):
        n = 1 << lg
        bases = h2g.DevBuf(n * 64)
        try:
            h2g.srs_setup_dev(O.random_fr(r, 1)[0], n, bases.ptr)
            bs = bases.download((n, 8))
        finally:
            bases.close()
        if kind == "random":
            sc = O.random_fr(r, n)
        else:
            can = np.zeros((n, 4), dtype=np.uint64)
            can[:, 0] = r.integers(0, 16, size=n).astype(np.uint64)
            sc = O.fr_from_canonical(can)
            if kind == "mixed":
                sc[: n // 2] = O.random_fr(r, n // 2)
        want = O.msm_best(sc, bs, 16)
        if fixed:
            hb = h2g.base_descriptor(bs)
            try:
                got = h2g.msm_with_cached_base(sc, hb)
            finally:
                h2g.descriptor_free(hb)
        else:
            got = h2g.msm(sc, bs)
        assert np.array_equal(got, want), (kind, lg, fixed)
