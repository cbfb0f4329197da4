"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and
the C restatement oracle, bit-exact (integer modular arithmetic).

At sizes the oracle finishes in seconds the comparison is element-for-element;
at BASELINE sizes (2^20..2^24) size-independent properties are used:
  MSM  : sum_i c_i [s^i]G == [c(s)]G  (SRS structure; c(s) by the CPU oracle)
  NTT  : ifft(fft(a)) == a, and fft(a)[j] == a(w^j) at sampled j (CPU Horner)
"""
import numpy as np
import pytest

import _oracle as O
import h2g

pytestmark = pytest.mark.gpu

GEN = np.array([0xd35d438dc58f0d9d, 0x0a78eb28f5c70b3d, 0x666ea36f7879462c, 0x0e0a77c19a07df2f,
                0xa6ba871b8b1e1b3a, 0x14f1d651eb8e167b, 0xccdd46def0f28c58, 0x1c14ef83340fbe5e], dtype=np.uint64)


@pytest.fixture(scope="module", autouse=True)
def engine():
    h2g.init()
    yield
    h2g.shutdown()


def rng(seed=1):
    return np.random.default_rng(seed)


# ---------------------------------------------------------------- MSM
def test_msm_golden_all_cases(golden):
    g = golden["msm"]
    for name in g["__names"]:
        got = h2g.msm(g[f"{name}__scalars"], g[f"{name}__bases"])
        assert np.array_equal(got, g[f"{name}__result"]), name


def test_msm_descriptor_api(golden):
    """MsmAccel caching API (zal.rs:83-102) == msm()."""
    g = golden["msm"]
    sc, bs = g["srs_random_k10__scalars"], g["srs_random_k10__bases"]
    want = g["srs_random_k10__result"]
    hb = h2g.base_descriptor(bs)
    hc = h2g.coeffs_descriptor(sc)
    try:
        assert np.array_equal(h2g.msm_with_cached_base(sc, hb), want)
        assert np.array_equal(h2g.msm_with_cached_scalars(hc, bs), want)
        assert np.array_equal(h2g.msm_with_cached_inputs(hc, hb), want)
        # prefix of a registered SRS, as commit_lagrange uses &g_lagrange[0..n]
        n = 256
        assert np.array_equal(h2g.msm_with_cached_base(sc[:n], hb, 0), O.msm_best(sc[:n], bs[:n], 8))
        assert np.array_equal(h2g.msm_with_cached_base(sc[:n], hb, 100), O.msm_best(sc[:n], bs[100:100 + n], 8))
    finally:
        h2g.descriptor_free(hb)
        h2g.descriptor_free(hc)
    with pytest.raises(h2g.H2GError):
        h2g.msm_with_cached_base(sc, 987654)


def _srs(n, s):
    d = h2g.DevBuf(n * 64)
    h2g.srs_setup_dev(s, n, d.ptr)
    return d


def test_srs_setup_matches_golden(golden):
    g = golden["msm"]
    want = g["srs_random_k10__bases"]
    d = _srs(len(want), g["srs_s"])
    assert np.array_equal(d.download((len(want), 8)), want)


@pytest.mark.parametrize("k", [11, 14, 16])
def test_msm_random_vs_oracle(k):
    r = rng(k)
    n = 1 << k
    s = O.random_fr(r, 1)[0]
    bases = _srs(n, s).download((n, 8))
    sc = O.random_fr(r, n)
    assert np.array_equal(h2g.msm(sc, bases), O.msm_best(sc, bases, 8))


@pytest.mark.parametrize("dist", ["ones", "small", "repeated", "sparse", "rminus1", "powers"])
def test_msm_skewed_distributions(dist):
    """Skewed scalars (many equal digits) exercise the big-bucket path."""
    r = rng(7)
    n = 1 << 13
    s = O.random_fr(r, 1)[0]
    bases = _srs(n, s).download((n, 8))
    if dist == "ones":
        sc = O.fr_from_canonical(np.tile(np.array([1, 0, 0, 0], dtype=np.uint64), (n, 1)))
    elif dist == "small":
        c = np.zeros((n, 4), dtype=np.uint64)
        c[:, 0] = r.integers(0, 16, size=n).astype(np.uint64)
        sc = O.fr_from_canonical(c)
    elif dist == "repeated":
        sc = np.tile(O.random_fr(r, 3), (n // 3 + 1, 1))[:n].copy()
    elif dist == "sparse":
        sc = O.random_fr(r, n)
        sc[r.random(n) < 0.9] = 0
    elif dist == "rminus1":
        rm1 = O.fr_from_canonical(np.array([0x43e1f593f0000000, 0x2833e84879b97091, 0xb85045b68181585d,
                                            0x30644e72e131a029], dtype=np.uint64))
        sc = np.tile(rm1, (n, 1))
    else:
        c = np.zeros((n, 4), dtype=np.uint64)
        bit = r.integers(0, 253, size=n)
        for i, b in enumerate(bit):
            c[i, b // 64] = np.uint64(1) << np.uint64(b % 64)
        sc = O.fr_from_canonical(c)
    want = O.msm_best(sc, bases, 8)
    assert np.array_equal(h2g.msm(sc, bases), want), dist
    # fixed-base windows (one shared bucket set): the same skew through the descriptor path
    hb = h2g.base_descriptor(bases)
    try:
        assert np.array_equal(h2g.msm_with_cached_base(sc, hb), want), dist
    finally:
        h2g.descriptor_free(hb)


@pytest.mark.parametrize("window_bits", [4, 9, 13, 17])
def test_msm_window_sizes(window_bits):
    r = rng(window_bits)
    n = 3000  # not a power of two
    s = O.random_fr(r, 1)[0]
    bases = _srs(n, s).download((n, 8))
    sc = O.random_fr(r, n)
    want = O.msm_best(sc, bases, 8)
    dsc, dbs, dout = h2g.DevBuf.from_array(sc), h2g.DevBuf.from_array(bases), h2g.DevBuf(64)
    h2g.msm_dev(dsc.ptr, dbs.ptr, n, dout.ptr, window_bits=window_bits)  # device-side final combine
    assert np.array_equal(dout.download(8), want)
    assert np.array_equal(h2g.msm_dev_host(dsc.ptr, dbs.ptr, n, window_bits), want)  # host-side combine


@pytest.mark.parametrize("k", [20, 22])
def test_msm_full_size_srs_identity(k):
    """sum_i c_i [s^i] G == [c(s)] G at BASELINE sizes (no O(n) CPU MSM needed)."""
    r = rng(100 + k)
    n = 1 << k
    s = O.random_fr(r, 1)[0]
    dbs = _srs(n, s)
    sc = O.random_fr(r, n)
    dsc = h2g.DevBuf.from_array(sc)
    got = h2g.msm_dev_host(dsc.ptr, dbs.ptr, n)
    want = O.g1_mul(GEN, O.eval_poly(sc, s))
    assert np.array_equal(got, want)


# ---------------------------------------------------------------- NTT
def test_fft_golden(golden):
    g = golden["ntt"]
    for name in g["__names"]:
        got = h2g.fft(g[f"{name}__input"], g[f"{name}__omega"])
        assert np.array_equal(got, g[f"{name}__fft"]), name


@pytest.mark.parametrize("k", [11, 12, 13, 15, 16, 17, 18, 19, 20])
def test_fft_random_vs_oracle(k):
    r = rng(k)
    a = O.random_fr(r, 1 << k)
    _, consts, _ = O.domain_constants(2, k)
    w = consts[0]
    assert np.array_equal(h2g.fft(a, w), O.fft(a, w, 8)), k


def test_domain_golden(golden):
    g = golden["ntt"]
    for name in g["__domains"]:
        j, k, ek = (int(v) for v in g[f"{name}__meta"])
        d = h2g.Domain(j, k)
        try:
            assert d.extended_k == ek
            assert np.array_equal(d.consts, g[f"{name}__consts"]), name
            assert np.array_equal(d.lagrange_to_coeff(g[f"{name}__lagrange"]), g[f"{name}__coeff"]), name
            assert np.array_equal(d.coeff_to_extended(g[f"{name}__coeff"]), g[f"{name}__extended"]), name
            assert np.array_equal(d.divide_by_vanishing_poly(g[f"{name}__ext_in"]), g[f"{name}__divided"]), name
            assert np.array_equal(d.extended_to_coeff(g[f"{name}__ext_in"]), g[f"{name}__ext_to_coeff"]), name
        finally:
            d.close()


@pytest.mark.parametrize("j,k", [(3, 11), (3, 14), (5, 12), (3, 18), (9, 13)])
def test_domain_ops_vs_oracle(j, k):
    r = rng(j * 100 + k)
    d = h2g.Domain(j, k)
    try:
        lag = O.random_fr(r, 1 << k)
        coeff = d.lagrange_to_coeff(lag)
        assert np.array_equal(coeff, O.lagrange_to_coeff(lag, j, k, 8))
        ext = d.coeff_to_extended(coeff)
        assert np.array_equal(ext, O.coeff_to_extended(coeff, j, k, 8))
        h = O.random_fr(r, d.extended_len)
        assert np.array_equal(d.divide_by_vanishing_poly(h), O.divide_by_vanishing_poly(h, j, k))
        assert np.array_equal(d.extended_to_coeff(h), O.extended_to_coeff(h, j, k, 8))
        rt = d.extended_to_coeff(ext)
        assert np.array_equal(rt[: 1 << k], coeff) and not rt[1 << k:].any()
    finally:
        d.close()


@pytest.mark.parametrize("k", [22, 24])
def test_fft_full_size_properties(k):
    r = rng(k)
    n = 1 << k
    a = O.random_fr(r, n)
    _, consts, _ = O.domain_constants(2, k)
    w, winv = consts[0], consts[1]
    da = h2g.DevBuf.from_array(a)
    h2g.fft_dev(da.ptr, k, w)
    y = da.download((n, 4))
    # sampled evaluations y_j = a(w^j)
    for j in [0, 1, 2, n // 2 + 3, n - 1, int(r.integers(0, n))]:
        x = _fr_pow(w, j)  # w^j by square-and-multiply on the oracle
        assert np.array_equal(y[j], O.eval_poly(a, x)), j
    # inverse transform round trip (times n)
    h2g.fft_dev(da.ptr, k, winv)
    back = da.download((n, 4))
    ninv = O.domain_constants(2, k)[1][6]
    assert np.array_equal(O.scale(back, ninv), a)


def _fr_pow(x, e):
    acc = O.fr_from_canonical(np.array([1, 0, 0, 0], dtype=np.uint64))[0]
    base = x.copy()
    while e:
        if e & 1:
            acc = O.binop("or_fr_mul", acc.reshape(1, 4), base.reshape(1, 4))[0]
        base = O.binop("or_fr_mul", base.reshape(1, 4), base.reshape(1, 4))[0]
        e >>= 1
    return acc


# ---------------------------------------------------------------- poly ops
def test_poly_golden(golden):
    g = golden["poly"]
    for name in g["__names"]:
        a, b, x = g[f"{name}__a"], g[f"{name}__b"], g[f"{name}__x"]
        assert np.array_equal(h2g.fr_op(h2g.OP_ADD, a, b), g[f"{name}__add"])
        assert np.array_equal(h2g.fr_op(h2g.OP_SUB, a, b), g[f"{name}__sub"])
        assert np.array_equal(h2g.fr_op(h2g.OP_MUL, a, b), g[f"{name}__mul"])
        assert np.array_equal(h2g.fr_op(h2g.OP_SCALE, a, c=x), g[f"{name}__scale"])
        assert np.array_equal(h2g.batch_invert(a), g[f"{name}__inv"])
        assert np.array_equal(h2g.prefix_product(a), g[f"{name}__prefix_product"])


@pytest.mark.parametrize("n", [1, 63, 4097, 1 << 16, (1 << 20) + 5])
def test_poly_ops_vs_oracle(n):
    r = rng(n)
    a, b = O.random_fr(r, n), O.random_fr(r, n)
    c = O.random_fr(r, 1)[0]
    a[:: 7] = 0  # zeros must stay zero under batch inversion
    assert np.array_equal(h2g.fr_op(h2g.OP_SUB_CONST, a, c=c), O.binop("or_fr_sub", a, np.tile(c, (n, 1))))
    assert np.array_equal(h2g.fr_op(h2g.OP_ADD_CONST, a, c=c), O.binop("or_fr_add", a, np.tile(c, (n, 1))))
    assert np.array_equal(h2g.fr_op(h2g.OP_AXPY, a, b, c), O.binop("or_fr_add", O.scale(a, c), b))
    assert np.array_equal(h2g.batch_invert(a), O.batch_invert(a))
    b[:: 5] = O.fr_from_canonical(np.array([1, 0, 0, 0], dtype=np.uint64))[0]
    assert np.array_equal(h2g.prefix_product(b), O.prefix_product(b))


def test_batch_invert_edge_values():
    """the divsteps inversion (bn254.h inv_by) on values at the edges of its limb ranges:
    a one-element batch inverts the element itself (inv_regs_kernel), against the oracle"""
    R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
    vals = [1, 2, 3, R - 1, R - 2, (R - 1) // 2, 1 << 30, (1 << 30) - 1, 1 << 60, 1 << 240, (1 << 253) + 12345,
            0x3fffffff3fffffff3fffffff3fffffff3fffffff3fffffff3fffffff3fff]
    for v in vals:
        limbs = np.array([[(v >> (64 * i)) & (2**64 - 1) for i in range(4)]], dtype=np.uint64)
        a = O.fr_from_canonical(limbs)
        assert np.array_equal(h2g.batch_invert(a), O.batch_invert(a)), hex(v)
    # and every value of a longer batch at once (the middle level inverts 16-element products)
    a = O.fr_from_canonical(np.array([[(v >> (64 * i)) & (2**64 - 1) for i in range(4)] for v in vals * 50],
                                     dtype=np.uint64))
    assert np.array_equal(h2g.batch_invert(a), O.batch_invert(a))


# ---------------------------------------------------------------- fixed-base MSM (resident bases)
def _skewed(dist, r, n):
    if dist == "random":
        return O.random_fr(r, n)
    if dist == "ones":
        return O.fr_from_canonical(np.tile(np.array([1, 0, 0, 0], dtype=np.uint64), (n, 1)))
    if dist == "zeros":
        return np.zeros((n, 4), dtype=np.uint64)
    if dist == "rminus1":
        rm1 = O.fr_from_canonical(np.array([0x43e1f593f0000000, 0x2833e84879b97091, 0xb85045b68181585d,
                                            0x30644e72e131a029], dtype=np.uint64))
        return np.tile(rm1, (n, 1))
    sc = O.random_fr(r, n)   # sparse
    sc[r.random(n) < 0.9] = 0
    return sc


@pytest.mark.parametrize("window_bits", [0, 3, 8, 13, 20, 22])
@pytest.mark.parametrize("dist", ["random", "ones", "zeros", "rminus1", "sparse"])
def test_msm_fixed_base_vs_oracle(window_bits, dist):
    """Fixed-base windows (h2g_msm_base_descriptor_dev) incl. offsets into the table."""
    r = rng(window_bits * 7 + len(dist))
    N = 5000
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(N, s)
    bases = bases_dev.download((N, 8))
    h = h2g.base_descriptor_dev(bases_dev.ptr, N, window_bits)
    try:
        for off, n in ((0, N), (0, 1024), (1234, 3000), (N - 2, 2), (7, 1)):
            sc = _skewed(dist, r, n)
            d_sc = h2g.DevBuf.from_array(sc)
            got = h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, off)
            want = O.msm_best(sc, bases[off:off + n], 8)
            assert np.array_equal(got, want), (dist, window_bits, off, n)
            d_sc.close()
        with pytest.raises(h2g.H2GError):
            h2g.msm_with_cached_base_dev(0, 10, h, N - 5)
    finally:
        h2g.descriptor_free(h)
        bases_dev.close()


def test_msm_fixed_base_srs_identity_2_20():
    """2^20 fixed-base MSM over the SRS: sum c_i [s^i]G == [c(s)]G."""
    r = rng(20)
    n = 1 << 20
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(n, s)
    h = h2g.base_descriptor_dev(bases_dev.ptr, n, 0)
    sc = O.random_fr(r, n)
    d_sc = h2g.DevBuf.from_array(sc)
    got = h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, 0)
    cs = O.eval_poly(sc, s)
    want = O.g1_mul(GEN, cs)
    assert np.array_equal(got, want)
    h2g.descriptor_free(h)
    d_sc.close()
    bases_dev.close()


@pytest.mark.parametrize("window_bits", [0, 9, 16])
@pytest.mark.parametrize("dist", ["random", "ones", "sparse", "rminus1"])
def test_msm_fixed_base_windows_and_skew(window_bits, dist):
    """Fixed-base MSMs over a sub-slice of the bases at several window sizes and skewed
    scalar distributions (ones put every digit in bucket 0: one coarse bin holds all
    entries) == the oracle's best_multiexp."""
    r = rng(31 + window_bits + len(dist))
    N = 5000
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(N, s)
    bases = bases_dev.download((N, 8))
    h = h2g.base_descriptor_dev(bases_dev.ptr, N, window_bits)
    try:
        for off, n in ((0, N), (1234, 3000)):
            sc = _skewed(dist, r, n)
            d_sc = h2g.DevBuf.from_array(sc)
            got = h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, off)
            assert np.array_equal(got, O.msm_best(sc, bases[off:off + n], 8)), (window_bits, dist, off)
            d_sc.close()
    finally:
        h2g.descriptor_free(h)
        bases_dev.close()


@pytest.mark.parametrize("k", [22, 24])
def test_msm_fixed_base_srs_identity_at_size(k):
    """The bench's MSMs at size: 2^22 (c = 20, bit-plane reduction) and 2^24 (c = 22, the
    rscale reduction); sum c_i [s^i]G == [c(s)]G."""
    r = rng(400 + k)
    n = 1 << k
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(n, s)
    sc = O.random_fr(r, n)
    want = O.g1_mul(GEN, O.eval_poly(sc, s))
    d_sc = h2g.DevBuf.from_array(sc)
    h = h2g.base_descriptor_dev(bases_dev.ptr, n, 0)
    try:
        assert np.array_equal(h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, 0), want)
    finally:
        h2g.descriptor_free(h)
        d_sc.close()
        bases_dev.close()


@pytest.mark.parametrize("k", [18, 20])
def test_msm_equal_scalars_srs_identity(k):
    """One scalar value for every point (a constant column): each window's digits all
    land in one bucket of n entries, cut into items and combined (msm_big_item_kernel,
    msm_big_combine_kernel).  sum_i c [s^i]G == [c sum_i s^i]G."""
    r = rng(300 + k)
    n = 1 << k
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(n, s)
    sc = np.tile(O.random_fr(r, 1), (n, 1))
    want = O.g1_mul(GEN, O.eval_poly(sc, s))
    d_sc = h2g.DevBuf.from_array(sc)
    assert np.array_equal(h2g.msm_dev_host(d_sc.ptr, bases_dev.ptr, n), want)
    h = h2g.base_descriptor_dev(bases_dev.ptr, n, 0)
    try:
        assert np.array_equal(h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, 0), want)
    finally:
        h2g.descriptor_free(h)
        d_sc.close()
        bases_dev.close()


@pytest.mark.parametrize("frac", [0.5, 0.97])
def test_msm_mixed_big_and_small_bins_srs_identity(frac):
    """A constant run of scalars among random ones at 2^20 points: the constant's digits
    fill a few coarse bins past the per-bin kernel's capacity (tile path, cursors rebased
    onto their bins) while the random ones fill every bin below it (per-bin kernel) --
    both partition paths in one MSM, generic and fixed-base windows."""
    r = rng(400 + int(frac * 100))
    n = 1 << 20
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(n, s)
    sc = O.random_fr(r, n)
    m = int(n * frac)
    sc[:m] = O.random_fr(r, 1)[0]
    want = O.g1_mul(GEN, O.eval_poly(sc, s))
    d_sc = h2g.DevBuf.from_array(sc)
    assert np.array_equal(h2g.msm_dev_host(d_sc.ptr, bases_dev.ptr, n), want)
    h = h2g.base_descriptor_dev(bases_dev.ptr, n, 0)
    try:
        assert np.array_equal(h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, 0), want)
    finally:
        h2g.descriptor_free(h)
        d_sc.close()
        bases_dev.close()


def test_msm_profile_counts_sorted_entries():
    """h2g_profile_msm_entries: the accumulation's mixed additions are the nonzero signed
    digits -- n for scalars equal to 1 (one digit each), 0 for zeros, W n for random
    scalars up to the rare zero digit (what the bench's modmul rates divide by)."""
    r = rng(77)
    n = 4096
    s = O.random_fr(r, 1)[0]
    bases_dev = _srs(n, s)
    h = h2g.base_descriptor_dev(bases_dev.ptr, n, 0)
    try:
        import bn254_ref as B
        one = np.tile(np.asarray(B.fr_mont_limbs(1), dtype=np.uint64), (n, 1))
        cases = ((one, lambda e: e == n), (np.zeros((n, 4), dtype=np.uint64), lambda e: e == 0))
        for sc, ok in cases:
            d_sc = h2g.DevBuf.from_array(sc)
            h2g.profile_enable(True)
            h2g.msm_with_cached_base_dev(d_sc.ptr, n, h, 0)
            h2g.profile_enable(False)
            calls, _, union = h2g.profile_msm_collect(with_union=True)
            assert calls == 1 and ok(union["entries"]), union
            d_sc.close()
    finally:
        h2g.descriptor_free(h)
        bases_dev.close()


# ---------------------------------------------------------------- counts -> offsets scan
@pytest.mark.parametrize("n", [1, 4096, 4097, (1 << 24) + 12345, (1 << 25) + 7])
def test_u32_exclusive_scan_any_length(n):
    """h2g_u32_exclusive_scan_dev (the lookup sort's and compactions' scan): exact against
    numpy at lengths around the 4096-element block and past 2^24, where the block sums
    no longer fit one block and are scanned recursively (in place, as the sort uses it)."""
    r = rng(n % 1000)
    a = r.integers(0, 300, size=n, dtype=np.uint32)
    want = np.zeros(n, dtype=np.uint64)
    want[1:] = np.cumsum(a[:-1], dtype=np.uint64)
    want = (want & 0xffffffff).astype(np.uint32)
    d_in = h2g.DevBuf.from_array(a)
    d_out = h2g.DevBuf(a.nbytes)
    try:
        h2g.u32_exclusive_scan_dev(d_in.ptr, d_out.ptr, n)
        assert np.array_equal(d_out.download(n, np.uint32), want)
        h2g.u32_exclusive_scan_dev(d_in.ptr, d_in.ptr, n)  # in place
        assert np.array_equal(d_in.download(n, np.uint32), want)
    finally:
        d_in.close()
        d_out.close()
