"""Descriptor lifetimes through the C ABI (MsmAccel's CoeffsDescriptor / BaseDescriptor,
halo2_middleware/src/zal.rs:47-50,83-102): a descriptor owns device memory until
h2g_msm_descriptor_free, and freeing gives all of it back -- what the Rust shim's Drop
 relies on."""
import numpy as np
import pytest

import _oracle as O
import h2g

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def engine():
    h2g.init()
    yield
    h2g.shutdown()


def _free_bytes():
    return h2g.device_mem_info()[0]


def test_ten_thousand_descriptors_return_device_memory():
    r = np.random.default_rng(3)
    n = 256
    bases = h2g.DevBuf(n * 64)
    h2g.srs_setup_dev(O.random_fr(r, 1)[0], n, bases.ptr)
    bs = bases.download((n, 8))
    bases.close()
    sc = O.random_fr(r, n)
    want = O.msm_best(sc, bs, 4)

    def cycle(count):
        for i in range(count):
            h = h2g.base_descriptor(bs) if i % 2 else h2g.coeffs_descriptor(sc)
            h2g.descriptor_free(h)

    cycle(200)  # the runtime's own first-use allocations settle
    start = _free_bytes()
    cycle(10_000)
    after = _free_bytes()
    # descriptors held at once take memory (the measurement sees them) ...
    held = [h2g.base_descriptor(bs) for _ in range(200)]
    during = _free_bytes()
    assert np.array_equal(h2g.msm_with_cached_base(sc, held[-1]), want)
    for h in held:
        h2g.descriptor_free(h)
    end = _free_bytes()
    per_base = (start - during) / 200
    assert per_base > 8 * 1024, per_base  # a base descriptor keeps its fixed-base table
    # ... and 10^4 create / free cycles leak none of it (tolerance: the allocator's own
    # granularity, far below one descriptor per hundred cycles)
    assert start - after < 100 * per_base, (start, after, per_base)
    assert start - end < 100 * per_base, (start, end, per_base)
    with pytest.raises(h2g.H2GError):
        h2g.descriptor_free(held[0])  # freed once: the handle is gone
