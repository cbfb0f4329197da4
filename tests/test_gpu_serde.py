"""SerdeFormat::RawBytes and ::Processed serialisation of ParamsKZG and ProvingKey on the device path
(h2g_params_write/read, h2g_pk_write/read; helpers.rs:8-21, kzg/commitment.rs:166-267,
plonk.rs:73-129,311-359).  The byte layout is checked field by field against the
reference's writers (lengths, endianness, section order) and against the oracle
(SRS points, G2 points from big-integer arithmetic, Lagrange commitments of the fixed
columns, the permutation's sigma values); a key or params read back from the bytes
proves byte-identical proofs.  The reference's own round-trip test is
halo2_proofs/tests/serialization.rs:130-175 (pk RawBytes write -> read -> prove)."""
import copy

import numpy as np
import pytest

import _oracle as O
import bn254_ref as B
import h2g
import h2g_circuit as hc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2g.init()
    yield


def _u64(b):
    return np.frombuffer(bytes(b), dtype=np.uint64)


def test_params_roundtrip_and_layout():
    k = 6
    s_int, g, gl = O.srs(k)
    p = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    data = p.write()
    n = 1 << k
    assert len(data) == 4 + 2 * n * 64 + 2 * 128
    assert int.from_bytes(data[:4], "little") == k
    assert np.array_equal(_u64(data[4:4 + n * 64]).reshape(n, 8), g)
    assert np.array_equal(_u64(data[4 + n * 64:4 + 2 * n * 64]).reshape(n, 8), gl)
    g2 = _u64(data[4 + 2 * n * 64:4 + 2 * n * 64 + 128])
    sg2 = _u64(data[4 + 2 * n * 64 + 128:])
    assert list(g2) == B.g2_affine_mont_limbs(B.G2_GEN)
    assert list(sg2) == B.g2_affine_mont_limbs(B.g2_mul(B.G2_GEN, s_int))
    q = h2g.Params.read(data)
    dg, dgl = q.export()
    assert np.array_equal(dg, g) and np.array_equal(dgl, gl)
    a, b = q.g2()
    assert list(a) == list(g2) and list(b) == list(sg2)
    assert q.write() == data
    # a key and proof made with the read params are those of the original
    circ, wit = hc.simple_example(k)
    pk1, pk2 = h2g.ProvingKey(p, circ), h2g.ProvingKey(q, circ)
    assert pk1.create_proof(wit) == pk2.create_proof(wit) == O.create_proof(circ, wit, g, gl)
    for o in (pk1, pk2, p, q):
        o.close()


def test_params_read_checks():
    k = 4
    s_int, g, gl = O.srs(k)
    p = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    data = bytearray(p.write())
    p.close()
    bad_point = bytearray(data)
    bad_point[4 + 3 * 64 + 40] ^= 0x01  # y of g[3]: off the curve
    with pytest.raises(h2g.H2GError):
        h2g.Params.read(bytes(bad_point))
    h2g.Params.read(bytes(bad_point), h2g.RAW_BYTES_UNCHECKED).close()  # no checks
    unreduced = bytearray(data)
    unreduced[4 + 5 * 64:4 + 5 * 64 + 32] = b"\xff" * 32  # x of g[5] >= p
    with pytest.raises(h2g.H2GError):
        h2g.Params.read(bytes(unreduced))
    bad_g2 = bytearray(data)
    bad_g2[-1] ^= 0x01
    with pytest.raises(h2g.H2GError):
        h2g.Params.read(bytes(bad_g2))
    with pytest.raises(h2g.H2GError):
        h2g.Params.read(bytes(data[:-5]))  # truncated
    # created params have no G2 half until it is supplied
    q = h2g.Params(k, g, gl)
    with pytest.raises(h2g.H2GError):
        q.write()
    q.set_g2(B.g2_affine_mont_limbs(B.G2_GEN), B.g2_affine_mont_limbs(B.g2_mul(B.G2_GEN, s_int)))
    assert q.write() == bytes(data)
    q.close()


def _parse_pk(data, circ, ext):
    """ProvingKey::write layout, section by section (plonk.rs:73-86, 311-321)"""
    n = 1 << circ.k
    pos = 0

    def take(cnt):
        nonlocal pos
        out = data[pos:pos + cnt]
        assert len(out) == cnt
        pos += cnt
        return out

    def poly(length):
        assert int.from_bytes(take(4), "big") == length
        return _u64(take(length * 32)).reshape(length, 4)

    def polys(count, length):
        assert int.from_bytes(take(4), "big") == count
        return [poly(length) for _ in range(count)]

    assert take(1) == bytes([4]) and take(1) == bytes([circ.k])
    F = int.from_bytes(take(4), "little")
    assert F == circ.num_fixed
    P = len(circ.perm_columns)
    sec = {"fixed_com": _u64(take(64 * F)).reshape(F, 8), "perm_com": _u64(take(64 * P)).reshape(P, 8)}
    sec["l0"], sec["l_last"], sec["l_active"] = poly(ext), poly(ext), poly(ext)
    sec["fixed_values"], sec["fixed_polys"], sec["fixed_cosets"] = polys(F, n), polys(F, n), polys(F, ext)
    sec["sigma"], sec["sigma_polys"], sec["sigma_cosets"] = polys(P, n), polys(P, n), polys(P, ext)
    assert pos == len(data)
    return sec


PK_CASES = {
    "simple_k6": lambda: hc.simple_example(6),
    "mixed_k7": lambda: hc.mixed_circuit(7),
    "lookup_k8": lambda: hc.lookup_circuit(8),
    "c3_k9": lambda: hc.synthetic_c3(9, O.OracleOps),
}


@pytest.mark.parametrize("name", list(PK_CASES))
def test_pk_roundtrip_and_layout(name):
    circ, wit = PK_CASES[name]()
    k, n = circ.k, 1 << circ.k
    s_int, g, gl = O.srs(k)
    params = h2g.Params(k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    data = pk.write()
    ext = 1 << pk.extended_k
    sec = _parse_pk(data, circ, ext)
    fixed = np.asarray(circ.fixed_values, dtype=np.uint64).reshape(circ.num_fixed, n, 4)
    kg = O.Keygen(circ, wit, g, gl)
    j = pk.degree  # EvaluationDomain::new(j = cs degree, k)
    for i in range(circ.num_fixed):
        assert np.array_equal(sec["fixed_values"][i], fixed[i])
        assert np.array_equal(sec["fixed_polys"][i], O.lagrange_to_coeff(fixed[i], j, k))
        assert np.array_equal(sec["fixed_cosets"][i], O.coeff_to_extended(sec["fixed_polys"][i], j, k))
        assert np.array_equal(sec["fixed_com"][i], O.msm_best(fixed[i], gl, 8))  # commit_lagrange
    for i in range(len(circ.perm_columns)):
        assert np.array_equal(sec["sigma"][i], kg.sigma(i))
        assert np.array_equal(sec["perm_com"][i], O.msm_best(sec["sigma"][i], gl, 8))
    kg.close()
    unit = np.zeros((n, 4), dtype=np.uint64)
    unit[0] = hc.ints_to_mont([1])[0]
    assert np.array_equal(sec["l0"], O.coeff_to_extended(O.lagrange_to_coeff(unit, j, k), j, k))
    # read back: the arrays come from the bytes, the constraint system from the circuit
    bare = copy.copy(circ)  # fixed values and copies wiped: they must not be used
    bare.fixed_values = np.zeros_like(circ.fixed_values)
    bare.copies = np.zeros((0, 6), dtype=np.int32)
    # vk.transcript_repr (plonk.rs:189-200) is the caller's input here; the reference
    # derives it from the read vk, whose pinned form is the same as the original's
    bare.transcript_repr = circ.transcript_repr
    pk2 = h2g.ProvingKey(params, bare, data=data)
    assert pk2.write() == data
    want = O.create_proof(circ, wit, g, gl)
    assert pk.create_proof(wit) == want
    assert pk2.create_proof(wit) == want
    for o in (pk, pk2, params):
        o.close()


def test_pk_read_checks():
    circ, wit = hc.simple_example(5)
    s_int, g, gl = O.srs(5)
    params = h2g.Params(5, g, gl)
    pk = h2g.ProvingKey(params, circ)
    data = pk.write()
    pk.close()
    for bad in (b"\x05" + data[1:],                    # version byte
                data[:1] + bytes([6]) + data[2:],     # k
                data[:-1],                            # truncated
                data + b"\x00"):                      # trailing bytes
        with pytest.raises(h2g.H2GError):
            h2g.ProvingKey(params, circ, data=bad)
    unreduced = bytearray(data)
    off = len(data) - 32  # last element of the last sigma coset
    unreduced[off:off + 32] = b"\xff" * 32
    with pytest.raises(h2g.H2GError):
        h2g.ProvingKey(params, circ, data=bytes(unreduced))
    h2g.ProvingKey(params, circ, data=bytes(unreduced), fmt=h2g.RAW_BYTES_UNCHECKED).close()
    params.close()


# ---- SerdeFormat::Processed (helpers.rs:36-100): compressed points, canonical scalars ----


def _g1_int(limbs):
    """G1Affine raw limbs (8 u64, Montgomery) -> affine ints, None = identity"""
    limbs = [int(v) for v in limbs]
    if not any(limbs):
        return None
    return B.from_mont(B.from_limbs(limbs[:4]), B.P), B.from_mont(B.from_limbs(limbs[4:]), B.P)


def _g2_int(limbs):
    limbs = [int(v) for v in limbs]
    if not any(limbs):
        return None
    f = [B.from_mont(B.from_limbs(limbs[4 * i:4 * i + 4]), B.P) for i in range(4)]
    return (f[0], f[1]), (f[2], f[3])


def _fr_repr_bytes(arr):
    return b"".join(B.fr_to_repr(B.from_mont(B.from_limbs(row), B.R)) for row in arr)


def test_params_processed_layout_and_roundtrip():
    k = 6
    n = 1 << k
    s_int, g, gl = O.srs(k)
    p = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    raw = p.write()
    data = p.write(h2g.PROCESSED)
    want = (k.to_bytes(4, "little") + b"".join(B.g1_to_bytes(_g1_int(r)) for r in g)
            + b"".join(B.g1_to_bytes(_g1_int(r)) for r in gl)
            + B.g2_to_bytes(B.G2_GEN) + B.g2_to_bytes(B.g2_mul(B.G2_GEN, s_int)))
    assert len(data) == 4 + 2 * n * 32 + 2 * 64
    assert data == want
    q = h2g.Params.read(data, h2g.PROCESSED)
    dg, dgl = q.export()
    assert np.array_equal(dg, g) and np.array_equal(dgl, gl)
    assert q.write() == raw and q.write(h2g.PROCESSED) == data
    circ, wit = hc.simple_example(k)
    pk = h2g.ProvingKey(q, circ)
    assert pk.create_proof(wit) == O.create_proof(circ, wit, g, gl)
    for o in (pk, p, q):
        o.close()


def test_params_processed_read_checks():
    k = 4
    n = 1 << k
    s_int, g, gl = O.srs(k)
    p = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    data = p.write(h2g.PROCESSED)
    p.close()
    x = 1
    while B.fq_sqrt(x ** 3 + 3) is not None:
        x += 1
    cases = []
    for off in (4 + 3 * 32, 4 + n * 32 + 7 * 32):  # a point of g, a point of g_lagrange
        for enc in (B.P.to_bytes(32, "little"), x.to_bytes(32, "little"), bytes(31) + b"\x80"):
            bad = bytearray(data)
            bad[off:off + 32] = enc
            cases.append(bytes(bad))
    bad_g2 = bytearray(data)
    bad_g2[-64:-32] = B.P.to_bytes(32, "little")  # s_g2.x.c0 >= p
    cases.append(bytes(bad_g2))
    cases.append(data[:-3])
    for bad in cases:
        with pytest.raises(h2g.H2GError):
            h2g.Params.read(bad, h2g.PROCESSED)
    # a sign flip is a valid encoding of the negated point
    flip = bytearray(data)
    flip[4 + 2 * 32 + 31] ^= 0x80
    q = h2g.Params.read(bytes(flip), h2g.PROCESSED)
    dg, _ = q.export()
    assert _g1_int(dg[2]) == B.g1_neg(_g1_int(g[2]))
    q.close()


@pytest.mark.parametrize("name", ["simple_k6", "lookup_k8", "c3_k9"])
def test_pk_processed_layout_and_roundtrip(name):
    circ, wit = PK_CASES[name]()
    k, n = circ.k, 1 << circ.k
    s_int, g, gl = O.srs(k)
    params = h2g.Params(k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    raw = pk.write()
    ext = 1 << pk.extended_k
    sec = _parse_pk(raw, circ, ext)
    F, P = circ.num_fixed, len(circ.perm_columns)
    want = bytearray([4, k]) + F.to_bytes(4, "little")
    want += b"".join(B.g1_to_bytes(_g1_int(c)) for c in sec["fixed_com"])
    want += b"".join(B.g1_to_bytes(_g1_int(c)) for c in sec["perm_com"])

    def poly(a):
        return len(a).to_bytes(4, "big") + _fr_repr_bytes(a)

    def polys(v):
        return len(v).to_bytes(4, "big") + b"".join(poly(a) for a in v)

    want += poly(sec["l0"]) + poly(sec["l_last"]) + poly(sec["l_active"])
    want += polys(sec["fixed_values"]) + polys(sec["fixed_polys"]) + polys(sec["fixed_cosets"])
    want += polys(sec["sigma"]) + polys(sec["sigma_polys"]) + polys(sec["sigma_cosets"])
    data = pk.write(h2g.PROCESSED)
    assert data == bytes(want)
    pk2 = h2g.ProvingKey(params, circ, data=data, fmt=h2g.PROCESSED)
    assert pk2.write() == raw
    want_proof = O.create_proof(circ, wit, g, gl)
    assert pk2.create_proof(wit) == want_proof
    for o in (pk, pk2, params):
        o.close()


def test_pk_processed_read_checks():
    circ, wit = hc.simple_example(5)
    s_int, g, gl = O.srs(5)
    params = h2g.Params(5, g, gl)
    pk = h2g.ProvingKey(params, circ)
    data = pk.write(h2g.PROCESSED)
    pk.close()
    unreduced = bytearray(data)
    unreduced[-32:] = B.R.to_bytes(32, "little")  # last sigma coset element = r
    bad_com = bytearray(data)
    bad_com[6:38] = B.P.to_bytes(32, "little")  # the first fixed commitment's x = p
    for bad in (bytes(unreduced), bytes(bad_com), data[:-1], data + b"\x00"):
        with pytest.raises(h2g.H2GError):
            h2g.ProvingKey(params, circ, data=bad, fmt=h2g.PROCESSED)
    ok = bytearray(data)
    ok[-32:] = (B.R - 1).to_bytes(32, "little")  # r - 1 is a valid repr
    h2g.ProvingKey(params, circ, data=bytes(ok), fmt=h2g.PROCESSED).close()
    params.close()
