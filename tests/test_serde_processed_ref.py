"""SerdeFormat::Processed restatement (oracle/py/bn254_ref.py; helpers.rs:36-100): the
compressed G1/G2 encodings and canonical field elements round-trip, and the decoders refuse
what GroupEncoding::from_bytes / PrimeField::from_repr refuse.  CPU only; the device
writers and readers are compared with these in tests/test_gpu_serde.py.  halo2curves 0.6
is not vendored in the reference, so the flag convention is unpinned by a reference vector;
it is the encoding of every point in the proofs the verifier accepts."""
import random

import bn254_ref as B


def _pts(cnt, seed):
    r = random.Random(seed)
    return [B.g1_mul(B.G1_GEN, r.randrange(1, B.R)) for _ in range(cnt)]


def test_g1_roundtrip_and_sign():
    for pt in _pts(24, 1) + [None]:
        b = B.g1_to_bytes(pt)
        assert len(b) == 32
        assert B.g1_from_bytes(b) == (True, pt)
        if pt is not None:
            assert (b[31] >> 7) == (pt[1] & 1)
            neg = B.g1_neg(pt)
            nb = B.g1_to_bytes(neg)
            assert nb[:31] == b[:31] and (nb[31] ^ b[31]) == 0x80
            assert B.g1_from_bytes(nb) == (True, neg)


def test_g1_rejects():
    assert B.g1_from_bytes(B.P.to_bytes(32, "little"))[0] is False  # x = p (non-canonical)
    x = 1
    while B.fq_sqrt(x ** 3 + 3) is not None:  # the first x with no curve point
        x += 1
    assert B.g1_from_bytes(x.to_bytes(32, "little"))[0] is False
    assert B.fq_sqrt(3) is None  # x = 0 is no curve point: the all-zero encoding is unambiguous
    assert B.g1_from_bytes(bytes(31) + b"\x80")[0] is False  # x = 0 with the sign set


def test_g2_roundtrip():
    r = random.Random(2)
    for pt in [B.G2_GEN] + [B.g2_mul(B.G2_GEN, r.randrange(1, B.R)) for _ in range(4)] + [None]:
        b = B.g2_to_bytes(pt)
        assert len(b) == 64
        assert B.g2_from_bytes(b) == (True, pt)
    bad = bytearray(B.g2_to_bytes(B.G2_GEN))
    bad[0] ^= 1
    ok, _ = B.g2_from_bytes(bytes(bad))
    # a perturbed x is on the twist about half the time; when it is, the decoded point is on it
    assert ok is False or B.g2_on_curve(B.g2_from_bytes(bytes(bad))[1])


def test_fr_repr():
    assert B.fr_to_repr(5) == (5).to_bytes(32, "little")
    assert B.fr_to_repr(B.R + 3) == (3).to_bytes(32, "little")
