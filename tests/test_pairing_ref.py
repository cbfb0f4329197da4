"""The verifier's pairing (oracle/py/pairing_ref.py, BN254 optimal ate) and DualMSM::check
decided from the params' G2 elements instead of the SRS secret, as the reference's
verify_proof does (kzg/multiopen/{shplonk,gwc}/verifier.rs, poly/kzg/msm.rs).  The
pairing is pinned by bilinearity, non-degeneracy and order r."""
import os
import sys

import pytest

import _oracle as O
import h2g_circuit as hc

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "py"))
import bn254_ref as B  # noqa: E402
import pairing_ref as PR  # noqa: E402
import verifier as V  # noqa: E402


def test_pairing_bilinear_nondegenerate_order_r():
    e = PR.pairing(B.G1_GEN, B.G2_GEN)
    assert not PR.f12_is_one(e)
    assert PR.f12_is_one(PR.f12_pow(e, B.R))
    a, b = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    assert PR.pairing(B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)) == PR.f12_pow(e, a * b % B.R)
    assert PR.pairing(B.g1_mul(B.G1_GEN, a * b % B.R), B.G2_GEN) == PR.pairing(B.G1_GEN, B.g2_mul(B.G2_GEN, a * b))
    # e(P, Q) e(-P, Q) = 1, and the identity pairs to one
    assert PR.pairing_check([(B.G1_GEN, B.G2_GEN), (B.g1_neg(B.G1_GEN), B.G2_GEN)])
    assert PR.f12_is_one(PR.pairing(None, B.G2_GEN))


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_verify_with_params_g2(multiopen):
    circ, wit = hc.lookup_circuit(6)
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, wit, g, gl, multiopen=multiopen)
    g2 = (B.G2_GEN, B.g2_mul(B.G2_GEN, s))
    inst = [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]
    assert V.verify(circ, inst, proof, s, multiopen=multiopen, g2=g2)
    # another secret's [s]G2 fails the pairing equation; so does a tampered opening
    bad = (B.G2_GEN, B.g2_mul(B.G2_GEN, s + 1))
    assert not V.verify(circ, inst, proof, s, multiopen=multiopen, g2=bad)
    t = bytearray(proof)
    t[-40] ^= 1
    try:
        ok = V.verify(circ, inst, bytes(t), s, multiopen=multiopen, g2=g2)
    except V.VerifyError:
        ok = False
    assert not ok
