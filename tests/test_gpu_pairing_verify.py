"""Device proofs verified as the reference's verify_proof does: VK commitments from the
device key and DualMSM::check by the pairing against the device params' G2 elements
(h2g_params_g2: g2, s_g2 = [s]g2), no SRS secret in the checker."""
import numpy as np
import pytest

import h2g
import h2g_circuit as hc
import verifier as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2g.init()
    yield


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_device_proof_pairing_verifies(multiopen):
    circ, wit = hc.synthetic_c3(12, h2g.DeviceOps, seed=7)
    params = h2g.Params(circ.k, s=np.asarray(hc.fr_to_limbs(0xC0FFEE), dtype=np.uint64))
    pk = h2g.ProvingKey(params, circ)
    proof = pk.create_proof(wit, multiopen=multiopen)
    f, p = pk.vk_commitments()
    vk = ([V.affine_from_limbs(c) for c in f], [V.affine_from_limbs(c) for c in p])
    g2, s_g2 = params.g2()
    g2p = (V.g2_from_limbs(g2), V.g2_from_limbs(s_g2))
    assert V.verify(circ, [], proof, None, vk=vk, g2=g2p, multiopen=multiopen)
    t = bytearray(proof)
    t[100] ^= 4
    try:
        ok = V.verify(circ, [], bytes(t), None, vk=vk, g2=g2p, multiopen=multiopen)
    except V.VerifyError:
        ok = False
    assert not ok
    pk.close()
    params.close()
