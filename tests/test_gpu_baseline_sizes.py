"""Parity at the BASELINE.json sizes (configs[2]..[4]) on the device, through the C ABI.

  * C3 at k = 20 (configs[2]): device proof bytes == the oracle's create_proof bytes (C
    restatement of halo2_backend/src/plonk/prover.rs), on the device-generated SRS, whose
    entries are spot-checked against [s^i]G and [L_i(s)]G computed here.
  * C3 at k = 22 (the bench proof, configs[3]), C3 at k = 24 (north_star's k-range top) and
    the keccak-style circuit (32 advice columns, 16 lookups) at k = 18 (configs[4]): device
    proof bytes == the oracle's, and the device proof is accepted by the independent Python
    verifier (oracle/py/verifier.py, halo2_backend/src/plonk/verifier.rs)
    and a tampered proof is rejected -- the prove -> verify relation of
    halo2_proofs/tests/plonk_api.rs:580-640.  The verifying key is computed twice: by the
    device keygen (h2g_pk_vk_commitments) and on the CPU from the oracle keygen's sigma
    columns as [f(s)]G; the two must agree.
"""
import os
import random

import numpy as np
import pytest

import _oracle as O
import h2g
import h2g_circuit as hc
import verifier as V
from bn254_ref import G1_GEN, R, g1_mul

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2g.init()
    yield


def _s(k):
    return 0x5EED0000 + k


def _dev_vk(pk):
    f, p = pk.vk_commitments()
    return [V.affine_from_limbs(c) for c in f], [V.affine_from_limbs(c) for c in p]


def _tampered(proof, at):
    b = bytearray(proof)
    b[at] ^= 0x01
    return bytes(b)


def _rejects(circ, proof, s, vk):
    try:
        return not V.verify(circ, [], proof, s, vk=vk)
    except V.VerifyError:
        return True


def _check_srs(params, s_int, k, g, gl):
    """device SRS entries vs [s^i]G and [L_i(s)]G (ParamsKZG::setup, kzg/commitment.rs:64-131)"""
    n = 1 << k
    from bn254_ref import Domain
    omega = Domain(3, k).omega
    rnd = random.Random(k)
    for i in [0, 1, 2, n - 1] + rnd.sample(range(3, n - 1), 4):
        assert V.affine_from_limbs(g[i]) == g1_mul(G1_GEN, pow(s_int, i, R)), i
        w = pow(omega, i, R)
        li = w * (pow(s_int, n, R) - 1) % R * pow(n * (s_int - w) % R, -1, R) % R
        assert V.affine_from_limbs(gl[i]) == g1_mul(G1_GEN, li), i


@pytest.mark.timeout(900)
def test_c3_k20_bytes_match_oracle():
    """BASELINE configs[2]: synthetic 3-advice/1-fixed circuit at k = 20, bit-exact vs CPU"""
    k = 20
    s_int = _s(k)
    circ, wit = hc.synthetic_c3(k, O.OracleOps, seed=20)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    g, gl = params.export()
    _check_srs(params, s_int, k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    got = pk.create_proof(wit)
    want = O.create_proof(circ, wit, g, gl, threads=THREADS)
    assert len(got) == 864 and got == want
    vk = _dev_vk(pk)
    assert vk == O.vk_commitments(circ, wit, s_int, g, gl, threads=THREADS)
    assert V.verify(circ, [], got, s_int, vk=vk)
    pk.close()
    params.close()


@pytest.mark.timeout(900)
def test_c3_k22_proof_bytes_match_oracle_and_verify():
    """the bench proof (C3, k = 22, BASELINE configs[3]): device proof bytes == the oracle's
    create_proof bytes (same circuit, witness, SRS and RNG seed), accepted by the verifier,
    tampered copies rejected, identical across repeated proofs with the same key"""
    k = 22
    s_int = _s(k)
    circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=22)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    pk = h2g.ProvingKey(params, circ)
    proof = pk.create_proof(wit)
    assert pk.create_proof(wit) == proof
    vk = _dev_vk(pk)
    g, gl = params.export()
    assert proof == O.create_proof(circ, wit, g, gl, threads=THREADS)
    assert vk == O.vk_commitments(circ, wit, s_int, g, gl, threads=THREADS)
    del g, gl
    assert V.verify(circ, [], proof, s_int, vk=vk)
    # an advice commitment, an evaluation and the final opening point, each altered
    for at in (0, 32 * 11 + 3, len(proof) - 32):
        assert _rejects(circ, _tampered(proof, at), s_int, vk), at
    # a wrong witness (broken gate on one row) gives a proof that does not verify
    bad = hc.Witness(wit.advice.copy(), wit.instance, wit.instance_lens)
    bad.advice[2, 1000] = hc.fr_to_limbs(12345)
    assert _rejects(circ, pk.create_proof(bad), s_int, vk)
    pk.close()
    params.close()


@pytest.mark.timeout(900)
def test_keccak_style_k18_proof_bytes_match_oracle_and_verify():
    """BASELINE configs[4]'s circuit shape at its size: 32 advice columns, 16 three-column
    lookups, degree 5 (extended domain 4n), at k = 18; device bytes == oracle bytes"""
    k = 18
    s_int = _s(k)
    circ, wit = hc.keccak_style(k, words=16)
    assert circ.num_advice == 32 and len(circ.lookups) == 16
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    pk = h2g.ProvingKey(params, circ)
    proof = pk.create_proof(wit)
    assert pk.create_proof(wit) == proof
    vk = _dev_vk(pk)
    g, gl = params.export()
    assert proof == O.create_proof(circ, wit, g, gl, threads=THREADS)
    assert vk == O.vk_commitments(circ, wit, s_int, g, gl, threads=THREADS)
    assert V.verify(circ, [], proof, s_int, vk=vk)
    for at in (5, 32 * 40 + 7, len(proof) - 40):
        assert _rejects(circ, _tampered(proof, at), s_int, vk), at
    pk.close()
    params.close()


@pytest.mark.timeout(1200)
def test_c3_k24_proof_bytes_match_oracle_and_verify():
    """north_star's k-range top (k = 24, extended domain 2^25): device bytes == oracle
    bytes, the proof verifies with the device verifying key (which equals the CPU-computed
    key at k = 18, 20, 22 above) and a tampered copy is rejected"""
    k = 24
    s_int = _s(k)
    circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=24)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    pk = h2g.ProvingKey(params, circ)
    proof = pk.create_proof(wit)
    assert len(proof) == 864 and pk.create_proof(wit) == proof
    g, gl = params.export()
    assert proof == O.create_proof(circ, wit, g, gl, threads=THREADS)
    del g, gl
    vk = _dev_vk(pk)
    assert V.verify(circ, [], proof, s_int, vk=vk)
    assert _rejects(circ, _tampered(proof, 32 * 11 + 3), s_int, vk)
    pk.close()
    params.close()
