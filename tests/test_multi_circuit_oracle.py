"""CPU tests of create_proof's full argument list in the restatement (oracle/c/prover.c):
several circuits of one key in one proof (circuits: &[C], instances: &[&[&[F]]],
halo2_proofs/src/plonk/prover.rs:19-36; halo2_backend/src/plonk/prover.rs:187-899) and the
caller's `rng: R: RngCore`.  Pinned by the reference's relational tests: the two-circuit
batch of halo2_proofs/tests/plonk_api.rs:504-510 must verify (and a tampered one must not),
and the OneNg-driven MyCircuit proof of halo2_proofs/tests/frontend_backend_split.rs:477-560
must verify with the SRS OneNg itself sets up."""
import ctypes

import numpy as np
import pytest

import _oracle as O
import h2g_circuit as hc
import verifier as V


def _instances(circ, wit):
    return [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]


class ChaChaStream:
    """ChaCha20Rng::from_seed(seed) as a caller RNG (blocks from the oracle's ChaCha20)"""

    def __init__(self, seed):
        self.seed, self.ctr, self.buf = bytes(seed), 0, b""

    def fill_bytes(self, n):
        while len(self.buf) < n:
            out = ctypes.create_string_buffer(64)
            O.lib().or_chacha20_block(self.seed, self.ctr, out)
            self.ctr += 1
            self.buf += out.raw
        b, self.buf = self.buf[:n], self.buf[n:]
        return b


def test_two_circuits_verify_and_tamper():
    """plonk_api.rs:504-510 batches the same circuit twice; here two different C3 witnesses
    of one key (same fixed columns and copies) go into one proof"""
    circ, w0 = hc.synthetic_c3(8, O.OracleOps, seed=3)
    _, w1 = hc.synthetic_c3(8, O.OracleOps, seed=11)
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, w0, g, gl, wits=[w0, w1])
    single = O.create_proof(circ, w0, g, gl)
    assert len(proof) > len(single) and proof != single
    assert V.verify(circ, None, proof, s, instances_multi=[[], []])
    bad = bytearray(proof)
    bad[100] ^= 1
    try:
        assert not V.verify(circ, None, bytes(bad), s, instances_multi=[[], []])
    except V.VerifyError:
        pass
    # one circuit through the multi-circuit path is the single-circuit proof
    assert O.create_proof(circ, w0, g, gl, wits=[w0]) == single
    # the order of the circuits matters
    assert O.create_proof(circ, w0, g, gl, wits=[w1, w0]) != proof


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_two_circuits_with_instances_lookups_shuffles(multiopen):
    """every argument per circuit: instances, lookups, shuffles, a second phase with a
    challenge, both circuits' witnesses from per-circuit witness sources"""
    circ, wit, fill = hc.my_circuit(6)
    s, g, gl = O.srs(circ.k)
    ch = []
    proof = O.create_proof(circ, wit, g, gl, wits=[wit, wit], fills=[fill, fill], challenges_out=ch,
                           multiopen=multiopen)
    inst = _instances(circ, wit)
    assert V.verify(circ, None, proof, s, instances_multi=[inst, inst], multiopen=multiopen)
    full = fill.full(ch)
    assert O.create_proof(circ, full, g, gl, wits=[full, full], multiopen=multiopen) == proof
    # a wrong instance of the second circuit is rejected
    inst2 = [list(inst[0])]
    inst2[0][3] = (inst2[0][3] + 1) % hc.R_MOD
    assert not V.verify(circ, None, proof, s, instances_multi=[inst, inst2], multiopen=multiopen)


def test_my_circuit_single_verifies():
    circ, wit, fill = hc.my_circuit(6)
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, wit, g, gl, fill=fill)
    assert V.verify(circ, _instances(circ, wit), proof, s)


def test_caller_rng_chacha_equals_seed():
    """an RngCore callback producing the ChaCha20 stream gives the seeded proof"""
    circ, wit = hc.mixed_circuit(7)
    _, g, gl = O.srs(circ.k)
    seed = bytes(range(32))
    assert O.create_proof(circ, wit, g, gl, rng=ChaChaStream(seed)) == O.create_proof(circ, wit, g, gl, seed=seed)


def test_one_ng_proof():
    """frontend_backend_split.rs:513-560: OneNg drives ParamsKZG::setup (s = Fr::random(OneNg))
    and create_proof; the proof verifies.  fill_bytes-only and F::random answered directly
    give the same proof (every F::random of OneNg is the same constant)."""
    circ, wit, fill = hc.my_circuit(6)
    s, g, gl = O.srs(circ.k, hc.ONE_NG_FR)
    p1 = O.create_proof(circ, wit, g, gl, fill=fill, rng=hc.OneNg())
    p2 = O.create_proof(circ, wit, g, gl, fill=fill, rng=hc.OneNgFr())
    assert p1 == p2
    assert V.verify(circ, _instances(circ, wit), p1, s)
    assert p1 != O.create_proof(circ, wit, g, gl, fill=fill)


def test_rng_failure_fails_the_proof():
    circ, wit = hc.simple_example(6)
    _, g, gl = O.srs(circ.k)

    class Broken:
        def __init__(self):
            self.left = 10

        def fill_bytes(self, n):
            self.left -= 1
            if self.left < 0:
                raise RuntimeError("entropy source failed")
            return bytes(n)

    with pytest.raises(ValueError):
        O.create_proof(circ, wit, g, gl, rng=Broken())

    class Unreduced:
        def fill_bytes(self, n):
            return bytes(n)

        def random_fr(self):
            return np.full(4, 0xFFFFFFFFFFFFFFFF, dtype=np.uint64)   # not below r

    with pytest.raises(ValueError):
        O.create_proof(circ, wit, g, gl, rng=Unreduced())
