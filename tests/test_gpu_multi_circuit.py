"""GPU parity of create_proof's full argument list (h2g_create_proof_multi): several
circuits of one key in one proof and the caller's RngCore, device proof bytes against the
C restatement (oracle/c/prover.c) and the independent verifier (oracle/py/verifier.py).
Reference shapes: the two-circuit batch of halo2_proofs/tests/plonk_api.rs:504-510 and the
OneNg-driven MyCircuit proof of halo2_proofs/tests/frontend_backend_split.rs:477-560."""
import numpy as np
import pytest

import _oracle as O
import h2g
import h2g_circuit as hc
import verifier as V
from test_multi_circuit_oracle import ChaChaStream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2g.init()
    yield


def _instances(circ, wit):
    return [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]


@pytest.mark.parametrize("k", [8, 11])
def test_two_c3_circuits_match_oracle(k):
    circ, w0 = hc.synthetic_c3(k, O.OracleOps, seed=3)
    _, w1 = hc.synthetic_c3(k, O.OracleOps, seed=11)
    s, g, gl = O.srs(k)
    params = h2g.Params(k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, w0, g, gl, wits=[w0, w1])
    got = pk.create_proof_multi([w0, w1])
    assert got == want
    assert V.verify(circ, None, got, s, instances_multi=[[], []])
    # the single-circuit entry point still gives the one-circuit proof after a 2-circuit proof
    assert pk.create_proof(w0) == O.create_proof(circ, w0, g, gl)
    # three circuits: workspaces grow on demand
    assert pk.create_proof_multi([w1, w0, w1]) == O.create_proof(circ, w0, g, gl, wits=[w1, w0, w1])
    pk.close()
    params.close()


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_two_my_circuits_phases_lookups_shuffles(multiopen):
    """instances, a lookup, a shuffle and a second advice phase per circuit; witnesses from
    per-circuit witness sources"""
    circ, wit, fill = hc.my_circuit(6)
    s, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, wit, g, gl, wits=[wit, wit], fills=[fill, fill], multiopen=multiopen)
    got = pk.create_proof_multi([wit, wit], fills=[fill, fill], multiopen=multiopen)
    assert got == want
    inst = _instances(circ, wit)
    assert V.verify(circ, None, got, s, instances_multi=[inst, inst], multiopen=multiopen)
    pk.close()
    params.close()


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_two_my_circuits_distinct_inputs(multiopen):
    """two circuits with different witnesses and instances (MyCircuit with input 42 and
    1000): a swapped circuit index -- the instance hashing order, fill(circuit, phase), the
    lookup index ci * NL + l, the shuffle products' order -- changes the bytes"""
    circ, w0, f0 = hc.my_circuit(6, input_value=42)
    _, w1, f1 = hc.my_circuit(6, input_value=1000)
    assert not np.array_equal(w0.instance, w1.instance)
    s, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, w0, g, gl, wits=[w0, w1], fills=[f0, f1], multiopen=multiopen)
    got = pk.create_proof_multi([w0, w1], fills=[f0, f1], multiopen=multiopen)
    assert got == want
    assert got != pk.create_proof_multi([w1, w0], fills=[f1, f0], multiopen=multiopen)
    inst = [_instances(circ, w0), _instances(circ, w1)]
    assert V.verify(circ, None, got, s, instances_multi=inst, multiopen=multiopen)
    try:
        swapped = V.verify(circ, None, got, s, instances_multi=inst[::-1], multiopen=multiopen)
    except V.VerifyError:
        swapped = False
    assert not swapped
    pk.close()
    params.close()


def test_one_ng_my_circuit_matches_oracle():
    """frontend_backend_split.rs:513-560: OneNg sets up the SRS (s = Fr::random(OneNg)) and
    drives create_proof; device bytes == oracle bytes, with F::random drawn through
    fill_bytes and through the shim's random_fr"""
    circ, wit, fill = hc.my_circuit(6)
    s_int = hc.ONE_NG_FR
    params = h2g.Params(circ.k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    g, gl = params.export()
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, wit, g, gl, fill=fill, rng=hc.OneNg())
    assert pk.create_proof_multi([wit], fills=[fill], rng=hc.OneNg()) == want
    assert pk.create_proof_multi([wit], fills=[fill], rng=hc.OneNgFr()) == want
    assert V.verify(circ, _instances(circ, wit), want, s_int)
    pk.close()
    params.close()


def test_caller_chacha_rng_equals_seed_on_device():
    circ, wit = hc.lookup_circuit(8)
    _, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    seed = bytes(range(32))
    want = O.create_proof(circ, wit, g, gl, seed=seed)
    assert pk.create_proof_multi([wit], rng=ChaChaStream(seed)) == want
    assert pk.create_proof(wit, seed=seed) == want
    # the library's own ChaCha20 behind the h2g_rng callbacks (h2g_rng_chacha20)
    assert pk.create_proof_multi([wit], seed=seed, rng="native") == want
    pk.close()
    params.close()


def test_rng_failure_fails_the_device_proof():
    circ, wit = hc.simple_example(6)
    _, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)

    class Broken:
        def fill_bytes(self, n):
            raise RuntimeError("entropy source failed")

    with pytest.raises(h2g.H2GError, match="RNG"):
        pk.create_proof_multi([wit], rng=Broken())
    # the key still proves afterwards
    assert pk.create_proof(wit) == O.create_proof(circ, wit, g, gl)
    pk.close()
    params.close()
