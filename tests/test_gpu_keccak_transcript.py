"""Keccak256Write on the device prover (h2g_pk_set_transcript 1): proof bytes identical to
the C restatement over the same transcript (oracle/c/prover.c tr_*), accepted by the
Python Keccak256Read verifier, and the key returns to Blake2bWrite afterwards.  The
Keccak-256 sponge itself is pinned in tests/test_keccak_transcript.py."""
import pytest

import _oracle as O
import h2g
import h2g_circuit as hc
import verifier as V

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _init():
    h2g.init()
    yield


def _instances(circ, wit):
    return [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]


@pytest.mark.parametrize("name,multiopen", [("simple", "shplonk"), ("lookup", "shplonk"), ("c3", "gwc"),
                                            ("keccak", "shplonk")])
def test_keccak_transcript_matches_oracle(name, multiopen):
    circ, wit = {"simple": lambda: hc.simple_example(7), "lookup": lambda: hc.lookup_circuit(9),
                 "c3": lambda: hc.synthetic_c3(10, O.OracleOps, seed=2),
                 "keccak": lambda: hc.keccak_style(10, words=16, seed=3)}[name]()
    s, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, wit, g, gl, multiopen=multiopen, transcript="keccak256")
    got = pk.create_proof(wit, multiopen=multiopen, transcript="keccak256")
    assert got == want
    assert V.verify(circ, _instances(circ, wit), got, s, multiopen=multiopen, transcript="keccak256")
    assert pk.create_proof(wit, multiopen=multiopen) == O.create_proof(circ, wit, g, gl, multiopen=multiopen)
    pk.close()
    params.close()


def test_keccak_transcript_phased_and_multi():
    circ, wit, fill = hc.my_circuit(6)
    s, g, gl = O.srs(circ.k)
    params = h2g.Params(circ.k, g, gl)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, wit, g, gl, wits=[wit, wit], fills=[fill, fill], transcript="keccak256")
    assert pk.create_proof_multi([wit, wit], fills=[fill, fill], transcript="keccak256") == want
    inst = _instances(circ, wit)
    assert V.verify(circ, None, want, s, instances_multi=[inst, inst], transcript="keccak256")
    pk.close()
    params.close()
