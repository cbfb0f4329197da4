"""GPU parity of the device create_proof pipeline (through the C ABI) against the
C restatement prover (oracle/c/prover.c): proof bytes must be identical, and
proofs must verify under the independent Python verifier (oracle/py/verifier.py)."""
import numpy as np
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


_PARAMS = {}


def _params(k):
    if k not in _PARAMS:
        s, g, gl = O.srs(k)
        _PARAMS[k] = (s, g, gl, h2g.Params(k, g, gl))
    return _PARAMS[k]


def test_params_setup_matches_oracle_srs():
    for k in (4, 8):
        s_int, g, gl = O.srs(k)
        p = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
        dg, dgl = p.export()
        assert np.array_equal(dg, g)
        assert np.array_equal(dgl, gl)
        p.close()


CASES = {
    "simple_k6": lambda: hc.simple_example(6),
    "simple_k8": lambda: hc.simple_example(8),
    "mixed_k7": lambda: hc.mixed_circuit(7),
    "mixed_k10": lambda: hc.mixed_circuit(10, seed=5),
    "c3_k8": lambda: hc.synthetic_c3(8, O.OracleOps),
    "c3_k12": lambda: hc.synthetic_c3(12, O.OracleOps, seed=9),
    "lookup_k8": lambda: hc.lookup_circuit(8),
    "lookup_k11": lambda: hc.lookup_circuit(11, seed=8),
    "keccak_k9": lambda: hc.keccak_style(9, words=8),
    "keccak_k12": lambda: hc.keccak_style(12, words=16, seed=9),
}


@pytest.mark.parametrize("name", list(CASES))
def test_proof_bytes_match_oracle(name):
    circ, wit = CASES[name]()
    s, g, gl, params = _params(circ.k)
    pk = h2g.ProvingKey(params, circ)
    assert pk.degree == circ.degree() and pk.bf == circ.blinding_factors()
    want = O.create_proof(circ, wit, g, gl)
    got = pk.create_proof(wit)
    assert len(got) == len(want)
    assert got == want
    # a second proof with the same key reuses the workspace and is identical
    assert pk.create_proof(wit) == want
    # another rng seed / vanishing split: still identical to the oracle
    want2 = O.create_proof(circ, wit, g, gl, seed=bytes(range(32)), vanishing_threads=3)
    assert pk.create_proof(wit, seed=bytes(range(32)), vanishing_threads=3) == want2
    # the vanishing argument's random polynomial committed early from the keystream position
    # the previous proof drew its seeds at (seeded RNG): again with that split, then with
    # the first seed but a third split (position reused, seeds from this proof's keystream)
    assert pk.create_proof(wit, seed=bytes(range(32)), vanishing_threads=3) == want2
    want3 = O.create_proof(circ, wit, g, gl, vanishing_threads=3)
    assert pk.create_proof(wit, vanishing_threads=3) == want3
    assert pk.create_proof(wit) == want and pk.create_proof(wit) == want
    pk.close()


def test_golden_proofs_on_device():
    d = np.load(O.os.path.join(O.REPO, "tests", "golden", "proof_golden.npz"), allow_pickle=False)
    for name in ("simple_k8", "mixed_k7", "lookup_k8"):
        circ, wit = CASES[name]()
        s = int(d[f"{name}_s"].tobytes()[::-1].hex(), 16)
        _, g, gl = O.srs(circ.k, s)
        params = h2g.Params(circ.k, g, gl)
        pk = h2g.ProvingKey(params, circ)
        assert pk.create_proof(wit) == d[f"{name}_proof"].tobytes()
        pk.close()
        params.close()


def test_device_proof_verifies_and_rejects_bad_witness():
    circ, wit = hc.mixed_circuit(8, seed=11)
    s, g, gl, params = _params(8)
    pk = h2g.ProvingKey(params, circ)
    proof = pk.create_proof(wit)
    assert V.verify(circ, _instances(circ, wit), proof, s)
    bad = hc.Witness(wit.advice.copy(), wit.instance.copy(), wit.instance_lens.copy())
    bad.advice[0, 3] = hc.fr_to_limbs(4242)
    assert not V.verify(circ, _instances(circ, bad), pk.create_proof(bad), s)
    pk.close()


def test_advice_resident_on_device():
    circ, wit = hc.synthetic_c3(10, O.OracleOps, seed=4)
    s, g, gl, params = _params(10)
    pk = h2g.ProvingKey(params, circ)
    buf = h2g.DevBuf.from_array(np.ascontiguousarray(wit.advice))
    got = pk.create_proof(advice_dev_ptr=buf.ptr, wit=wit)
    assert got == O.create_proof(circ, wit, g, gl)
    buf.close()
    pk.close()


def test_errors():
    circ, wit = hc.simple_example(6)
    s, g, gl, params = _params(6)
    pk = h2g.ProvingKey(params, circ)
    bad = hc.Witness(wit.advice, wit.instance, np.asarray([circ.n - circ.blinding_factors()], np.uint32))
    with pytest.raises(h2g.H2GError, match="InstanceTooLarge"):
        pk.create_proof(bad)
    # device advice is read in 16-byte chunks: a misaligned pointer is refused, not misread
    adv = h2g.DevBuf.from_array(np.ascontiguousarray(wit.advice))
    with pytest.raises(h2g.H2GError, match="16-byte aligned"):
        pk.create_proof(wit=wit, advice_dev_ptr=adv.ptr + 8)
    adv.close()
    pk.close()
    other = h2g.Params(7, *O.srs(7)[1:])
    with pytest.raises(h2g.H2GError, match="params k"):
        h2g.ProvingKey(other, circ)
    other.close()


def test_lookup_missing_table_value_fails():
    """permute_expression_pair's ConstraintSystemFailure: reported as an argument error"""
    circ, wit = hc.lookup_circuit(8)
    s, g, gl, params = _params(8)
    pk = h2g.ProvingKey(params, circ)
    bad = hc.Witness(wit.advice.copy(), wit.instance, wit.instance_lens)
    bad.advice[0, 5] = hc.fr_to_limbs(300)
    bad.advice[1, 5] = hc.fr_to_limbs(90000)
    with pytest.raises(h2g.H2GError, match="not in the table"):
        pk.create_proof(bad)
    # the key stays usable
    assert pk.create_proof(wit) == O.create_proof(circ, wit, g, gl)
    pk.close()


GWC_CASES = ["simple_k6", "mixed_k10", "c3_k8", "lookup_k11", "keccak_k9"]


@pytest.mark.parametrize("name", GWC_CASES)
def test_gwc_proof_bytes_match_oracle(name):
    """ProverGWC on the device (h2g_pk_set_multiopen 1): bytes identical to the oracle's
    GWC proof, which the independent GWC verifier accepts; the same key still proves
    SHPLONK afterwards."""
    circ, wit = CASES[name]()
    s, g, gl, params = _params(circ.k)
    pk = h2g.ProvingKey(params, circ)
    want = O.create_proof(circ, wit, g, gl, multiopen="gwc")
    got = pk.create_proof(wit, multiopen="gwc")
    assert got == want
    assert pk.create_proof(wit, multiopen="gwc") == want
    assert V.verify(circ, _instances(circ, wit), got, s, multiopen="gwc")
    assert pk.create_proof(wit) == O.create_proof(circ, wit, g, gl)
    pk.close()


def test_phased_proof_matches_oracle():
    """h2g_create_proof_phased (Prover::commit_phase per phase with the caller's witness
    source) produces the oracle's bytes and challenges; h2g_create_proof with the complete
    witness (challenges known) produces the same proof."""
    circ, wit, fill = hc.challenge_circuit(6)
    s, g, gl, params = _params(circ.k)
    ch = []
    want = O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch)
    pk = h2g.ProvingKey(params, circ)
    got, got_ch = pk.create_proof_phased(fill, wit)
    assert got_ch == ch
    assert got == want
    full = hc.Witness(np.stack([hc.ints_to_mont(fill.a), hc.ints_to_mont(fill.z_values(ch))]), wit.instance, [])
    assert pk.create_proof(full) == want
    assert V.verify(circ, [], got, s)
    pk.close()


@pytest.mark.parametrize("k,multiopen", [(7, "shplonk"), (11, "shplonk"), (7, "gwc")])
def test_three_phase_proof_matches_oracle(k, multiopen):
    circ, wit, fill = hc.challenge_circuit(k, seed=k, extended=True)
    s, g, gl, params = _params(circ.k)
    ch = []
    want = O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch, multiopen=multiopen)
    pk = h2g.ProvingKey(params, circ)
    got, got_ch = pk.create_proof_phased(fill, wit, multiopen=multiopen)
    assert got_ch == ch
    assert got == want
    assert pk.create_proof(fill.full(ch), multiopen=multiopen) == want
    assert V.verify(circ, _instances(circ, wit), got, s, multiopen=multiopen)
    pk.close()


def test_phased_witness_failure_is_an_error():
    circ, wit, fill = hc.challenge_circuit(6)
    _, _, _, params = _params(circ.k)
    pk = h2g.ProvingKey(params, circ)

    def broken(phase, ch):
        if phase == 1:
            raise RuntimeError("witness generator failed")
        return fill(phase, ch)

    with pytest.raises(h2g.H2GError, match="witness source failed at phase 1"):
        pk.create_proof_phased(broken, wit)
    # the key still proves afterwards
    ch = []
    s, g, gl, _ = _params(circ.k)
    assert pk.create_proof_phased(fill, wit)[0] == O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch)
    pk.close()


def test_witness_source_writing_usable_rows_only():
    """h2g_create_proof_phased's staging outlives proofs: a witness source that writes only
    the usable rows gets the reference's zero tail in its unblinded column (prover.rs:
    417-421), not what an earlier proof left there."""
    k = 7
    circ, wit, fill = hc.challenge_circuit(k, seed=3, extended=True)
    s, g, gl, params = _params(circ.k)
    usable = circ.usable_rows()
    rng = np.random.default_rng(0)

    def poison(phase, ch):  # full-length columns with garbage in the unusable rows
        out = {c: v.copy() for c, v in fill(phase, ch).items()}
        for v in out.values():
            v[usable:] = hc.random_mont(rng, circ.n - usable)
        return out

    def usable_only(phase, ch):
        return {c: v[:usable] for c, v in fill(phase, ch).items()}

    ch = []
    want = O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch)
    pk = h2g.ProvingKey(params, circ)
    pk.create_proof_phased(poison, wit)
    assert pk.create_proof_phased(usable_only, wit)[0] == want
    assert pk.create_proof_phased(usable_only, wit)[0] == want
    pk.close()
