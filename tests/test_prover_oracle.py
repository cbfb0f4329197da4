"""CPU tests of the create_proof restatement (oracle/c/prover.c) and its pins:
the transcript hash / RNG known answers, keygen's permutation vs an independent
restatement, and prove -> verify with the independent Python verifier
(oracle/py/verifier.py) -- the reference's own relational test
(halo2_proofs/tests/plonk_api.rs: proofs must verify; corrupted ones must not)."""
import hashlib
import os

import numpy as np
import pytest

import _oracle as O
import h2g_circuit as hc
import verifier as V

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _instances(circ, wit):
    return [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]


def test_blake2b_personal_matches_hashlib():
    import ctypes
    rng = np.random.default_rng(0)
    for ln in (0, 1, 33, 65, 127, 128, 129, 300):
        d = rng.bytes(ln)
        out = ctypes.create_string_buffer(64)
        O.lib().or_blake2b(d, ln, b"Halo2-Transcript", out)
        assert out.raw == hashlib.blake2b(d, digest_size=64, person=b"Halo2-Transcript").digest()


def test_chacha20_known_answer():
    """RFC 7539 zero-key keystream (= rand_chacha ChaCha20Rng::from_seed([0; 32]) test vector)"""
    import ctypes
    out = ctypes.create_string_buffer(64)
    O.lib().or_chacha20_block(bytes(32), 0, out)
    assert out.raw[:32].hex() == "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
    O.lib().or_chacha20_block(bytes(32), 1, out)
    assert out.raw[:16].hex() == "9f07e7be5551387a98ba977c732d080d"


def test_fr_random_is_le512_mod_r():
    import ctypes
    seed = bytes(range(32))
    out = np.zeros((5, 4), dtype=np.uint64)
    O.lib().or_fr_random_stream(seed, 5, O._p(out))
    # keystream: blocks 0..4 of ChaCha20(seed)
    ks = b""
    buf = ctypes.create_string_buffer(64)
    for c in range(5):
        O.lib().or_chacha20_block(seed, c, buf)
        ks += buf.raw
    want = [int.from_bytes(ks[64 * i: 64 * i + 64], "little") % hc.R_MOD for i in range(5)]
    assert hc.mont_to_ints(out) == want


def test_one_rng_constant():
    """with OneNg every Fr::random = LE512(0x01000000 x16) mod r"""
    v = int.from_bytes(bytes([1, 0, 0, 0]) * 16, "little") % hc.R_MOD
    assert v == 0x0FDD950C1DA3E00B1D2FB9CF61452B1EC0C9DFB910ECFB36B574601AEDF0313B


CIRCUITS = {
    "simple_k6": lambda: hc.simple_example(6),
    "simple_k8": lambda: hc.simple_example(8),
    "mixed_k7": lambda: hc.mixed_circuit(7),
    "c3_k8": lambda: hc.synthetic_c3(8, O.OracleOps),
    "lookup_k8": lambda: hc.lookup_circuit(8),
    "lookup_k9": lambda: hc.lookup_circuit(9, seed=6),
    "keccak_k9": lambda: hc.keccak_style(9, words=5),
}


@pytest.mark.parametrize("name", list(CIRCUITS))
def test_keygen_permutation_matches_restatement(name):
    circ, wit = CIRCUITS[name]()
    _, g, gl = O.srs(circ.k)
    kg = O.Keygen(circ, wit, g, gl)
    assert kg.degree == circ.degree() and kg.bf == circ.blinding_factors()
    sig = V.sigma_lagrange(circ)
    for i in range(len(circ.perm_columns)):
        assert hc.mont_to_ints(kg.sigma(i)) == sig[i]


@pytest.mark.parametrize("name", list(CIRCUITS))
def test_prove_verify(name):
    circ, wit = CIRCUITS[name]()
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, wit, g, gl)
    assert V.verify(circ, _instances(circ, wit), proof, s)


def test_proof_deterministic_and_seed_dependent():
    circ, wit = hc.simple_example(6)
    s, g, gl = O.srs(circ.k)
    p1 = O.create_proof(circ, wit, g, gl, seed=bytes([7] * 32), threads=1)
    p2 = O.create_proof(circ, wit, g, gl, seed=bytes([7] * 32), threads=8)
    p3 = O.create_proof(circ, wit, g, gl, seed=bytes([8] * 32))
    p4 = O.create_proof(circ, wit, g, gl, vanishing_threads=3)
    assert p1 == p2
    assert p1 != p3 and p1 != p4
    for p in (p3, p4):
        assert V.verify(circ, _instances(circ, wit), p, s)


def test_unsatisfied_gate_rejected():
    circ, wit = hc.simple_example(6)
    s, g, gl = O.srs(circ.k)
    wit.advice[1, 0] = hc.fr_to_limbs(12345)   # a1[0] breaks s_mul * (a0 * a1 - a0[next])
    proof = O.create_proof(circ, wit, g, gl)
    assert not V.verify(circ, _instances(circ, wit), proof, s)


def test_broken_copy_rejected():
    circ, wit = hc.mixed_circuit(7)
    s, g, gl = O.srs(circ.k)
    lt, li, lr, rt, ri, rr = circ.copies[0]
    assert lt == hc.ADVICE and rt == hc.ADVICE
    wit.advice[ri, rr] = hc.fr_to_limbs(999)
    proof = O.create_proof(circ, wit, g, gl)
    assert not V.verify(circ, _instances(circ, wit), proof, s)


def test_wrong_instance_rejected():
    circ, wit = hc.simple_example(6)
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, wit, g, gl)
    ins = _instances(circ, wit)
    ins[0][0] = (ins[0][0] + 1) % hc.R_MOD
    assert not V.verify(circ, ins, proof, s)


def test_tampered_proof_rejected():
    circ, wit = hc.mixed_circuit(7)
    s, g, gl = O.srs(circ.k)
    proof = bytearray(O.create_proof(circ, wit, g, gl))
    proof[-40] ^= 1
    try:
        assert not V.verify(circ, _instances(circ, wit), bytes(proof), s)
    except V.VerifyError:
        pass


def test_instance_too_large_fails():
    circ, wit = hc.simple_example(6)
    _, g, gl = O.srs(circ.k)
    wit.instance_lens[0] = circ.n - circ.blinding_factors()   # > n - (bf + 1)
    with pytest.raises(ValueError):
        O.create_proof(circ, wit, g, gl)


def test_lookup_shuffle_negative_cases():
    """a broken shuffle does not verify; an input missing from the table fails like the
    reference (permute_expression_pair -> Error::ConstraintSystemFailure)"""
    circ, wit = hc.lookup_circuit(8)
    s, g, gl = O.srs(circ.k)
    bad = hc.Witness(wit.advice.copy(), wit.instance, wit.instance_lens)
    bad.advice[3, 5] = hc.fr_to_limbs(77)
    assert not V.verify(circ, [], O.create_proof(circ, bad, g, gl), s)
    bad = hc.Witness(wit.advice.copy(), wit.instance, wit.instance_lens)
    bad.advice[0, 5] = hc.fr_to_limbs(300)
    bad.advice[1, 5] = hc.fr_to_limbs(90000)
    with pytest.raises(ValueError, match="-7"):
        O.create_proof(circ, bad, g, gl)


def test_lookup_degree_and_queries():
    circ, _ = hc.lookup_circuit(8)
    assert circ.degree() == 5   # 2 + deg(q a) + deg(t) = 5 (circuit.rs:327-373)
    adv, fix, ins = circ.queries()
    assert adv == [(1, 0), (0, 0), (0, 1), (2, 0), (3, 0)]   # gates, lookups, shuffles, permutation
    assert fix == [(0, 0), (1, 0), (2, 0), (3, 0)]


def test_golden_proofs():
    """committed fixtures (tests/golden/gen_proofs.py): the restatement reproduces them"""
    d = np.load(os.path.join(GOLDEN, "proof_golden.npz"), allow_pickle=False)
    for name in ("simple_k8", "mixed_k7", "lookup_k8"):
        circ, wit = CIRCUITS[name]()
        s, g, gl = O.srs(circ.k, int(d[f"{name}_s"].tobytes()[::-1].hex(), 16))
        proof = O.create_proof(circ, wit, g, gl)
        assert proof == d[f"{name}_proof"].tobytes()


@pytest.mark.parametrize("name", ["simple_k6", "mixed_k7", "c3_k8", "lookup_k8", "keccak_k9"])
def test_prove_verify_gwc(name):
    """ProverGWC / VerifierGWC (poly/kzg/multiopen/gwc): the multi-open the reference's
    serialization test uses (halo2_proofs/tests/serialization.rs:158-175)"""
    circ, wit = CIRCUITS[name]()
    s, g, gl = O.srs(circ.k)
    proof = O.create_proof(circ, wit, g, gl, multiopen="gwc")
    ins = _instances(circ, wit)
    assert V.verify(circ, ins, proof, s, multiopen="gwc")
    # the two multi-opens share everything up to the opening: same prefix, different tail
    shplonk = O.create_proof(circ, wit, g, gl)
    npts = len(proof) - (len(shplonk) - 64)
    assert npts > 0 and npts % 32 == 0 and proof[: len(shplonk) - 64] == shplonk[:-64]


def test_gwc_negative_cases():
    circ, wit = hc.mixed_circuit(7)
    s, g, gl = O.srs(circ.k)
    proof = bytearray(O.create_proof(circ, wit, g, gl, multiopen="gwc"))
    proof[-40] ^= 1
    try:
        assert not V.verify(circ, _instances(circ, wit), bytes(proof), s, multiopen="gwc")
    except V.VerifyError:
        pass
    bad = hc.Witness(wit.advice.copy(), wit.instance, wit.instance_lens)
    bad.advice[0, 3] = hc.fr_to_limbs(4242)
    assert not V.verify(circ, _instances(circ, bad), O.create_proof(circ, bad, g, gl, multiopen="gwc"), s,
                        multiopen="gwc")


def test_phases_and_challenges():
    """Prover::commit_phase over two advice phases (prover.rs:309-494): the phase-1 witness
    is computed from the phase-0 challenge the prover hands back; challenges enter gates and
    compressed lookup expressions.  The proof verifies, equals the proof from the complete
    witness computed with the same challenges, and a witness that ignores the challenge is
    rejected.  (Phases are my restatement's; parity with the Rust prover is unpinned here:
    the reference holds no multi-phase golden proof.)"""
    circ, wit, fill = hc.challenge_circuit(6)
    s, g, gl = O.srs(circ.k)
    ch = []
    proof = O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch)
    assert len(ch) == 2 and all(0 < c < hc.R_MOD for c in ch)
    assert V.verify(circ, [], proof, s)
    full = hc.Witness(np.stack([hc.ints_to_mont(fill.a), hc.ints_to_mont(fill.z_values(ch))]), wit.instance, [])
    assert O.create_proof(circ, full, g, gl) == proof
    bad = hc.Witness(np.stack([hc.ints_to_mont(fill.a), hc.ints_to_mont(fill.z_values([5, 0]))]), wit.instance, [])
    assert not V.verify(circ, [], O.create_proof(circ, bad, g, gl), s)


def test_single_phase_transcript_repr_unchanged():
    """circuits without phases keep their description hash (no phase bytes appended)"""
    circ, _ = hc.simple_example(6)
    assert circ.max_phase == 0 and circ.num_challenges == 0
    c2, _, _ = hc.challenge_circuit(6)
    assert c2.max_phase == 1 and c2.num_challenges == 2


@pytest.mark.parametrize("multiopen", ["shplonk", "gwc"])
def test_three_phases_shuffle_unblinded(multiopen):
    """three advice phases, an unblinded phase-1 column shuffled against a phase-0 column,
    an instance column, a phase-1 challenge used by a phase-2 column"""
    circ, wit, fill = hc.challenge_circuit(7, extended=True)
    s, g, gl = O.srs(circ.k)
    ch = []
    proof = O.create_proof(circ, wit, g, gl, fill=fill, challenges_out=ch, multiopen=multiopen)
    inst = _instances(circ, wit)
    assert V.verify(circ, inst, proof, s, multiopen=multiopen)
    assert O.create_proof(circ, fill.full(ch), g, gl, multiopen=multiopen) == proof
    # a w that is not a permutation of a's active rows breaks the shuffle
    bad = fill.full(ch)
    bad.advice[2, 0] = hc.ints_to_mont([(fill.a[1] + 1) % 16])[0]
    assert not V.verify(circ, inst, O.create_proof(circ, bad, g, gl, multiopen=multiopen), s, multiopen=multiopen)


def test_witness_source_failure_fails_the_proof():
    circ, wit, fill = hc.challenge_circuit(6)
    _, g, gl = O.srs(circ.k)

    def broken(phase, ch):
        if phase == 1:
            raise RuntimeError("witness generator failed")
        return fill(phase, ch)

    with pytest.raises(ValueError):
        O.create_proof(circ, wit, g, gl, fill=broken)
