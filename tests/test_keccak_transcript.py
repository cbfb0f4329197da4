"""Keccak256Write / Keccak256Read (halo2_backend/src/transcript.rs:109-463, the EVM
transcript): the Keccak-256 sponge pinned two ways -- the permutation against
hashlib.sha3_256 (same Keccak-f[1600], SHA3 padding), the Keccak padding against the
public constants Keccak-256("") and Keccak-256("abc") -- for both the C oracle and the
Python restatement; then oracle proofs over the Keccak transcript verify under the
Python Keccak256Read and fail under Blake2bRead (and vice versa)."""
import hashlib
import os
import sys

import pytest

import _oracle as O
import h2g_circuit as hc

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "py"))
import keccak_ref as K  # noqa: E402
import verifier as V  # noqa: E402

KECCAK_EMPTY = "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
KECCAK_ABC = "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"


@pytest.mark.parametrize("n", [0, 1, 31, 135, 136, 137, 271, 272, 273, 1000])
def test_sponge_vs_hashlib_sha3(n):
    data = bytes((7 * i + n) & 0xFF for i in range(n))
    want = hashlib.sha3_256(data).digest()
    assert K.Keccak(0x06).update(data).digest() == want
    assert O.keccak(data, 0x06) == want
    assert O.keccak(data) == K.keccak256(data)


def test_keccak256_known_answers():
    for impl in (K.keccak256, O.keccak):
        assert impl(b"").hex() == KECCAK_EMPTY
        assert impl(b"abc").hex() == KECCAK_ABC


def test_incremental_updates_and_copies():
    h = K.Keccak().update(b"Halo2-Transcript")
    c = h.copy()
    h.update(b"\x00" * 200)
    assert c.update(b"\x00" * 200).digest() == h.digest() == K.keccak256(b"Halo2-Transcript" + b"\x00" * 200)


@pytest.mark.parametrize("name", ["simple", "lookup"])
def test_oracle_keccak_transcript_proof_verifies(name):
    circ, wit = hc.simple_example(5) if name == "simple" else hc.lookup_circuit(6)
    s, g, gl = O.srs(circ.k)
    pk = O.create_proof(circ, wit, g, gl, transcript="keccak256")
    pb = O.create_proof(circ, wit, g, gl)
    assert pk != pb and len(pk) == len(pb)
    inst = [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]
    assert V.verify(circ, inst, pk, s, transcript="keccak256")
    assert V.verify(circ, inst, pb, s)
    for proof, tr in ((pk, "blake2b"), (pb, "keccak256")):
        try:
            ok = V.verify(circ, inst, proof, s, transcript=tr)
        except V.VerifyError:
            ok = False
        assert not ok
