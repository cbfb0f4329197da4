"""Generates tests/golden/proof_golden.npz: proofs of the C1 simple-example circuit
(k=8), the mixed-feature circuit (k=7) and the lookup/shuffle circuit (k=8) from the C
restatement prover, each
checked by the independent Python verifier before it is written.  Inputs are fully
determined by the circuit generators' seeds, the SRS secret s (stored) and the
prover RNG seed [7; 32] with vanishing thread count 8.

    python tests/golden/gen_proofs.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle", "py"),
                os.path.join(REPO, "yet-another-halo2-fork_amd")]

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402
import h2g_circuit as hc  # noqa: E402
import verifier as V  # noqa: E402


def main():
    out = {}
    for name, make in (("simple_k8", lambda: hc.simple_example(8)), ("mixed_k7", lambda: hc.mixed_circuit(7)),
                       ("lookup_k8", lambda: hc.lookup_circuit(8))):
        circ, wit = make()
        s, g, gl = O.srs(circ.k)
        proof = O.create_proof(circ, wit, g, gl)
        ins = [hc.mont_to_ints(wit.instance[i])[: int(wit.instance_lens[i])] for i in range(circ.num_instance)]
        assert V.verify(circ, ins, proof, s), name
        out[f"{name}_proof"] = np.frombuffer(proof, dtype=np.uint8)
        out[f"{name}_s"] = np.frombuffer(s.to_bytes(32, "little"), dtype=np.uint8)
        print(name, len(proof), "bytes")
    np.savez_compressed(os.path.join(HERE, "proof_golden.npz"), **out)


if __name__ == "__main__":
    main()
