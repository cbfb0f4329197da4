"""One proof across several ranks (BASELINE configs[3]): create_proof with
its commitment MSMs split into point slabs over h2g_dist's transport gives the same
proof bytes as the single-device prover.  The ranks run as separate processes (the
one-process-per-GPU layout) over gloo with host-staged slabs, so they can share this
box's one GPU; the RCCL transport differs only in where the slab tensors live."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpus():
    import torch
    return torch.cuda.device_count()


def _run(world, cases, backend="gloo", transport="torch", mode="slab", extra=()):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "_shard_prove.py"), "--backend", backend, "--transport", transport,
           "--mode", mode] + list(extra) + cases
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("SHARD_RESULT ")]
    assert line, p.stdout[-3000:] + p.stderr[-3000:]
    return json.loads(line[-1][len("SHARD_RESULT "):])


def test_sharded_proof_two_ranks():
    cases = ["simple_k6", "mixed_k10", "lookup_k11", "keccak_k12", "c3_k14", "challenge_k9"]
    res = _run(2, cases)
    for nm in cases:
        assert res[nm]["same"], nm
        assert all(m > 0 for m in res[nm]["msms"]), (nm, res[nm])


def test_sharded_proof_three_ranks():
    cases = ["simple_k6", "lookup_k11"]
    res = _run(3, cases)
    for nm in cases:
        assert res[nm]["same"], nm
        assert len(res[nm]["msms"]) == 2 and all(m > 0 for m in res[nm]["msms"]), (nm, res[nm])


def test_spmd_proof_two_and_three_ranks():
    """SPMD: every rank proves with its slab of each MSM and the all-gathered partials, and
    the extended domain's sub-cosets divided over the ranks (h broadcast from each owner);
    every rank's bytes == the single-device proof.  Three ranks leave a rank without a
    sub-coset for the degree-3 circuits (2 sub-cosets) and give one rank two of the
    keccak-style circuit's four."""
    cases = ["simple_k6", "mixed_k10", "lookup_k11", "keccak_k12", "c3_k14", "challenge_k9"]
    res = _run(2, cases, mode="spmd")
    for nm in cases:
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
        assert res[nm]["gathers"] > 0 and res[nm]["bcasts"] > 0, (nm, res[nm])
    res = _run(3, ["simple_k6", "lookup_k11", "keccak_k12", "c3_k14"], mode="spmd")
    for nm in ("simple_k6", "lookup_k11", "keccak_k12", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
    # the MSM-only split (extended domain replicated)
    res = _run(2, ["lookup_k11", "c3_k14"], mode="spmd", extra=["--no-subcosets"])
    for nm in ("lookup_k11", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"] and res[nm]["bcasts"] == 0, (nm, res[nm])


@pytest.mark.parametrize("mode", ["slab", "spmd"])
@pytest.mark.parametrize("transport", ["torch", "native"])
def test_sharded_proof_rccl_two_gpus(transport, mode):
    """the RCCL paths (one GPU per rank): torch.distributed slabs, and libh2g's own
    communicators (h2g_comm_*); needs >= 2 GPUs (RCCL refuses two ranks on one GPU)"""
    if _gpus() < 2:
        pytest.skip("needs two GPUs")
    cases = ["simple_k6", "lookup_k11", "c3_k14", "challenge_k9"]
    res = _run(2, cases, backend="nccl", transport=transport, mode=mode)
    for nm in cases:
        assert res[nm]["same"], nm
        if mode == "spmd":
            assert res[nm]["same_ranks"], nm
        else:
            assert all(m > 0 for m in res[nm]["msms"]), (nm, res[nm])
