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
import time

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


def _run(world, cases, backend="gloo", transport="torch", mode="slab", extra=(), timeout=900):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "_shard_prove.py"), "--backend", backend, "--transport", transport,
           "--mode", mode] + list(extra) + cases
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    # the ranks' output goes to a log under gpurun_out/ as it is written (a multi-minute
    # at-size case shows its progress there), read back when the ranks have finished
    logdir = os.path.join(os.path.dirname(HERE), "gpurun_out", "sharded")
    os.makedirs(logdir, exist_ok=True)
    log = os.path.join(logdir, f"{mode}_{world}_{'_'.join(cases)[:60]}.log")
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, text=True, env=env)
        t0 = time.monotonic()
        while True:
            try:
                p.wait(timeout=30)
                break
            except subprocess.TimeoutExpired:
                if time.monotonic() - t0 > timeout:
                    p.kill()
                    p.wait()
                    break
                f.write(f"[test] ranks running {time.monotonic() - t0:.0f} s\n")
                f.flush()
    with open(log) as f:
        out = f.read()
    assert p.returncode == 0, out[-6000:]
    line = [ln for ln in out.splitlines() if ln.startswith("SHARD_RESULT ")]
    assert line, out[-6000:]
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
    """SPMD: every rank proves with its slab of each MSM and the all-gathered partials, the
    extended domain's sub-cosets divided over the ranks (each owner interpolates its h
    evaluations and every rank receives its coefficient slab of them), and the
    evaluations / SHPLONK on coefficient slabs; every rank's bytes == the single-device
    proof.  Three ranks leave a rank without a sub-coset for the degree-3 circuits (2
    sub-cosets) and give one rank two of the keccak-style circuit's four."""
    cases = ["simple_k6", "mixed_k10", "lookup_k11", "keccak_k12", "c3_k14", "challenge_k9"]
    res = _run(2, cases, mode="spmd")
    for nm in cases:
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
        assert res[nm]["gathers"] > 0 and res[nm]["exchanges"] > 0 and res[nm]["host_gathers"] > 0, (nm, res[nm])
        assert res[nm]["bcasts"] == 0, (nm, res[nm])
    res = _run(3, ["simple_k6", "lookup_k11", "keccak_k12", "c3_k14"], mode="spmd")
    for nm in ("simple_k6", "lookup_k11", "keccak_k12", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
    # h broadcast as evaluations, tail on slabs; and everything but the MSMs and sub-cosets
    # replicated (the round-2 split)
    res = _run(2, ["lookup_k11", "c3_k14"], mode="spmd", extra=["--bcast-h"])
    for nm in ("lookup_k11", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"] and res[nm]["bcasts"] > 0, (nm, res[nm])
        assert res[nm]["exchanges"] == 0 and res[nm]["host_gathers"] > 0, (nm, res[nm])
    res = _run(3, ["keccak_k12", "c3_k14"], mode="spmd", extra=["--no-slabs"])
    for nm in ("keccak_k12", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"] and res[nm]["bcasts"] > 0, (nm, res[nm])
        assert res[nm]["host_gathers"] == 0, (nm, res[nm])
    # uneven slab weights (h2g_spmd_set_weights): the MSM slabs, the tail's coefficient
    # slabs and the h slab exchange all follow the weighted partition
    res = _run(3, ["lookup_k11", "keccak_k12", "c3_k14"], mode="spmd", extra=["--weights", "3,1,2"])
    for nm in ("lookup_k11", "keccak_k12", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
    # the MSM-only split (extended domain replicated), tail on slabs
    res = _run(2, ["lookup_k11", "c3_k14"], mode="spmd", extra=["--no-subcosets"])
    for nm in ("lookup_k11", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"] and res[nm]["bcasts"] == 0, (nm, res[nm])
        assert res[nm]["exchanges"] == 0, (nm, res[nm])


def test_spmd_row_pieces_four_and_eight_ranks():
    """more ranks than sub-coset (world a multiple of 2^e): every rank evaluates h on a row
    piece of one sub-coset (rotation halos around it), every column's transforms run once
    on its owner and reach the pieces through one exchange per stage, the pieces' h rows
    gather at each sub-coset's leader; bytes == one GPU.  Degree-3 circuits have 2
    sub-cosets: 2 pieces each at 4 ranks, 4 at 8"""
    cases = ["simple_k6", "mixed_k10", "c3_k14", "challenge_k9", "multi_my_k6", "keccak_k12"]
    res = _run(4, cases, mode="spmd")
    for nm in cases:
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
    res = _run(8, ["c3_k14", "mixed_k10"], mode="spmd", extra=["--one-variant"])
    for nm in ("c3_k14", "mixed_k10"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
    # the column exchanges completing on return instead of overlapped (post / wait before h)
    res = _run(4, ["c3_k14", "keccak_k12"], mode="spmd", extra=["--one-variant", "--sync-exchange"])
    for nm in ("c3_k14", "keccak_k12"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])


def test_spmd_column_owners_off_matches():
    """the same proofs with column ownership off (h2g_spmd_set_column_owners(0)): point
    slabs for every MSM, sub-coset owners transforming every column"""
    res = _run(4, ["keccak_k12", "c3_k14"], mode="spmd", extra=["--no-column-owners"])
    for nm in ("keccak_k12", "c3_k14"):
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])


def test_spmd_two_circuits_distinct_witnesses():
    """two MyCircuit instances with different inputs (witnesses and instances), a lookup,
    a shuffle and a second phase each, in one SPMD proof: every rank == one GPU"""
    res = _run(2, ["multi_my_k6"], mode="spmd")
    assert res["multi_my_k6"]["same"] and res["multi_my_k6"]["same_ranks"], res


def test_spmd_diverged_ranks_refuse_the_proof():
    """a rank with other RNG draws: the digest in every all-gather payload makes every rank
    fail the proof (H2G_ERR_STATE) instead of summing slabs of different polynomials"""
    res = _run(2, ["simple_k6", "lookup_k11"], mode="spmd", extra=["--diverge"])
    for nm in ("simple_k6", "lookup_k11"):
        assert res[nm]["refused_all"], (nm, res[nm])


@pytest.mark.parametrize("world,names", [(2, ["c3_k14", "lookup_k11"]), (4, ["keccak_k12", "c3_k14"])])
def test_spmd_diverged_witness_refuses_the_proof(world, names):
    """a rank fed another witness (same RNG, same instances): with the commitments and
    evaluations summed from slabs its transcript matches the others', so only the witness
    digest (every advice column at a fixed point, folded into the all-gather payload)
    makes every rank fail the proof.  At 4 ranks the keccak-style advice and lookup stages
    are wide (each column committed by its owner alone) and the sub-cosets are cut into
    row pieces: the checksum of the owner's copy is then the only witness evidence"""
    res = _run(world, names, mode="spmd", extra=["--diverge-witness"])
    for nm in names:
        assert res[nm]["refused_all"], (nm, res[nm])


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("world", [2, 4])
def test_spmd_c3_k22_at_size(world):
    """BASELINE configs[3] at its size: the C3 k = 22 proof with every commitment MSM split
    into `world` point slabs and the extended domain's sub-cosets divided over the ranks
    (gloo ranks sharing this box's GPU); every rank's bytes == the single-GPU proof.  With
    more ranks than the 2 sub-cosets, the non-owners receive their coefficient slabs of the
    circuit's columns (a second exchange).  At 2 ranks rank 0 also checks its bytes against
    the CPU oracle directly (tests/_oracle.py create_proof on the same SRS and witness)"""
    extra = ["--one-variant"] + (["--oracle"] if world == 2 else [])
    res = _run(world, ["c3_k22"], mode="spmd", extra=extra, timeout=1100)
    print("c3_k22", world, res["c3_k22"])
    assert res["c3_k22"]["same"] and res["c3_k22"]["same_ranks"], res
    # 11 MSMs: the stages' commitments travel together (advice 3, permutation + vanishing
    # 4, h 2: one host all-gather each), SHPLONK's two lone ones in the per-MSM all-gather;
    # exchanges: 1 (h by coefficient slabs) at 2 ranks; at 4 ranks the row pieces add the 3
    # advice columns' pieces and the h rows gathered at the leaders
    assert res["c3_k22"]["gathers"] == 2, res
    assert res["c3_k22"]["host_gathers"] == (6 if world == 2 else 7), res
    assert res["c3_k22"]["exchanges"] == (1 if world == 2 else 5), res
    if world == 2:  # rank 0's sharded bytes == the CPU oracle's create_proof (tests/_oracle.py)
        assert res["c3_k22"]["oracle_same"], res


@pytest.mark.timeout(1200)
def test_spmd_keccak_k18_eight_ranks():
    """BASELINE configs[4] at its size and GPU count: the keccak-style circuit at k = 18
    over 8 SPMD ranks (MSM slabs, 4 sub-cosets over the first 4 ranks); bytes == one GPU"""
    res = _run(8, ["keccak_k18"], mode="spmd", extra=["--one-variant"], timeout=1100)
    assert res["keccak_k18"]["same"] and res["keccak_k18"]["same_ranks"], res


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


@pytest.mark.parametrize("exchange", ["overlapped", "blocking"])
def test_spmd_rccl_four_gpus_column_exchanges(exchange):
    """libh2g's RCCL communicators with column ownership (from 4 ranks): the column
    exchanges posted on the second communicator (h2g_comm_set_exchange_overlap(1), what
    bench.py --overlap-exchange selects) and blocking on the first (the default); needs
    >= 4 GPUs, one per rank"""
    if _gpus() < 4:
        pytest.skip("needs four GPUs")
    cases = ["c3_k14", "keccak_k12"]
    extra = ["--one-variant"] + (["--sync-exchange"] if exchange == "blocking" else [])
    res = _run(4, cases, backend="nccl", transport="native", mode="spmd", extra=extra)
    for nm in cases:
        assert res[nm]["same"] and res[nm]["same_ranks"], (nm, res[nm])
