"""One create_proof split over WORLD_SIZE ranks must give the same proof bytes as the
single-device prover: --mode slab (rank 0 proves, h2g_dist slab transport or libh2g's
RCCL communicators) or --mode spmd (every rank proves its point slab of each MSM,
partials all-gathered).  Launched by tests/test_gpu_sharded.py:
  python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
      --master-port P tests/_shard_prove.py --backend gloo case...
With --backend gloo every rank may share one GPU (host-staged slabs); with nccl each
rank needs its own GPU (RCCL)."""
import argparse
import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "yet-another-halo2-fork_amd"), HERE, os.path.join(REPO, "oracle", "py")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import h2g  # noqa: E402
import h2g_circuit as hc  # noqa: E402
import h2g_dist as D  # noqa: E402

CASES = {
    "simple_k6": lambda: hc.simple_example(6),
    "mixed_k10": lambda: hc.mixed_circuit(10, seed=5),
    "lookup_k11": lambda: hc.lookup_circuit(11, seed=8),
    "keccak_k12": lambda: hc.keccak_style(12, words=16, seed=9),
    "c3_k14": lambda: hc.synthetic_c3(14, h2g.DeviceOps, seed=4),
    "challenge_k9": lambda: hc.challenge_circuit(9, seed=9, extended=True),  # phases: witness source
    # BASELINE sizes: configs[3] (C3 at k = 22) and configs[4] (the keccak-style circuit at k = 18)
    "c3_k22": lambda: hc.synthetic_c3(22, h2g.DeviceOps, seed=22),
    "keccak_k18": lambda: hc.keccak_style(18, words=16),
    # two MyCircuit instances with different inputs (witnesses, instances) in one proof
    "multi_my_k6": lambda: _multi_my(),
}


def _multi_my():
    circ, w0, f0 = hc.my_circuit(6, input_value=42)
    _, w1, f1 = hc.my_circuit(6, input_value=1000)
    return circ, [w0, w1], [f0, f1], "multi"


def _prove(pk, case, **kw):
    if len(case) == 4:  # (circuit, witnesses, fills, "multi"): several circuits in one proof
        return pk.create_proof_multi(case[1], fills=case[2], **kw)
    if len(case) == 3:  # (circuit, instance witness, fill): Prover::commit_phase per phase
        return pk.create_proof_phased(case[2], case[1], **kw)[0]
    return pk.create_proof(case[1], **kw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--transport", default="torch", choices=("torch", "native"),
                    help="h2g_dist over torch.distributed, or libh2g's RCCL communicators (nccl only)")
    ap.add_argument("--mode", default="slab", choices=("slab", "spmd"),
                    help="slab: rank 0 proves, peers serve slabs; spmd: every rank proves its slab")
    ap.add_argument("--no-subcosets", action="store_true",
                    help="spmd: replicate the extended-domain work instead of splitting the sub-cosets")
    ap.add_argument("--no-slabs", action="store_true",
                    help="spmd: replicate the evaluations / SHPLONK tail (no host all-gather)")
    ap.add_argument("--bcast-h", action="store_true",
                    help="spmd: broadcast the sub-cosets' h evaluations instead of exchanging coefficient slabs")
    ap.add_argument("--weights", default="", help="spmd: slab weights (h2g.spmd_set_weights), comma separated")
    ap.add_argument("--diverge", action="store_true",
                    help="spmd: the last rank proves with another RNG seed; every rank must refuse the proof")
    ap.add_argument("--diverge-witness", action="store_true",
                    help="spmd: the last rank proves another witness (one advice value changed); every rank "
                         "must refuse the proof")
    ap.add_argument("--no-column-owners", action="store_true",
                    help="spmd: point slabs for every MSM, no column ownership (h2g_spmd_set_column_owners(0))")
    ap.add_argument("--oracle", action="store_true",
                    help="spmd: rank 0 also compares the sharded proof with the CPU oracle's create_proof "
                         "(tests/_oracle.py) on the same SRS, witness and seed")
    ap.add_argument("--one-variant", action="store_true",
                    help="prove each case once (default seed) instead of twice (large cases)")
    ap.add_argument("--sync-exchange", action="store_true",
                    help="spmd: every column-ownership exchange completes on return (no overlapped post / wait)")
    ap.add_argument("cases", nargs="+")
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local if args.backend == "nccl" else 0
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")
    h2g.init([dev])
    native = args.transport == "native"
    if native:  # the library's communicators; the id travels over torch.distributed
        uid = torch.zeros(256, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(h2g.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        h2g.comm_init(bytes(uid.cpu().numpy().tobytes()), world, rank)
    if args.mode == "spmd":
        spmd_main(args, rank, world, native)
        return
    results = {}
    for name in args.cases:
        case = CASES[name]()
        circ = case[0]
        params = h2g.Params(circ.k, s=np.asarray(hc.fr_to_limbs(0x5eed + circ.k), dtype=np.uint64))
        P = 1 << circ.k
        if rank == 0:
            pk = h2g.ProvingKey(params, circ)
            want = [_prove(pk, case), _prove(pk, case, seed=bytes(range(32)), vanishing_threads=3)]
            params.set_slab(*D.slab(P, world, 0))
            if native:
                h2g.comm_install(params)
            else:
                cl = D.SlabClient(dist, points=P)
                cl.install()
            try:
                got = [_prove(pk, case), _prove(pk, case, seed=bytes(range(32)), vanishing_threads=3)]
            finally:
                if native:
                    h2g.comm_stop()
                else:
                    D.SlabClient.uninstall()
                    cl.stop()
            results[name] = {"same": got == want, "bytes": len(got[0]), "msms": None}
            pk.close()
        else:
            params.set_slab(*D.slab(P, world, rank))
            if native:  # a rank 0 that aborted would otherwise leave this peer waiting forever
                h2g.comm_set_serve_timeout(120.0)
            served = h2g.comm_serve(params) if native else D.SlabWorker(dist, params=params).serve()
            results[name] = {"served": served}
        params.close()
        dist.barrier()
    if rank != 0:  # peers report how many slabs they served
        counts = [results[nm]["served"] for nm in args.cases]
    else:
        counts = [0] * len(args.cases)
    t = torch.tensor(counts, dtype=torch.int64)
    if args.backend == "nccl":
        t = t.cuda()
    gathered = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gathered, t)
    if rank == 0:
        for i, nm in enumerate(args.cases):
            results[nm]["msms"] = [int(g[i]) for g in gathered[1:]]
        print("SHARD_RESULT " + json.dumps(results), flush=True)
    if native:
        h2g.comm_destroy()
    h2g.shutdown()
    dist.destroy_process_group()


def spmd_main(args, rank, world, native):
    """every rank: the single-device proofs first, then the same proofs with its slab of
    every MSM and the all-gathered partials; all ranks must print identical bytes"""
    import hashlib
    results = {}
    variants = [{}] if args.one_variant else [{}, {"seed": bytes(range(32)), "vanishing_threads": 3}]
    weights = [int(x) for x in args.weights.split(",")] if args.weights else None
    h2g.spmd_set_weights(weights)
    h2g.spmd_set_column_owners(not args.no_column_owners)
    for name in args.cases:
        case = CASES[name]()
        circ = case[0]
        params = h2g.Params(circ.k, s=np.asarray(hc.fr_to_limbs(0x5eed + circ.k), dtype=np.uint64))
        P = 1 << circ.k
        params.set_slab(*D.slab(P, world, rank, weights=weights))
        pk = h2g.ProvingKey(params, circ)
        want = [_prove(pk, case, **kw) for kw in variants]
        g = None
        if native:  # the RCCL test runs both: overlapped (default here) and --sync-exchange
            h2g.comm_set_exchange_overlap(not args.sync_exchange)
            h2g.comm_spmd_install(not args.no_subcosets)
        else:
            g = D.SpmdGather(dist, subcosets=not args.no_subcosets, slabs=not args.no_slabs,
                             h_exchange=not args.bcast_h, exchange_async=not args.sync_exchange)
            g.install()
        if args.diverge or args.diverge_witness:  # the digest check must catch a diverged rank
            try:
                if args.diverge:  # the last rank draws other randomness
                    seed = bytes([9] * 32) if rank == world - 1 else bytes([7] * 32)
                    _prove(pk, case, seed=seed)
                else:  # the last rank holds another witness: advice column 0, row 3 changed
                    c2 = list(case)
                    if rank == world - 1:
                        w = copy.deepcopy(case[1])
                        w.advice[0, 3, 0] ^= np.uint64(1)
                        c2[1] = w
                    _prove(pk, tuple(c2))
                err = ""
            except h2g.H2GError as e:
                err = str(e)
            finally:
                if native:
                    h2g.comm_spmd_uninstall()
                else:
                    D.SpmdGather.uninstall()
            ok = torch.tensor([1 if "diverged" in err else 0], dtype=torch.int64)
            if args.backend == "nccl":
                ok = ok.cuda()
            allok = [torch.empty_like(ok) for _ in range(world)]
            dist.all_gather(allok, ok)
            results[name] = {"refused_all": all(int(a.item()) == 1 for a in allok), "error": err[:200]}
            pk.close()
            params.close()
            dist.barrier()
            continue
        try:
            got = [_prove(pk, case, **kw) for kw in variants]
        finally:
            if native:
                h2g.comm_spmd_uninstall()
            else:
                D.SpmdGather.uninstall()
        digest = hashlib.sha256(b"".join(got)).digest()
        t = torch.frombuffer(bytearray(digest), dtype=torch.uint8).to(torch.int64)
        if args.backend == "nccl":
            t = t.cuda()
        allh = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allh, t)
        same_ranks = all(bool(torch.equal(a.cpu(), allh[0].cpu())) for a in allh)
        ok = torch.tensor([1 if got == want else 0], dtype=torch.int64)
        if args.backend == "nccl":
            ok = ok.cuda()
        allok = [torch.empty_like(ok) for _ in range(world)]
        dist.all_gather(allok, ok)
        results[name] = {"same": all(int(a.item()) == 1 for a in allok), "same_ranks": same_ranks,
                         "bytes": len(got[0]), "gathers": None if g is None else g.calls,
                         "bcasts": None if g is None else g.bcasts,
                         "host_gathers": None if g is None else g.host_gathers,
                         "exchanges": None if g is None else g.exchanges}
        if args.oracle and rank == 0 and len(case) == 2:  # the sharded bytes against the checker itself
            import _oracle as O
            gg, gl = params.export()
            threads = max(1, min(16, len(os.sched_getaffinity(0))))
            print(f"[rank 0] oracle create_proof k={circ.k} on {threads} threads", flush=True)
            results[name]["oracle_same"] = got[0] == O.create_proof(circ, case[1], gg, gl, threads=threads)
            del gg, gl
        pk.close()
        params.close()
        dist.barrier()
    if rank == 0:
        print("SHARD_RESULT " + json.dumps(results), flush=True)
    if native:
        h2g.comm_destroy()
    h2g.shutdown()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
