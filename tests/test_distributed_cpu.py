"""The N > 1 bench path on CPU with gloo, world_size 2: MSM point slabs
sharded over ranks, per-rank partial sums exchanged with all_gather and combined
with the host EC add of the C ABI (h2g_g1_add_affine -- host code, no GPU), timing
reduced with max over ranks.  The result must equal the unsharded MSM."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, sc, bases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import h2g
        n = len(sc) // world
        lo = rank * n
        part = O.msm_best(sc[lo:lo + n], bases[lo:lo + n], 2)   # this rank's slab
        parts = bench.gather_partials(part, dist, world, "cpu")
        total = bench.combine_partials(parts, h2g.g1_add_affine)
        t = bench.max_over_ranks(0.5 + rank, dist, world, "cpu")
        q.put((rank, total.tobytes(), t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_msm_gloo(world):
    r = np.random.default_rng(3)
    n = 512
    s = O.random_fr(r, 1)[0]
    bases = O.srs_powers(s, n)
    sc = O.random_fr(r, n)
    want = O.msm_best(sc, bases, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(i, world, port, sc, bases, q)) for i in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, total, t in out:
        assert np.array_equal(np.frombuffer(total, dtype=np.uint64), want), rank
        assert t == 0.5 + (world - 1)   # max over ranks


# ---------------------------------------------------------------- one proof, N ranks
def _slab_worker(rank, world, port, jobs, bases, q):
    """h2g_dist's slab protocol over gloo: rank 0 = SlabClient (the prover's transport),
    ranks 1.. = SlabWorker with the oracle MSM as engine (no GPU here)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import h2g
        import h2g_dist as D

        def engine(base_set, lo, n, buf):
            sc = buf.numpy().view(np.uint64).reshape(n, 4)
            pt = O.msm_best(sc, bases[base_set][lo:lo + n], 1)
            return pt, not pt.any()

        if rank == 0:
            P = len(bases[0])
            cl = D.SlabClient(dist, points=P)
            totals = []
            # several MSMs outstanding at once (the prover launches ahead of collecting)
            for seq, (base_set, sc) in enumerate(jobs):
                cl.launch_host(seq, base_set, sc)
            for seq, (base_set, sc) in enumerate(jobs):
                lo, hi = D.slab(len(sc), world, 0, P)
                own = O.msm_best(sc[lo:hi], bases[base_set][lo:hi], 1) if hi > lo else np.zeros(8, np.uint64)
                total = own
                for pt, is_id in cl.collect(seq):
                    if not is_id:
                        total = pt.copy() if not total.any() else h2g.g1_add_affine(total, pt)
                totals.append(total.tobytes())
            cl.stop()
            q.put((rank, totals))
        else:
            q.put((rank, D.SlabWorker(dist, engine=engine).serve()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_protocol_gloo(world):
    """every MSM of a proof split over `world` ranks sums to the unsharded MSM, for both
    base sets, slab sizes down to empty slabs (n < world), launches pipelined"""
    r = np.random.default_rng(11 + world)
    n = 256
    s = O.random_fr(r, 1)[0]
    bases = [O.srs_powers(s, n), O.srs_powers(O.random_fr(r, 1)[0], n)]
    jobs = [(0, O.random_fr(r, n)), (1, O.random_fr(r, n)), (1, O.random_fr(r, 2)), (0, O.random_fr(r, 77)),
            (1, np.zeros((n, 4), np.uint64))]
    want = [O.msm_best(sc, bases[b][:len(sc)], 2).tobytes() for b, sc in jobs]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_worker, args=(i, world, port, jobs, bases, q)) for i in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == want
    for rk in range(1, world):
        assert out[rk] == len(jobs)   # every MSM reached every peer (empty slabs answer identity)


# ---------------------------------------------------------------- SPMD: every rank proves
def _spmd_worker(rank, world, port, jobs, bases, q):
    """h2g_dist.SpmdGather over gloo with the prover's slab rule (h2g_dist.slab of the
    params' P) and its rank-order sum (csrc/prover.cpp commit_collect), the oracle MSM as
    each rank's slab engine (no GPU here): every rank must hold the unsharded MSM"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import h2g
        import h2g_dist as D

        g = D.SpmdGather(dist)
        P = len(bases[0])
        totals = []
        for seq, (base_set, sc) in enumerate(jobs):
            lo, hi = D.slab(len(sc), world, rank, P)
            own = O.msm_best(sc[lo:hi], bases[base_set][lo:hi], 1) if hi > lo else np.zeros(8, np.uint64)
            # payload = partial, identity flag, 4 digest words (h2g.SPMD_WORDS, H2G_SPMD_WORDS)
            digest = np.array([seq, 1, 2, 3], np.uint64)
            mine = np.concatenate([own, np.array([0 if own.any() else 1], np.uint64), digest])
            assert len(mine) == h2g.SPMD_WORDS
            allp = g.allgather(seq, mine)
            assert allp.shape == (world, h2g.SPMD_WORDS)
            assert all(np.array_equal(allp[r, 9:], digest) for r in range(world))
            assert np.array_equal(allp[rank], mine)
            total = np.zeros(8, np.uint64)
            for r in range(world):
                if not allp[r, 8]:
                    total = allp[r, :8].copy() if not total.any() else h2g.g1_add_affine(total, allp[r, :8])
            totals.append(total.tobytes())
        q.put((rank, totals, g.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_spmd_gather_gloo(world):
    r = np.random.default_rng(29 + world)
    n = 256
    s = O.random_fr(r, 1)[0]
    bases = [O.srs_powers(s, n), O.srs_powers(O.random_fr(r, 1)[0], n)]
    jobs = [(0, O.random_fr(r, n)), (1, O.random_fr(r, n - 1)), (1, O.random_fr(r, 2)),
            (0, np.zeros((n, 4), np.uint64))]
    want = [O.msm_best(sc, bases[b][:len(sc)], 2).tobytes() for b, sc in jobs]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spmd_worker, args=(i, world, port, jobs, bases, q)) for i in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, totals, calls in out:
        assert totals == want, rank
        assert calls == len(jobs)


# ---------------------------------------------------------------- SPMD slab partition
def test_weighted_slabs_partition_the_points():
    """h2g_dist.slab with SPMD weights (h2g_spmd_set_weights): contiguous, disjoint,
    covering, proportional to the weights; owner_weights lightens the sub-coset owners"""
    import h2g_dist as D
    P = 1 << 22
    for world, w in [(8, D.owner_weights(8, 23, 22, row_pieces=False)), (3, [3, 1, 2]), (4, None)]:
        sl = [D.slab(P, world, r, weights=w) for r in range(world)]
        assert sl[0][0] == 0 and sl[-1][1] == P
        assert all(sl[r][1] == sl[r + 1][0] for r in range(world - 1))
        ws = w or [1] * world
        for r in range(world):
            assert abs((sl[r][1] - sl[r][0]) - P * ws[r] / sum(ws)) <= 1
        # an MSM shorter than P: the same boundaries clipped to its length
        assert [D.slab(P - 1, world, r, P, w) for r in range(world)][-1][1] == P - 1
    nop = dict(row_pieces=False)  # sub-coset owners (no row pieces)
    assert D.owner_weights(8, 23, 22, **nop) == [10, 10] + [100] * 6  # 4x the owners: measured best 0.1
    assert D.owner_weights(4, 23, 22, **nop) == [50, 50, 100, 100]  # 2x the owners: 0.5
    assert D.owner_weights(8, 23, 22, 0.5, **nop) == [50, 50] + [100] * 6
    assert D.owner_weights(2, 23, 22) is None  # every rank owns a sub-coset
    assert D.owner_weights(8, 20, 18, **nop) == [50] * 4 + [100] * 4
    # row pieces: every rank holds an equal piece of one sub-coset -> uniform slabs
    assert D.owner_weights(8, 23, 22) is None and D.owner_weights(8, 20, 18) is None
    assert D.owner_weights(6, 20, 18) == D.owner_weights(6, 20, 18, row_pieces=False) is not None  # 6 % 4 != 0
    # the library cuts row pieces only with column owners on, SHPLONK and world >= 4
    # (prove_impl): otherwise the sub-coset owners keep their lighter slabs
    assert D.owner_weights(8, 23, 22, column_owners=False) == [10, 10] + [100] * 6
    assert D.owner_weights(8, 23, 22, multiopen="gwc") == [10, 10] + [100] * 6
    assert D.row_pieces_active(8, 23, 22) and not D.row_pieces_active(2, 23, 22)
    assert not D.row_pieces_active(8, 23, 22, column_owners=False)


def _host_gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import h2g_dist as D
        g = D.SpmdGather(dist)
        parts = g.allgather_host(bytes([rank]) * (5 + rank % 1))
        q.put((rank, parts, g.host_gathers))
    finally:
        dist.destroy_process_group()


def test_spmd_host_allgather_gloo():
    """the multi-open tail's scalar all-gather (h2g_spmd_transport.allgather_host) over gloo:
    every rank receives every rank's bytes in rank order"""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_gather_worker, args=(i, world, port, q)) for i in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, parts, calls in out:
        assert parts == [bytes([r]) * 5 for r in range(world)], rank
        assert calls == 1


def _a2a_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        import h2g_dist as D
        members = [1, 2, 3]  # a sub-group: group index != global rank
        grp = dist.new_group(members)
        if rank in members:
            me = members.index(rank)
            W = len(members)
            send_bytes = [me + p + 1 for p in range(W)]  # to member p: me + p + 1 bytes of value 10 me + p
            recv_bytes = [p + me + 1 for p in range(W)]
            sb = torch.cat([torch.full((send_bytes[p],), 10 * me + p, dtype=torch.uint8) for p in range(W)])
            rb = torch.zeros(sum(recv_bytes), dtype=torch.uint8)
            D.host_all_to_all(dist, grp, me, W, sb, send_bytes, rb, recv_bytes)
            q.put((rank, rb.tolist()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_spmd_host_all_to_all_subgroup_gloo():
    """SpmdGather.exchange's host (gloo) path on a process group that is not the default
    one: the peers are addressed by their global ranks, the byte offsets by group index"""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(i, world, port, q)) for i in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in out.items():
        me = [1, 2, 3].index(rank)
        want = []
        for p in range(3):
            want += [10 * p + me] * (p + me + 1)
        assert got == want, (rank, got)
