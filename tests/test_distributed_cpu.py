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
