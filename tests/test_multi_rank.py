"""CPU, world_size 2 over gloo: the N>1 path of bench.py.

Each rank extracts its x-slab of the synthetic lattice (boundary mark plane
replicated, tropical/synthetic.py::slab_lattice == tnp_engine_lattice's
layout) and takes the reference's two whole-complex decisions per step --
"does anything split" (subpoly.py:110) and the failover override
(subpoly_debug.py:43-49) -- through bench.Collective, the same host code the
RCCL bench runs.  The union of the shards' complexes must equal the
unsharded complex exactly (bitwise coordinates; edges as coordinate pairs).
The per-slab engine work is the oracle here (no GPU); the GPU engine runs
the same decomposition in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_io import load
from helpers import oracle_net

CASE = "synth24"
CUT = 11  # slab 0 = marks [0, 11], slab 1 = [11, 23]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _canon(V, E):
    key = [tuple(r) for r in np.asarray(V, dtype=np.float32).view(np.int32)]
    verts = set(key)
    edges = {frozenset((key[a], key[b])) for a, b in np.asarray(E)}
    return verts, edges


def _slab_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle.subdivide as od
        from tropical.synthetic import slab_lattice
        torch.set_num_threads(2)
        d = load(CASE)
        net = oracle_net(d)
        n = int(d["lattice_n"])
        x0, x1 = (0, CUT) if rank == 0 else (CUT, n - 1)
        V, E = slab_lattice(d["marks"], x0, x1)
        coll = bench.Collective(torch.device("cpu"))

        def sync(kind, value):
            return int(coll(np.array([value], dtype=np.int64), "max")[0])

        with torch.no_grad():
            V, E, _ = od.run_steps(torch.from_numpy(V), torch.from_numpy(E), net, 1e-4, sync=sync)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), V=V.numpy(), E=E.numpy())
    finally:
        dist.destroy_process_group()


def test_bench_slab_cuts_cover_the_lattice():
    import bench
    for G, world in ((128, 1), (161, 2), (203, 4), (256, 8)):
        cuts = [bench.slab(G, r, world) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == G - 1
        for (a0, a1), (b0, b1) in zip(cuts, cuts[1:]):
            assert a1 == b0 and a0 < a1  # one shared boundary mark plane


@pytest.mark.slow
def test_two_gloo_ranks_reproduce_the_unsharded_complex(tmp_path):
    import oracle.subdivide as od
    from tropical.synthetic import lattice_edges, lattice_vertices
    mp.spawn(_slab_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    d = load(CASE)
    net = oracle_net(d)
    n = int(d["lattice_n"])
    with torch.no_grad():
        V, E, _ = od.run_steps(torch.from_numpy(lattice_vertices(d["marks"])),
                               torch.from_numpy(lattice_edges(n)), net, 1e-4)
    assert (V.shape[0], E.shape[0]) == tuple(d["pre_VE"])
    whole_v, whole_e = _canon(V.numpy(), E.numpy())
    union_v, union_e = set(), set()
    for r in range(2):
        z = np.load(tmp_path / f"rank{r}.npz")
        sv, se = _canon(z["V"], z["E"])
        assert sv <= whole_v and se <= whole_e  # nothing a shard invents
        union_v |= sv
        union_e |= se
    assert union_v == whole_v
    assert union_e == whole_e
