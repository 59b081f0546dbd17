"""CPU, world_size 2 over gloo: the N>1 path of bench.py.

Each rank extracts its x-slab of the synthetic lattice with a two-cell halo
(tropical/distributed.py::slab_marks; tropical/synthetic.py::slab_lattice ==
tnp_engine_lattice's layout) and takes the reference's two whole-complex
decisions per step -- "does anything split" (subpoly.py:110) and the
failover override (subpoly_debug.py:43-49) -- through bench.Collective, the
same host code the RCCL bench runs.  The product's stitch
(tropical/distributed.py) then builds one global complex, which must equal
the unsharded complex exactly: same vertex and edge counts, bitwise
coordinates, edges as coordinate pairs.  The per-slab engine work is the
oracle here (no GPU); the GPU engine runs the same decomposition in
bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_io import load
from helpers import oracle_net

CASE = "synth24"
# world 2: cells of marks [0, 11] -> rank 0, [11, 23] -> rank 1; world 3:
# three slabs, so the middle rank has a halo and a shared plane on both sides
CUTS = {2: [0, 11, 23], 3: [0, 7, 15, 23]}


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


def _slab_worker(rank, world, port, outdir, cuts):
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
        from tropical.distributed import gather_complex, slab_marks, stitch
        assert cuts[-1] == n - 1
        x0, x1 = slab_marks(cuts, rank)
        V, E = slab_lattice(d["marks"], x0, x1)
        coll = bench.Collective(torch.device("cpu"))

        def sync(kind, value):
            return int(coll(np.array([value], dtype=np.int64), "max")[0])

        with torch.no_grad():
            V, E, _ = od.run_steps(torch.from_numpy(V), torch.from_numpy(E), net, 1e-4, sync=sync)
        owned, first, gE = stitch(V, E, torch.from_numpy(d["marks"]), cuts)
        SV, SE = gather_complex(owned, first, gE)
        if rank == 0:
            np.savez(os.path.join(outdir, "stitched.npz"), V=SV.numpy(), E=SE.numpy())
    finally:
        dist.destroy_process_group()


def test_slab_cuts_cover_the_lattice():
    from tropical.distributed import slab_cuts, slab_marks
    for G, world in ((128, 1), (161, 2), (203, 4), (256, 8)):
        cuts = slab_cuts(G, world)
        assert cuts[0] == 0 and cuts[-1] == G - 1 and cuts == sorted(set(cuts))
        for r in range(world):
            x0, x1 = slab_marks(cuts, r)
            assert x0 == max(cuts[r] - 2, 0) and x1 == min(cuts[r + 1] + 2, G - 1)


def test_owner_rule_matches_cells_and_planes():
    import torch
    from tropical.distributed import owner_of
    marks = torch.linspace(0, 1, 11)
    cuts = [0, 4, 10]
    x01 = torch.tensor([0.0, 0.05, 0.4, 0.40004, 0.45, 0.9, 1.0])
    V = torch.stack([x01 * 2 - 1, torch.zeros(7), torch.zeros(7)], 1)
    # plane 0 -> 0; cell 0 -> 0; plane 4 (and within eps) -> 0; cell 4 -> 1; planes 9, 10 -> 1
    assert owner_of(V, marks, cuts).tolist() == [0, 0, 0, 0, 1, 1, 1]


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_reproduce_the_unsharded_complex(tmp_path, world):
    import oracle.subdivide as od
    from tropical.synthetic import lattice_edges, lattice_vertices
    mp.spawn(_slab_worker, args=(world, _free_port(), str(tmp_path), CUTS[world]), nprocs=world,
             join=True)
    d = load(CASE)
    net = oracle_net(d)
    n = int(d["lattice_n"])
    with torch.no_grad():
        V, E, _ = od.run_steps(torch.from_numpy(lattice_vertices(d["marks"])),
                               torch.from_numpy(lattice_edges(n)), net, 1e-4)
    assert (V.shape[0], E.shape[0]) == tuple(d["pre_VE"])
    whole_v, whole_e = _canon(V.numpy(), E.numpy())
    # stitched: one global numbering, no vertex or edge twice, same complex
    z = np.load(tmp_path / "stitched.npz")
    assert z["V"].shape[0] == V.shape[0] and z["E"].shape[0] == E.shape[0]
    sv, se = _canon(z["V"], z["E"])
    assert sv == whole_v and se == whole_e
