"""CPU, world_size 2 over gloo: the N>1 path of bench.py.

Each rank extracts its x-slab of the synthetic lattice with the default HALO (three cells)
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
    """cuts: x-slab cuts, or ("blocks", dims) for a block split."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle.subdivide as od
        from tropical.synthetic import block_lattice, slab_lattice
        torch.set_num_threads(2 if world <= 4 else 1)
        d = load(CASE)
        net = oracle_net(d)
        n = int(d["lattice_n"])
        from tropical.distributed import HALO, Blocks, gather_complex, slab_marks, stitch
        if cuts[0] == "blocks":
            cuts = Blocks(n, cuts[1])
            V, E = block_lattice(d["marks"], *cuts.box(rank, HALO))
        else:
            assert cuts[-1] == n - 1
            x0, x1 = slab_marks(cuts, rank)
            V, E = slab_lattice(d["marks"], x0, x1)
        coll = bench.Collective(torch.device("cpu"))

        def sync(kind, value):
            return int(coll(np.array([value], dtype=np.int64), "max")[0])

        with torch.no_grad():
            V, E, _ = od.run_steps(torch.from_numpy(V), torch.from_numpy(E), net, 1e-4, sync=sync)
        from tropical.distributed import halo_check
        halo_check(V, E, torch.from_numpy(d["marks"]), cuts)
        owned, first, gE = stitch(V, E, torch.from_numpy(d["marks"]), cuts)
        SV, SE = gather_complex(owned, first, gE)
        if rank == 0:
            np.savez(os.path.join(outdir, "stitched.npz"), V=SV.numpy(), E=SE.numpy())
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def whole():
    """The unsharded complex of CASE (oracle), computed once for the module."""
    import oracle.subdivide as od
    from tropical.synthetic import lattice_edges, lattice_vertices
    d = load(CASE)
    net = oracle_net(d)
    with torch.no_grad():
        V, E, _ = od.run_steps(torch.from_numpy(lattice_vertices(d["marks"])),
                               torch.from_numpy(lattice_edges(int(d["lattice_n"]))), net, 1e-4)
    return V, E


def test_slab_cuts_cover_the_lattice():
    from tropical.distributed import HALO, HALOS, slab_cuts, slab_marks
    assert HALOS[0] == HALO and list(HALOS) == sorted(set(HALOS))
    for G, world in ((128, 1), (161, 2), (203, 4), (256, 8)):
        cuts = slab_cuts(G, world)
        assert cuts[0] == 0 and cuts[-1] == G - 1 and cuts == sorted(set(cuts))
        for r in range(world):
            x0, x1 = slab_marks(cuts, r)
            assert x0 == max(cuts[r] - HALO, 0) and x1 == min(cuts[r + 1] + HALO, G - 1)


def test_block_split():
    """block_dims is the most cubic factorisation; every cell of the grid has
    exactly one owning block; the 256^3 / 8-rank split at a 3-cell halo
    extracts 6.7-6.8 % redundant cells per rank (x-slabs: 15.8 %)."""
    from tropical.distributed import Blocks, block_dims, slab_cuts
    assert [block_dims(w) for w in (1, 2, 3, 4, 6, 8, 12, 16)] == [
        (1, 1, 1), (2, 1, 1), (3, 1, 1), (2, 2, 1), (3, 2, 1), (2, 2, 2), (3, 2, 2), (4, 2, 2)]
    B = Blocks(256, (2, 2, 2))
    assert [B.rank_of(B.index(r)) for r in range(8)] == list(range(8))
    cells = np.zeros((255, 255, 255), dtype=np.int32)
    for r in range(8):
        lo, hi = B.owned(r)
        cells[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] += 1
    assert (cells == 1).all()
    assert abs(B.redundant_frac(0, 3) - 0.0672) < 1e-3
    assert abs(Blocks.xslabs(slab_cuts(256, 8)).redundant_frac(1, 3) - 0.158) < 1e-3
    with pytest.raises(ValueError, match="non-empty"):
        Blocks(3, (4, 1, 1))  # more blocks than cells along x


def test_block_owner_and_edge_rules():
    """Per axis the x-slab owner rule; an edge belongs to the block of the
    highest cell whose closure holds both endpoints."""
    from tropical.distributed import Blocks, edge_owner, owner_of
    marks = torch.linspace(0, 1, 11)
    B = Blocks(11, (2, 2, 1), [[0, 4, 10], [0, 6, 10], [0, 10]])
    p = lambda i: float(marks[i]) * 2 - 1  # on mark plane i
    c = lambda i: (float(marks[i]) + 0.05) * 2 - 1  # inside cell i
    V = torch.tensor([[p(4), p(6), 0.0],    # planes x4, y6 -> block (0, 0)
                      [c(4), p(6), 0.0],    # cell x4, plane y6 -> (1, 0)
                      [c(4), c(6), 0.0],    # (1, 1)
                      [p(4), c(6), 0.0],    # (0, 1)
                      [p(0), p(0), 0.0],    # (0, 0)
                      [p(10), p(10), 0.0]])  # (1, 1)
    assert owner_of(V, marks, B).tolist() == [0, 2, 3, 1, 0, 3]
    E = torch.tensor([[0, 1], [0, 2], [0, 3], [1, 2], [3, 2], [5, 5]])
    # each edge lies in cell (x4, y6) (per axis the lower endpoint offset),
    # block (1, 1) = rank 3; the last one on the grid's far corner line
    assert edge_owner(V, E, marks, B).tolist() == [3, 3, 3, 3, 3, 3]


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
@pytest.mark.parametrize("world", [2, 3, "blocks4", "blocks8"])
def test_gloo_ranks_reproduce_the_unsharded_complex(tmp_path, world, whole):
    """x-slabs (2, 3 ranks) and blocks (2 x 2 x 1, 2 x 2 x 2 ranks: cut faces
    along two and three axes, edges and corners where 4 and 8 blocks meet)."""
    if isinstance(world, str):
        from tropical.distributed import block_dims
        world = int(world[len("blocks"):])
        part = ("blocks", block_dims(world))
    else:
        part = CUTS[world]
    mp.spawn(_slab_worker, args=(world, _free_port(), str(tmp_path), part), nprocs=world,
             join=True)
    d = load(CASE)
    V, E = whole
    assert (V.shape[0], E.shape[0]) == tuple(d["pre_VE"])
    whole_v, whole_e = _canon(V.numpy(), E.numpy())
    # stitched: one global numbering, no vertex or edge twice, same complex
    z = np.load(tmp_path / "stitched.npz")
    assert z["V"].shape[0] == V.shape[0] and z["E"].shape[0] == E.shape[0]
    sv, se = _canon(z["V"], z["E"])
    assert sv == whole_v and se == whole_e


def _halo_worker(rank, world, port, outdir, corrupt):
    """Both ranks hold the same unsharded complex (exact views); rank 1
    optionally drops one edge next to the cut: halo_check must raise."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tropical.distributed import halo_check, x_grid
        d = load(CASE)
        z = np.load(os.path.join(outdir, "whole.npz"))
        V, E = torch.from_numpy(z["V"]), torch.from_numpy(z["E"])
        marks = torch.from_numpy(d["marks"])
        cuts = CUTS[2]
        if corrupt and rank == 1:
            off, on = x_grid(V, marks)
            near = (off[E[:, 0]] == cuts[1]) & ~on[E[:, 0]] & (off[E[:, 1]] == cuts[1])
            drop = int(torch.nonzero(near)[0])
            E = torch.cat([E[:drop], E[drop + 1:]])
        try:
            halo_check(V, E, marks, cuts)
            res = "ok"
        except RuntimeError as ex:
            res = str(ex)
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_halo_check_detects_a_missing_edge(tmp_path, corrupt, whole):
    V, E = whole
    np.savez(tmp_path / "whole.npz", V=V.numpy(), E=E.numpy())
    mp.spawn(_halo_worker, args=(2, _free_port(), str(tmp_path), corrupt), nprocs=2, join=True)
    res = [(tmp_path / f"r{r}.txt").read_text() for r in range(2)]
    if corrupt:
        assert all("halo_check" in r and f"cut {CUTS[2][1]}" in r for r in res)
    else:
        assert res == ["ok", "ok"]


def test_balanced_cuts():
    from tropical.distributed import balanced_cuts
    load_ = torch.tensor([0, 0, 10, 10, 0, 0, 10, 10, 0, 0])
    assert balanced_cuts(load_, 1) == [0, 10]
    c = balanced_cuts(load_, 2)
    assert c[0] == 0 and c[-1] == 10 and 3 <= c[1] <= 6
    c = balanced_cuts(torch.zeros(5, dtype=torch.int64), 5)
    assert c == [0, 1, 2, 3, 4, 5]
    c = balanced_cuts(torch.tensor([100, 0, 0, 0, 0, 0]), 3)
    assert c == sorted(set(c)) and len(c) == 4


def test_slab_restrict_matches_slab_lattice():
    """The skeleton shard's restriction of a mark-plane complex equals the
    lattice slab layout (order-preserving ids, edges in order)."""
    from tropical.distributed import slab_restrict
    from tropical.synthetic import lattice_edges, lattice_vertices, slab_lattice
    d = load(CASE)
    n = int(d["lattice_n"])
    V = torch.from_numpy(lattice_vertices(d["marks"]))
    E = torch.from_numpy(lattice_edges(n))
    for x0, x1 in ((0, 5), (7, 15), (20, n - 1)):
        v, e = slab_restrict(V, E, torch.from_numpy(d["marks"]), x0, x1)
        sv, se = slab_lattice(d["marks"], x0, x1)
        assert torch.equal(v, torch.from_numpy(sv))
        # the lattice slab orders x-edges, then y, then z: the same subsequence
        assert sorted(map(tuple, e.tolist())) == sorted(map(tuple, se.tolist()))
        assert e.shape[0] == se.shape[0]
    # boxes (blocks with their halo) likewise
    from tropical.distributed import box_restrict
    from tropical.synthetic import block_lattice
    for lo, hi in (((0, 3, 5), (9, 14, 20)), ((12, 0, 0), (n - 1, 11, n - 1))):
        v, e = box_restrict(V, E, torch.from_numpy(d["marks"]), lo, hi)
        sv, se = block_lattice(d["marks"], lo, hi)
        assert torch.equal(v, torch.from_numpy(sv))
        assert sorted(map(tuple, e.tolist())) == sorted(map(tuple, se.tolist()))


def _shm_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        shm = bench.Collective(torch.device("cpu"), shm=True)
        ref = bench.Collective(torch.device("cpu"), shm=False)
        rs = np.random.RandomState(rank)
        bad = []
        for it in range(200):  # many calls: both banks reused, ranks racing
            v = rs.randint(-2**40, 2**40, size=3).astype(np.int64)
            m = np.array([rs.randint(0, 2**62) | (1 << (rank + it % 7))], dtype=np.uint64)
            for vec, op in ((v, "max"), (m, "or")):
                a, b = shm(vec, op), ref(vec, op)
                if not np.array_equal(a, b) or a.dtype != vec.dtype:
                    bad.append((it, op, a.tolist(), b.tolist()))
        shm.shm.close()
        with open(os.path.join(outdir, f"shm{rank}.txt"), "w") as f:
            f.write(repr(bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shm_collective_matches_the_library_collective(tmp_path, world):
    """tnp_shm_allreduce (host shared memory, one node) returns what the
    all_gather + host reduction returns, over 400 racing calls per rank."""
    mp.spawn(_shm_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"shm{r}.txt").read_text() == "[]"
