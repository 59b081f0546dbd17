"""Multi-GPU x-slab sharding of the extraction.

One process per GPU.  The cells between mark planes cuts[r] and cuts[r+1]
of the x axis belong to rank r, which also owns the mark planes
(cuts[r], cuts[r+1]] (rank 0 also plane 0).  Each rank extracts the lattice
of its cells plus a HALO of HALO cell columns on either side (slab_marks),
with the reference's two whole-complex decisions made global (``allreduce``
of run_steps: "does anything split", subpoly.py:110, and the failover
override, subpoly_debug.py:43-49).

Why the halo: a vertex within eps of a mark plane is ON that plane in the
reference's grid regions (tropical.py:227-236), so it joins regions -- and
connecting edges -- of the cells on both sides, whichever side created it.
A slab cut exactly at the plane misses those edges (measured: 930 of 21.9M
splits at 161^3 / 2 ranks).  A halo computes them; what the halo itself
misses at its OUTER plane can reach one cell further in only through another
such eps coincidence (a vertex split off a missing edge within eps of the
next plane), at most one cell per active step, so each halo column divides
the residual by the chance of a coincidence (one column still left 3
vertices of 23.6M at 161^3; two suffice there, three at 203^3 and 256^3 with
seed 6).  The width is therefore FOUND: bench.py and subpoly_sharded() try
the widths of HALOS in turn until halo_check (below) passes.

Stitching (one pair of all_gathers, RCCL over xGMI / gloo on CPU):
* vertex owner = the rank owning its cell or plane (grid sense, eps rule);
* edge owner = the larger owner of its endpoints; a rank keeps its edges;
* owned vertices get global ids by an exclusive scan of the owned counts;
* a rank's kept edges can reference vertices of the lower neighbour only on
  the shared plane: the lower rank's owned upper-plane records (coordinate
  bits + global id) are matched bitwise on the device.

Regions are (grid cell x sign pattern), so pairs, connecting edges and faces
never span cells: the stitched complex equals the unsharded one up to the
vertex numbering (the reference interleaves tiles), which is why parity at
N > 1 is checked after canonicalisation (tests/test_multi_rank.py).

Exactness is CHECKED, not assumed: halo_check() has both neighbours of every
cut fingerprint the complex they each computed in the two cells next to the
cut (and the cut plane), and raises on any difference.  A slab's own errors
start at its outer halo boundary; to reach anything a rank keeps they must
cross those two cells, where the neighbour -- for which they are interior --
computed them from a different boundary.

Stanford nets (BASELINE config 4): every rank computes the reference's
skeleton on its 128-mark tiles (tropical.py:176-181, per-tile max_grad),
cuts the x axis into slabs of equal skeleton-edge count (balanced_cuts) and
keeps its slab plus halo (slab_restrict) -- subpoly_sharded().
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
from torch import Tensor


class ShmCollective:
    """The per-step agreements (run_steps' ``allreduce(vec, op)``) between
    the ranks of ONE node through host shared memory (csrc/shm.cpp,
    tnp_shm_*): every rank writes its <= 16 words and spins on one atomic
    counter -- no library collective, no device copies.  Same results as an
    all_gather + host reduction: "max" (int64), "or" / "and" (64-bit masks),
    "sum"."""

    OPS = {"max": 0, "or": 1, "sum": 2, "and": 3}

    def __init__(self, group=None):
        import ctypes as C
        import os
        import secrets
        from . import _hip
        self._C, self._lib = C, _hip.lib()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        name = [f"/tnp_{os.getpid()}_{secrets.token_hex(6)}" if rank == 0 else None]
        dist.broadcast_object_list(name, src=dist.get_global_rank(group, 0) if group else 0, group=group)
        self.name = name[0].encode()
        h = C.c_void_p()
        if rank == 0:
            _hip.check(self._lib.tnp_shm_open(self.name, rank, world, 1, C.byref(h)), "tnp_shm_open")
        dist.barrier(group=group)
        if rank != 0:
            _hip.check(self._lib.tnp_shm_open(self.name, rank, world, 0, C.byref(h)), "tnp_shm_open")
        dist.barrier(group=group)
        if rank == 0:
            self._lib.tnp_shm_unlink(self.name)  # the mappings stay; nothing left in /dev/shm
        self.h = h
        self._in = np.zeros(16, dtype=np.int64)  # csrc/shm.cpp SHM_WORDS
        self._out = np.zeros(16, dtype=np.int64)

    def __call__(self, vec, op: str):
        from . import _hip
        vec = np.asarray(vec)
        n = vec.size
        bits = op in ("or", "and")
        words = np.ascontiguousarray(vec.astype(np.uint64 if bits else np.int64)).view(np.int64)
        self._in[:n] = words
        _hip.check(self._lib.tnp_shm_allreduce(self.h, self._in.ctypes.data, n, self.OPS[op],
                                               self._out.ctypes.data), "tnp_shm_allreduce")
        res = self._out[:n].copy()
        return res.view(np.uint64).astype(vec.dtype) if bits else res

    def close(self):
        if self.h:
            self._lib.tnp_shm_close(self.h)
            self.h = None


def slab_cuts(n_marks: int, world: int) -> list:
    """Mark indices cutting the x axis into `world` slabs of cells."""
    return [round(r * (n_marks - 1) / world) for r in range(world + 1)]


HALO = 2  # first halo tried: cell columns extracted beyond each cut plane
# the widths tried in turn while halo_check still sees a difference (the
# error front of a slab's outer boundary moves inward by at most one cell per
# active step, and only through eps coincidences: how far it gets depends on
# the net and the lattice, so the width is found, then checked again)
HALOS = (2, 3, 4, 6, 8, 12, 16, 24, 33)


def slab_marks(cuts: list, rank: int, halo: int = HALO):
    """Marks [x0, x1] a rank extracts: its cells plus `halo` cells each side."""
    return max(cuts[rank] - halo, cuts[0]), min(cuts[rank + 1] + halo, cuts[-1])


def balanced_cuts(cell_load: Tensor, world: int) -> list:
    """Cut the x cells 0..n-1 (n = n_marks - 1) into `world` slabs of about
    equal load (e.g. skeleton edges per x cell); every slab gets >= 1 cell."""
    n = int(cell_load.shape[0])
    if world > n:
        raise ValueError(f"{world} slabs of {n} cells")
    c = torch.cumsum(cell_load.to(torch.float64).cpu(), 0)
    tot = float(c[-1]) if n else 0.0
    cuts = [0]
    for r in range(1, world):
        k = int(torch.searchsorted(c, torch.tensor(tot * r / world, dtype=torch.float64)).item()) + 1
        cuts.append(min(max(k, cuts[-1] + 1), n - (world - r)))
    cuts.append(n)
    return cuts


def x_grid(vertices: Tensor, marks: Tensor, eps: float = 1e-4):
    """(offset, on_mark) of the x coordinate in the grid-region sense of
    TropicalHashGrid.region (tropical.py:227-236) on x01 = (x + 1) / 2
    (Net.preprocess, model.py:78-79) -- the engine's grid word, bit for bit."""
    x01 = (vertices[:, 0] + 1.0) / 2.0
    off = torch.searchsorted(marks, x01 + eps) - 1
    mk = marks[torch.where(off < 0, off + marks.shape[0], off)]
    return off, ~((mk - x01).abs() > eps)


def owner_of(vertices: Tensor, marks: Tensor, cuts: list, eps: float = 1e-4) -> Tensor:
    """Owning rank of each vertex: plane p -> rank r with cuts[r] < p <=
    cuts[r+1] (plane cuts[0] -> rank 0); cell c -> rank r with cuts[r] <= c
    < cuts[r+1] (the engine's tnp_engine_set_owned rule)."""
    off, on = x_grid(vertices, marks, eps)
    c = torch.tensor(cuts, dtype=torch.int64, device=vertices.device)
    # planes: count of cuts strictly below p, minus one; cells: cuts <= c, minus one
    r_plane = torch.searchsorted(c, off, right=False) - 1
    r_cell = torch.searchsorted(c, off, right=True) - 1
    r = torch.where(on, r_plane, r_cell)
    return r.clamp(0, len(cuts) - 2)


def slab_restrict(vertices: Tensor, edges: Tensor, marks: Tensor, x0: int, x1: int,
                  eps: float = 1e-4):
    """The sub-complex of a complex whose vertices lie on mark planes (a
    skeleton) between x planes x0 and x1: vertices kept in order (ids
    renumbered order-preserving, as slab_lattice numbers the lattice),
    edges with both endpoints kept, in order (duplicates included)."""
    off, on = x_grid(vertices, marks.to(vertices.device), eps)
    if not bool(on.all()):
        raise ValueError("slab_restrict: vertices off the x mark planes")
    keep = (off >= x0) & (off <= x1)
    nid = torch.cumsum(keep.to(torch.int64), 0) - 1
    e = edges.to(vertices.device)
    ke = keep[e[:, 0]] & keep[e[:, 1]]
    return vertices[keep], nid[e[ke]]


def comm_device(group, device) -> torch.device:
    """Where a collective's tensors must live: the GPU for RCCL ("nccl"),
    host memory for gloo (multi-rank rehearsals sharing one GPU)."""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else torch.device(device)


def _all_gather_padded(t: Tensor, group=None) -> list:
    """all_gather of a per-rank [n, C] tensor with varying n (count gather +
    one padded payload gather)."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    pad = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return [o[:c] for o, c in zip(out, counts)]


def _mix(h: Tensor) -> Tensor:
    h = h ^ (h >> 31)
    h = h * -7046029254386353131  # 0x9E3779B97F4A7C15 as int64 (wrapping)
    return h ^ (h >> 29)


def complex_hash(vertices: Tensor, edges: Tensor, vmask: Tensor = None, emask: Tensor = None):
    """Order-independent 64-bit fingerprints (vertex set, edge set) of a
    complex: vertices by coordinate bits, edges as unordered coordinate
    pairs -- numbering-free, so a stitched N-rank complex and the 1-rank one
    can be compared by summing the ranks' partial fingerprints."""
    b = vertices.contiguous().view(torch.int32).to(torch.int64)
    hv = _mix(b[:, 0] * 1000003 + b[:, 1] * 998244353 + b[:, 2])
    e = edges.to(vertices.device)
    ha, hb = hv[e[:, 0]], hv[e[:, 1]]
    he = _mix(torch.minimum(ha, hb) * 1000000007 + torch.maximum(ha, hb))
    if vmask is not None:
        hv = hv[vmask]
    if emask is not None:
        he = he[emask]
    return int(hv.sum().item()), int(he.sum().item())


def cut_fingerprint(vertices: Tensor, edges: Tensor, marks: Tensor, cut: int, eps: float = 1e-4):
    """(#vertices, #edges, vertex-set hash, edge-set hash) of the complex
    strictly between mark planes cut-1 and cut+1: cells cut-1 and cut and
    the cut plane, edges with both endpoints there."""
    off, on = x_grid(vertices, marks.to(vertices.device), eps)
    sel = torch.where(on, off == cut, (off == cut - 1) | (off == cut))
    e = edges.to(vertices.device)
    emask = sel[e[:, 0]] & sel[e[:, 1]]
    hv, he = complex_hash(vertices, e, sel, emask)
    return [int(sel.sum().item()), int(emask.sum().item()), hv, he]


def halo_check(vertices: Tensor, edges: Tensor, marks: Tensor, cuts: list, eps: float = 1e-4,
               group=None, raise_: bool = True):
    """Compare, across every cut, the two neighbours' complexes next to the
    cut (cut_fingerprint); raise RuntimeError on any difference (raise_=False:
    return None instead, on every rank).  Returns the per-cut fingerprints
    (rank 0's view) for logging."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mine = torch.zeros(2, 4, dtype=torch.int64, device=comm_device(group, vertices.device))
    if rank > 0:
        mine[0] = torch.tensor(cut_fingerprint(vertices, edges, marks, cuts[rank], eps))
    if rank < world - 1:
        mine[1] = torch.tensor(cut_fingerprint(vertices, edges, marks, cuts[rank + 1], eps))
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    bad = []
    for r in range(world - 1):
        lo, hi = allv[r][1].tolist(), allv[r + 1][0].tolist()
        if lo != hi:
            bad.append(f"cut {cuts[r + 1]}: rank {r} sees {lo[:2]} (hash {lo[2]:x}/{lo[3]:x}), "
                       f"rank {r + 1} sees {hi[:2]} (hash {hi[2]:x}/{hi[3]:x})")
    if bad:
        if not raise_:
            return None
        raise RuntimeError("halo_check: the shards disagree next to a cut (halo too narrow): "
                           + "; ".join(bad))
    return [allv[r][1].tolist() for r in range(world - 1)]


def stitch(vertices: Tensor, edges: Tensor, marks: Tensor, cuts: list, eps: float = 1e-4,
           group=None, masks: bool = False):
    """Stitch this rank's (halo) slab complex into the global one.

    vertices [V, 3] fp32, edges [E, 2] int64 (local ids), marks [M] fp32
    (net.enc.marks), cuts from slab_cuts.  Returns (owned_vertices [V', 3],
    first_global_id, global_edges [E', 2] int64): the owned vertices carry
    global ids first_global_id + arange(V'); global_edges are this rank's
    share of the global edge list.  masks=True appends the (owned vertex,
    kept edge) masks over the local arrays."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = vertices.device
    marks = marks.to(dev)
    nv = vertices.shape[0]
    owner = owner_of(vertices, marks, cuts, eps)
    own = owner == rank
    n_own = int(own.sum().item())
    cnt = torch.tensor([n_own], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    first = sum(int(c.item()) for c in counts[:rank])
    gid = torch.full((nv,), -1, dtype=torch.int64, device=dev)
    gid[own] = first + torch.arange(n_own, dtype=torch.int64, device=dev)

    # owned records on the upper cut plane, for the upper neighbour
    bits = vertices.contiguous().view(torch.int32).to(torch.int64)
    if rank < world - 1:
        off, on = x_grid(vertices, marks, eps)
        up = own & on & (off == cuts[rank + 1])
    else:
        up = torch.zeros(nv, dtype=torch.bool, device=dev)
    recs = _all_gather_padded(torch.cat([bits[up], gid[up, None]], dim=1), group)

    e_all = edges.to(dev)
    keep = torch.maximum(owner[e_all[:, 0]], owner[e_all[:, 1]]) == rank
    e = e_all[keep]
    used = torch.zeros(nv, dtype=torch.bool, device=dev)
    used[e.reshape(-1)] = True
    need = used & ~own
    if bool(need.any()):
        if rank == 0 or bool((owner[need] != rank - 1).any()):
            raise RuntimeError("stitch: a kept edge references a vertex beyond the lower cut plane")
        prev = recs[rank - 1]
        ni = torch.nonzero(need).squeeze(1)
        keys = torch.cat([prev[:, :3], bits[ni]], dim=0)
        uniq, inv = torch.unique(keys, dim=0, return_inverse=True)
        table = torch.full((uniq.shape[0],), -1, dtype=torch.int64, device=dev)
        table[inv[: prev.shape[0]]] = prev[:, 3]
        got = table[inv[prev.shape[0]:]]
        if bool((got < 0).any()):
            raise RuntimeError(f"stitch: {int((got < 0).sum())} vertices on cut plane "
                               f"{cuts[rank]} have no counterpart on rank {rank - 1}")
        gid[ni] = got
    if masks:
        return vertices[own], first, gid[e], own, keep
    return vertices[own], first, gid[e]


def gather_complex(owned: Tensor, first: int, gedges: Tensor, dst: int = 0, group=None):
    """Collect the stitched complex on rank `dst` (vertices in global id
    order, edges in rank order); other ranks get (None, None)."""
    rank = dist.get_rank(group)
    vs = _all_gather_padded(owned, group)
    es = _all_gather_padded(gedges, group)
    if rank != dst:
        return None, None
    return torch.cat(vs, dim=0), torch.cat(es, dim=0)


def subpoly_sharded(net, size: float = 1.2, group=None, allreduce=None, stats: list = None,
                    halo: int = None, force: bool = True, eps: float = 1e-4):
    """The hot loop of subpoly() (subpoly.py:45-69) sharded over the ranks of
    `group` (one GPU each): the skeleton (tropical.py:158-225, computed whole
    on every rank -- a few lattice passes), x-slabs of equal skeleton-edge
    load, each rank's slab + halo through every hyperplane step with the
    reference's global decisions made by `allreduce(vec, op)`, then
    halo_check and stitch; while halo_check sees a difference, the slabs are
    redone with the next width of HALOS (halo=None), or it raises (a fixed
    halo).  Returns (engine, owned vertices, first global id, global edges,
    cuts): the engine still holds this rank's slab complex.  force=False:
    the curve branch, its in-step decisions through the same allreduce.
    eps: subpoly's eps argument (None: Net.eps), as in subpoly()."""
    from ._engine import engine_for
    from .subpoly import _eps
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    eng = engine_for(net)
    eng.set_shards(world)
    eng.set_curve(not force)
    eng.set_eps(_eps(net, eps))
    V0, E0 = eng.skeleton(unit=128, size=size)
    v, e, _ = eng.export()
    marks = net.enc.marks.to(v.device)
    off, on = x_grid(v, marks, net.eps)
    if not bool(on.all()):
        raise NotImplementedError("subpoly_sharded: the skeleton fell back to get_hypercube "
                                  "(subpoly.py:51-52); nothing to shard")
    n_cells = marks.shape[0] - 1
    # an edge's x cell: the lower of its endpoints' x planes (x-edges span one
    # cell; y/z edges lie in a plane, charged to the cell on its right)
    ex = torch.minimum(off[e[:, 0]], off[e[:, 1]]).clamp(0, n_cells - 1)
    load = torch.bincount(ex, minlength=n_cells)
    cuts = balanced_cuts(load, world)
    widths = HALOS if halo is None else (halo,)
    for k, h in enumerate(widths):
        x0, x1 = slab_marks(cuts, rank, h)
        vs, es = slab_restrict(v, e, marks, x0, x1, net.eps)
        eng.load(vs, es)
        eng.set_xspan(x0, x1)
        eng.set_owned(cuts[rank], cuts[rank + 1])
        st = []
        eng.run_steps(st, allreduce)
        Vl, El, _ = eng.export()
        cd = comm_device(group, Vl.device)
        Vl, El = Vl.to(cd), El.to(cd)
        if halo_check(Vl, El, marks, cuts, net.eps, group, raise_=k == len(widths) - 1) is not None:
            break
    if stats is not None:
        stats.extend(st)
    owned, first, gE = stitch(Vl, El, marks, cuts, net.eps, group)
    return eng, owned, first, gE, cuts
