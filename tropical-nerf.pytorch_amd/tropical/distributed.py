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
next plane), so each halo column divides the residual by the chance of a
coincidence (one column still left 3 vertices of 23.6M at 161^3; two:
see tools/multi_rehearsal.sh).  stitch() raises if a residual remains.

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
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import Tensor


def slab_cuts(n_marks: int, world: int) -> list:
    """Mark indices cutting the x axis into `world` slabs of cells."""
    return [round(r * (n_marks - 1) / world) for r in range(world + 1)]


HALO = 2  # cell columns extracted beyond each cut plane


def slab_marks(cuts: list, rank: int, halo: int = HALO):
    """Marks [x0, x1] a rank extracts: its cells plus `halo` cells each side."""
    return max(cuts[rank] - halo, cuts[0]), min(cuts[rank + 1] + halo, cuts[-1])


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
