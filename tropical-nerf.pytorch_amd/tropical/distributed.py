"""Multi-GPU sharding of the extraction: x-slabs or blocks.

One process per GPU.  The cells between mark planes cuts[r] and cuts[r+1]
of the x axis belong to rank r, which also owns the mark planes
(cuts[r], cuts[r+1]] (rank 0 also plane 0).  Blocks (class Blocks) apply
the same rule along every cut axis: a px x py x pz split of the lattice,
whose cut faces -- and so halos -- are smallest (bench.py's N > 1 path:
2 x 2 x 2 blocks of the 256^3 lattice at N = 8, 6.7 % redundant cells per
rank at a 3-cell halo, against 15.8 % for 8 x-slabs).  Each rank extracts
the lattice of its cells plus a HALO of HALO cell columns on either side (slab_marks),
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
* edge owner = the owner of the cell the edge lies in (edge_owner); a rank
  keeps its edges;
* owned vertices get global ids by an exclusive scan of the owned counts;
* a rank's kept edges can reference other ranks' vertices only on its lower
  faces: the owners' records on their upper faces (coordinate bits + global
  id) are matched bitwise on the device.

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

Stanford nets (BASELINE config 4): the reference's skeleton on its
128-mark tiles (tropical.py:176-181, per-tile max_grad) is split over the
ranks -- each evaluates every world-th tile whole for its max |grad sdf| and
per-plane load, the ranks agree on both, cut the grid at equal load
(balanced_cuts) and each builds only the part of the skeleton inside its
block plus halo (tnp_engine_skeleton_box) -- subpoly_sharded().
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


HALO = 3  # first halo tried: cell columns extracted beyond each cut plane
# the widths tried in turn while halo_check still sees a difference (the
# error front of a slab's outer boundary moves inward by at most one cell per
# active step, and only through eps coincidences: how far it gets depends on
# the net and the lattice, so the width is found, then checked again).  The
# search starts at 3, the widest any measured workload needed (161^3: 2;
# 203^3, 256^3: 3 -- a 2-cell halo left 1-2 vertices different at 203^3), so
# none of them pays a rejected extraction; at 161^3 / 2 slabs the extra
# column costs 1.2 % more redundant cells, at 256^3 / 8 blocks 3 is the
# minimum anyway (6.7 % redundant)
HALOS = (3, 4, 6, 8, 12, 16, 24, 33)


def slab_marks(cuts: list, rank: int, halo: int = HALO):
    """Marks [x0, x1] a rank extracts: its cells plus `halo` cells each side."""
    return max(cuts[rank] - halo, cuts[0]), min(cuts[rank + 1] + halo, cuts[-1])


def block_dims(world: int) -> tuple:
    """(px, py, pz), px * py * pz == world: the most cubic split of the ranks
    into blocks (px >= py >= pz; 8 -> 2 x 2 x 2, 4 -> 2 x 2 x 1, 2 -> 2 x 1 x 1)."""
    best = None
    for px in range(1, world + 1):
        if world % px:
            continue
        for py in range(1, px + 1):
            if (world // px) % py:
                continue
            pz = world // px // py
            if pz > py:
                continue
            key = (px - pz, -px)
            if best is None or key < best[0]:
                best = (key, (px, py, pz))
    return best[1]


class Blocks:
    """A split of the mark grid into px x py x pz blocks, one per rank.

    Along axis d block i OWNS the cells cuts[d][i] <= c < cuts[d][i+1] and
    the mark planes cuts[d][i] < p <= cuts[d][i+1] (block 0 also plane 0) --
    x-slabs are the (world, 1, 1) case (``Blocks.xslabs``).  rank =
    (ix * py + iy) * pz + iz.  Why blocks: a shard extracts its block plus a
    halo of cells beyond every cut face, and a block of a 256^3 lattice on 8
    ranks has three such faces of 128^2 cells where an x-slab has two of
    256^2 -- 6 % redundant cells at a 3-cell halo instead of 16 %."""

    def __init__(self, n_marks: int, dims, cuts=None):
        self.n_marks = int(n_marks)
        self.dims = tuple(int(p) for p in dims)
        self.cuts = [list(c) for c in cuts] if cuts is not None else [slab_cuts(n_marks, p) for p in self.dims]
        self.world = self.dims[0] * self.dims[1] * self.dims[2]
        for d in range(3):
            c = self.cuts[d]
            if len(c) != self.dims[d] + 1 or any(b <= a for a, b in zip(c, c[1:])):
                raise ValueError(f"Blocks: axis {'xyz'[d]} cuts {c} do not give {self.dims[d]} non-empty "
                                 f"blocks of the {self.n_marks - 1} cells")

    @classmethod
    def xslabs(cls, cuts: list):
        n = cuts[-1] + 1
        return cls(n, (len(cuts) - 1, 1, 1), [list(cuts), [0, n - 1], [0, n - 1]])

    def index(self, rank: int) -> tuple:
        _, py, pz = self.dims
        return rank // (py * pz), (rank // pz) % py, rank % pz

    def rank_of(self, idx) -> int:
        _, py, pz = self.dims
        return (idx[0] * py + idx[1]) * pz + idx[2]

    def owned(self, rank: int):
        """(lo, hi) of tnp_engine_set_owned_box: per axis the owned planes
        (lo, hi]; lo > hi on an axis that is not cut."""
        idx = self.index(rank)
        lo, hi = [1, 1, 1], [0, 0, 0]
        for d in range(3):
            if self.dims[d] > 1:
                lo[d], hi[d] = self.cuts[d][idx[d]], self.cuts[d][idx[d] + 1]
        return lo, hi

    def box(self, rank: int, halo: int):
        """Mark indices [lo[d], hi[d]] the rank extracts: its block plus
        `halo` cells beyond every cut face."""
        idx = self.index(rank)
        lo, hi = [0, 0, 0], [0, 0, 0]
        for d in range(3):
            c = self.cuts[d]
            lo[d] = max(c[idx[d]] - halo, c[0])
            hi[d] = min(c[idx[d] + 1] + halo, c[-1])
        return lo, hi

    def redundant_frac(self, rank: int, halo: int) -> float:
        """Share of the rank's extracted cells that another rank owns."""
        lo, hi = self.box(rank, halo)
        idx = self.index(rank)
        mine = tot = 1
        for d in range(3):
            mine *= self.cuts[d][idx[d] + 1] - self.cuts[d][idx[d]]
            tot *= hi[d] - lo[d]
        return 1.0 - mine / tot


def as_blocks(part) -> Blocks:
    """x-slab cuts (a list) or a Blocks split."""
    return part if isinstance(part, Blocks) else Blocks.xslabs(part)


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


def axis_grid(vertices: Tensor, marks: Tensor, eps: float = 1e-4, d: int = 0):
    """(offset, on_mark) of coordinate d in the grid-region sense of
    TropicalHashGrid.region (tropical.py:227-236) on x01 = (x + 1) / 2
    (Net.preprocess, model.py:78-79) -- the engine's grid word, bit for bit."""
    x01 = (vertices[:, d] + 1.0) / 2.0
    off = torch.searchsorted(marks, x01 + eps) - 1
    mk = marks[torch.where(off < 0, off + marks.shape[0], off)]
    return off, ~((mk - x01).abs() > eps)


def x_grid(vertices: Tensor, marks: Tensor, eps: float = 1e-4):
    return axis_grid(vertices, marks, eps, 0)


def _axis_index(off: Tensor, on: Tensor, cuts: list, plane: bool = True) -> Tensor:
    """Block index along one axis: plane p -> i with cuts[i] < p <= cuts[i+1]
    (plane cuts[0] -> 0), cell c -> i with cuts[i] <= c < cuts[i+1]."""
    c = torch.tensor(cuts, dtype=torch.int64, device=off.device)
    r_cell = torch.searchsorted(c, off, right=True) - 1
    if plane:
        r = torch.where(on, torch.searchsorted(c, off, right=False) - 1, r_cell)
    else:
        r = r_cell
    return r.clamp(0, len(cuts) - 2)


def owner_of(vertices: Tensor, marks: Tensor, cuts, eps: float = 1e-4) -> Tensor:
    """Owning rank of each vertex: along every cut axis, plane p -> block i
    with cuts[i] < p <= cuts[i+1] (plane cuts[0] -> block 0), cell c -> block
    i with cuts[i] <= c < cuts[i+1] (the engine's tnp_engine_set_owned_box
    rule).  cuts: x-slab cuts (a list) or Blocks."""
    B = as_blocks(cuts)
    idx = []
    for d in range(3):
        if B.dims[d] == 1:
            idx.append(torch.zeros(vertices.shape[0], dtype=torch.int64, device=vertices.device))
            continue
        off, on = axis_grid(vertices, marks, eps, d)
        idx.append(_axis_index(off, on, B.cuts[d]))
    return B.rank_of(idx)


def edge_owner(vertices: Tensor, edges: Tensor, marks: Tensor, cuts, eps: float = 1e-4) -> Tensor:
    """Owning rank of each edge: the owner of the cell it lies in, taken as
    the highest cell whose closure holds both endpoints (per axis the lower
    of the endpoints' offsets) -- a cell of the owner's block, so the edge is
    one of its own cells' and both endpoints lie in that block or on its
    lower faces."""
    B = as_blocks(cuts)
    e = edges.to(vertices.device)
    idx = []
    for d in range(3):
        if B.dims[d] == 1:
            idx.append(torch.zeros(e.shape[0], dtype=torch.int64, device=vertices.device))
            continue
        off, _ = axis_grid(vertices, marks, eps, d)
        cell = torch.minimum(off[e[:, 0]], off[e[:, 1]])
        idx.append(_axis_index(cell, None, B.cuts[d], plane=False))
    return B.rank_of(idx)


def owned_masks(vertices: Tensor, edges: Tensor, marks: Tensor, cuts, rank: int, eps: float = 1e-4):
    """(owned vertex mask, kept edge mask) of `rank` over its local arrays:
    the share stitch() contributes to the global complex."""
    marks = marks.to(vertices.device)
    return (owner_of(vertices, marks, cuts, eps) == rank,
            edge_owner(vertices, edges, marks, cuts, eps) == rank)


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


def box_restrict(vertices: Tensor, edges: Tensor, marks: Tensor, lo, hi, eps: float = 1e-4):
    """slab_restrict for a box of mark planes [lo[d], hi[d]] per axis (a
    block with its halo): vertices of a mark-plane complex kept in order,
    edges with both endpoints kept, in order."""
    marks = marks.to(vertices.device)
    keep = torch.ones(vertices.shape[0], dtype=torch.bool, device=vertices.device)
    for d in range(3):
        off, on = axis_grid(vertices, marks, eps, d)
        if not bool(on.all()):
            raise ValueError("box_restrict: vertices off the mark planes")
        keep &= (off >= lo[d]) & (off <= hi[d])
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


def cut_fingerprint(vertices: Tensor, edges: Tensor, marks: Tensor, cut: int, eps: float = 1e-4,
                    axis: int = 0, across=None):
    """(#vertices, #edges, vertex-set hash, edge-set hash) of the complex
    strictly between mark planes cut-1 and cut+1 of `axis`: cells cut-1 and
    cut and the cut plane, edges with both endpoints there.  across: {axis b:
    (lo, hi)} further restricts the region along the other cut axes of a
    block split to the two blocks' common range plus one cell beyond each
    of its faces (cells lo-1 .. hi, planes lo .. hi)."""
    marks = marks.to(vertices.device)
    off, on = axis_grid(vertices, marks, eps, axis)
    sel = torch.where(on, off == cut, (off == cut - 1) | (off == cut))
    for b, (lo, hi) in (across or {}).items():
        ob, nb = axis_grid(vertices, marks, eps, b)
        sel &= torch.where(nb, (ob >= lo) & (ob <= hi), (ob >= lo - 1) & (ob <= hi))
    e = edges.to(vertices.device)
    emask = sel[e[:, 0]] & sel[e[:, 1]]
    hv, he = complex_hash(vertices, e, sel, emask)
    return [int(sel.sum().item()), int(emask.sum().item()), hv, he]


def halo_check(vertices: Tensor, edges: Tensor, marks: Tensor, cuts, eps: float = 1e-4,
               group=None, raise_: bool = True):
    """Compare, across every cut face, the two neighbouring blocks'
    complexes next to the face (cut_fingerprint over the face's range);
    raise RuntimeError on any difference (raise_=False: return None instead,
    on every rank).  Returns the per-face fingerprints (rank 0's view) for
    logging.  cuts: x-slab cuts (a list) or Blocks.

    A block's own errors start at its outer halo boundary; to reach a cell it
    owns they must cross one of its faces, where the neighbour across that
    face -- for which those cells are interior along that axis -- computed
    them from a different boundary (an error from a corner of the halo
    differs from at least one of the two or three neighbours whose faces
    meet there)."""
    B = as_blocks(cuts)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if world != B.world:
        raise ValueError(f"halo_check: {world} ranks for a split into {B.world} blocks")
    idx = B.index(rank)
    mine = torch.zeros(3, 2, 4, dtype=torch.int64, device=comm_device(group, vertices.device))

    def across(i):
        return {b: (B.cuts[b][i[b]], B.cuts[b][i[b] + 1]) for b in range(3) if B.dims[b] > 1 and b != a}

    for a in range(3):
        if B.dims[a] == 1:
            continue
        if idx[a] > 0:
            mine[a, 0] = torch.tensor(cut_fingerprint(vertices, edges, marks, B.cuts[a][idx[a]], eps, a, across(idx)))
        if idx[a] < B.dims[a] - 1:
            mine[a, 1] = torch.tensor(cut_fingerprint(vertices, edges, marks, B.cuts[a][idx[a] + 1], eps, a,
                                                      across(idx)))
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    bad, seen = [], []
    for r in range(world):
        ir = B.index(r)
        for a in range(3):
            if B.dims[a] == 1 or ir[a] == B.dims[a] - 1:
                continue
            up = list(ir)
            up[a] += 1
            q = B.rank_of(up)
            lo, hi = allv[r][a, 1].tolist(), allv[q][a, 0].tolist()
            seen.append(lo)
            if lo != hi:
                bad.append(f"cut {B.cuts[a][ir[a] + 1]} of axis {'xyz'[a]}: rank {r} sees {lo[:2]} "
                           f"(hash {lo[2]:x}/{lo[3]:x}), rank {q} sees {hi[:2]} (hash {hi[2]:x}/{hi[3]:x})")
    if bad:
        if not raise_:
            return None
        raise RuntimeError("halo_check: the shards disagree next to a cut (halo too narrow): "
                           + "; ".join(bad))
    return seen


def stitch(vertices: Tensor, edges: Tensor, marks: Tensor, cuts, eps: float = 1e-4,
           group=None, masks: bool = False):
    """Stitch this rank's (halo) slab or block complex into the global one.

    vertices [V, 3] fp32, edges [E, 2] int64 (local ids), marks [M] fp32
    (net.enc.marks), cuts: x-slab cuts from slab_cuts, or Blocks.  Returns
    (owned_vertices [V', 3], first_global_id, global_edges [E', 2] int64):
    the owned vertices carry global ids first_global_id + arange(V');
    global_edges are this rank's share of the global edge list (edge_owner:
    the edges of its own cells).  masks=True appends the (owned vertex, kept
    edge) masks over the local arrays.

    A kept edge lies in one of the rank's cells, so an endpoint it does not
    own lies on one of its LOWER faces, owned by the block below along that
    axis (or diagonally below): every rank publishes its owned vertices on
    its upper faces (coordinate bits + global id) and looks the others up
    there, bitwise, on the device."""
    B = as_blocks(cuts)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = vertices.device
    marks = marks.to(dev)
    nv = vertices.shape[0]
    owner = owner_of(vertices, marks, B, eps)
    own = owner == rank
    n_own = int(own.sum().item())
    cnt = torch.tensor([n_own], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    first = sum(int(c.item()) for c in counts[:rank])
    gid = torch.full((nv,), -1, dtype=torch.int64, device=dev)
    gid[own] = first + torch.arange(n_own, dtype=torch.int64, device=dev)

    # owned records on an upper cut face, for the blocks above
    bits = vertices.contiguous().view(torch.int32).to(torch.int64)
    idx = B.index(rank)
    up = torch.zeros(nv, dtype=torch.bool, device=dev)
    for d in range(3):
        if idx[d] < B.dims[d] - 1:
            off, on = axis_grid(vertices, marks, eps, d)
            up |= on & (off == B.cuts[d][idx[d] + 1])
    up &= own
    recs = _all_gather_padded(torch.cat([bits[up], gid[up, None]], dim=1), group)

    e_all = edges.to(dev)
    keep = edge_owner(vertices, e_all, marks, B, eps) == rank
    e = e_all[keep]
    used = torch.zeros(nv, dtype=torch.bool, device=dev)
    used[e.reshape(-1)] = True
    need = used & ~own
    if bool(need.any()):
        ni = torch.nonzero(need).squeeze(1)
        below = [r for r in range(world) if r != rank and all(a <= b for a, b in zip(B.index(r), idx))]
        if not below:
            raise RuntimeError("stitch: a kept edge references a vertex beyond the block's lower faces")
        prev = torch.cat([recs[r] for r in below], dim=0)
        src = torch.cat([torch.full((recs[r].shape[0],), r, dtype=torch.int64, device=dev) for r in below])
        keys = torch.cat([prev[:, :3], bits[ni]], dim=0)
        uniq, inv = torch.unique(keys, dim=0, return_inverse=True)
        table = torch.full((uniq.shape[0],), -1, dtype=torch.int64, device=dev)
        table[inv[: prev.shape[0]]] = prev[:, 3]
        tsrc = torch.full((uniq.shape[0],), -1, dtype=torch.int64, device=dev)
        tsrc[inv[: prev.shape[0]]] = src
        q = inv[prev.shape[0]:]
        got = table[q]
        if bool((got < 0).any()):
            raise RuntimeError(f"stitch: {int((got < 0).sum())} vertices on the lower faces of rank "
                               f"{rank} have no counterpart on the ranks below")
        # each needed vertex must come from the rank owner_of names: a record
        # is published only by its owner, so another source means the ranks
        # disagree on ownership (a bitwise match against the wrong block)
        wrong = tsrc[q] != owner[ni]
        if bool(wrong.any()):
            raise RuntimeError(f"stitch: {int(wrong.sum())} vertices on the lower faces of rank {rank} "
                               f"matched a record of a rank other than their owner")
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
                    halo: int = None, force: bool = True, eps: float = 1e-4, blocks: bool = False,
                    info: dict = None, box_skeleton: bool = True):
    """The hot loop of subpoly() (subpoly.py:45-69) sharded over the ranks of
    `group` (one GPU each): the skeleton (tropical.py:158-225), x-slabs of
    equal skeleton load, each rank's slab + halo through every hyperplane
    step with the reference's global decisions made by `allreduce(vec, op)`,
    then halo_check and stitch; while halo_check sees a difference, the slabs
    are redone with the next width of HALOS (halo=None), or it raises (a fixed
    halo).  Returns (engine, owned vertices, first global id, global edges,
    cuts): the engine still holds this rank's slab complex.  force=False:
    the curve branch, its in-step decisions through the same allreduce.
    eps: subpoly's eps argument (None: Net.eps), as in subpoly().
    blocks=True: the most cubic block split instead of x-slabs, each axis
    cut at equal marginal load; `cuts` is then the Blocks.
    box_skeleton (default): the skeleton is split over the ranks too -- each
    rank evaluates every world-th reference tile whole (its max |grad sdf|
    and its per-plane load), the ranks agree on the tiles' maxima (MAX) and
    the loads (SUM), cut the grid at equal load, and each rank then builds
    only the part of the skeleton inside its box (tnp_engine_skeleton_box:
    tile & box, the whole skeleton restricted, order kept).  False: every
    rank computes the whole skeleton and restricts it (box_restrict), cuts at
    equal skeleton-edge load.
    info (a dict): filled with the accepted halo, the extractions the halo
    search ran (halo_attempts: 1 unless a width was rejected) and their
    wall time (halo_ms)."""
    import time
    from ._engine import engine_for
    from .subpoly import _eps
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    eng = engine_for(net)
    eng.set_shards(world)
    eng.set_curve(not force)
    eng.set_eps(_eps(net, eps))
    marks = net.enc.marks
    n_cells = marks.shape[0] - 1

    def reduce(vec: np.ndarray, op: str) -> np.ndarray:
        if allreduce is not None:
            return np.asarray(allreduce(vec, op))
        t = torch.from_numpy(np.ascontiguousarray(vec)).to(comm_device(group, marks.device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=group)
        return t.cpu().numpy()

    if box_skeleton:
        gmax, load = eng.skeleton_gmax(128, rank, world)
        gmax = reduce(gmax.astype(np.int64), "max").astype(np.uint32)
        load = reduce(load.reshape(-1), "sum").reshape(3, -1)

        def axis_cuts(d, parts):
            # plane m's load charged to cell m (the cell on its right)
            return balanced_cuts(torch.from_numpy(load[d][:n_cells].copy()), parts)
    else:
        V0, E0 = eng.skeleton(unit=128, size=size)
        v, e, _ = eng.export()
        mk = marks.to(v.device)
        off, on = x_grid(v, mk, net.eps)
        if not bool(on.all()):
            raise NotImplementedError("subpoly_sharded: the skeleton fell back to get_hypercube "
                                      "(subpoly.py:51-52); nothing to shard")

        def axis_cuts(d, parts):
            # an edge's cell along d: the lower of its endpoints' planes (edges
            # along d span one cell; the others lie in a plane, charged to the
            # cell on its right)
            o, _ = axis_grid(v, mk, net.eps, d)
            ed = torch.minimum(o[e[:, 0]], o[e[:, 1]]).clamp(0, n_cells - 1)
            return balanced_cuts(torch.bincount(ed, minlength=n_cells), parts)

    if blocks:
        dims = block_dims(world)
        part = Blocks(n_cells + 1, dims, [axis_cuts(d, dims[d]) if dims[d] > 1 else [0, n_cells]
                                          for d in range(3)])
    else:
        part = Blocks.xslabs(axis_cuts(0, world))
    cuts = part.cuts[0] if not blocks else part
    widths = HALOS if halo is None else (halo,)
    t0 = time.perf_counter()
    for k, h in enumerate(widths):
        lo, hi = part.box(rank, h)
        if box_skeleton:
            Vb, Eb = eng.skeleton_box(lo, hi, gmax)
            if k == 0 and int(reduce(np.array([Eb], dtype=np.int64), "sum")[0]) == 0:
                # the boxes cover the grid: no edge in any is no skeleton at all
                raise NotImplementedError("subpoly_sharded: the skeleton fell back to get_hypercube "
                                          "(subpoly.py:51-52); nothing to shard")
        else:
            vs, es = box_restrict(v, e, mk, lo, hi, net.eps)
            eng.load(vs, es)
        eng.set_span(lo, hi)
        eng.set_owned_box(*part.owned(rank))
        st = []
        eng.run_steps(st, allreduce)
        Vl, El, _ = eng.export()
        cd = comm_device(group, Vl.device)
        Vl, El = Vl.to(cd), El.to(cd)
        if halo_check(Vl, El, marks, cuts, net.eps, group, raise_=k == len(widths) - 1) is not None:
            break
    if info is not None:
        info.update(halo=h, halo_attempts=k + 1, halo_ms=(time.perf_counter() - t0) * 1e3)
    if stats is not None:
        stats.extend(st)
    owned, first, gE = stitch(Vl, El, marks, cuts, net.eps, group)
    return eng, owned, first, gE, cuts
