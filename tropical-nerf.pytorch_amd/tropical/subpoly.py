"""Drop-in for the reference's ``tropical.subpoly`` (tropical/subpoly.py).

``subpoly(net, d, size, eps, force)`` keeps the reference's signature, stdout
line and return types; the whole extraction -- skeleton, every hyperplane
step, surface and faces -- runs in the device-resident HIP engine
(csrc/*.hip through include/tropical_hip.h).  Empty steps are skipped
without a launch: the engine knows from the packed eps-sign keys which
future planes split an edge (subpoly.py:104-110 has no side effects when
nothing splits).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch
from torch import Tensor

from ._engine import engine_for


def _eps(net, eps):
    """subpoly's eps argument (None: Net.eps).  The reference mixes both:
    the steps' sign test, split point, hits and failover, extract_skeleton
    and extract_faces take the argument, Net.region (the pair tests and the
    pruning) net.eps (subpoly.py:24, 90-279, 556-606); the engine does the
    same (tnp_engine_set_eps)."""
    return float(net.eps) if eps is None else float(eps)


def _faces_to_numpy(tri: Tensor, faces: Tensor):
    if tri.shape[0] == 0:
        return [], []
    return faces.numpy(), tri.numpy()  # (host tensors: faces(host=True))


@torch.no_grad()
def subpoly(net, d: int, size: float, eps: float = 1e-4, force: bool = False,
            stats: list = None) -> List:
    """Skeleton -> all hyperplane steps -> surface -> faces (subpoly.py:23-86).

    Returns ``(faces float np F x 3 x 3, vertices V x 3 on net.device(),
    faces_with_indices int64 np F x 3)``; ``stats`` (optional list) receives
    one counter dict per active step."""
    if d != 3:
        raise NotImplementedError("d must be 3 (the reference's hash grid is 3-D)")
    eng = engine_for(net).set_curve(not force).set_eps(_eps(net, eps))
    eng.skeleton(unit=128, size=size)
    eng.run_steps(stats)
    return _finish(eng, net)


def _finish(eng, net):
    nV, nE = eng.sizes()
    print()
    print(f"# of vertices and edges = {nV}/{nE} => ", end="")
    sV, sE = eng.surface()
    print(f"{sV}/{sE}", end=", ")
    if sV == 0:
        print("0 faces", end=", ")
        return [], torch.zeros(0, dtype=torch.int64, device=eng.device), []
    verts, _, _ = eng.export(edges=False)  # (the faces need no edge list)
    tri, fc = eng.faces(host=True)
    faces, fwi = _faces_to_numpy(tri, fc)
    print(f"{len(faces)} faces", end=", ")
    return faces, verts, fwi


@torch.no_grad()
def subpoly_lattice(net, x0: int = 0, x1: int = -1, stats: list = None, faces: bool = True):
    """The hot loop on the full lattice of the marks (no skeleton pruning):
    the north-star synthetic workload."""
    eng = engine_for(net)
    eng.lattice(x0, x1)
    eng.run_steps(stats)
    if not faces:
        return eng
    return _finish(eng, net)


def subpoly_(vertices, edges, net, l, h, eps, outputs_=None, pruning=True, strict=True,
             force=False):
    """One hyperplane step (subpoly.py:90-279); ``force=False`` is the curve
    branch, with the strict filter when ``strict`` (the reference's default;
    strict=False keeps every split, subpoly.py:198-203).

    Like the reference, a step that splits rewrites the caller's ``edges``
    in place: the second endpoint of every split edge becomes its new vertex
    (``masked_scatter_``, subpoly.py:209-212)."""
    eng = engine_for(net).set_curve(not force).set_strict(strict).set_eps(_eps(net, eps))
    eng.load(vertices, edges, outputs_, keep_all=True)
    idx = l * net.num_hidden + h
    S, fail = eng.split(idx)
    if S == 0:
        v, e, o = eng.export(pre=True)
        return v, e, o
    # the split mask of subpoly.py:102-105 over the caller's cached column
    col = outputs_[:, idx] if outputs_ is not None else None
    if col is None:
        col = torch.cat(net(vertices.to(net.device()), gather=True)[1], dim=-1)[:, idx]
    d = col.to(edges.device)[edges]
    m = (d[:, 0] * d[:, 1]) < 0
    m &= (d[:, 0].abs() > eps) & (d[:, 1].abs() > eps)
    eng.finish(idx, bool(h < net.num_hidden and pruning), fail)
    if not force:  # the strict filter's survivors (subpoly_debug.py:234-271)
        m[m.clone()] = eng.split_keep(S).to(edges.device)
    n_new = int(m.sum())
    edges[:, 1].masked_scatter_(m, torch.arange(n_new, device=edges.device).to(edges)
                                + vertices.shape[0])
    return eng.export(pre=True)


def extract_skeleton(vertices, edges, net, eps, outputs=None):
    """subpoly.py:556-581; returns (vertices, edges, v_idx)."""
    eps = _eps(net, eps)
    on = (outputs[:, -1].abs() < eps) if outputs is not None else (net.sdf(vertices)[:, 0].abs() < eps)
    v = net.preprocess(vertices)
    on[(v > 1).sum(dim=-1) > 0] = False
    on[(v < 0).sum(dim=-1) > 0] = False
    if 3 > on.sum():
        return torch.Tensor([]).to(edges), torch.Tensor([]).to(edges), None
    edges = edges[on[edges].sum(dim=-1) == 2]
    v_idx, r_idx = edges.view(-1).unique(return_inverse=True)
    return vertices[v_idx], r_idx.view(-1, 2), v_idx


def extract_faces(vertices, edges, net, outputs=None, eps=None):
    """subpoly.py:584-652 on the device engine (regions at ``eps``,
    subpoly.py:606)."""
    if vertices.shape[0] == 0:
        return [], []
    eng = engine_for(net).set_eps(_eps(net, eps))
    eng.load(vertices, edges, outputs, keep_all=True)
    tri, fc = eng.faces(host=True)
    return _faces_to_numpy(tri, fc)


def get_hypercube(d, size):
    """subpoly.py:731-750."""
    x = torch.Tensor([-size, size])
    vertices = torch.stack(torch.meshgrid(x, x, x, indexing="ij"), dim=-1).view(-1, 3)
    pairs = [[i, j] for i in range(8) for j in range(i + 1, 8)
             if int((vertices[i] * vertices[j] < 0).sum()) == 1]
    faces = [[0, 3, 5, 1], [0, 2, 8, 4], [3, 4, 10, 7],
             [1, 2, 9, 6], [8, 9, 11, 10], [7, 11, 6, 5]]
    return vertices, torch.LongTensor(pairs), faces
