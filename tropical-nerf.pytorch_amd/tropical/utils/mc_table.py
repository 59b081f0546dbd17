"""Marching-cubes case table, derived procedurally (no copied table).

The reference's `-e` evaluation meshes SDF samples with PyMCubes
(`mcubes.marching_cubes(-sdfs, 0)`, train.py:284), a third-party package
absent here; its Lorensen-Cline case table is not restated from memory but
re-derived from the cube geometry:

* corners 0..7 at (x, y, z) = (0,0,0) (1,0,0) (1,1,0) (0,1,0) (0,0,1)
  (1,0,1) (1,1,1) (0,1,1); a corner is INSIDE when its value < iso (bit i of
  the case index);
* edges 0..11 = (0,1) (1,2) (2,3) (3,0) (4,5) (5,6) (6,7) (7,4) (0,4) (1,5)
  (2,6) (3,7) -- the usual numbering;
* on every cube face (walked counter-clockwise seen from outside) each
  inside->outside crossing is joined to the preceding outside->inside
  crossing, which separates the inside corners of an ambiguous face (the
  classic table's choice on faces with diagonal inside corners);
* the face segments chain into closed loops over the cube; each loop is fan
  triangulated and oriented so the normal points from outside (value >=
  iso) to inside (value < iso), i.e. along -grad(value).  The reference
  meshes -sdf (train.py:284) of an inside-positive SDF (dataset.py:91), so
  these normals follow +grad(sdf), the orientation of the subpoly faces
  (whose normals come from grad(sdf), subpoly.py:584-728): the angular
  distance of "Ours" against the MC pseudo ground truth is then small, as
  in the reference's results.

Vertex count per cube = crossing edges, as in the table; ambiguous-face
topology follows the separated-corners rule, which may differ from
PyMCubes' table in the rare ambiguous configurations (parity of the MC
baseline rows is therefore not bitwise; the metric that uses them is
Chamfer / angular distance).
"""
from functools import lru_cache

import numpy as np

CORNERS = np.array([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0),
                    (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)], dtype=np.int64)
EDGES = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4),
         (0, 4), (1, 5), (2, 6), (3, 7)]
# faces as corner cycles, counter-clockwise seen from outside the cube
FACES = [(0, 3, 2, 1),   # z = 0 (outward -z)
         (4, 5, 6, 7),   # z = 1
         (0, 1, 5, 4),   # y = 0
         (2, 3, 7, 6),   # y = 1
         (0, 4, 7, 3),   # x = 0
         (1, 2, 6, 5)]   # x = 1
_EDGE_OF = {frozenset(e): i for i, e in enumerate(EDGES)}


def _case_loops(case: int):
    inside = [(case >> i) & 1 == 1 for i in range(8)]
    nxt = {}
    for f in FACES:
        cr = []  # (edge, kind) in CCW order; kind +1: in->out, -1: out->in
        for k in range(4):
            a, b = f[k], f[(k + 1) % 4]
            if inside[a] != inside[b]:
                cr.append((_EDGE_OF[frozenset((a, b))], 1 if inside[a] else -1))
        for k, (e, kind) in enumerate(cr):
            if kind == 1:  # join to the preceding out->in crossing
                j = (k - 1) % len(cr)
                while cr[j][1] != -1:
                    j = (j - 1) % len(cr)
                nxt[e] = cr[j][0]
    loops, seen = [], set()
    for s in sorted(nxt):
        if s in seen:
            continue
        loop, e = [], s
        while e not in seen:
            seen.add(e)
            loop.append(e)
            e = nxt[e]
        loops.append(loop)
    return loops, inside


def _mid(e):
    a, b = EDGES[e]
    return (CORNERS[a] + CORNERS[b]) / 2.0


def _loops_outward() -> bool:
    """Do the loops of the construction wind so that fan normals point away
    from the inside corners?  (One rule builds every loop, so one case --
    corner 0 alone inside -- decides for all.)  The table wants the
    opposite."""
    (loop,), _ = _case_loops(1)
    p = [_mid(e) for e in loop[:3]]
    n = np.cross(p[1] - p[0], p[2] - p[0])
    return float(np.dot(n, (p[0] + p[1] + p[2]) / 3.0 - CORNERS[0])) > 0


@lru_cache(maxsize=None)
def case_table() -> np.ndarray:
    """int8 [256, 16]: up to 5 triangles as cube-edge triples, -1 padded.
    Shared faces of neighbouring cubes pair their crossings identically, so
    the surface is closed and consistently oriented (normals towards value
    < iso)."""
    tab = np.full((256, 16), -1, dtype=np.int8)
    flip = _loops_outward()
    for case in range(256):
        loops, inside = _case_loops(case)
        tris = []
        for loop in loops:
            if flip:
                loop = loop[::-1]
            for i in range(1, len(loop) - 1):
                tris.append([loop[0], loop[i], loop[i + 1]])
        flat = [e for t in tris for e in t]
        assert len(flat) <= 15, (case, flat)
        tab[case, :len(flat)] = flat
    return tab


def edge_table() -> np.ndarray:
    """int32 [256]: bit e set when cube edge e is crossed."""
    out = np.zeros(256, dtype=np.int32)
    for case in range(256):
        for e, (a, b) in enumerate(EDGES):
            if ((case >> a) & 1) != ((case >> b) & 1):
                out[case] |= 1 << e
    return out
