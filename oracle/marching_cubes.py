"""TEST INFRASTRUCTURE ONLY (oracle): numpy marching cubes over the
procedural case table of tropical/utils/mc_table.py -- the checker for the
HIP kernels in csrc/evaluate.hip (tnp_mc_*), never called by the product.

Same conventions as the kernels: volume vol[i, j, k] (x, y, z index space),
inside = value < iso, one vertex per crossed lattice edge, numbered by
(point-major, axis-minor) lattice-edge order, position p + t * e_axis with
t = (iso - v0) / (v1 - v0) in fp64 (from the fp32 samples); triangles per cube in cube order (x
slowest), table order within a cube.  PyMCubes (the reference's
`mcubes.marching_cubes`, train.py:284) is absent here and unpinned."""
import numpy as np


def marching_cubes(vol: np.ndarray, iso: float, table: np.ndarray):
    vol = np.ascontiguousarray(vol, dtype=np.float32)
    n0, n1, n2 = vol.shape
    iso = np.float32(iso)
    inside = vol < iso
    # lattice edges: point (i,j,k) x axis a -> id 3*flat(p) + a
    flags = np.zeros((n0, n1, n2, 3), dtype=bool)
    flags[:-1, :, :, 0] = inside[:-1] != inside[1:]
    flags[:, :-1, :, 1] = inside[:, :-1] != inside[:, 1:]
    flags[:, :, :-1, 2] = inside[:, :, :-1] != inside[:, :, 1:]
    ff = flags.reshape(-1)
    vid = np.cumsum(ff) - 1
    ids = np.nonzero(ff)[0]
    p = ids // 3
    a = ids % 3
    i, j, k = p // (n1 * n2), (p // n2) % n1, p % n2
    v0 = vol[i, j, k]
    step = np.stack([a == 0, a == 1, a == 2], 1).astype(np.int64)
    v1 = vol[i + step[:, 0], j + step[:, 1], k + step[:, 2]]
    v0, v1 = v0.astype(np.float64), v1.astype(np.float64)
    t = (np.float64(iso) - v0) / (v1 - v0)
    base = np.stack([i, j, k], 1).astype(np.float64)
    verts = base + step.astype(np.float64) * t[:, None]
    # cubes
    c = inside.astype(np.int64)
    case = (c[:-1, :-1, :-1] | c[1:, :-1, :-1] << 1 | c[1:, 1:, :-1] << 2 | c[:-1, 1:, :-1] << 3 |
            c[:-1, :-1, 1:] << 4 | c[1:, :-1, 1:] << 5 | c[1:, 1:, 1:] << 6 | c[:-1, 1:, 1:] << 7)
    # cube edge -> (di, dj, dk, axis)
    E = [(0, 0, 0, 0), (1, 0, 0, 1), (0, 1, 0, 0), (0, 0, 0, 1), (0, 0, 1, 0), (1, 0, 1, 1),
         (0, 1, 1, 0), (0, 0, 1, 1), (0, 0, 0, 2), (1, 0, 0, 2), (1, 1, 0, 2), (0, 1, 0, 2)]
    tris = []
    ci, cj, ck = np.nonzero((case != 0) & (case != 255))
    for x, y, z in zip(ci, cj, ck):
        row = table[case[x, y, z]]
        for q in range(0, 15, 3):
            if row[q] < 0:
                break
            tri = []
            for e in row[q:q + 3]:
                di, dj, dk, ax = E[e]
                lid = 3 * (((x + di) * n1 + (y + dj)) * n2 + (z + dk)) + ax
                tri.append(vid[lid])
            tris.append(tri)
    return verts, np.asarray(tris, dtype=np.int64).reshape(-1, 3)
