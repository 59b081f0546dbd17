"""Triangle mesh container + PLY writer (the trimesh.Trimesh(process=False)
/ .export surface train.py:254-269 uses)."""
from __future__ import annotations

import os

import numpy as np


class Mesh:
    def __init__(self, vertices, faces, process: bool = False):
        self.vertices = np.asarray(vertices, dtype=np.float64).reshape(-1, 3)
        self.faces = np.asarray(faces, dtype=np.int64).reshape(-1, 3)
        if process:
            raise NotImplementedError("process=True (vertex merging) is not part of the path")

    def export(self, path: str):
        """Binary little-endian PLY (float32 vertices, int32 index lists)."""
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        head = ("ply\nformat binary_little_endian 1.0\n"
                f"element vertex {len(self.vertices)}\n"
                "property float x\nproperty float y\nproperty float z\n"
                f"element face {len(self.faces)}\n"
                "property list uchar int vertex_indices\nend_header\n").encode()
        fv = np.empty(len(self.faces), dtype=[("n", "u1"), ("i", "<i4", (3,))])
        fv["n"] = 3
        fv["i"] = self.faces
        with open(path, "wb") as f:
            f.write(head)
            f.write(self.vertices.astype("<f4").tobytes())
            f.write(fv.tobytes())


_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def merge_vertices(verts: np.ndarray, tris: np.ndarray, digits: int = 8):
    """trimesh's process=True vertex merge (the default of the trimesh.load
    calls in dataset.py:39-67): vertices equal after rounding to `digits`
    decimals (trimesh's merge tolerance, 1e-8) become one, vertices no face
    references are dropped (a mesh with faces), first-occurrence order is
    kept and the faces are remapped.  trimesh is absent here, so the exact
    rounding rule is restated, not pinned against it."""
    verts = np.asarray(verts, dtype=np.float64)
    tris = np.asarray(tris, dtype=np.int64).reshape(-1, 3)
    keep = np.ones(len(verts), dtype=bool)
    if len(tris):
        keep[:] = False
        keep[tris.reshape(-1)] = True
    idx = np.nonzero(keep)[0]
    key = np.round(verts[idx], digits) + 0.0  # + 0.0: -0.0 and 0.0 merge
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")  # groups in first-occurrence order
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    remap = np.full(len(verts), -1, dtype=np.int64)
    remap[idx] = rank[inv.reshape(-1)]
    return verts[idx[first[order]]], remap[tris] if len(tris) else tris


def load_ply(path: str, process: bool = True) -> Mesh:
    """PLY reader for the meshes the training data comes from (the
    trimesh.load calls of dataset.py:39-67): ascii or binary (either
    endianness), any extra vertex properties (the Stanford scans carry
    confidence / intensity), faces as index lists (polygons fan-triangulated).
    Elements other than vertex and face are skipped.  process=True (trimesh's
    default): duplicate vertices merged and unreferenced ones dropped
    (merge_vertices), so the dataset samples the same vertex list."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header") + len(b"end_header")
    end = data.index(b"\n", end) + 1
    fmt, elems = None, []
    for line in data[:end].decode("ascii", "replace").splitlines():
        w = line.split()
        if not w or w[0] in ("ply", "comment", "obj_info", "end_header"):
            continue
        if w[0] == "format":
            fmt = w[1]
        elif w[0] == "element":
            elems.append([w[1], int(w[2]), []])
        elif w[0] == "property":
            if w[1] == "list":
                elems[-1][2].append((w[4], ("list", _PLY_TYPES[w[2]], _PLY_TYPES[w[3]])))
            else:
                elems[-1][2].append((w[2], _PLY_TYPES[w[1]]))
    if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
        raise ValueError(f"{path}: unsupported PLY format {fmt!r}")
    verts, faces = None, []
    if fmt == "ascii":
        toks = data[end:].split()
        pos = 0
        for name, n, props in elems:
            rows = []
            for _ in range(n):
                row = []
                for pname, t in props:
                    if isinstance(t, tuple):
                        k = int(toks[pos])
                        row.append([float(v) for v in toks[pos + 1:pos + 1 + k]])
                        pos += 1 + k
                    else:
                        row.append(float(toks[pos]))
                        pos += 1
                rows.append(row)
            if name == "vertex":
                ix = [i for i, (pn, _) in enumerate(props) if pn in ("x", "y", "z")]
                verts = np.array([[r[i] for i in ix] for r in rows], dtype=np.float64).reshape(-1, 3)
            elif name == "face":
                li = next(i for i, (_, t) in enumerate(props) if isinstance(t, tuple))
                faces = [[int(v) for v in r[li]] for r in rows]
    else:
        bo = "<" if fmt == "binary_little_endian" else ">"
        pos = end
        for name, n, props in elems:
            if all(not isinstance(t, tuple) for _, t in props):
                dt = np.dtype([(pn, bo + t) for pn, t in props])
                arr = np.frombuffer(data, dtype=dt, count=n, offset=pos)
                pos += dt.itemsize * n
                if name == "vertex":
                    verts = np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float64)
                continue
            if name == "face" and len(props) == 1:
                # the common triangle-only layout in one read
                t = props[0][1]
                dt = np.dtype([("n", bo + t[1]), ("i", bo + t[2], (3,))])
                if pos + dt.itemsize * n <= len(data):
                    arr = np.frombuffer(data, dtype=dt, count=n, offset=pos)
                    if (arr["n"] == 3).all():
                        faces = arr["i"].astype(np.int64).tolist()
                        pos += dt.itemsize * n
                        continue
            # elements with list properties: one record at a time
            rows = []
            for _ in range(n):
                row = None
                for pname, t in props:
                    if isinstance(t, tuple):
                        ct, it = np.dtype(bo + t[1]), np.dtype(bo + t[2])
                        k = int(np.frombuffer(data, dtype=ct, count=1, offset=pos)[0])
                        pos += ct.itemsize
                        v = np.frombuffer(data, dtype=it, count=k, offset=pos)
                        pos += it.itemsize * k
                        if row is None:
                            row = v.astype(np.int64).tolist()
                    else:
                        pos += np.dtype(t).itemsize
                rows.append(row or [])
            if name == "face":
                faces = rows
    if verts is None:
        raise ValueError(f"{path}: no vertex element")
    tris = [(f[0], f[i], f[i + 1]) for f in faces for i in range(1, len(f) - 1)]
    tris = np.array(tris, dtype=np.int64).reshape(-1, 3)
    if process:
        verts, tris = merge_vertices(verts, tris)
    return Mesh(verts, tris)
