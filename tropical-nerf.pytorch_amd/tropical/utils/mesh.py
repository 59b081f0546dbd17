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


def load_ply(path: str) -> Mesh:
    """Reader for the binary PLY files Mesh.export writes."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode().splitlines()
    nv = int(next(l for l in head if l.startswith("element vertex")).split()[-1])
    nf = int(next(l for l in head if l.startswith("element face")).split()[-1])
    V = np.frombuffer(data, dtype="<f4", count=3 * nv, offset=end).reshape(nv, 3)
    fv = np.frombuffer(data, dtype=[("n", "u1"), ("i", "<i4", (3,))], count=nf, offset=end + 12 * nv)
    return Mesh(V, fv["i"])
