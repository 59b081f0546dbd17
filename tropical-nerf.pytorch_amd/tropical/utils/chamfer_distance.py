"""Chamfer distance and ray-cast surface sampling on the GPU
(tropical/utils/chamfer_distance.py:39-48, 184-212 of the reference).

* `chamfer_distance(x, y)` = (mean NN distance y->x + mean NN distance
  x->y) / 2 with exact nearest neighbours (the reference uses sklearn's
  kd-tree; here a brute-force HIP kernel, tnp_nn_min_dist).
* `sample_surface_from_rays(rays_o, rays_d, mesh, return_normal)`: nearest
  hit of every ray (the reference's cubvh BVH; here a uniform-grid HIP ray
  caster, tnp_raycaster_*), positions of the hits, per-ray face normals
  (face 0 for misses, as the reference) and the hit mask."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _hip


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


def _t(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        return x.detach().to(_dev(), dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x)).to(_dev(), dtype).contiguous()


def nn_min_dist(a, b) -> torch.Tensor:
    """Exact distance of every point of a [n, 3] to its nearest point of b."""
    A, B = _t(a).reshape(-1, 3), _t(b).reshape(-1, 3)
    out = torch.empty(A.shape[0], dtype=torch.float32, device=A.device)
    _hip.check(_hip.lib().tnp_nn_min_dist(_hip.ptr(A), A.shape[0], _hip.ptr(B), B.shape[0],
                                          _hip.ptr(out), C.c_void_p(_hip.stream_ptr(A.device))),
               "tnp_nn_min_dist")
    return out


def chamfer_distance(x, y) -> float:
    min_yx = nn_min_dist(y, x).double().mean()
    min_xy = nn_min_dist(x, y).double().mean()
    return float((min_yx + min_xy) / 2.0)


class RayCaster:
    """cubvh.cuBVH(vertices, faces) replacement: nearest-hit ray casting."""

    def __init__(self, vertices, faces):
        self.V = _t(vertices).reshape(-1, 3)
        self.F = _t(faces, torch.int32).reshape(-1, 3)
        dev = self.V.device
        h = C.c_void_p()
        _hip.check(_hip.lib().tnp_raycaster_create(C.byref(h), dev.index), "tnp_raycaster_create")
        self.h = h
        lo = self.V.min(0).values.cpu().numpy() if len(self.V) else np.zeros(3, np.float32)
        hi = self.V.max(0).values.cpu().numpy() if len(self.V) else np.ones(3, np.float32)
        flo, fhi = (C.c_float * 3)(*lo.tolist()), (C.c_float * 3)(*hi.tolist())
        _hip.check(_hip.lib().tnp_raycaster_build(h, _hip.ptr(self.V), self.V.shape[0], _hip.ptr(self.F),
                                                  self.F.shape[0], flo, fhi,
                                                  C.c_void_p(_hip.stream_ptr(dev))),
                   "tnp_raycaster_build")

    def __del__(self):
        if getattr(self, "h", None) is not None:
            _hip.lib().tnp_raycaster_destroy(self.h)
            self.h = None

    def ray_trace(self, rays_o, rays_d):
        """-> (positions [n, 3], face_id [n] int64 (-1: miss), depth [n])."""
        o, d = _t(rays_o).reshape(-1, 3), _t(rays_d).reshape(-1, 3)
        n = o.shape[0]
        t = torch.empty(n, dtype=torch.float32, device=o.device)
        f = torch.empty(n, dtype=torch.int32, device=o.device)
        _hip.check(_hip.lib().tnp_raycaster_cast(self.h, _hip.ptr(o), _hip.ptr(d), n, _hip.ptr(t),
                                                 _hip.ptr(f), C.c_void_p(_hip.stream_ptr(o.device))),
                   "tnp_raycaster_cast")
        hit = f >= 0
        depth = torch.where(hit, t, torch.zeros_like(t))
        pos = o + d * depth[:, None]
        return pos, f.long(), depth


def sample_surface_from_rays(rays_o, rays_d, mesh, return_normal: bool = False):
    RT = RayCaster(mesh.vertices, mesh.faces)
    positions, face_id, depth = RT.ray_trace(rays_o, rays_d)
    mask = face_id >= 0
    pos = positions[mask].cpu().numpy().reshape(-1, 3)
    if return_normal:
        fid = face_id.clone()
        fid[~mask] = 0
        faces = np.asarray(mesh.vertices)[np.asarray(mesh.faces)[fid.cpu().numpy()]]
        normals = np.cross(faces[:, 1] - faces[:, 0], faces[:, 2] - faces[:, 0])
        normals /= (np.linalg.norm(normals, axis=-1, keepdims=True) + 1e-9)
        return pos, normals, mask.cpu().numpy()
    return pos
