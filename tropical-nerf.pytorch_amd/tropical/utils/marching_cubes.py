"""GPU marching cubes (replaces `mcubes.marching_cubes`, train.py:284).

`marching_cubes(volume, iso)` meshes the iso level of a [n0, n1, n2] sample
volume (x slowest, the meshgrid 'ij' layout of train.py:281) on the HIP
kernels of csrc/evaluate.hip with the procedural case table of
mc_table.py.  Vertices are in index space, as PyMCubes returns them; inside
is value < iso.  One vertex per crossed lattice edge (PyMCubes' vertex
count); triangle normals point towards value < iso (mc_table.py)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _hip
from .mc_table import case_table

_TABLES = {}


def _table(device) -> torch.Tensor:
    t = _TABLES.get(device)
    if t is None:
        t = torch.from_numpy(case_table()).to(device).contiguous()
        _TABLES[device] = t
    return t


def marching_cubes_torch(volume: torch.Tensor, iso: float = 0.0):
    """volume: fp32 ROCm tensor [n0, n1, n2] -> (vertices fp64 [V, 3],
    triangles int64 [F, 3]) on the same device."""
    _hip.require_cuda(volume, "marching_cubes")
    vol = volume.detach().to(torch.float32).contiguous()
    n0, n1, n2 = vol.shape
    dev = vol.device
    tab = _table(dev)
    eoff = torch.empty(3 * n0 * n1 * n2 + 1, dtype=torch.int64, device=dev)
    coff = torch.empty((n0 - 1) * (n1 - 1) * (n2 - 1) + 1, dtype=torch.int64, device=dev)
    nv, nt = C.c_int64(), C.c_int64()
    s = C.c_void_p(_hip.stream_ptr(dev))
    L = _hip.lib()
    _hip.check(L.tnp_mc_count(_hip.ptr(vol), n0, n1, n2, float(iso), _hip.ptr(tab), _hip.ptr(eoff),
                              _hip.ptr(coff), C.byref(nv), C.byref(nt), s), "tnp_mc_count")
    verts = torch.empty(nv.value, 3, dtype=torch.float64, device=dev)
    tris = torch.empty(nt.value, 3, dtype=torch.int64, device=dev)
    _hip.check(L.tnp_mc_emit(_hip.ptr(vol), n0, n1, n2, float(iso), _hip.ptr(tab), _hip.ptr(eoff),
                             _hip.ptr(coff), _hip.ptr(verts), _hip.ptr(tris), s), "tnp_mc_emit")
    return verts, tris


def marching_cubes(volume, iso: float = 0.0):
    """mcubes.marching_cubes signature: numpy or tensor volume -> numpy
    (vertices float64 [V, 3], triangles int64 [F, 3])."""
    if not isinstance(volume, torch.Tensor):
        volume = torch.from_numpy(np.ascontiguousarray(volume, dtype=np.float32)).cuda()
    v, t = marching_cubes_torch(volume, iso)
    return v.cpu().numpy(), t.cpu().numpy()
