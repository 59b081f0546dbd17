"""TropicalHashGrid: the hash-grid encoding wrapper of the reference
(tropical/tropical.py:20-239), MI355X-native.

Same constructor, attributes (``marks``, ``module.params`` -> state_dict key
``enc.module.params``), and methods (``forward``, ``skeleton``, ``region``,
``p2v``, ``v2p``).  The encoding arithmetic is the tcnn Grid/Hash definition
restated in SURVEY Appendix A; the compute runs in HIP kernels
(csrc/net.hip) through the C ABI -- there is no CPU fallback.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor

from . import _hip


def level_meta(n_levels: int, n_min: int, per_level_scale: float, log2_T: int):
    """tcnn GridEncoding per-level constants (fp32 scale, res, size, offset,
    dense) -- SURVEY Appendix A."""
    lb = np.log2(np.float32(per_level_scale))
    scales, res, sizes, offsets, dense = [], [], [], [], []
    off = 0
    for l in range(n_levels):
        s = np.float32(np.exp2(np.float32(l) * lb) * np.float32(n_min) - np.float32(1.0))
        r = int(np.ceil(s)) + 1
        n = min((r ** 3 + 7) // 8 * 8, 1 << log2_T)
        scales.append(s)
        res.append(r)
        sizes.append(n)
        offsets.append(off)
        dense.append(r ** 3 <= n)
        off += n
    return np.array(scales, dtype=np.float32), res, sizes, offsets, dense, off


def compute_marks(L: int, n_min: int, b: float, scale: float = 1.0, eps: float = 1e-4) -> Tensor:
    """Kink positions of all levels (tropical.py:49-79), host-side setup.

    Same float64 cell size / fp32 ``arange`` construction and the same
    sequential merge of marks closer than eps, so the marks are bitwise the
    reference's.

    Attribution: this construction restates seonghunn/tropical-nerf.pytorch
    (tropical/tropical.py:49-79, Copyright (c) 2024-present NAVER Cloud Corp.),
    licensed CC BY-SA 4.0; the marks have to be the reference's bit for bit."""
    cand = []
    for l in range(L):
        n_cells = np.exp2(l * np.log2(b)) * n_min - 1.0
        u = 1 / n_cells
        cand.append(torch.arange(0, 1.5, u) - 0.5 * u)
    cand.append(torch.Tensor([0, scale]))
    mk, _ = torch.cat(cand).unique().sort()
    keep = torch.ones(len(mk), dtype=torch.bool)
    for i in range(len(mk) - 1):
        if eps > (mk[i] - mk[i + 1]).abs():
            mk[i + 1] = (mk[i] + mk[i + 1]) / 2
            keep[i] = False
    mk = mk[keep]
    mk = mk[mk >= 0]
    return mk[mk <= scale]


class GridParams(nn.Module):
    """Holds the flat fp32 hash table like ``tcnn.Encoding`` (``params``)."""

    def __init__(self, n_params: int):
        super().__init__()
        g = torch.Generator().manual_seed(1337)
        self.params = nn.Parameter((torch.rand(n_params, generator=g) * 2 - 1) * 1e-4)


class TropicalHashGrid(nn.Module):
    def __init__(self, scale: float = 1.0, D: int = 3, L: int = 16, F: int = 2, T: int = 19,
                 N_min: int = 16, N_max: int = 2048, eps: float = 1e-4):
        super().__init__()
        if D != 3 or F != 2:
            raise NotImplementedError("TropicalHashGrid: D=3, F=2 only (as the reference's Net)")
        self.scale, self.D, self.L, self.F, self.T = scale, D, L, F, T
        self.N_min, self.N_max, self.eps = N_min, N_max, eps
        self.b = np.exp2(np.log2(N_max * scale / N_min) / (L - 1))
        self.meta = level_meta(L, N_min, self.b, T)
        self.module = GridParams(self.meta[-1] * F)
        self.register_buffer("marks", compute_marks(L, N_min, self.b, scale, eps), persistent=False)

    # -- C ABI descriptor ---------------------------------------------------
    def tnp_fields(self, s: "_hip.TnpNet"):
        scales, res, sizes, offsets, dense, _ = self.meta
        if self.L > _hip.MAX_LEVELS:
            raise NotImplementedError(f"at most {_hip.MAX_LEVELS} levels")
        s.n_levels, s.n_features, s.n_marks = self.L, self.F, len(self.marks)
        for l in range(self.L):
            s.scales[l] = float(scales[l])
            s.res[l] = res[l]
            s.sizes[l] = sizes[l]
            s.offsets[l] = offsets[l]
            s.dense[l] = int(dense[l])

    def forward(self, x: Tensor) -> Tensor:
        """Raw encoding of x in [0,1]^3 -> N x (L*F) (tcnn column order)."""
        net = _GridOnlyNet(self)
        return net.encode(x)

    # -- skeleton ------------------------------------------------------------
    def p2v(self, indices: Tensor) -> Tensor:
        L = len(self.marks)
        idx = indices.clone()
        for i in range(self.D):
            idx[..., -1 - i] *= L ** i
        return idx.sum(dim=-1).long()

    def v2p(self, v_idx: Tensor) -> Tensor:
        # the reference's float32 true division (tropical.py:149-156)
        L = len(self.marks)
        p = []
        v = v_idx.clone()
        for i in range(self.D - 1, -1, -1):
            p.append(v.div(L ** i).floor().long())
            v.sub_(p[-1] * L ** i)
        return torch.stack(p, dim=-1)

    def skeleton(self, net: nn.Module, unit: int = 128, mode: str = "distance") -> Tuple[Tensor, Tensor]:
        """Pruned initial edge set (tropical.py:158-225), on device.  mode is
        the reference's PRUNING_MODE: "distance" (its value) or "sign" (its
        dormant branch, tropical.py:198-202: edges whose endpoints' eps-sign
        vectors differ)."""
        from ._engine import engine_for
        eng = engine_for(net)
        V, E = eng.skeleton(unit=unit, size=None, mode=mode)
        if E == 0:
            dev = self.marks.device
            return torch.zeros(0, device=dev), torch.zeros(0, dtype=torch.int64, device=dev)
        verts, edges, _ = eng.export()
        return verts, edges

    def region(self, x: Tensor, eps: float = None) -> Tuple[Tensor, Tensor]:
        """eps-tolerant grid offsets/masks of x in [0,1]^3 (tropical.py:227-236)."""
        eps = self.eps if eps is None else eps
        _hip.require_cuda(x, "TropicalHashGrid.region")
        off = torch.searchsorted(self.marks, x + eps) - 1
        mask = ((self.marks[off] - x).abs() > eps).long()
        return mask, off

    def device(self):
        return next(self.parameters()).device


class _GridOnlyNet:
    """Minimal tnp_net view for encoding-only calls."""

    def __init__(self, grid: TropicalHashGrid):
        self.grid = grid

    def encode(self, x: Tensor) -> Tensor:
        _hip.require_cuda(x, "TropicalHashGrid.forward")
        s = _hip.TnpNet()
        self.grid.tnp_fields(s)
        s.num_layers, s.num_hidden, s.eps = 3, 16, float(self.grid.eps)
        table = self.grid.module.params.detach().contiguous()
        marks = self.grid.marks.contiguous()
        dummy = torch.zeros(1, device=x.device)
        s.d_table, s.d_marks, s.d_weights = table.data_ptr(), marks.data_ptr(), dummy.data_ptr()
        x = x.detach().float().contiguous()
        out = torch.empty(x.shape[0], self.grid.L * self.grid.F, device=x.device)
        _hip.check(_hip.lib().tnp_encode(C_ref(s), _hip.ptr(x), x.shape[0], _hip.ptr(out),
                                         C_void(_hip.stream_ptr(x.device))), "tnp_encode")
        return out


def C_ref(s):
    import ctypes
    return ctypes.byref(s)


def C_void(p: int):
    import ctypes
    return ctypes.c_void_p(p)
