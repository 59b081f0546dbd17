"""ORACLE (test infrastructure only) -- CPU restatement of the tiny-cuda-nn
multi-resolution Grid/Hash encoding that the reference instantiates at
tropical/tropical.py:32-40 and calls at tropical/tropical.py:46-47.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  The product path
(``tropical-nerf.pytorch_amd/tropical``) never does.

tinycudann is an un-vendored, unpinned third-party dependency of the
reference (absent from requirements.txt:1-8), so the encoding arithmetic is
**parity unpinned** with respect to real tcnn.  What this module pins is the
build's *definition* of the encoding, which both the golden generator (as the
``tinycudann`` stub injected into the reference) and the HIP kernel
(``csrc/encode_mlp.hip``) implement bit-for-bit:

* per level l (float32, host side):
  ``scale_l = exp2(l * log2(b)) * N_min - 1``; ``res_l = ceil(scale_l) + 1``;
  ``size_l = min(next_multiple(res_l**3, 8), 2**T)``; ``offset_l`` = prefix sum.
* forward, per coordinate: ``pos = x*scale_l + 0.5`` (two roundings, not an
  fma -- the one deliberate deviation from tcnn's ``fmaf``, chosen so that a
  plain CPU restatement is bitwise reproducible), ``g = floor(pos)``,
  ``t = pos - g``.
* corner c = 0..7, bit d of c picks ``g_d + 1`` with factor ``t_d`` else
  ``g_d`` with ``1 - t_d``; weight ``((1*w0)*w1)*w2``.
* index: dense ``g0 + g1*res + g2*res^2`` when ``res^3 <= size_l`` else the
  tcnn coherent prime hash ``g0 ^ g1*2654435761 ^ g2*805459861`` (uint32
  wrap-around), then ``% size_l``.
* accumulation: ``acc = acc + w*val`` (non-fused) in corner order.
* table layout ``params[(offset_l + index)*F + f]``; output column ``l*F + f``.
"""
from __future__ import annotations

import numpy as np
import torch

PRIMES = (1, 2654435761, 805459861)
U32 = 0xFFFFFFFF


def level_meta(n_levels: int, n_min: int, per_level_scale: float, log2_T: int):
    """Per-level (scale fp32, res, size, offset, dense) -- tcnn GridEncoding
    constructor semantics."""
    lb = np.log2(np.float32(per_level_scale))
    scales, res, sizes, offsets, dense = [], [], [], [], []
    off = 0
    for l in range(n_levels):
        s = np.float32(np.exp2(np.float32(l) * lb) * np.float32(n_min) - np.float32(1.0))
        r = int(np.ceil(s)) + 1
        n = r ** 3
        n = (n + 7) // 8 * 8
        n = min(n, 1 << log2_T)
        scales.append(s)
        res.append(r)
        sizes.append(n)
        offsets.append(off)
        dense.append(r ** 3 <= n)
        off += n
    return (np.array(scales, dtype=np.float32), res, sizes, offsets, dense, off)


def _corner_index(g: torch.Tensor, res: int, size: int, dense: bool) -> torch.Tensor:
    """uint32 index arithmetic carried in int64 (g: N x 3 int64)."""
    g = g & U32
    if dense:
        idx = (g[:, 0] + g[:, 1] * res + g[:, 2] * (res * res)) & U32
    else:
        idx = ((g[:, 0] * PRIMES[0]) & U32) ^ ((g[:, 1] * PRIMES[1]) & U32) ^ \
              ((g[:, 2] * PRIMES[2]) & U32)
    return idx % size


class _GridFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, params, meta, F):
        scales, res, sizes, offsets, dense, _ = meta
        N = x.shape[0]
        L = len(res)
        out = torch.zeros(N, L * F, dtype=torch.float32)
        for l in range(L):
            pos = x * torch.tensor(scales[l]) + 0.5
            g = torch.floor(pos)
            t = pos - g
            gi = g.to(torch.int64)
            acc = torch.zeros(N, F, dtype=torch.float32)
            for c in range(8):
                w = torch.ones(N, dtype=torch.float32)
                gc = gi.clone()
                for d in range(3):
                    if (c >> d) & 1:
                        w = w * t[:, d]
                        gc[:, d] += 1
                    else:
                        w = w * (1 - t[:, d])
                row = _corner_index(gc, res[l], sizes[l], dense[l]) + offsets[l]
                val = params.view(-1, F)[row]
                acc = acc + w[:, None] * val
            out[:, l * F:(l + 1) * F] = acc
        ctx.save_for_backward(x, params)
        ctx.meta = meta
        ctx.F = F
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, params = ctx.saved_tensors
        scales, res, sizes, offsets, dense, _ = ctx.meta
        F = ctx.F
        N = x.shape[0]
        gx = torch.zeros_like(x) if ctx.needs_input_grad[0] else None
        gp = torch.zeros_like(params) if ctx.needs_input_grad[1] else None
        for l in range(len(res)):
            s = torch.tensor(scales[l])
            pos = x * s + 0.5
            g = torch.floor(pos)
            t = pos - g
            gi = g.to(torch.int64)
            go = grad_out[:, l * F:(l + 1) * F]
            for c in range(8):
                f = [t[:, d] if (c >> d) & 1 else 1 - t[:, d] for d in range(3)]
                gc = gi.clone()
                for d in range(3):
                    gc[:, d] += (c >> d) & 1
                row = _corner_index(gc, res[l], sizes[l], dense[l]) + offsets[l]
                if gp is not None:
                    w = f[0] * f[1] * f[2]
                    gp.view(-1, F).index_add_(0, row, w[:, None] * go)
                if gx is not None:
                    val = params.view(-1, F)[row]
                    dv = (val * go).sum(-1)
                    for d in range(3):
                        sgn = 1.0 if (c >> d) & 1 else -1.0
                        o = [f[e] for e in range(3) if e != d]
                        gx[:, d] += sgn * o[0] * o[1] * dv * s
        return gx, gp, None, None


class GridHashEncoding(torch.nn.Module):
    """Drop-in for ``tcnn.Encoding(3, {"otype": "Grid", "type": "Hash", ...})``
    with a flat fp32 ``params`` parameter (the reference's state_dict key
    ``enc.module.params``)."""

    def __init__(self, n_input_dims: int = 3, encoding_config: dict = None,
                 dtype=torch.float32):
        super().__init__()
        cfg = dict(encoding_config or {})
        assert n_input_dims == 3
        self.n_levels = int(cfg.get("n_levels", 16))
        self.F = int(cfg.get("n_features_per_level", 2))
        self.log2_T = int(cfg.get("log2_hashmap_size", 19))
        self.n_min = int(cfg.get("base_resolution", 16))
        self.b = float(cfg.get("per_level_scale", 2.0))
        self.meta = level_meta(self.n_levels, self.n_min, self.b, self.log2_T)
        self.n_output_dims = self.n_levels * self.F
        n_params = self.meta[-1] * self.F
        g = torch.Generator().manual_seed(1337)
        self.params = torch.nn.Parameter(
            (torch.rand(n_params, generator=g, dtype=torch.float32) * 2 - 1) * 1e-4)

    def forward(self, x):
        return _GridFn.apply(x.float().contiguous(), self.params, self.meta, self.F)
