"""``torch.ops.tropical_hip``: the hot path's entry points on the PyTorch dispatcher.

SURVEY §8(b) specifies a ``tropical_hip`` operator set next to the C ABI.
These ops are registered with ``torch.library.custom_op`` over the same
C ABI (``include/tropical_hip.h``, bound in ``_hip.py``), so there is no
second native library and no second implementation: every op launches the
same gfx950 kernels the drop-in Python surface uses.

The net travels as plain tensors, ``net_args(net)`` builds them:

* ``table``      f32[P]     the hash-grid parameters (``enc.module.params``)
* ``level_meta`` i32[L, 4]  per level (offset, size, res, dense)  (host)
* ``scales``     f32[L]     per-level scale                         (host)
* ``weights``    f32[NW]    ``fc.{i}.weight``, ``fc.{i}.bias`` concatenated
* ``marks``      f32[M]     the sorted kink positions per axis
* ``eps``, ``num_layers``, ``num_hidden``

Ops (reference call site each one replaces):

* ``encode_mlp``    Net.forward(x, gather=True)       model.py:52-76
* ``region``        Net.region                        model.py:90-103
* ``sdf_grad``      Net.sdf / Net.normal              model.py:84-88, 105-123
* ``subpoly_step``  subpoly_ (flat or curve branch)   subpoly.py:90-279
* ``subpoly``       subpoly (skeleton -> faces)       subpoly.py:24-86

They are functional: outputs are freshly allocated on the inputs' device and
stream, inputs are never written (the Python ``subpoly_`` keeps the
reference's in-place rewrite of the caller's edges; ``subpoly_step`` does
not).  Errors of the library surface as ``RuntimeError``; CPU tensors are
refused (there is no CPU fallback).  ``register_fake`` gives every op its
output shapes for meta / FakeTensor tracing.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import torch
from torch import Tensor

from . import _hip

NS = "tropical_hip"


class _OpNet:
    """The duck-typed net the engine and the C ABI need, from op tensors."""

    def __init__(self, table, level_meta, scales, weights, marks, eps, num_layers, num_hidden):
        self.table, self.weights, self.marks = table, weights, marks
        self.level_meta = level_meta.cpu().to(torch.int64)
        self.scales = scales.cpu().to(torch.float32)
        self.eps, self.num_layers, self.num_hidden = float(eps), int(num_layers), int(num_hidden)
        L = self.level_meta.shape[0]
        if L > _hip.MAX_LEVELS or self.level_meta.shape[1] != 4 or self.scales.shape[0] != L:
            raise RuntimeError(f"{NS}: level_meta must be [L, 4] (L <= {_hip.MAX_LEVELS}) "
                               f"with one scale per level")
        nin = 2 * L
        sizes = [nin] + [self.num_hidden] * (self.num_layers - 1) + [2]
        nw = sum(a * b + b for a, b in zip(sizes[:-1], sizes[1:]))
        if weights.numel() != nw:
            raise RuntimeError(f"{NS}: weights hold {weights.numel()} floats, the "
                               f"{self.num_layers}-layer net needs {nw}")
        for name, t in (("table", table), ("weights", weights), ("marks", marks)):
            _hip.require_cuda(t, f"{NS} {name}")
            if t.dtype != torch.float32:
                raise RuntimeError(f"{NS}: {name} must be float32")

    @property
    def K(self) -> int:
        return (self.num_layers - 1) * self.num_hidden + 1

    def device(self):
        return self.table.device

    def tnp_desc(self):
        s = _hip.TnpNet()
        L = self.level_meta.shape[0]
        s.n_levels, s.n_features, s.n_marks = L, 2, self.marks.numel()
        for l in range(L):
            off, size, res, dense = (int(v) for v in self.level_meta[l])
            s.scales[l] = float(self.scales[l])
            s.res[l], s.sizes[l], s.offsets[l], s.dense[l] = res, size, off, dense
        s.num_layers, s.num_hidden, s.eps = self.num_layers, self.num_hidden, self.eps
        table, w, marks = (t.detach().contiguous() for t in (self.table, self.weights, self.marks))
        s.d_table, s.d_weights, s.d_marks = table.data_ptr(), w.data_ptr(), marks.data_ptr()
        return s, (table, w, marks)


def net_args(net) -> tuple:
    """(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    of a ``tropical.stanford.model.Net`` for the ``tropical_hip`` ops."""
    scales, res, sizes, offsets, dense, _ = net.enc.meta
    L = net.enc.L
    meta = torch.tensor([[int(offsets[l]), int(sizes[l]), int(res[l]), int(dense[l])]
                         for l in range(L)], dtype=torch.int32)
    sc = torch.tensor([float(scales[l]) for l in range(L)], dtype=torch.float32)
    dev = net.device()
    table = net.enc.module.params.detach().float().contiguous()
    w = torch.cat([t.detach().float().reshape(-1) for lin in net.fc
                   for t in (lin.weight, lin.bias)]).contiguous()
    marks = net.enc.marks.to(dev).float().contiguous()
    return table, meta, sc, w, marks, float(net.eps), int(net.num_layers), int(net.num_hidden)


def _stream(t: Tensor):
    return C.c_void_p(_hip.stream_ptr(t.device))


def _K(num_layers: int, num_hidden: int) -> int:
    return (num_layers - 1) * num_hidden + 1


# -- encode_mlp ---------------------------------------------------------------

@torch.library.custom_op(f"{NS}::encode_mlp", mutates_args=())
def encode_mlp(coords: Tensor, table: Tensor, level_meta: Tensor, scales: Tensor, weights: Tensor,
               marks: Tensor, eps: float, num_layers: int, num_hidden: int,
               group: int = 1) -> Tuple[Tensor, Tensor]:
    """Fused hash-grid encoding + MLP of coords f32[N, 3] (vertex space,
    [-1, 1]^3): pre-activations f32[K, N] plane-major (rows: the hidden
    layers' pre-activations, then o1 - o0) and the outputs f32[N, 2];
    group=8: the reference's grouped forward over box corners."""
    _hip.require_cuda(coords, f"{NS}::encode_mlp")
    net = _OpNet(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    x = coords.detach().float().contiguous()
    n = x.shape[0]
    pre = torch.empty(net.K, n, device=x.device)
    out2 = torch.empty(n, 2, device=x.device)
    if group not in (1, 8):
        raise RuntimeError(f"{NS}::encode_mlp: group must be 1 or 8")
    s, keep = net.tnp_desc()
    fn = _hip.lib().tnp_forward_grouped if group == 8 else _hip.lib().tnp_forward
    _hip.check(fn(C.byref(s), _hip.ptr(x), n, _hip.ptr(pre), n, _hip.ptr(out2), _stream(x)),
               "tnp_forward")
    del keep
    return pre, out2


@encode_mlp.register_fake
def _(coords, table, level_meta, scales, weights, marks, eps, num_layers, num_hidden, group=1):
    n = coords.shape[0]
    return coords.new_empty(_K(num_layers, num_hidden), n), coords.new_empty(n, 2)


# -- region -------------------------------------------------------------------

@torch.library.custom_op(f"{NS}::region", mutates_args=())
def region(coords: Tensor, pre: Tensor, table: Tensor, level_meta: Tensor, scales: Tensor,
           weights: Tensor, marks: Tensor, eps: float, num_layers: int,
           num_hidden: int) -> Tuple[Tensor, Tensor]:
    """eps-sign region vectors (Net.region): m i64[N, 3 + K] (grid columns
    {0, 1}, plane columns {-1, 0, 1}) and grid offsets i64[N, 3], from the
    plane-major pre-activations f32[K, N] of ``encode_mlp``."""
    _hip.require_cuda(coords, f"{NS}::region")
    net = _OpNet(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    v = coords.detach().float().contiguous()
    p = pre.detach().float().contiguous()
    n = v.shape[0]
    if p.shape != (net.K, n):
        raise RuntimeError(f"{NS}::region: pre must be [K={net.K}, N={n}], got {tuple(p.shape)}")
    m = torch.empty(n, 3 + net.K, dtype=torch.int64, device=v.device)
    off = torch.empty(n, 3, dtype=torch.int64, device=v.device)
    s, keep = net.tnp_desc()
    _hip.check(_hip.lib().tnp_region(C.byref(s), _hip.ptr(v), _hip.ptr(p), n, n, float(eps),
                                     _hip.ptr(m), _hip.ptr(off), _stream(v)), "tnp_region")
    del keep
    return m, off


@region.register_fake
def _(coords, pre, table, level_meta, scales, weights, marks, eps, num_layers, num_hidden):
    n = coords.shape[0]
    return (coords.new_empty(n, 3 + _K(num_layers, num_hidden), dtype=torch.int64),
            coords.new_empty(n, 3, dtype=torch.int64))


# -- sdf_grad -----------------------------------------------------------------

@torch.library.custom_op(f"{NS}::sdf_grad", mutates_args=())
def sdf_grad(coords: Tensor, table: Tensor, level_meta: Tensor, scales: Tensor, weights: Tensor,
             marks: Tensor, eps: float, num_layers: int, num_hidden: int) -> Tuple[Tensor, Tensor]:
    """SDF = tanh(o1 - o0) f32[N] and its input gradient f32[N, 3]."""
    _hip.require_cuda(coords, f"{NS}::sdf_grad")
    net = _OpNet(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    x = coords.detach().float().contiguous()
    n = x.shape[0]
    y = torch.empty(n, device=x.device)
    J = torch.empty(n, 3, device=x.device)
    s, keep = net.tnp_desc()
    _hip.check(_hip.lib().tnp_sdf_grad(C.byref(s), _hip.ptr(x), n, _hip.ptr(y), _hip.ptr(J),
                                       _stream(x)), "tnp_sdf_grad")
    del keep
    return y, J


@sdf_grad.register_fake
def _(coords, table, level_meta, scales, weights, marks, eps, num_layers, num_hidden):
    n = coords.shape[0]
    return coords.new_empty(n), coords.new_empty(n, 3)


# -- subpoly_step / subpoly ---------------------------------------------------

def _engine(net: _OpNet, curve: bool):
    from ._engine import Engine, _ENGINES
    dev = net.device()
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    eng = _ENGINES.get(key)
    if eng is None:
        eng = Engine(torch.device("cuda", key))
        _ENGINES[key] = eng
    return eng.set_net(net).set_curve(curve)


@torch.library.custom_op(f"{NS}::subpoly_step", mutates_args=())
def subpoly_step(vertices: Tensor, edges: Tensor, cache: Tensor, table: Tensor, level_meta: Tensor,
                 scales: Tensor, weights: Tensor, marks: Tensor, eps: float, num_layers: int,
                 num_hidden: int, idx: int, prune: bool, force: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """One hyperplane step on plane idx (= l * num_hidden + h) of the complex
    (vertices f32[V, 3], edges i64[E, 2], cache f32[V, K] of the net's
    pre-activations): the updated (vertices, edges, cache).  force=False is
    the curve branch (with the strict filter)."""
    _hip.require_cuda(vertices, f"{NS}::subpoly_step")
    net = _OpNet(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    if not 0 <= idx < net.K:
        raise RuntimeError(f"{NS}::subpoly_step: plane {idx} outside [0, {net.K})")
    eng = _engine(net, not force)
    eng.load(vertices, edges, cache, keep_all=True)
    S, fail = eng.split(idx)
    if S > 0:
        eng.finish(idx, bool(prune and idx < net.K - 1), fail)
    v, e, o = eng.export(pre=True)
    return v, e, o


def _no_graph(ctx, inputs, output):
    # the reference's subpoly_ takes outputs_ as the net's forward left it --
    # a graph-carrying tensor (subpoly.py:93) -- and nothing it returns is
    # differentiated: the step's outputs carry no graph whatever the inputs
    ctx.mark_non_differentiable(*output)


def _no_grads(ctx, *grads):
    return (None,) * 14


subpoly_step.register_autograd(_no_grads, setup_context=_no_graph)


@subpoly_step.register_fake
def _(vertices, edges, cache, table, level_meta, scales, weights, marks, eps, num_layers,
      num_hidden, idx, prune, force):
    ctx = torch.library.get_ctx()
    V, E = ctx.new_dynamic_size(), ctx.new_dynamic_size()
    return (vertices.new_empty(V, 3), edges.new_empty(E, 2),
            cache.new_empty(V, _K(num_layers, num_hidden)))


@torch.library.custom_op(f"{NS}::subpoly", mutates_args=())
def subpoly(table: Tensor, level_meta: Tensor, scales: Tensor, weights: Tensor, marks: Tensor,
            eps: float, num_layers: int, num_hidden: int, size: float,
            force: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """The whole extraction (skeleton -> every hyperplane step -> surface ->
    faces): (vertices f32[V, 3], faces_with_indices i64[F, 3], faces
    f32[F, 3, 3]), the tensors the reference's subpoly returns as
    (vertices, np faces_with_indices, np faces)."""
    net = _OpNet(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden)
    eng = _engine(net, not force)
    eng.skeleton(unit=128, size=size)
    eng.run_steps()
    dev = eng.device
    sV, _ = eng.surface()
    if sV == 0:
        return (torch.zeros(0, 3, device=dev), torch.zeros(0, 3, dtype=torch.int64, device=dev),
                torch.zeros(0, 3, 3, device=dev))
    verts, _, _ = eng.export()
    tri, fc = eng.faces()
    return verts, tri, fc


@subpoly.register_fake
def _(table, level_meta, scales, weights, marks, eps, num_layers, num_hidden, size, force):
    ctx = torch.library.get_ctx()
    V, F = ctx.new_dynamic_size(), ctx.new_dynamic_size()
    return (table.new_empty(V, 3), table.new_empty(F, 3, dtype=torch.int64),
            table.new_empty(F, 3, 3))


OPS: List[str] = ["encode_mlp", "region", "sdf_grad", "subpoly_step", "subpoly"]
