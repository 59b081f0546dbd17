"""Net: the piecewise-trilinear SDF network of the reference
(tropical/stanford/model.py:18-135), MI355X-native.

Same constructor, attributes (``enc``, ``fc``, ``num_layers``,
``num_hidden``, ``num_nodes``, ``eps``, ``scale``), state_dict keys
(``enc.module.params``, ``fc.{i}.weight``, ``fc.{i}.bias``) and methods
(``forward(x, gather, group)``, ``preprocess``, ``preprocess_inverse``,
``sdf``, ``region``, ``normal``).  Every evaluation is a fused HIP kernel
(encoding + MLP, csrc/net.hip) on the net's ROCm device; the forward is
bitwise equal to the reference's PyTorch-CPU evaluation.

Autograd, as the reference's (autograd through tcnn and nn.Linear there):
``sdf`` is differentiable w.r.t. its input (the analytic input gradient of
``tnp_sdf_grad``) and the parameters (``tnp_sdf_vjp``: the encoding table
and the fc weights); ``forward(x, gather)`` w.r.t. both through every
gathered plane and the output (``tnp_forward_vjp``); ``normal(...,
create_graph=True)`` returns J with a graph whose backward -- the
reference's double backward, the eikonal term of train.py:196 -- is
``tnp_normal_vjp`` (parameters, and the Hessian along the upstream for the
points).  Every instantiated net shape.  ``region`` and ``normal`` without
``create_graph`` return values without a graph, as the extraction uses them.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
from torch import Tensor

from .. import _hip
from ..tropical import TropicalHashGrid


class _SDF(torch.autograd.Function):
    """Net.sdf with its backward: d sdf / d x from tnp_sdf_grad (computed in
    the forward's kernel), d sdf / d theta as one tnp_sdf_vjp call."""

    @staticmethod
    def forward(ctx, net, x, table, *weights):
        y, J = net._sdf_eval(x, want_grad=bool(ctx.needs_input_grad[1]))
        ctx.net = net
        # the parameters' versions at forward time: the backward's VJP reads
        # the parameters as they are then, so an in-place change in between
        # must fail as autograd's saved-tensor check would
        ctx.versions = tuple(t._version for t in (table,) + weights)
        ctx.save_for_backward(x, J)
        return y.unsqueeze(-1)

    @staticmethod
    def backward(ctx, gy):
        net = ctx.net
        x, J = ctx.saved_tensors
        now = tuple(t._version for t in net._params())
        if any(ctx.needs_input_grad[2:]) and now != ctx.versions:
            raise RuntimeError("Net.sdf backward: a parameter was modified in place after the forward "
                               "(its version changed); the gradient would be taken at other weights")
        if torch.is_grad_enabled() and ctx.needs_input_grad[1]:
            # create_graph=True (the reference's Net.normal / eikonal term,
            # train.py:196): the input gradient g * J with a graph through
            # _Normal (whose backward is the double backward); the parameter
            # gradients are returned as values (their own derivatives are not
            # tracked -- autograd.grad(..., x, create_graph=True) discards them)
            Jg, _ = _Normal.apply(net, x, *net._params())
            gx = gy.reshape(-1, 1).to(Jg.dtype) * Jg
            with torch.no_grad():
                grads = _SDF._param_vjp(ctx, net, x, gy)
            return (None, gx.to(x.dtype), *grads)
        g = gy.detach().reshape(-1).float().contiguous()
        gx = (g[:, None] * J).to(x.dtype) if ctx.needs_input_grad[1] else None
        return (None, gx, *_SDF._param_vjp(ctx, net, x, gy))

    @staticmethod
    def _param_vjp(ctx, net, x, gy):
        grads = [None] * (len(ctx.needs_input_grad) - 2)
        if not any(ctx.needs_input_grad[2:]):
            return grads
        g = gy.detach().reshape(-1).float().contiguous()
        params = net._params()
        g_table = torch.zeros(params[0].numel(), device=x.device)
        g_w = torch.zeros(sum(t.numel() for t in params[1:]), device=x.device)
        s, keep = net.tnp_desc()
        xs = x.detach().float().contiguous()
        _hip.check(_hip.lib().tnp_sdf_vjp(ctypes.byref(s), _hip.ptr(xs), _hip.ptr(g), xs.shape[0],
                                          _hip.ptr(g_table), _hip.ptr(g_w),
                                          ctypes.c_void_p(_hip.stream_ptr(x.device))), "tnp_sdf_vjp")
        del keep
        return _param_grads(net, g_table, g_w, ctx.needs_input_grad[2:])


def _param_grads(net, g_table, g_w, needs):
    """Split the C ABI's packed gradients over the parameters (table, then
    fc.{i}.weight / bias); None where no gradient is needed."""
    params = net._params()
    out = [None] * len(params)
    if needs[0]:
        out[0] = g_table.view_as(params[0]).to(params[0].dtype)
    off = 0
    for k, t in enumerate(params[1:]):
        if needs[1 + k]:
            out[1 + k] = g_w[off:off + t.numel()].view_as(t).to(t.dtype)
        off += t.numel()
    return out


class _Forward(torch.autograd.Function):
    """Net.forward with its backward (the reference's is autograd through tcnn
    and nn.Linear, model.py:52-76): outputs the gathered planes (plane-major
    [K, n], as tnp_forward writes them) and the output [n, 2]; the backward
    is one tnp_forward_vjp call (table, fc parameters and the points)."""

    @staticmethod
    def forward(ctx, net, x, table, *weights):
        pre, out = net._forward_planes(x, 1, want_out=True)
        ctx.net = net
        ctx.versions = tuple(t._version for t in (table,) + weights)
        ctx.save_for_backward(x)
        return pre, out

    @staticmethod
    def backward(ctx, g_pre, g_out):
        if torch.is_grad_enabled():
            raise NotImplementedError("double backward through Net.forward")
        net = ctx.net
        (x,) = ctx.saved_tensors
        if any(ctx.needs_input_grad[2:]) and tuple(t._version for t in net._params()) != ctx.versions:
            raise RuntimeError("Net.forward backward: a parameter was modified in place after the forward")
        n = x.shape[0]
        gp = None if g_pre is None else g_pre.detach().float().contiguous()
        go = None if g_out is None else g_out.detach().float().contiguous()
        params = net._params()
        g_table = torch.zeros(params[0].numel(), device=x.device)
        g_w = torch.zeros(sum(t.numel() for t in params[1:]), device=x.device)
        gx = torch.zeros(n, 3, device=x.device) if ctx.needs_input_grad[1] else None
        if gp is None and go is None:
            return (None, None, *([None] * len(params)))
        s, keep = net.tnp_desc()
        xs = x.detach().float().contiguous()
        _hip.check(_hip.lib().tnp_forward_vjp(ctypes.byref(s), _hip.ptr(xs), n, _hip.ptr(gp), n, _hip.ptr(go),
                                              _hip.ptr(g_table), _hip.ptr(g_w), _hip.ptr(gx),
                                              ctypes.c_void_p(_hip.stream_ptr(x.device))), "tnp_forward_vjp")
        del keep
        grads = _param_grads(net, g_table, g_w, ctx.needs_input_grad[2:])
        return (None, None if gx is None else gx.to(x.dtype), *grads)


class _Normal(torch.autograd.Function):
    """Net.normal(create_graph=True): J = d sdf / d x as a differentiable
    output (the reference's autograd.grad(..., create_graph=True) through
    tcnn, model.py:105-123); its backward -- the reference's double
    backward -- is one tnp_normal_vjp call (the parameters' gradient of
    gJ . J and the Hessian of sdf along gJ for the points)."""

    @staticmethod
    def forward(ctx, net, x, table, *weights):
        y, J = net._sdf_eval(x, want_grad=True)
        ctx.net = net
        ctx.versions = tuple(t._version for t in (table,) + weights)
        ctx.save_for_backward(x)
        return J, y.unsqueeze(-1)

    @staticmethod
    def backward(ctx, gJ, gy):
        if torch.is_grad_enabled():
            raise NotImplementedError("third-order derivatives through Net.normal")
        net = ctx.net
        (x,) = ctx.saved_tensors
        if any(ctx.needs_input_grad[2:]) and tuple(t._version for t in net._params()) != ctx.versions:
            raise RuntimeError("Net.normal backward: a parameter was modified in place after the forward")
        n = x.shape[0]
        params = net._params()
        g_table = torch.zeros(params[0].numel(), device=x.device)
        g_w = torch.zeros(sum(t.numel() for t in params[1:]), device=x.device)
        gx = torch.zeros(n, 3, device=x.device) if ctx.needs_input_grad[1] else None
        s, keep = net.tnp_desc()
        xs = x.detach().float().contiguous()
        stream = ctypes.c_void_p(_hip.stream_ptr(x.device))
        if gJ is not None:
            g = gJ.detach().float().contiguous()
            _hip.check(_hip.lib().tnp_normal_vjp(ctypes.byref(s), _hip.ptr(xs), _hip.ptr(g), n, _hip.ptr(g_table),
                                                 _hip.ptr(g_w), _hip.ptr(gx), stream), "tnp_normal_vjp")
        if gy is not None:  # the returned y (return_y=True): Net.sdf's backward
            g1 = gy.detach().reshape(-1).float().contiguous()
            _hip.check(_hip.lib().tnp_sdf_vjp(ctypes.byref(s), _hip.ptr(xs), _hip.ptr(g1), n, _hip.ptr(g_table),
                                              _hip.ptr(g_w), stream), "tnp_sdf_vjp")
            if gx is not None:
                _, J = net._sdf_eval(x, want_grad=True)
                gx += g1[:, None] * J
        del keep
        grads = _param_grads(net, g_table, g_w, ctx.needs_input_grad[2:])
        return (None, None if gx is None else gx.to(x.dtype), *grads)


class Net(nn.Module):
    def __init__(self, num_layers: int = 3, num_hidden: int = 16, levels: int = 4,
                 r_min: int = 2, r_max: int = 32, T: int = 19, eps: float = 1e-4):
        super().__init__()
        self.num_layers = num_layers
        self.num_hidden = num_hidden
        self.eps = eps
        self.scale = 1
        self.enc = TropicalHashGrid(1.0, 3, levels, 2, T, r_min, r_max, eps)
        self.num_nodes = [levels * 2] + [num_hidden] * (num_layers - 1) + [2]
        self.fc = nn.ModuleList(nn.Linear(a, b) for a, b in
                                zip(self.num_nodes[:-1], self.num_nodes[1:]))
        self._flatten_fc()

    def _params(self):
        return [self.enc.module.params] + [t for lin in self.fc for t in (lin.weight, lin.bias)]

    def _flatten_fc(self):
        """Every fc weight and bias becomes a view of ONE flat buffer, in the
        C ABI's order (W0, b0, W1, b1, ...): the kernels read that buffer
        directly, so any in-place change -- including through ``p.data``,
        which bumps no version counter -- is what they see, with no copy to
        go stale (tnp_desc)."""
        ts = [t for lin in self.fc for t in (lin.weight, lin.bias)]
        if len({(t.device, t.dtype) for t in ts}) != 1:
            self._fc_flat = None
            return
        flat = torch.empty(sum(t.numel() for t in ts), dtype=ts[0].dtype, device=ts[0].device)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                flat[off:off + n].copy_(t.reshape(-1))
                t.data = flat[off:off + n].view_as(t)
                off += n
        self._fc_flat = flat

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cuda() / .float() give every parameter new storage
        out = super()._apply(fn, *args, **kwargs)
        self._flatten_fc()
        return out

    def _fc_buffer(self):
        """The flat fp32 weight buffer the kernels read: the parameters' own
        storage when they are still views of it, else a fresh copy."""
        flat = getattr(self, "_fc_flat", None)
        ts = [t for lin in self.fc for t in (lin.weight, lin.bias)]
        if flat is not None and flat.dtype == torch.float32:
            off, ok = 0, True
            for t in ts:
                if t.data_ptr() != flat.data_ptr() + 4 * off or not t.is_contiguous():
                    ok = False
                    break
                off += t.numel()
            if ok:
                return flat
        return torch.cat([t.detach().float().reshape(-1) for t in ts]).contiguous()

    @property
    def K(self) -> int:
        return (self.num_layers - 1) * self.num_hidden + 1

    def device(self):
        return next(self.parameters()).device

    # -- C ABI descriptor ----------------------------------------------------
    def tnp_desc(self):
        """(tnp_net struct, keep-alive tensors) for the current parameters.
        The kernels read the parameters' own storage (the table, and the fc
        weights' flat buffer, _flatten_fc), so edits in place are always
        seen; the descriptor is rebuilt when a parameter got new storage (or,
        for parameters that no longer share the flat buffer, a new version)."""
        dev = self.device()
        if dev.type != "cuda":
            raise RuntimeError("Net: move the net to a ROCm GPU (.cuda()); the tropical HIP "
                               "path has no CPU fallback")
        params = self._params()
        sig = (self.num_layers, self.num_hidden, float(self.eps),
               tuple((t.data_ptr(), t._version, t.dtype) for t in params), self.enc.marks.data_ptr())
        cached = getattr(self, "_tnp_cache", None)
        if cached is not None and cached[0] == sig:
            return cached[1]
        s = _hip.TnpNet()
        self.enc.tnp_fields(s)
        s.num_layers, s.num_hidden, s.eps = self.num_layers, self.num_hidden, float(self.eps)
        table = self.enc.module.params.detach().float().contiguous()
        w = self._fc_buffer()
        marks = self.enc.marks.to(dev).contiguous()
        s.d_table, s.d_weights, s.d_marks = table.data_ptr(), w.data_ptr(), marks.data_ptr()
        self._tnp_cache = (sig, (s, (table, w, marks)))
        return s, (table, w, marks)

    # -- evaluation ----------------------------------------------------------
    def _forward_planes(self, x: Tensor, group: int = 1, want_out: bool = False):
        _hip.require_cuda(x, "Net.forward")
        s, keep = self.tnp_desc()
        x = x.detach().float().contiguous()
        n = x.shape[0]
        pre = torch.empty(self.K, n, device=x.device)
        out2 = torch.empty(n, 2, device=x.device) if want_out else None
        fn = _hip.lib().tnp_forward_grouped if group == 8 else _hip.lib().tnp_forward
        if group not in (1, 8):
            raise NotImplementedError("group must be 1 or 8 (box corners)")
        _hip.check(fn(ctypes.byref(s), _hip.ptr(x), n, _hip.ptr(pre), n, _hip.ptr(out2),
                      ctypes.c_void_p(_hip.stream_ptr(x.device))), "tnp_forward")
        del keep
        return pre, out2

    def forward(self, x, gather: bool = False, group: int = 1):
        params = self._params()
        if (group == 1 and torch.is_grad_enabled()
                and (x.requires_grad or any(p.requires_grad for p in params))):
            # differentiable as the reference's (autograd through tcnn and nn.Linear)
            pre, out = _Forward.apply(self, x, *params)
        else:
            pre, out = self._forward_planes(x, group, want_out=True)
        if not gather:
            return out
        H = self.num_hidden
        cols = pre.t()
        inputs = [cols[:, i * H:(i + 1) * H] for i in range(self.num_layers - 1)]
        inputs.append(cols[:, -1:])
        return out, inputs

    def preprocess(self, x):
        return (x + self.scale) / (self.scale * 2)

    def preprocess_inverse(self, x):
        return x * (self.scale * 2) - self.scale

    def _sdf_eval(self, x, want_grad: bool = False):
        """(sdf [n], d sdf / d x [n, 3] or None) from one tnp_sdf_grad call."""
        _hip.require_cuda(x, "Net.sdf")
        s, keep = self.tnp_desc()
        x = x.detach().float().contiguous()
        y = torch.empty(x.shape[0], device=x.device)
        J = torch.empty(x.shape[0], 3, device=x.device) if want_grad else None
        _hip.check(_hip.lib().tnp_sdf_grad(ctypes.byref(s), _hip.ptr(x), x.shape[0], _hip.ptr(y),
                                           _hip.ptr(J), ctypes.c_void_p(_hip.stream_ptr(x.device))),
                   "tnp_sdf_grad")
        del keep
        return y, J

    def sdf(self, x):
        """tanh(o1 - o0) (model.py:84-88); differentiable w.r.t. x and the
        parameters under grad mode (module docstring)."""
        params = self._params()
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _SDF.apply(self, x, *params)
        return self._sdf_eval(x)[0].unsqueeze(-1)

    def region(self, vertices: Tensor, output: Tensor = None, eps=None):
        eps = self.eps if eps is None else eps
        _hip.require_cuda(vertices, "Net.region")
        v = vertices.detach().float().contiguous()
        if output is None:
            planes, _ = self._forward_planes(v)
            output = planes.t()
        else:
            planes = output.detach().float().t().contiguous()
        s, keep = self.tnp_desc()
        n = v.shape[0]
        m = torch.empty(n, 3 + self.K, dtype=torch.int64, device=v.device)
        off = torch.empty(n, 3, dtype=torch.int64, device=v.device)
        _hip.check(_hip.lib().tnp_region(ctypes.byref(s), _hip.ptr(v), _hip.ptr(planes), n, n,
                                         float(eps), _hip.ptr(m), _hip.ptr(off),
                                         ctypes.c_void_p(_hip.stream_ptr(v.device))), "tnp_region")
        return m, off, output

    def normal(self, vertices: Tensor, l: int = None, h: int = None, create_graph=False,
               return_y=False) -> Tensor:
        if l is not None and h is not None and h != self.num_hidden:
            raise NotImplementedError("Net.normal: per-neuron gradients (the reference's "
                                      "l/h branch references an undefined global)")
        _hip.require_cuda(vertices, "Net.normal")
        if create_graph:
            # J with a graph (the reference's create_graph=True): differentiable
            # w.r.t. the parameters and the points (_Normal's double backward)
            if not vertices.requires_grad:
                vertices.requires_grad_(True)
            with torch.enable_grad():
                J, y = _Normal.apply(self, vertices, *self._params())
            return (J, y) if return_y else J
        s, keep = self.tnp_desc()
        x = vertices.detach().float().contiguous()
        y = torch.empty(x.shape[0], device=x.device)
        J = torch.empty(x.shape[0], 3, device=x.device)
        _hip.check(_hip.lib().tnp_sdf_grad(ctypes.byref(s), _hip.ptr(x), x.shape[0], _hip.ptr(y),
                                           _hip.ptr(J), ctypes.c_void_p(_hip.stream_ptr(x.device))),
                   "tnp_sdf_grad")
        return (J, y.unsqueeze(-1)) if return_y else J
