"""SDF training on the MI355X path: the optimisation step of the reference's
training loop (tropical/stanford/train.py:86-90, 177-205) and the mesh
signed distance its dataset samples (dataset.py:77, 92).

The batch gradient of the data terms -- L1 on clamped SDFs and the eikonal
term, whose parameter gradient the reference gets by double backward
through tcnn -- is one C-ABI call (``tnp_sdf_train_grad``, csrc/train.hip,
closed form); the weight-norm term (train.py:200-201) only involves the fc
weights and is added here.  Adam and the cosine schedule are the
reference's own torch.optim objects over the net's parameters.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _hip

CLAMP = 0.2      # train.py:184-185 (minT, maxT)
EIK_W = 1e-2     # train.py:197
BATCH_SIZE = 1000  # train.py:66: the eikonal term's divisor (train.py:197), whatever the batch length
WN_W = 1e-1      # train.py:200


def _weights(net):
    return [t for lin in net.fc for t in (lin.weight, lin.bias)]


class SDFTrainer:
    """Adam(lr) + CosineAnnealingLR(T_max) over ``net.parameters()``
    (train.py:86-90); ``step(x, gt)`` is one iteration of train.py:177-205."""

    def __init__(self, net, lr: float = 1e-3, T_max: float = 500.0, batch_size: int = BATCH_SIZE):
        self.net = net
        self.batch_size = int(batch_size)
        self.opt = torch.optim.Adam(net.parameters(), lr=lr)
        self.sched = torch.optim.lr_scheduler.CosineAnnealingLR(self.opt, T_max)
        dev = net.device()
        params = net.enc.module.params
        self.g_table = torch.zeros_like(params, dtype=torch.float32)
        self.g_w = torch.zeros(sum(t.numel() for t in _weights(net)), dtype=torch.float32, device=dev)
        self.stats = torch.zeros(2, dtype=torch.float64, device=dev)

    def data_grads(self, x, gt):
        """Gradients of the L1 + eikonal terms of one batch into the
        trainer's buffers; returns (l1, eik) as device scalars."""
        net = self.net
        _hip.require_cuda(x, "SDFTrainer")
        x = x.detach().float().contiguous()
        gt = gt.detach().float().contiguous().reshape(-1)
        if x.shape[0] != gt.shape[0]:
            raise ValueError("SDFTrainer: inputs and labels differ in length")
        self.g_table.zero_()
        self.g_w.zero_()
        s, keep = net.tnp_desc()
        _hip.check(_hip.lib().tnp_sdf_train_grad(
            ctypes.byref(s), _hip.ptr(x), _hip.ptr(gt), x.shape[0], CLAMP, EIK_W, self.batch_size,
            _hip.ptr(self.g_table),
            _hip.ptr(self.g_w), _hip.ptr(self.stats), ctypes.c_void_p(_hip.stream_ptr(x.device))),
            "tnp_sdf_train_grad")
        del keep
        n = max(x.shape[0], 1)
        l1 = self.stats[0] / n  # nn.L1Loss: the mean over the actual batch
        eik = EIK_W * (self.stats[1].sqrt() - 1) ** 2 / self.batch_size
        return l1.float(), eik.float()

    def step(self, x, gt):
        """zero_grad, gradients of every loss term, Adam step, schedule step
        (train.py:178-205); returns (loss, l1) as device scalars."""
        net = self.net
        self.opt.zero_grad(set_to_none=False)
        l1, eik = self.data_grads(x, gt)
        params = net.enc.module.params
        params.grad = self.g_table.clone() if params.grad is None else params.grad.copy_(self.g_table)
        off = 0
        for t in _weights(net):
            g = self.g_w[off:off + t.numel()].view_as(t)
            off += t.numel()
            t.grad = g.clone() if t.grad is None else t.grad.copy_(g)
        # weight-norm term: d/dW_r of WN_W/L * mean_r (1 - |W_r|)^2
        wn = 0.0
        L = len(net.fc)
        for lin in net.fc:
            W = lin.weight.detach()
            nr = W.norm(p=2, dim=1, keepdim=True)
            wn = wn + (1 - nr).pow(2).mean()
            coef = WN_W / L * 2 * (nr - 1) / (W.shape[0] * nr.clamp_min(1e-30))
            lin.weight.grad.add_(coef * W)
        wn = WN_W * wn / L
        self.opt.step()
        self.sched.step()
        return l1 + eik + wn, l1


def mesh_signed_distance(V: torch.Tensor, F: torch.Tensor, P: torch.Tensor) -> torch.Tensor:
    """Signed distance (inside positive) of points P to the closed mesh
    (V, F) on the GPU -- cubvh.cuBVH(V, F).signed_distance(P)[0]
    (dataset.py:77, 92)."""
    for t, w in ((V, "V"), (F, "F"), (P, "P")):
        _hip.require_cuda(t, f"mesh_signed_distance({w})")
    V = V.detach().float().contiguous()
    F = F.detach().to(torch.int32).contiguous()
    P = P.detach().float().contiguous()
    if F.numel() and (int(F.min()) < 0 or int(F.max()) >= V.shape[0]):
        raise ValueError("mesh_signed_distance: face index out of range")
    out = torch.empty(P.shape[0], device=P.device)
    work = torch.empty(2 * P.shape[0], device=P.device)
    _hip.check(_hip.lib().tnp_mesh_signed_distance(
        _hip.ptr(V), V.shape[0], _hip.ptr(F), F.shape[0], _hip.ptr(P), P.shape[0], _hip.ptr(work),
        _hip.ptr(out), ctypes.c_void_p(_hip.stream_ptr(P.device))), "tnp_mesh_signed_distance")
    return out
