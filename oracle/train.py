"""ORACLE (test infrastructure only) -- PyTorch-CPU restatement of the
reference's SDF training loss and its parameter gradients
(tropical/stanford/train.py:181-203; Net.sdf = tanh(o1 - o0),
tropical/stanford/model.py:84-87) and of the dataset's mesh signed distance
(tropical/stanford/dataset.py:80-96, cubvh signed_distance).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product path never does.

The reference takes the eikonal term's gradient by double backward through
tcnn (train.py:196, ``create_graph=True``).  tinycudann is absent and
unpinned, so that arithmetic is **parity unpinned**; this module pins the
mathematics instead: the encoding forward of oracle/encoding.py restated
with differentiable gathers (cell corners and hash indices from the fp32
positions, as the kernel), evaluated in float64 with autograd's double
backward.  cubvh is absent too: the signed distance here is the exact
closest-triangle distance with the winding-number sign (inside positive,
dataset.py:96), in float64.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle.encoding import _corner_index


def encode_diff(x01: torch.Tensor, params: torch.Tensor, meta, F: int = 2) -> torch.Tensor:
    """Differentiable Grid/Hash encoding of x01 (N x 3 in [0, 1], float64 with
    grad): cells and indices from the fp32 positions, weights in float64."""
    scales, res, sizes, offsets, dense, _ = meta
    P = params.view(-1, F)
    cols = []
    for l in range(len(scales)):
        s32 = np.float32(scales[l])
        pos32 = x01.detach().float() * torch.tensor(s32) + 0.5
        g = torch.floor(pos32)
        t = x01 * float(s32) + 0.5 - g.double()
        gi = g.to(torch.int64)
        acc = 0.0
        for c in range(8):
            w = torch.ones_like(t[:, 0])
            gc = gi.clone()
            for d in range(3):
                if (c >> d) & 1:
                    w = w * t[:, d]
                    gc[:, d] += 1
                else:
                    w = w * (1 - t[:, d])
            idx = _corner_index(gc, res[l], sizes[l], dense[l]) + offsets[l]
            acc = acc + w[:, None] * P[idx]
        cols.append(acc)
    return torch.cat(cols, 1)


def sdf64(table, weights, meta, x):
    """Net.sdf (model.py:84-88) in float64 with autograd through the
    encoding (encode_diff), the MLP and tanh: the checker of the product's
    autograd (tnp_sdf_grad / tnp_sdf_vjp)."""
    h = encode_diff((x + 1) / 2, table, meta)
    n = len(weights) // 2
    for i in range(n):
        h = torch.nn.functional.linear(h, weights[2 * i], weights[2 * i + 1])
        if i < n - 1:
            h = torch.relu(h)
    return torch.tanh(h[:, 1] - h[:, 0])


def train_loss_grads(table, weights, meta, x, gt, clamp_t=0.2, eik_w=1e-2, batch_size=None):
    """(l1, eik, grads) of one batch: the L1 and eikonal terms of
    train.py:181-197 and their gradients w.r.t. the table and the fc
    parameters [W0, b0, W1, b1, W2, b2] (the weight-norm term,
    train.py:200-201, is left out: it does not involve the data)."""
    tab = table.detach().double().clone().requires_grad_(True)
    ws = [w.detach().double().clone().requires_grad_(True) for w in weights]
    x = x.detach().double().clone().requires_grad_(True)
    gt = gt.detach().double()

    def sdf(p):
        h = encode_diff((p + 1) / 2, tab, meta)
        n = len(ws) // 2
        for i in range(n):
            h = torch.nn.functional.linear(h, ws[2 * i], ws[2 * i + 1])
            if i < n - 1:
                h = torch.relu(h)
        return torch.tanh(h[:, 1] - h[:, 0])

    y = sdf(x)
    l1 = (torch.clamp(y, -clamp_t, clamp_t) - torch.clamp(gt, -clamp_t, clamp_t)).abs().mean()
    J = torch.autograd.grad(y.sum(), x, create_graph=True)[0]
    # train.py:197 divides by the BATCH_SIZE constant (the L1 mean by the actual batch)
    eik = eik_w * (J.norm(p=2) - 1).pow(2) / (x.shape[0] if batch_size is None else batch_size)
    grads = torch.autograd.grad(l1 + eik, [tab] + ws)
    return l1.detach(), eik.detach(), grads


def weight_norm_loss(weights):
    """train.py:200-201 on [W0, W1, W2]."""
    return 1e-1 * sum((1 - w.norm(p=2, dim=1)).pow(2).mean() for w in weights) / len(weights)


def _closest_dist2(p, a, b, c):
    """Squared distance from points p (N x 3) to triangle (a, b, c), float64,
    by minimising over the triangle's face, edges and vertices."""
    ab, ac = b - a, c - a
    n = np.cross(ab, ac)
    nn = np.dot(n, n)
    best = np.full(len(p), np.inf)
    if nn > 0:
        ap = p - a
        # barycentric projection onto the plane
        v = np.dot(np.cross(ap, ac), n) / nn
        w = np.dot(np.cross(ab, ap), n) / nn
        inside = (v >= 0) & (w >= 0) & (v + w <= 1)
        proj = a + v[:, None] * ab + w[:, None] * ac
        d = ((p - proj) ** 2).sum(1)
        best = np.where(inside, d, best)
    for u, q in ((a, b), (b, c), (c, a)):
        e = q - u
        ee = np.dot(e, e)
        t = np.clip(((p - u) @ e) / ee, 0, 1) if ee > 0 else np.zeros(len(p))
        d = ((p - (u + t[:, None] * e)) ** 2).sum(1)
        best = np.minimum(best, d)
    return best


def signed_distance(V: np.ndarray, F: np.ndarray, P: np.ndarray) -> np.ndarray:
    """Exact signed distance (inside positive) of points P to the closed
    mesh (V, F), float64 brute force -- for small meshes only."""
    V, P = V.astype(np.float64), P.astype(np.float64)
    d2 = np.full(len(P), np.inf)
    wind = np.zeros(len(P))
    for f in F:
        a, b, c = V[f[0]], V[f[1]], V[f[2]]
        d2 = np.minimum(d2, _closest_dist2(P, a, b, c))
        u, v, w = a - P, b - P, c - P
        lu, lv, lw = (np.linalg.norm(q, axis=1) for q in (u, v, w))
        det = np.einsum("ij,ij->i", u, np.cross(v, w))
        den = lu * lv * lw + (u * v).sum(1) * lw + (u * w).sum(1) * lv + (v * w).sum(1) * lu
        wind += 2 * np.arctan2(det, den) / (4 * np.pi)
    d = np.sqrt(d2)
    return np.where(np.abs(wind) > 0.5, d, -d), wind
