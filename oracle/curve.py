"""ORACLE (test infrastructure only) -- PyTorch-CPU restatement of the
reference's curve-approximation branch (``subpoly_(..., force=False)``).

Only ``tests/`` and the checker legs of ``bench.py`` / ``smoke()`` import
this.  Same op sequence as the reference, so that on the golden-generating
host it reproduces the reference bit for bit (tests/test_oracle_golden.py):

* ``corner_points``          tropical/geometry.py:350-372
* ``plane_intersection``     tropical/geometry.py:24-138 ("xz" assumption;
                             bilinear cells marked -1 as the reference's
                             ``failover = False`` branch does)
* ``polynomial_roots``       tropical/geometry.py:259-299 (companion-matrix
                             eigenvalues, last real root in [0, 1])
* ``last_nonzero``           tropical/torch_ext.py:18-29 (vectorised)
* ``descend``                tropical/subpoly_debug.py:121-165
* ``strict_keep``            tropical/subpoly_debug.py:234-271
* ``curve_vertices``         tropical/subpoly.py:120-177, 204-207
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

ROOT_EPS = 1e-9  # geometry.py:259, 271


def corner_points(ends: torch.Tensor) -> torch.Tensor:
    """B x 2 x 3 edge endpoints -> B x 8 x 3 box corners; corner
    4i + 2j + k takes x from endpoint k, y from j, z from i."""
    out = []
    for i in range(2):
        for j in range(2):
            for k in range(2):
                sel = ends.new_zeros(1, 2, 3)
                sel[0, k, 0] = 1
                sel[0, j, 1] = 1
                sel[0, i, 2] = 1
                out.append((ends * sel).sum(dim=1, keepdim=True))
    return torch.cat(out, dim=1)


def last_nonzero(mask: torch.Tensor) -> torch.Tensor:
    """(row, last nonzero column) for every row with a nonzero, in row order."""
    rows = mask.any(-1).nonzero()[:, 0]
    cols = mask.shape[1] - 1 - mask.flip(-1).float().argmax(-1)
    return torch.stack([rows, cols[rows]], -1)


def _companion_roots(c: torch.Tensor) -> torch.Tensor:
    """Rows of c = [a_0 .. a_N] (a_0 leading, non-zero): last real eigenvalue
    in [0, 1] of the companion matrix, -1 if none (geometry.py:271-299)."""
    c = torch.flip(c, [1])
    N = c.shape[1] - 1
    valid = c.abs().mean(-1) > ROOT_EPS
    cv = c[valid]
    C = c.new_zeros(cv.shape[0], N, N)
    for i in range(N - 1):
        C[:, i, i + 1] = 1
    lead = last_nonzero(cv.abs() > ROOT_EPS)
    assert lead.shape[0] == cv.shape[0]
    C[:, -1] = -cv[:, :-1] / cv.gather(1, lead[:, 1:])
    ev = torch.linalg.eigvals(C)
    ok = (ev.imag.abs() <= ROOT_EPS) & (ev.real >= 0) & (ev.real <= 1)
    pick = last_nonzero(ok)
    has = ok.sum(-1) > 0
    out = c.new_full((c.shape[0],), -1.0)
    sel = valid.clone()
    sel[valid] = has
    out[sel] = ev[has].real.gather(1, pick[:, 1:]).squeeze()
    return out


def polynomial_roots(coeffs: torch.Tensor) -> torch.Tensor:
    """geometry.py:259-268: tiny coefficients zeroed in place, then the degree
    is set by the first non-zero coefficient."""
    coeffs[coeffs.abs() < ROOT_EPS] = 0
    roots = coeffs.new_full((coeffs.shape[0],), -1.0)
    for i in range(coeffs.shape[1] - 1):
        m = (coeffs[:, :i].abs().sum(-1) <= ROOT_EPS) & (coeffs[:, i].abs() > ROOT_EPS)
        roots[m] = _companion_roots(coeffs[m][:, i:])
    return roots


_T = [[1.0, -2.0, 1.0], [-1.0, 1.0, 0.0], [1.0, 0.0, 0.0]]
_LO = [0, 1, 4, 5]
_HI = [2, 3, 6, 7]


def _fold3(v):  # [v0, v1 + v2, v3]
    return torch.stack([v[:, 0], v[:, 1] + v[:, 2], v[:, 3]], dim=-1)


def plane_intersection(p: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """B x 8 corner values of the edge plane p and the current plane q ->
    B x 3 box parameters (x, y, x) of their intersection on the box's xz
    diagonal plane (geometry.py:24-73); -1 rows where both planes are
    bilinear in one of xz / xy / yz (geometry.py:110-136)."""
    T = p.new_tensor([_T])
    lo, hi = p.new_tensor(_LO).long(), p.new_tensor(_HI).long()
    A = _fold3(q[:, lo]).unsqueeze(2) * _fold3(p[:, hi]).unsqueeze(1) \
        - _fold3(q[:, hi]).unsqueeze(2) * _fold3(p[:, lo]).unsqueeze(1)
    B = T.transpose(1, 2) @ A @ T
    coeffs = torch.stack([B[:, 0, 0], B[:, 1, 0] + B[:, 0, 1],
                          B[:, 2, 0] + B[:, 1, 1] + B[:, 0, 2],
                          B[:, 1, 2] + B[:, 2, 1], B[:, 2, 2]], dim=-1)
    x = polynomial_roots(coeffs)
    z = x.clone()
    X = torch.stack([(1 - x) ** 2, x * (1 - x), x * (1 - x), x ** 2], dim=-1)
    a = (q[:, lo] * X).sum(-1)
    b = (q[:, hi] * X).sum(-1)
    y = a / (a - b)
    for t, u in (([0, 1, 4, 5], [2, 3, 6, 7]), ([0, 1, 2, 3], [4, 5, 6, 7]),
                 ([0, 4, 2, 6], [1, 5, 3, 7])):
        t, u = p.new_tensor(t).long(), p.new_tensor(u).long()
        flat = ((p[:, t] == p[:, u]) & (q[:, t] == q[:, u])).sum(-1) == 4
        x[flat] = -1
        y[flat] = -1
        z[flat] = -1
    return torch.stack([x, y, z], dim=-1)


def descend(net, ends, x, plane, idx, eps, iters=500, step=1e-2):
    """subpoly_debug.py:121-165 on the rows given: normalised gradient descent
    of d_plane^2 + d_idx^2 over the box parameters, clamped to [0, 1];
    all rows stop together (max over rows).  Returns (x after the last
    update, the distances evaluated before it)."""
    x = x.clone()
    x.requires_grad = True
    d0 = d1 = torch.tensor(1.0)
    i = 0
    with torch.enable_grad():
        while ((d0.abs().max() > eps) | (d1.abs().max() > eps)) and i < iters:
            pts = ends[:, 0] + x * (ends[:, 1] - ends[:, 0])
            out = torch.cat(net(pts, gather=True)[1], dim=-1)
            d0 = out.gather(-1, plane.view(-1, 1)).squeeze(1)
            d1 = out[:, idx]
            y = (d0.pow(2) + d1.pow(2)).sum()
            x.data -= step * F.normalize(torch.autograd.grad(y, x)[0])
            x.data.clamp_(0, 1)
            i += 1
    return x.detach(), d0.detach(), d1.detach(), i


def curve_vertices(V, E, split, cache, rgn, net, idx, eps, stats=None, off=None):
    """subpoly.py:120-177, 204-207: new vertices of the split edges with the
    trilinear correction on non-axis-aligned edges.  Returns
    (v_new S x 3, c mask S, ints B x 3, d_new B x 2)."""
    ds = cache[:, idx][E][split] / eps
    ends = V[E][split]
    w = ds[:, :1].abs() / (ds[:, 1:] - ds[:, :1]).abs()
    c = 1 < ((ends[:, 1, :] - ends[:, 0, :]).abs() > eps).sum(dim=-1)
    B = int(c.sum())
    v_new = ends[:, 0] * (1 - w) + ends[:, 1] * w
    if B == 0:
        return v_new, c, ends.new_empty(0, 3), ends.new_zeros(1, 2), None
    corners = corner_points(ends[c]).view(-1, 3)
    dc = torch.cat(net(corners, gather=True, group=8)[1], dim=-1)
    dc = dc.view(-1, 8, dc.shape[-1])
    if off is not None:
        # check_new_vertices_on_two_planes (subpoly.py:134-135,
        # subpoly_debug.py:96-104): fewer than two shared zero columns -> the
        # reference's diagnostic print raises (Tensor has no .astype)
        ar, ao = rgn[E][split][c], off[E][split][c]
        chk = (ar[:, 0] == 0) & (ar[:, 1] == 0)
        chk[:, :3] &= ao[:, 0] == ao[:, 1]
        if bool((chk.sum(-1) < 2).any()):
            raise AttributeError(f"curve path, plane {idx}: a split edge's endpoints share fewer than two "
                                 "zero columns (reference subpoly_debug.py:96-104 fails on Tensor.astype)")
    er = rgn[E][split][c][:, :, 3:]
    both_zero = (er[:, 0] == 0) & (er[:, 1] == 0)
    plane = last_nonzero(both_zero[:, :idx])
    if plane.shape[0] != B:
        raise RuntimeError(f"curve path: {B - plane.shape[0]} split edges share no plane below "
                           f"{idx} (the reference prints them and exit()s, subpoly.py:141-148)")
    plane = plane[:, 1]
    p = dc.gather(-1, plane.view(-1, 1, 1).repeat(1, 8, 1)).squeeze(-1)
    q = dc[:, :, idx]
    ints = plane_intersection(p, q)
    ec = ends[c]
    _, _, out = net.region(ec[:, 0] * (1 - ints) + ec[:, 1] * ints)
    d_new = torch.stack([out.gather(-1, plane.view(-1, 1)).squeeze(1), out[:, idx]], dim=-1)
    gg = 0 < ((ints < 0) | (ints > 1)).sum(-1)
    gd = ~gg & (0 < (d_new.abs() > eps).sum(dim=-1))
    n_iter = 0
    if int(gd.sum()) > 0:
        xg, d0, d1, n_iter = descend(net, ec[gd], ints[gd], plane[gd], idx, eps)
        ints[gd] = xg
        d_new[gd, 0] = d0
        d_new[gd, 1] = d1
    if stats is not None:
        stats.update(B=B, gg=int(gg.sum()), gd=int(gd.sum()), gd_iters=n_iter)
    v_new[c] = ec[:, 0] + ints * (ec[:, 1] - ec[:, 0])
    return v_new, c, ints, d_new, gg


def strict_keep(pre_new, c, ints, d_new, gg, idx, eps):
    """subpoly_debug.py:234-271: which new vertices survive (S bool)."""
    chk = pre_new[:, idx]
    B = ints.shape[0]
    keep = chk.abs() < eps
    if not ((chk.abs().max() >= eps) | (d_new[:, 0].abs().max() >= eps) | (B > 0)):
        return torch.ones_like(keep)
    if B > 0:
        d_new[:, 0][gg] = 0
    tight = bool(eps < d_new[:, 0].abs().max())
    if B > 0:
        kc = (chk[c].abs() < eps) & ~gg
        if tight:
            kc &= d_new[:, 0].abs() < eps
        keep[c] = kc
    return keep
