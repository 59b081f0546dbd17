"""Diagnostic (GPU box): where the HIP descent (tnp_debug_descend) first
departs from the oracle's torch-autograd descent on a descend_cases.npz
fixture.  Runs the oracle loop on CPU iteration by iteration and the HIP
descent for 1, 2, ... iterations from the same start; prints the first
iteration whose x differs, with the distances and gradients of that step.

    python tools/descend_diag.py s3_r1 [s1_r5 ...]
"""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tropical-nerf.pytorch_amd"), os.path.join(REPO, "tests")]

from golden_io import GOLDEN  # noqa: E402
import oracle.subdivide as od  # noqa: E402
try:
    from tropical import _hip  # noqa: E402
except Exception:  # (--save runs without the library)
    _hip = None
from tropical.stanford.model import Net  # noqa: E402
from tropical.synthetic import random_params  # noqa: E402
from tropical.tropical import level_meta  # noqa: E402


def case(name):
    with np.load(os.path.join(GOLDEN, "descend_cases.npz"), allow_pickle=False) as z:
        g = {k.split(":")[1]: z[k] for k in z.files if k.startswith(name + ":")}
    cfg = dict(zip(("num_layers", "num_hidden", "levels", "r_min", "r_max", "T"), (int(v) for v in g["cfg"])))
    b = np.exp2(np.log2(cfg["r_max"] / cfg["r_min"]) / (cfg["levels"] - 1))
    n_params = level_meta(cfg["levels"], cfg["r_min"], b, cfg["T"])[-1] * 2
    nodes = [cfg["levels"] * 2] + [cfg["num_hidden"]] * (cfg["num_layers"] - 1) + [2]
    p = random_params(n_params, nodes, int(g["gen"][0]), float(g["gen"][1]))
    return g, cfg, p


def oracle_steps(ref, ends, x0, plane, idx, iters, step=1e-2):
    """oracle/curve.py descend, one record per iteration: (x after, d0, d1, grad)."""
    x = x0.clone()
    x.requires_grad = True
    out_rec = []
    with torch.enable_grad():
        for _ in range(iters):
            pts = ends[:, 0] + x * (ends[:, 1] - ends[:, 0])
            out = torch.cat(ref(pts, gather=True)[1], dim=-1)
            d0 = out.gather(-1, plane.view(-1, 1)).squeeze(1)
            d1 = out[:, idx]
            y = (d0.pow(2) + d1.pow(2)).sum()
            gr = torch.autograd.grad(y, x)[0]
            x.data -= step * F.normalize(gr)
            x.data.clamp_(0, 1)
            out_rec.append((x.detach().clone(), d0.detach().clone(), d1.detach().clone(), gr.clone()))
    return out_rec


def main(names):
    dev = torch.device("cuda", 0)
    for name in names:
        g, cfg, p = case(name)
        ref = od.load_params(od.RefNet(**cfg), p)
        net = Net(**cfg)
        net.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in p.items()})
        net = net.to(dev)
        rows = g["x0"].shape[0]
        idx, it = (int(v) for v in g["idx_it"])
        ends = torch.from_numpy(g["ends"])
        plane = torch.from_numpy(g["plane"]).long()
        traj = os.path.join(REPO, "gpurun_traj.npz")  # trajectories made where the fixture was (--save)
        if os.path.exists(traj):
            with np.load(traj, allow_pickle=False) as z:
                rec = [tuple(torch.from_numpy(z[f"{name}:{k}:{q}"]) for q in ("x", "d0", "d1", "g")) for k in range(it)]
        else:
            rec = oracle_steps(ref, ends, torch.from_numpy(g["x0"]), plane, idx, it)
        s, keep = net.tnp_desc()
        de = ends.reshape(-1, 3).contiguous().to(dev)
        pl = torch.from_numpy(g["plane"]).to(dev)
        print(f"== {name} {cfg} rows {rows} idx {idx} iters {it}; oracle final == golden:",
              bool(torch.equal(rec[-1][0], torch.from_numpy(g["x"]))))
        for k in range(1, it + 1):
            x = torch.from_numpy(g["x0"]).to(dev)
            d0 = torch.empty(rows, device=dev)
            d1 = torch.empty(rows, device=dev)
            _hip.check(_hip.lib().tnp_debug_descend(ctypes.byref(s), _hip.ptr(de), _hip.ptr(x), _hip.ptr(pl), rows,
                                                    idx, 1e-4, k, _hip.ptr(d0), _hip.ptr(d1), 1,
                                                    ctypes.c_void_p(_hip.stream_ptr(dev))), "tnp_debug_descend")
            xg, d0g, d1g = x.cpu(), d0.cpu(), d1.cpu()
            xc, d0c, d1c, gr = rec[k - 1]
            if not (torch.equal(xg, xc) and torch.equal(d0g, d0c) and torch.equal(d1g, d1c)):
                bad = torch.nonzero((xg != xc).any(1) | (d0g != d0c) | (d1g != d1c)).flatten().tolist()
                print(f"  first difference at iteration {k}, rows {bad[:8]}")
                xp = rec[k - 2][0] if k > 1 else torch.from_numpy(g["x0"])
                for r in bad[:3]:
                    print(f"   row {r}: x_prev {xp[r].tolist()}")
                    print(f"     gpu x {xg[r].tolist()} d0 {d0g[r].item()!r} d1 {d1g[r].item()!r}")
                    print(f"     cpu x {xc[r].tolist()} d0 {d0c[r].item()!r} d1 {d1c[r].item()!r}")
                    print(f"     cpu grad {gr[r].tolist()} normalized {F.normalize(gr)[r].tolist()}")
                    print(f"     gpu step/1e-2 {((xp[r] - xg[r]) / 1e-2).tolist()}")
                break
        else:
            print("  no difference")


def save(names):
    """Record the oracle trajectories on this host (the fixture's) for a GPU run."""
    out = {}
    for name in names:
        g, cfg, p = case(name)
        ref = od.load_params(od.RefNet(**cfg), p)
        idx, it = (int(v) for v in g["idx_it"])
        rec = oracle_steps(ref, torch.from_numpy(g["ends"]), torch.from_numpy(g["x0"]),
                           torch.from_numpy(g["plane"]).long(), idx, it)
        assert torch.equal(rec[-1][0], torch.from_numpy(g["x"])), name
        for k, r in enumerate(rec):
            for q, v in zip(("x", "d0", "d1", "g"), r):
                out[f"{name}:{k}:{q}"] = v.numpy()
    np.savez(os.path.join(REPO, "gpurun_traj.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--save"]:
        save(sys.argv[2:])
    else:
        main(sys.argv[1:])
