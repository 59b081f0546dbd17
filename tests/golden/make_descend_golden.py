"""Descent fixtures: the oracle's deal_with_gradient_descent (oracle/curve.py
descend -- torch autograd on CPU, i.e. the reference's backward schedules,
subpoly_debug.py:121-165) on random rows of every shape family, computed
in the build container (the host of every other golden) and stored for the
GPU test (tests/test_gpu_curve.py test_descend_matches_golden): the box's
own CPU may run other BLAS kernels.

    python tests/golden/make_descend_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tropical-nerf.pytorch_amd")]

import oracle.curve as oc  # noqa: E402
import oracle.subdivide as od  # noqa: E402
from tropical.synthetic import random_params  # noqa: E402
from tropical.tropical import level_meta  # noqa: E402

SHAPES = [dict(num_layers=3, num_hidden=16, levels=4, r_min=2, r_max=32, T=19),
          dict(num_layers=3, num_hidden=8, levels=3, r_min=2, r_max=24, T=19),
          dict(num_layers=2, num_hidden=32, levels=4, r_min=2, r_max=32, T=19),
          dict(num_layers=4, num_hidden=8, levels=5, r_min=2, r_max=32, T=19),
          dict(num_layers=4, num_hidden=16, levels=8, r_min=4, r_max=64, T=13)]
ROWS = [1, 5, 20]
KEYS = ("num_layers", "num_hidden", "levels", "r_min", "r_max", "T")


def main():
    torch.set_num_threads(1)
    out = {}
    for si, cfg in enumerate(SHAPES):
        b = np.exp2(np.log2(cfg["r_max"] / cfg["r_min"]) / (cfg["levels"] - 1))
        n_params = level_meta(cfg["levels"], cfg["r_min"], b, cfg["T"])[-1] * 2
        nodes = [cfg["levels"] * 2] + [cfg["num_hidden"]] * (cfg["num_layers"] - 1) + [2]
        for rows in ROWS:
            seed = 61 + rows
            p = random_params(n_params, nodes, seed, 0.1)
            ref = od.load_params(od.RefNet(**cfg), p)
            K = (cfg["num_layers"] - 1) * cfg["num_hidden"] + 1
            rng = np.random.default_rng(rows * 7 + cfg["num_hidden"] + 100 * si)
            e0 = rng.uniform(-0.8, 0.8, (rows, 3)).astype(np.float32)
            ends = np.stack([e0, e0 + rng.uniform(-0.05, 0.05, (rows, 3)).astype(np.float32)], axis=1)
            x0 = rng.uniform(0, 1, (rows, 3)).astype(np.float32)
            idx = int(rng.integers(1, K))
            plane = rng.integers(0, idx, rows).astype(np.int64)
            x, d0, d1, it = oc.descend(ref, torch.from_numpy(ends), torch.from_numpy(x0), torch.from_numpy(plane),
                                       idx, 1e-4, iters=40)
            key = f"s{si}_r{rows}"
            out[key + ":cfg"] = np.array([cfg[k] for k in KEYS], dtype=np.int64)
            out[key + ":gen"] = np.array([seed, 0.1])
            out[key + ":ends"] = ends
            out[key + ":x0"] = x0
            out[key + ":plane"] = plane.astype(np.int32)
            out[key + ":idx_it"] = np.array([idx, it], dtype=np.int64)
            out[key + ":x"] = x.numpy()
            out[key + ":d"] = np.stack([d0.numpy(), d1.numpy()])
            print(key, cfg, "idx", idx, "iters", it, flush=True)
    np.savez_compressed(os.path.join(HERE, "descend_cases.npz"), **out)


if __name__ == "__main__":
    main()
