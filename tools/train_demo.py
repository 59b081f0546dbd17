"""Train an SDF on a sphere scan stand-in with the reference's loop and
evaluate it (`python -m tropical.stanford.train -d bunny -c --mesh ... -e`),
timing the phases.  The Stanford scans are not in this repository; a closed
icosphere mesh (20,480 triangles, the size class of the res3 / res10 scans)
takes their place.

    python tools/train_demo.py [out_dir]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tropical-nerf.pytorch_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_train import icosphere  # noqa: E402
from tropical.stanford import sdf_train  # noqa: E402
from tropical.stanford.train import main  # noqa: E402
from tropical.utils.mesh import Mesh  # noqa: E402


def main_demo(out="gpurun_out/train_demo"):
    os.makedirs(out, exist_ok=True)
    V, F = icosphere(5, r=0.37)
    Mesh(V, F).export(os.path.join(out, "sphere.ply"))
    # per-step time of the optimisation step, measured around SDFTrainer.step
    times = []
    orig = sdf_train.SDFTrainer.step

    def timed(self, x, gt):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = orig(self, x, gt)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        return r
    sdf_train.SDFTrainer.step = timed
    t0 = time.perf_counter()
    main(["-d", "bunny", "-c", "--mesh", os.path.join(out, "sphere.ply"), "--out", os.path.join(out, "meshes"),
          "-e"])
    total = time.perf_counter() - t0
    ts = np.array(times[5:]) * 1e3
    print(f"train_demo: {len(times)} optimisation steps of 1000 points, median {np.median(ts):.3f} ms "
          f"(p90 {np.percentile(ts, 90):.3f} ms); whole command {total:.1f} s")


if __name__ == "__main__":
    main_demo(*sys.argv[1:])
