#!/usr/bin/env python3
"""Bunny-scale latency breakdown of the drop-in subpoly() on one GPU.

    python tools/small_profile.py [reps] [flat|curve]

For the committed stand-in small nets (small_sphere flat, small_sphere_curve
curve-approx on): median wall time of each phase (skeleton, the hyperplane
loop, surface + export + faces) over `reps` runs, the number of active steps,
and the engine's HIP-event kernel times summed per kernel over one run (the
difference to the loop's wall time is host turnaround: launches and the
per-step counter readbacks)."""
import contextlib
import io
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tropical-nerf.pytorch_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2] if len(sys.argv) > 2 else None  # "flat" | "curve"
    from golden_io import load
    from helpers import product_net
    import tropical.subpoly as sp
    from tropical._engine import engine_for
    dev = torch.device("cuda", 0)
    for name, force in (("small_sphere", True), ("small_sphere_curve", False)):
        if only and only != ("flat" if force else "curve"):
            continue
        d = load(name)
        net = product_net(d, dev)
        ph = {"skeleton": [], "loop": [], "finish": [], "total": []}
        nsteps = 0
        for r in range(reps + 1):
            with contextlib.redirect_stdout(io.StringIO()):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                eng = engine_for(net).set_curve(not force)
                eng.skeleton(unit=128, size=1.2)
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                st = []
                eng.run_steps(st)
                torch.cuda.synchronize(dev)
                t2 = time.perf_counter()
                sp._finish(eng, net)
                torch.cuda.synchronize(dev)
                t3 = time.perf_counter()
            if r == 0:
                continue  # warm
            nsteps = len(st)
            for k, v in (("skeleton", t1 - t0), ("loop", t2 - t1), ("finish", t3 - t2), ("total", t3 - t0)):
                ph[k].append(v * 1e3)
        # kernel times of one loop
        eng = engine_for(net).set_curve(not force)
        eng.skeleton(unit=128, size=1.2)
        eng.kernel_timer(True)
        st = []
        eng.run_steps(st)
        kt = eng.kernel_timer(False)
        ksum = sum(v["ms"] for v in kt.values())
        S = sum(s["S"] for s in st)
        out = {"net": name, "force": force, "active_steps": nsteps, "splits": int(S),
               "median_ms": {k: round(statistics.median(v), 3) for k, v in ph.items()},
               "loop_kernel_ms": round(ksum, 3),
               "kernels": {k: [round(v["ms"], 3), v["launches"]] for k, v in
                           sorted(kt.items(), key=lambda kv: -kv[1]["ms"])}}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
