#!/usr/bin/env python3
"""Bunny-scale breakdown of subpoly()'s finish (surface -> export -> faces ->
host arrays) on one GPU: median wall time of each call over `reps` runs of
the stand-in small net, plus the engine's kernel timers over one finish.

    python tools/finish_profile.py [reps]"""
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
    from golden_io import load
    from helpers import product_net
    import tropical.subpoly as sp
    from tropical._engine import engine_for
    dev = torch.device("cuda", 0)
    d = load("small_sphere")
    net = product_net(d, dev)
    ph = {}
    kt = None
    for r in range(reps + 1):
        with contextlib.redirect_stdout(io.StringIO()):
            eng = engine_for(net).set_curve(False)
            eng.skeleton(unit=128, size=1.2)
            eng.run_steps([])
            torch.cuda.synchronize(dev)
            if r == reps:
                eng.kernel_timer(True)
            t = [time.perf_counter()]
            eng.sizes()
            t.append(time.perf_counter())
            eng.surface()
            torch.cuda.synchronize(dev)
            t.append(time.perf_counter())
            eng.export()
            torch.cuda.synchronize(dev)
            t.append(time.perf_counter())
            tri, fc = eng.faces(host=True)
            torch.cuda.synchronize(dev)
            t.append(time.perf_counter())
            sp._faces_to_numpy(tri, fc)
            t.append(time.perf_counter())
            if r == reps:
                kt = eng.kernel_timer(False)
        if r == 0:
            continue
        for k, (a, b) in zip(("sizes", "surface", "export", "faces", "to_host"), zip(t, t[1:])):
            ph.setdefault(k, []).append((b - a) * 1e3)
    out = {"median_ms": {k: round(statistics.median(v), 3) for k, v in ph.items()},
           "kernels": {k: [round(v["ms"], 3), v["launches"]] for k, v in
                       sorted((kt or {}).items(), key=lambda kv: -kv[1]["ms"])}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
