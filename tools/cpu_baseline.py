"""The CPU baseline alone, at a chosen lattice size (BASELINE.md §3's 64^3
fallback; the default bench line keeps the bounded 48^3 sample):
    python tools/cpu_baseline.py [G] [seed]
prints one JSON line: the oracle (PyTorch-CPU restatement of the reference)
on the whole G^3 lattice on the host's cores, and the GPU engine on the same
workload (equal split counts asserted)."""
import json
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"),
                os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402

import bench  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 6
thr = bench.cpu_threads()
bench.log(f"CPU baseline: the oracle on the {G}^3 lattice, {thr} threads")
cps, S_cpu, t_cpu = bench.cpu_baseline(G, seed, thr)
bench.log(f"CPU baseline: {S_cpu} splits in {t_cpu:.1f} s")
dev = torch.device("cuda", 0)
S_g, t_g = bench.gpu_same_workload(G, seed, dev)
if S_g != S_cpu:
    raise SystemExit(f"{S_cpu} splits on the host, {S_g} on the GPU")
print(json.dumps({"marks": G, "seed": seed, "cpu": bench.cpu_model(), "cores": thr, "kind": "port",
                  "cpu_edges_subdivided": S_cpu, "cpu_seconds": round(t_cpu, 2), "cpu_edges_per_s": round(cps, 1),
                  "gpu_seconds": round(t_g, 5), "gpu_edges_per_s": round(S_g / t_g, 1),
                  "gpu_over_cpu": round((S_g / t_g) / cps, 1)}), flush=True)
