"""Kernel ms per pass (HIP events, median of 5 timed passes) of the synthetic
lattice on the GPU, for A/B runs of library variants and timing experiments:
    TNP_LIB=... python tools/kernel_ms.py [G] [seed] [tag]
prints one JSON line {tag, pass_ms, kernels: {name: ms}}."""
import json
import os
import statistics
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"),
                os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402

from bench import make_net  # noqa: E402
from tropical._engine import engine_for  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 6
tag = sys.argv[3] if len(sys.argv) > 3 else os.environ.get("TNP_LIB", "default")
dev = torch.device("cuda", 0)
net = make_net(G, dev, seed)
eng = engine_for(net)


def one_pass():
    eng.lattice()
    eng.run_steps([])


for _ in range(3):
    one_pass()
torch.cuda.synchronize()
walls, per = [], {}
for _ in range(5):
    t = time.perf_counter()
    one_pass()
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t) * 1e3)
for _ in range(5):
    eng.kernel_timer(True)
    one_pass()
    kt = eng.kernel_timer(False)
    for k, v in kt.items():
        per.setdefault(k, []).append(v["ms"])
V, E = eng.sizes()
print(json.dumps({"tag": tag, "env": {k: v for k, v in os.environ.items() if k.startswith("TNP_")},
                  "pass_ms": round(statistics.median(walls), 4), "V": V, "E": E,
                  "kernels": {k: round(statistics.median(v), 4)
                              for k, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1]))}}),
      flush=True)
