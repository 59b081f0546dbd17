"""Per-step engine stats and per-step kernel times (HIP events) for the
synthetic lattice on the GPU: python tools/step_profile.py [G] [seed]."""
import json
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"),
                os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402

from bench import make_net  # noqa: E402
from tropical._engine import engine_for  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda", 0)
net = make_net(G, dev, seed)
eng = engine_for(net)
def full_pass():
    try:
        eng.lattice()
        eng.run_steps([])
    except RuntimeError as ex:  # TNP_EXP timing runs compute wrong values
        print("pass stopped:", ex)


for _ in range(2):  # warm (capacities)
    full_pass()
torch.cuda.synchronize()
t = time.time()
full_pass()
torch.cuda.synchronize()
print("wall pass ms", round((time.time() - t) * 1e3, 3))
t = time.time()
for _ in range(5):
    engine_for(net)
torch.cuda.synchronize()
print("set_net ms (tied copy + cell tables)", round((time.time() - t) / 5 * 1e3, 3))
eng.kernel_timer(True)
eng.lattice()
mask = eng.active_planes(0)
lat = eng.kernel_timer(False)
print("setup", json.dumps({k: round(v["ms"], 3) for k, v in lat.items()}))
K = net.K
tot = {}
for idx in range(K):
    if not (mask >> idx) & 1:
        continue
    eng.kernel_timer(True)
    try:
        S, fail = eng.split(idx)
        st = eng.finish(idx, idx < K - 1, fail) if S else None
    except RuntimeError as ex:  # TNP_EXP timing runs compute wrong values
        print("stopped:", ex)
        print("   ", json.dumps({k: round(v["ms"], 3) for k, v in eng.kernel_timer(False).items()}))
        break
    kt = eng.kernel_timer(False)
    if st:
        mask = (mask & ((1 << (idx + 1)) - 1)) | st["next_active"]
        print({k: st[k] for k in ("idx", "V_in", "E_in", "S", "H", "X", "V_out", "E_out", "A", "P",
                                  "pair_tests", "T")})
    ms = {k: round(v["ms"], 3) for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["ms"])}
    print("   ", json.dumps(ms), "sum", round(sum(ms.values()), 3))
    for k, v in kt.items():
        tot[k] = tot.get(k, 0) + v["ms"]
print("total", json.dumps({k: round(v, 3) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])}),
      "sum", round(sum(tot.values()), 3))
