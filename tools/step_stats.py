"""Print per-step engine stats for the synthetic lattice (GPU)."""
import sys, os, json, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd")]
import torch
from bench import make_net
from tropical._engine import engine_for
G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda", 0)
net = make_net(G, dev, int(sys.argv[2]) if len(sys.argv) > 2 else 6)
eng = engine_for(net)
eng.lattice()
stats = []
eng.kernel_timer(True)
t = time.time(); eng.run_steps(stats); torch.cuda.synchronize(); dt = time.time() - t
kt = eng.kernel_timer(False)
for s in stats:
    print({k: s[k] for k in ("idx", "V_in", "E_in", "S", "H", "X", "V_out", "E_out", "A", "P", "pair_tests")})
print("wall", dt)
print(json.dumps({k: round(v["ms"], 2) for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["ms"])}))
