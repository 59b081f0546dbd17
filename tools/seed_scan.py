"""Scan synthetic-net seeds at G^3: splits, connecting edges, wall time (GPU)."""
import sys, os, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd")]
import torch
from bench import make_net
from tropical._engine import engine_for
G = int(sys.argv[1]); seeds = range(int(sys.argv[2]), int(sys.argv[3]))
dev = torch.device("cuda", 0)
for seed in seeds:
    net = make_net(G, dev, seed)
    eng = engine_for(net)
    eng.lattice(); stats = []
    torch.cuda.synchronize(); t = time.time()
    try:
        eng.run_steps(stats)
        torch.cuda.synchronize()
        S = sum(s["S"] for s in stats); X = sum(s["X"] for s in stats); P = sum(s["P"] for s in stats)
        V, E = eng.sizes()
        print(f"seed {seed}: active {len(stats)} S {S} X {X} P {P} maxX/S {max(s['X']/max(s['S'],1) for s in stats):.1f} final V {V} E {E} {time.time()-t:.3f}s", flush=True)
    except RuntimeError as e:
        print(f"seed {seed}: error {e} {time.time()-t:.3f}s", flush=True)
