"""Repeat one shard's pass on one GPU (diagnostic for the 4-block rehearsal):
the bench net at G^3, the block of `rank` in the most cubic split of
`world`, `passes` passes of lattice_box + run_steps (local decisions), an
export after the second (as bench's halo check does); prints per pass the
split count, final sizes and device memory.  Identical passes expected."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tropical-nerf.pytorch_amd"))


def main():
    G, world, rank, halo, passes = (int(a) for a in (sys.argv[1:] + ["203", "4", "0", "3", "6"])[:5])
    import bench
    from tropical._engine import engine_for
    from tropical.distributed import Blocks, block_dims
    dev = torch.device("cuda", 0)
    net = bench.make_net(G, dev, 6)
    part = Blocks(G, block_dims(world))
    eng = engine_for(net)
    eng.set_owned_box(*part.owned(rank))
    eng.set_shards(world)
    lo, hi = part.box(rank, halo)
    for p in range(passes):
        t0 = time.perf_counter()
        eng.lattice_box(lo, hi)
        st = []
        try:
            eng.run_steps(st, None)
        except RuntimeError as ex:
            print(f"pass {p}: {ex}", flush=True)
            raise SystemExit(1)
        V, E = eng.sizes()
        fr, tot = torch.cuda.mem_get_info(dev)
        print(f"pass {p}: S {sum(s['S'] for s in st)} steps {len(st)} V {V} E {E} "
              f"{(time.perf_counter() - t0) * 1e3:.1f} ms, {(tot - fr) / 2**30:.1f} GiB in use", flush=True)
        if p == 1:
            eng.export()


if __name__ == "__main__":
    main()
