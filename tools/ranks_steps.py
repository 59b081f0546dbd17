"""Per-step trace of a multi-rank block run (diagnostic): under
torch.distributed.run with gloo, every rank runs its block of the bench
lattice `passes` times with the bench's global decisions and prints, for
`--rank`, per step (pass, plane, local S, global S, global failover, V, E)
and the process's device memory -- to find where a shard's passes diverge.
python -m torch.distributed.run --nproc-per-node 4 ... tools/ranks_steps.py 203 3 4 2"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tropical-nerf.pytorch_amd"))


def main():
    G, halo, passes, show = (int(a) for a in (sys.argv[1:] + ["203", "3", "4", "2"])[:4])
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import bench
    from tropical.distributed import Blocks, block_dims
    from tropical._engine import engine_for
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    coll = bench.Collective(torch.device("cpu"))
    net = bench.make_net(G, dev, 6)
    part = Blocks(G, block_dims(world))
    eng = engine_for(net)
    eng.set_owned_box(*part.owned(rank))
    eng.set_shards(world)
    K = eng.K
    for p in range(passes):
        # as bench: a pass at halo - 1, then at halo, each exported (the halo
        # check's view), then the warmup and timed passes
        lo, hi = part.box(rank, halo - 1 if p == 0 else halo)
        eng.lattice_box(lo, hi)
        mask = int(coll(np.array([eng.active_planes(0)], dtype=np.uint64), "or")[0])
        for idx in range(K):
            if not (mask >> idx) & 1:
                continue
            S, fail = eng.split(idx)
            g = coll(np.array([S, int(fail)], dtype=np.int64), "max")
            if int(g[0]) == 0:
                continue
            st = eng.finish(idx, idx < K - 1, int(g[1]))
            if rank == show:
                V, E = eng.sizes()
                fr, tot = torch.cuda.mem_get_info(dev)
                print(f"pass {p} plane {idx}: S {S} fail {int(fail)} | S_glob {int(g[0])} fail_glob {int(g[1])} "
                      f"| V {V} E {E} X {st.get('X')} | {(tot - fr) / 2**30:.1f} GiB", flush=True)
            if idx < K - 1:
                m2 = int(coll(np.array([st["next_active"]], dtype=np.uint64), "or")[0])
                mask = (mask & ((1 << (idx + 1)) - 1)) | m2
        if p < 2:
            eng.export()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
