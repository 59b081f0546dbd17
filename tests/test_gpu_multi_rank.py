"""GPU, 2-3 ranks sharing one MI355X over gloo: the sharded HIP engine.

Each rank runs the device engine on its x-slab (plus halo) with the
reference's whole-complex decisions taken through bench.Collective; the
neighbours' views next to every cut are compared (distributed.halo_check,
fails loudly), the slabs are stitched (distributed.stitch) and the stitched
complex must equal the unsharded engine's -- which the single-device tests
pin to the reference -- as a vertex/edge set (counts + order-free
fingerprints; N > 1 parity is up to numbering):
* the synthetic lattice (bench.py's N > 1 path): synth32h (hashed levels) and
  the 64^3 hashed golden, whose unsharded counts/fingerprint come from the
  reference itself;
* Stanford-style nets (BASELINE config 4): subpoly_sharded -- skeleton on the
  reference's 128-mark tiles, slabs of equal skeleton-edge load -- on the
  201-mark large net and the small net.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_io import load

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, case, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from helpers import product_net
        from tropical import distributed as D
        from tropical._engine import engine_for
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        d = load(case)
        net = product_net(d, dev)
        coll = bench.Collective(torch.device("cpu"))
        stats = []
        if mode == "lattice":
            n = int(d["lattice_n"])
            cuts = D.slab_cuts(n, world)
            x0, x1 = D.slab_marks(cuts, rank)
            eng = engine_for(net)
            eng.set_owned(cuts[rank], cuts[rank + 1])
            eng.set_shards(world)
            eng.lattice(x0, x1)
            eng.run_steps(stats, coll)
            Vl, El, _ = eng.export()
            Vl, El = Vl.cpu(), El.cpu()
            D.halo_check(Vl, El, net.enc.marks.cpu(), cuts)
            owned, first, gE, own, keep = D.stitch(Vl, El, net.enc.marks.cpu(), cuts, masks=True)
        else:
            eng, owned, first, gE, cuts = D.subpoly_sharded(net, 1.2, allreduce=coll, stats=stats)
            Vl, El, _ = eng.export()
            Vl, El = Vl.cpu(), El.cpu()
            own = D.owner_of(Vl, net.enc.marks.cpu(), cuts) == rank
            keep = torch.maximum(D.owner_of(Vl, net.enc.marks.cpu(), cuts)[El[:, 0]],
                                 D.owner_of(Vl, net.enc.marks.cpu(), cuts)[El[:, 1]]) == rank
        hv, he = D.complex_hash(Vl, El, own, keep)
        splits = sum(s["S"] - s["S_dup"] for s in stats)
        tot = torch.tensor([owned.shape[0], gE.shape[0], hv, he, splits], dtype=torch.int64)
        dist.all_reduce(tot)
        SV, SE = D.gather_complex(owned.cpu(), first, gE.cpu())
        if rank == 0:
            np.savez(os.path.join(outdir, "out.npz"), tot=tot.numpy(), V=SV.numpy(), E=SE.numpy(),
                     cuts=np.array(cuts))
    finally:
        dist.destroy_process_group()


def _run(tmp_path, case, mode, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), case, mode), nprocs=world, join=True)
    return np.load(tmp_path / "out.npz")


def _unsharded(cuda, case, mode):
    from helpers import product_net
    from tropical.distributed import complex_hash
    from tropical._engine import engine_for
    d = load(case)
    net = product_net(d, cuda)
    eng = engine_for(net)
    if mode == "lattice":
        eng.lattice()
    else:
        eng.skeleton(128, 1.2)
    stats = []
    eng.run_steps(stats)
    V, E, _ = eng.export()
    hv, he = complex_hash(V, E)
    return d, V, E, (V.shape[0], E.shape[0], hv, he, sum(s["S"] for s in stats))


@pytest.mark.parametrize("case,world", [("synth32h", 2), ("synth32h", 3), ("synth64h", 2)])
def test_sharded_lattice_engine(cuda, tmp_path, case, world):
    d, V, E, want = _unsharded(cuda, case, "lattice")
    assert (want[0], want[1]) == tuple(int(x) for x in d["pre_VE"])
    assert (want[2], want[3]) == tuple(int(x) for x in d["complex_hash"])  # the reference's
    z = _run(tmp_path, case, "lattice", world)
    assert tuple(int(x) for x in z["tot"]) == want
    # the gathered complex has one global numbering: every edge resolves
    assert z["V"].shape[0] == want[0] and z["E"].shape[0] == want[1]
    assert z["E"].min() >= 0 and z["E"].max() < want[0]


@pytest.mark.parametrize("case,world", [("large_sphere", 2), ("large_sphere", 3), ("small_sphere", 2)])
def test_sharded_stanford_net(cuda, tmp_path, case, world):
    d, V, E, want = _unsharded(cuda, case, "skeleton")
    z = _run(tmp_path, case, "skeleton", world)
    assert tuple(int(x) for x in z["tot"]) == want
    cuts = z["cuts"].tolist()
    assert cuts[0] == 0 and cuts[-1] == len(d["marks"]) - 1 and len(cuts) == world + 1
