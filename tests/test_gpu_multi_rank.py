"""GPU, 2-8 ranks sharing one MI355X over gloo: the sharded HIP engine.

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
  201-mark large net (2, 3 and the config's 8 ranks) and the small net;
* BASELINE config 5 at full size: the 256^3 seed-6 synthetic lattice cut
  into 8 x-slabs must stitch to exactly the complex the unsharded engine
  extracts on one GPU (counts + order-free fingerprints).
Lattice shards use the halo search of bench.py (HALOS, halo_check).
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


def _sharded_lattice(net, rank, world, coll, stats, blocks=False):
    """This rank's x-slab (blocks: its block of the most cubic split,
    bench.py's N > 1 path) of the net's full lattice, with the narrowest halo
    of HALOS that halo_check accepts."""
    from tropical import distributed as D
    from tropical._engine import engine_for
    n = int(net.enc.marks.shape[0])
    part = D.Blocks(n, D.block_dims(world)) if blocks else D.Blocks.xslabs(D.slab_cuts(n, world))
    eng = engine_for(net)
    eng.set_owned_box(*part.owned(rank))
    eng.set_shards(world)
    marks = net.enc.marks.cpu()
    for k, h in enumerate(D.HALOS):
        st = []
        eng.lattice_box(*part.box(rank, h))
        eng.run_steps(st, coll)
        Vl, El, _ = eng.export()
        Vl, El = Vl.cpu(), El.cpu()
        if D.halo_check(Vl, El, marks, part, raise_=k == len(D.HALOS) - 1) is not None:
            break
    stats.extend(st)
    _sharded_lattice.attempts = k + 1  # extractions the halo search ran
    return part, Vl, El, h


def _worker(rank, world, port, outdir, case, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from helpers import product_net
        from tropical import distributed as D
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        coll = bench.Collective(torch.device("cpu"))
        stats = []
        blocks = mode.endswith("_blocks")
        if mode.startswith("bench"):  # the synthetic bench net of `case` = (marks, seed[, passes])
            G, seed = case[:2]
            net = bench.make_net(G, dev, seed)
            part, Vl, El, halo = _sharded_lattice(net, rank, world, coll, stats, blocks)
            # further passes of the accepted halo on the same engine (bench.py's
            # timed loop): the engine's device footprint must stay what the
            # first pass left (round 4's 4-block run grew a buffer by half per
            # step until hipMallocAsync failed)
            from tropical._engine import engine_for
            eng = engine_for(net)
            foot = [eng.scratch_bytes()]
            for _ in range(case[2] if len(case) > 2 else 0):
                eng.lattice_box(*part.box(rank, halo))
                eng.run_steps([], coll)
                foot.append(eng.scratch_bytes())
            if len(foot) > 1:
                Vl, El, _ = eng.export()
                Vl, El = Vl.cpu(), El.cpu()
            steady = torch.tensor([int(all(f == foot[1] for f in foot[1:]))])
            dist.all_reduce(steady, op=dist.ReduceOp.MIN)
            own, keep = D.owned_masks(Vl, El, net.enc.marks.cpu(), part, rank)
            hv, he = D.complex_hash(Vl, El, own, keep)
            splits = sum(s["S"] - s["S_dup"] for s in stats)
            tot = torch.tensor([int(own.sum()), int(keep.sum()), hv, he, splits], dtype=torch.int64)
            dist.all_reduce(tot)
            if rank == 0:
                np.savez(os.path.join(outdir, "out.npz"), tot=tot.numpy(), dims=np.array(part.dims),
                         halo=np.array(halo), redundant=np.array(part.redundant_frac(rank, halo)),
                         attempts=np.array(_sharded_lattice.attempts),
                         steady=steady.numpy(), foot=np.array([f["bytes"] for f in foot]))
            return
        d = load(case)
        net = product_net(d, dev)
        if mode == "empty":
            # a net whose SDF never crosses zero (o1 - o0 = 5 everywhere): its
            # skeleton is empty, subpoly falls back to get_hypercube
            # (subpoly.py:51-52), and the sharded driver must say so
            with torch.no_grad():
                net.fc[-1].weight.zero_()
                net.fc[-1].bias.copy_(torch.tensor([0.0, 5.0]))
            raised = []
            for box in (True, False):
                try:
                    D.subpoly_sharded(net, 1.2, allreduce=coll, box_skeleton=box)
                    raised.append(0)
                except NotImplementedError:
                    raised.append(1)
            if rank == 0:
                np.savez(os.path.join(outdir, "out.npz"), raised=np.array(raised))
            return
        if mode.startswith("lattice"):
            part, Vl, El, _ = _sharded_lattice(net, rank, world, coll, stats, blocks)
            cuts = part.cuts[0]
            owned, first, gE, own, keep = D.stitch(Vl, El, net.enc.marks.cpu(), part, masks=True)
        else:  # "skeleton" (flat) or "curve" (force=False: the curve branch's decisions go
            # through the engine's collective callback)
            curve = mode.startswith("curve")
            info = {}
            eng, owned, first, gE, cuts = D.subpoly_sharded(net, 1.2, allreduce=coll, stats=stats,
                                                            force=not curve, blocks=blocks, info=info,
                                                            box_skeleton=not mode.endswith("_whole"))
            Vl, El, _ = eng.export()
            Vl, El = Vl.cpu(), El.cpu()
            own, keep = D.owned_masks(Vl, El, net.enc.marks.cpu(), cuts, rank)
        hv, he = D.complex_hash(Vl, El, own, keep)
        splits = sum(s["S"] - s["S_dup"] for s in stats)
        tot = torch.tensor([owned.shape[0], gE.shape[0], hv, he, splits], dtype=torch.int64)
        dist.all_reduce(tot)
        SV, SE = D.gather_complex(owned.cpu(), first, gE.cpu())
        # then a plain single-device subpoly(force=False) in the same process:
        # engine_for must hand it an engine without the sharded run's shard
        # count, owned range and x span
        import contextlib
        import io
        from golden_io import sha
        import tropical.subpoly as sp
        single_ok = torch.tensor([1])
        if not mode.startswith("lattice"):  # (the lattice goldens hold the full-lattice surface, not subpoly's)
            with contextlib.redirect_stdout(io.StringIO()):
                _, verts, fwi = sp.subpoly(net, 3, 1.2, force=not curve)
            single_ok[0] = int(verts.shape[0] == int(d["n_surf"][0]) and
                               sha(np.asarray(fwi, dtype=np.int64)) == str(d["sha_tri"]))
        dist.all_reduce(single_ok, op=dist.ReduceOp.MIN)
        attempts = _sharded_lattice.attempts if mode.startswith("lattice") else info["halo_attempts"]
        if rank == 0:
            np.savez(os.path.join(outdir, "out.npz"), tot=tot.numpy(), V=SV.numpy(), E=SE.numpy(),
                     cuts=np.array(cuts.cuts[0] if isinstance(cuts, D.Blocks) else cuts),
                     single_ok=single_ok.numpy(), attempts=np.array(attempts))
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
    eng.set_owned()
    eng.set_shards(1)
    eng.set_curve(mode == "curve")
    if mode == "lattice":
        eng.lattice()
    else:
        eng.skeleton(128, 1.2)
    stats = []
    eng.run_steps(stats)
    V, E, _ = eng.export()
    eng.set_curve(False)
    hv, he = complex_hash(V, E)
    return d, V, E, (V.shape[0], E.shape[0], hv, he, sum(s["S"] for s in stats))


@pytest.mark.parametrize("case,world,mode", [("synth32h", 2, "lattice"), ("synth32h", 3, "lattice"),
                                             ("synth64h", 2, "lattice"), ("synth64h", 8, "lattice"),
                                             ("synth32h", 4, "lattice_blocks"), ("synth64h", 8, "lattice_blocks"),
                                             # K = 65 (two-word sign keys) on shards
                                             ("synth16_h32l3", 2, "lattice"),
                                             ("synth16_h32l3", 4, "lattice_blocks")])
def test_sharded_lattice_engine(cuda, tmp_path, case, world, mode):
    """x-slabs, and blocks (2 x 2 x 1, 2 x 2 x 2: the box lattice, owned box
    and span of the engine, halo_check over every cut face, the stitch's
    cell-owner edge rule with vertices shared by up to 8 blocks)."""
    d, V, E, want = _unsharded(cuda, case, "lattice")
    assert (want[0], want[1]) == tuple(int(x) for x in d["pre_VE"])
    assert (want[2], want[3]) == tuple(int(x) for x in d["complex_hash"])  # the reference's
    z = _run(tmp_path, case, mode, world)
    assert tuple(int(x) for x in z["tot"]) == want
    # the gathered complex has one global numbering: every edge resolves
    assert z["V"].shape[0] == want[0] and z["E"].shape[0] == want[1]
    assert z["E"].min() >= 0 and z["E"].max() < want[0]


@pytest.mark.parametrize("case,world,mode", [("large_sphere", 2, "skeleton"), ("large_sphere", 3, "skeleton"),
                                             ("large_sphere", 8, "skeleton"), ("small_sphere", 2, "skeleton"),
                                             ("large_sphere", 8, "skeleton_blocks"),
                                             # the whole skeleton on every rank, cuts at equal edge load
                                             ("large_sphere", 3, "skeleton_whole"),
                                             ("small_sphere", 2, "skeleton_whole")])
def test_sharded_stanford_net(cuda, tmp_path, case, world, mode):
    """x-slabs of equal skeleton load, and (skeleton_blocks) 2 x 2 x 2
    blocks cut at equal marginal load per axis.  The default splits the
    skeleton itself over the ranks (box_skeleton: per-plane point loads);
    skeleton_whole computes it whole on every rank and cuts at equal
    skeleton-edge load -- both stitch to the unsharded complex, so they
    stitch to the same one."""
    d, V, E, want = _unsharded(cuda, case, "skeleton")
    z = _run(tmp_path, case, mode, world)
    assert tuple(int(x) for x in z["tot"]) == want
    if mode == "skeleton_blocks":  # the halo search accepts its first width: one extraction
        assert int(z["attempts"]) == 1
    cuts = z["cuts"].tolist()
    assert cuts[0] == 0 and cuts[-1] == len(d["marks"]) - 1
    assert len(cuts) == (3 if mode == "skeleton_blocks" else world + 1)


def test_sharded_empty_skeleton_raises(cuda, tmp_path):
    """A net whose skeleton is empty: subpoly() falls back to get_hypercube
    (subpoly.py:51-52), which subpoly_sharded does not shard -- it raises
    NotImplementedError on every rank, with the skeleton split over the ranks
    (box_skeleton, the default: no box holds an edge) and whole."""
    z = _run(tmp_path, "small_sphere", "empty", 2)
    assert z["raised"].tolist() == [1, 1]


@pytest.mark.parametrize("case,world,mode", [("small_sphere_curve", 2, "curve"), ("small_sphere_curve", 3, "curve"),
                                             ("small_torus_curve", 2, "curve"),
                                             ("small_sphere_curve", 4, "curve_blocks"),
                                             ("small_torus_curve", 8, "curve_blocks"),
                                             # K = 65: two-word keys through the curve branch's shards
                                             ("h16l5_sphere_curve", 2, "curve")])
def test_sharded_curve_branch(cuda, tmp_path, case, world, mode):
    """The curve branch (force=False) on x-slabs: the per-step decisions the
    reference takes over the whole batch -- the curve rows' and descent rows'
    counts (MKL's row-count schedules), the descent's stop iteration (an AND
    of the shards' convergence words, subpoly_debug.py:141) and the strict
    filter's flag (subpoly_debug.py:253-257) -- go through the engine's
    collective callback (tnp_engine_set_collective); the stitched complex must
    equal the unsharded curve run's.  curve_blocks: 2 x 2 x 1 and 2 x 2 x 2
    blocks, where the failover test counts only each shard's owned new
    vertices (k_fail_check)."""
    d, V, E, want = _unsharded(cuda, case, "curve")
    z = _run(tmp_path, case, mode, world)
    assert tuple(int(x) for x in z["tot"]) == want
    assert z["V"].shape[0] == want[0] and z["E"].shape[0] == want[1]
    # a single-device subpoly(force=False) after the sharded run, same process
    assert int(z["single_ok"][0]) == 1


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["bench", "bench_blocks"])
def test_lattice256_eight_slabs_stitch_to_the_unsharded_complex(cuda, tmp_path, mode):
    """BASELINE config 5 at its full size (the 8-GPU weak-scaling lattice of
    bench.py --gpus 8): the 256^3 seed-6 synthetic lattice cut into 8 x-slabs,
    or the 2 x 2 x 2 blocks bench.py uses (8 gloo ranks sharing this GPU,
    halo search as bench.py), must hold exactly the complex the unsharded
    engine extracts on one GPU -- same vertex and edge counts, same
    order-free fingerprints -- and count every split once; the blocks' halo
    must leave at most 7 % of a rank's cells redundant."""
    import bench
    from tropical.distributed import complex_hash
    from tropical._engine import engine_for
    net = bench.make_net(256, cuda, 6)
    eng = engine_for(net)
    eng.set_owned()
    eng.set_shards(1)
    eng.lattice()
    stats = []
    eng.run_steps(stats)
    V, E, _ = eng.export()
    hv, he = complex_hash(V, E)
    want = (V.shape[0], E.shape[0], hv, he, sum(s["S"] for s in stats))
    del V, E
    torch.cuda.empty_cache()
    z = _run(tmp_path, (256, 6), mode, 8)
    assert tuple(int(x) for x in z["tot"]) == want
    if mode == "bench_blocks":
        assert z["dims"].tolist() == [2, 2, 2]
        assert float(z["redundant"]) <= 0.07, (int(z["halo"]), float(z["redundant"]))
        assert int(z["attempts"]) == 1  # no rejected extraction in the halo search


def _unsharded_bench(cuda, G, seed):
    import bench
    from tropical.distributed import complex_hash
    from tropical._engine import engine_for
    net = bench.make_net(G, cuda, seed)
    eng = engine_for(net)
    eng.set_owned()
    eng.set_shards(1)
    eng.lattice()
    stats = []
    eng.run_steps(stats)
    V, E, _ = eng.export()
    hv, he = complex_hash(V, E)
    want = (V.shape[0], E.shape[0], hv, he, sum(s["S"] for s in stats))
    del V, E
    torch.cuda.empty_cache()
    return want


@pytest.mark.timeout(600)
def test_four_blocks_203_steady_footprint(cuda, tmp_path):
    """The run that blew up in round 4 (bench.py --gpus 4: 2 x 2 x 1 blocks of
    the 203^3 seed-6 lattice, gpurun_out/rs.log: hipMallocAsync of 66 GB after
    the connect key buffer grew by half per step): 4 gloo ranks sharing this
    GPU run the halo search and then 5 more passes each on the same engine;
    every rank's device footprint (tnp_engine_scratch_bytes) must stay what
    its first timed pass left, and the stitched complex must equal the
    unsharded one."""
    want = _unsharded_bench(cuda, 203, 6)
    z = _run(tmp_path, (203, 6, 5), "bench_blocks", 4)
    assert z["dims"].tolist() == [2, 2, 1]
    assert int(z["steady"][0]) == 1, z["foot"].tolist()
    assert tuple(int(x) for x in z["tot"]) == want


def test_slab_buckets_do_not_change_the_result(cuda):
    """The spatial buckets of an x-slab cover only its cells (lattice() sets
    the x span; an 8-rank 256^3 slab: 5 x 33 x 33 buckets of 8^3 cells
    instead of 17^3 of 16^3).  Geometry is performance only: the slab's
    complex with the narrow buckets equals the one with the whole grid's,
    and a vertex outside the span fails loudly instead of being dropped."""
    from helpers import product_net
    from tropical.distributed import complex_hash
    from tropical._engine import engine_for
    net = product_net(load("synth64h"), cuda)
    eng = engine_for(net)
    eng.set_owned()
    eng.set_shards(2)  # a slab may hold no connecting pair on some step
    got = []
    for narrow in (True, False):
        eng.lattice(20, 41)
        if not narrow:
            eng.set_xspan()  # the whole grid
        eng.run_steps([])
        V, E, _ = eng.export()
        got.append((V.shape[0], E.shape[0]) + complex_hash(V, E))
    assert got[0] == got[1]
    # a block: buckets over its box along all three axes
    got = []
    for narrow in (True, False):
        eng.lattice_box([20, 10, 5], [41, 40, 30])
        if not narrow:
            eng.set_span([0, 0, 0], [-1, -1, -1])
        eng.run_steps([])
        V, E, _ = eng.export()
        got.append((V.shape[0], E.shape[0]) + complex_hash(V, E))
    assert got[0] == got[1]
    eng.lattice_box([20, 10, 5], [41, 40, 30])
    eng.set_span([20, 10, 5], [41, 25, 30])
    with pytest.raises(RuntimeError, match="outside the mark planes"):
        eng.run_steps([])
    eng.lattice(20, 41)
    eng.set_xspan(30, 41)
    with pytest.raises(RuntimeError, match="outside the mark planes"):
        eng.run_steps([])
    eng.set_shards(1)


def _nccl_worker(rank, world, port, outdir):
    """ONE process on the one GPU, world size 1, backend nccl (RCCL): every
    collective call site of the sharded path -- bench.Collective's
    all_gather_into_tensor on device tensors, the engine's in-step
    collective callback (curve branch), halo_check's and stitch's
    all_gathers, the final all_reduce -- runs through RCCL on device tensors,
    as on the 8-GPU node (the gloo tests put them on host copies)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        import bench
        from helpers import product_net
        from tropical import distributed as D
        from tropical._engine import engine_for
        coll = bench.Collective(dev, shm=False)
        assert coll.shm is None and D.comm_device(None, dev).type == "cuda"
        # the collective itself: OR / AND / SUM / MAX of one rank's words
        v = np.array([5, 1 << 62, 3], dtype=np.uint64)
        out = {op: coll(v, op) for op in ("or", "and")}
        w = np.array([7, -2, 40], dtype=np.int64)
        out.update({op: coll(w, op) for op in ("sum", "max")})
        ok = all(np.array_equal(out[o], v) for o in ("or", "and")) and \
            all(np.array_equal(out[o], w) for o in ("sum", "max"))
        # the synthetic lattice through the host loop with the RCCL collective
        net = bench.make_net(24, dev, 6)
        part = D.Blocks(24, D.block_dims(1))
        eng = engine_for(net)
        eng.set_owned_box(*part.owned(0))
        eng.set_shards(1)
        eng.lattice_box(*part.box(0, 3))
        st = []
        eng.run_steps(st, coll)
        Vl, El, _ = eng.export()
        marks = net.enc.marks
        seen = D.halo_check(Vl, El, marks, part)  # device tensors: RCCL all_gather
        owned, first, gE, own, keep = D.stitch(Vl, El, marks, part, masks=True)
        hv, he = D.complex_hash(Vl, El, own, keep)
        tot = torch.tensor([owned.shape[0], gE.shape[0], hv, he, sum(s["S"] for s in st)], device=dev,
                           dtype=torch.int64)
        dist.all_reduce(tot)
        SV, SE = D.gather_complex(owned, first, gE)
        # the curve branch's in-step decisions through the engine's collective
        # callback, then the skeleton split, all on RCCL
        d = load("small_sphere_curve")
        cnet = product_net(d, dev)
        cst = []
        ceng, cown, cfirst, cgE, ccuts = D.subpoly_sharded(cnet, 1.2, allreduce=coll, stats=cst, force=False)
        CV, CE, _ = ceng.export()
        ch = D.complex_hash(CV, CE)
        # the engine calls the collective back from inside a curve step only
        # on shards: the same extraction as 2 "shards" of which this rank is
        # the only one (its totals are the batch's), every in-step decision
        # (curve rows, descent rows, convergence AND, strict OR) over RCCL
        ceng.set_owned()
        ceng.set_span([0, 0, 0], [-1, -1, -1])
        ceng.set_shards(2)
        ceng.set_curve(True)
        ceng.skeleton(128, 1.2)
        cst2 = []
        ceng.run_steps(cst2, coll)
        CV2, CE2, _ = ceng.export()
        ch2 = D.complex_hash(CV2, CE2)
        ceng.set_shards(1)
        ceng.set_curve(False)
        np.savez(os.path.join(outdir, "out.npz"), ok=np.array(int(ok)), tot=tot.cpu().numpy(),
                 seen=np.array(seen is not None), first=np.array(first),
                 nV=np.array(SV.shape[0]), nE=np.array(SE.shape[0]), dev=np.array(str(SV.device)),
                 curve=np.array([CV.shape[0], CE.shape[0], ch[0], ch[1], sum(s["S"] for s in cst)],
                                dtype=np.int64),
                 curve2=np.array([CV2.shape[0], CE2.shape[0], ch2[0], ch2[1], sum(s["S"] for s in cst2)],
                                 dtype=np.int64),
                 cown=np.array(cown.shape[0]), cgE=np.array(cgE.shape[0]))
    finally:
        dist.destroy_process_group()


def test_rccl_world_size_one_runs_every_collective_call_site(cuda, tmp_path):
    """the RCCL branch of every collective (bench.Collective
    without shared memory, halo_check, stitch, gather_complex, the curve
    branch's engine callback) on device tensors, in one nccl process group of
    world size 1 on the one GPU; the results equal the unsharded engine's."""
    mp.spawn(_nccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    z = np.load(tmp_path / "out.npz")
    assert int(z["ok"]) == 1
    assert bool(z["seen"])
    assert str(z["dev"]).startswith("cuda")
    import bench
    from tropical.distributed import complex_hash
    from tropical._engine import engine_for
    net = bench.make_net(24, cuda, 6)
    eng = engine_for(net)
    eng.set_owned()
    eng.set_shards(1)
    eng.lattice()
    st = []
    eng.run_steps(st)
    V, E, _ = eng.export()
    ref = [V.shape[0], E.shape[0], *complex_hash(V, E), sum(s["S"] for s in st)]
    assert z["tot"].tolist() == ref
    assert int(z["first"]) == 0 and int(z["nV"]) == V.shape[0] and int(z["nE"]) == E.shape[0]
    d, Vc, Ec, cref = _unsharded(cuda, "small_sphere_curve", "curve")
    assert z["curve"].tolist() == list(cref)
    assert z["curve2"].tolist() == list(cref)
    assert int(z["cown"]) == Vc.shape[0] and int(z["cgE"]) == Ec.shape[0]
