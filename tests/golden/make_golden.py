"""Generate golden fixtures by running the REFERENCE (/root/reference) on CPU.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py [case ...]

Each case writes ``tests/golden/<case>.npz`` holding
* the inputs: net config, weights (``p:<state_dict key>``), optional lattice size;
* the reference's outputs: skeleton (V0, E0) for skeleton cases, per-step
  (idx, V, E) counts and SHA-256 of (vertices, edges int64, cache) after every
  ``subpoly_`` call, the final surface vertices, ``faces_with_indices`` and
  float ``faces``.

Rules: argsort forced stable; the tinycudann stub is the
oracle's encoding (oracle/encoding.py); weights come from numpy PCG64
(tropical/synthetic.py) or from a short CPU fit of the oracle net to an
analytic SDF (weights are stored, so the fit itself needs no determinism).
"""
from __future__ import annotations

import hashlib
import importlib.util
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

_spec = importlib.util.spec_from_file_location(
    "_synthetic", os.path.join(REPO, "tropical-nerf.pytorch_amd", "tropical", "synthetic.py"))
syn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(syn)

FULL_MAX_TRI = 20_000
SMALL = dict(num_layers=3, num_hidden=16, levels=4, r_min=2, r_max=32, T=19)
LARGE = dict(num_layers=3, num_hidden=16, levels=4, r_min=8, r_max=128, T=19)


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def fit_sdf(cfg, fn, seed, iters=1000, batch=4096, lr=1e-2):
    """Fit the oracle net to an analytic SDF on CPU (stand-in pretrained net)."""
    from oracle.subdivide import RefNet, load_params
    net = RefNet(**cfg)
    load_params(net, syn.random_params(net.enc.module.params.numel(), net.num_nodes, seed, 1e-4))
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, iters)
    g = torch.Generator().manual_seed(seed)
    for it in range(iters):
        x = torch.rand(batch, 3, generator=g) * 2.0 - 1.0
        loss = (net.sdf(x)[:, 0] - torch.tanh(fn(x))).abs().mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
    print(f"  fit loss {loss.item():.5f}")
    return {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}


def sphere(x):
    return x.norm(dim=-1) - 0.6


def torus(x):
    q = torch.stack([torch.sqrt(x[:, 0] ** 2 + x[:, 1] ** 2) - 0.5, x[:, 2]], -1)
    return q.norm(dim=-1) - 0.2


CASES = {
    # name: (kind, cfg, weights, extra); lattice extra = marks per axis or
    # (marks, T): T < 19 hashes the lattice's levels (res = marks - 1)
    "synth24": ("lattice", None, ("rand", 1, 0.1), 24),
    "synth32": ("lattice", None, ("rand", 2, 0.1), 32),
    "synth32u": ("lattice", None, ("rand_uncentered", 0, 0.1), 32),
    "small_sphere": ("subpoly", SMALL, ("fit", sphere, 7), None),
    "small_torus": ("subpoly", SMALL, ("fit", torus, 11), None),
    "small_rand": ("subpoly", SMALL, ("rand", 5, 0.05), None),
    # curve path (force=False): same nets, trilinear correction on
    "small_sphere_curve": ("curve", SMALL, ("same", "small_sphere"), None),
    "small_torus_curve": ("curve", SMALL, ("same", "small_torus"), None),
    "small_rand_curve": ("curve", SMALL, ("same", "small_rand"), None),
    # hashed levels (31^3 > 2^14, 63^3 > 2^17): the prime-XOR branch of the
    # encoding and the tied-table layout under hashing
    "synth32h": ("lattice", None, ("rand", 3, 0.1), (32, 14)),
    "synth64h": ("lattice", None, ("rand", 4, 0.1), (64, 17)),
    # BASELINE config 3 net class: 201 marks, level 3 hashed (128^3 > 2^19),
    # 2x2x2 skeleton tiles with the 127-stride overlap; weights fitted to a
    # sphere and stored as fp16 (exactly representable in fp32)
    "large_sphere": ("subpoly", LARGE, ("fit16", sphere, 13), None),
    # the bench headline workload (bench.py: 128^3 lattice, seed 6, amp 0.1,
    # uncentred): per-step hashes + order-free final fingerprints
    "bench128": ("lattice", None, ("rand_uncentered", 6, 0.1), (128, 19)),
    # net shapes beyond 3 layers x 16 hidden x {2,4} levels (the reference's
    # Net is generic, model.py:19-50; subpoly loops num_layers-1 x num_hidden,
    # subpoly.py:60-69): BASELINE config 3's "deeper MLP" (4 layers, K = 49
    # planes), a 32-wide 2-layer net, a 3-level 8-wide net (odd level count:
    # MKL's zero-padded schedules), an 8-level net, and lattices of them
    "small4l_sphere": ("subpoly", dict(SMALL, num_layers=4), ("fit", sphere, 17), None),
    "small4l_sphere_curve": ("curve", dict(SMALL, num_layers=4), ("same", "small4l_sphere"), None),
    "h32_torus": ("subpoly", dict(SMALL, num_layers=2, num_hidden=32), ("fit", torus, 19), None),
    "h8l3_sphere": ("subpoly", dict(SMALL, num_hidden=8, levels=3, r_max=24), ("fit", sphere, 23), None),
    "lv8_rand": ("subpoly", dict(SMALL, levels=8, r_max=48, T=15), ("rand", 29, 0.05), None),
    # the curve branch (with its gradient-descent fallback) on 8- and
    # 32-hidden nets and an odd level count (the descent's backward
    # schedules per shape, csrc/curve.hip)
    "h8l3_sphere_curve": ("curve", dict(SMALL, num_hidden=8, levels=3, r_max=24), ("same", "h8l3_sphere"), None),
    "h32_torus_curve": ("curve", dict(SMALL, num_layers=2, num_hidden=32), ("same", "h32_torus"), None),
    # random weights: rows that need the gradient-descent fallback
    "h8l3_rand_curve": ("curve", dict(SMALL, num_hidden=8, levels=3, r_max=24), ("rand", 41, 0.05), None),
    "h32_rand_curve": ("curve", dict(SMALL, num_layers=2, num_hidden=32), ("rand", 43, 0.05), None),
    "synth24_l4h8": ("lattice", None, ("rand", 31, 0.1), (24, 19, dict(num_layers=4, num_hidden=8))),
    "synth20_h32": ("lattice", None, ("rand", 37, 0.1), (20, 19, dict(num_layers=2, num_hidden=32))),
    # K > 63 planes (two-word sign keys, csrc/common.h Key<2>): Net(3 layers,
    # 32 hidden) K = 65, Net(5 layers, 16 hidden) K = 65, Net(4, 32) K = 97 --
    # the flat path from the skeleton and from lattices
    "h32l3_rand": ("subpoly", dict(SMALL, num_layers=3, num_hidden=32), ("rand", 47, 0.05), None),
    "h16l5_sphere": ("subpoly", dict(SMALL, num_layers=5), ("fit", sphere, 61), None),
    "synth16_h32l3": ("lattice", None, ("rand", 53, 0.1), (16, 19, dict(num_layers=3, num_hidden=32))),
    "synth8_h32l4": ("lattice", None, ("rand", 59, 0.1), (8, 19, dict(num_layers=4, num_hidden=32))),
    # the curve branch (force=False) on K = 65 nets: two-word sign keys through
    # the corner forward, the failover shared planes and the 32- / 16-wide
    # descent
    "h32l3_rand_curve": ("curve", dict(SMALL, num_layers=3, num_hidden=32), ("same", "h32l3_rand"), None),
    "h16l5_sphere_curve": ("curve", dict(SMALL, num_layers=5), ("same", "h16l5_sphere"), None),
    # the curve branch with strict=False (subpoly_(..., strict=False),
    # subpoly.py:198-203): every split stays, no strict_check -- driven step
    # by step through subpoly_ from the skeleton (subpoly() never passes it)
    "small_torus_curve_loose": ("curve_loose", SMALL, ("same", "small_torus"), None),
    # subpoly(net, d, size, eps) with eps != net.eps (subpoly.py:24): the
    # steps' sign test, split point, hits, failover, surface and faces use
    # the argument, Net.region (the pair tests and the pruning) net.eps
    "small_sphere_eps3": ("subpoly", SMALL, ("same", "small_sphere"), None),
    "small_torus_eps05": ("subpoly", SMALL, ("same", "small_torus"), None),
}
# the eps argument of subpoly() per case (default: 1e-4 = Net's eps)
# (the curve branch with eps=3e-4 fails in the reference itself: its
# check_new_vertices_on_two_planes diagnostic raises AttributeError)
EPS = {"small_sphere_eps3": 3e-4, "small_torus_eps05": 5e-5}
# table params above this many floats are stored as the generator spec
# (tropical/synthetic.py random_params) instead of the values
GEN_MAX = 200_000


def _surface_check(*args, **kwargs):
    """Stand-in for the name subpoly.py:173 calls unqualified (a NameError in
    the reference); the helper it means (subpoly_debug.py:166-190) only
    prints diagnostics, so the goldens continue as that helper would."""
    print("[check_new_vertices_on_surface]", end=" ")


def build_params(cfg, spec, net):
    if spec[0] == "same":
        with np.load(os.path.join(HERE, spec[1] + ".npz"), allow_pickle=False) as z:
            return {k[2:]: z[k] for k in z.files if k.startswith("p:")}
    if spec[0] == "rand_uncentered":
        return syn.random_params(net.enc.module.params.numel(), net.num_nodes, spec[1], spec[2])
    if spec[0] == "rand":
        p = syn.random_params(net.enc.module.params.numel(), net.num_nodes, spec[1], spec[2])

        def col(x):
            net.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
            with torch.no_grad():
                return net(torch.from_numpy(x), gather=True)[1][-1][:, 0].numpy()
        return syn.center_sdf_bias(p, col, spec[1])
    if spec[0] == "fit16":
        p = fit_sdf(cfg, spec[1], spec[2])
        return {k: v.astype(np.float16) for k, v in p.items()}
    return fit_sdf(cfg, spec[1], spec[2])


def run_case(name):
    sp, model = __import__("ref_loader").import_reference()
    kind, cfg, wspec, n = CASES[name]
    T = 19
    if kind == "lattice":
        n, T, over = (n, 19, {}) if isinstance(n, int) else (tuple(n) + ({},))[:3]
        cfg = dict(syn.net_config_for_lattice(n, T), **over)
    net = model.Net(**cfg)
    params = build_params(cfg, wspec, net)
    net.load_state_dict({k: torch.from_numpy(v.astype(np.float32)) for k, v in params.items()})
    out = {"case": name, "kind": kind, "eps": np.float64(EPS.get(name, 1e-4)),
           "cfg_keys": np.array(list(cfg.keys())),
           "cfg_vals": np.array(list(cfg.values()), dtype=np.int64),
           "marks": net.enc.marks.numpy()}
    n_table = params["enc.module.params"].size
    if wspec[0] in ("rand", "rand_uncentered") and n_table > GEN_MAX:
        # regenerated by tests/golden_io.py (synthetic.random_params); the
        # centred output bias is stored as a value
        out["gen"] = np.array([wspec[1], wspec[2], n_table], dtype=np.float64)
        if wspec[0] == "rand":
            last = f"fc.{len(net.fc) - 1}.bias"
            out["p:" + last] = params[last]
    else:
        for k, v in params.items():
            out["p:" + k] = v

    steps = []
    orig = sp.subpoly_
    memo = {}

    def wrapped(vertices, edges, net_, l, h, eps, outputs_=None, **kw):
        v, e, o = orig(vertices, edges, net_, l, h, eps, outputs_, **kw)
        key = (id(v), id(e), id(o), v.data_ptr(), e.data_ptr(), o.data_ptr())
        if key != memo.get("key"):  # an S == 0 step returns its inputs unchanged
            memo["key"] = key
            memo["sha"] = sha(v.numpy(), e.numpy().astype(np.int64), o.numpy())
        steps.append((l * net_.num_hidden + h, v.shape[0], e.shape[0], memo["sha"]))
        print(f"  step {steps[-1][0]}: V={v.shape[0]} E={e.shape[0]} ({time.time() - t0:.0f}s)",
              flush=True)
        return v, e, o

    sp.subpoly_ = wrapped
    force = kind not in ("curve", "curve_loose")
    if not force:
        sp.check_new_vertices_on_surface = _surface_check
        out["patched"] = np.array("check_new_vertices_on_surface -> diagnostic print")
    t0 = time.time()
    with torch.no_grad():
        if kind == "lattice":
            V = torch.from_numpy(syn.lattice_vertices(net.enc.marks.numpy()))
            E = torch.from_numpy(syn.lattice_edges(n))
            out["lattice_n"] = n
            o = None
            for l in range(net.num_layers - 1):
                for h in range(net.num_hidden):
                    V, E, o = sp.subpoly_(V, E, net, l, h, 1e-4, o, force=True)
            V, E, o = sp.subpoly_(V, E, net, net.num_layers - 2, net.num_hidden, 1e-4, o,
                                  force=True)
            out["pre_VE"] = np.array([V.shape[0], E.shape[0]])
            # the product's fingerprint, loaded by path (``tropical`` here is
            # the reference package)
            dspec = importlib.util.spec_from_file_location(
                "_distributed", os.path.join(REPO, "tropical-nerf.pytorch_amd", "tropical",
                                             "distributed.py"))
            dmod = importlib.util.module_from_spec(dspec)
            dspec.loader.exec_module(dmod)
            complex_hash = dmod.complex_hash
            out["complex_hash"] = np.array(complex_hash(V, E), dtype=np.int64)
            Vs, Es, used = sp.extract_skeleton(V, E, net, 1e-4, o)
            out["surf_V"] = Vs.numpy()
            out["surf_E"] = Es.numpy()
            faces, fwi = sp.extract_faces(Vs, Es, net, o[used], 1e-4)
        else:
            for m in net.modules():
                if isinstance(m, sys.modules["tropical"].TropicalHashGrid):
                    V0, E0 = m.skeleton(net)
                    break
            out["skel_V"] = V0.numpy().copy()
            out["skel_E"] = E0.numpy().copy()  # (subpoly_ rewrites its edges argument in place)
            # duplicate edges from the 127-stride tile overlap (tropical.py:176-181)
            out["skel_dups"] = np.int64(E0.shape[0] - np.unique(E0.numpy(), axis=0).shape[0])
            if not force:
                last = {}
                orig_ex = sp.extract_skeleton

                def grab(vertices, edges, net_, eps, outputs=None):
                    last["V"], last["E"] = vertices.numpy().copy(), edges.numpy().copy()
                    return orig_ex(vertices, edges, net_, eps, outputs)

                sp.extract_skeleton = grab
            if kind == "curve_loose":
                # subpoly.py:58-86 with strict=False in every subpoly_ call;
                # the reference may fail part-way (its diagnostics): record where
                V, E, o = V0.clone(), E0.clone(), None
                try:
                    for l in range(net.num_layers - 1):
                        for h in range(net.num_hidden):
                            cur = l * net.num_hidden + h
                            V, E, o = sp.subpoly_(V, E, net, l, h, 1e-4, o, force=False, strict=False)
                    cur = (net.num_layers - 1) * net.num_hidden
                    V, E, o = sp.subpoly_(V, E, net, net.num_layers - 2, net.num_hidden, 1e-4, o,
                                          force=False, strict=False)
                    Vs, Es, used = sp.extract_skeleton(V, E, net, 1e-4, o)
                    faces, fwi = sp.extract_faces(Vs, Es, net, o[used], 1e-4)
                except AttributeError as ex:
                    out["raises_at"] = np.int64(cur)
                    out["raises"] = np.array(f"{type(ex).__name__}: {ex}")
                    Vs, faces, fwi = torch.zeros(0, 3), [], []
            else:
                faces, Vs, fwi = sp.subpoly(net, 3, 1.2, EPS.get(name, 1e-4), force=force)
            if not force:
                sp.extract_skeleton = orig_ex
                if "V" in last and last["V"].shape[0] <= 50_000:  # small enough to commit in full
                    out["pre_V"], out["pre_E"] = last["V"], last["E"].astype(np.int32)
            out["surf_V"] = Vs.numpy()
    sp.subpoly_ = orig
    faces = np.asarray(faces, dtype=np.float32)
    tri = np.asarray(fwi, dtype=np.int64)
    surf = out.pop("surf_V")
    out["n_surf"] = np.array([surf.shape[0], tri.shape[0]])
    out["sha_surf"] = sha(surf)
    out["sha_tri"] = sha(tri)
    out["sha_faces"] = sha(faces)
    if tri.shape[0] <= FULL_MAX_TRI:   # small enough to commit in full
        out["surf_V"], out["tri"], out["faces"] = surf, tri, faces
    if "surf_E" in out:
        out["sha_surf_E"] = sha(out.pop("surf_E").astype(np.int64))
    if "skel_E" in out and out["skel_E"].shape[0] > 200_000:
        out["sha_skel"] = sha(out.pop("skel_V"), out.pop("skel_E").astype(np.int64))
    out["step_idx"] = np.array([s[0] for s in steps])
    out["step_V"] = np.array([s[1] for s in steps])
    out["step_E"] = np.array([s[2] for s in steps])
    out["step_sha"] = np.array([s[3] for s in steps])
    out["ref_seconds"] = time.time() - t0
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: V_surf={out['n_surf'][0]} tris={out['n_surf'][1]} "
          f"steps={len(steps)} {out['ref_seconds']:.1f}s -> {os.path.getsize(path)/1e3:.0f} kB")


def annotate_skeleton(name):
    """Add ``skel_dups`` to an existing skeleton golden: re-run the
    reference's skeleton on the stored weights, check it against the stored
    hash, count duplicate edges."""
    sp, model = __import__("ref_loader").import_reference()
    sys.path.insert(0, os.path.dirname(HERE))
    from golden_io import load
    d = load(name)
    net = model.Net(**d["cfg"])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in d["params"].items()})
    for m in net.modules():
        if isinstance(m, sys.modules["tropical"].TropicalHashGrid):
            V0, E0 = m.skeleton(net)
            break
    if "sha_skel" in d:
        assert sha(V0.numpy(), E0.numpy().astype(np.int64)) == str(d["sha_skel"])
    path = os.path.join(HERE, f"{name}.npz")
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    out["skel_dups"] = np.int64(E0.shape[0] - np.unique(E0.numpy(), axis=0).shape[0])
    out["skel_VE"] = np.array([V0.shape[0], E0.shape[0]])
    np.savez_compressed(path, **out)
    print(f"{name}: skeleton {tuple(out['skel_VE'])}, {out['skel_dups']} duplicate edges")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--annotate"]:
        for nm in sys.argv[2:]:
            annotate_skeleton(nm)
        sys.exit(0)
    if os.environ.get("GOLDEN_TRACE"):
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["GOLDEN_TRACE"]), exit=True)
    names = sys.argv[1:] or list(CASES)
    for nm in names:
        run_case(nm)
