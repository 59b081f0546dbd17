"""python -m tropical.stanford.train -- the reference's entry point
(tropical/stanford/train.py) on the MI355X path.

Same flags (train.py:39-51, including the inverted `-c` and `-f`): -d
dataset, -s seed, -c disables the checkpoint cache, -m model size, -e runs
the evaluation, -f turns the flat assumption OFF (curve approximation on).
Same flow for a cached model: load the state_dict, extract the mesh with
tropical.subpoly.subpoly (prints " take T"), scale by 1/R, write
meshes/{d}/our_mesh_{m}_{seed}.ply, and with -e mesh the SDF by marching
cubes at the reference's resolutions (pseudo ground truth at 512), sample
both surfaces with 100k rays from the origin and print the
"#samples, #vertices, CD, AD, time" table (train.py:275-354).  Every step
runs on the GPU: subpoly on the HIP engine, the SDF grid through the fused
net kernel, marching cubes, ray casting and nearest neighbours in
csrc/evaluate.hip.

Without a cached model (or with -c) the net is trained first, as the
reference's loop (train.py:153-231): StanfordDataset samples (dataset.py,
signed distances by the HIP mesh kernel), batches of 1000, Adam + cosine
schedule, one closed-form gradient call per batch (csrc/train.hip), the
reference's progress lines, one subpoly per 10 batches once past 5 * EPOCH
of them, the state_dict saved to the cache path.  The Stanford scans are not
part of this repository: pass --mesh PATH (any closed PLY mesh) when the
dataset's own file is absent.  Extra flags: --weights PATH loads a
state_dict from PATH instead of the cache location; --epochs overrides
EPOCH (train.py:67).
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time

import numpy as np
import torch

import tropical.subpoly as sp
from tropical.stanford.model import Net
from tropical.utils.chamfer_distance import chamfer_distance, sample_surface_from_rays
from tropical.utils.marching_cubes import marching_cubes_torch
from tropical.utils.mesh import Mesh

DIM = 3
CANVAS_SIZE = 1.2
R = 0.8  # StanfordDataset.R (dataset.py:27): the scans are scaled into [-R, R]
MC_SIZES = [512, 16, 24, 32, 40, 48, 56, 64, 128, 192, 224, 256]


def parse_args(argv=None):
    p = argparse.ArgumentParser(prog="python -m tropical.stanford.train",
                                description="Polyhedral complex derivation from piecewise trilinear networks")
    p.add_argument("-d", "--dataset", default="dragon",
                   choices=["bunny", "dragon", "happy", "armadillo", "drill", "lucy", "bunny_npy"],
                   help="Stanford 3D scanning model name")
    p.add_argument("-s", "--seed", default=45, type=int, help="Seed")
    p.add_argument("-c", "--cache", default=True, action="store_false", help="Cache the trained SDF?")
    p.add_argument("-m", "--model_size", default="small", choices=["small", "medium", "large"],
                   help="Model size")
    p.add_argument("-e", "--eval", default=False, action="store_true", help="Run evaluation?")
    p.add_argument("-f", "--force", default=True, action="store_false",
                   help="Force flat assumption to skip curve approximation.")
    p.add_argument("--weights", default=None, help="state_dict to load instead of the cache path")
    p.add_argument("--mesh", default=None, help="training mesh (PLY) instead of the dataset's scan file")
    p.add_argument("--epochs", default=None, type=int, help="training epochs (default: the reference's EPOCH)")
    p.add_argument("--out", default="meshes", help="mesh output directory")
    return p.parse_args(argv)


def net_config(model_size: str, dataset: str) -> dict:
    """train.py:70-82 (T defaults to 19 where the reference leaves it unset)."""
    r_min, r_max = {"small": (2, 32), "medium": (4, 64), "large": (8, 128)}[model_size]
    T = 21 if (model_size == "large" and "bunny" in dataset.lower()) else 19
    return dict(num_layers=3, num_hidden=16, levels=4, r_min=r_min, r_max=r_max, T=T)


def model_path(dataset: str, model_size: str, seed: int) -> str:
    return os.path.join(os.path.dirname(__file__),
                        f"models/{dataset}/{dataset}_sdf_{model_size}_{seed}.pth")


@torch.no_grad()
def run_marching_cubes(net, n: int) -> Mesh:
    """train.py:275-293: SDF on an n^3 grid over [-C, C]^3, MC of -sdf at 0."""
    s = torch.linspace(-CANVAS_SIZE, CANVAS_SIZE, n)
    gx, gy, gz = torch.meshgrid(s, s, s, indexing="ij")
    pts = torch.stack([gx, gy, gz], dim=-1).reshape(-1, 3).to(net.device())
    sdfs = net.sdf(pts)[:, 0].reshape(n, n, n)
    v, t = marching_cubes_torch(-sdfs, 0.0)
    v = v / (n - 1.0) * 2 * CANVAS_SIZE - CANVAS_SIZE
    v = v / R
    return Mesh(v.cpu().numpy(), t.cpu().numpy())  # float64, as the reference's trimesh


def get_rays(n: int = 100000):
    """train.py:296-304 (CPU RNG, as the reference)."""
    theta = torch.rand(n) * 2 * torch.pi
    phi = torch.rand(n) * 2 * torch.pi
    x = torch.cos(theta) * torch.sin(phi)
    y = torch.sin(theta) * torch.sin(phi)
    z = torch.cos(phi)
    d = torch.stack([x, y, z], 1)
    return torch.zeros_like(d), d


def angular_distance(x, y):
    deg = np.degrees(np.arccos(np.clip(np.sum(x * y, axis=-1), -1, 1)))
    return np.mean(deg), np.std(deg)


def evaluate(net, our_mesh: Mesh, our_t: float, out_dir: str, tag: str, sizes=None):
    sizes = MC_SIZES if sizes is None else sizes
    rays_o, rays_d = get_rays()
    our_samples, our_normals, our_mask = sample_surface_from_rays(rays_o, rays_d, our_mesh,
                                                                  return_normal=True)
    print("Marching Cubes Results:")
    print("#samples, #vertices, CD, AD, time")
    gt = None
    rows = []
    for i in sizes:
        t = time.time()
        mc_mesh = run_marching_cubes(net, i)
        torch.cuda.synchronize()
        t = time.time() - t
        mc_samples, mc_normals, mc_mask = sample_surface_from_rays(rays_o, rays_d, mc_mesh,
                                                                   return_normal=True)
        if len(mc_samples) == 0:
            print(f"{i:4d}, {0:5d}, {0:0.6f}, {0:4.1f}, {t:.2f}")
            continue
        if gt is None:  # the first (512) is the pseudo ground truth
            gt = (mc_samples, mc_normals, mc_mask)
            our_cd = chamfer_distance(our_samples, gt[0])
            common = our_mask & gt[2]
            our_ad, _ = angular_distance(our_normals[common], gt[1][common])
            print(f"{'Ours'}, {our_mesh.vertices.shape[0]:5d}, {our_cd:0.6f}, {our_ad:4.1f}, {our_t:.2f}")
            rows.append(("ours", our_mesh.vertices.shape[0], our_cd, our_ad, our_t))
        mc_cd = chamfer_distance(mc_samples, gt[0])
        common = mc_mask & gt[2]
        mc_ad, _ = angular_distance(mc_normals[common], gt[1][common])
        print(f"{i:4d}, {mc_mesh.vertices.shape[0]:5d}, {mc_cd:0.6f}, {mc_ad:4.1f}, {t:.2f}")
        rows.append((i, mc_mesh.vertices.shape[0], mc_cd, mc_ad, t))
        mc_mesh.export(os.path.join(out_dir, f"mc{i:03d}_mesh_{tag}.ply"))
    print()
    return rows


BATCH_SIZE = 1000  # train.py:66


def draw_canvas(net, force: bool):
    """train.py:117-129 without the matplotlib canvas: subpoly, timed."""
    t = time.time()
    polygons, vertices, faces_with_indices = sp.subpoly(net, DIM, CANVAS_SIZE, force=force)
    torch.cuda.synchronize()
    our_t = time.time() - t
    print(f" take {our_t:.2f}")
    return polygons, vertices, faces_with_indices, our_t


def train_sdf(net, args, path: str):
    """The training loop of train.py:153-231 (no checkpoint, or -c)."""
    from tropical.stanford.dataset import StanfordDataset
    from tropical.stanford.sdf_train import SDFTrainer
    epochs = args.epochs or (6 if "drill" == args.dataset else 10)  # train.py:67
    print(f"warning: cannot find a pretrained model for seed ({args.seed})! This training code is not "
          f"guarantee the convergence of training nor a reliable SDF.", flush=True)
    training_data = StanfordDataset(args.dataset, mesh=args.mesh)
    loader = torch.utils.data.DataLoader(training_data, batch_size=BATCH_SIZE, shuffle=True)
    trainer = SDFTrainer(net, lr=1e-3, T_max=epochs * len(training_data) / BATCH_SIZE, batch_size=BATCH_SIZE)
    result = None
    for epoch in range(epochs):
        running_loss = torch.zeros((), device=net.device())
        training_data.resample()  # train.py:170 (also before the first epoch)
        for i, (inputs, labels) in enumerate(loader):
            loss, l1 = trainer.step(inputs.cuda(), labels.cuda())
            running_loss += loss
            if i % 10 == 9:
                print(f"[{epoch + 1}, {i + 1:5d}] lr: {trainer.sched.get_last_lr()[0]:.4f}, "
                      f"loss: {running_loss.item() / 10:.5f}", f"l1: {l1.item() / 10:.5f}", end="")
                running_loss.zero_()
                it = len(training_data) * epoch // BATCH_SIZE // 10 + (i + 1) // 10
                if 5 * epochs > it:
                    print(" mesh calculation skipped.")
                    continue
                result = draw_canvas(net, args.force)
    print("Finished training.", flush=True)
    if args.cache:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        torch.save(net.state_dict(), path)
    return result


def main(argv=None):
    args = parse_args(argv)
    print(args)
    seed = args.seed
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)
    if not torch.cuda.is_available():
        raise SystemExit("tropical.stanford.train needs a ROCm GPU (no CPU fallback)")
    net = Net(**net_config(args.model_size, args.dataset)).cuda()
    path = args.weights or model_path(args.dataset, args.model_size, seed)
    if (args.cache or args.weights) and os.path.isfile(path):
        sd = torch.load(path, map_location=net.device(), weights_only=True)
        net.load_state_dict(sd)
        print(f"The pretrained model loaded from {path}")
        polygons, vertices, faces_with_indices, our_t = draw_canvas(net, args.force)
    else:
        if args.weights:
            raise SystemExit(f"--weights: no file at {path}")
        result = train_sdf(net, args, path)
        if result is None:
            result = draw_canvas(net, args.force)
        polygons, vertices, faces_with_indices, our_t = result

    verts = vertices.cpu().numpy() / R
    our_mesh = Mesh(verts, np.asarray(faces_with_indices, dtype=np.int64))
    print(f"Ours: {our_mesh.vertices.shape}/{our_mesh.faces.shape}")
    out_dir = os.path.join(args.out, args.dataset)
    tag = f"{args.model_size}_{seed}"
    our_mesh.export(os.path.join(out_dir, f"our_mesh_{tag}.ply"))
    if not args.eval:
        return 0
    evaluate(net, our_mesh, our_t, out_dir, tag)
    return 0


if __name__ == "__main__":
    sys.exit(main())
