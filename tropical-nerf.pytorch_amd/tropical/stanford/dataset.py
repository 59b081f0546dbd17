"""StanfordDataset: the training samples of the reference's SDF training
(tropical/stanford/dataset.py:25-99) -- points near the scanned surface and
their signed distances (inside positive), resampled every epoch.

Same names, paths and sampling as the reference: the mesh of each dataset
name under tropical/stanford/ (dataset.py:36-67; ``mesh=`` takes any PLY
path or a Mesh instead -- the scans are not part of this repository),
normalised to [-1, 1] (dataset.py:71-74), 50,000 points per epoch drawn
from the (10x repeated) vertices plus uniform jitter of width 0.4
(dataset.py:80-90).  The signed distances are the HIP kernel's
(``mesh_signed_distance``, replacing cubvh); the samples stay on the host
as in the reference.

Attribution: the normalisation and the resampling rule restate
seonghunn/tropical-nerf.pytorch (tropical/stanford/dataset.py:69-96),
licensed CC BY-SA 4.0; the training distribution has to match it.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils.mesh import Mesh, load_ply
from .sdf_train import mesh_signed_distance

BASE_DIR = os.path.dirname(__file__)


def mesh_path(name: str) -> str:
    """The reference's file for each dataset name (dataset.py:37-67)."""
    n = name.lower()
    if n == "bunny":
        return os.path.join(BASE_DIR, f"{n}/reconstruction/bun_zipper.ply")
    if n == "bunny_npy":
        return os.path.join(BASE_DIR, "models/bunny.npy")
    if n == "armadillo":
        return os.path.join(BASE_DIR, f"{n}/{name.capitalize()}.ply")
    if n == "drill":
        return os.path.join(BASE_DIR, f"{n}/reconstruction/{name}_shaft_vrip.ply")
    if n == "lucy":
        return os.path.join(BASE_DIR, f"{n}/{name}_res10.ply")
    return os.path.join(BASE_DIR, f"{name}_recon/{name}_vrip_res3.ply")


class StanfordDataset(torch.utils.data.Dataset):
    def __init__(self, name: str = "dragon", mesh=None, device=None):
        self.R = .8
        self.name = name
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.init(mesh)
        self.resample()

    def __len__(self):
        return 50000

    def init(self, mesh=None):
        if isinstance(mesh, Mesh):
            m = mesh
        else:
            path = mesh or mesh_path(self.name)
            if not os.path.isfile(path):
                raise FileNotFoundError(f"{self.name}: no mesh at {path} (the Stanford scans are not part of "
                                        f"this repository; pass mesh=PATH)")
            print(f"Loading {os.path.basename(path)} ...")
            if path.endswith(".npy"):
                # bunny_npy: marching cubes of the density grid (dataset.py:41-48)
                from ..utils.marching_cubes import marching_cubes_torch
                grid = np.load(path)  # allow_pickle=False
                v, t = marching_cubes_torch(torch.from_numpy(np.ascontiguousarray(grid, dtype=np.float32))
                                            .to(self.device), 0.0)
                v = (v.cpu().numpy() / 32 - 1).astype(np.float32) * self.R
                m = Mesh(v, t.cpu().numpy())
            else:
                m = load_ply(path)
        print("Done.", flush=True)
        vertices = torch.tensor(m.vertices, dtype=torch.float32)
        if "bunny_npy" != self.name.lower():
            scale = (vertices.max(dim=0)[0] - vertices.min(dim=0)[0]).max()
            vertices = vertices / scale * 2
            vertices -= (vertices.max(dim=0)[0] + vertices.min(dim=0)[0]) / 2
        self.vertices = vertices
        self.faces = torch.as_tensor(np.asarray(m.faces, dtype=np.int64))
        self.V = vertices.to(self.device)
        self.F = self.faces.to(self.device, torch.int32)
        print("BVH initialized.", flush=True)

    def resample(self):
        vertices = self.vertices
        if "lucy" != self.name.lower():  # lucy has too many vertices (dataset.py:83)
            vertices = vertices.repeat(10, 1)
        d = 0.4
        if vertices.shape[0] < len(self):  # few vertices (dataset.py:86-88)
            vertices = self.vertices.repeat(30, 1)
            d = 0.2
        points = vertices[torch.randperm(vertices.shape[0])[:len(self)]] + \
            (torch.rand(len(self), 3) * d - d / 2)
        distances = mesh_signed_distance(self.V, self.F, points.to(self.device))
        self.X = points
        self.Y = distances.cpu()  # inside is positive

    def __getitem__(self, idx):
        return self.X[idx], self.Y[idx]
