"""Deterministic synthetic SDF nets and lattices (numpy only, no package imports).

Used by ``bench.py`` (the north-star "synthetic random-weight trilinear net at
an N^3 initial grid") and by the golden generator.

* Net shape: ``Net(num_layers=3, num_hidden=16, levels=2, r_min=N-1,
  r_max=N-1, T=19)`` gives exactly N marks per axis.
* Hash table: U(-amp, amp) fp32, MLP: ``nn.Linear`` default bounds
  U(+-1/sqrt(fan_in)) -- drawn from a fixed-seed numpy PCG64 generator in a
  fixed fill order (table, then W0, b0, W1, b1, W2, b2).
* Initial edges: the full lattice in the reference's ``_skeleton(...,
  pruning=False)`` layout (tropical/tropical.py:103-109): x-edges, then y,
  then z, each ``(hi, lo)`` in meshgrid-ij order, vertex id ``i*N^2+j*N+k``.
"""
from __future__ import annotations

import numpy as np


def net_config_for_lattice(n_marks: int, T: int = 19) -> dict:
    """T < 19 hashes smaller lattices: level res = n_marks - 1 is prime-hashed
    once (n_marks - 1)^3 > 2^T (tcnn semantics)."""
    return dict(num_layers=3, num_hidden=16, levels=2, r_min=n_marks - 1,
                r_max=n_marks - 1, T=T)


def random_params(n_table: int, num_nodes, seed: int, amp: float = 0.1) -> dict:
    """Table + MLP weights drawn in a fixed order from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {"enc.module.params": rng.uniform(-amp, amp, n_table).astype(np.float32)}
    for i in range(len(num_nodes) - 1):
        fan_in, fan_out = num_nodes[i], num_nodes[i + 1]
        bound = 1.0 / np.sqrt(fan_in)
        out[f"fc.{i}.weight"] = rng.uniform(-bound, bound, (fan_out, fan_in)).astype(np.float32)
        out[f"fc.{i}.bias"] = rng.uniform(-bound, bound, fan_out).astype(np.float32)
    return out


def probe_points(seed: int, n: int = 4096) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed + 1_000_003))
    return rng.uniform(-1.0, 1.0, (n, 3)).astype(np.float32)


def center_sdf_bias(params: dict, sdf_column, seed: int) -> dict:
    """Shift the output bias so the zero level set crosses the box.

    A random-weight net is almost always one-signed on [-1,1]^3, which would
    leave the final (o1-o0) step and the surface empty.  ``sdf_column(points)``
    is the pre-tanh o1-o0 of the net with ``params`` (computed by whichever
    forward the caller owns -- the GPU kernel and the oracle are bitwise
    equal); ``fc.2.bias[1]`` is lowered by its median over a fixed probe.
    Only plane 32 changes; planes 0..31 (and their splits) are untouched.
    """
    last = max(int(k.split(".")[1]) for k in params if k.startswith("fc."))
    col = np.asarray(sdf_column(probe_points(seed)), dtype=np.float32)
    med = np.float32(np.median(col.astype(np.float64)))
    out = dict(params)
    b = out[f"fc.{last}.bias"].copy()
    b[1] = np.float32(b[1] - med)
    out[f"fc.{last}.bias"] = b
    return out


def lattice_edges(n: int) -> np.ndarray:
    """Full-lattice axis edges (E x 2 int64) in the reference's layout."""
    ids = np.arange(n ** 3, dtype=np.int64).reshape(n, n, n)
    ex = np.stack([ids[1:, :, :].reshape(-1), ids[:-1, :, :].reshape(-1)], -1)
    ey = np.stack([ids[:, 1:, :].reshape(-1), ids[:, :-1, :].reshape(-1)], -1)
    ez = np.stack([ids[:, :, 1:].reshape(-1), ids[:, :, :-1].reshape(-1)], -1)
    return np.concatenate([ex, ey, ez], 0)


def lattice_vertices(marks: np.ndarray) -> np.ndarray:
    """Vertices ``marks[idx]*2-1`` for every lattice point, id order i,j,k."""
    m = np.asarray(marks, dtype=np.float32)
    n = m.shape[0]
    g = np.stack(np.meshgrid(m, m, m, indexing="ij"), -1).reshape(-1, 3)
    return (g * np.float32(2) - np.float32(1)).astype(np.float32)


def slab_lattice(marks: np.ndarray, x0: int, x1: int):
    """The x-slab [x0, x1] (mark indices) of the full lattice, laid out as
    tnp_engine_lattice does: vertex (i, j, k) -> id (i - x0) N^2 + j N + k;
    x-edges, then y, then z, each (hi, lo) -- an order-preserving subsequence
    of lattice_edges(N) restricted to the slab, so shards number and orient
    every shared element exactly as the unsharded run does."""
    n = np.asarray(marks).shape[0]
    return block_lattice(marks, (x0, 0, 0), (x1, n - 1, n - 1))


def block_lattice(marks: np.ndarray, lo, hi):
    """The box of mark indices [lo[d], hi[d]] of the full lattice, laid out
    as tnp_engine_lattice_box does: vertex (i, j, k) -> id (i - lo0) ny nz +
    (j - lo1) nz + (k - lo2); x-edges, then y, then z, each (hi, lo)."""
    m = np.asarray(marks, dtype=np.float32)
    n = [hi[d] - lo[d] + 1 for d in range(3)]
    g = np.stack(np.meshgrid(m[lo[0]:hi[0] + 1], m[lo[1]:hi[1] + 1], m[lo[2]:hi[2] + 1], indexing="ij"),
                 -1).reshape(-1, 3)
    verts = (g * np.float32(2) - np.float32(1)).astype(np.float32)
    ids = np.arange(n[0] * n[1] * n[2], dtype=np.int64).reshape(*n)
    ex = np.stack([ids[1:, :, :].reshape(-1), ids[:-1, :, :].reshape(-1)], -1)
    ey = np.stack([ids[:, 1:, :].reshape(-1), ids[:, :-1, :].reshape(-1)], -1)
    ez = np.stack([ids[:, :, 1:].reshape(-1), ids[:, :, :-1].reshape(-1)], -1)
    return verts, np.concatenate([ex, ey, ez], 0)
