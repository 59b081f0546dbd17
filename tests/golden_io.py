"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
from __future__ import annotations

import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def cases(kind=None):
    out = []
    for f in sorted(os.listdir(GOLDEN)):
        if f.endswith(".npz"):
            d = load(f[:-4])
            if kind is None or str(d["kind"]) == kind:
                out.append(f[:-4])
    return out


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["cfg"] = {str(k): int(v) for k, v in zip(d["cfg_keys"], d["cfg_vals"])}
    d["params"] = {k[2:]: v for k, v in d.items() if k.startswith("p:")}
    return d
