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
            with np.load(os.path.join(GOLDEN, f), allow_pickle=False) as z:
                if "kind" not in z.files:  # not a subpoly case (descend_cases.npz)
                    continue
            d = load(f[:-4])
            if kind is None or str(d["kind"]) == kind:
                out.append(f[:-4])
    return out


def golden_eps(d) -> float:
    """The eps argument the golden's subpoly calls used (make_golden.py EPS)."""
    return float(d["eps"]) if "eps" in d else 1e-4


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["cfg"] = {str(k): int(v) for k, v in zip(d["cfg_keys"], d["cfg_vals"])}
    params = {}
    if "gen" in d:
        # large tables are stored as their generator spec (make_golden.py GEN_MAX)
        from tropical.synthetic import random_params
        c = d["cfg"]
        nodes = [c["levels"] * 2] + [c["num_hidden"]] * (c["num_layers"] - 1) + [2]
        seed, amp, n_table = d["gen"]
        params = random_params(int(n_table), nodes, int(seed), float(amp))
    # stored values override (fp16-stored fits are exact in fp32)
    params.update({k[2:]: v.astype(np.float32) for k, v in d.items() if k.startswith("p:")})
    d["params"] = params
    return d


def heavy(name: str) -> bool:
    """Cases whose reference run took minutes (large net, 64^3+ lattices):
    the CPU suite skips re-running the oracle on them unless TNP_SLOW=1."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return float(z["ref_seconds"]) > 60.0
