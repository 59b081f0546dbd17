"""Shared test helpers: build product / oracle nets from golden fixtures and
run the device engine step by step."""
from __future__ import annotations

import numpy as np
import torch

from golden_io import sha


def product_net(d, device):
    from tropical.stanford.model import Net
    net = Net(**d["cfg"])
    net.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in d["params"].items()})
    return net.to(device)


def oracle_net(d):
    from oracle.subdivide import RefNet, load_params
    return load_params(RefNet(**d["cfg"]), d["params"])


def engine_steps(eng, record=True):
    """Every subpoly_ call of subpoly.py:60-69 on a keep_all engine; returns
    the (V, E, sha) after each call (the goldens' step records)."""
    out = []
    K = eng.K
    for idx in range(K):
        S, fail = eng.split(idx)
        if S > 0:
            eng.finish(idx, idx < K - 1, fail)
        elif out:  # nothing split: the state (and its hash) is unchanged
            out.append(out[-1])
            continue
        if record:
            v, e, p = eng.export(pre=True)
            out.append((v.shape[0], e.shape[0],
                        sha(v.cpu().numpy(), e.cpu().numpy(), p.cpu().numpy())))
    return out
