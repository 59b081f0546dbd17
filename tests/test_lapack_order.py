"""CPU: the fp32 restatement of reference LAPACK's sgeev for the curve
path's companion matrices (tools/lapack_eig_port.py; the device code is
csrc/curve.hip SmallEig) picks the same "last real root in [0, 1]"
(geometry.py:292-296) as torch.linalg.eigvals -- the reference's call -- on
this host.  Roots that are clustered within 1e-3 are ill-conditioned in
fp32: there the order position is compared, not the value."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from lapack_eig_port import companion, f32, sgeev_values  # noqa: E402


def _last_index(r):
    m = (np.abs(r.imag) <= 1e-9) & (r.real >= 0) & (r.real <= 1)
    idx = np.nonzero(m)[0]
    return None if len(idx) == 0 else int(idx[-1])


def test_last_root_in_unit_interval_matches_torch():
    rng = np.random.default_rng(11)
    n = same = 0
    for _ in range(600):
        N = int(rng.choice([3, 4]))
        roots = rng.uniform(-0.5, 1.5, N)
        if np.min(np.diff(np.sort(roots))) < 1e-3:
            continue
        c = (np.poly(roots)[::-1] * rng.uniform(0.5, 2)).astype(f32)
        C = companion(c)
        a = torch.linalg.eigvals(torch.from_numpy(C)).numpy()
        b = sgeev_values(C)
        ia, ib = _last_index(a), _last_index(b)
        n += 1
        if ia == ib and (ia is None or abs(a[ia].real - b[ib].real) < 1e-3):
            same += 1
    assert n > 500 and same >= n - 2, f"{same}/{n}"
