"""Import the *reference* package (``/root/reference/tropical``) in THIS
container only, to generate golden fixtures.  Never used on the GPU box and
never imported by the product.

The reference imports a few third-party modules that are absent here
(SURVEY §8c): ``tinycudann`` (replaced by the oracle's restatement of the
tcnn Grid/Hash encoding, so goldens and the build share one encoding
definition), ``deprecation`` (a no-op decorator factory) and
``trimesh``/``cubvh``/``mcubes`` (imported but unused on the extraction path).

``torch.Tensor.argsort`` is patched to ``stable=True`` so that
``r_idx_as_tensor`` (subpoly.py:357) has the reference-on-CUDA semantics
(SURVEY finding 4).
"""
from __future__ import annotations

import os
import sys
import types

REF_ROOT = os.environ.get("TROPICAL_REFERENCE", "/root/reference")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def import_reference():
    sys.dont_write_bytecode = True
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    from oracle.encoding import GridHashEncoding
    import torch

    tcnn = types.ModuleType("tinycudann")
    tcnn.Encoding = GridHashEncoding
    sys.modules["tinycudann"] = tcnn

    dep = types.ModuleType("deprecation")
    dep.deprecated = lambda *a, **k: (lambda f: f)
    sys.modules["deprecation"] = dep
    for name in ("trimesh", "cubvh", "mcubes"):
        sys.modules.setdefault(name, types.ModuleType(name))

    if not getattr(torch.Tensor.argsort, "_stable_patch", False):
        _orig = torch.Tensor.argsort

        def _stable_argsort(self, *args, **kwargs):
            kwargs["stable"] = True
            return _orig(self, *args, **kwargs)

        _stable_argsort._stable_patch = True
        torch.Tensor.argsort = _stable_argsort

    sys.path.insert(0, REF_ROOT)
    import tropical  # noqa: F401  (the reference package)
    import tropical.subpoly as sp
    import tropical.stanford.model as model
    assert os.path.abspath(tropical.__file__).startswith(os.path.abspath(REF_ROOT))
    return sp, model
