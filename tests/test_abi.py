"""CPU: the C-ABI library builds, loads and exports exactly what
include/tropical_hip.h declares (no compute calls without a GPU)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tropical_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tnp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_engine_and_net_ops():
    syms = declared_symbols()
    for s in ("tnp_forward", "tnp_region", "tnp_sdf_grad", "tnp_engine_split",
              "tnp_engine_finish", "tnp_engine_skeleton", "tnp_engine_faces"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from tropical import _hip
    lib = _hip.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.tnp_abi_version() == 1


def test_ctypes_table_matches_header():
    from tropical import _hip
    assert sorted(_hip.SIGNATURES) == declared_symbols()


def test_product_has_no_cpu_fallback():
    import torch
    from tropical.stanford.model import Net
    net = Net()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        net(torch.zeros(2, 3))


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "tropical-nerf.pytorch_amd", "tropical")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r'""".*?"""', "", txt, flags=re.S).replace(
                    "# oracle", ""), f
