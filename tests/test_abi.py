"""CPU: the C-ABI library builds, loads and exports exactly what
include/*.h declare -- the product surface tropical_hip.h and the
diagnostics tropical_hip_debug.h (no compute calls without a GPU)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("tropical_hip.h", "tropical_hip_debug.h")]


def declared_symbols(headers=HEADERS):
    syms = set()
    for h in headers:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms |= set(re.findall(r"\b(tnp_[a-z0-9_]+)\s*\(", src))
    return sorted(syms)


def test_header_declares_engine_and_net_ops():
    syms = declared_symbols()
    for s in ("tnp_forward", "tnp_region", "tnp_sdf_grad", "tnp_engine_split",
              "tnp_engine_finish", "tnp_engine_skeleton", "tnp_engine_faces"):
        assert s in syms


def test_debug_entry_points_stay_out_of_the_product_header():
    product = declared_symbols(HEADERS[:1])
    debug = declared_symbols(HEADERS[1:])
    assert debug and not set(debug) & set(product)
    assert all("debug" in s for s in debug)


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


def test_build_id_rules_agree():
    """csrc/build_id.sh (compiled into the library) and tropical/_buildid.py
    (the loader's check) hash the same sources the same way."""
    import subprocess
    from tropical._buildid import CSRC, build_id
    sh = subprocess.run(["sh", os.path.join(CSRC, "build_id.sh")], capture_output=True, text=True, check=True)
    assert sh.stdout.strip() == build_id()


def test_stale_library_is_refused(monkeypatch):
    """A prebuilt library whose sources differ from the tree's (tnp_build_id)
    must not load: the GPU box runs whatever .so travels with the tree."""
    from tropical import _buildid, _hip
    good = _hip.lib()
    assert good.tnp_build_id().decode() == _buildid.build_id()
    monkeypatch.setattr(_hip, "_lib", None)
    monkeypatch.setattr(_buildid, "build_id", lambda: "0000000000000000")
    with pytest.raises(RuntimeError, match="stale"):
        _hip.lib()
