"""Build provenance of libtropical_hip.so.

The Makefile compiles a hash of the library's sources into it
(csrc/build_id.sh -> ``tnp_build_id()``); ``build_id()`` below is the same
rule over the sources next to this package.  ``_hip.lib()`` compares the two
and refuses a library built from other sources (a stale prebuilt .so).
"""
from __future__ import annotations

import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # tropical-nerf.pytorch_amd
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")


def source_files():
    """(label, path) of every hashed source; None when the sources are not
    next to the package (an installed copy)."""
    if not (os.path.isdir(CSRC) and os.path.isdir(INCLUDE)):
        return None
    out = [(f"include/{f}", os.path.join(INCLUDE, f)) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    out += [(f"csrc/{f}", os.path.join(CSRC, f)) for f in os.listdir(CSRC)
            if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile"]
    return out


def build_id():
    files = source_files()
    if files is None:
        return None
    lines = []
    for label, path in files:
        with open(path, "rb") as fh:
            lines.append(f"{label} {hashlib.sha256(fh.read()).hexdigest()}\n")
    return hashlib.sha256("".join(sorted(lines)).encode()).hexdigest()[:16]


if __name__ == "__main__":
    print(build_id())
