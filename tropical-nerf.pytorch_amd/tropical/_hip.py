"""ctypes binding of libtropical_hip.so (C ABI: include/tropical_hip.h).

The product path has NO CPU fallback: every op below launches a gfx950 HIP
kernel and raises if the library or a GPU is missing.  ``torch`` is imported
first so that the process uses torch's own libamdhip64 (same soname) and
torch's device memory / streams are valid handles for the library.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import torch  # noqa: F401  (must load before the HIP library)

# TNP_LIB names an alternative build of the same library (A/B kernel variants
# built in-tree under _lib/); the default is the Makefile's output
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                         os.environ.get("TNP_LIB", "libtropical_hip.so"))
MAX_LEVELS = 8


class TnpNet(C.Structure):
    _fields_ = [
        ("n_levels", C.c_int32), ("n_features", C.c_int32), ("num_layers", C.c_int32),
        ("num_hidden", C.c_int32), ("n_marks", C.c_int32), ("eps", C.c_float),
        ("scales", C.c_float * MAX_LEVELS), ("res", C.c_int32 * MAX_LEVELS),
        ("sizes", C.c_uint32 * MAX_LEVELS), ("offsets", C.c_uint32 * MAX_LEVELS),
        ("dense", C.c_int32 * MAX_LEVELS),
        ("d_table", C.c_void_p), ("d_weights", C.c_void_p), ("d_marks", C.c_void_p),
    ]


class TnpStepStats(C.Structure):
    _fields_ = [
        ("idx", C.c_int32),
        ("V_in", C.c_int64), ("E_in", C.c_int64), ("S", C.c_int64), ("H", C.c_int64),
        ("X", C.c_int64), ("V_out", C.c_int64), ("E_out", C.c_int64),
        ("A", C.c_int64), ("P", C.c_int64), ("pair_tests", C.c_int64),
        ("override_applied", C.c_int32), ("next_active", C.c_uint64), ("S_dup", C.c_int64),
        ("T", C.c_int64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# symbol -> (restype, argtypes); exactly the functions include/tropical_hip.h declares
_VP, _I64, _I32, _F = C.c_void_p, C.c_int64, C.c_int32, C.c_float
_P64, _P32, _PU64 = C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_uint64)
_NETP = C.POINTER(TnpNet)
SIGNATURES = {
    "tnp_last_error": (C.c_char_p, []),
    "tnp_abi_version": (C.c_int, []),
    "tnp_build_id": (C.c_char_p, []),
    "tnp_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "tnp_forward": (C.c_int, [_NETP, _VP, _I64, _VP, _I64, _VP, _VP]),
    "tnp_encode": (C.c_int, [_NETP, _VP, _I64, _VP, _VP]),
    "tnp_forward_grouped": (C.c_int, [_NETP, _VP, _I64, _VP, _I64, _VP, _VP]),
    "tnp_region": (C.c_int, [_NETP, _VP, _VP, _I64, _I64, _F, _VP, _VP, _VP]),
    "tnp_sdf_grad": (C.c_int, [_NETP, _VP, _I64, _VP, _VP, _VP]),
    "tnp_sdf_train_grad": (C.c_int, [_NETP, _VP, _VP, _I64, _F, _F, _I64, _VP, _VP, _VP, _VP]),
    "tnp_mesh_signed_distance": (C.c_int, [_VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP, _VP]),
    "tnp_sdf_vjp": (C.c_int, [_NETP, _VP, _VP, _I64, _VP, _VP, _VP]),
    "tnp_normal_vjp": (C.c_int, [_NETP, _VP, _VP, _I64, _VP, _VP, _VP, _VP]),
    "tnp_forward_vjp": (C.c_int, [_NETP, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _VP, _VP]),
    "tnp_engine_create": (C.c_int, [C.POINTER(_VP), C.c_int]),
    "tnp_engine_destroy": (None, [_VP]),
    "tnp_engine_set_net": (C.c_int, [_VP, _NETP]),
    "tnp_engine_scratch_bytes": (C.c_int, [_VP, _P64, _P64, _P64]),
    "tnp_engine_skeleton_gmax": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, _VP, _VP, C.c_int,
                                           C.POINTER(C.c_int), _VP]),
    "tnp_engine_skeleton_box": (C.c_int, [_VP, C.c_int, _P32, _P32, _VP, C.c_int, _VP, _P64, _P64]),
    "tnp_engine_load": (C.c_int, [_VP, _VP, _I64, _VP, _I64, _VP, C.c_int, _VP]),
    "tnp_engine_skeleton": (C.c_int, [_VP, C.c_int, _F, _VP, _P64, _P64]),
    "tnp_shm_open": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "tnp_shm_unlink": (C.c_int, [C.c_char_p]),
    "tnp_shm_close": (None, [_VP]),
    "tnp_shm_allreduce": (C.c_int, [_VP, _VP, C.c_int, C.c_int, _VP]),
    "tnp_engine_skeleton_mode": (C.c_int, [_VP, C.c_int, _F, C.c_int, _VP, _P64, _P64]),
    "tnp_engine_lattice": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, _VP, _P64, _P64]),
    "tnp_engine_lattice_box": (C.c_int, [_VP, _P32, _P32, C.c_int, _VP, _P64, _P64]),
    "tnp_engine_active_planes": (C.c_int, [_VP, C.c_int, _PU64, _VP]),
    "tnp_engine_split": (C.c_int, [_VP, C.c_int, _VP, _P64, _P32]),
    "tnp_engine_finish": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, _VP, C.POINTER(TnpStepStats)]),
    "tnp_engine_sizes": (C.c_int, [_VP, _P64, _P64]),
    "tnp_engine_split_keep": (C.c_int, [_VP, _VP, _I64, _VP]),
    "tnp_engine_export": (C.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "tnp_engine_surface": (C.c_int, [_VP, _VP, _P64, _P64]),
    "tnp_engine_faces": (C.c_int, [_VP, _VP, _P64, _P64]),
    "tnp_engine_faces_export": (C.c_int, [_VP, _VP, _VP, _VP]),
    "tnp_engine_set_owned": (C.c_int, [_VP, C.c_int, C.c_int]),
    "tnp_engine_set_xspan": (C.c_int, [_VP, C.c_int, C.c_int]),
    "tnp_engine_set_owned_box": (C.c_int, [_VP, _P32, _P32]),
    "tnp_engine_set_span": (C.c_int, [_VP, _P32, _P32]),
    "tnp_engine_set_eps": (C.c_int, [_VP, C.c_float]),
    "tnp_engine_run_steps": (C.c_int, [_VP, _VP, C.POINTER(TnpStepStats), C.c_int, _P32]),
    "tnp_engine_set_curve": (C.c_int, [_VP, C.c_int]),
    "tnp_engine_set_strict": (C.c_int, [_VP, C.c_int]),
    "tnp_engine_set_collective": (C.c_int, [_VP, _VP, _VP]),
    "tnp_engine_set_shards": (C.c_int, [_VP, C.c_int]),
    "tnp_debug_ops": (C.c_int, [_VP, _VP, _VP, C.c_int64, _VP, _VP]),
    "tnp_debug_descend": (C.c_int, [_NETP, _VP, _VP, _VP, C.c_int64, C.c_int, C.c_float, C.c_int, _VP, _VP,
                                    C.c_int, _VP]),
    "tnp_engine_faces_debug": (C.c_int, [_VP, _VP, C.c_int64, _P64, _P64, _VP]),
    "tnp_engine_debug_set_lb_spin": (C.c_int, [_VP, C.c_int]),
    "tnp_debug_buf_growth": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.c_int, _P64, _P64]),
    "tnp_engine_debug_set_lds_records": (C.c_int, [_VP, C.c_int]),
    "tnp_engine_debug_vertex_capacity": (C.c_int, [_VP, _P64, _P64]),
    "tnp_engine_debug_lb_recomputes": (C.c_int, [_VP, _P64, C.c_int, _VP]),
    "tnp_engine_kernel_timer": (C.c_int, [_VP, C.c_int, _VP, _P32]),
    "tnp_mc_count": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, _F, _VP, _VP, _VP, _P64, _P64, _VP]),
    "tnp_mc_emit": (C.c_int, [_VP, C.c_int, C.c_int, C.c_int, _F, _VP, _VP, _VP, _VP, _VP, _VP]),
    "tnp_raycaster_create": (C.c_int, [C.POINTER(_VP), C.c_int]),
    "tnp_raycaster_destroy": (None, [_VP]),
    "tnp_raycaster_build": (C.c_int, [_VP, _VP, _I64, _VP, _I64, C.POINTER(C.c_float),
                                      C.POINTER(C.c_float), _VP]),
    "tnp_raycaster_cast": (C.c_int, [_VP, _VP, _VP, _I64, _VP, _VP, _VP]),
    "tnp_nn_min_dist": (C.c_int, [_VP, _I64, _VP, _I64, _VP, _VP]),
    "tnp_engine_kernel_stat": (C.c_int, [_VP, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_double),
                                         _P64, C.POINTER(C.c_double)]),
}

_lib = None


def lib():
    """Load the library (raises loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.isfile(_LIB_PATH):
            raise RuntimeError(
                f"tropical HIP library not built: {_LIB_PATH} is missing "
                "(run `make -C tropical-nerf.pytorch_amd/csrc` or __graft_entry__.build())")
        L = C.CDLL(_LIB_PATH)
        # TNP_LIB_ANY_BUILD=1 (timing experiments on a TNP_LIB variant built
        # from other sources, tools/): no build-id check, missing entry
        # points left unbound.  Never the default: the product loads only a
        # library built from this tree's sources.
        any_build = os.environ.get("TNP_LIB_ANY_BUILD") == "1" and "TNP_LIB" in os.environ
        if any_build:
            import warnings
            warnings.warn(f"TNP_LIB_ANY_BUILD=1: loading {_LIB_PATH} without the build-id check "
                          "(timing experiments only; missing entry points stay unbound)", RuntimeWarning,
                          stacklevel=2)
            print(f"[tropical] TNP_LIB_ANY_BUILD=1: {os.path.basename(_LIB_PATH)} loaded without the "
                  "build-id check", file=sys.stderr, flush=True)
        for name, (res, args) in SIGNATURES.items():
            if any_build and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        from ._buildid import build_id
        want, got = build_id(), L.tnp_build_id().decode()
        if want is not None and got != want and not any_build:
            raise RuntimeError(
                f"tropical HIP library {_LIB_PATH} is stale: built from sources {got}, the tree's "
                f"are {want} (rebuild: `make -C tropical-nerf.pytorch_amd/csrc` or __graft_entry__.build())")
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().tnp_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}")


def require_cuda(t: torch.Tensor, what: str):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError(f"{what}: the tropical HIP path needs tensors on a ROCm GPU "
                           f"(got {getattr(t, 'device', type(t))}); there is no CPU fallback")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())
