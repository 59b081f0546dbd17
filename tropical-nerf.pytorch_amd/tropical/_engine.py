"""Python handle on the device-resident extraction engine (tnp_engine_*).

The engine keeps the polyhedral complex (vertices, edges, the plane-major
pre-activation cache and packed eps-sign keys) in HBM across all hyperplane
steps; Python only sequences the steps and reads back the sizes the next
allocation needs.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np
import torch

from . import _hip



# tnp_collective_fn (include/tropical_hip.h): ops TNP_COLL_SUM / _MAX / _AND / _OR
_COLL_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_int64), C.c_int, C.c_int, C.c_void_p)
_COLL_OPS = {0: "sum", 1: "max", 2: "and", 3: "or"}


def _collective_callback(allreduce):
    """The engine's collective as a C callback over the host-language
    ``allreduce(vec, op)``; the returned object must stay alive while the
    engine may call it."""
    def fn(ptr, n, op, ctx):
        try:
            name = _COLL_OPS[op]
            v = np.ctypeslib.as_array(ptr, shape=(n,))
            if name in ("and", "or"):
                r = np.asarray(allreduce(v.copy().view(np.uint64), name), dtype=np.uint64).view(np.int64)
            else:
                r = np.asarray(allreduce(v.copy(), name), dtype=np.int64)
            v[:] = r
            return 0
        except Exception:  # noqa: BLE001 -- reported by the engine as a failed collective
            import traceback
            traceback.print_exc()
            return 1
    return _COLL_FN(fn)

class Engine:
    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("Engine needs a ROCm GPU device")
        h = C.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        with torch.cuda.device(idx):
            _hip.check(_hip.lib().tnp_engine_create(C.byref(h), idx), "tnp_engine_create")
        self.h = h
        self._keep = None
        self._sharded = False
        self.K = None
        self._fin = weakref.finalize(self, _hip.lib().tnp_engine_destroy, h)

    @property
    def _s(self):
        return C.c_void_p(_hip.stream_ptr(self.device))

    def set_net(self, net):
        s, keep = net.tnp_desc()
        self._keep = (s, keep)  # the engine reads these device buffers later
        self.K = net.K
        self.net_eps = float(net.eps)
        self.num_hidden = net.num_hidden
        self.num_layers = net.num_layers
        _hip.check(_hip.lib().tnp_engine_set_net(self.h, C.byref(s)), "tnp_engine_set_net")
        return self

    # -- complex I/O ---------------------------------------------------------
    def load(self, vertices: torch.Tensor, edges: torch.Tensor, pre: torch.Tensor = None,
             keep_all: bool = False):
        v = vertices.detach().to(self.device, torch.float32).contiguous()
        e = edges.detach().to(self.device, torch.int64).contiguous()
        p = None if pre is None else pre.detach().to(self.device, torch.float32).contiguous()
        _hip.check(_hip.lib().tnp_engine_load(self.h, _hip.ptr(v), v.shape[0], _hip.ptr(e),
                                              e.shape[0], _hip.ptr(p), int(keep_all), self._s),
                   "tnp_engine_load")
        return v.shape[0], e.shape[0]

    def lattice(self, x0: int = 0, x1: int = -1, keep_all: bool = False):
        n_marks = int(self._keep[0].n_marks)
        x1 = n_marks - 1 if x1 < 0 else x1
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_lattice(self.h, x0, x1, int(keep_all), self._s,
                                                 C.byref(V), C.byref(E)), "tnp_engine_lattice")
        return V.value, E.value

    @staticmethod
    def _i3(v):
        a = (C.c_int32 * 3)(*[int(x) for x in v])
        return a

    def lattice_box(self, lo, hi, keep_all: bool = False):
        """The lattice over the marks restricted to the box of mark indices
        [lo[d], hi[d]] per axis (a block of a sharded lattice; the whole grid
        is lattice())."""
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_lattice_box(self.h, self._i3(lo), self._i3(hi), int(keep_all), self._s,
                                                     C.byref(V), C.byref(E)), "tnp_engine_lattice_box")
        return V.value, E.value

    SKELETON_MODES = {"distance": 0, "sign": 1}

    def skeleton(self, unit: int = 128, size: float = None, mode: str = "distance"):
        """mode: the reference's PRUNING_MODE (tropical.py:184-205)."""
        if mode not in self.SKELETON_MODES:
            raise ValueError(f"skeleton pruning mode {mode!r}: 'distance' or 'sign'")
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_skeleton_mode(self.h, unit, float(size or 0.0),
                                                       self.SKELETON_MODES[mode], self._s,
                                                       C.byref(V), C.byref(E)),
                   "tnp_engine_skeleton_mode")
        return V.value, E.value

    def skeleton_gmax(self, unit: int = 128, rank: int = 0, world: int = 1):
        """The tiles t % world == rank of the distance-mode skeleton evaluated
        whole (tnp_engine_skeleton_gmax): (uint32 max |grad sdf| bits per tile,
        0 for the others; int64 [3, n_marks] per-plane load of those tiles)."""
        n_marks = int(self._keep[0].n_marks)
        cap = 4096
        gmax = np.zeros(cap, dtype=np.uint32)
        load = np.zeros((3, n_marks), dtype=np.int64)
        nt = C.c_int()
        _hip.check(_hip.lib().tnp_engine_skeleton_gmax(self.h, unit, rank, world, gmax.ctypes.data,
                                                       load.ctypes.data, cap, C.byref(nt), self._s),
                   "tnp_engine_skeleton_gmax")
        return gmax[: nt.value].copy(), load

    def skeleton_box(self, lo, hi, gmax, unit: int = 128):
        """The skeleton inside the mark box [lo, hi] (tnp_engine_skeleton_box),
        every tile's max |grad sdf| bits in gmax: (V, E) loaded."""
        g = np.ascontiguousarray(np.asarray(gmax, dtype=np.uint32))
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_skeleton_box(self.h, unit, self._i3(lo), self._i3(hi), g.ctypes.data,
                                                      int(g.shape[0]), self._s, C.byref(V), C.byref(E)),
                   "tnp_engine_skeleton_box")
        return V.value, E.value

    def sizes(self):
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_sizes(self.h, C.byref(V), C.byref(E)), "tnp_engine_sizes")
        return V.value, E.value

    def scratch_bytes(self) -> dict:
        """Device memory the engine holds (tnp_engine_scratch_bytes): the sum
        over its buffers, how many are allocated, the connect key buffer."""
        b, n, k = C.c_int64(), C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_scratch_bytes(self.h, C.byref(b), C.byref(n), C.byref(k)),
                   "tnp_engine_scratch_bytes")
        return {"bytes": b.value, "buffers": n.value, "key_bytes": k.value}

    def vertex_capacity(self) -> dict:
        """(debug) the vertex set's row capacity and the steps whose split
        count exceeded the early forward's row bound (forward run again)."""
        r, x = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_debug_vertex_capacity(self.h, C.byref(r), C.byref(x)),
                   "tnp_engine_debug_vertex_capacity")
        return {"rows": r.value, "early_redo": x.value}

    def export(self, pre: bool = False, edges: bool = True):
        """(vertices [V, 3], edges [E, 2] int64 or None when edges=False,
        cache [V, K] when pre) of the compacted complex."""
        V, E = self.sizes()
        verts = torch.empty(V, 3, device=self.device)
        edges = torch.empty(E, 2, dtype=torch.int64, device=self.device) if edges else None
        cache = torch.empty(V, self.K, device=self.device) if pre else None
        _hip.check(_hip.lib().tnp_engine_export(self.h, _hip.ptr(verts), _hip.ptr(edges),
                                                _hip.ptr(cache), self._s), "tnp_engine_export")
        return verts, edges, cache

    def set_curve(self, on: bool):
        """subpoly_(force=False) semantics for the following steps."""
        _hip.check(_hip.lib().tnp_engine_set_curve(self.h, int(on)), "tnp_engine_set_curve")
        self.curve = bool(on)
        return self

    def set_strict(self, on: bool):
        """Curve path: subpoly_(strict=on) (subpoly.py:198-203); False keeps
        every split (no strict_check)."""
        _hip.check(_hip.lib().tnp_engine_set_strict(self.h, int(on)), "tnp_engine_set_strict")
        return self

    def set_shards(self, world: int):
        _hip.check(_hip.lib().tnp_engine_set_shards(self.h, int(world)), "tnp_engine_set_shards")
        self._sharded = int(world) > 1
        return self

    def set_owned(self, lo: int = 1, hi: int = 0):
        """This shard owns mark planes (lo, hi] and the cells between
        (lo > hi: everything); splits outside are reported as S_dup."""
        _hip.check(_hip.lib().tnp_engine_set_owned(self.h, int(lo), int(hi)), "tnp_engine_set_owned")

    def set_owned_box(self, lo, hi):
        """Along axis d this shard owns mark planes (lo[d], hi[d]] and the
        cells between (lo[d] > hi[d]: the axis is not cut)."""
        _hip.check(_hip.lib().tnp_engine_set_owned_box(self.h, self._i3(lo), self._i3(hi)),
                   "tnp_engine_set_owned_box")

    def set_eps(self, eps: float = None):
        """subpoly's eps argument (None: Net.eps): the steps' sign test, split
        point, hits and failover, the surface and the faces take it; the
        region keys stay at Net.eps (subpoly.py:24, 90, 556-606)."""
        e = self.net_eps if eps is None else float(eps)
        _hip.check(_hip.lib().tnp_engine_set_eps(self.h, C.c_float(e)), "tnp_engine_set_eps")
        return self

    def set_xspan(self, x0: int = 0, x1: int = -1):
        """The loaded complex lies between x mark planes x0 and x1 (a slab
        with its halo; x1 < x0: anywhere): the step's spatial buckets cover
        only those cells.  lattice() sets it, load()/skeleton() reset it."""
        _hip.check(_hip.lib().tnp_engine_set_xspan(self.h, int(x0), int(x1)), "tnp_engine_set_xspan")
        return self

    def set_span(self, lo, hi):
        """Per axis, the loaded complex lies between mark planes lo[d] and
        hi[d] (hi[d] < lo[d]: anywhere along d)."""
        _hip.check(_hip.lib().tnp_engine_set_span(self.h, self._i3(lo), self._i3(hi)), "tnp_engine_set_span")
        return self

    def kernel_timer(self, on: bool):
        """on=True: start HIP-event timing of every engine launch; on=False:
        stop and return {kernel: {"ms", "launches", "bytes"}}."""
        n = C.c_int32()
        _hip.check(_hip.lib().tnp_engine_kernel_timer(self.h, int(on), self._s, C.byref(n)),
                   "tnp_engine_kernel_timer")
        out = {}
        for i in range(n.value):
            name = C.create_string_buffer(64)
            ms, nl, by = C.c_double(), C.c_int64(), C.c_double()
            _hip.check(_hip.lib().tnp_engine_kernel_stat(self.h, i, name, 64, C.byref(ms), C.byref(nl),
                                                         C.byref(by)), "tnp_engine_kernel_stat")
            out[name.value.decode()] = {"ms": ms.value, "launches": nl.value, "bytes": by.value}
        return out

    def debug_lds_records(self, on: bool):
        """The grouping kernel's LDS-record path on / off (csrc/bucket.hip;
        off: every bucket's records go through memory)."""
        _hip.check(_hip.lib().tnp_engine_debug_set_lds_records(self.h, int(bool(on))),
                   "tnp_engine_debug_set_lds_records")
        return self

    def debug_lb(self, spin: int = None, reset: bool = True) -> int:
        """Diagnostics of the ticket-free look-back (common.h lb_prefix_rc):
        spin != None sets the polls before a recompute (0: always recompute,
        -1: the kernels' defaults); returns the recomputes counted since the
        last reset."""
        if spin is not None:
            _hip.check(_hip.lib().tnp_engine_debug_set_lb_spin(self.h, int(spin)),
                       "tnp_engine_debug_set_lb_spin")
        n = C.c_int64()
        _hip.check(_hip.lib().tnp_engine_debug_lb_recomputes(self.h, C.byref(n), int(reset), self._s),
                   "tnp_engine_debug_lb_recomputes")
        return n.value

    # -- steps ---------------------------------------------------------------
    def active_planes(self, start: int = 0) -> int:
        m = C.c_uint64()
        _hip.check(_hip.lib().tnp_engine_active_planes(self.h, start, C.byref(m), self._s),
                   "tnp_engine_active_planes")
        return m.value

    def split(self, idx: int):
        S, fail = C.c_int64(), C.c_int32()
        _hip.check(_hip.lib().tnp_engine_split(self.h, idx, self._s, C.byref(S), C.byref(fail)),
                   "tnp_engine_split")
        return S.value, int(fail.value)  # -1: left on the device (single-device flat)

    def finish(self, idx: int, prune: bool, override: bool) -> dict:
        st = _hip.TnpStepStats()
        _hip.check(_hip.lib().tnp_engine_finish(self.h, idx, int(prune), int(override), self._s,
                                                C.byref(st)), "tnp_engine_finish")
        return st.as_dict()

    def split_keep(self, n: int) -> torch.Tensor:
        """Curve path: the strict filter's keep flags of the last step's n
        candidate splits (edge order)."""
        keep = torch.empty(n, dtype=torch.int32, device=self.device)
        _hip.check(_hip.lib().tnp_engine_split_keep(self.h, _hip.ptr(keep), n, self._s),
                   "tnp_engine_split_keep")
        return keep.bool()

    def surface(self):
        V, E = C.c_int64(), C.c_int64()
        _hip.check(_hip.lib().tnp_engine_surface(self.h, self._s, C.byref(V), C.byref(E)),
                   "tnp_engine_surface")
        return V.value, E.value

    def faces(self, host: bool = False):
        """(faces_with_indices [F, 3] int64, faces [F', 3, 3] float); host=True:
        in pinned host memory, copied by DMA straight from the engine's
        buffers (what subpoly() returns as numpy arrays)."""
        nt, nf = C.c_int64(), C.c_int64()
        s = self._s
        _hip.check(_hip.lib().tnp_engine_faces(self.h, s, C.byref(nt), C.byref(nf)),
                   "tnp_engine_faces")
        where = dict(device="cpu", pin_memory=True) if host else dict(device=self.device)
        tri = torch.empty(nt.value, 3, dtype=torch.int64, **where)
        fc = torch.empty(nf.value, 3, 3, **where)
        _hip.check(_hip.lib().tnp_engine_faces_export(self.h, _hip.ptr(tri), _hip.ptr(fc), s),
                   "tnp_engine_faces_export")
        if host:
            torch.cuda.current_stream(self.device).synchronize()  # (the stream of self._s)
        return tri, fc

    # -- the hot loop (subpoly.py:58-69) -------------------------------------
    def run_steps(self, stats: list = None, allreduce=None):
        """All hyperplane steps with empty steps skipped (they have no side
        effects, subpoly.py:110).  ``allreduce(vec, op)`` (multi-GPU) makes
        the split count, the override predicate and the active mask global."""
        K, H = self.K, self.num_hidden
        if allreduce is not None and getattr(self, "curve", False):
            # the curve branch's in-step decisions (curve rows, descent rows,
            # the descent's stop, the strict filter's flag) go through the
            # same collective, called back from the engine
            cb = _collective_callback(allreduce)
            _hip.check(_hip.lib().tnp_engine_set_collective(self.h, C.cast(cb, C.c_void_p), None),
                       "tnp_engine_set_collective")
            try:
                return self._run_steps_host(stats, allreduce)
            finally:
                _hip.lib().tnp_engine_set_collective(self.h, None, None)
        return self._run_steps_host(stats, allreduce)

    def _run_steps_host(self, stats, allreduce):
        K = self.K
        if allreduce is None and not self._sharded:
            # one device: the loop runs in the library (tnp_engine_run_steps)
            buf = (_hip.TnpStepStats * max(self.K, 1))()
            n = C.c_int32()
            rc = _hip.lib().tnp_engine_run_steps(self.h, self._s, buf, len(buf), C.byref(n))
            if stats is not None:  # the completed steps, also when a later one failed
                stats.extend(buf[i].as_dict() for i in range(min(n.value, len(buf))))
            _hip.check(rc, "tnp_engine_run_steps")
            return stats
        mask = self.active_planes(0)
        if allreduce is not None:
            mask = int(allreduce(np.array([mask], dtype=np.uint64), "or")[0])
        for idx in range(K):
            # active-plane words keep planes 0..62 and fold 63.. into bit 63
            # (common.h act_bit): a wide net's planes >= 63 are never skipped
            if not (mask >> min(idx, 63)) & 1:
                continue
            S, fail = self.split(idx)
            if allreduce is not None:
                g = allreduce(np.array([S, int(fail)], dtype=np.int64), "max")
                S_glob, fail = int(g[0]), int(g[1])
            else:
                S_glob = S
            if S_glob == 0:
                continue
            prune = idx < K - 1  # h == num_hidden (final step) never prunes
            st = self.finish(idx, prune, fail)
            if stats is not None:
                stats.append(st)
            if prune:
                m2 = st["next_active"]
                if allreduce is not None:
                    m2 = int(allreduce(np.array([m2], dtype=np.uint64), "or")[0])
                keep = (1 << 63) - 1 if idx >= 62 else (1 << (idx + 1)) - 1
                mask = (mask & keep) | m2
        return stats


_ENGINES = {}


def engine_for(net) -> Engine:
    dev = net.device()
    key = (dev.index if dev.index is not None else torch.cuda.current_device())
    eng = _ENGINES.get(key)
    if eng is None:
        eng = Engine(torch.device("cuda", key))
        _ENGINES[key] = eng
    # every per-run setting back to the single-device default: a sharded run
    # (subpoly_sharded, a bench rank) leaves shards, the owned range and the
    # bucket x span behind on the cached engine otherwise
    eng.set_shards(1)
    eng.set_owned()
    eng.set_xspan()
    return eng.set_net(net).set_curve(False).set_strict(True)
