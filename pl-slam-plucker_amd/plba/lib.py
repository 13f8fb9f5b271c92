"""ctypes binding of libplba.so (the HIP backend, C ABI of include/plba.h).

This is the product path: it fails loudly when the HIP library is missing or no GPU is
visible — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import capi
from .synth import Graph

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "libplba.so")

_lib = None

PLBA_ERRORS = {-1: "PLBA_E_INVALID", -2: "PLBA_E_DEVICE", -3: "PLBA_E_STATE", -4: "PLBA_E_NOMEM", -5: "PLBA_E_COMM"}

EXPORTED = [
    "plba_default_opts", "plba_create", "plba_destroy", "plba_last_error", "plba_upload", "plba_reset_estimates",
    "plba_set_edge_levels", "plba_set_robust", "plba_initialize_optimization", "plba_optimize",
    "plba_refresh_edge_errors", "plba_get_edge_chi2", "plba_download", "plba_lba_plucker", "plba_get_trace",
    "plba_synchronize", "plba_enable_kernel_timing", "plba_kernel_times", "plba_structure_stats",
    "plba_shard_plan", "plba_comm_unique_id", "plba_comm_init_rccl", "plba_comm_init_host",
    "plba_comm_info",
    "plba_hlm_default_params", "plba_hlm_lba",
    "plba_pgo_default_params", "plba_pgo_optimize",
]

# int (*plba_host_allreduce_fn)(void *user, double *buf, int64_t n)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)


class PlbaError(RuntimeError):
    pass


def load(path: Optional[str] = None):
    """Load libplba.so (raises if it is missing — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("PLBA_LIB") or LIB_PATH  # (PLBA_LIB: A/B builds of the same library)
    if not os.path.exists(path):
        raise PlbaError(f"libplba.so not found at {path}: run `make -C pl-slam-plucker_amd` "
                        "(or __graft_entry__.build()) first")
    L = C.CDLL(path)
    vp = C.c_void_p
    dp = C.POINTER(C.c_double)
    bp = C.POINTER(C.c_uint8)
    ip = C.POINTER(C.c_int32)
    L.plba_default_opts.argtypes = [C.POINTER(capi.PlbaOpts)]
    L.plba_default_opts.restype = None
    L.plba_create.argtypes = [C.POINTER(vp), C.POINTER(capi.PlbaOpts)]
    L.plba_destroy.argtypes = [vp]
    L.plba_last_error.argtypes = [vp]
    L.plba_last_error.restype = C.c_char_p
    L.plba_upload.argtypes = [vp, C.POINTER(capi.PlbaGraph)]
    L.plba_reset_estimates.argtypes = [vp]
    L.plba_set_edge_levels.argtypes = [vp, bp, bp]
    L.plba_set_robust.argtypes = [vp, C.c_int32]
    L.plba_initialize_optimization.argtypes = [vp, C.c_int32]
    L.plba_optimize.argtypes = [vp, C.c_int32, ip, dp]
    L.plba_refresh_edge_errors.argtypes = [vp, C.c_int32]
    L.plba_get_edge_chi2.argtypes = [vp, dp, bp, dp]
    L.plba_download.argtypes = [vp, dp, dp, dp]
    L.plba_lba_plucker.argtypes = [vp, C.POINTER(capi.PlbaResult)]
    L.plba_get_trace.argtypes = [vp, C.POINTER(capi.PlbaIterTrace), C.c_int32, ip]
    L.plba_synchronize.argtypes = [vp]
    L.plba_enable_kernel_timing.argtypes = [vp, C.c_int32]
    L.plba_kernel_times.argtypes = [vp, C.POINTER(C.c_char_p), dp, ip, C.c_int32, ip]
    L.plba_structure_stats.argtypes = [vp, C.POINTER(C.c_int64), C.c_int32]
    L.plba_shard_plan.argtypes = [C.POINTER(capi.PlbaGraph), C.c_int32, ip, ip]
    L.plba_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
    L.plba_comm_init_rccl.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]
    L.plba_comm_init_host.argtypes = [vp, C.c_int32, C.c_int32, HOST_ALLREDUCE_FN, vp]
    L.plba_comm_info.argtypes = [vp, ip, C.c_int32]
    L.plba_hlm_default_params.argtypes = [C.POINTER(capi.PlbaHlmParams)]
    L.plba_hlm_default_params.restype = None
    L.plba_hlm_lba.argtypes = [vp, C.POINTER(capi.PlbaHlmState), C.POINTER(capi.PlbaHlmParams),
                               C.POINTER(capi.PlbaHlmResult)]
    L.plba_pgo_default_params.argtypes = [C.POINTER(capi.PlbaPgoParams)]
    L.plba_pgo_default_params.restype = None
    L.plba_pgo_optimize.argtypes = [vp, C.POINTER(capi.PlbaPgoGraph), C.POINTER(capi.PlbaPgoParams),
                                    C.POINTER(capi.PlbaPgoResult)]
    for name in EXPORTED:
        f = getattr(L, name)
        if name not in ("plba_default_opts", "plba_last_error", "plba_hlm_default_params", "plba_pgo_default_params"):
            f.restype = C.c_int
    _lib = L
    return L


def _p(a, t=C.c_double):
    return a.ctypes.data_as(C.POINTER(t))


def shard_plan(g: Graph, nranks: int):
    """Landmark -> rank assignment of a sharded window (pure host code; no GPU needed)."""
    L = load()
    gv = capi.GraphView(g)
    po = np.zeros(max(g.n_pt, 1), np.int32)
    lo = np.zeros(max(g.n_ln, 1), np.int32)
    rc = L.plba_shard_plan(C.byref(gv.struct), nranks, _p(po, C.c_int32), _p(lo, C.c_int32))
    if rc != 0:
        raise PlbaError(f"plba_shard_plan failed: {PLBA_ERRORS.get(rc, rc)}")
    return po[:g.n_pt], lo[:g.n_ln]


def comm_unique_id() -> bytes:
    """RCCL unique id (create on rank 0, broadcast the 128 bytes)."""
    buf = (C.c_uint8 * 128)()
    rc = load().plba_comm_unique_id(buf)
    if rc != 0:
        raise PlbaError(f"plba_comm_unique_id failed: {PLBA_ERRORS.get(rc, rc)}")
    return bytes(buf)


class Solver:
    """One plba context bound to a device (g2o::SparseOptimizer equivalent)."""

    def __init__(self, device: int = 0, corrected_line_jacobian: bool = False, verbose: bool = False,
                 kernel_timing: bool = False, tau: Optional[float] = None, max_trials: Optional[int] = None):
        self.L = load()
        o = capi.PlbaOpts()
        self.L.plba_default_opts(C.byref(o))
        o.device = device
        o.corrected_line_jacobian = int(corrected_line_jacobian)
        o.verbose = int(verbose)
        if tau is not None:
            o.tau = float(tau)          # OptimizationAlgorithmLevenberg τ (λ init = τ·max|H_jj|)
        if max_trials is not None:
            o.max_trials = int(max_trials)
        self.ctx = C.c_void_p()
        rc = self.L.plba_create(C.byref(self.ctx), C.byref(o))
        if rc != 0:
            raise PlbaError(f"plba_create failed: {PLBA_ERRORS.get(rc, rc)} (no usable HIP device?)")
        self.graph: Optional[Graph] = None
        if kernel_timing:
            self._check(self.L.plba_enable_kernel_timing(self.ctx, 1), "plba_enable_kernel_timing")

    def _check(self, rc, what):
        if rc != 0:
            msg = self.L.plba_last_error(self.ctx).decode(errors="replace")
            raise PlbaError(f"{what} failed: {PLBA_ERRORS.get(rc, rc)}: {msg}")

    def close(self):
        if self.ctx:
            self.L.plba_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- sharded windows (call one of these before upload)
    def comm_init_rccl(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.L.plba_comm_init_rccl(self.ctx, nranks, rank, buf), "plba_comm_init_rccl")

    def comm_init_host(self, nranks: int, rank: int, allreduce):
        """allreduce(np.ndarray[float64]) sums the array over ranks in place."""
        def tramp(user, buf, n):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(n,)))
                return 0
            except Exception:  # never unwind through C
                import traceback
                traceback.print_exc()
                return -1
        self._host_cb = HOST_ALLREDUCE_FN(tramp)
        self._check(self.L.plba_comm_init_host(self.ctx, nranks, rank, self._host_cb, None), "plba_comm_init_host")

    def comm_info(self) -> dict:
        """What the transport reports (plba_comm_info): RCCL's own rank count, rank and device, and
        the HIP device / PCI location this context runs on."""
        v = np.zeros(8, np.int32)
        self._check(self.L.plba_comm_info(self.ctx, _p(v, C.c_int32), 8), "plba_comm_info")
        return dict(transport={0: "none", 1: "rccl", 2: "host"}.get(int(v[0]), str(int(v[0]))),
                    ranks=int(v[1]), rank=int(v[2]), comm_device=int(v[3]), hip_device=int(v[4]),
                    pci=f"{int(v[5]):04x}:{int(v[6]):02x}:{int(v[7]):02x}" if v[5] >= 0 else None)

    # -- g2o-style calls
    def upload(self, g: Graph):
        self.graph = g
        gv = capi.GraphView(g)
        self._check(self.L.plba_upload(self.ctx, C.byref(gv.struct)), "plba_upload")

    def reset(self):
        self._check(self.L.plba_reset_estimates(self.ctx), "plba_reset_estimates")

    def set_edge_levels(self, ept_level, eln_level):
        a = np.ascontiguousarray(ept_level, np.uint8)
        b = np.ascontiguousarray(eln_level, np.uint8)
        self._check(self.L.plba_set_edge_levels(self.ctx, _p(a, C.c_uint8), _p(b, C.c_uint8)), "plba_set_edge_levels")

    def set_robust(self, on: bool):
        self._check(self.L.plba_set_robust(self.ctx, int(on)), "plba_set_robust")

    def initialize_optimization(self, level: int = 0):
        self._check(self.L.plba_initialize_optimization(self.ctx, level), "plba_initialize_optimization")

    def optimize(self, iterations: int):
        it = C.c_int32(0)
        chi = C.c_double(0)
        self._check(self.L.plba_optimize(self.ctx, iterations, C.byref(it), C.byref(chi)), "plba_optimize")
        return it.value, chi.value

    def refresh_edge_errors(self, level: int):
        self._check(self.L.plba_refresh_edge_errors(self.ctx, level), "plba_refresh_edge_errors")

    def edge_chi2(self):
        g = self.graph
        pc, pd, lc = np.zeros(g.n_ept), np.zeros(g.n_ept, np.uint8), np.zeros(g.n_eln)
        self._check(self.L.plba_get_edge_chi2(self.ctx, _p(pc), _p(pd, C.c_uint8), _p(lc)), "plba_get_edge_chi2")
        return pc, pd, lc

    def download(self):
        g = self.graph
        T, P, O = np.zeros((g.n_kf, 3, 4)), np.zeros((g.n_pt, 3)), np.zeros((g.n_ln, 4))
        self._check(self.L.plba_download(self.ctx, _p(T), _p(P), _p(O)), "plba_download")
        return T, P, O

    def lba_plucker(self, want_outputs: bool = True, with_trace: bool = True) -> dict:
        """Full two-stage schedule (src/mapHandler.cpp:6119-6160) on the uploaded window."""
        g = self.graph
        if want_outputs:
            rb = capi.ResultBuffers(g)
            self._check(self.L.plba_lba_plucker(self.ctx, C.byref(rb.struct)), "plba_lba_plucker")
            out = rb.as_dict()
        else:
            r = capi.PlbaResult()
            self._check(self.L.plba_lba_plucker(self.ctx, C.byref(r)), "plba_lba_plucker")
            out = dict(iters=np.array([r.iters[0], r.iters[1]]), chi2=np.array([r.chi2[0], r.chi2[1]]),
                       solve_ms=r.solve_ms)
        if with_trace:
            out["trace"] = self.trace()
        return out

    def hlm_lba(self, win, params=None, with_trace: bool = True) -> dict:
        """levMarquardtOptimizationLBAForPluker (src/mapHandler.cpp:1618-2332) on the uploaded window.

        ``win`` is a plba.hlm.HlmWindow whose ``graph`` was uploaded with :meth:`upload`."""
        g = self.graph
        if params is None:
            params = capi.PlbaHlmParams()
            self.L.plba_hlm_default_params(C.byref(params))
        sv = capi.HlmStateView(win.kf_x, win.ln_pluker, getattr(win, "ln_line3d", None))
        rb = capi.HlmResultBuffers(g)
        self._check(self.L.plba_hlm_lba(self.ctx, C.byref(sv.struct), C.byref(params), C.byref(rb.struct)),
                    "plba_hlm_lba")
        out = rb.as_dict()
        if with_trace:
            out["trace"] = self.trace()
        return out

    def pgo_optimize(self, pg, params=None) -> dict:
        """Loop-closure pose graph (plba_pgo_optimize; src/mapHandler.cpp:5070-5531) of a
        plba.pgo.PoseGraph: computeInitialGuess + optimize on this context's device. Needs no
        uploaded window and leaves one intact."""
        if params is None:
            params = capi.PlbaPgoParams()
            self.L.plba_pgo_default_params(C.byref(params))
        gv = capi.PgoGraphView(pg)
        rb = capi.PgoResultBuffers(len(gv.v_id))
        self._check(self.L.plba_pgo_optimize(self.ctx, C.byref(gv.struct), C.byref(params), C.byref(rb.struct)),
                    "plba_pgo_optimize")
        return rb.as_dict()

    def trace(self) -> np.ndarray:
        n = C.c_int32(0)
        self._check(self.L.plba_get_trace(self.ctx, None, 0, C.byref(n)), "plba_get_trace")
        buf = (capi.PlbaIterTrace * max(n.value, 1))()
        self._check(self.L.plba_get_trace(self.ctx, buf, n.value, C.byref(n)), "plba_get_trace")
        return capi.trace_to_array(buf, n.value)

    def kernel_times(self) -> dict:
        cap = 32
        names = (C.c_char_p * cap)()
        ms = np.zeros(cap)
        nl = np.zeros(cap, np.int32)
        n = C.c_int32(0)
        self._check(self.L.plba_kernel_times(self.ctx, names, _p(ms), _p(nl, C.c_int32), cap, C.byref(n)),
                    "plba_kernel_times")
        return {names[i].decode(): (float(ms[i]), int(nl[i])) for i in range(n.value)}

    def structure_stats(self) -> dict:
        st = (C.c_int64 * 22)()
        self._check(self.L.plba_structure_stats(self.ctx, st, 22), "plba_structure_stats")
        return dict(nf=st[0], bw=st[1], nblk=st[2], triples=st[3], edges=st[4], landmarks=st[5], banded=st[6],
                    chunks=st[7], free_edges=st[8], point_edges=st[9], graph=st[10], sharded=st[11],
                    twisted=st[12], column_lane=st[13], bcr_rows=st[14], dense_mfma=st[15],
                    bcr_fallbacks=st[16], spec_slots=st[17], spec_policy=st[18], device_steps=st[19],
                    unused20=st[20], device_build=st[21])

    def synchronize(self):
        self._check(self.L.plba_synchronize(self.ctx), "plba_synchronize")
