"""ctypes mirror of include/plba.h (structs only; no library is loaded here)."""
from __future__ import annotations

import ctypes as C
from typing import List

import numpy as np

from .synth import Graph

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_bp = C.POINTER(C.c_uint8)


class PlbaGraph(C.Structure):
    _fields_ = [
        ("n_kf", C.c_int32), ("n_pt", C.c_int32), ("n_ln", C.c_int32), ("n_ept", C.c_int32), ("n_eln", C.c_int32),
        ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
        ("kf_Tcw", _dp), ("kf_fixed", _bp), ("kf_id", _ip),
        ("pt_xyz", _dp), ("pt_id", _ip),
        ("ln_orth", _dp), ("ln_id", _ip),
        ("ept_lm", _ip), ("ept_kf", _ip), ("ept_obs", _dp), ("ept_info", _dp),
        ("eln_lm", _ip), ("eln_kf", _ip), ("eln_obs", _dp), ("eln_info", _dp),
        ("huber_pt", C.c_double), ("huber_ln", C.c_double),
    ]


class PlbaIterTrace(C.Structure):
    _fields_ = [("stage", C.c_int32), ("iter", C.c_int32), ("trials", C.c_int32), ("result", C.c_int32),
                ("chi2_start", C.c_double), ("chi2_end", C.c_double),
                ("lambda_start", C.c_double), ("lambda_end", C.c_double)]


class PlbaResult(C.Structure):
    _fields_ = [("kf_Tcw", _dp), ("pt_xyz", _dp), ("ln_orth", _dp),
                ("ept_chi2", _dp), ("ept_depth_ok", _bp), ("ept_level", _bp),
                ("eln_chi2", _dp), ("eln_level", _bp),
                ("iters", C.c_int32 * 2), ("chi2", C.c_double * 2), ("solve_ms", C.c_double)]


class PlbaOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("corrected_line_jacobian", C.c_int32), ("verbose", C.c_int32),
                ("max_trials", C.c_int32), ("tau", C.c_double)]


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class GraphView:
    """Keeps contiguous copies of a Graph's arrays alive and exposes a PlbaGraph."""

    def __init__(self, g: Graph):
        self.keep: List[np.ndarray] = []

        def f64(a, shape_last=None):
            a = np.ascontiguousarray(a, dtype=np.float64)
            self.keep.append(a)
            return _ptr(a, _dp)

        def i32(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            self.keep.append(a)
            return _ptr(a, _ip)

        def u8(a):
            a = np.ascontiguousarray(a, dtype=np.uint8)
            self.keep.append(a)
            return _ptr(a, _bp)

        s = PlbaGraph()
        s.n_kf, s.n_pt, s.n_ln, s.n_ept, s.n_eln = g.n_kf, g.n_pt, g.n_ln, g.n_ept, g.n_eln
        s.fx, s.fy, s.cx, s.cy = g.fx, g.fy, g.cx, g.cy
        s.kf_Tcw = f64(g.kf_Tcw.reshape(-1, 12))
        s.kf_fixed = u8(g.kf_fixed)
        s.kf_id = i32(g.kf_id)
        s.pt_xyz = f64(g.pt_xyz.reshape(-1, 3))
        s.pt_id = i32(g.pt_id)
        s.ln_orth = f64(g.ln_orth.reshape(-1, 4))
        s.ln_id = i32(g.ln_id)
        s.ept_lm, s.ept_kf = i32(g.ept_lm), i32(g.ept_kf)
        s.ept_obs, s.ept_info = f64(g.ept_obs.reshape(-1, 2)), f64(g.ept_info)
        s.eln_lm, s.eln_kf = i32(g.eln_lm), i32(g.eln_kf)
        s.eln_obs, s.eln_info = f64(g.eln_obs.reshape(-1, 4)), f64(g.eln_info)
        s.huber_pt, s.huber_ln = g.huber_pt, g.huber_ln
        self.struct = s


class ResultBuffers:
    """Host output arrays for plba_result."""

    def __init__(self, g: Graph):
        self.kf_Tcw = np.zeros((g.n_kf, 3, 4))
        self.pt_xyz = np.zeros((g.n_pt, 3))
        self.ln_orth = np.zeros((g.n_ln, 4))
        self.ept_chi2 = np.zeros(g.n_ept)
        self.ept_depth_ok = np.zeros(g.n_ept, np.uint8)
        self.ept_level = np.zeros(g.n_ept, np.uint8)
        self.eln_chi2 = np.zeros(g.n_eln)
        self.eln_level = np.zeros(g.n_eln, np.uint8)
        r = PlbaResult()
        r.kf_Tcw = _ptr(self.kf_Tcw, _dp)
        r.pt_xyz = _ptr(self.pt_xyz, _dp)
        r.ln_orth = _ptr(self.ln_orth, _dp)
        r.ept_chi2 = _ptr(self.ept_chi2, _dp)
        r.ept_depth_ok = _ptr(self.ept_depth_ok, _bp)
        r.ept_level = _ptr(self.ept_level, _bp)
        r.eln_chi2 = _ptr(self.eln_chi2, _dp)
        r.eln_level = _ptr(self.eln_level, _bp)
        self.struct = r

    def as_dict(self) -> dict:
        s = self.struct
        return dict(kf_Tcw=self.kf_Tcw, pt_xyz=self.pt_xyz, ln_orth=self.ln_orth,
                    ept_chi2=self.ept_chi2, ept_depth_ok=self.ept_depth_ok, ept_level=self.ept_level,
                    eln_chi2=self.eln_chi2, eln_level=self.eln_level,
                    iters=np.array([s.iters[0], s.iters[1]], np.int32),
                    chi2=np.array([s.chi2[0], s.chi2[1]]), solve_ms=float(s.solve_ms))


def trace_to_array(tr, n: int) -> np.ndarray:
    """Structured numpy array from a PlbaIterTrace buffer."""
    dt = np.dtype([("stage", np.int32), ("iter", np.int32), ("trials", np.int32), ("result", np.int32),
                   ("chi2_start", np.float64), ("chi2_end", np.float64),
                   ("lambda_start", np.float64), ("lambda_end", np.float64)])
    out = np.zeros(n, dt)
    for i in range(n):
        t = tr[i]
        out[i] = (t.stage, t.iter, t.trials, t.result, t.chi2_start, t.chi2_end, t.lambda_start, t.lambda_end)
    return out


# ---- hand-rolled LM (plba_hlm_*)
class PlbaHlmState(C.Structure):
    _fields_ = [("kf_x", _dp), ("ln_pluker", _dp), ("ln_line3d", _dp)]


class PlbaHlmParams(C.Structure):
    _fields_ = [("lambda0", C.c_double), ("lambda_k", C.c_double), ("homog_th", C.c_double),
                ("min_error", C.c_double), ("min_error_change", C.c_double),
                ("max_iters", C.c_int32), ("err_per_obs", C.c_int32), ("variant", C.c_int32), ("pad", C.c_int32)]


HLM_LBA_PLUCKER = 0
HLM_GBA = 1
DBL_EPSILON = float(np.finfo(np.float64).eps)


class PlbaHlmResult(C.Structure):
    _fields_ = [("kf_x", _dp), ("kf_Tcw", _dp), ("pt_xyz", _dp), ("ln_orth", _dp),
                ("linearizations", C.c_int32), ("solves", C.c_int32), ("accepted", C.c_int32), ("pad", C.c_int32),
                ("err", C.c_double), ("lambda_", C.c_double), ("dx_norm", C.c_double), ("solve_ms", C.c_double),
                ("ln_line3d", _dp)]


def gba_params(**kw) -> "PlbaHlmParams":
    """levMarquardtOptimizationGBA: the LBA defaults with ε stop tests (src/mapHandler.cpp:3664,3694)."""
    p = hlm_params(min_error=DBL_EPSILON, min_error_change=DBL_EPSILON, variant=HLM_GBA)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def hlm_params(**kw) -> PlbaHlmParams:
    """Defaults of src/slamConfig.cpp:65-67 and src2/config.cpp:80-85 (plba_hlm_default_params)."""
    p = PlbaHlmParams(lambda0=1e-5, lambda_k=10.0, homog_th=1e-7, min_error=1e-7, min_error_change=1e-7,
                      max_iters=15, err_per_obs=0, variant=HLM_LBA_PLUCKER)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class HlmStateView:
    def __init__(self, kf_x: np.ndarray, ln_pluker: np.ndarray, ln_line3d=None):
        self.kf_x = np.ascontiguousarray(kf_x, np.float64).reshape(-1, 6)
        self.ln_pluker = np.ascontiguousarray(ln_pluker, np.float64).reshape(-1, 6)
        self.ln_line3d = np.ascontiguousarray(ln_line3d if ln_line3d is not None else np.zeros((0, 6)),
                                              np.float64).reshape(-1, 6)
        self.struct = PlbaHlmState(kf_x=_ptr(self.kf_x, _dp), ln_pluker=_ptr(self.ln_pluker, _dp),
                                   ln_line3d=_ptr(self.ln_line3d, _dp) if self.ln_line3d.size else None)


class HlmResultBuffers:
    def __init__(self, g: Graph):
        self.kf_x = np.zeros((g.n_kf, 6))
        self.kf_Tcw = np.zeros((g.n_kf, 3, 4))
        self.pt_xyz = np.zeros((g.n_pt, 3))
        self.ln_orth = np.zeros((g.n_ln, 4))
        self.ln_line3d = np.zeros((g.n_ln, 6))
        self.struct = PlbaHlmResult(kf_x=_ptr(self.kf_x, _dp), kf_Tcw=_ptr(self.kf_Tcw, _dp),
                                    pt_xyz=_ptr(self.pt_xyz, _dp), ln_orth=_ptr(self.ln_orth, _dp),
                                    ln_line3d=_ptr(self.ln_line3d, _dp))

    def as_dict(self) -> dict:
        s = self.struct
        return dict(kf_x=self.kf_x, kf_Tcw=self.kf_Tcw, pt_xyz=self.pt_xyz, ln_orth=self.ln_orth,
                    ln_line3d=self.ln_line3d,
                    linearizations=int(s.linearizations), solves=int(s.solves), accepted=int(s.accepted),
                    err=float(s.err), lam=float(s.lambda_), dx_norm=float(s.dx_norm), solve_ms=float(s.solve_ms))


# ---- loop-closure pose graph (plba_pgo_*)
class PlbaPgoGraph(C.Structure):
    _fields_ = [("n_v", C.c_int32), ("n_e", C.c_int32), ("v_id", _ip), ("v_T", _dp), ("v_fixed", _bp),
                ("e_v", _ip), ("e_Z", _dp), ("e_info", _dp)]


class PlbaPgoParams(C.Structure):
    _fields_ = [("user_lambda_init", C.c_double), ("max_iters", C.c_int32), ("initial_guess", C.c_int32),
                ("max_trials", C.c_int32), ("pad", C.c_int32)]


class PlbaPgoResult(C.Structure):
    _fields_ = [("v_T", _dp), ("trace", C.POINTER(PlbaIterTrace)), ("trace_cap", C.c_int32), ("n_trace", C.c_int32),
                ("iterations", C.c_int32), ("trials", C.c_int32), ("solve_fails", C.c_int32), ("n_free", C.c_int32),
                ("chi2_initial", C.c_double), ("chi2_final", C.c_double), ("lambda_final", C.c_double),
                ("solve_ms", C.c_double)]


def pgo_params(**kw) -> PlbaPgoParams:
    """plba_pgo_default_params: the reference's values (setUserLambdaInit(1e-10), maxItersPGO 100)."""
    p = PlbaPgoParams(user_lambda_init=1e-10, max_iters=100, initial_guess=1, max_trials=10, pad=0)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class PgoGraphView:
    """Contiguous copies of a plba.pgo.PoseGraph's arrays and the PlbaPgoGraph over them."""

    def __init__(self, pg):
        self.v_id = np.ascontiguousarray(pg.v_id, dtype=np.int32)
        self.v_T = np.ascontiguousarray(pg.v_T, dtype=np.float64).reshape(-1, 12)
        self.v_fixed = np.ascontiguousarray(pg.v_fixed, dtype=np.uint8)
        self.e_v = np.ascontiguousarray(pg.e_v, dtype=np.int32).reshape(-1, 2)
        self.e_Z = np.ascontiguousarray(pg.e_Z, dtype=np.float64).reshape(-1, 12)
        self.e_info = None if pg.e_info is None else np.ascontiguousarray(pg.e_info, dtype=np.float64).reshape(-1, 36)
        self.struct = PlbaPgoGraph(
            n_v=len(self.v_id), n_e=len(self.e_v), v_id=_ptr(self.v_id, _ip), v_T=_ptr(self.v_T, _dp),
            v_fixed=_ptr(self.v_fixed, _bp), e_v=_ptr(self.e_v, _ip), e_Z=_ptr(self.e_Z, _dp),
            e_info=_ptr(self.e_info, _dp) if self.e_info is not None else C.cast(None, _dp))


class PgoResultBuffers:
    def __init__(self, n_v: int, trace_cap: int = 256):
        self.v_T = np.zeros((n_v, 12))
        self.trace = (PlbaIterTrace * trace_cap)()
        self.struct = PlbaPgoResult(v_T=_ptr(self.v_T, _dp), trace=self.trace, trace_cap=trace_cap)

    def as_dict(self) -> dict:
        s = self.struct
        return dict(v_T=self.v_T.copy(), iterations=s.iterations, trials=s.trials, solve_fails=s.solve_fails,
                    n_free=s.n_free, chi2_initial=s.chi2_initial, chi2_final=s.chi2_final,
                    lambda_final=s.lambda_final, solve_ms=s.solve_ms, trace=trace_to_array(self.trace, s.n_trace))
