"""Map-level view of an LBA window: the KeyFrame / MapPoint / MapLine state that
``MapHandler::localBundleAdjustmentForPlukerWithG2O`` reads and mutates
(include/keyFrame.h:50-71, include/mapFeatures.h:39-107, include/mapHandler.h:141-151),
and the ctypes binding of the C++ host mirror (include/plslam_host.h, libplslam_host.so).

``make_map`` turns a synthetic window (synth.Graph) into such a map: free keyframes are
``local``, KF 0 is local (and therefore fixed by id, src/mapHandler.cpp:5943-5945), the other
fixed keyframes are non-local observers that the gather step pulls in as fixed
(:5888-5919); non-local landmarks and keyframes outside the window are added so the gather
has something to skip.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
from typing import Callable, Dict, List, Optional

import numpy as np

from . import capi
from . import geometry as geo
from .lib import PKG_DIR, PLBA_ERRORS, PlbaError
from .synth import Graph

HOST_LIB_PATH = os.path.join(PKG_DIR, "libplslam_host.so")
DESC_BYTES = 32


@dataclasses.dataclass
class KF:
    kf_idx: int
    T_kf_w: np.ndarray            # (4,4) camera -> world
    local: bool
    pt_idx: List[int]
    ls_idx: List[int]


@dataclasses.dataclass
class Landmark:
    idx: int
    local: bool
    inlier: bool
    pos: np.ndarray               # point3D (3,) or NDw (6,)
    desc_list: List[np.ndarray]
    obs_list: List[np.ndarray]    # (2,) for points, (4,) for lines
    kf_obs_list: List[int]
    sigma_list: List[float]
    dir_list: Optional[List[np.ndarray]] = None   # points only
    med_desc: Optional[np.ndarray] = None
    med_dir: Optional[np.ndarray] = None


@dataclasses.dataclass
class SlamMap:
    fx: float
    fy: float
    cx: float
    cy: float
    keyframes: List[Optional[KF]]
    points: List[Optional[Landmark]]
    lines: List[Optional[Landmark]]
    map_points_kf_idx: Dict[int, List[int]]
    full_graph: np.ndarray        # (n_kf, n_kf) uint32
    map_lines_kf_idx: Dict[int, List[int]] = dataclasses.field(default_factory=dict)
    max_kf_idx: int = 0           # MapHandler::max_kf_idx (the newest KF)

    def copy(self) -> "SlamMap":
        import copy
        return copy.deepcopy(self)


def median_descriptor(desc_list) -> int:
    """Index of the descriptor with the least median Hamming distance to the others
    (MapPoint::updateAverageDescDir, src/mapFeatures.cpp:57-86; the n == 1 read past the end
    of dist_idx is clamped to the only entry)."""
    n = len(desc_list)
    D = np.array([[int(np.unpackbits(np.bitwise_xor(a, b)).sum()) for b in desc_list] for a in desc_list])
    best, best_i = 99999, 0
    k = min(int(1 + 0.5 * (n - 1)), n - 1)
    for i in range(n):
        med = int(np.sort(D[i])[k])
        if med < best:
            best, best_i = med, i
    return best_i


def make_map(g: Graph, seed: int = 0, n_extra_kf: int = 2, n_extra_pt: int = 5, sigma2: float = 1.0) -> SlamMap:
    rng = np.random.default_rng(seed)
    kf_ids = [int(i) for i in g.kf_id]
    n_kf = max(kf_ids) + 1 + n_extra_kf
    kfs: List[Optional[KF]] = [None] * n_kf
    for k in range(g.n_kf):
        Twc = np.eye(4)
        Twc[:3, :] = geo.invert_rigid(g.kf_Tcw[k])
        kid = kf_ids[k]
        local = (not g.kf_fixed[k]) or kid == 0
        kfs[kid] = KF(kid, Twc, bool(local), [], [])
    for kid in range(n_kf):   # keyframes outside the window (not observed by local landmarks)
        if kfs[kid] is None:
            T = np.eye(4)
            T[:3, 3] = rng.normal(size=3)
            kfs[kid] = KF(kid, T, False, [], [])

    def new_lm(idx, pos, obs_rows, kf_rows, is_point):
        lm = Landmark(idx=idx, local=True, inlier=True, pos=np.array(pos, np.float64), desc_list=[], obs_list=[],
                      kf_obs_list=[], sigma_list=[], dir_list=[] if is_point else None)
        for o, k in zip(obs_rows, kf_rows):
            lm.desc_list.append(rng.integers(0, 256, DESC_BYTES, dtype=np.uint8))
            lm.obs_list.append(np.array(o, np.float64))
            lm.kf_obs_list.append(int(k))
            lm.sigma_list.append(float(sigma2 if rng.random() > 0.1 else 1.7))
            if is_point:
                d = rng.normal(size=3)
                lm.dir_list.append(d / np.linalg.norm(d))
        return lm

    points: List[Optional[Landmark]] = []
    for p in range(g.n_pt):
        sel = np.nonzero(g.ept_lm == p)[0]
        points.append(new_lm(p, g.pt_xyz[p], g.ept_obs[sel], g.kf_id[g.ept_kf[sel]], True))
    lines: List[Optional[Landmark]] = []
    for l in range(g.n_ln):
        sel = np.nonzero(g.eln_lm == l)[0]
        lines.append(new_lm(l, geo.orth_to_pluker(g.ln_orth[l]), g.eln_obs[sel], g.kf_id[g.eln_kf[sel]], False))
    # non-local landmarks (skipped by the gather) and a hole in the vectors (NULL pointer)
    for j in range(n_extra_pt):
        k1, k2 = rng.integers(0, n_kf, 2)
        lm = new_lm(len(points), rng.normal(size=3) * 3, [rng.uniform(0, 700, 2)] * 2, [k1, k2], True)
        lm.local = False
        points.append(lm)
    points.append(None)
    for lms in (points, lines):   # state after the constructor + addObservation replay
        for lm in lms:
            if lm is None:
                continue
            lm.med_desc = lm.desc_list[median_descriptor(lm.desc_list)]
            if lm.dir_list is not None:
                lm.med_dir = np.sum(lm.dir_list, axis=0) / len(lm.dir_list)
    # keyframe stereo features: every landmark seen, plus an untracked feature (-1)
    for lm in points:
        if lm is not None:
            for k in lm.kf_obs_list:
                kfs[k].pt_idx.append(lm.idx)
    for lm in lines:
        if lm is not None:
            for k in lm.kf_obs_list:
                kfs[k].ls_idx.append(lm.idx)
    for kf in kfs:
        kf.pt_idx.append(-1)
        rng.shuffle(kf.pt_idx)
    # map_points_kf_idx / map_lines_kf_idx: base KF -> its points / lines (the LBA's outlier
    # pass looks lines up in map_points_kf_idx, src/mapHandler.cpp:6239-6251)
    kidx: Dict[int, List[int]] = {k: [] for k in range(n_kf)}
    lidx: Dict[int, List[int]] = {k: [] for k in range(n_kf)}
    for lm in points:
        if lm is not None:
            kidx[lm.kf_obs_list[0]].append(lm.idx)
    for lm in lines:
        lidx[lm.kf_obs_list[0]].append(lm.idx)
    fg = np.zeros((n_kf, n_kf), np.uint32)
    for lm in points + lines:
        if lm is not None:
            for a in lm.kf_obs_list:
                for b in lm.kf_obs_list:
                    if a != b:
                        fg[a, b] += 1
    fg += 3   # so a few decrements never wrap
    return SlamMap(g.fx, g.fy, g.cx, g.cy, kfs, points, lines, kidx, fg, lidx, n_kf - 1)


# ------------------------------------------------------------------------------------ binding
class PlslamLbaStats(C.Structure):
    _fields_ = [("n_free_kf", C.c_int32), ("n_fixed_kf", C.c_int32), ("n_pt", C.c_int32), ("n_ln", C.c_int32),
                ("n_ept", C.c_int32), ("n_eln", C.c_int32), ("bad_line_stage1", C.c_int32),
                ("bad_point_obs", C.c_int32), ("actually_bad_point_obs", C.c_int32),
                ("bad_line_obs", C.c_int32), ("actually_bad_line_obs", C.c_int32),
                ("iters", C.c_int32 * 2), ("chi2", C.c_double * 2),
                ("gather_ms", C.c_double), ("solve_ms", C.c_double), ("bookkeeping_ms", C.c_double),
                ("upload_ms", C.c_double), ("dirty_landmarks", C.c_int32)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["iters"] = list(self.iters)
        d["chi2"] = list(self.chi2)
        return d


SOLVE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(capi.PlbaGraph), C.POINTER(capi.PlbaResult))
HLM_SOLVE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(capi.PlbaGraph), C.POINTER(capi.PlbaHlmState),
                           C.POINTER(capi.PlbaHlmParams), C.POINTER(capi.PlbaHlmResult))


PGO_SOLVE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(capi.PlbaPgoGraph), C.POINTER(capi.PlbaPgoParams),
                           C.POINTER(capi.PlbaPgoResult))


class PlslamPgoStats(C.Structure):
    _fields_ = [("kf_prev_idx", C.c_int32), ("kf_curr_idx", C.c_int32), ("n_vertices", C.c_int32),
                ("n_fixed", C.c_int32), ("n_edges", C.c_int32), ("n_loop_edges", C.c_int32),
                ("iterations", C.c_int32), ("trials", C.c_int32),
                ("chi2_initial", C.c_double), ("chi2_final", C.c_double), ("solve_ms", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class PlslamHlmStats(C.Structure):
    _fields_ = [("ret", C.c_int32), ("n_kf_list", C.c_int32), ("n_fixed_kf", C.c_int32), ("n_pt", C.c_int32),
                ("n_ln", C.c_int32), ("n_pt_obs", C.c_int32), ("n_ls_obs", C.c_int32),
                ("linearizations", C.c_int32), ("solves", C.c_int32), ("accepted", C.c_int32),
                ("pt_outliers", C.c_int32), ("ln_outliers", C.c_int32),
                ("err", C.c_double), ("lambda_", C.c_double), ("gather_ms", C.c_double), ("solve_ms", C.c_double),
                ("writeback_ms", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}

HOST_EXPORTED = [
    "plslam_map_create", "plslam_map_destroy", "plslam_map_last_error", "plslam_set_solver", "plslam_add_keyframe",
    "plslam_add_point", "plslam_point_add_observation", "plslam_add_line", "plslam_line_add_observation",
    "plslam_set_local", "plslam_set_full_graph", "plslam_get_full_graph", "plslam_kf_idx_set", "plslam_kf_idx_get",
    "plslam_local_ba_plucker_g2o", "plslam_get_keyframe", "plslam_get_point", "plslam_get_line",
    "plslam_pluker_to_orth", "plslam_orth_to_pluker",
    "plslam_set_inlier", "plslam_set_params", "plslam_set_max_kf_idx", "plslam_kf_lines_idx_set", "plslam_kf_lines_idx_get",
    "plslam_form_local_map", "plslam_remove_bad_landmarks_pluker", "plslam_local_mapping_step", "plslam_exists",
    "plslam_set_keyframe_x", "plslam_get_keyframe_x", "plslam_set_hlm_solver", "plslam_set_hlm_params",
    "plslam_local_ba_plucker",
    "plslam_set_loop_closure", "plslam_get_lc_idx_list", "plslam_set_pgo_params", "plslam_set_pgo_solver",
    "plslam_loop_closure_optimization", "plslam_set_line_geometry", "plslam_get_line_geometry",
    "plslam_set_incremental", "plslam_mark_landmark_changed", "plslam_check_incremental_gather",
]


@dataclasses.dataclass
class SlamParams:
    """SlamConfig values of the local-mapping step (src/slamConfig.cpp:48,61-62 defaults)."""
    min_lm_obs: int = 5
    min_lm_cov_graph: int = 75
    min_kf_local_map: int = 3

_hl = None


def load_host(path: Optional[str] = None):
    global _hl
    if _hl is not None:
        return _hl
    path = path or HOST_LIB_PATH
    if not os.path.exists(path):
        raise PlbaError(f"libplslam_host.so not found at {path}: run `make -C pl-slam-plucker_amd/host`")
    L = C.CDLL(path)
    vp, dp, ip, bp = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_uint8)
    u32p = C.POINTER(C.c_uint32)
    L.plslam_map_create.argtypes = [C.POINTER(vp), C.c_double, C.c_double, C.c_double, C.c_double,
                                    C.POINTER(capi.PlbaOpts)]
    L.plslam_map_destroy.argtypes = [vp]
    L.plslam_map_last_error.argtypes = [vp]
    L.plslam_map_last_error.restype = C.c_char_p
    L.plslam_set_solver.argtypes = [vp, SOLVE_FN, vp]
    L.plslam_add_keyframe.argtypes = [vp, C.c_int32, dp, C.c_int32, ip, C.c_int32, ip]
    L.plslam_add_point.argtypes = [vp, C.c_int32, dp, bp, C.c_int32, C.c_int32, dp, dp, C.c_double]
    L.plslam_point_add_observation.argtypes = [vp, C.c_int32, bp, C.c_int32, dp, dp, C.c_double]
    L.plslam_add_line.argtypes = [vp, C.c_int32, dp, bp, C.c_int32, C.c_int32, dp, C.c_double]
    L.plslam_line_add_observation.argtypes = [vp, C.c_int32, bp, C.c_int32, dp, C.c_double]
    L.plslam_set_local.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.plslam_set_full_graph.argtypes = [vp, C.c_int32, u32p]
    L.plslam_get_full_graph.argtypes = [vp, C.c_int32, u32p]
    L.plslam_kf_idx_set.argtypes = [vp, C.c_int32, ip, C.c_int32]
    L.plslam_kf_idx_get.argtypes = [vp, C.c_int32, ip, C.c_int32, ip]
    L.plslam_local_ba_plucker_g2o.argtypes = [vp, C.POINTER(PlslamLbaStats)]
    L.plslam_get_keyframe.argtypes = [vp, C.c_int32, dp, ip, ip, C.c_int32, ip, C.c_int32]
    L.plslam_get_point.argtypes = [vp, C.c_int32, dp, ip, ip, ip, ip, dp, dp, dp, C.c_int32, bp, dp]
    L.plslam_get_line.argtypes = [vp, C.c_int32, dp, ip, ip, ip, ip, dp, dp, C.c_int32, bp]
    L.plslam_pluker_to_orth.argtypes = [dp, dp]
    L.plslam_pluker_to_orth.restype = None
    L.plslam_orth_to_pluker.argtypes = [dp, dp]
    L.plslam_orth_to_pluker.restype = None
    L.plslam_set_inlier.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.plslam_set_params.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.plslam_set_max_kf_idx.argtypes = [vp, C.c_int32]
    L.plslam_kf_lines_idx_set.argtypes = [vp, C.c_int32, ip, C.c_int32]
    L.plslam_kf_lines_idx_get.argtypes = [vp, C.c_int32, ip, C.c_int32, ip]
    L.plslam_form_local_map.argtypes = [vp, C.c_int32]
    L.plslam_remove_bad_landmarks_pluker.argtypes = [vp, ip, ip]
    L.plslam_local_mapping_step.argtypes = [vp, C.c_int32, C.POINTER(PlslamLbaStats), ip, ip]
    L.plslam_exists.argtypes = [vp, C.c_int32, C.c_int32, ip]
    L.plslam_set_keyframe_x.argtypes = [vp, C.c_int32, dp]
    L.plslam_get_keyframe_x.argtypes = [vp, C.c_int32, dp]
    L.plslam_set_hlm_solver.argtypes = [vp, HLM_SOLVE_FN, vp]
    L.plslam_set_hlm_params.argtypes = [vp, C.POINTER(capi.PlbaHlmParams), C.c_int32]
    L.plslam_local_ba_plucker.argtypes = [vp, C.POINTER(PlslamHlmStats)]
    L.plslam_set_loop_closure.argtypes = [vp, C.c_int32, ip, C.c_int32, ip, C.c_int32, dp]
    L.plslam_get_lc_idx_list.argtypes = [vp, ip, C.c_int32, ip]
    L.plslam_set_pgo_params.argtypes = [vp, C.c_int32, C.c_int32]
    L.plslam_set_pgo_solver.argtypes = [vp, PGO_SOLVE_FN, vp]
    L.plslam_loop_closure_optimization.argtypes = [vp, C.c_int32, C.POINTER(PlslamPgoStats)]
    L.plslam_set_line_geometry.argtypes = [vp, C.c_int32, dp, dp]
    L.plslam_get_line_geometry.argtypes = [vp, C.c_int32, dp, dp]
    L.plslam_set_incremental.argtypes = [vp, C.c_int32]
    L.plslam_mark_landmark_changed.argtypes = [vp, C.c_int32, C.c_int32]
    L.plslam_check_incremental_gather.argtypes = [vp, ip]
    for n in HOST_EXPORTED:
        if n not in ("plslam_map_last_error", "plslam_pluker_to_orth", "plslam_orth_to_pluker"):
            getattr(L, n).restype = C.c_int
    _hl = L
    return L


def _d(a):
    a = np.ascontiguousarray(a, np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


class HostMap:
    """A MapHandler (C++ host mirror) holding a SlamMap."""

    def __init__(self, m: SlamMap, corrected_line_jacobian: bool = False, device: int = 0,
                 params: Optional[SlamParams] = None):
        self.L = load_host()
        o = capi.PlbaOpts()
        from .lib import load
        load().plba_default_opts(C.byref(o))
        o.device = device
        o.corrected_line_jacobian = int(corrected_line_jacobian)
        self.h = C.c_void_p()
        self._check(self.L.plslam_map_create(C.byref(self.h), m.fx, m.fy, m.cx, m.cy, C.byref(o)), "create")
        self._cb = None
        self.n_kf = len(m.keyframes)
        self.n_pt = len(m.points)
        self.n_ln = len(m.lines)
        self._push(m)
        p = params or SlamParams()
        self._check(self.L.plslam_set_params(self.h, p.min_lm_obs, p.min_lm_cov_graph, p.min_kf_local_map), "params")

    def _check(self, rc, what):
        if rc != 0:
            msg = self.L.plslam_map_last_error(self.h).decode(errors="replace") if self.h else ""
            raise PlbaError(f"plslam {what} failed: {PLBA_ERRORS.get(rc, rc)}: {msg}")

    def close(self):
        if self.h:
            self.L.plslam_map_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _push(self, m: SlamMap):
        L, h = self.L, self.h
        ip = C.POINTER(C.c_int32)
        for kf in m.keyframes:
            if kf is None:
                continue
            T, Tp = _d(kf.T_kf_w.reshape(16))
            pi = np.asarray(kf.pt_idx, np.int32)
            li = np.asarray(kf.ls_idx, np.int32)
            self._check(L.plslam_add_keyframe(h, kf.kf_idx, Tp, len(pi), pi.ctypes.data_as(ip), len(li),
                                              li.ctypes.data_as(ip)), "add_keyframe")
            self._check(L.plslam_set_local(h, 0, kf.kf_idx, int(kf.local)), "set_local")
        bp = C.POINTER(C.c_uint8)
        for kind, lms in ((1, m.points), (2, m.lines)):
            for lm in lms:
                if lm is None:
                    continue
                for i in range(len(lm.kf_obs_list)):
                    desc = np.ascontiguousarray(lm.desc_list[i], np.uint8)
                    o, op = _d(lm.obs_list[i])
                    s = lm.sigma_list[i]
                    if kind == 1:
                        dvec, dpp = _d(lm.dir_list[i])
                        if i == 0:
                            x, xp = _d(lm.pos)
                            rc = L.plslam_add_point(h, lm.idx, xp, desc.ctypes.data_as(bp), len(desc),
                                                    lm.kf_obs_list[i], op, dpp, s)
                        else:
                            rc = L.plslam_point_add_observation(h, lm.idx, desc.ctypes.data_as(bp),
                                                                lm.kf_obs_list[i], op, dpp, s)
                    else:
                        if i == 0:
                            x, xp = _d(lm.pos)
                            rc = L.plslam_add_line(h, lm.idx, xp, desc.ctypes.data_as(bp), len(desc),
                                                   lm.kf_obs_list[i], op, s)
                        else:
                            rc = L.plslam_line_add_observation(h, lm.idx, desc.ctypes.data_as(bp),
                                                               lm.kf_obs_list[i], op, s)
                    self._check(rc, "add landmark")
                self._check(L.plslam_set_local(h, kind, lm.idx, int(lm.local)), "set_local")
                self._check(L.plslam_set_inlier(h, kind, lm.idx, int(lm.inlier)), "set_inlier")
        fg = np.ascontiguousarray(m.full_graph, np.uint32)
        self._check(L.plslam_set_full_graph(h, fg.shape[0], fg.ctypes.data_as(C.POINTER(C.c_uint32))), "full_graph")
        for k, lst in m.map_points_kf_idx.items():
            a = np.asarray(lst, np.int32)
            self._check(L.plslam_kf_idx_set(h, k, a.ctypes.data_as(ip), len(a)), "kf_idx_set")
        for k, lst in m.map_lines_kf_idx.items():
            a = np.asarray(lst, np.int32)
            self._check(L.plslam_kf_lines_idx_set(h, k, a.ctypes.data_as(ip), len(a)), "kf_lines_idx_set")
        self._check(L.plslam_set_max_kf_idx(h, int(m.max_kf_idx)), "max_kf_idx")

    def add_background(self, n_kf: int, n_pt: int, n_ln: int, seed: int = 0, obs_per_lm=(2, 5)):
        """Non-local keyframes and landmarks around the window (appended after the existing slots):
        e.g. a C5-sized map (BASELINE.json configs[4]: 1000 KF / 200k points / 40k lines) holding a
        C3 window, so that the per-call cost of the LBA is measured on a map of real size. Each
        background landmark is observed by 2-4 of the new keyframes; none is local."""
        L, h = self.L, self.h
        rng = np.random.default_rng(seed)
        ip, dp = C.POINTER(C.c_int32), C.POINTER(C.c_double)
        k0 = self.n_kf
        for k in range(n_kf):
            T = np.eye(4)
            T[:3, 3] = rng.normal(size=3) * 10
            Tc = np.ascontiguousarray(T.reshape(16))
            self._check(L.plslam_add_keyframe(h, k0 + k, Tc.ctypes.data_as(dp), 0, None, 0, None), "add_keyframe")
        self.n_kf += n_kf
        for kind, n, width in ((1, n_pt, 2), (2, n_ln, 4)):
            base = self.n_pt if kind == 1 else self.n_ln
            nobs = rng.integers(obs_per_lm[0], obs_per_lm[1], size=n)
            kfs = (k0 + rng.integers(0, max(n_kf, 1), size=int(nobs.sum()))).astype(np.int32)
            obs = np.ascontiguousarray(rng.uniform(0, 700, size=(int(nobs.sum()), width)))
            pos = np.ascontiguousarray(rng.normal(size=(n, 3 if kind == 1 else 6)) * 5)
            d3 = np.ascontiguousarray(np.array([0.0, 0.0, 1.0]))
            po, oo, dd = pos.ctypes.data, obs.ctypes.data, d3.ctypes.data_as(dp)
            e = 0
            for i in range(n):
                idx = base + i
                xp = C.cast(po + i * pos.shape[1] * 8, dp)
                for j in range(int(nobs[i])):
                    op = C.cast(oo + e * width * 8, dp)
                    if j == 0:
                        rc = (L.plslam_add_point(h, idx, xp, None, DESC_BYTES, int(kfs[e]), op, dd, 1.0) if kind == 1
                              else L.plslam_add_line(h, idx, xp, None, DESC_BYTES, int(kfs[e]), op, 1.0))
                    else:
                        rc = (L.plslam_point_add_observation(h, idx, None, int(kfs[e]), op, dd, 1.0) if kind == 1
                              else L.plslam_line_add_observation(h, idx, None, int(kfs[e]), op, 1.0))
                    if rc:
                        self._check(rc, "add background landmark")
                    e += 1
            if kind == 1:
                self.n_pt += n
            else:
                self.n_ln += n

    def set_solver(self, fn: Optional[Callable]):
        """fn(graph: PlbaGraph, result: PlbaResult) -> int, or None for the MI355X backend."""
        if fn is None:
            self._cb = None
            self._check(self.L.plslam_set_solver(self.h, C.cast(None, SOLVE_FN), None), "set_solver")
            return

        def tramp(user, gp, rp):
            try:
                return int(fn(gp.contents, rp.contents))
            except Exception as e:  # never unwind through C
                import traceback
                traceback.print_exc()
                self._cb_error = e
                return -1
        self._cb = SOLVE_FN(tramp)
        self._check(self.L.plslam_set_solver(self.h, self._cb, None), "set_solver")

    def set_incremental(self, on: bool):
        self._check(self.L.plslam_set_incremental(self.h, int(on)), "set_incremental")

    def mark_landmark_changed(self, kind: int, idx: int):
        self._check(self.L.plslam_mark_landmark_changed(self.h, kind, idx), "mark_landmark_changed")

    def check_incremental_gather(self) -> bool:
        e = C.c_int32()
        self._check(self.L.plslam_check_incremental_gather(self.h, C.byref(e)), "check_incremental_gather")
        if not e.value:
            self._why = self.L.plslam_map_last_error(self.h).decode(errors="replace")
        return bool(e.value)

    def local_ba(self) -> dict:
        st = PlslamLbaStats()
        self._check(self.L.plslam_local_ba_plucker_g2o(self.h, C.byref(st)), "local_ba_plucker_g2o")
        return st.as_dict()

    # -- hand-rolled LM LBA (MapHandler::localBundleAdjustmentForPluker)
    def set_hlm_solver(self, fn: Optional[Callable]):
        """fn(graph, state, params, result) -> int, or None for the MI355X backend (plba_hlm_lba)."""
        if fn is None:
            self._hcb = None
            self._check(self.L.plslam_set_hlm_solver(self.h, C.cast(None, HLM_SOLVE_FN), None), "set_hlm_solver")
            return

        def tramp(user, gp, sp, pp, rp):
            try:
                return int(fn(gp.contents, sp.contents, pp.contents, rp.contents))
            except Exception:  # never unwind through C
                import traceback
                traceback.print_exc()
                return -1
        self._hcb = HLM_SOLVE_FN(tramp)
        self._check(self.L.plslam_set_hlm_solver(self.h, self._hcb, None), "set_hlm_solver")

    def set_hlm_params(self, params=None, vo_inserting_kf: bool = False):
        self._check(self.L.plslam_set_hlm_params(self.h, C.byref(params) if params is not None else None,
                                                 int(vo_inserting_kf)), "set_hlm_params")

    def local_ba_hlm(self) -> dict:
        st = PlslamHlmStats()
        self._check(self.L.plslam_local_ba_plucker(self.h, C.byref(st)), "local_ba_plucker")
        return st.as_dict()

    # ---- loop-closure pose graph (src/mapHandler.cpp:5070-5531)
    def set_loop_closure(self, lc_idxs, lc_idx_list, lc_pose_list):
        a = np.ascontiguousarray(np.asarray(lc_idxs, np.int32).reshape(-1, 3))
        b = np.ascontiguousarray(np.asarray(lc_idx_list, np.int32).reshape(-1, 3))
        c = np.ascontiguousarray(np.asarray(lc_pose_list, np.float64).reshape(-1, 6))
        ip = C.POINTER(C.c_int32)
        self._check(self.L.plslam_set_loop_closure(self.h, len(a), a.ctypes.data_as(ip), len(b), b.ctypes.data_as(ip),
                                                   len(c), c.ctypes.data_as(C.POINTER(C.c_double))), "set_loop_closure")

    def lc_idx_list(self) -> np.ndarray:
        n = C.c_int32(0)
        self._check(self.L.plslam_get_lc_idx_list(self.h, None, 0, C.byref(n)), "get_lc_idx_list")
        out = np.zeros((max(n.value, 1), 3), np.int32)
        self._check(self.L.plslam_get_lc_idx_list(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), n.value,
                                                  C.byref(n)), "get_lc_idx_list")
        return out[:n.value]

    def set_pgo_params(self, min_lm_ess_graph: int = 150, max_iters_pgo: int = 100):
        self._check(self.L.plslam_set_pgo_params(self.h, min_lm_ess_graph, max_iters_pgo), "set_pgo_params")

    def set_pgo_solver(self, fn: Optional[Callable]):
        """fn(graph, params, result) -> int, or None for the MI355X backend (plba_pgo_optimize)."""
        if fn is None:
            self._pcb = None
            self._check(self.L.plslam_set_pgo_solver(self.h, C.cast(None, PGO_SOLVE_FN), None), "set_pgo_solver")
            return

        def tramp(user, gp, pp, rp):
            try:
                return int(fn(gp.contents, pp.contents, rp.contents))
            except Exception:  # never unwind through C
                import traceback
                traceback.print_exc()
                return -1
        self._pcb = PGO_SOLVE_FN(tramp)
        self._check(self.L.plslam_set_pgo_solver(self.h, self._pcb, None), "set_pgo_solver")

    def loop_closure(self, ess: bool = True) -> dict:
        st = PlslamPgoStats()
        self._check(self.L.plslam_loop_closure_optimization(self.h, int(ess), C.byref(st)), "loop_closure")
        return st.as_dict()

    def set_line_geometry(self, idx: int, line3d, med_obs_dir):
        a, pa = _d(line3d)
        b, pb = _d(med_obs_dir)
        self._check(self.L.plslam_set_line_geometry(self.h, idx, pa, pb), "set_line_geometry")

    def line_geometry(self, idx: int):
        a, b = np.zeros(6), np.zeros(3)
        self._check(self.L.plslam_get_line_geometry(self.h, idx, a.ctypes.data_as(C.POINTER(C.c_double)),
                                                    b.ctypes.data_as(C.POINTER(C.c_double))), "get_line_geometry")
        return a, b

    def keyframe_x(self, kf_idx: int) -> np.ndarray:
        x = np.zeros(6)
        self._check(self.L.plslam_get_keyframe_x(self.h, kf_idx, x.ctypes.data_as(C.POINTER(C.c_double))), "get_x")
        return x

    def set_keyframe_x(self, kf_idx: int, x):
        a, ap = _d(x)
        self._check(self.L.plslam_set_keyframe_x(self.h, kf_idx, ap), "set_x")

    def form_local_map(self, kf_idx: int):
        self._check(self.L.plslam_form_local_map(self.h, kf_idx), "form_local_map")

    def remove_bad_landmarks(self):
        a, b = C.c_int32(), C.c_int32()
        self._check(self.L.plslam_remove_bad_landmarks_pluker(self.h, C.byref(a), C.byref(b)), "remove_bad")
        return a.value, b.value

    def local_mapping_step(self, kf_idx: int) -> dict:
        st = PlslamLbaStats()
        a, b = C.c_int32(), C.c_int32()
        self._check(self.L.plslam_local_mapping_step(self.h, kf_idx, C.byref(st), C.byref(a), C.byref(b)),
                    "local_mapping_step")
        d = st.as_dict()
        d["points_removed"], d["lines_removed"] = a.value, b.value
        return d

    def exists(self, kind: int, idx: int) -> bool:
        e = C.c_int32()
        self._check(self.L.plslam_exists(self.h, kind, idx, C.byref(e)), "exists")
        return bool(e.value)

    def read(self, like: SlamMap) -> SlamMap:
        """Read the map state back (same object layout as `like`)."""
        L, h = self.L, self.h
        out = like.copy()
        ip = C.POINTER(C.c_int32)
        for kf in out.keyframes:
            if kf is None:
                continue
            T = np.zeros(16)
            loc = C.c_int32()
            pi = np.zeros(len(kf.pt_idx), np.int32)
            li = np.zeros(len(kf.ls_idx), np.int32)
            self._check(L.plslam_get_keyframe(h, kf.kf_idx, T.ctypes.data_as(C.POINTER(C.c_double)), C.byref(loc),
                                              pi.ctypes.data_as(ip), len(pi), li.ctypes.data_as(ip), len(li)),
                        "get_keyframe")
            kf.T_kf_w = T.reshape(4, 4)
            kf.local = bool(loc.value)
            kf.pt_idx = [int(v) for v in pi]
            kf.ls_idx = [int(v) for v in li]
        dp, bp = C.POINTER(C.c_double), C.POINTER(C.c_uint8)
        for kind, lms in ((1, out.points), (2, out.lines)):
            for j, lm in enumerate(lms):
                if lm is None:
                    continue
                if not self.exists(kind, lm.idx):   # deleted by removeBadMapLandmarksForPluker
                    lms[j] = None
                    continue
                cap = len(lm.kf_obs_list) + len(lm.sigma_list) + 4
                inl, loc, nobs = C.c_int32(), C.c_int32(), C.c_int32()
                kfo = np.zeros(cap, np.int32)
                sig = np.zeros(cap)
                md = np.zeros(DESC_BYTES, np.uint8)
                if kind == 1:
                    pos = np.zeros(3)
                    obs = np.zeros((cap, 2))
                    dirs = np.zeros((cap, 3))
                    mdir = np.zeros(3)
                    self._check(L.plslam_get_point(h, lm.idx, pos.ctypes.data_as(dp), C.byref(inl), C.byref(loc),
                                                   C.byref(nobs), kfo.ctypes.data_as(ip), obs.ctypes.data_as(dp),
                                                   dirs.ctypes.data_as(dp), sig.ctypes.data_as(dp), cap,
                                                   md.ctypes.data_as(bp), mdir.ctypes.data_as(dp)), "get_point")
                    n = nobs.value
                    lm.dir_list = [dirs[i].copy() for i in range(n)]
                    lm.med_dir = mdir
                else:
                    pos = np.zeros(6)
                    obs = np.zeros((cap, 4))
                    self._check(L.plslam_get_line(h, lm.idx, pos.ctypes.data_as(dp), C.byref(inl), C.byref(loc),
                                                  C.byref(nobs), kfo.ctypes.data_as(ip), obs.ctypes.data_as(dp),
                                                  sig.ctypes.data_as(dp), cap, md.ctypes.data_as(bp)), "get_line")
                    n = nobs.value
                lm.pos = pos
                lm.inlier = bool(inl.value)
                lm.local = bool(loc.value)
                lm.kf_obs_list = [int(v) for v in kfo[:n]]
                lm.obs_list = [obs[i].copy() for i in range(n)]
                lm.sigma_list = [float(v) for v in sig[:len(lm.sigma_list)]]
                lm.med_desc = md
                lm.desc_list = None   # not exposed; med_desc covers the descriptor logic
        fg = np.zeros_like(out.full_graph)
        self._check(L.plslam_get_full_graph(h, fg.shape[0], fg.ctypes.data_as(C.POINTER(C.c_uint32))), "full_graph")
        out.full_graph = fg
        n = C.c_int32()
        for k in list(out.map_points_kf_idx.keys()):
            buf = np.zeros(4096, np.int32)
            self._check(L.plslam_kf_idx_get(h, k, buf.ctypes.data_as(ip), len(buf), C.byref(n)), "kf_idx_get")
            out.map_points_kf_idx[k] = [int(v) for v in buf[:n.value]]
        for k in list(out.map_lines_kf_idx.keys()):
            buf = np.zeros(4096, np.int32)
            self._check(L.plslam_kf_lines_idx_get(h, k, buf.ctypes.data_as(ip), len(buf), C.byref(n)),
                        "kf_lines_idx_get")
            out.map_lines_kf_idx[k] = [int(v) for v in buf[:n.value]]
        return out
