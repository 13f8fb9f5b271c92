"""Seeded EuRoC-shaped synthetic LBA windows.

A *window* is what ``MapHandler::localBundleAdjustmentForPlukerWithG2O`` hands to
g2o after its gather step (src/mapHandler.cpp:5868-6117):

* pose vertices  -- ``Tcw = T_kf_w.inverse()`` (:5940), fixed for the observer
  KFs outside the local set and for KF id 0 (:5943-5945, :5954-5968);
* point vertices -- ``point3D`` (:5982), id ``idx + max_kf_id + 1`` (:5983);
* line vertices  -- ``changePlukerToOrth(NDw)`` (:6039-6046), id
  ``idx + maxPointId + 1`` (:6047);
* point edges    -- pixel ``obs_list[i]`` (:6002), Ω = I·(float)(1/σ²) (:6009);
* line edges     -- endpoints ``NDw_obs_list[i]`` (:6066), Ω = I·(float)(1/σ²).

Edges are emitted landmark-major in observation order -- the g2o insertion order.

Generator (per config Ck, seed 1000+k):
  camera      fx=458.654 fy=457.296 cx=367.215 cy=248.375, 752x480
              (config/dataset_params/euroc_params.yaml:2,9,11)
  trajectory  circle of radius 3 m, 0.15 m per KF, height ±0.5 m, outward-looking
              camera with yaw wobble (≈5° per KF)
  fixed KFs   the first max(1, round(0.1·N_kf)) -- always including id 0
  landmarks   each seen by a contiguous track of L~U{2..8} KFs (E = 5·N on average)
  points      2-8 m depth; lines 0.5-2 m segments, Plücker as src/mapHandler.cpp:451-459
  noise       N(0,1 px) on every observation; 2 % outliers displaced by U(20,50) px
  init        free poses rot N(0,0.3°) trans N(0,1 cm); points N(0,3 cm);
              lines orth N(0,0.3°)
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, Optional

import numpy as np

from . import geometry as geo

CAMERA = dict(fx=458.654, fy=457.296, cx=367.215, cy=248.375, width=752, height=480)

# (n_kf, n_pt, n_ln, seed).  Seeds follow SURVEY.md §8d (1000+k for Ck).
CONFIGS: Dict[str, tuple] = {
    "C1": (10, 500, 0, 1001),
    "C1L": (10, 200, 40, 1011),
    "C2": (50, 5000, 1000, 1002),
    "C3": (100, 20000, 4000, 1003),
    "C4": (400, 80000, 16000, 1004),
    "C5": (1000, 200000, 40000, 1005),
    # "revisit" windows: the trajectory closes its loop (period ≈126 KFs) and a share of the
    # landmarks is re-observed one loop later, so poses ~126 apart share landmarks and the
    # reduced camera system loses its narrow band (the dense / reordered factorisation paths)
    "C2R": (150, 3000, 600, 1012),
    "C3R": (160, 20000, 4000, 1013),
}
REVISIT_PERIOD = 126          # 2π / 0.05 rad per KF (_trajectory)
REVISIT_FRAC = 0.15

HUBER_DELTA = float(np.float32(math.sqrt(5.991)))  # const float thHuberMono (src/mapHandler.cpp:5978)
CHI2_THRESHOLD = 5.991                              # src/mapHandler.cpp:6129,6142


@dataclasses.dataclass
class Graph:
    """One LBA window in g2o-vertex/edge form (SoA, float64 / int32)."""
    fx: float
    fy: float
    cx: float
    cy: float
    kf_Tcw: np.ndarray        # (N_kf,3,4)  vertex estimate Tcw = [R|t]
    kf_fixed: np.ndarray      # (N_kf,) uint8
    kf_id: np.ndarray         # (N_kf,) int32 g2o vertex id (= kf_idx)
    pt_xyz: np.ndarray        # (N_p,3)
    pt_id: np.ndarray         # (N_p,) int32
    ln_orth: np.ndarray       # (N_l,4)
    ln_id: np.ndarray         # (N_l,) int32
    ept_lm: np.ndarray        # (E_p,) int32 index into pt arrays
    ept_kf: np.ndarray        # (E_p,) int32 index into kf arrays
    ept_obs: np.ndarray       # (E_p,2)
    ept_info: np.ndarray      # (E_p,)
    eln_lm: np.ndarray        # (E_l,) int32
    eln_kf: np.ndarray        # (E_l,) int32
    eln_obs: np.ndarray       # (E_l,4)
    eln_info: np.ndarray      # (E_l,)
    huber_pt: float = HUBER_DELTA
    huber_ln: float = HUBER_DELTA
    # ground truth (generator only; not part of the solver input)
    gt_Tcw: Optional[np.ndarray] = None
    gt_xyz: Optional[np.ndarray] = None
    gt_orth: Optional[np.ndarray] = None
    ept_outlier: Optional[np.ndarray] = None
    eln_outlier: Optional[np.ndarray] = None
    # initial line endpoints [P; Q] (N_l,6): the non-Plücker map's line3D, read by the hand-rolled
    # GBA (src/mapHandler.cpp:3089); not an input of the Plücker LBA
    ln_seg0: Optional[np.ndarray] = None

    @property
    def n_kf(self) -> int:
        return int(self.kf_Tcw.shape[0])

    @property
    def n_pt(self) -> int:
        return int(self.pt_xyz.shape[0])

    @property
    def n_ln(self) -> int:
        return int(self.ln_orth.shape[0])

    @property
    def n_ept(self) -> int:
        return int(self.ept_lm.shape[0])

    @property
    def n_eln(self) -> int:
        return int(self.eln_lm.shape[0])

    def copy(self) -> "Graph":
        return Graph(**{f.name: (getattr(self, f.name).copy() if isinstance(getattr(self, f.name), np.ndarray)
                                 else getattr(self, f.name)) for f in dataclasses.fields(self)})

    def save(self, path: str) -> None:
        d = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if v is None:
                continue
            d[f.name] = np.asarray(v)
        np.savez_compressed(path, **d)

    @staticmethod
    def load(path: str) -> "Graph":
        with np.load(path, allow_pickle=False) as z:
            kw = {}
            for f in dataclasses.fields(Graph):
                if f.name in z.files:
                    v = z[f.name]
                    kw[f.name] = float(v) if v.ndim == 0 else v
            return Graph(**kw)


def _trajectory(n: int):
    """Twc for n KFs on an MH-like loop; returns (R_wc (n,3,3), p_wc (n,3))."""
    k = np.arange(n, dtype=np.float64)
    phi = 0.05 * k                                    # 3 m * 0.05 rad = 0.15 m per KF
    pos = np.stack([3.0 * np.cos(phi), 3.0 * np.sin(phi), 0.5 * np.sin(0.11 * k)], -1)
    yaw = phi + 0.15 * np.sin(0.5 * k)
    pitch = 0.05 * np.sin(0.3 * k)
    roll = 0.03 * np.sin(0.2 * k)
    # camera looking along +X of its base frame: right=-Y, down=-Z, forward=+X
    R0 = np.array([[0.0, 0.0, 1.0], [-1.0, 0.0, 0.0], [0.0, -1.0, 0.0]])
    Rz = geo.rodrigues(np.stack([np.zeros(n), np.zeros(n), yaw], -1))
    Ry = geo.rodrigues(np.stack([np.zeros(n), pitch, np.zeros(n)], -1))
    Rx = geo.rodrigues(np.stack([roll, np.zeros(n), np.zeros(n)], -1))
    Rwc = Rz @ Ry @ Rx @ R0
    return Rwc, pos


def _project(Rcw, tcw, P, cam):
    Pc = np.einsum("...ij,...j->...i", Rcw, P) + tcw
    z = Pc[..., 2]
    zs = np.where(np.abs(z) < 1e-9, 1e-9, z)
    u = cam["fx"] * Pc[..., 0] / zs + cam["cx"]
    v = cam["fy"] * Pc[..., 1] / zs + cam["cy"]
    return u, v, z


def _tracks(rng, n_kf, count, lmin=2, lmax=8):
    Lmax = min(lmax, n_kf)
    Lmin = min(lmin, n_kf)
    L = rng.integers(Lmin, Lmax + 1, size=count)
    s = (rng.random(count) * (n_kf - L + 1)).astype(np.int64)
    return L, s


def _visible(Rcw, tcw, P, s, L, cam, margin):
    """P (M,3); tracks (s,L) -> bool (M,), all track KFs see P in the image."""
    M = P.shape[0]
    ok = np.ones(M, dtype=bool)
    for j in range(int(L.max()) if M else 0):
        m = j < L
        if not m.any():
            break
        kf = np.where(m, s + j, s)
        u, v, z = _project(Rcw[kf], tcw[kf], P, cam)
        good = (z > 0.5) & (u >= margin) & (u < cam["width"] - margin) & (v >= margin) & (v < cam["height"] - margin)
        ok &= np.where(m, good, True)
    return ok


def _sample_anchor(rng, Rwc, pwc, s, L, cam, depth_lo=2.0, depth_hi=8.0, margin=40.0):
    M = s.shape[0]
    a = s + L // 2
    u = rng.uniform(margin, cam["width"] - margin, M)
    v = rng.uniform(margin, cam["height"] - margin, M)
    z = rng.uniform(depth_lo, depth_hi, M)
    Pc = np.stack([(u - cam["cx"]) / cam["fx"] * z, (v - cam["cy"]) / cam["fy"] * z, z], -1)
    return np.einsum("mij,mj->mi", Rwc[a], Pc) + pwc[a]


def generate(name: str = "C3", *, n_kf: Optional[int] = None, n_pt: Optional[int] = None,
             n_ln: Optional[int] = None, seed: Optional[int] = None, fixed_frac: float = 0.1,
             noise_px: float = 1.0, outlier_frac: float = 0.02, perturb: bool = True,
             track_min: int = 2, track_max: int = 8, revisit_frac: Optional[float] = None,
             revisit_period: int = REVISIT_PERIOD) -> Graph:
    """Generate one window. ``name`` picks a config; keyword args override it.

    ``revisit_frac`` (default REVISIT_FRAC for the ``*R`` configs, else 0): that share of the
    point landmarks gets one more observation from the KF one loop (``revisit_period`` KFs) after
    the middle of its track, when that KF sees the point."""
    base = CONFIGS.get(name, (10, 500, 0, 1000))
    n_kf = base[0] if n_kf is None else n_kf
    n_pt = base[1] if n_pt is None else n_pt
    n_ln = base[2] if n_ln is None else n_ln
    seed = base[3] if seed is None else seed
    rng = np.random.default_rng(seed)
    cam = CAMERA

    Rwc, pwc = _trajectory(n_kf)
    Rcw = np.swapaxes(Rwc, -1, -2)
    tcw = -np.einsum("nij,nj->ni", Rcw, pwc)
    n_fix = max(1, int(round(fixed_frac * n_kf)))

    # ---------------- points
    pts, pt_s, pt_L = [], [], []
    have = 0
    while have < n_pt:
        M = max(1024, 2 * (n_pt - have))
        L, s = _tracks(rng, n_kf, M, track_min, track_max)
        P = _sample_anchor(rng, Rwc, pwc, s, L, cam)
        ok = _visible(Rcw, tcw, P, s, L, cam, margin=5.0)
        take = np.nonzero(ok)[0][: n_pt - have]
        pts.append(P[take]); pt_s.append(s[take]); pt_L.append(L[take])
        have += take.size
    gt_xyz = np.concatenate(pts) if n_pt else np.zeros((0, 3))
    pt_s = np.concatenate(pt_s) if n_pt else np.zeros(0, np.int64)
    pt_L = np.concatenate(pt_L) if n_pt else np.zeros(0, np.int64)

    # ---------------- lines (segments)
    segs, ln_s, ln_L = [], [], []
    have = 0
    while have < n_ln:
        M = max(1024, 2 * (n_ln - have))
        L, s = _tracks(rng, n_kf, M, track_min, track_max)
        C = _sample_anchor(rng, Rwc, pwc, s, L, cam, margin=80.0)
        dvec = rng.normal(size=(M, 3))
        dvec /= np.linalg.norm(dvec, axis=1, keepdims=True)
        length = rng.uniform(0.5, 2.0, M)
        P1 = C - 0.5 * length[:, None] * dvec
        P2 = C + 0.5 * length[:, None] * dvec
        ok = _visible(Rcw, tcw, P1, s, L, cam, 5.0) & _visible(Rcw, tcw, P2, s, L, cam, 5.0)
        # projected segment length >= 15 px in every track KF (well-defined image line)
        for j in range(int(L.max())):
            m = j < L
            kf = np.where(m, s + j, s)
            u1, v1, _ = _project(Rcw[kf], tcw[kf], P1, cam)
            u2, v2, _ = _project(Rcw[kf], tcw[kf], P2, cam)
            ok &= np.where(m, np.hypot(u2 - u1, v2 - v1) >= 15.0, True)
        take = np.nonzero(ok)[0][: n_ln - have]
        segs.append(np.stack([P1[take], P2[take]], 1)); ln_s.append(s[take]); ln_L.append(L[take])
        have += take.size
    seg = np.concatenate(segs) if n_ln else np.zeros((0, 2, 3))
    ln_s = np.concatenate(ln_s) if n_ln else np.zeros(0, np.int64)
    ln_L = np.concatenate(ln_L) if n_ln else np.zeros(0, np.int64)
    gt_plk = geo.pluker_from_endpoints(seg[:, 0], seg[:, 1]) if n_ln else np.zeros((0, 6))
    gt_orth = geo.pluker_to_orth(gt_plk) if n_ln else np.zeros((0, 4))

    # ---------------- point edges (landmark-major, track order; a revisit observation last)
    if revisit_frac is None:
        revisit_frac = REVISIT_FRAC if name.endswith("R") else 0.0
    E_p = int(pt_L.sum())
    ept_lm = np.repeat(np.arange(n_pt, dtype=np.int32), pt_L)
    offs = np.arange(E_p) - np.repeat(np.cumsum(pt_L) - pt_L, pt_L)
    ept_kf = (np.repeat(pt_s, pt_L) + offs).astype(np.int32)
    if revisit_frac > 0 and n_pt:
        kr = pt_s + pt_L // 2 + revisit_period
        cand = (rng.random(n_pt) < revisit_frac) & (kr < n_kf)
        krc = np.where(cand, kr, 0)
        u, v, z = _project(Rcw[krc], tcw[krc], gt_xyz, cam)
        cand &= (z > 0.5) & (u >= 5) & (u < cam["width"] - 5) & (v >= 5) & (v < cam["height"] - 5)
        extra = np.nonzero(cand)[0]
        if extra.size:
            ends = np.cumsum(pt_L)
            ept_lm = np.insert(ept_lm, ends[extra], extra.astype(np.int32))
            ept_kf = np.insert(ept_kf, ends[extra], krc[extra].astype(np.int32))
            E_p = int(ept_lm.size)
    u, v, _ = _project(Rcw[ept_kf], tcw[ept_kf], gt_xyz[ept_lm], cam)
    ept_obs = np.stack([u, v], -1) + rng.normal(0.0, noise_px, (E_p, 2))
    ept_outlier = rng.random(E_p) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, E_p)
    mag = rng.uniform(20.0, 50.0, E_p)
    ept_obs += (ept_outlier * mag)[:, None] * np.stack([np.cos(ang), np.sin(ang)], -1)

    # ---------------- line edges
    E_l = int(ln_L.sum())
    eln_lm = np.repeat(np.arange(n_ln, dtype=np.int32), ln_L)
    offs = np.arange(E_l) - np.repeat(np.cumsum(ln_L) - ln_L, ln_L)
    eln_kf = (np.repeat(ln_s, ln_L) + offs).astype(np.int32)
    if E_l:
        u1, v1, _ = _project(Rcw[eln_kf], tcw[eln_kf], seg[eln_lm, 0], cam)
        u2, v2, _ = _project(Rcw[eln_kf], tcw[eln_kf], seg[eln_lm, 1], cam)
        eln_obs = np.stack([u1, v1, u2, v2], -1) + rng.normal(0.0, noise_px, (E_l, 4))
        eln_outlier = rng.random(E_l) < outlier_frac
        nrm = np.stack([-(v2 - v1), u2 - u1], -1)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        shift = rng.uniform(20.0, 50.0, E_l) * np.where(rng.random(E_l) < 0.5, -1.0, 1.0) * eln_outlier
        eln_obs[:, 0:2] += shift[:, None] * nrm
        eln_obs[:, 2:4] += shift[:, None] * nrm
    else:
        eln_obs = np.zeros((0, 4))
        eln_outlier = np.zeros(0, dtype=bool)

    # ---------------- initial estimates
    gt_Tcw = np.concatenate([Rcw, tcw[..., None]], -1)
    Rwc0, pwc0 = Rwc.copy(), pwc.copy()
    xyz0 = gt_xyz.copy()
    orth0 = gt_orth.copy()
    if perturb:
        free = np.arange(n_kf) >= n_fix
        dR = geo.rodrigues(rng.normal(0.0, math.radians(0.3), (n_kf, 3)))
        dt = rng.normal(0.0, 0.01, (n_kf, 3))
        Rwc0 = np.where(free[:, None, None], dR @ Rwc, Rwc)
        pwc0 = np.where(free[:, None], pwc + dt, pwc)
        xyz0 = gt_xyz + rng.normal(0.0, 0.03, gt_xyz.shape)
        orth0 = gt_orth + rng.normal(0.0, math.radians(0.3), gt_orth.shape)
    Tcw0 = geo.invert_rigid(np.concatenate([Rwc0, pwc0[..., None]], -1))
    seg0 = seg.reshape(-1, 6) + (rng.normal(0.0, 0.03, (n_ln, 6)) if perturb else 0.0)
    # the map stores NDw; the LBA converts it to orth (src/mapHandler.cpp:6039-6040)
    ln_orth = geo.pluker_to_orth(geo.orth_to_pluker(orth0)) if n_ln else orth0

    kf_id = np.arange(n_kf, dtype=np.int32)
    max_kf_id = n_kf                                  # max(idKF+1)  (src/mapHandler.cpp:5946-5948)
    pt_id = (np.arange(n_pt) + max_kf_id + 1).astype(np.int32)
    max_point_id = int(pt_id[-1]) + 1 if n_pt else max_kf_id   # stray ';' at :6025-6026
    ln_id = (np.arange(n_ln) + max_point_id + 1).astype(np.int32)
    info = float(np.float32(1.0 / 1.0))                # (float)(1/sigma2), sigma2 = 1

    return Graph(
        fx=cam["fx"], fy=cam["fy"], cx=cam["cx"], cy=cam["cy"],
        kf_Tcw=np.ascontiguousarray(Tcw0), kf_fixed=(np.arange(n_kf) < n_fix).astype(np.uint8), kf_id=kf_id,
        pt_xyz=np.ascontiguousarray(xyz0), pt_id=pt_id,
        ln_orth=np.ascontiguousarray(ln_orth), ln_id=ln_id,
        ept_lm=ept_lm, ept_kf=ept_kf, ept_obs=np.ascontiguousarray(ept_obs), ept_info=np.full(E_p, info),
        eln_lm=eln_lm, eln_kf=eln_kf, eln_obs=np.ascontiguousarray(eln_obs), eln_info=np.full(E_l, info),
        gt_Tcw=gt_Tcw, gt_xyz=gt_xyz, gt_orth=gt_orth,
        ept_outlier=ept_outlier.astype(np.uint8), eln_outlier=eln_outlier.astype(np.uint8),
        ln_seg0=np.ascontiguousarray(seg0),
    )


def algorithmic_bytes_per_iter(g: Graph) -> int:
    """SURVEY.md §8d roofline basis: bytes one LM iteration must move at minimum.

    B = 2·(32·E_p + 48·E_l) + 3·(96·N_kf + 24·N_p + 32·N_l) + 288·nnzb + 48·N_free
    with nnzb = Σ_{o=0..7}(N_free−o) for the track band.
    """
    n_free = int((g.kf_fixed == 0).sum())
    nnzb = sum(max(n_free - o, 0) for o in range(8))
    return (2 * (32 * g.n_ept + 48 * g.n_eln) + 3 * (96 * g.n_kf + 24 * g.n_pt + 32 * g.n_ln)
            + 288 * nnzb + 48 * n_free)
