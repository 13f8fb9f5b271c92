"""Synthetic loop-closure pose graphs in the shape
MapHandler::loopClosureOptimizationEssGraphG2O builds (src/mapHandler.cpp:5070-5185):

* one VertexSE3 per keyframe from the loop's first to its last keyframe, estimate = the map pose
  (drifted by accumulated odometry noise);
* EdgeSE3 between every pair that is covisible enough (here: |i-j| <= cov_window) or
  consecutive, measurement = T_i⁻¹·T_j of the CURRENT map poses (so these edges start at zero
  error, :5152-5158);
* one loop edge (loop_i, loop_j) whose measurement is the true relative pose (the loop
  detector's estimate, :5166-5178); vertex 0 and loop_i fixed, loop_j fixed at the
  loop-corrected pose (:5124-5136) — `ess=True`; the CovGraph variant (`ess=False`) leaves
  loop_j free and fixes only vertex 0 (:5354-5368).
Poses are Isometry3, row-major 3x4 [R | t] (camera -> world)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class PoseGraph:
    v_id: np.ndarray      # [n_v] int32
    v_T: np.ndarray       # [n_v][12]
    v_fixed: np.ndarray   # [n_v] uint8
    e_v: np.ndarray       # [n_e][2] int32 (vertex positions)
    e_Z: np.ndarray       # [n_e][12]
    e_info: Optional[np.ndarray] = None
    T_true: Optional[np.ndarray] = None

    def copy(self) -> "PoseGraph":
        return PoseGraph(self.v_id.copy(), self.v_T.copy(), self.v_fixed.copy(), self.e_v.copy(), self.e_Z.copy(),
                         None if self.e_info is None else self.e_info.copy(),
                         None if self.T_true is None else self.T_true.copy())


def rot(axis_angle) -> np.ndarray:
    w = np.asarray(axis_angle, dtype=np.float64)
    th = np.linalg.norm(w)
    if th < 1e-15:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def to4(T12) -> np.ndarray:
    M = np.eye(4)
    M[:3, :] = np.asarray(T12).reshape(3, 4)
    return M


def to12(M) -> np.ndarray:
    return np.asarray(M)[:3, :].reshape(12).copy()


def inv4(M) -> np.ndarray:
    R, t = M[:3, :3], M[:3, 3]
    o = np.eye(4)
    o[:3, :3] = R.T
    o[:3, 3] = -R.T @ t
    return o


def loop_graph(n_kf: int = 40, seed: int = 7, cov_window: int = 3, rot_noise_deg: float = 0.4,
               trans_noise: float = 0.01, ess: bool = True, info: bool = False, extra_loops: int = 0) -> PoseGraph:
    rng = np.random.default_rng(seed)
    # true trajectory: a loop of radius 3 m, yaw following the tangent, small height wobble
    Tt = []
    for k in range(n_kf):
        a = 2 * np.pi * k / n_kf
        M = np.eye(4)
        M[:3, :3] = rot([0, 0, a + np.pi / 2]) @ rot([np.pi / 2, 0, 0])
        M[:3, 3] = [3 * np.cos(a), 3 * np.sin(a), 0.3 * np.sin(3 * a)]
        Tt.append(M)
    # map poses: integrated noisy odometry from the true first pose (drift)
    Te = [Tt[0].copy()]
    for k in range(1, n_kf):
        odo = inv4(Tt[k - 1]) @ Tt[k]
        N = np.eye(4)
        N[:3, :3] = rot(rng.normal(0, np.deg2rad(rot_noise_deg), 3))
        N[:3, 3] = rng.normal(0, trans_noise, 3)
        Te.append(Te[-1] @ odo @ N)
    v_T = np.array([to12(M) for M in Te])
    ev, ez = [], []
    for i in range(n_kf):
        for j in range(i + 1, n_kf):
            if j - i <= cov_window:
                ev.append((i, j))
                ez.append(to12(inv4(Te[i]) @ Te[j]))
    loops = [(0, n_kf - 1)] + [(int(a), int(b)) for a, b in
                               zip(rng.integers(0, n_kf // 3, extra_loops), rng.integers(2 * n_kf // 3, n_kf, extra_loops))]
    fixed = np.zeros(n_kf, np.uint8)
    fixed[0] = 1
    for li, lj in loops:
        ev.append((li, lj))
        ez.append(to12(inv4(Tt[li]) @ Tt[lj]))  # the loop detector's relative pose (true here)
    if ess:
        li, lj = loops[0]
        fixed[li] = 1
        fixed[lj] = 1
        v_T[lj] = to12(Te[li] @ inv4(Tt[li]) @ Tt[lj])  # loop-corrected pose of the loop KF
    e_info = None
    if info:
        m = len(ev)
        e_info = np.zeros((m, 36))
        for e in range(m):
            A = rng.normal(0, 0.3, (6, 6))
            e_info[e] = (np.eye(6) + A @ A.T).reshape(36)
    return PoseGraph(np.arange(n_kf, dtype=np.int32), v_T, fixed, np.array(ev, np.int32), np.array(ez),
                     e_info, np.array([to12(M) for M in Tt]))


def loop_map(n_loop: int = 24, n_after: int = 3, seed: int = 3, pts_per_kf: int = 3, lns_per_kf: int = 1):
    """A SlamMap (plba.slam_map) whose keyframes drift around a loop of n_loop KFs (KF 0 ..
    n_loop-1 closes on KF 0) followed by n_after KFs past the loop, with points / lines attached
    to each KF (map_points_kf_idx / map_lines_kf_idx), a covisibility full_graph (>= 150 shared
    landmarks for |i-j| <= 2) and the loop lists: lc_idxs = lc_idx_list = [(0, n_loop-1, 1)],
    lc_pose_list = [logmap(T_true_j · T_true_0⁻¹)] so expmap(lc_pose)·T_kf_w(0) is the true pose of
    the loop KF. Returns (SlamMap, lc_idxs, lc_idx_list, lc_pose_list, line3d[n_ln][6])."""
    from . import geometry as geo
    from .slam_map import DESC_BYTES, KF, Landmark, SlamMap
    rng = np.random.default_rng(seed)
    pg = loop_graph(n_kf=n_loop + n_after, seed=seed, ess=False)
    n_kf = n_loop + n_after
    Te = [to4(T) for T in pg.v_T]
    Tt = [to4(T) for T in pg.T_true]
    kfs, points, lines, mpk, mlk = [], [], [], {}, {}
    line3d = []
    for k in range(n_kf):
        kfs.append(KF(k, Te[k].copy(), False, [], []))
        mpk[k], mlk[k] = [], []
        for _ in range(pts_per_kf):
            idx = len(points)
            pos = Te[k][:3, :3] @ rng.normal(0, 1, 3) + Te[k][:3, 3]
            d = rng.normal(size=3)
            points.append(Landmark(idx, False, True, pos, [rng.integers(0, 256, DESC_BYTES, dtype=np.uint8)],
                                   [rng.normal(300, 50, 2)], [k], [1.0], [d / np.linalg.norm(d)]))
            mpk[k].append(idx)
        for _ in range(lns_per_kf):
            idx = len(lines)
            P, Q = rng.normal(0, 1, 3) + Te[k][:3, 3], rng.normal(0, 1, 3) + Te[k][:3, 3]
            dv = (Q - P) / np.linalg.norm(Q - P)
            lines.append(Landmark(idx, False, True, np.concatenate([np.cross(P, dv), dv]),
                                  [rng.integers(0, 256, DESC_BYTES, dtype=np.uint8)], [rng.normal(0, 1, 4)], [k], [1.0]))
            line3d.append(np.concatenate([P, Q]))
            mlk[k].append(idx)
    fg = np.zeros((n_kf, n_kf), np.uint32)
    for i in range(n_kf):
        for j in range(n_kf):
            if i != j and abs(i - j) <= 2:
                fg[i, j] = 200
    m = SlamMap(458.654, 457.296, 367.215, 248.375, kfs, points, lines, mpk, fg, mlk, max_kf_idx=n_kf - 1)
    lj = n_loop - 1
    lc = np.array([[0, lj, 1]], np.int32)
    x = geo.logmap_se3(Tt[lj] @ inv4(Tt[0]))
    return m, lc.copy(), lc.copy(), np.array([x]), np.array(line3d)
