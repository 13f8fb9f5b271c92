"""Window of the hand-rolled Levenberg–Marquardt LBA from a map window.

``MapHandler::localBundleAdjustmentForPluker`` (src/mapHandler.cpp:1505-1615) hands
``levMarquardtOptimizationLBAForPluker`` (:1618-2332) the KeyFrame pose vectors ``x_kf_w``
(:1518), the map poses ``T_kf_w`` (read through ``inverse_se3`` at :1657-1659, 1750-1752), the
points ``point3D`` and the lines as ``orthNDw = changePlukerToOrth(NDw)`` (:1577). A KeyFrame
stores ``x_kf_w = logmap_se3(T)`` and ``T_kf_w = expmap_se3(x_kf_w)`` when it is inserted
(:140-141, :179-180); ``NDw`` is the map's Plücker vector with a unit direction (:451-459).
``hlm_window`` derives exactly those inputs from a synthetic window (whose ``kf_Tcw`` are the
camera poses): the product path then sees the reference's own representation.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import geometry as geo
from .synth import Graph


@dataclass
class HlmWindow:
    graph: Graph            # kf_Tcw = inverse_se3(T_kf_w); ln_orth = changePlukerToOrth(NDw)
    kf_x: np.ndarray        # (n_kf, 6) x_kf_w
    ln_pluker: np.ndarray   # (n_ln, 6) NDw
    ln_line3d: Optional[np.ndarray] = None   # (n_ln, 6) line3D endpoints (GBA)


def hlm_window(g: Graph) -> HlmWindow:
    h = g.copy()
    Tcw = np.zeros((g.n_kf, 4, 4))
    Tcw[:, :3, :] = g.kf_Tcw.reshape(-1, 3, 4)
    Tcw[:, 3, 3] = 1.0
    x = geo.logmap_se3(geo.inverse_se3(Tcw))            # x_kf_w = logmap_se3(T_kf_w)
    T_kf_w = geo.expmap_se3(x)                          # T_kf_w = expmap_se3(x_kf_w)
    h.kf_Tcw = np.ascontiguousarray(geo.inverse_se3(T_kf_w)[:, :3, :])
    L = geo.orth_to_pluker(g.ln_orth.reshape(-1, 4)) if g.n_ln else np.zeros((0, 6))
    if g.n_ln:
        L = L / np.linalg.norm(L[:, 3:], axis=1, keepdims=True)   # unit direction, |n| = distance
        h.ln_orth = np.ascontiguousarray(geo.pluker_to_orth(L))
    return HlmWindow(h, np.ascontiguousarray(x), np.ascontiguousarray(L))


def gba_window(g: Graph) -> HlmWindow:
    """``MapHandler::globalBundleAdjustment`` (src/mapHandler.cpp:3022-3126) on a synthetic map:
    every KF but kf_idx 0 is free, lines are their endpoints ``line3D`` (the generator's perturbed
    segments) and each line observation is the image line through the observed endpoints,
    normalised to a² + b² = 1 (StVO's ``le``), in ``eln_obs[:, :3]``."""
    w = hlm_window(g)
    h = w.graph
    h.kf_fixed = (h.kf_id == 0).astype(np.uint8)
    if g.n_eln:
        p1 = np.concatenate([g.eln_obs[:, 0:2], np.ones((g.n_eln, 1))], 1)
        p2 = np.concatenate([g.eln_obs[:, 2:4], np.ones((g.n_eln, 1))], 1)
        le = np.cross(p1, p2)
        le /= np.hypot(le[:, 0], le[:, 1])[:, None]
        h.eln_obs = np.ascontiguousarray(np.concatenate([le, np.zeros((g.n_eln, 1))], 1))
    seg = g.ln_seg0 if g.ln_seg0 is not None else np.zeros((g.n_ln, 6))
    return HlmWindow(h, w.kf_x, w.ln_pluker, np.ascontiguousarray(seg, np.float64).reshape(-1, 6))
