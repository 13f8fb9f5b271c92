"""Vectorised SE(3) / Plücker / orthonormal-line helpers (host side, numpy).

These restate the map-model conversions the LBA path uses at its boundary:

* ``pluker_to_orth``  — ``MapLine::changePlukerToOrth``  (src/mapFeatures.cpp:186-201)
* ``orth_to_pluker``  — ``MapLine::changeOrthToPluker``  (src/mapFeatures.cpp:203-224)
* ``orth_R_from_pluker`` / ``orth_W_from_pluker``        (src/mapFeatures.cpp:226-249)

All functions take arrays with a leading batch dimension. Everything is float64.
"""
from __future__ import annotations

import numpy as np


def skew(v: np.ndarray) -> np.ndarray:
    """``vechat`` (g2o_types/g2o_types.h:18-24), batched: (...,3) -> (...,3,3)."""
    v = np.asarray(v, dtype=np.float64)
    z = np.zeros(v.shape[:-1])
    return np.stack([
        np.stack([z, -v[..., 2], v[..., 1]], -1),
        np.stack([v[..., 2], z, -v[..., 0]], -1),
        np.stack([-v[..., 1], v[..., 0], z], -1),
    ], -2)


def rot_xyz(theta: np.ndarray) -> np.ndarray:
    """U(θ1,θ2,θ3) as written in ``changeOrthToPluker`` (src/mapFeatures.cpp:205-215)."""
    theta = np.asarray(theta, dtype=np.float64)
    s1, c1 = np.sin(theta[..., 0]), np.cos(theta[..., 0])
    s2, c2 = np.sin(theta[..., 1]), np.cos(theta[..., 1])
    s3, c3 = np.sin(theta[..., 2]), np.cos(theta[..., 2])
    return np.stack([
        np.stack([c2 * c3, s1 * s2 * c3 - c1 * s3, c1 * s2 * c3 + s1 * s3], -1),
        np.stack([c2 * s3, s1 * s2 * s3 + c1 * c3, c1 * s2 * s3 - s1 * c3], -1),
        np.stack([-s2, s1 * c2, c1 * c2], -1),
    ], -2)


def orth_to_pluker(orth: np.ndarray) -> np.ndarray:
    """(...,4) orth -> (...,6) Plücker [n; d] (src/mapFeatures.cpp:203-224)."""
    orth = np.asarray(orth, dtype=np.float64)
    R = rot_xyz(orth[..., :3])
    w1 = np.cos(orth[..., 3])[..., None]
    w2 = np.sin(orth[..., 3])[..., None]
    return np.concatenate([w1 * R[..., :, 0], w2 * R[..., :, 1]], -1)


def orth_R_from_pluker(L: np.ndarray) -> np.ndarray:
    """``getOrhtRFromPluker`` (src/mapFeatures.cpp:226-239)."""
    n0 = L[..., :3]
    d0 = L[..., 3:]
    n = n0 / np.linalg.norm(n0, axis=-1, keepdims=True)
    d = d0 / np.linalg.norm(d0, axis=-1, keepdims=True)
    c = np.cross(n0, d0)
    c = c / np.linalg.norm(c, axis=-1, keepdims=True)
    return np.stack([n, d, c], -1)


def orth_W_from_pluker(L: np.ndarray) -> np.ndarray:
    """``getOrthWFromPluker`` (src/mapFeatures.cpp:241-249) -> (...,2,2)."""
    nn = np.linalg.norm(L[..., :3], axis=-1)
    dn = np.linalg.norm(L[..., 3:], axis=-1)
    f = np.sqrt(nn * nn + dn * dn)
    return np.stack([np.stack([nn / f, -dn / f], -1), np.stack([dn / f, nn / f], -1)], -2)


def pluker_to_orth(L: np.ndarray) -> np.ndarray:
    """(...,6) Plücker -> (...,4) orth (src/mapFeatures.cpp:186-201)."""
    L = np.asarray(L, dtype=np.float64)
    R = orth_R_from_pluker(L)
    W = orth_W_from_pluker(L)
    u1, u2, u3 = R[..., :, 0], R[..., :, 1], R[..., :, 2]
    return np.stack([
        np.arctan2(u2[..., 2], u3[..., 2]),
        np.arcsin(-u1[..., 2]),
        np.arctan2(u1[..., 1], u1[..., 0]),
        np.arcsin(W[..., 1, 0]),
    ], -1)


def pluker_from_endpoints(P1: np.ndarray, P2: np.ndarray) -> np.ndarray:
    """Normalised Plücker line through two points, built as the reference builds
    ``NDw`` (src/mapHandler.cpp:451-459): unit direction, moment scaled so that
    ``|n| = |n_raw| / |d_raw|`` (the distance of the line from the origin)."""
    d = P2 - P1
    n = np.cross(P1, P2)
    dn = np.linalg.norm(d, axis=-1, keepdims=True)
    nn = np.linalg.norm(n, axis=-1, keepdims=True)
    ratio = nn / dn
    return np.concatenate([n / nn * ratio, d / dn], -1)


def rodrigues(w: np.ndarray) -> np.ndarray:
    """Rotation matrix exp([w]x), batched (...,3)->(...,3,3)."""
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w, axis=-1)[..., None, None]
    K = skew(w)
    th_safe = np.where(th < 1e-12, 1.0, th)
    A = np.where(th < 1e-12, 1.0, np.sin(th_safe) / th_safe)
    B = np.where(th < 1e-12, 0.5, (1.0 - np.cos(th_safe)) / (th_safe * th_safe))
    eye = np.broadcast_to(np.eye(3), K.shape)
    return eye + A * K + B * (K @ K)


def invert_rigid(T: np.ndarray) -> np.ndarray:
    """Inverse of rigid transforms given as (...,3,4) [R|t] -> (...,3,4)."""
    R = T[..., :3, :3]
    t = T[..., :3, 3]
    Rt = np.swapaxes(R, -1, -2)
    return np.concatenate([Rt, -(Rt @ t[..., None])], -1)


def transform_pluker(Tcw: np.ndarray, L: np.ndarray) -> np.ndarray:
    """L_c = [[R, [t]x R], [0, R]] L_w  (g2o_types/g2o_types.h:357-365)."""
    R = Tcw[..., :3, :3]
    t = Tcw[..., :3, 3]
    n = L[..., :3]
    d = L[..., 3:]
    nc = (R @ n[..., None])[..., 0] + (skew(t) @ R @ d[..., None])[..., 0]
    dc = (R @ d[..., None])[..., 0]
    return np.concatenate([nc, dc], -1)


def expmap_se3(x: np.ndarray) -> np.ndarray:
    """``expmap_se3`` (src2/auxiliar.cpp:124-141), batched (...,6) [t; ω] -> (...,4,4)."""
    x = np.asarray(x, dtype=np.float64)
    w = x[..., 3:]
    t = x[..., :3]
    th = np.linalg.norm(w, axis=-1)[..., None, None]
    small = th < 0.000001
    ths = np.where(small, 1.0, th)
    s = skew(w) / ths
    ss = s @ s
    eye = np.broadcast_to(np.eye(3), s.shape)
    R = np.where(small, eye, eye + s * np.sin(ths) + ss * (1.0 - np.cos(ths)))
    V = eye + s * (1.0 - np.cos(ths)) / ths + ss * (ths - np.sin(ths)) / ths
    tt = np.where(small[..., 0], t, (V @ t[..., None])[..., 0])
    T = np.zeros(x.shape[:-1] + (4, 4))
    T[..., :3, :3] = R
    T[..., :3, 3] = tt
    T[..., 3, 3] = 1.0
    return T


def logmap_se3(T: np.ndarray) -> np.ndarray:
    """``logmap_se3`` (src2/auxiliar.cpp:143-173), batched (...,4,4) -> (...,6) [t; ω]."""
    T = np.asarray(T, dtype=np.float64)
    R = T[..., :3, :3]
    Vt = T[..., :3, 3]
    cosine = np.clip((np.trace(R, axis1=-2, axis2=-1) - 1.0) / 2.0, -1.0, 1.0)
    sine = np.clip(np.sqrt(1.0 - cosine * cosine), -1.0, 1.0)
    theta = np.arccos(cosine)
    big = theta > 0.000001
    ths = np.where(big, theta, 1.0)
    sn = np.where(big, sine, 1.0)
    w_hat = ths[..., None, None] * (R - np.swapaxes(R, -1, -2)) / (2.0 * sn[..., None, None])
    w = np.stack([w_hat[..., 2, 1], w_hat[..., 0, 2], w_hat[..., 1, 0]], -1)
    w = np.where(big[..., None], w, 0.0)
    s = skew(w) / ths[..., None, None]
    eye = np.broadcast_to(np.eye(3), R.shape)
    V = eye + s * ((1.0 - cosine) / ths)[..., None, None] + (s @ s) * ((ths - sine) / ths)[..., None, None]
    V = np.where(big[..., None, None], V, eye)
    t = (np.linalg.inv(V) @ Vt[..., None])[..., 0]
    return np.concatenate([t, w], -1)


def inverse_se3(T: np.ndarray) -> np.ndarray:
    """``inverse_se3`` (src2/auxiliar.cpp:113-122), batched (...,4,4) -> (...,4,4)."""
    T = np.asarray(T, dtype=np.float64)
    out = np.zeros_like(T)
    Rt = np.swapaxes(T[..., :3, :3], -1, -2)
    out[..., :3, :3] = Rt
    out[..., :3, 3] = -(Rt @ T[..., :3, 3][..., None])[..., 0]
    out[..., 3, 3] = 1.0
    return out
