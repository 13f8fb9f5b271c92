"""Graph mutations for edge-case parity tests (shuffles, duplicates, fixed/idle vertices)."""
import numpy as np

from plba.synth import Graph


def shuffled(g: Graph, seed=0) -> Graph:
    """Permute edge order, vertex array order and vertex ids (keeps the same optimisation
    problem up to g2o's id-based ordering)."""
    rng = np.random.default_rng(seed)
    h = g.copy()
    # permute keyframe array order, keep ids attached
    pk = rng.permutation(g.n_kf)
    inv_k = np.argsort(pk)
    h.kf_Tcw, h.kf_fixed, h.kf_id = g.kf_Tcw[pk], g.kf_fixed[pk], g.kf_id[pk]
    h.ept_kf = inv_k[g.ept_kf].astype(np.int32)
    h.eln_kf = inv_k[g.eln_kf].astype(np.int32)
    pp = rng.permutation(g.n_pt)
    inv_p = np.argsort(pp)
    h.pt_xyz, h.pt_id = g.pt_xyz[pp], g.pt_id[pp]
    h.ept_lm = inv_p[g.ept_lm].astype(np.int32)
    # edges in random order
    pe = rng.permutation(g.n_ept)
    h.ept_lm, h.ept_kf, h.ept_obs, h.ept_info = h.ept_lm[pe], h.ept_kf[pe], g.ept_obs[pe], g.ept_info[pe]
    pl = rng.permutation(g.n_eln)
    h.eln_lm, h.eln_kf, h.eln_obs, h.eln_info = g.eln_lm[pl], h.eln_kf[pl], g.eln_obs[pl], g.eln_info[pl]
    h._perm = dict(pk=pk, pp=pp, pe=pe, pl=pl)
    return h


def with_duplicate_observations(g: Graph, every=7) -> Graph:
    """Append a second, slightly different observation of some landmarks by the same KF."""
    h = g.copy()
    sel = np.arange(0, g.n_ept, every)
    h.ept_lm = np.concatenate([g.ept_lm, g.ept_lm[sel]]).astype(np.int32)
    h.ept_kf = np.concatenate([g.ept_kf, g.ept_kf[sel]]).astype(np.int32)
    h.ept_obs = np.concatenate([g.ept_obs, g.ept_obs[sel] + 0.3])
    h.ept_info = np.concatenate([g.ept_info, g.ept_info[sel]])
    return h


def drop_lines(g: Graph) -> Graph:
    h = g.copy()
    h.ln_orth, h.ln_id = g.ln_orth[:0], g.ln_id[:0]
    h.eln_lm, h.eln_kf, h.eln_obs, h.eln_info = g.eln_lm[:0], g.eln_kf[:0], g.eln_obs[:0], g.eln_info[:0]
    return h


def drop_points(g: Graph) -> Graph:
    h = g.copy()
    h.pt_xyz, h.pt_id = g.pt_xyz[:0], g.pt_id[:0]
    h.ept_lm, h.ept_kf, h.ept_obs, h.ept_info = g.ept_lm[:0], g.ept_kf[:0], g.ept_obs[:0], g.ept_info[:0]
    return h


def all_fixed(g: Graph) -> Graph:
    h = g.copy()
    h.kf_fixed = np.ones_like(g.kf_fixed)
    return h


def add_idle_free_pose(g: Graph) -> Graph:
    """A free keyframe that no edge observes (inactive in g2o, must stay untouched)."""
    h = g.copy()
    h.kf_Tcw = np.concatenate([g.kf_Tcw, g.kf_Tcw[-1:]])
    h.kf_fixed = np.concatenate([g.kf_fixed, np.zeros(1, np.uint8)])
    h.kf_id = np.concatenate([g.kf_id, np.array([g.kf_id.max() + 1], np.int32)])
    return h


def fixed_only_landmarks(g: Graph) -> Graph:
    """Re-point the edges of the first landmarks to fixed keyframes only."""
    h = g.copy()
    fixed = np.nonzero(g.kf_fixed)[0]
    sel = g.ept_lm < 20
    h.ept_kf = np.where(sel, fixed[np.arange(g.n_ept) % len(fixed)], g.ept_kf).astype(np.int32)
    return h


def zero_information_keyframe(g: Graph) -> Graph:
    """Ω = 0 on every edge of one free keyframe: the vertex stays active (it has edges) but its
    reduced-camera block row is exactly zero, so with λ = 0 the LDLᵀ meets an exact zero pivot
    in any elimination order (g2o's LinearSolverEigen fails there too)."""
    h = g.copy()
    free = np.nonzero(g.kf_fixed == 0)[0]
    k = free[len(free) // 2]
    h.ept_info = np.where(g.ept_kf == k, 0.0, g.ept_info)
    h.eln_info = np.where(g.eln_kf == k, 0.0, g.eln_info)
    return h
