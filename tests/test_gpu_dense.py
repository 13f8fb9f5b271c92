"""Wide reduced camera systems: reverse Cuthill–McKee pose reordering and the dense
multi-workgroup LDLᵀ with MFMA trailing updates (csrc/plba_dense.hpp), vs the CPU oracle.

LinearSolverEigen orders the reduced camera system by AMD and factorises it
exactly; any symmetric reordering and any exact factorisation give the same solution up to
rounding, so the bar is the usual one (1e-4 relative on every estimate, identical iteration
counts and outlier classification)."""
import numpy as np
import pytest

import oracle_api as oa
from parity import EST_RTOL, assert_parity, compare
from plba import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from plba.lib import Solver
    s = Solver()
    yield s
    s.close()


def _check(out, ref):
    m = compare(out, ref)
    assert m["pt_level_diff"] == 0 and m["ln_level_diff"] == 0, m
    assert_parity(m)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    return m


def _scramble_ids(g, seed=11):
    """Random keyframe ids (the fixed flags stay with their keyframes): the id order g2o builds
    the Hessian in no longer follows the trajectory, so the natural envelope is wide."""
    h = g.copy()
    rng = np.random.default_rng(seed)
    h.kf_id = rng.permutation(g.n_kf).astype(np.int32)
    return h


@pytest.mark.parametrize("cfg,kw", [("C2", {}), ("C1L", dict(n_kf=40, n_pt=800, n_ln=160, seed=43))])
def test_rcm_recovers_band_for_scrambled_ids(solver, monkeypatch, cfg, kw):
    g = _scramble_ids(synth.generate(cfg, **kw))
    ref = oa.lba_plucker(g)
    solver.upload(g)
    st = solver.structure_stats()
    # the reordering finds a band the banded kernels take again (C2: the column-lane one)
    assert st["banded"] == 1 and st["bw"] <= (9 if cfg == "C2" else 20), st
    _check(solver.lba_plucker(), ref)
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    solver.upload(g)
    st2 = solver.structure_stats()
    assert st2["bw"] > st["bw"], (st, st2)
    _check(solver.lba_plucker(), ref)


def test_revisit_window_reordered(solver):
    """C2R: landmarks re-observed one loop later couple poses ~126 apart (natural envelope ~129
    blocks); RCM folds the loop into a band the banded kernels take."""
    g = synth.generate("C2R")
    ref = oa.lba_plucker(g)
    solver.upload(g)
    st = solver.structure_stats()
    assert st["banded"] == 1 and st["bw"] <= 20, st
    _check(solver.lba_plucker(), ref)


@pytest.mark.parametrize("cfg,kw", [("C2R", {}), ("C1", dict(n_kf=30, n_pt=400, seed=35, track_max=30)),
                                    ("C1", dict(n_kf=70, n_pt=1200, seed=36, track_max=70))])
def test_dense_mfma_factorisation(solver, monkeypatch, cfg, kw):
    """The dense path (no reordering, or an envelope no order can narrow): blocked LDLᵀ on many
    workgroups with v_mfma_f64_16x16x4 trailing updates, and the scalar single-workgroup kernel,
    both against the oracle."""
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    monkeypatch.setenv("PLBA_FORCE_DENSE", "1")  # (the 30-KF window's bw 26 is banded otherwise)
    g = synth.generate(cfg, **kw)
    ref = oa.lba_plucker(g)
    solver.upload(g)
    st = solver.structure_stats()
    assert st["banded"] == 0 and st["dense_mfma"] == 1, st
    mf = solver.lba_plucker()
    _check(mf, ref)
    monkeypatch.setenv("PLBA_DENSE_SCALAR", "1")
    solver.upload(g)
    assert solver.structure_stats()["dense_mfma"] == 0
    sc = solver.lba_plucker()
    _check(sc, ref)
    assert np.abs(mf["kf_Tcw"] - sc["kf_Tcw"]).max() < 1e-9


def test_revisit_window_wide_band(solver):
    """C3R: the loop revisit folds (RCM) into a band of 23 pose blocks — wider than the 20 the
    former LDS window held — so it runs k_rcs_factor_band's register-resident window (bw up to
    kBandMax = 27) instead of the dense path; parity with the oracle."""
    g = synth.generate("C3R")
    ref = oa.lba_plucker(g)
    solver.upload(g)
    st = solver.structure_stats()
    assert st["banded"] == 1 and 20 < st["bw"] <= 24 and st["dense_mfma"] == 0, st
    _check(solver.lba_plucker(), ref)


def _ids_in_order(g, order):
    """Keyframe ids that put the free poses in `order` (the id order g2o builds the Hessian in);
    fixed keyframes after them."""
    h = g.copy()
    free = np.where(g.kf_fixed == 0)[0]
    fixed = np.where(g.kf_fixed != 0)[0]
    ids = np.empty(g.n_kf, np.int32)
    ids[free[order]] = np.arange(len(free), dtype=np.int32)
    ids[fixed] = len(free) + np.arange(len(fixed), dtype=np.int32)
    h.kf_id = ids
    return h


def test_band_window_at_the_widest_band(solver, monkeypatch):
    """Bandwidths 25..kBandMax = 27 run 512-thread band workgroups owning whole 6x6 blocks (bw <= 24:
    768 threads, half blocks). C3R in SciPy's reverse Cuthill-McKee order (bandwidth 27; this
    library's own RCM finds 23) with the reordering off: banded at bw 27, parity with the oracle."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    g = synth.generate("C3R")
    free = np.where(g.kf_fixed == 0)[0]
    hid = -np.ones(g.n_kf, np.int64)
    hid[free] = np.arange(len(free))
    lm = np.concatenate([g.ept_lm, g.n_pt + g.eln_lm])
    kf = np.concatenate([g.ept_kf, g.eln_kf])
    m = hid[kf] >= 0
    A = sp.csr_matrix((np.ones(int(m.sum())), (hid[kf[m]], lm[m])), shape=(len(free), g.n_pt + g.n_ln))
    order = np.asarray(reverse_cuthill_mckee((A @ A.T).tocsr(), symmetric_mode=True))
    h = _ids_in_order(g, order)
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    ref = oa.lba_plucker(h)
    solver.upload(h)
    st = solver.structure_stats()
    assert st["banded"] == 1 and 24 < st["bw"] <= 27 and st["dense_mfma"] == 0, st
    _check(solver.lba_plucker(), ref)


def test_dense_mfma_hand_rolled_lm(solver, monkeypatch):
    """The hand-rolled LM (plba_hlm_lba) through the dense path."""
    from plba import capi
    from plba.hlm import hlm_window
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    monkeypatch.setenv("PLBA_FORCE_DENSE", "1")
    win = hlm_window(synth.generate("C1", n_kf=30, n_pt=400, seed=35, track_max=30))
    p = capi.hlm_params(err_per_obs=1)
    ref = oa.hlm_lba(win, p)
    solver.upload(win.graph)
    assert solver.structure_stats()["dense_mfma"] == 1
    out = solver.hlm_lba(win, p)
    assert out["linearizations"] == ref["linearizations"] and out["accepted"] == ref["accepted"]
    d = np.abs(ref["pt_xyz"] - win.graph.pt_xyz).max()
    assert np.abs(out["pt_xyz"] - ref["pt_xyz"]).max() <= 1e-4 * d + 1e-12


def test_dense_solve_with_y_in_global_memory(solver, monkeypatch):
    """Windows with n > kSolveLdsN keep the substitution vector in global memory instead of LDS;
    PLBA_SOLVE_LDS_N=0 takes that path at a size the oracle finishes. Same operations in the same
    order as the LDS path, so the two agree bitwise."""
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    monkeypatch.setenv("PLBA_FORCE_DENSE", "1")
    g = synth.generate("C1", n_kf=30, n_pt=400, seed=35, track_max=30)
    ref = oa.lba_plucker(g)
    solver.upload(g)
    assert solver.structure_stats()["dense_mfma"] == 1
    lds = solver.lba_plucker()
    monkeypatch.setenv("PLBA_SOLVE_LDS_N", "0")
    solver.upload(g)
    glob = solver.lba_plucker()
    _check(glob, ref)
    np.testing.assert_array_equal(glob["kf_Tcw"], lds["kf_Tcw"])
    np.testing.assert_array_equal(glob["pt_xyz"], lds["pt_xyz"])
