"""GPU parity on edge cases and API paths (HIP path vs CPU oracle, same inputs)."""
import numpy as np
import pytest

import golden_io
import graph_mut as gm
import oracle_api as oa
from parity import EST_RTOL, assert_parity, compare, assert_trace_parity
from plba import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from plba.lib import Solver
    s = Solver()
    yield s
    s.close()


def _amax(x):
    return float(np.abs(x).max(initial=0.0))


def _check(out, ref, tol=EST_RTOL, elem=1.0):
    m = compare(out, ref)
    assert m["pt_level_diff"] == 0 and m["ln_level_diff"] == 0, m
    assert_parity(m, elem=elem, north=tol)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    np.testing.assert_array_equal(out["ept_depth_ok"], ref["ept_depth_ok"])
    bad_g = (out["ept_chi2"] > 5.991) | (out["ept_depth_ok"] == 0)
    bad_r = (ref["ept_chi2"] > 5.991) | (ref["ept_depth_ok"] == 0)
    np.testing.assert_array_equal(bad_g, bad_r)
    np.testing.assert_array_equal(out["eln_chi2"] > 5.991, ref["eln_chi2"] > 5.991)
    return m


def _run(solver, g, **kw):
    ref = oa.lba_plucker(g, **kw)
    solver.upload(g)
    return solver.lba_plucker(), ref


@pytest.mark.parametrize("cfg", ["C1", "C1L"])
def test_matches_committed_golden(solver, cfg):
    g, exp = golden_io.load(cfg)
    solver.upload(g)
    out = solver.lba_plucker()
    for k in ("kf_Tcw", "pt_xyz", "ln_orth"):
        assert _amax(out[k] - exp[k]) <= EST_RTOL * max(_amax(exp[k]), 1.0), k
    for k in ("ept_level", "eln_level", "ept_depth_ok", "iters"):
        np.testing.assert_array_equal(out[k], exp[k])
    np.testing.assert_allclose(out["ept_chi2"], exp["ept_chi2"], rtol=1e-6, atol=1e-9)


def test_lines_only(solver):
    _check(*_run(solver, gm.drop_points(synth.generate("C1L"))))


def test_points_only_with_lines_config(solver):
    _check(*_run(solver, gm.drop_lines(synth.generate("C1L"))))


def test_no_free_poses(solver):
    # every keyframe fixed: the reduced camera system is empty, landmarks still move
    _check(*_run(solver, gm.all_fixed(synth.generate("C1L"))))


def test_landmarks_seen_only_by_fixed_keyframes(solver):
    _check(*_run(solver, gm.fixed_only_landmarks(synth.generate("C1L"))))


def test_idle_free_pose_untouched(solver):
    g = gm.add_idle_free_pose(synth.generate("C1L"))
    out, ref = _run(solver, g)
    _check(out, ref)
    np.testing.assert_array_equal(out["kf_Tcw"][-1], g.kf_Tcw[-1])


def test_duplicate_observations(solver):
    _check(*_run(solver, gm.with_duplicate_observations(synth.generate("C1L"))))


def test_shuffled_edges_and_ids(solver):
    g = synth.generate("C1L")
    h = gm.shuffled(g, seed=3)
    out, ref = _run(solver, h)
    _check(out, ref)
    # same problem as the unshuffled window (up to rounding)
    solver.upload(g)
    base = solver.lba_plucker()
    pk, pp = h._perm["pk"], h._perm["pp"]
    assert np.abs(out["kf_Tcw"] - base["kf_Tcw"][pk]).max() < 1e-8
    assert np.abs(out["pt_xyz"] - base["pt_xyz"][pp]).max() < 1e-8


@pytest.mark.parametrize("tmax,n_kf,banded", [(12, 24, 1), (12, 12, 1), (16, 16, 1), (30, 30, 1), (60, 60, 0)])
def test_wide_bands_and_dense_fallback(solver, monkeypatch, tmax, n_kf, banded):
    # tmax 12 -> banded kernel with bw 11; 12 / 16 KF -> the band spans every free pose (bw = nf-1:
    # the register window starts full and no row ever enters); tmax 30 -> bw 21 (register-resident band window, up
    # to kBandMax = 27); the 60-KF window with scrambled keyframe ids and no reordering -> an
    # envelope wider than kBandMax (dense path)
    g = synth.generate("C1", n_kf=n_kf, n_pt=400, seed=5 + tmax, track_min=2, track_max=tmax, fixed_frac=0.1)
    if not banded:
        g = g.copy()
        g.kf_id = np.random.default_rng(3).permutation(g.n_kf).astype(np.int32)
        monkeypatch.setenv("PLBA_NO_RCM", "1")
    out, ref = _run(solver, g)
    _check(out, ref)
    st = solver.structure_stats()
    assert st["banded"] == banded and (st["bw"] <= 27) == bool(banded), st


@pytest.mark.parametrize("cfg,kw", [("C2", {}), ("C1", dict(n_kf=60, n_pt=1500, seed=77, track_max=12))])
def test_twisted_factorisation_matches_single_sweep(solver, monkeypatch, cfg, kw):
    # two-sided band LDLᵀ (2 workgroups + separator) vs the one-sided sweep, both vs the oracle;
    # the second case has bw 11 (separator solved by the multi-wave Gauss–Jordan)
    g = synth.generate(cfg, **kw)
    ref = oa.lba_plucker(g)
    solver.upload(g)
    assert solver.structure_stats()["twisted"] == 1
    tw = solver.lba_plucker()
    _check(tw, ref)
    monkeypatch.setenv("PLBA_NO_TWIST", "1")
    solver.upload(g)
    assert solver.structure_stats()["twisted"] == 0
    one = solver.lba_plucker()
    _check(one, ref)
    monkeypatch.delenv("PLBA_NO_TWIST")
    assert np.abs(tw["kf_Tcw"] - one["kf_Tcw"]).max() < 1e-10


@pytest.mark.parametrize("tmax", [2, 3, 5, 8, 10])
@pytest.mark.parametrize("n_kf", [14, 48])
def test_column_lane_factorisation_bandwidths(solver, monkeypatch, tmax, n_kf):
    # column-lane band LDLᵀ (plba_band_cl.hpp) at bandwidths 1..9, single sweep (14 KF) and
    # two-sided (48 KF, bw <= 9 -> nf >= 2bw + 16), vs the oracle and vs the 16-wave kernel
    g = synth.generate("C1L", n_kf=n_kf, n_pt=30 * n_kf, n_ln=6 * n_kf, seed=300 + tmax + n_kf,
                       track_min=2, track_max=tmax, fixed_frac=0.1)
    ref = oa.lba_plucker(g)
    monkeypatch.setenv("PLBA_FACTOR", "cl")
    solver.upload(g)
    st = solver.structure_stats()
    assert st["banded"] == 1 and st["column_lane"] == 1 and st["bw"] <= 9, st
    assert st["twisted"] == (1 if st["nf"] >= 2 * st["bw"] + 16 else 0), st
    cl = solver.lba_plucker()
    # (48 KF / tracks <= 5 is the one ill-conditioned window of the sweep: its stage χ² already
    # differ by 2e-9 relative from the oracle's — rounding of a different elimination order
    # amplified — so its elements agree to 1e-6, not 1e-8; every other case to 4e-10)
    elem = 1e3 if (n_kf, tmax) == (48, 5) else 1.0
    _check(cl, ref, elem=elem)
    monkeypatch.setenv("PLBA_NO_CL", "1")
    solver.upload(g)
    assert solver.structure_stats()["column_lane"] == 0
    old = solver.lba_plucker()
    monkeypatch.delenv("PLBA_NO_CL")
    monkeypatch.delenv("PLBA_FACTOR")
    _check(old, ref, elem=elem)
    assert np.abs(cl["kf_Tcw"] - old["kf_Tcw"]).max() < 1e-9


# Every environment switch the library reads (DESIGN §6 "Switches"), on a window the oracle
# finishes in seconds: the A/B and diagnostic switches must keep the oracle parity, and those that
# only change scheduling, load paths, staging or logging must be bitwise the default solve.
ENV_SWITCHES = [
    ({"PLBA_NO_FOLD_INIT": "1"}, False),       # k_iter_init as its own launch
    ({"PLBA_CHUNK_DIRECT": "1"}, True),        # Schur assembly with per-lane row loads
    ({"PLBA_CHUNK_HALF_MIN": "0"}, False),     # two-lane Schur assembly at any size
    ({"PLBA_CHUNK_TRIPLES": "64"}, False),     # shorter assembly chunks
    ({"PLBA_GRAPH_LEVELS": "1"}, True),        # step graphs of 1-2 steps only
    ({"PLBA_POISON": "1"}, True),              # unwritten arrays start as NaN
    ({"PLBA_TIMING": "1"}, True),              # host-side phase log
    ({"PLBA_HOST_BUILD": "1"}, True),          # host window build
    ({"PLBA_FORCE_DENSE": "1"}, False),        # dense MFMA factorisation of a banded window
    ({"PLBA_DENSE_SCALAR": "1", "PLBA_FORCE_DENSE": "1"}, False),
    ({"PLBA_FACTOR": "bcr", "PLBA_SPEC_BCR": "0"}, False),
    ({"PLBA_FACTOR": "band"}, False),           # 16-wave band kernel
    ({"PLBA_NO_TWIST": "1"}, False),
    ({"PLBA_SPEC": "1"}, True),                # one trial slot
]


@pytest.mark.parametrize("env,bitwise", ENV_SWITCHES, ids=lambda x: ",".join(x) if isinstance(x, dict) else str(x))
def test_environment_switches_keep_parity(solver, monkeypatch, env, bitwise):
    g = synth.generate("C2")
    solver.upload(g)
    base = solver.lba_plucker()
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    solver.upload(g)
    out = solver.lba_plucker()
    for k in env:
        monkeypatch.delenv(k)
    if bitwise:
        for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "eln_level", "iters", "chi2"):
            assert np.array_equal(np.asarray(out[k]), np.asarray(base[k])), (env, k)
    _check(out, oa.lba_plucker(g))


def test_empty_graph(solver):
    g = synth.generate("C1", n_pt=0, n_ln=0)
    out, ref = _run(solver, g)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    assert list(out["iters"]) == [-1, -1]
    np.testing.assert_array_equal(out["kf_Tcw"], g.kf_Tcw)


def test_corrected_line_jacobian_option():
    from plba.lib import Solver
    g = synth.generate("C1L")
    ref = oa.lba_plucker(g, corrected_line_jacobian=1)
    with Solver(corrected_line_jacobian=True) as s:
        s.upload(g)
        out = s.lba_plucker()
    _check(out, ref)
    # and it is a different trajectory from the bug-compatible default
    dflt = oa.lba_plucker(g)
    assert np.abs(dflt["ln_orth"] - ref["ln_orth"]).max() > 1e-9


def test_g2o_style_call_sequence(solver):
    """The reference's call sequence as separate g2o-style calls (src/mapHandler.cpp:6119-6160):
    setRobustKernel(Huber) / initializeOptimization(0) / optimize(5), classification on the host
    from chi2() / isDepthPositive(), setLevel(1), setRobustKernel(0), initializeOptimization(0) /
    optimize(10), computeError() of the level-1 edges, chi2() — equals the oracle's schedule."""
    g = synth.generate("C1L")
    ref1 = oa.lba_plucker(g, stage_iters=(5, 0))
    ref = oa.lba_plucker(g)
    solver.upload(g)
    solver.set_robust(True)
    solver.initialize_optimization(0)
    it, chi = solver.optimize(5)
    assert it == ref1["iters"][0]
    assert abs(chi - ref1["chi2"][0]) <= 1e-6 * ref1["chi2"][0]
    T, P, O = solver.download()
    assert _amax(P - ref1["pt_xyz"]) <= EST_RTOL * _amax(ref1["pt_xyz"])
    assert _amax(O - ref1["ln_orth"]) <= EST_RTOL * max(_amax(ref1["ln_orth"]), 1.0)
    # per-edge chi2 after optimize() follows g2o's last-evaluated semantics
    pc, pd, lc = solver.edge_chi2()
    np.testing.assert_allclose(pc, ref1["ept_chi2"], rtol=1e-6, atol=1e-9)
    # classification (src/mapHandler.cpp:6125-6147) on the host, then stage 2 through the C ABI
    pl = ((pc > 5.991) | (pd == 0)).astype(np.uint8)
    ll = (lc > 5.991).astype(np.uint8)
    np.testing.assert_array_equal(pl, ref["ept_level"])
    np.testing.assert_array_equal(ll, ref["eln_level"])
    solver.set_edge_levels(pl, ll)
    solver.set_robust(False)
    solver.initialize_optimization(0)
    it2, chi2 = solver.optimize(10)
    assert it2 == ref["iters"][1]
    assert abs(chi2 - ref["chi2"][1]) <= 1e-6 * ref["chi2"][1]
    solver.refresh_edge_errors(1)
    pc2, pd2, lc2 = solver.edge_chi2()
    np.testing.assert_allclose(pc2, ref["ept_chi2"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(lc2, ref["eln_chi2"], rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(pd2, ref["ept_depth_ok"])
    T2, P2, O2 = solver.download()
    assert _amax(T2 - ref["kf_Tcw"]) <= EST_RTOL * _amax(ref["kf_Tcw"])
    assert _amax(P2 - ref["pt_xyz"]) <= EST_RTOL * _amax(ref["pt_xyz"])
    assert _amax(O2 - ref["ln_orth"]) <= EST_RTOL * max(_amax(ref["ln_orth"]), 1.0)


def test_set_edge_levels_after_reset_is_ordered(solver):
    """plba_set_edge_levels right after plba_reset_estimates (whose level memset is queued on the
    solver stream): the levels must land after the reset, so stage 2 sees them."""
    g = synth.generate("C1L")
    ref = oa.lba_plucker(g)
    solver.upload(g)
    for _ in range(3):
        solver.reset()
        solver.set_edge_levels(ref["ept_level"], ref["eln_level"])
        solver.set_robust(False)
        solver.initialize_optimization(1)   # only the level-1 edges: non-empty iff the levels landed
        it, _ = solver.optimize(1)
        assert it == 1


def test_zero_pivot_rejects_every_trial():
    """LinearSolverEigen fails iff an LDLᵀ pivot is exactly 0: with τ = 0
    (λ = 0) a free keyframe whose edges all carry Ω = 0 stays active but leaves an exactly zero
    6x6 block on the reduced camera diagonal, so every solve of the Huber stage fails, every
    trial is rejected with the previous x (g2o still calls update), and optimize(5) stops after
    maxTrials with Terminate — the same path as the oracle's stage 1."""
    from plba.lib import Solver
    g = gm.zero_information_keyframe(synth.generate("C1L", track_min=3, seed=41))
    ref = oa.lba_plucker(g, tau=0.0, stage_iters=(5, 0))
    tr_ref = ref["trace"]
    assert len(tr_ref) == 1 and tr_ref[0]["trials"] == 10 and tr_ref[0]["result"] == 1, tr_ref
    with Solver(tau=0.0) as s:
        s.upload(g)
        s.set_robust(True)
        s.initialize_optimization(0)
        it, chi = s.optimize(5)
        tr = s.trace()
        T, P, O = s.download()
    assert it == ref["iters"][0] == 1
    assert len(tr) == 1 and tr[0]["trials"] == 10 and tr[0]["result"] == 1, tr
    assert tr[0]["lambda_start"] == 0.0 and tr[0]["lambda_end"] == 0.0
    assert abs(chi - ref["chi2"][0]) <= 1e-9 * ref["chi2"][0]
    # nothing moved: every trial was popped
    np.testing.assert_array_equal(T, g.kf_Tcw)
    np.testing.assert_array_equal(P, g.pt_xyz)
    np.testing.assert_array_equal(O, g.ln_orth)


@pytest.mark.slow
@pytest.mark.parametrize("cfg", ["C3", "C4", "C5"])
def test_large_configs_match_oracle(solver, cfg):
    """C3 (two-sided column-lane), C4 and C5 (block cyclic reduction): estimates, iteration counts,
    classification and depth flags, and the per-iteration trace of both stages."""
    g = synth.generate(cfg)
    out, ref = _run(solver, g)
    _check(out, ref)
    assert_trace_parity(out, ref)


def test_idle_free_pose_is_inactive_at_zero_lambda():
    """A free keyframe with no edge is not an active vertex in g2o, so it is not in the linear
    system at all: even at λ = 0 (τ = 0) it must not make the solve fail (its block is I, x = 0),
    and the solve must be the one of the same window without it. (At λ = 0 the Huber stage is a
    Gauss–Newton step on a barely conditioned system, so the comparison is GPU vs GPU; the oracle
    agrees on the trial count and on the pose staying put.)"""
    from plba.lib import Solver
    base = synth.generate("C1L", track_min=3, seed=41)
    g = gm.add_idle_free_pose(base)
    ref = oa.lba_plucker(g, tau=0.0, stage_iters=(5, 0))
    res = []
    for h in (g, base):
        with Solver(tau=0.0) as s:
            s.upload(h)
            s.set_robust(True)
            s.initialize_optimization(0)
            it, chi = s.optimize(5)
            tr = s.trace()
            T, P, O = s.download()
        res.append((it, chi, tr, T, P, O))
    (it, chi, tr, T, P, O), (it0, chi0, tr0, T0, P0, O0) = res
    assert it == it0 == ref["iters"][0]
    assert [int(t["trials"]) for t in tr] == [int(t["trials"]) for t in tr0] == [int(t["trials"]) for t in ref["trace"]]
    assert abs(chi - chi0) <= 1e-9 * chi0
    assert _amax(T[:-1] - T0) <= 1e-9 and _amax(P - P0) <= 1e-9 * _amax(P0)
    np.testing.assert_array_equal(T[-1], g.kf_Tcw[-1])
    np.testing.assert_array_equal(ref["kf_Tcw"][-1], g.kf_Tcw[-1])


def test_column_lane_large_nf_lds(solver):
    """Two-sided column-lane factorisation with an x_p staging area past 64 KB of LDS (nf > 432 at
    bw 9): the kernel's dynamic-LDS attribute must be raised for it."""
    g = synth.generate("C1", n_kf=520, n_pt=9000, seed=909, track_min=2, track_max=10, fixed_frac=0.1)
    out, ref = _run(solver, g)
    st = solver.structure_stats()
    assert st["bw"] == 9 and st["nf"] > 432, st
    _check(out, ref, elem=1e3)  # 468 free poses, tracks up to 10 KFs: elements agree to 1e-7


@pytest.mark.parametrize("tmax,n_kf", [(2, 12), (3, 30), (5, 40), (8, 64), (8, 100), (10, 60), (10, 130)])
def test_block_cyclic_reduction_matches_oracle(solver, monkeypatch, tmax, n_kf):
    """Block cyclic reduction over super-rows of bw pose blocks (plba_bcr.hpp), forced on, at
    bandwidths 1..9 and super-row counts 2..16 (odd and even, powers of two and not), against
    the oracle and against the column-lane factorisation of the same window."""
    g = synth.generate("C1L", n_kf=n_kf, n_pt=25 * n_kf, n_ln=5 * n_kf, seed=500 + tmax + n_kf,
                       track_min=2, track_max=tmax, fixed_frac=0.1)
    ref = oa.lba_plucker(g)
    monkeypatch.setenv("PLBA_FACTOR", "bcr")
    solver.upload(g)
    st = solver.structure_stats()
    assert st["banded"] == 1 and st["bcr_rows"] == -(-st["nf"] // st["bw"]) >= 2, st
    out = solver.lba_plucker()
    _check(out, ref)
    solver.reset()
    again = solver.lba_plucker()          # epoch-tagged hand-offs: a rerun is bitwise identical
    for k in ("kf_Tcw", "pt_xyz", "ln_orth"):
        assert np.array_equal(out[k], again[k]), k
    monkeypatch.setenv("PLBA_FACTOR", "cl")
    solver.upload(g)
    assert solver.structure_stats()["bcr_rows"] == 0
    cl = solver.lba_plucker()
    monkeypatch.delenv("PLBA_FACTOR")
    assert np.abs(out["kf_Tcw"] - cl["kf_Tcw"]).max() < 1e-9


def test_bcr_handoff_timeout_falls_back_to_column_lane(monkeypatch):
    """The failure path of BCR's bounded hand-off waits (plba_bcr.hpp bcr_poll). With PLBA_DIAG
    bit 64 every wait times out at once: the guards must stop the rest of that batch, and the host
    must restore the schedule's starting state and re-solve the SAME window in the same context
    with the column-lane factorisation — the result equals the oracle, never PLBA_E_DEVICE.
    The context then keeps the column-lane factorisation: a rerun and a re-upload on it match the
    oracle too."""
    from plba.lib import Solver
    g = synth.generate("C1L", n_kf=64, n_pt=1600, n_ln=320, seed=640, track_min=2, track_max=8,
                       fixed_frac=0.1)
    ref = oa.lba_plucker(g)
    monkeypatch.setenv("PLBA_FACTOR", "bcr")
    monkeypatch.setenv("PLBA_DIAG", "64")
    s = Solver()
    try:
        s.upload(g)
        assert s.structure_stats()["bcr_rows"] >= 4
        out = s.lba_plucker()
        st = s.structure_stats()
        assert st["bcr_fallbacks"] == 1 and st["bcr_rows"] == 0 and st["column_lane"] == 1, st
        _check(out, ref)
        s.reset()
        again = s.lba_plucker()           # same context after the fallback
        _check(again, ref)
        for k in ("kf_Tcw", "pt_xyz", "ln_orth"):
            assert np.array_equal(out[k], again[k]), k
        s.upload(g)                       # re-upload: the context keeps the column-lane choice
        assert s.structure_stats()["bcr_rows"] == 0
        _check(s.lba_plucker(), ref)
    finally:
        s.close()
    monkeypatch.delenv("PLBA_DIAG")
    s = Solver()                          # a fresh context uses BCR again
    try:
        s.upload(g)
        assert s.structure_stats()["bcr_rows"] >= 4
        out2 = s.lba_plucker()
        assert s.structure_stats()["bcr_fallbacks"] == 0
    finally:
        s.close()
    _check(out2, ref)


def test_bcr_hand_rolled_lm_fallback(monkeypatch):
    """The same fallback under the hand-rolled LM (its uploaded se(3) state and NDw are part of
    the restored starting state)."""
    from plba import capi
    from plba.hlm import hlm_window
    from plba.lib import Solver
    g = synth.generate("C1L", n_kf=64, n_pt=1600, n_ln=320, seed=641, track_min=2, track_max=8,
                       fixed_frac=0.1)
    win = hlm_window(g)
    monkeypatch.setenv("PLBA_FACTOR", "bcr")
    p = capi.hlm_params(lambda0=1e-24, err_per_obs=1)
    with Solver() as s:
        s.upload(win.graph)
        assert s.structure_stats()["bcr_rows"] >= 4
        base = s.hlm_lba(win, p)
    monkeypatch.setenv("PLBA_DIAG", "64")
    with Solver() as s:
        s.upload(win.graph)
        out = s.hlm_lba(win, p)
        assert s.structure_stats()["bcr_fallbacks"] == 1
    assert (out["linearizations"], out["solves"], out["accepted"]) == (base["linearizations"], base["solves"],
                                                                      base["accepted"])
    for k in ("kf_x", "pt_xyz", "ln_orth", "kf_Tcw"):
        np.testing.assert_allclose(out[k], base[k], rtol=1e-9, atol=1e-12)


def test_bcr_residency_limit_selects_column_lane(monkeypatch, solver):
    """BCR is chosen only when its workgroups fit the device at once (CUs x occupancy); a limit
    below the window's super-row count (PLBA_BCR_RESIDENT) must select the column-lane path."""
    g = synth.generate("C1L", n_kf=100, n_pt=2500, n_ln=500, seed=642, track_min=2, track_max=8,
                       fixed_frac=0.1)
    monkeypatch.setenv("PLBA_FACTOR", "bcr")
    solver.upload(g)
    n_rows = solver.structure_stats()["bcr_rows"]
    assert n_rows >= 8
    monkeypatch.setenv("PLBA_BCR_RESIDENT", str(n_rows - 1))
    solver.upload(g)
    st = solver.structure_stats()
    assert st["bcr_rows"] == 0 and st["column_lane"] == 1, st
    _check(solver.lba_plucker(), oa.lba_plucker(g))
