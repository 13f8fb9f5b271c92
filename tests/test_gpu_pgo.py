"""Loop-closure pose graph on the GPU (plba_pgo_optimize) against the CPU
oracle (oracle/refpgo.cpp). MapHandler::loopClosureOptimization{EssGraph,CovGraph}G2O
(src/mapHandler.cpp:5070-5531) run g2o's computeInitialGuess + Levenberg over VertexSE3 /
EdgeSE3 with Cholmod; here the initial guess is the same host algorithm, the edge arithmetic is
compiled without contraction like the oracle, and the solve is a dense LDLᵀ (oracle: dense
Cholesky) — so the initial χ² agrees to rounding and the trajectories agree until the
decisions reach the rounding floor of χ² (the last, terminating iteration). Parity unpinned
against g2o itself (no fixtures)."""
import numpy as np
import pytest

import oracle_api as oa
from plba import capi, pgo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from plba.lib import Solver
    s = Solver()
    yield s
    s.close()


def _compare(out, ref, pose_tol=1e-7):
    assert out["n_free"] == ref["n_free"]
    assert abs(out["chi2_initial"] - ref["chi2_initial"]) <= 1e-12 * max(ref["chi2_initial"], 1e-30)
    # trajectory: the iterations that still make progress agree exactly in trials and to rounding
    # in χ²; once χ² sits at its rounding floor (relative change < 1e-10) the accept / reject
    # decisions compare numbers equal to rounding and may differ, so only the end state is checked
    tr, rt = out["trace"], ref["trace"]
    fin = ref["chi2_final"]
    k = int(np.sum(np.abs(rt["chi2_start"] - fin) > 1e-10 * fin))
    k = min(k, len(tr), len(rt))
    assert k >= 1, (tr, rt)
    np.testing.assert_array_equal(tr["trials"][:k], rt["trials"][:k])
    np.testing.assert_allclose(tr["chi2_end"][:k], rt["chi2_end"][:k], rtol=1e-9)
    assert abs(out["chi2_final"] - ref["chi2_final"]) <= 1e-8 * ref["chi2_final"] + 1e-14
    scale = max(np.abs(ref["v_T"]).max(), 1.0)
    assert np.abs(out["v_T"] - ref["v_T"]).max() <= pose_tol * scale


@pytest.mark.parametrize("kw", [dict(n_kf=40, seed=11, ess=True), dict(n_kf=40, seed=11, ess=False),
                                dict(n_kf=60, seed=5, cov_window=5, extra_loops=3, info=True),
                                dict(n_kf=150, seed=9, cov_window=4, extra_loops=6)])
def test_pgo_matches_oracle(solver, kw):
    pg = pgo.loop_graph(**kw)
    ref = oa.pgo_optimize(pg)
    out = solver.pgo_optimize(pg)
    assert out["chi2_final"] < 0.2 * out["chi2_initial"]
    _compare(out, ref)
    # the fixed vertices keep their estimates
    fx = pg.v_fixed.astype(bool)
    np.testing.assert_array_equal(out["v_T"][fx], pg.v_T[fx])


def test_pgo_without_initial_guess_and_tau_lambda(solver):
    pg = pgo.loop_graph(n_kf=30, seed=21, ess=False)
    p = capi.pgo_params(initial_guess=0, user_lambda_init=0.0, max_iters=20)
    _compare(solver.pgo_optimize(pg, p), oa.pgo_optimize(pg, p))


def test_pgo_non_positive_definite_rejects_trials(solver):
    """An indefinite information matrix makes H + λI indefinite at small λ: Cholmod fails, the
    trial is rejected (χ² = max) and λ grows until the system is positive definite."""
    pg = pgo.loop_graph(n_kf=20, seed=4, ess=False)
    m = len(pg.e_v)
    info = np.tile(np.eye(6).reshape(36), (m, 1))
    info[:, 35] = -0.5  # Ω_55 < 0 on every edge
    pg.e_info = info
    p = capi.pgo_params(max_iters=8)
    ref = oa.pgo_optimize(pg, p)
    out = solver.pgo_optimize(pg, p)
    assert ref["solve_fails"] > 0 and out["solve_fails"] == ref["solve_fails"], (out["solve_fails"], ref["solve_fails"])
    assert out["iterations"] == ref["iterations"] and out["trials"] == ref["trials"]
    np.testing.assert_allclose(out["trace"]["lambda_end"], ref["trace"]["lambda_end"], rtol=1e-12)


def test_pgo_rerun_is_bitwise_deterministic(solver):
    pg = pgo.loop_graph(n_kf=50, seed=13, extra_loops=2)
    a = solver.pgo_optimize(pg)
    b = solver.pgo_optimize(pg)
    assert np.array_equal(a["v_T"], b["v_T"]) and a["trials"] == b["trials"]


def test_pgo_leaves_an_uploaded_window_intact(solver):
    from plba import synth
    g = synth.generate("C1L")
    solver.upload(g)
    before = solver.lba_plucker()
    solver.pgo_optimize(pgo.loop_graph(n_kf=25, seed=2))
    solver.reset()
    after = solver.lba_plucker()
    assert np.array_equal(before["kf_Tcw"], after["kf_Tcw"])


def test_pgo_solve_with_y_in_global_memory(solver, monkeypatch):
    """Pose graphs with n > kSolveLdsN (about 1000 keyframes) substitute with y in global memory;
    PLBA_SOLVE_LDS_N=0 takes that path on a graph the oracle finishes: same as the LDS path
    bitwise, and the oracle's trajectory."""
    pg = pgo.loop_graph(n_kf=60, seed=5, cov_window=5, extra_loops=3)
    lds = solver.pgo_optimize(pg)
    monkeypatch.setenv("PLBA_SOLVE_LDS_N", "0")
    out = solver.pgo_optimize(pg)
    np.testing.assert_array_equal(out["v_T"], lds["v_T"])
    _compare(out, oa.pgo_optimize(pg))


def test_pgo_id_order_full_envelope_matches_oracle(solver, monkeypatch):
    """PLBA_NO_RCM=1: the Hessian in g2o's id order with the loop edges' full envelope (the dense
    factorisation over every tile), same oracle agreement as the RCM-ordered default."""
    monkeypatch.setenv("PLBA_NO_RCM", "1")
    pg = pgo.loop_graph(n_kf=150, seed=9, cov_window=4, extra_loops=6)
    ref = oa.pgo_optimize(pg)
    out = solver.pgo_optimize(pg)
    _compare(out, ref)
