"""Known-answer tests of the pose-graph oracle (oracle/refpgo.cpp) — the loop-closure g2o
optimisation of MapHandler::loopClosureOptimization{EssGraph,CovGraph}G2O
(src/mapHandler.cpp:5070-5531). Parity against g2o itself is unpinned; these
pin the restatement: Eigen's matrix -> quaternion against scipy, the MQT maps, the EdgeSE3
Jacobians against central differences, EstimatePropagator's initial guess on graphs with a
known answer, and convergence on consistent loops."""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import oracle_api as oa
from plba import pgo
from plba.pgo import inv4, to4, to12


def _rand_T(rng, max_angle=np.pi):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    M = np.eye(4)
    M[:3, :3] = pgo.rot(ax * rng.uniform(0, max_angle))
    M[:3, 3] = rng.normal(0, 2, 3)
    return M


def test_quaternion_from_matrix_matches_scipy():
    rng = np.random.default_rng(1)
    mats = [pgo.rot(rng.normal(size=3)) for _ in range(50)]
    mats += [pgo.rot([np.pi - 1e-3, 0, 0]), pgo.rot([0, np.pi - 1e-4, 0]), pgo.rot([0, 0, 3.1]),
             pgo.rot(np.array([1.0, 1.0, 1.0]) / np.sqrt(3) * 3.0)]  # trace <= 0 branches
    for R in mats:
        q = oa.quat_from_R(R)
        ref = Rotation.from_matrix(R).as_quat()  # x y z w
        s = 1.0 if np.dot(q, ref) >= 0 else -1.0
        np.testing.assert_allclose(q, s * ref, atol=1e-12)


def test_mqt_round_trip_and_oplus():
    rng = np.random.default_rng(2)
    for _ in range(30):
        T = _rand_T(rng)
        v = oa.to_mqt(to12(T))
        assert np.linalg.norm(v[3:]) <= 1.0 + 1e-15
        np.testing.assert_allclose(oa.from_mqt(v), to12(T), atol=1e-12)
    # VertexSE3::oplusImpl: X <- X·fromVectorMQT(δ)
    X = _rand_T(rng)
    d = np.array([0.1, -0.2, 0.05, 0.01, -0.02, 0.03])
    np.testing.assert_allclose(oa.se3_oplus(to12(X), d), to12(X @ to4(oa.from_mqt(d))), atol=1e-13)
    # |v| > 1 -> identity rotation (fromCompactQuaternion)
    np.testing.assert_allclose(to4(oa.from_mqt([1, 2, 3, 0.9, 0.9, 0]))[:3, :3], np.eye(3))


def test_edge_error_zero_at_measurement():
    rng = np.random.default_rng(3)
    Xi, Xj = _rand_T(rng), _rand_T(rng)
    e = oa.se3_edge_error(to12(inv4(Xi) @ Xj), to12(Xi), to12(Xj))
    np.testing.assert_allclose(e, 0.0, atol=1e-12)


@pytest.mark.parametrize("seed", range(6))
def test_edge_jacobians_central_differences(seed):
    rng = np.random.default_rng(100 + seed)
    Xi, Xj = _rand_T(rng), _rand_T(rng)
    # measurement near the current relative pose, with a sizeable error rotation (< 150°)
    D = np.eye(4)
    D[:3, :3] = pgo.rot(rng.normal(0, 0.8, 3))
    D[:3, 3] = rng.normal(0, 0.5, 3)
    Z = inv4(Xi) @ Xj @ D
    Ji, Jj = oa.se3_edge_jacobians(to12(Z), to12(Xi), to12(Xj))
    h = 1e-6
    for k in range(6):
        d = np.zeros(6)
        d[k] = h
        for J, which in ((Ji, 0), (Jj, 1)):
            Xp = [to12(Xi), to12(Xj)]
            Xm = [to12(Xi), to12(Xj)]
            Xp[which] = oa.se3_oplus(Xp[which], d)
            Xm[which] = oa.se3_oplus(Xm[which], -d)
            num = (oa.se3_edge_error(to12(Z), *Xp) - oa.se3_edge_error(to12(Z), *Xm)) / (2 * h)
            np.testing.assert_allclose(J[:, k], num, atol=2e-8, rtol=1e-6)


def _chain(n=8, seed=5, perturb=True):
    rng = np.random.default_rng(seed)
    Tt = [_rand_T(rng, 0.5)]
    for _ in range(n - 1):
        D = np.eye(4)
        D[:3, :3] = pgo.rot(rng.normal(0, 0.2, 3))
        D[:3, 3] = rng.normal(0, 0.5, 3)
        Tt.append(Tt[-1] @ D)
    v_T = np.array([to12(M) for M in Tt])
    if perturb:
        v_T[1:] += rng.normal(0, 0.05, (n - 1, 12))
    ev = np.array([(i, i + 1) for i in range(n - 1)], np.int32)
    ez = np.array([to12(inv4(Tt[i]) @ Tt[i + 1]) for i in range(n - 1)])
    fixed = np.zeros(n, np.uint8)
    fixed[0] = 1
    return pgo.PoseGraph(np.arange(n, dtype=np.int32), v_T, fixed, ev, ez, None, np.array([to12(M) for M in Tt]))


def test_initial_guess_propagates_the_chain():
    pg = _chain()
    out = oa.pgo_initial_guess(pg)
    np.testing.assert_allclose(out, pg.T_true, atol=1e-10)


def test_initial_guess_from_two_roots_takes_the_nearest():
    """Roots 0 and n-1 fixed; reversed edges (vertex(0) = the later KF) use Z⁻¹. Each free
    vertex is initialised from the root fewer hops away (ties: the root popped first, vertex 0)."""
    pg = _chain(n=9, seed=6)
    n = 9
    pg.v_fixed[n - 1] = 1
    last = to4(pg.T_true[n - 1]).copy()
    last[:3, 3] += [0.3, 0, 0]  # a different (loop-corrected) pose for the far root
    pg.v_T[n - 1] = to12(last)
    pg.e_v[-1] = pg.e_v[-1][::-1]  # edge (n-1 -> n-2): measurement must be inverted
    pg.e_Z[-1] = to12(inv4(to4(pg.e_Z[-1])))
    out = oa.pgo_initial_guess(pg)
    for k in range(1, 4 + 1):   # hops from 0 <= hops from n-1 (tie at k = 4 -> root 0, popped first)
        np.testing.assert_allclose(out[k], pg.T_true[k], atol=1e-10)
    for k in range(5, n - 1):
        # from the far root: T_k = T_{n-1} · (T_true_k⁻¹ T_true_{n-1})⁻¹
        exp = last @ inv4(inv4(to4(pg.T_true[k])) @ to4(pg.T_true[n - 1]))
        np.testing.assert_allclose(out[k], to12(exp), atol=1e-10)


def test_consistent_loop_converges_to_truth():
    """All measurements exact, estimates perturbed: LM drives χ² to ~0 and the poses to truth."""
    pg = pgo.loop_graph(n_kf=20, seed=3, rot_noise_deg=0.0, trans_noise=0.0, ess=False)
    pg.e_Z[:] = [to12(inv4(to4(pg.T_true[i])) @ to4(pg.T_true[j])) for i, j in pg.e_v]
    rng = np.random.default_rng(4)
    pg.v_T[1:] = [to12(to4(T) @ to4(oa.from_mqt(rng.normal(0, 0.02, 6)))) for T in pg.T_true[1:]]
    r = oa.pgo_optimize(pg, oa.capi.pgo_params(initial_guess=0))
    assert r["chi2_initial"] > 1e-4 and r["chi2_final"] < 1e-16, r
    np.testing.assert_allclose(r["v_T"], pg.T_true, atol=1e-8)


@pytest.mark.parametrize("ess", [True, False])
def test_drift_loop_reduces_error(ess):
    pg = pgo.loop_graph(n_kf=40, seed=11, ess=ess)
    r = oa.pgo_optimize(pg)
    tr = r["trace"]
    assert r["n_free"] == (38 if ess else 39), r["n_free"]  # vertex 0 = loop_i, and loop_j fixed
    assert r["chi2_final"] < 0.2 * r["chi2_initial"], (r["chi2_initial"], r["chi2_final"])
    assert len(tr) == r["iterations"] and np.all(np.diff(tr["chi2_end"]) <= 0)
    assert tr["result"][-1] == 1 or r["iterations"] == 100
    # the fixed vertices keep their estimates
    fx = pg.v_fixed.astype(bool)
    np.testing.assert_array_equal(r["v_T"][fx], pg.v_T[fx])
