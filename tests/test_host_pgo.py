"""Host mirror of MapHandler::loopClosureOptimizationEssGraphG2O / CovGraphG2O
(src/mapHandler.cpp:5070-5299 / :5301-5531): the graph it builds for g2o, the write-back of the
optimised poses and the landmark / later-KF corrections. CPU tests drive the mirror through the
pose-graph oracle (a solver hook); the GPU test runs plba_pgo_optimize and compares with that
model. Parity against the reference itself is unpinned (no fixtures)."""
import ctypes as C

import numpy as np
import pytest

import oracle_api as oa
from plba import capi, pgo
from plba import geometry as geo
from plba.pgo import inv4, to4
from plba.slam_map import HostMap


def _hostmap(n_loop=24, n_after=3, seed=3, ess=True):
    m, lc_idxs, lc_list, lc_pose, line3d = pgo.loop_map(n_loop=n_loop, n_after=n_after, seed=seed)
    h = HostMap(m)
    h.set_loop_closure(lc_idxs, lc_list, lc_pose)
    for i, L in enumerate(line3d):
        h.set_line_geometry(i, L, L[:3] * 0.5)
    return m, h, lc_pose, line3d


def _oracle_hook(store):
    def fn(g, p, r):
        nv, ne = g.n_v, g.n_e
        store["v_T"] = np.ctypeslib.as_array(g.v_T, (nv * 12,)).reshape(nv, 12).copy()
        store["v_fixed"] = np.ctypeslib.as_array(g.v_fixed, (nv,)).copy()
        store["v_id"] = np.ctypeslib.as_array(g.v_id, (nv,)).copy()
        store["e_v"] = np.ctypeslib.as_array(g.e_v, (ne * 2,)).reshape(ne, 2).copy()
        store["e_Z"] = np.ctypeslib.as_array(g.e_Z, (ne * 12,)).reshape(ne, 12).copy()
        store["max_iters"] = p.max_iters
        rc = oa._pgo_lib().refpgo_optimize(C.byref(g), C.byref(p), C.byref(r))
        store["out"] = np.ctypeslib.as_array(r.v_T, (nv * 12,)).reshape(nv, 12).copy()
        return rc
    return fn


def _kf(h, k):
    T = np.zeros(16)
    h.L.plslam_get_keyframe(h.h, k, T.ctypes.data_as(C.POINTER(C.c_double)), None, None, 0, None, 0)
    return T.reshape(4, 4)


def _pt(h, i):
    xyz = np.zeros(3)
    h.L.plslam_get_point(h.h, i, xyz.ctypes.data_as(C.POINTER(C.c_double)), None, None, None, None, None, None,
                         None, 0, None, None)
    return xyz


@pytest.mark.parametrize("ess", [True, False])
def test_loop_closure_graph_and_write_back(ess):
    m, h, lc_pose, line3d = _hostmap()
    n_loop, n_kf = 24, 27
    T0 = [_kf(h, k) for k in range(n_kf)]
    P0 = [_pt(h, i) for i in range(len(m.points))]
    store = {}
    h.set_pgo_solver(_oracle_hook(store))
    st = h.loop_closure(ess=ess)
    # ---- the graph (:5087-5179): KFs 0..n_loop-1, vertex 0 (and, EssGraph, both loop KFs) fixed
    assert st["kf_prev_idx"] == 0 and st["kf_curr_idx"] == n_loop - 1
    np.testing.assert_array_equal(store["v_id"], np.arange(n_loop))
    exp_fixed = np.zeros(n_loop, np.uint8)
    exp_fixed[0] = 1
    if ess:
        exp_fixed[n_loop - 1] = 1
    np.testing.assert_array_equal(store["v_fixed"], exp_fixed)
    assert store["max_iters"] == 100
    # covisible (>= 150 shared, |i-j| <= 2) and consecutive pairs + the loop edge
    pairs = [(i, j) for i in range(n_loop) for j in range(i + 1, n_loop) if j - i <= 2]
    assert st["n_edges"] == len(pairs) and st["n_loop_edges"] == 1
    np.testing.assert_array_equal(store["e_v"][:-1], np.array(pairs))
    for (i, j), Z in zip(pairs, store["e_Z"]):
        np.testing.assert_allclose(to4(Z), inv4(T0[i]) @ T0[j], atol=1e-9)
    np.testing.assert_allclose(to4(store["e_Z"][-1]), geo.expmap_se3(lc_pose[0]), atol=1e-9)
    # vertex estimates: SE3Quat::exp(reverse_se3(x_kf_w)) = the map pose; the loop KF, EssGraph
    # and CovGraph alike, at expmap(lc_pose)·T_kf_w(0)
    for k in range(n_loop - 1):
        np.testing.assert_allclose(to4(store["v_T"][k]), T0[k], atol=1e-9)
    np.testing.assert_allclose(to4(store["v_T"][n_loop - 1]), geo.expmap_se3(lc_pose[0]) @ T0[0], atol=1e-9)
    # ---- write-back (:5187-5240): optimised poses, landmarks moved with their KF
    corr = None
    for k in range(n_loop):
        Tn = _kf(h, k)
        np.testing.assert_allclose(Tn, to4(store["out"][k]), atol=1e-9)
        corr = Tn @ inv4(T0[k])
        for i in m.map_points_kf_idx[k]:
            np.testing.assert_allclose(_pt(h, i), corr[:3, :3] @ P0[i] + corr[:3, 3], atol=1e-9)
        for i in m.map_lines_kf_idx[k]:
            L, d = h.line_geometry(i)
            np.testing.assert_allclose(L[:3], corr[:3, :3] @ line3d[i][:3] + corr[:3, 3], atol=1e-9)
            np.testing.assert_allclose(d, corr[:3, :3] @ (0.5 * line3d[i][:3]) + corr[:3, 3], atol=1e-9)
    # ---- later KFs (:5243-5287) take the last KF's correction
    for k in range(n_loop, n_kf):
        np.testing.assert_allclose(_kf(h, k), corr @ T0[k], atol=1e-9)
        np.testing.assert_allclose(h.keyframe_x(k), geo.logmap_se3(corr @ T0[k]), atol=1e-9)
    np.testing.assert_array_equal(h.lc_idx_list()[:, 2], 0)
    assert st["chi2_final"] < st["chi2_initial"]
    h.close()


def test_loop_closure_rejects_missing_loop_pose():
    m, lc_idxs, lc_list, lc_pose, _ = pgo.loop_map(n_loop=10, n_after=0, seed=5)
    h = HostMap(m)
    h.set_loop_closure(lc_idxs, lc_list, np.zeros((0, 6)))
    h.set_pgo_solver(_oracle_hook({}))
    with pytest.raises(Exception):
        h.loop_closure(ess=True)
    h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ess", [True, False])
def test_gpu_loop_closure_matches_model_with_oracle(ess):
    m, ref, _, _ = _hostmap(seed=7)
    ref.set_pgo_solver(_oracle_hook({}))
    st_ref = ref.loop_closure(ess=ess)
    _, gpu, _, _ = _hostmap(seed=7)
    st = gpu.loop_closure(ess=ess)   # plba_pgo_optimize on the GPU
    assert st["n_vertices"] == st_ref["n_vertices"] and st["n_edges"] == st_ref["n_edges"]
    assert abs(st["chi2_final"] - st_ref["chi2_final"]) <= 1e-8 * st_ref["chi2_final"] + 1e-14
    for k in range(27):
        np.testing.assert_allclose(_kf(gpu, k), _kf(ref, k), atol=1e-7)
    for i in range(len(m.points)):
        np.testing.assert_allclose(_pt(gpu, i), _pt(ref, i), atol=1e-7)
    ref.close()
    gpu.close()
