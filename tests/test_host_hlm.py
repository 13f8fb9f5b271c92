"""C++ host mirror of MapHandler::localBundleAdjustmentForPluker (src/mapHandler.cpp:1505-1615) and
the write-back of levMarquardtOptimizationLBAForPluker (:2160-2330), SURVEY.md §8f row 1.

CPU tests drive it through the solver hook with the CPU oracle (oracle/refhlm.cpp) and check
the window it hands the optimiser and the map state it leaves against a test-side model of the
reference; the GPU test runs the real plba_hlm_lba solve and compares with that model."""
import numpy as np
import pytest

import oracle_api as oa
from plba import capi, synth
from plba import geometry as geo
from plba.hlm import HlmWindow
from plba.slam_map import HostMap, make_map

from test_host_mirror import graph_from_struct


def _arr(p, n):
    return np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0)


def capture_hook(record, solve=True, params=None):
    """Solver hook: records the window; solves it with the oracle (or fails, solve=False)."""
    def fn(gs, ss, ps, rs):
        g = graph_from_struct(gs)
        win = HlmWindow(g, _arr(ss.kf_x, 6 * g.n_kf).reshape(-1, 6), _arr(ss.ln_pluker, 6 * g.n_ln).reshape(-1, 6))
        record["win"] = win
        record["params"] = (ps.lambda0, ps.lambda_k, ps.homog_th, ps.min_error, ps.min_error_change, ps.max_iters,
                            ps.err_per_obs)
        if not solve:
            return -7
        out = oa.hlm_lba(win, ps)
        record["out"] = out
        for name, a in (("kf_x", out["kf_x"]), ("kf_Tcw", out["kf_Tcw"]), ("pt_xyz", out["pt_xyz"]),
                        ("ln_orth", out["ln_orth"])):
            a = np.ascontiguousarray(a, np.float64).reshape(-1)
            if a.size:
                np.ctypeslib.as_array(getattr(rs, name), shape=(a.size,))[:] = a
        rs.linearizations, rs.solves, rs.accepted = out["linearizations"], out["solves"], out["accepted"]
        rs.err, rs.lambda_, rs.dx_norm = out["err"], out["lam"], out["dx_norm"]
        return 0
    return fn


def expected_window(m, xs):
    """The reference's lists (:1511-1607) for the SlamMap m (x_kf_w from the host, xs)."""
    kf_list = [k for k in m.keyframes if k is not None and k.local and k.kf_idx != 0]
    pts = [p for p in m.points if p is not None and p.local]
    lns = [l for l in m.lines if l is not None and l.local]
    return kf_list, pts, lns


def check_window(win, m, xs):
    kf_list, pts, lns = expected_window(m, xs)
    g = win.graph
    free = g.kf_fixed == 0
    assert list(g.kf_id[free]) == [k.kf_idx for k in kf_list]
    observers = sorted({o for lm in pts + lns for o in lm.kf_obs_list} - {k.kf_idx for k in kf_list})
    assert sorted(g.kf_id[~free]) == observers
    for i, kid in enumerate(g.kf_id):
        T = m.keyframes[kid].T_kf_w
        np.testing.assert_allclose(g.kf_Tcw[i], geo.inverse_se3(T)[:3, :], rtol=0, atol=1e-14)
        np.testing.assert_array_equal(win.kf_x[i], xs[kid])
    np.testing.assert_array_equal(g.pt_xyz, np.array([p.pos for p in pts]).reshape(-1, 3))
    np.testing.assert_array_equal(win.ln_pluker, np.array([l.pos for l in lns]).reshape(-1, 6))
    np.testing.assert_allclose(g.ln_orth, geo.pluker_to_orth(np.array([l.pos for l in lns]).reshape(-1, 6)),
                               rtol=0, atol=1e-12)
    assert g.n_ept == sum(len(p.kf_obs_list) for p in pts)
    assert g.n_eln == sum(len(l.kf_obs_list) for l in lns)


def check_writeback(before, after, win, out, tol=0.0):
    """:2165-2198 applied to the optimiser's output `out`."""
    kf_list, pts, lns = expected_window(before, None)
    for i, k in enumerate(kf_list):
        T = geo.expmap_se3(out["kf_x"][i])
        np.testing.assert_allclose(after.keyframes[k.kf_idx].T_kf_w, T, rtol=0, atol=max(tol, 1e-14))
    free_ids = {k.kf_idx for k in kf_list}
    for k in before.keyframes:
        if k is not None and k.kf_idx not in free_ids:
            np.testing.assert_array_equal(after.keyframes[k.kf_idx].T_kf_w, k.T_kf_w)
    for i, p in enumerate(pts):
        q = after.points[p.idx]
        np.testing.assert_allclose(q.pos, out["pt_xyz"][i], rtol=0, atol=max(tol, 0.0))
        moved = np.linalg.norm(out["pt_xyz"][i] - p.pos) > 0.01
        assert q.inlier == (p.inlier and not moved)
    for i, l in enumerate(lns):
        q = after.lines[l.idx]
        orth0 = win.graph.ln_orth[i]
        dx = out["ln_orth"][i] - orth0
        np.testing.assert_allclose(q.pos, geo.orth_to_pluker(dx), rtol=0, atol=max(tol, 1e-15))
        assert q.inlier == (l.inlier and not np.linalg.norm(dx) > 0.01)
    for lms_b, lms_a in ((before.points, after.points), (before.lines, after.lines)):
        for b, a in zip(lms_b, lms_a):
            if b is not None and not b.local:
                np.testing.assert_array_equal(a.pos, b.pos)


@pytest.mark.parametrize("cfg,params", [("C1", {}), ("C1L", {"lambda0": 1e-24, "err_per_obs": 1})])
def test_host_hlm_window_and_writeback_with_oracle_hook(cfg, params):
    m = make_map(synth.generate(cfg))
    hmap = HostMap(m)
    xs = {k.kf_idx: hmap.keyframe_x(k.kf_idx) for k in m.keyframes if k is not None}
    for kid, x in xs.items():   # x_kf_w = logmap_se3(T_kf_w) at insertion
        np.testing.assert_allclose(x, geo.logmap_se3(m.keyframes[kid].T_kf_w), rtol=0, atol=1e-12)
    p = capi.hlm_params(**params)
    hmap.set_hlm_params(p)
    rec = {}
    hmap.set_hlm_solver(capture_hook(rec))
    st = hmap.local_ba_hlm()
    assert st["ret"] == 0
    assert rec["params"] == (p.lambda0, p.lambda_k, p.homog_th, p.min_error, p.min_error_change, p.max_iters,
                             p.err_per_obs)
    check_window(rec["win"], m, xs)
    assert st["linearizations"] == rec["out"]["linearizations"] and st["accepted"] == rec["out"]["accepted"]
    after = hmap.read(m)
    check_writeback(m, after, rec["win"], rec["out"])
    for kid, x in xs.items():   # the reference never writes x_kf_w back
        np.testing.assert_array_equal(hmap.keyframe_x(kid), x)
    hmap.close()


def test_host_hlm_vo_inserting_kf_writes_nothing():
    m = make_map(synth.generate("C1L"))
    hmap = HostMap(m)
    hmap.set_hlm_params(None, vo_inserting_kf=True)
    rec = {}
    hmap.set_hlm_solver(capture_hook(rec))
    st = hmap.local_ba_hlm()
    assert st["ret"] == -1 and "out" in rec
    after = hmap.read(m)
    for b, a in zip(m.points, after.points):
        if b is not None:
            np.testing.assert_array_equal(a.pos, b.pos)
    for b, a in zip(m.keyframes, after.keyframes):
        np.testing.assert_array_equal(a.T_kf_w, b.T_kf_w)


def test_host_hlm_no_observations_returns_minus_one():
    m = make_map(synth.generate("C1"))
    for lm in m.points + m.lines:
        if lm is not None:
            lm.local = False
    hmap = HostMap(m)
    rec = {}
    hmap.set_hlm_solver(capture_hook(rec))
    st = hmap.local_ba_hlm()
    assert st["ret"] == -1 and "win" not in rec


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,params", [("C1", {}), ("C2", {"lambda0": 1e-24, "err_per_obs": 1})])
def test_gpu_host_hlm_matches_model_with_oracle(cfg, params):
    m = make_map(synth.generate(cfg))
    p = capi.hlm_params(**params)
    probe = HostMap(m)            # the window the host builds, captured (hook fails: no write-back)
    probe.set_hlm_params(p)
    rec = {}
    probe.set_hlm_solver(capture_hook(rec, solve=False))
    with pytest.raises(Exception):
        probe.local_ba_hlm()
    probe.close()
    ref = oa.hlm_lba(rec["win"], p)
    hmap = HostMap(m)             # the real thing: plba_hlm_lba on the GPU
    hmap.set_hlm_params(p)
    st = hmap.local_ba_hlm()
    assert st["ret"] == 0 and st["linearizations"] == ref["linearizations"] and st["accepted"] == ref["accepted"]
    after = hmap.read(m)
    scale = max(np.abs(ref["pt_xyz"] - rec["win"].graph.pt_xyz).max(), 1e-12)
    check_writeback(m, after, rec["win"], ref, tol=1e-4 * scale + 1e-12)
    hmap.close()
