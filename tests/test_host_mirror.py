"""C++ host mirror of MapHandler::localBundleAdjustmentForPlukerWithG2O (gather, marshalling,
outlier bookkeeping, write-back; src/mapHandler.cpp:5851-6323) against the test-side
restatement in host_model.py. CPU tests drive it with a deterministic stub solver; the GPU
test runs the real MI355X solve and compares with the model driven by the CPU oracle."""
import ctypes as C

import numpy as np
import pytest

import host_model as hm
from plba import capi, synth
from plba import geometry as geo
from plba.slam_map import HOST_EXPORTED, HostMap, load_host, make_map


def _frac(x):
    return x - np.floor(x)


def stub_solve(g: synth.Graph) -> dict:
    """Deterministic fake solve: moves the estimates a little and produces a spread of χ²,
    depth flags and levels so every bookkeeping branch is taken."""
    Tcw = g.kf_Tcw.reshape(-1, 3, 4).copy()
    free = g.kf_fixed == 0
    Tcw[free, :, 3] += 1e-3 * (1 + np.arange(free.sum()))[:, None]
    h_p = _frac(np.sin(g.ept_obs[:, 0] * 12.9898 + g.ept_obs[:, 1] * 78.233) * 43758.5453)
    h_l = _frac(np.sin(g.eln_obs[:, 0] * 12.9898 + g.eln_obs[:, 3] * 78.233) * 43758.5453)
    return dict(
        kf_Tcw=Tcw.reshape(-1, 12),
        pt_xyz=g.pt_xyz + 0.01 * np.sin(np.arange(g.n_pt))[:, None],
        ln_orth=g.ln_orth + 1e-3,
        ept_chi2=20.0 * h_p ** 4,
        ept_depth_ok=(_frac(h_p * 97.0) > 0.05).astype(np.uint8),
        ept_level=(h_p > 0.8).astype(np.uint8),
        eln_chi2=20.0 * h_l ** 4,
        eln_level=(h_l > 0.8).astype(np.uint8),
        iters=np.array([5, 10], np.int32),
        chi2=np.array([123.0, 45.0]),
    )


def graph_from_struct(s: capi.PlbaGraph) -> synth.Graph:
    def arr(p, n, w=1, dt=np.float64):
        if n * w == 0:
            return np.zeros((0, w) if w > 1 else 0, dt)
        a = np.ctypeslib.as_array(p, shape=(n * w,)).astype(dt).copy()
        return a.reshape(n, w) if w > 1 else a
    return synth.Graph(
        fx=s.fx, fy=s.fy, cx=s.cx, cy=s.cy,
        kf_Tcw=arr(s.kf_Tcw, s.n_kf, 12).reshape(-1, 3, 4), kf_fixed=arr(s.kf_fixed, s.n_kf, 1, np.uint8),
        kf_id=arr(s.kf_id, s.n_kf, 1, np.int32),
        pt_xyz=arr(s.pt_xyz, s.n_pt, 3).reshape(-1, 3), pt_id=arr(s.pt_id, s.n_pt, 1, np.int32),
        ln_orth=arr(s.ln_orth, s.n_ln, 4).reshape(-1, 4), ln_id=arr(s.ln_id, s.n_ln, 1, np.int32),
        ept_lm=arr(s.ept_lm, s.n_ept, 1, np.int32), ept_kf=arr(s.ept_kf, s.n_ept, 1, np.int32),
        ept_obs=arr(s.ept_obs, s.n_ept, 2).reshape(-1, 2), ept_info=arr(s.ept_info, s.n_ept),
        eln_lm=arr(s.eln_lm, s.n_eln, 1, np.int32), eln_kf=arr(s.eln_kf, s.n_eln, 1, np.int32),
        eln_obs=arr(s.eln_obs, s.n_eln, 4).reshape(-1, 4), eln_info=arr(s.eln_info, s.n_eln),
        huber_pt=s.huber_pt, huber_ln=s.huber_ln)


def write_result(r: capi.PlbaResult, res: dict, g: synth.Graph):
    def put(p, a, dt=np.float64):
        a = np.ascontiguousarray(a, dt).reshape(-1)
        if a.size and p:
            np.ctypeslib.as_array(p, shape=(a.size,))[:] = a
    put(r.kf_Tcw, res["kf_Tcw"])
    put(r.pt_xyz, res["pt_xyz"])
    put(r.ln_orth, res["ln_orth"])
    put(r.ept_chi2, res["ept_chi2"])
    put(r.ept_depth_ok, res["ept_depth_ok"], np.uint8)
    put(r.ept_level, res["ept_level"], np.uint8)
    put(r.eln_chi2, res["eln_chi2"])
    put(r.eln_level, res["eln_level"], np.uint8)
    r.iters[0], r.iters[1] = int(res["iters"][0]), int(res["iters"][1])
    r.chi2[0], r.chi2[1] = float(res["chi2"][0]), float(res["chi2"][1])


def host_with(m, solve):
    hmap = HostMap(m)
    seen = {}

    def cb(gs, rs):
        g = graph_from_struct(gs)
        seen["graph"] = g
        write_result(rs, solve(g), g)
        return 0
    hmap.set_solver(cb)
    return hmap, seen


@pytest.fixture(scope="module")
def window():
    return synth.generate("C1L", fixed_frac=0.3)


def test_host_library_exports_every_header_symbol():
    L = load_host()
    for name in HOST_EXPORTED:
        assert hasattr(L, name), name
    import re
    hdr = open(__file__.replace("tests/test_host_mirror.py", "include/plslam_host.h")).read()
    declared = set(re.findall(r"\b(plslam_[a-z0-9_]+)\s*\(", hdr))
    assert declared <= set(HOST_EXPORTED), declared - set(HOST_EXPORTED)


def test_pluker_orth_conversions_match_reference_formulas():
    L = load_host()
    rng = np.random.default_rng(0)
    for _ in range(50):
        o = rng.uniform([-3, -1.5, -3, -1.5], [3, 1.5, 3, 1.5])
        Lp = np.zeros(6)
        L.plslam_orth_to_pluker(o.ctypes.data_as(C.POINTER(C.c_double)), Lp.ctypes.data_as(C.POINTER(C.c_double)))
        np.testing.assert_allclose(Lp, geo.orth_to_pluker(o), rtol=0, atol=1e-15)
        o2 = np.zeros(4)
        L.plslam_pluker_to_orth(Lp.ctypes.data_as(C.POINTER(C.c_double)), o2.ctypes.data_as(C.POINTER(C.c_double)))
        np.testing.assert_allclose(o2, geo.pluker_to_orth(Lp), rtol=0, atol=1e-13)


def test_marshalled_window_matches_reference_gather(window):
    m = make_map(window, seed=1)
    hmap, seen = host_with(m, stub_solve)
    hmap.local_ba()
    g_model, win = hm.gather(m.copy())
    g = seen["graph"]
    for k in ("kf_fixed", "kf_id", "pt_id", "ln_id", "ept_lm", "ept_kf", "eln_lm", "eln_kf"):
        np.testing.assert_array_equal(getattr(g, k), getattr(g_model, k), err_msg=k)
    for k in ("ept_obs", "ept_info", "eln_obs", "eln_info", "pt_xyz"):
        np.testing.assert_array_equal(getattr(g, k), getattr(g_model, k), err_msg=k)
    np.testing.assert_allclose(g.kf_Tcw, g_model.kf_Tcw, rtol=0, atol=1e-13)
    np.testing.assert_allclose(g.ln_orth, g_model.ln_orth, rtol=0, atol=1e-13)
    assert g.huber_pt == g_model.huber_pt == float(np.float32(np.sqrt(5.991)))
    # the window: free KFs (KF 0 among them, fixed by id) then the pulled-in observers
    assert g.kf_fixed[0] == 1 and g.kf_id[0] == 0
    assert win["n_fixed"] > 0
    # info is the float-rounded 1/σ² (const float& invSigma2, src/mapHandler.cpp:6009)
    assert np.any(g.ept_info != 1.0) and np.all(g.ept_info == g.ept_info.astype(np.float32))


@pytest.mark.parametrize("cfg,seed", [("C1L", 1), ("C1", 2)])
def test_bookkeeping_matches_model(cfg, seed):
    g = synth.generate(cfg, fixed_frac=0.3)
    m = make_map(g, seed=seed)
    hmap, _ = host_with(m, stub_solve)
    st = hmap.local_ba()
    got = hmap.read(m)
    want = m.copy()
    st_model = hm.lba(want, stub_solve)
    for k, v in st_model.items():
        assert st[k] == v, (k, st[k], v)
    assert st["actually_bad_point_obs"] > 0 and st["bad_point_obs"] > st["actually_bad_point_obs"] or cfg == "C1"
    hm.compare_maps(got, want, pose_tol=1e-12, lm_tol=1e-12)


def test_second_lba_on_updated_map(window):
    m = make_map(window, seed=4)
    hmap, _ = host_with(m, stub_solve)
    want = m.copy()
    for _ in range(2):
        st = hmap.local_ba()
        st_model = hm.lba(want, stub_solve)
        assert st["bad_point_obs"] == st_model["bad_point_obs"]
    hm.compare_maps(hmap.read(m), want, pose_tol=1e-12, lm_tol=1e-12)


def test_inconsistent_map_is_refused_and_untouched(window):
    m = make_map(window, seed=5)
    bad = m.copy()
    p = next(p for p in bad.points if p is not None and p.local)
    p.kf_obs_list[0] = len(bad.keyframes) + 7       # no such keyframe (reference: exit(0))
    hmap, seen = host_with(bad, stub_solve)
    with pytest.raises(Exception, match="PLBA_E_INVALID"):
        hmap.local_ba()
    assert "graph" not in seen
    after = hmap.read(bad)
    assert [k.local for k in after.keyframes] == [k.local for k in bad.keyframes]


def test_inconsistent_line_observation_is_refused_and_untouched(window):
    """The single-pass gather checks line observations after every point's (the reference's
    order, src/mapHandler.cpp:5891-5911) and leaves the local flags untouched."""
    m = make_map(window, seed=7)
    bad = m.copy()
    ln = [l for l in bad.lines if l is not None and l.local]
    if not ln:
        pytest.skip("window without lines")
    ln[-1].kf_obs_list[-1] = -3
    hmap, seen = host_with(bad, stub_solve)
    with pytest.raises(Exception, match="MapLine obs"):
        hmap.local_ba()
    assert "graph" not in seen
    after = hmap.read(bad)
    assert [k.local for k in after.keyframes] == [k.local for k in bad.keyframes]


def test_solver_failure_leaves_map_untouched(window):
    m = make_map(window, seed=6)
    hmap = HostMap(m)
    hmap.set_solver(lambda gs, rs: -2)
    with pytest.raises(Exception, match="PLBA_E_DEVICE"):
        hmap.local_ba()
    after = hmap.read(m)
    for a, b in zip(after.points, m.points):
        if a is not None:
            assert np.array_equal(a.pos, b.pos) and a.kf_obs_list == b.kf_obs_list


def test_default_solver_fails_loudly_without_gpu(window):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    hmap = HostMap(make_map(window, seed=7))
    with pytest.raises(Exception, match="plba_create|PLBA_E"):
        hmap.local_ba()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C1L", "C2"])
def test_gpu_host_path_matches_model_with_oracle(cfg):
    import oracle_api as oa
    g = synth.generate(cfg, fixed_frac=0.2)
    m = make_map(g, seed=11)
    hmap = HostMap(m)
    st = hmap.local_ba()
    got = hmap.read(m)
    want = m.copy()
    st_model = hm.lba(want, lambda gg: oa.lba_plucker(gg))
    for k in ("n_free_kf", "n_fixed_kf", "n_ept", "n_eln", "bad_line_stage1", "bad_point_obs",
              "actually_bad_point_obs", "bad_line_obs", "actually_bad_line_obs", "iters"):
        assert st[k] == st_model[k], (k, st[k], st_model[k])
    hm.compare_maps(got, want, pose_tol=1e-4, lm_tol=1e-4)


# ----------------------------------------------------------------- the local-mapping step
# formLocalMap(kf) -> LBA -> removeBadMapLandmarksForPluker (src/mapHandler.cpp:1274-1279)
from plba.slam_map import SlamParams  # noqa: E402


def _step_params(m, kf_idx):
    # a covisibility threshold inside the range of the last full_graph row, so both branches
    # of the window test (:1117) are taken
    row = m.full_graph[-1, :-1].astype(np.int64)
    return SlamParams(min_lm_obs=4, min_lm_cov_graph=int(np.median(row)) + 1, min_kf_local_map=2)


def _aged(m, extra=15):
    m.max_kf_idx = len(m.keyframes) - 1 + extra   # every landmark's base KF is > 10 KFs old
    return m


@pytest.mark.parametrize("cfg,seed", [("C1L", 21), ("C1", 22)])
def test_form_local_map_matches_model(cfg, seed):
    m = make_map(synth.generate(cfg, fixed_frac=0.3), seed=seed)
    for kf_idx in (len(m.keyframes) - 1, 3):
        p = _step_params(m, kf_idx)
        hmap = HostMap(m, params=p)
        hmap.form_local_map(kf_idx)
        want = m.copy()
        hm.form_local_map(want, kf_idx, p)
        got = hmap.read(m)
        assert [k.local for k in got.keyframes] == [k.local for k in want.keyframes]
        for a, b in zip(got.points + got.lines, want.points + want.lines):
            assert (a is None) == (b is None)
            if a is not None:
                assert a.local == b.local, a.idx
        assert any(k.local for k in want.keyframes) and not all(k.local for k in want.keyframes)


@pytest.mark.parametrize("cfg,seed", [("C1L", 23), ("C1", 24)])
def test_remove_bad_landmarks_matches_model(cfg, seed):
    m = _aged(make_map(synth.generate(cfg, fixed_frac=0.3), seed=seed))
    # some outliers and short tracks among the non-local landmarks
    rng = np.random.default_rng(seed)
    for lm in m.points + m.lines:
        if lm is not None and rng.random() < 0.3:
            lm.inlier = False
        if lm is not None and rng.random() < 0.4:
            lm.local = False
    p = SlamParams(min_lm_obs=4)
    hmap = HostMap(m, params=p)
    npt, nln = hmap.remove_bad_landmarks()
    want = m.copy()
    rem = hm.remove_bad(want, p)
    assert [npt, nln] == rem and npt > 0 and (nln > 0 or cfg == "C1")
    hm.compare_maps(hmap.read(m), want, pose_tol=0, lm_tol=0)


def test_local_mapping_step_matches_model():
    m = _aged(make_map(synth.generate("C1L", fixed_frac=0.3), seed=25), extra=5)
    kf_seq = [len(m.keyframes) - 1, len(m.keyframes) - 3]
    p = _step_params(m, kf_seq[0])
    hmap, _ = host_with(m, stub_solve)
    hmap.L.plslam_set_params(hmap.h, p.min_lm_obs, p.min_lm_cov_graph, p.min_kf_local_map)
    want = m.copy()
    for kf_idx in kf_seq:
        st = hmap.local_mapping_step(kf_idx)
        st_model = hm.local_mapping_step(want, kf_idx, stub_solve, p)
        for k, v in st_model.items():
            assert st[k] == v, (k, st[k], v)
    hm.compare_maps(hmap.read(m), want, pose_tol=1e-12, lm_tol=1e-12)


def test_remove_bad_refuses_missing_kf_idx_key():
    m = _aged(make_map(synth.generate("C1L", fixed_frac=0.3), seed=26))
    for lm in m.lines:
        lm.local, lm.inlier = False, False
    del m.map_lines_kf_idx[m.lines[0].kf_obs_list[0]]   # .at() would throw in the reference
    hmap = HostMap(m)
    with pytest.raises(Exception, match="PLBA_E_STATE"):
        hmap.remove_bad_landmarks()
    got = hmap.read(m)
    assert all(a is not None for a in got.points + got.lines if a is not None) and \
        sum(a is None for a in got.lines) == 0


def test_form_local_map_refuses_missing_covisible_keyframe():
    m2 = make_map(synth.generate("C1L", fixed_frac=0.3), seed=27)
    m2.keyframes[2] = None   # a NULL slot the reference would dereference (:1120)
    for lm in m2.points + m2.lines:
        if lm is not None and 2 in lm.kf_obs_list:
            lm.local = False
    hmap2 = HostMap(m2, params=SlamParams(min_kf_local_map=100))   # every KF is in the window
    before = hmap2.read(m2)
    with pytest.raises(Exception, match="PLBA_E_INVALID"):
        hmap2.form_local_map(len(m2.keyframes) - 1)
    after = hmap2.read(m2)
    assert [k.local if k else None for k in after.keyframes] == [k.local if k else None for k in before.keyframes]


@pytest.mark.gpu
def test_gpu_local_mapping_step_matches_model_with_oracle():
    import oracle_api as oa
    m = _aged(make_map(synth.generate("C2", fixed_frac=0.2), seed=28), extra=5)
    kf = len(m.keyframes) - 1
    p = _step_params(m, kf)
    hmap = HostMap(m, params=p)
    st = hmap.local_mapping_step(kf)
    want = m.copy()
    st_model = hm.local_mapping_step(want, kf, lambda gg: oa.lba_plucker(gg), p)
    for k in ("n_free_kf", "n_fixed_kf", "n_ept", "n_eln", "bad_point_obs", "actually_bad_point_obs",
              "bad_line_obs", "actually_bad_line_obs", "iters", "points_removed", "lines_removed"):
        assert st[k] == st_model[k], (k, st[k], st_model[k])
    hm.compare_maps(hmap.read(m), want, pose_tol=1e-4, lm_tol=1e-4)


# ---- incremental window (round 6)
def _mapping_sequence(hmap, m, rng):
    """A few local-mapping steps with map edits in between: new observations through the C ABI,
    local flags set and cleared, and the LBA's own outlier pass / write-back / culling."""
    L, h = hmap.L, hmap.h
    seq = [len(m.keyframes) - 1, len(m.keyframes) - 3, len(m.keyframes) - 2]
    for step, kf_idx in enumerate(seq):
        yield f"step{step}:before"
        hmap.local_mapping_step(kf_idx)
        yield f"step{step}:after"
        # a new observation of a few live points and lines (addMapPointObservation / addMapLineObservation)
        live_pt = [i for i in range(hmap.n_pt) if hmap.exists(1, i)]
        for idx in rng.choice(live_pt, size=3, replace=False):
            o = np.array([100.0 + idx, 50.0 + step])
            d = np.array([0.0, 0.0, 1.0])
            desc = np.zeros(32, np.uint8)
            assert L.plslam_point_add_observation(h, int(idx), desc.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                  int(kf_idx), o.ctypes.data_as(C.POINTER(C.c_double)),
                                                  d.ctypes.data_as(C.POINTER(C.c_double)), 1.3) == 0
        live_ln = [i for i in range(hmap.n_ln) if hmap.exists(2, i)]
        if live_ln:
            idx = int(rng.choice(live_ln))
            o = np.array([10.0, 20.0, 300.0, 40.0 + step])
            desc = np.zeros(32, np.uint8)
            assert L.plslam_line_add_observation(h, idx, desc.ctypes.data_as(C.POINTER(C.c_uint8)), int(kf_idx),
                                                 o.ctypes.data_as(C.POINTER(C.c_double)), 0.7) == 0
        yield f"step{step}:observations"
        # local flags written through the ABI (the registry follows them)
        for idx in rng.choice(live_pt, size=4, replace=False):
            assert L.plslam_set_local(h, 1, int(idx), int(rng.random() < 0.5)) == 0
        yield f"step{step}:flags"


@pytest.mark.parametrize("cfg,seed", [("C1L", 31), ("C2", 32)])
def test_incremental_gather_equals_the_scan_gather(cfg, seed):
    """The registry + cached-run gather hands the solver exactly what the reference's map scan
    would, after every kind of map change the local-mapping loop makes."""
    m = _aged(make_map(synth.generate(cfg, fixed_frac=0.3), seed=seed, n_extra_pt=40), extra=5)
    hmap, _ = host_with(m, stub_solve)
    p = _step_params(m, len(m.keyframes) - 1)
    hmap.L.plslam_set_params(hmap.h, p.min_lm_obs, p.min_lm_cov_graph, p.min_kf_local_map)
    assert hmap.check_incremental_gather()
    for tag in _mapping_sequence(hmap, m, np.random.default_rng(seed)):
        assert hmap.check_incremental_gather(), (tag, getattr(hmap, "_why", ""))


def test_incremental_and_scan_modes_leave_the_same_map():
    """The same local-mapping sequence on two handlers, one gathering incrementally (default) and
    one scanning the map as the reference: identical marshalled windows, statistics and maps."""
    m = _aged(make_map(synth.generate("C1L", fixed_frac=0.3), seed=33, n_extra_pt=40), extra=5)
    p = _step_params(m, len(m.keyframes) - 1)
    runs = []
    for inc in (True, False):
        hmap, seen = host_with(m, stub_solve)
        hmap.set_incremental(inc)
        hmap.L.plslam_set_params(hmap.h, p.min_lm_obs, p.min_lm_cov_graph, p.min_kf_local_map)
        graphs, stats = [], []
        orig = hmap._cb

        for tag in _mapping_sequence(hmap, m, np.random.default_rng(33)):
            if tag.endswith(":after"):
                graphs.append(seen["graph"])
        st = hmap.local_ba()
        stats.append({k: v for k, v in st.items() if not k.endswith("_ms") and k != "dirty_landmarks"})
        graphs.append(seen["graph"])
        runs.append((graphs, stats, hmap.read(m), st["dirty_landmarks"]))
        assert orig is hmap._cb
    (ga, sa, ma, da), (gb, sb, mb, db) = runs
    assert sa == sb
    for a, b in zip(ga, gb):
        for f in ("kf_Tcw", "kf_fixed", "kf_id", "pt_xyz", "pt_id", "ln_orth", "ln_id", "ept_lm", "ept_kf", "ept_obs",
                  "ept_info", "eln_lm", "eln_kf", "eln_obs", "eln_info"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
    hm.compare_maps(ma, mb, pose_tol=0, lm_tol=0)
    assert db == 0 and 0 < da < ga[-1].n_pt + ga[-1].n_ln   # the repeat call re-read only the changed landmarks
