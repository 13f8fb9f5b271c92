"""Test-side restatement of the reference's host logic around the g2o solve (checker for the
C++ host mirror, pl-slam-plucker_amd/host/):

  gather     src/mapHandler.cpp:5868-5921   (A1)
  marshal    src/mapHandler.cpp:5931-6117   (A1b)
  outliers   src/mapHandler.cpp:6154-6293   (A1d)
  write-back src/mapHandler.cpp:6296-6319   (A1e)
  formLocalMap(kf)                src/mapHandler.cpp:1073-1137   
  removeBadMapLandmarksForPluker  src/mapHandler.cpp:3816-3897   (§8f row 3)

operating on plba.slam_map.SlamMap objects. `solve` is any callable Graph -> result dict
(a stub on CPU, the CPU oracle in GPU tests).
"""
from __future__ import annotations

import math
from typing import Callable

import numpy as np

from plba import geometry as geo
from plba.slam_map import SlamMap, median_descriptor
from plba.synth import Graph

HUBER = float(np.float32(math.sqrt(5.991)))


def inv4(T):
    return np.linalg.inv(T)


def pluker_to_orth(L):   # src/mapFeatures.cpp:186-201
    return geo.pluker_to_orth(np.asarray(L, np.float64))


def orth_to_pluker(o):   # src/mapFeatures.cpp:203-221
    return geo.orth_to_pluker(np.asarray(o, np.float64))


def gather(m: SlamMap):
    """Returns (Graph, window) and applies the gather's side effect (observer KFs -> local)."""
    kfs = m.keyframes
    nofix = {k.kf_idx: k for k in kfs if k is not None and k.local}
    local_pt = [p for p in m.points if p is not None and p.local]
    local_ls = [l for l in m.lines if l is not None and l.local]
    fix = {}
    for lm in local_pt + local_ls:
        for o in lm.kf_obs_list:
            k = kfs[o]
            assert k.kf_idx == o
            if not k.local:
                fix[o] = k
                k.local = True
    kf_list = [(nofix[i], i == 0) for i in sorted(nofix)] + [(fix[i], True) for i in sorted(fix)]
    pos = {k.kf_idx: j for j, (k, _) in enumerate(kf_list)}
    max_kf_id = max([k.kf_idx + 1 for k, _ in kf_list], default=0)
    Tcw = np.array([inv4(k.T_kf_w)[:3, :] for k, _ in kf_list]).reshape(-1, 3, 4)
    fixed = np.array([f for _, f in kf_list], np.uint8)
    kf_id = np.array([k.kf_idx for k, _ in kf_list], np.int32)
    ept = dict(lm=[], kf=[], obs=[], info=[], kfp=[], oi=[])
    pt_id = []
    maxPointId = max_kf_id
    for li, p in enumerate(local_pt):
        pid = p.idx + max_kf_id + 1
        pt_id.append(pid)
        for i, o in enumerate(p.kf_obs_list):
            ept["lm"].append(li)
            ept["kf"].append(pos[o])
            ept["obs"].append(p.obs_list[i])
            ept["info"].append(float(np.float32(1.0 / p.sigma_list[i])))
            ept["kfp"].append(kfs[o])
            ept["oi"].append(i)
        maxPointId = pid + 1
    eln = dict(lm=[], kf=[], obs=[], info=[], kfp=[], oi=[])
    ln_id, ln_orth = [], []
    for li, l in enumerate(local_ls):
        ln_id.append(l.idx + maxPointId + 1)
        ln_orth.append(pluker_to_orth(l.pos))
        for i, o in enumerate(l.kf_obs_list):
            eln["lm"].append(li)
            eln["kf"].append(pos[o])
            eln["obs"].append(l.obs_list[i])
            eln["info"].append(float(np.float32(1.0 / l.sigma_list[i])))
            eln["kfp"].append(kfs[o])
            eln["oi"].append(i)
    g = Graph(fx=m.fx, fy=m.fy, cx=m.cx, cy=m.cy, kf_Tcw=Tcw, kf_fixed=fixed, kf_id=kf_id,
              pt_xyz=np.array([p.pos for p in local_pt], np.float64).reshape(-1, 3),
              pt_id=np.array(pt_id, np.int32),
              ln_orth=np.array(ln_orth, np.float64).reshape(-1, 4), ln_id=np.array(ln_id, np.int32),
              ept_lm=np.array(ept["lm"], np.int32), ept_kf=np.array(ept["kf"], np.int32),
              ept_obs=np.array(ept["obs"], np.float64).reshape(-1, 2), ept_info=np.array(ept["info"]),
              eln_lm=np.array(eln["lm"], np.int32), eln_kf=np.array(eln["kf"], np.int32),
              eln_obs=np.array(eln["obs"], np.float64).reshape(-1, 4), eln_info=np.array(eln["info"]),
              huber_pt=HUBER, huber_ln=HUBER)
    win = dict(kf_list=kf_list, local_pt=local_pt, local_ls=local_ls, ept=ept, eln=eln,
               n_free=len(nofix), n_fixed=len(fix))
    return g, win


def lba(m: SlamMap, solve: Callable[[Graph], dict]) -> dict:
    """MapHandler::localBundleAdjustmentForPlukerWithG2O on the Python map (mutates m)."""
    g, win = gather(m)
    r = solve(g)
    st = dict(n_free_kf=win["n_free"], n_fixed_kf=win["n_fixed"], n_pt=g.n_pt, n_ln=g.n_ln, n_ept=g.n_ept,
              n_eln=g.n_eln, bad_line_stage1=int((np.asarray(r["eln_level"]) == 1).sum()),
              bad_point_obs=0, actually_bad_point_obs=0, bad_line_obs=0, actually_bad_line_obs=0,
              iters=[int(v) for v in r["iters"]], chi2=[float(v) for v in r["chi2"]])

    def rebase(kf_obs, lm_idx, new_base):
        lst = m.map_points_kf_idx[kf_obs]
        for v in lst:
            if v == lm_idx:
                m.map_points_kf_idx[new_base].append(v)
                break

    def dec(a, b):
        m.full_graph[a, b] = np.uint32((int(m.full_graph[a, b]) - 1) & 0xFFFFFFFF)
        m.full_graph[b, a] = np.uint32((int(m.full_graph[b, a]) - 1) & 0xFFFFFFFF)

    for kind, E, lms in (("pt", win["ept"], win["local_pt"]), ("ln", win["eln"], win["local_ls"])):
        chi2 = r["ept_chi2"] if kind == "pt" else r["eln_chi2"]
        for i in range(len(E["lm"]) - 1, -1, -1):
            bad = chi2[i] > 5.991 or (kind == "pt" and not r["ept_depth_ok"][i])
            if not bad:
                continue
            st["bad_point_obs" if kind == "pt" else "bad_line_obs"] += 1
            kf = E["kfp"][i]
            lm = lms[E["lm"][i]]
            if len(lm.obs_list) > 1:
                st["actually_bad_point_obs" if kind == "pt" else "actually_bad_line_obs"] += 1
                kf_obs, lm_idx, oi = kf.kf_idx, lm.idx, E["oi"][i]
                if oi == 0:
                    rebase(kf_obs, lm_idx, lm.kf_obs_list[1])
                del lm.desc_list[oi]
                del lm.obs_list[oi]
                if kind == "pt":
                    del lm.dir_list[oi]
                del lm.kf_obs_list[oi]
                feats = kf.pt_idx if kind == "pt" else kf.ls_idx
                for j, f in enumerate(feats):
                    if f == lm_idx:
                        feats[j] = -1
                        break
                lm.med_desc = lm.desc_list[median_descriptor(lm.desc_list)]
                if kind == "pt":
                    lm.med_dir = np.sum(lm.dir_list, axis=0) / len(lm.desc_list)
                for idx in lm.kf_obs_list:
                    if kf_obs != idx:
                        dec(kf_obs, idx)
            else:
                lm.inlier = False
    # write-back
    for j, (k, _) in enumerate(win["kf_list"][:win["n_free"]]):
        est = inv4(k.T_kf_w)
        est[:3, :] = np.asarray(r["kf_Tcw"]).reshape(-1, 3, 4)[j]
        k.T_kf_w = inv4(est)
    for j, p in enumerate(win["local_pt"]):
        p.pos = np.asarray(r["pt_xyz"]).reshape(-1, 3)[j].copy()
    for j, l in enumerate(win["local_ls"]):
        l.pos = orth_to_pluker(np.asarray(r["ln_orth"]).reshape(-1, 4)[j])
    return st


def form_local_map(m: SlamMap, kf_idx: int, params) -> None:
    """MapHandler::formLocalMap(KeyFrame*) (src/mapHandler.cpp:1073-1137)."""
    for k in m.keyframes:
        if k is not None:
            k.local = False
    for lm in m.points + m.lines:
        if lm is not None:
            lm.local = False

    def mark(k):
        for i in k.pt_idx:
            if i != -1 and m.points[i] is not None:
                m.points[i].local = True
        for i in k.ls_idx:
            if i != -1 and m.lines[i] is not None:
                m.lines[i].local = True
    kf = m.keyframes[kf_idx]
    kf.local = True
    mark(kf)
    g_size = m.full_graph.shape[0] - 1
    for i in range(g_size):
        if int(m.full_graph[g_size, i]) >= params.min_lm_cov_graph or abs(g_size - i) <= params.min_kf_local_map:
            m.keyframes[i].local = True
            mark(m.keyframes[i])


def remove_bad(m: SlamMap, params):
    """MapHandler::removeBadMapLandmarksForPluker() (src/mapHandler.cpp:3816-3897)."""
    removed = [0, 0]
    for kind, lms, kidx in ((0, m.points, m.map_points_kf_idx), (1, m.lines, m.map_lines_kf_idx)):
        for j, lm in enumerate(lms):
            if lm is None:
                continue
            if not lm.local and m.max_kf_idx - lm.kf_obs_list[0] > 10 and \
                    (not lm.inlier or len(lm.obs_list) < params.min_lm_obs):
                kf_obs = lm.kf_obs_list[0]
                feats = m.keyframes[kf_obs].pt_idx if kind == 0 else m.keyframes[kf_obs].ls_idx
                for q, f in enumerate(feats):
                    if f == lm.idx:
                        feats[q] = -1
                        break
                lst = kidx[kf_obs]
                if lm.idx in lst:
                    lst.remove(lm.idx)          # first occurrence
                lms[j] = None
                removed[kind] += 1
    return removed


def local_mapping_step(m: SlamMap, kf_idx: int, solve, params) -> dict:
    """localMappingThread's USE_LINE_PLUKER body after lookForCommonMatches
    (src/mapHandler.cpp:1274-1279)."""
    form_local_map(m, kf_idx, params)
    st = lba(m, solve)
    st["points_removed"], st["lines_removed"] = remove_bad(m, params)
    return st


def compare_maps(a: SlamMap, b: SlamMap, pose_tol=1e-9, lm_tol=1e-9):
    """Raises AssertionError on the first mismatch (bookkeeping exact, states to tolerance)."""
    for ka, kb in zip(a.keyframes, b.keyframes):
        assert (ka is None) == (kb is None)
        if ka is None:
            continue
        assert ka.local == kb.local, ("kf local", ka.kf_idx)
        assert ka.pt_idx == kb.pt_idx, ("kf pt_idx", ka.kf_idx)
        assert ka.ls_idx == kb.ls_idx, ("kf ls_idx", ka.kf_idx)
        d = np.abs(ka.T_kf_w - kb.T_kf_w).max()
        assert d <= pose_tol * max(1.0, np.abs(kb.T_kf_w).max()), ("kf pose", ka.kf_idx, d)
    for kind, la, lb in (("pt", a.points, b.points), ("ln", a.lines, b.lines)):
        for x, y in zip(la, lb):
            assert (x is None) == (y is None)
            if x is None:
                continue
            tag = (kind, x.idx)
            assert x.local == y.local and x.inlier == y.inlier, (tag, "flags")
            assert x.kf_obs_list == y.kf_obs_list, (tag, "kf_obs_list", x.kf_obs_list, y.kf_obs_list)
            assert np.array_equal(np.array(x.obs_list), np.array(y.obs_list)), (tag, "obs_list")
            assert x.sigma_list == y.sigma_list, (tag, "sigma_list")
            assert np.array_equal(x.med_desc, y.med_desc), (tag, "med_desc")
            if kind == "pt":
                assert np.allclose(x.med_dir, y.med_dir, rtol=0, atol=1e-12), (tag, "med_dir")
                assert len(x.dir_list) == len(y.dir_list)
            d = np.abs(np.asarray(x.pos) - np.asarray(y.pos)).max()
            assert d <= lm_tol * max(1.0, np.abs(y.pos).max()), (tag, "pos", d)
    assert np.array_equal(a.full_graph, b.full_graph), "full_graph"
    assert a.map_points_kf_idx == b.map_points_kf_idx, "map_points_kf_idx"
    assert a.map_lines_kf_idx == b.map_lines_kf_idx, "map_lines_kf_idx"
