"""Device-side window build (csrc/plba_build.hip) against the host build.

plba_upload builds the window structure — landmark order, landmark-major edge CSR, free-pose
edge lists, the reduced-camera envelope and the block-sorted Schur triples — on the GPU unless
PLBA_HOST_BUILD=1. Both builds must produce the same structure (same orders, so every reduction
sums in the same order): the solves must be bitwise identical, on ordinary windows and on the
edge cases (shuffled ids and edges, duplicate observations, lines / points only, no free pose,
landmarks seen only by fixed keyframes, landmarks never observed, an idle free pose)."""
import numpy as np
import pytest

import graph_mut as gm
import oracle_api as oa
from plba import synth

pytestmark = pytest.mark.gpu

KEYS = ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "eln_level", "ept_depth_ok", "iters",
        "chi2")
STRUCT = ("nf", "bw", "nblk", "triples", "edges", "landmarks", "banded", "chunks", "free_edges", "point_edges",
          "twisted", "column_lane", "bcr_rows", "dense_mfma")


def _solve(monkeypatch, g, host):
    from plba.lib import Solver
    if host:
        monkeypatch.setenv("PLBA_HOST_BUILD", "1")
    else:
        monkeypatch.delenv("PLBA_HOST_BUILD", raising=False)
    with Solver() as s:
        s.upload(g)
        st = s.structure_stats()
        out = s.lba_plucker()
    monkeypatch.delenv("PLBA_HOST_BUILD", raising=False)
    return st, out


def _unobserved_landmarks(g):
    h = g.copy()
    h.pt_xyz = np.concatenate([g.pt_xyz, g.pt_xyz[:5] + 1.0])
    h.pt_id = np.concatenate([g.pt_id, np.arange(5, dtype=g.pt_id.dtype) + int(g.pt_id.max()) + 1000])
    return h


CASES = {
    "C1": lambda: synth.generate("C1"),
    "C1L": lambda: synth.generate("C1L"),
    "C2": lambda: synth.generate("C2"),
    "C3": lambda: synth.generate("C3"),
    "C4": lambda: synth.generate("C4"),
    "shuffled": lambda: gm.shuffled(synth.generate("C2"), seed=3),
    "duplicates": lambda: gm.with_duplicate_observations(synth.generate("C1L")),
    "lines_only": lambda: gm.drop_points(synth.generate("C1L")),
    "points_only": lambda: gm.drop_lines(synth.generate("C1L")),
    "all_fixed": lambda: gm.all_fixed(synth.generate("C1L")),
    "fixed_only_landmarks": lambda: gm.fixed_only_landmarks(synth.generate("C1L")),
    "idle_free_pose": lambda: gm.add_idle_free_pose(synth.generate("C1L")),
    "unobserved": lambda: _unobserved_landmarks(synth.generate("C1L")),
}


@pytest.mark.parametrize("case", list(CASES))
def test_device_build_equals_host_build(monkeypatch, case):
    g = CASES[case]()
    st_d, out_d = _solve(monkeypatch, g, host=False)
    st_h, out_h = _solve(monkeypatch, g, host=True)
    for k in STRUCT:
        assert st_d[k] == st_h[k], (k, st_d, st_h)
    for k in KEYS:
        assert np.array_equal(out_d[k], out_h[k]), k


def _scrambled_ids(g, seed=11):
    h = g.copy()
    h.kf_id = np.random.default_rng(seed).permutation(g.n_kf).astype(np.int32)
    return h


RCM_CASES = {
    "C2R": lambda: synth.generate("C2R"),
    "C3R": lambda: synth.generate("C3R"),
    "C2_scrambled": lambda: _scrambled_ids(synth.generate("C2")),
    "C1L_scrambled": lambda: _scrambled_ids(synth.generate("C1L", n_kf=40, n_pt=800, n_ln=160, seed=43)),
}


@pytest.mark.parametrize("case", list(RCM_CASES))
def test_device_build_rcm_equals_host_build(monkeypatch, case):
    """Windows whose id-order envelope is too wide for the banded kernels (a revisit loop,
    scrambled keyframe ids): the device build reorders the free poses by the host build's RCM
    permutation and builds again on the device — same structure, bitwise-equal solves."""
    g = RCM_CASES[case]()
    st_d, out_d = _solve(monkeypatch, g, host=False)
    st_h, out_h = _solve(monkeypatch, g, host=True)
    assert st_d["device_build"] == 1 and st_h["device_build"] == 0, (st_d, st_h)
    for k in STRUCT:
        assert st_d[k] == st_h[k], (k, st_d, st_h)
    for k in KEYS:
        assert np.array_equal(out_d[k], out_h[k]), k


def test_device_build_invalid_edge_reported(monkeypatch):
    from plba.lib import PlbaError, Solver
    g = synth.generate("C1L")
    g.eln_kf = g.eln_kf.copy()
    g.eln_kf[7] = g.n_kf + 3
    with Solver() as s:
        with pytest.raises(PlbaError, match="line edge 7 references a missing vertex"):
            s.upload(g)
        s.upload(synth.generate("C1"))   # the context stays usable
        out = s.lba_plucker()
    ref = oa.lba_plucker(synth.generate("C1"))
    np.testing.assert_array_equal(out["iters"], ref["iters"])


def test_device_build_reuses_context_across_sizes(monkeypatch):
    """Grow-only build memory: a large window after a small one and a small one after a large
    one, on one context, each equal to a fresh context's solve."""
    from plba.lib import Solver
    gs = [synth.generate("C1L"), synth.generate("C3"), synth.generate("C2")]
    with Solver() as s:
        outs = []
        for g in gs:
            s.upload(g)
            outs.append(s.lba_plucker())
    for g, o in zip(gs, outs):
        _, fresh = _solve(monkeypatch, g, host=False)
        for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_level"):
            assert np.array_equal(o[k], fresh[k]), k


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_step_graph_update_across_windows(monkeypatch, cfg):
    """Consecutive windows with the same launch signature (C2: column-lane, C4: BCR) reuse the
    executable step graphs through hipGraphExecUpdate: each solve equals a fresh context's."""
    from plba.lib import Solver
    seeds = [synth.CONFIGS[cfg][3] + 101 * k for k in range(3)]
    gs = [synth.generate(cfg, seed=sd) for sd in seeds]
    with Solver() as s:
        outs = []
        for g in gs:
            s.upload(g)
            outs.append(s.lba_plucker())
            assert s.structure_stats()["graph"] == 1
    for g, o in zip(gs, outs):
        _, fresh = _solve(monkeypatch, g, host=False)
        for k in KEYS:
            assert np.array_equal(o[k], fresh[k]), k


def test_step_graph_update_across_window_sizes(monkeypatch):
    """Windows of different keyframe counts with the same launch signature (same bandwidth and
    factorisation): the updated executable graphs carry the new grids and the new dynamic LDS size
    of the column-lane factorisation (its x_p staging grows with nf) — each solve equals a fresh
    context's, bitwise (the update path with a changed LDS size / grid)."""
    from plba.lib import Solver
    gs = [synth.generate("C2", n_kf=nk, n_pt=100 * nk, n_ln=20 * nk, seed=2000 + nk) for nk in (40, 56, 75)]
    with Solver() as s:
        outs, sts = [], []
        for g in gs:
            s.upload(g)
            outs.append(s.lba_plucker())
            sts.append(s.structure_stats())
    assert len({st["nf"] for st in sts}) == 3, sts
    for g, o in zip(gs, outs):
        _, fresh = _solve(monkeypatch, g, host=False)
        for k in KEYS:
            assert np.array_equal(o[k], fresh[k]), k
