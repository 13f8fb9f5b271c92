"""Synthetic window generator: determinism and shape invariants."""
import numpy as np
import pytest

from plba import geometry as geo
from plba import synth


def test_deterministic():
    a, b = synth.generate("C1L"), synth.generate("C1L")
    for f in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_obs", "eln_obs", "ept_kf", "eln_kf"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("cfg", ["C1", "C1L", "C2"])
def test_window_invariants(cfg):
    g = synth.generate(cfg)
    n_kf, n_pt, n_ln, _ = synth.CONFIGS[cfg]
    assert (g.n_kf, g.n_pt, g.n_ln) == (n_kf, n_pt, n_ln)
    # fixed set: first max(1, round(0.1 N)) KFs, incl. id 0
    assert g.kf_fixed[0] == 1 and g.kf_fixed.sum() == max(1, round(0.1 * n_kf))
    # tracks are contiguous runs of 2..8 KFs, edges landmark-major (g2o insertion order)
    for lm_arr, kf_arr, n in ((g.ept_lm, g.ept_kf, n_pt), (g.eln_lm, g.eln_kf, n_ln)):
        if n == 0:
            continue
        assert np.all(np.diff(lm_arr) >= 0)
        counts = np.bincount(lm_arr, minlength=n)
        assert counts.min() >= 2 and counts.max() <= 8
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        for s, c in zip(starts[:50], counts[:50]):
            assert np.array_equal(kf_arr[s:s + c], np.arange(kf_arr[s], kf_arr[s] + c))
    # vertex ids as src/mapHandler.cpp:5941,5983,6047
    assert g.pt_id[0] == n_kf + 1 if n_pt else True
    if n_ln:
        assert g.ln_id[0] == g.pt_id[-1] + 1 + 1
    # orth estimate is what changePlukerToOrth(changeOrthToPluker(.)) returns
    if n_ln:
        np.testing.assert_allclose(geo.pluker_to_orth(geo.orth_to_pluker(g.ln_orth)), g.ln_orth, atol=1e-12)
    # observations lie in the image (inliers) and Ω = I
    inl = g.ept_outlier == 0
    assert np.all((g.ept_obs[inl, 0] > -10) & (g.ept_obs[inl, 0] < 762))
    assert np.all(g.ept_info == 1.0)


def test_ground_truth_reprojects():
    g = synth.generate("C1", noise_px=0.0, outlier_frac=0.0, perturb=False)
    Pc = np.einsum("eij,ej->ei", g.kf_Tcw[g.ept_kf][:, :, :3], g.pt_xyz[g.ept_lm]) + g.kf_Tcw[g.ept_kf][:, :, 3]
    assert Pc[:, 2].min() > 0.5
    u = Pc[:, 0] / Pc[:, 2] * g.fx + g.cx
    np.testing.assert_allclose(u, g.ept_obs[:, 0], atol=1e-9)


def test_algorithmic_bytes_match_survey():
    # SURVEY.md §8d quotes C1 0.21 MB for E_p = 2.5k; ours has E_p = 2384
    g = synth.generate("C1")
    b = synth.algorithmic_bytes_per_iter(g)
    assert 0.19e6 < b < 0.22e6
