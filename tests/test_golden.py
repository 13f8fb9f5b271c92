"""The oracle reproduces the committed golden fixtures (tools/make_golden.py)."""
import numpy as np
import pytest

import golden_io
import oracle_api as oa
from plba import synth


@pytest.mark.parametrize("cfg", ["C1", "C1L"])
def test_fixture_inputs_are_the_seeded_generator(cfg):
    g, _ = golden_io.load(cfg)
    h = synth.generate(cfg)
    for f in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_obs", "eln_obs"):
        np.testing.assert_array_equal(getattr(g, f), getattr(h, f))


@pytest.mark.parametrize("cfg", ["C1", "C1L"])
def test_oracle_reproduces_golden(cfg):
    g, exp = golden_io.load(cfg)
    r = oa.lba_plucker(g)
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2"):
        np.testing.assert_allclose(r[k], exp[k], rtol=1e-9, atol=1e-12, err_msg=k)
    for k in ("ept_depth_ok", "ept_level", "eln_level", "iters"):
        np.testing.assert_array_equal(r[k], exp[k], err_msg=k)
    np.testing.assert_array_equal(np.stack([r["trace"]["trials"], r["trace"]["result"]], -1),
                                  exp["trace_int"][:, 2:])
