"""refcpu-fast (BASELINE.md §2 lower bound: oracle/refcpu.cpp built -DREFCPU_FAST, fixed-size
blocks) computes exactly what the g2o-structured oracle computes: same products in the same
summation order, so every output is bitwise equal. Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_api as oa
from plba import synth


@pytest.fixture(scope="module")
def fast_lib():
    subprocess.run(["make", "-C", oa.ORACLE_DIR, "-s", "fast"], check=True)
    return os.path.join(oa.ORACLE_DIR, "librefcpu_fast_native.so")


@pytest.mark.parametrize("cfg", ["C1", "C1L"])
def test_refcpu_fast_is_bitwise_equal(cfg, fast_lib):
    g = synth.generate(cfg)
    saved = (oa._lib, oa.ORACLE_SO)
    try:
        oa._lib, oa.ORACLE_SO = None, oa.build_oracle()
        ref = oa.lba_plucker(g)
        oa._lib, oa.ORACLE_SO = None, fast_lib
        oa._lib = None
        L = C.CDLL(fast_lib)  # loads (symbols exported like librefcpu.so)
        assert hasattr(L, "refcpu_lba_plucker")
        fast = oa.lba_plucker(g)
    finally:
        oa._lib, oa.ORACLE_SO = saved
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "iters", "chi2"):
        np.testing.assert_array_equal(np.asarray(fast[k]), np.asarray(ref[k]), err_msg=k)
