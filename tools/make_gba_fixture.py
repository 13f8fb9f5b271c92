"""Generate tests/golden/gba_C5_it2.npz: the bounded C5 GBA parity fixture.

levMarquardtOptimizationGBA (src/mapHandler.cpp:3128-3726) on the seeded C5 window
(synth.generate("C5"), plba.hlm.gba_window) with max_iters = 2, solved by the CPU oracle
(oracle/refhlm.cpp, ~100 s on one core): the control-flow counters, the trace, every pose and a
fixed seeded sample of 4000 points and 1000 lines (the full landmark arrays would be ~7 MB).
The GPU test (tests/test_gpu_hlm.py::test_gba_c5_bounded_matches_oracle_fixture) rebuilds the
same window, runs plba_hlm_lba and compares against this file.
Usage: python tools/make_gba_fixture.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from plba import capi, synth  # noqa: E402
from plba.hlm import gba_window  # noqa: E402

CFG, MAX_ITERS, NPT, NLN = "C5", 2, 4000, 1000


def sample(n_pt, n_ln):
    rng = np.random.default_rng(20261017)
    return (np.sort(rng.choice(n_pt, size=min(NPT, n_pt), replace=False)),
            np.sort(rng.choice(n_ln, size=min(NLN, n_ln), replace=False)))


def main():
    win = gba_window(synth.generate(CFG))
    ref = oa.hlm_lba(win, capi.gba_params(max_iters=MAX_ITERS))
    g = win.graph
    ip, il = sample(g.n_pt, g.n_ln)
    tr = ref["trace"]
    d = dict(
        counters=np.array([ref["linearizations"], ref["solves"], ref["accepted"]], np.int64),
        err=np.array([ref["err"], ref["dx_norm"]]),
        trace_int=np.stack([tr["iter"], tr["result"]], -1).astype(np.int32),
        trace_lam=np.stack([tr["lambda_start"], tr["lambda_end"]], -1),
        kf_Tcw=ref["kf_Tcw"], kf_x=ref["kf_x"],
        pt_idx=ip, pt_xyz=np.asarray(ref["pt_xyz"]).reshape(-1, 3)[ip],
        ln_idx=il, ln_line3d=np.asarray(ref["ln_line3d"]).reshape(-1, 6)[il],
        # the window's initial values of the same entries (the tolerance is relative to the change)
        init_kf_Tcw=np.asarray(g.kf_Tcw), init_pt=np.asarray(g.pt_xyz).reshape(-1, 3)[ip],
        init_ln=np.asarray(win.ln_line3d).reshape(-1, 6)[il],
    )
    path = os.path.join(ROOT, "tests", "golden", f"gba_{CFG}_it{MAX_ITERS}.npz")
    np.savez_compressed(path, **d)
    print(path, os.path.getsize(path), "bytes", d["counters"], d["err"])


if __name__ == "__main__":
    main()
