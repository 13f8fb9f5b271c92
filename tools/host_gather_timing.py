"""CPU-only timing of the host mirror's per-call bookkeeping (no GPU): MapHandler::
localBundleAdjustmentForPlukerWithG2O on a synthetic map with a solver hook that returns the
window's initial estimates (χ² 0, depth ok), so gather / marshalling and the outlier pass +
write-back are timed exactly as bench.py's host_mirror object times them, minus the device solve.
usage: python tools/host_gather_timing.py [config] [calls]"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
from plba import synth  # noqa: E402
from plba.slam_map import HostMap, make_map  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    g = synth.generate(cfg)
    hm = HostMap(make_map(g), device=0)

    def hook(gr, r):
        C.memmove(r.kf_Tcw, gr.kf_Tcw, 8 * 12 * gr.n_kf)
        C.memmove(r.pt_xyz, gr.pt_xyz, 8 * 3 * gr.n_pt)
        C.memmove(r.ln_orth, gr.ln_orth, 8 * 4 * gr.n_ln)
        C.memset(r.ept_chi2, 0, 8 * gr.n_ept)
        C.memset(r.eln_chi2, 0, 8 * gr.n_eln)
        C.memset(r.ept_depth_ok, 1, gr.n_ept)
        C.memset(r.ept_level, 0, gr.n_ept)
        C.memset(r.eln_level, 0, gr.n_eln)
        return 0

    hm.set_solver(hook)
    rows = [hm.local_ba() for _ in range(calls + 1)]
    hm.close()
    for k in ("gather_ms", "solve_ms", "bookkeeping_ms"):
        print("%-16s median %.3f ms  (first %.3f)" % (k, statistics.median(r[k] for r in rows[1:]), rows[0][k]))
    print({k: rows[-1][k] for k in ("n_free_kf", "n_fixed_kf", "n_pt", "n_ln", "n_ept", "n_eln")})


if __name__ == "__main__":
    main()
