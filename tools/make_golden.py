"""Generate the committed golden fixtures tests/golden/<cfg>.npz.

Each fixture holds the seeded input window (synth.generate) and the CPU oracle's outputs of
the full two-stage LBA (final estimates, per-edge χ² / depth / level, per-iteration trace).
The reference itself has no golden vectors, so these pin regressions of the
oracle and serve as the GPU parity fixtures.
Usage: python tools/make_golden.py [C1 C1L ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from plba import synth  # noqa: E402


def main(cfgs):
    os.makedirs(os.path.join(ROOT, "tests", "golden"), exist_ok=True)
    for cfg in cfgs:
        g = synth.generate(cfg)
        r = oa.lba_plucker(g)
        path = os.path.join(ROOT, "tests", "golden", f"{cfg}.npz")
        g.save(path)
        with np.load(path, allow_pickle=False) as z:
            d = dict(z)
        for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "ept_depth_ok", "ept_level", "eln_chi2",
                  "eln_level", "iters", "chi2"):
            d["out_" + k] = r[k]
        tr = r["trace"]
        d["out_trace_int"] = np.stack([tr["stage"], tr["iter"], tr["trials"], tr["result"]], -1).astype(np.int32)
        d["out_trace_f64"] = np.stack([tr["chi2_start"], tr["chi2_end"], tr["lambda_start"], tr["lambda_end"]], -1)
        np.savez_compressed(path, **d)
        print(cfg, path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main(sys.argv[1:] or ["C1", "C1L"])
