"""Diagnostic: one generated window, HIP band path vs HIP dense path vs oracle, traces side by side.

usage: python tools/diag_case.py n_kf n_pt track_max seed [fixed_frac]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from parity import compare  # noqa: E402
from plba import synth  # noqa: E402


def main():
    n_kf, n_pt, tmax, seed = (int(x) for x in sys.argv[1:5])
    ff = float(sys.argv[5]) if len(sys.argv) > 5 else 0.1
    g = synth.generate("C1", n_kf=n_kf, n_pt=n_pt, seed=seed, track_min=2, track_max=tmax, fixed_frac=ff)
    if os.environ.get("PLBA_DIAG_CHILD"):
        from plba.lib import Solver
        s = Solver()
        s.upload(g)
        out = s.lba_plucker()
        np.savez(os.environ["PLBA_DIAG_CHILD"], **{k: v for k, v in out.items() if k != "trace"},
                 trace=out["trace"])
        print("stats", s.structure_stats())
        return
    ref = oa.lba_plucker(g)
    res = {}
    for mode in os.environ.get("PLBA_DIAG_MODES", "band,dense").split(","):
        env = dict(os.environ, PLBA_DIAG_CHILD=f"/tmp/diag_{mode}.npz", PLBA_FORCE_DENSE="1" if mode == "dense" else "0")
        subprocess.run([sys.executable, __file__] + sys.argv[1:], env=env, check=True)
        with np.load(f"/tmp/diag_{mode}.npz") as z:
            res[mode] = {k: z[k] for k in z.files}
    for mode, out in res.items():
        print(mode, "vs oracle", compare(out, ref))
    if len(res) < 2:
        return
    print("band vs dense", compare(res["band"], res["dense"]))
    for a, b, c in zip(res["band"]["trace"], res["dense"]["trace"], ref["trace"]):
        print(f"st{a['stage']} it{a['iter']:2d} band {a['chi2_end']:.15g} tr{a['trials']} | dense {b['chi2_end']:.15g} "
              f"tr{b['trials']} | ref {c['chi2_end']:.15g} tr{c['trials']} lam {c['lambda_end']:.3g}")


if __name__ == "__main__":
    main()
