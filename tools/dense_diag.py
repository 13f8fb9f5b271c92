"""GPU box: structure and per-kernel times of the wide-envelope paths (RCM band / dense MFMA)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
from plba import synth
from plba.lib import Solver
for cfg in sys.argv[1:] or ["C2R", "C3R"]:
    g = synth.generate(cfg)
    for env in ({}, {"PLBA_NO_RCM": "1"}):
        os.environ.pop("PLBA_NO_RCM", None)
        os.environ.update(env)
        with Solver(kernel_timing=True) as s:
            s.upload(g)
            st = s.structure_stats()
            out = s.lba_plucker(want_outputs=False)
            kt = {k: (round(v[0] / max(v[1], 1) * 1e3, 1), v[1]) for k, v in s.kernel_times().items() if v[1]}
            it = int(out["iters"][0] + out["iters"][1])
            print(cfg, env, "nf", st["nf"], "bw", st["bw"], "banded", st["banded"], "twisted", st["twisted"],
                  "cl", st["column_lane"], "bcr", st["bcr_rows"], "dense_mfma", st["dense_mfma"],
                  "solve_ms %.2f" % out["solve_ms"], "iters", it, flush=True)
            print("   us/launch,launches:", kt, flush=True)
