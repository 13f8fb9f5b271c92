"""Diagnostics: host-side phases of plba_upload and the step-graph capture (PLBA_TIMING=1)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
os.environ["PLBA_TIMING"] = "1"
from plba import synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

for cfg in sys.argv[1:] or ["C3"]:
    seed = synth.CONFIGS[cfg][3]
    with Solver() as s:
        for rep in range(3):
            g = synth.generate(cfg, seed=seed + 7919 * rep)   # a new window each time, as bench.py
            print(f"== {cfg} upload {rep}", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            s.upload(g)
            t1 = time.perf_counter()
            out = s.lba_plucker(want_outputs=False)
            t2 = time.perf_counter()
            s.reset()
            out2 = s.lba_plucker(want_outputs=False)
            t3 = time.perf_counter()
            s.reset()
            out3 = s.lba_plucker(want_outputs=True)
            t4 = time.perf_counter()
            print(f"{cfg}: upload {1e3*(t1-t0):.2f} ms, first LBA (incl. graph update) {1e3*(t2-t1):.2f} ms "
                  f"(solve_ms {out['solve_ms']:.2f}), repeat LBA {1e3*(t3-t2):.2f} ms (solve_ms {out2['solve_ms']:.2f}), "
                  f"LBA + download {1e3*(t4-t3):.2f} ms", file=sys.stderr, flush=True)
