"""One-shot hand-rolled GBA (levMarquardtOptimizationGBA, src/mapHandler.cpp:3128-3726; run once on
the whole map at app end, app/plslam_dataset.cpp:174) on the GPU beside the CPU oracle
(oracle/refhlm.cpp, one thread), at the given configs. Prints one JSON line per config.

usage (GPU box): python tools/gba_timing.py C4 C5:2   (cfg:K = the oracle timed on a bounded sample of
K linearisations, reported per linearisation beside the GPU's; the full-size oracle run takes minutes)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from plba import capi, synth  # noqa: E402
from plba.hlm import gba_window  # noqa: E402
from plba.lib import Solver  # noqa: E402

for arg in sys.argv[1:] or ["C4"]:
    cfg, _, kcap = arg.partition(":")
    win = gba_window(synth.generate(cfg))
    for params in ({}, {"lambda0": 1e-7, "err_per_obs": 1}):
        p = capi.gba_params(**params)
        with Solver() as s:
            t0 = time.perf_counter()
            s.upload(win.graph)
            t1 = time.perf_counter()
            s.hlm_lba(win, p)            # warm (graph capture)
            t2 = time.perf_counter()
            out = s.hlm_lba(win, p)
            t3 = time.perf_counter()
        pr = capi.gba_params(**params, **({"max_iters": int(kcap)} if kcap else {}))
        c0 = time.perf_counter()
        ref = oa.hlm_lba(win, pr)
        c1 = time.perf_counter()
        same = (out["linearizations"], out["solves"], out["accepted"]) == (ref["linearizations"], ref["solves"],
                                                                           ref["accepted"]) if not kcap else None
        print(json.dumps({"config": cfg, "params": params, "n_kf": win.graph.n_kf, "n_pt": win.graph.n_pt,
                          "n_ln": win.graph.n_ln, "linearizations": out["linearizations"], "solves": out["solves"],
                          "gpu_upload_ms": (t1 - t0) * 1e3, "gpu_first_call_ms": (t2 - t1) * 1e3,
                          "gpu_gba_ms": (t3 - t2) * 1e3, "gpu_solve_ms": out["solve_ms"],
                          "cpu_oracle_ms": (c1 - c0) * 1e3, "cpu_oracle_linearizations": ref["linearizations"],
                          "gpu_ms_per_linearization": (t3 - t2) * 1e3 / max(out["linearizations"], 1),
                          "cpu_ms_per_linearization": (c1 - c0) * 1e3 / max(ref["linearizations"], 1),
                          "same_control_flow": same,
                          "max_abs_pt_diff": None if kcap else float(np.abs(out["pt_xyz"] - ref["pt_xyz"]).max())}),
              flush=True)
