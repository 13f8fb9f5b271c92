"""GPU box: loop-closure pose-graph timing (plba_pgo_optimize) against the CPU oracle
(oracle/refpgo.cpp, one thread) on synthetic drifted loops of growing size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from plba import pgo  # noqa: E402
from plba.lib import Solver  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [40, 150, 400]
with Solver() as s:
    s.pgo_optimize(pgo.loop_graph(n_kf=20, seed=1))  # warm-up (code objects, allocation)
    for n in sizes:
        pg = pgo.loop_graph(n_kf=n, seed=9, cov_window=4, extra_loops=max(1, n // 25))
        t = time.perf_counter()
        out = s.pgo_optimize(pg)
        gpu_ms = (time.perf_counter() - t) * 1e3
        rec = dict(n_kf=n, n_edges=int(len(pg.e_v)), n=6 * out["n_free"], iterations=out["iterations"],
                   trials=out["trials"], gpu_ms=round(gpu_ms, 2), gpu_ms_per_trial=round(gpu_ms / max(out["trials"], 1), 3),
                   chi2=[out["chi2_initial"], out["chi2_final"]])
        if n <= 200:
            t = time.perf_counter()
            ref = oa.pgo_optimize(pg)
            rec["cpu_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            rec["max_pose_diff"] = float(np.abs(out["v_T"] - ref["v_T"]).max())
        print(json.dumps(rec), flush=True)
