"""Fill BASELINE.md §4: per config C1..C5, the CPU oracle (refcpu-g2o proxy, 1 core pinned) and the
GPU path on the same window — ms per LM iteration, speedup, final χ² of both, max relative
difference of the estimates, HBM fraction of the iteration roofline. Prints a markdown table.
Usage (GPU box): python tools/baseline_table.py [C1 C2 C3 C4 C5]"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pl-slam-plucker_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from parity import compare  # noqa: E402
from plba import synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "native"], check=True)
oa.ORACLE_SO = os.path.join(ROOT, "oracle", "librefcpu_native.so")
HBM = 8000.0
rows = []
for cfg in sys.argv[1:] or ["C1", "C2", "C3", "C4", "C5"]:
    g = synth.generate(cfg)
    prev = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(prev)})
    nrun = 3  # median of 3 everywhere (single C5 runs differed by 31 %)
    oa.lba_plucker(g)
    cms = []
    for _ in range(nrun):
        ref = oa.lba_plucker(g)
        cms.append(ref["solve_ms"])
        print(f"# {cfg} cpu run {len(cms)}: {ref['solve_ms']:.1f} ms", file=sys.stderr, flush=True)
    os.sched_setaffinity(0, prev)
    cit = int(ref["iters"][0] + ref["iters"][1])
    with Solver() as s:
        s.upload(g)
        out = s.lba_plucker()
        gms = []
        for _ in range(5):
            s.reset()
            t0 = time.perf_counter()
            r = s.lba_plucker(want_outputs=False, with_trace=False)
            gms.append((time.perf_counter() - t0) * 1e3)
        st = s.structure_stats()
    git = int(r["iters"][0] + r["iters"][1])
    m = compare(out, ref)
    c_ms_it = statistics.median(cms) / cit
    g_ms_it = statistics.median(gms) / git
    B = synth.algorithmic_bytes_per_iter(g)
    rows.append(dict(cfg=cfg, cpu_ms_it=c_ms_it, cpu_ms_runs=[round(x, 1) for x in cms], gpu_ms_it=g_ms_it, speedup=c_ms_it / g_ms_it,
                     chi2_cpu=float(ref["chi2"][1]), chi2_gpu=float(out["chi2"][1]),
                     max_rel=max(m["Tcw"], m["pt"], m["ln"]), hbm_frac=B / (g_ms_it * 1e-3) / 1e9 / HBM,
                     factor="bcr" if st["bcr_rows"] else ("column-lane" if st["column_lane"] else "band/dense"),
                     iters=[cit, git], levels_equal=m["pt_level_diff"] == 0 and m["ln_level_diff"] == 0))
    print(json.dumps(rows[-1]), flush=True)
print("| cfg | refcpu-g2o ms/iter (1 core) | GPU ms/iter | speedup | final χ² CPU / GPU | max rel. Δ estimates | HBM fraction | factorisation |")
print("|---|---|---|---|---|---|---|---|")
for r in rows:
    print(f"| {r['cfg']} | {r['cpu_ms_it']:.2f} | {r['gpu_ms_it']:.4f} | {r['speedup']:.0f}× | "
          f"{r['chi2_cpu']:.6g} / {r['chi2_gpu']:.6g} | {r['max_rel']:.1e} | {r['hbm_frac']:.2e} | {r['factor']} |")
