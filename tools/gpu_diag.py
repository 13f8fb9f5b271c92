"""Diagnostic: HIP path vs oracle on several configs, with timings (run on the GPU box)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_api as oa  # noqa: E402
from parity import compare  # noqa: E402
from plba import synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

cfgs = sys.argv[1:] or ["C1", "C1L", "C2", "C3"]
s = Solver(kernel_timing=True)
for cfg in cfgs:
    t0 = time.time()
    g = synth.generate(cfg)
    t1 = time.time()
    ref = oa.lba_plucker(g)
    t2 = time.time()
    s.upload(g)
    t3 = time.time()
    out = s.lba_plucker()
    # second run for warm timing
    s.reset()
    out2 = s.lba_plucker()
    m = compare(out, ref)
    print(f"== {cfg}: E={g.n_ept}+{g.n_eln} gen {t1-t0:.2f}s oracle {ref['solve_ms']:.1f}ms upload {1e3*(t3-t2):.1f}ms "
          f"gpu {out['solve_ms']:.2f}ms / {out2['solve_ms']:.2f}ms iters gpu {out['iters']} ref {ref['iters']}", flush=True)
    print("   metrics", m, flush=True)
    print("   depth flags equal:", np.array_equal(out["ept_depth_ok"], ref["ept_depth_ok"]),
          "gpu bad", int((out["ept_depth_ok"] == 0).sum()), "ref bad", int((ref["ept_depth_ok"] == 0).sum()),
          "chi2 rel", float(np.abs(out["ept_chi2"] - ref["ept_chi2"]).max() / max(ref["ept_chi2"].max(), 1e-30)))
    print("   deterministic rerun:", all(np.array_equal(out[k], out2[k]) for k in ("kf_Tcw", "pt_xyz", "ln_orth")))
    for a, b in zip(out["trace"], ref["trace"]):
        print(f"   st{a['stage']} it{a['iter']:2d} gpu chi {a['chi2_start']:.10g}->{a['chi2_end']:.10g} lam {a['lambda_end']:.4g} tr {a['trials']} | "
              f"ref {b['chi2_start']:.10g}->{b['chi2_end']:.10g} lam {b['lambda_end']:.4g} tr {b['trials']}")
    kt = s.kernel_times()
    tot = sum(v[0] for v in kt.values())
    print("   kernel ms:", {k: (round(v[0], 3), v[1]) for k, v in kt.items()}, "sum", round(tot, 3), flush=True)
s.close()
