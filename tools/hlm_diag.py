"""GPU-box diagnostic: per-KF differences of the hand-rolled LM (GPU vs oracle)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
import numpy as np
import oracle_api as oa
from plba import capi, synth
from plba.hlm import hlm_window
from plba.lib import Solver

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
kw = dict(lambda0=1e-24, err_per_obs=1, max_iters=int(sys.argv[2]) if len(sys.argv) > 2 else 6)
w = hlm_window(synth.generate(cfg))
p = capi.hlm_params(**kw)
ref = oa.hlm_lba(w, p)
with Solver() as s:
    s.upload(w.graph)
    out = s.hlm_lba(w, p)
    print("structure", s.structure_stats())
th = np.linalg.norm(w.kf_x[:, 3:], axis=1)
dx = np.abs(out["kf_x"] - ref["kf_x"]).max(1)
dT = np.abs(out["kf_Tcw"] - ref["kf_Tcw"]).reshape(len(th), -1).max(1)
ch = np.abs(ref["kf_Tcw"] - w.graph.kf_Tcw).reshape(len(th), -1).max(1)
o = np.argsort(-dx)[:8]
for k in o:
    print(f"kf {k:4d} fixed={w.graph.kf_fixed[k]} theta={th[k]:.6f} dx={dx[k]:.3e} dTcw={dT[k]:.3e} oracle_change={ch[k]:.3e}")
print("trace gpu", out["trace"][["iter", "result", "lambda_start"]])
print("trace ref", ref["trace"][["iter", "result", "lambda_start"]])
print("dx_norm", out["dx_norm"], ref["dx_norm"], "err", out["err"], ref["err"])
print("pt", np.abs(out["pt_xyz"] - ref["pt_xyz"]).max(), "ln", np.abs(out["ln_orth"] - ref["ln_orth"]).max())
