"""Diagnostics: where the output download time of plba_lba_plucker goes (host buffers, copies)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
from plba import capi, synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
g = synth.generate(cfg)
with Solver() as s:
    s.upload(g)
    for rep in range(4):
        s.reset()
        t0 = time.perf_counter()
        r = capi.PlbaResult()
        s._check(s.L.plba_lba_plucker(s.ctx, C.byref(r)), "lba")
        t1 = time.perf_counter()
        rb = capi.ResultBuffers(g)
        t2 = time.perf_counter()
        s._check(s.L.plba_download(s.ctx, rb.struct.kf_Tcw, rb.struct.pt_xyz, rb.struct.ln_orth), "download")
        t3 = time.perf_counter()
        s._check(s.L.plba_download(s.ctx, rb.struct.kf_Tcw, rb.struct.pt_xyz, rb.struct.ln_orth), "download")
        t4 = time.perf_counter()
        s._check(s.L.plba_get_edge_chi2(s.ctx, rb.struct.ept_chi2, rb.struct.ept_depth_ok, rb.struct.eln_chi2), "chi2")
        t5 = time.perf_counter()
        s.reset()
        t6 = time.perf_counter()
        rb2 = capi.ResultBuffers(g)
        s._check(s.L.plba_lba_plucker(s.ctx, C.byref(rb2.struct)), "lba+out")
        t7 = time.perf_counter()
        print(f"{cfg}: lba {1e3*(t1-t0):.3f} (solve_ms {r.solve_ms:.3f}) | alloc {1e3*(t2-t1):.3f} | download (fresh "
              f"pages) {1e3*(t3-t2):.3f} | again {1e3*(t4-t3):.3f} | edge chi2 {1e3*(t5-t4):.3f} | lba with outputs "
              f"{1e3*(t7-t6):.3f} (solve_ms {rb2.struct.solve_ms:.3f})", flush=True)
