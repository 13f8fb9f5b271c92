"""GPU box, diagnostics: phase timestamps (s_memrealtime, 100 MHz) of one dense panel and one
trailing-update launch (K = 5, workgroup 0) on a wide-envelope window (PLBA_DIAG=8)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
os.environ["PLBA_DIAG"] = "8"
import numpy as np  # noqa: E402
from plba import synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

g = synth.generate(sys.argv[1] if len(sys.argv) > 1 else "C3R")
s = Solver()
s.upload(g)
s.lba_plucker(want_outputs=False)
L = s.L
L.plba_debug_bcr_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int32, C.POINTER(C.c_int32)]
buf = (C.c_ulonglong * 32)()
rows = C.c_int32(0)
assert L.plba_debug_bcr_stamps(s.ctx, buf, 32, C.byref(rows)) == 0
st = np.array(buf[:], dtype=np.float64)
p = (st[:7] - st[0]) / 100.0
u = (st[8:11] - st[8]) / 100.0
print("panel  us (from after the guard): solve_ok read %.2f loads-issued %.2f diag-LDLT %.2f L-scale %.2f TRSM %.2f stores %.2f" % tuple(p[1:7]))
print("update us: staged %.2f mfma %.2f" % tuple(u[1:3]))
v = (st[12:16] - st[12]) / 100.0
print("solve  us: forward %.2f backward %.2f pose-update %.2f" % (v[1], v[2] - v[1], v[3] - v[2]))
w = (st[16:20] - st[16]) / 100.0
print("forward tile K=5 us: wave0 chain done %.2f first barrier %.2f second barrier %.2f" % tuple(w[1:4]))
s.close()
