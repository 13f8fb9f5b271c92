"""Diagnostics: per-workgroup phase timeline of the block-cyclic-reduction factorisation.

Runs one LBA of a config with PLBA_FACTOR=bcr and PLBA_DIAG=8 (timestamps on), then prints, for
the last factorisation launch, every super-row's phase times in µs from the earliest start."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
os.environ["PLBA_FACTOR"] = "bcr"
os.environ.setdefault("PLBA_DIAG", "8")
from plba import synth  # noqa: E402
from plba.lib import Solver  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
g = synth.generate(cfg)
s = Solver()
s.upload(g)
s.lba_plucker(want_outputs=False)
L = s.L
L.plba_debug_bcr_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int32, C.POINTER(C.c_int32)]
cap = 32 * 256
buf = (C.c_ulonglong * cap)()
rows = C.c_int32(0)
rc = L.plba_debug_bcr_stamps(s.ctx, buf, cap, C.byref(rows))
assert rc == 0, rc
N = rows.value
st = np.array(buf[: N * 32], dtype=np.float64).reshape(N, 32)
t0 = st[:, 0].min()
us = (st - t0) / 100.0  # 100 MHz
names = {0: "start", 1: "loaded", 12: "elim", 13: "pub", 14: "X", 15: "bwait", 16: "xpub", 17: "end"}
Lv = int(np.ceil(np.log2(N))) if N > 1 else 0
print(f"{cfg}: N = {N} super-rows, {Lv} levels; µs from first start")
for m in range(N):
    lm = Lv if m == 0 else (m & -m).bit_length() - 1
    row = [f"m={m:3d} l={lm}", f"start {us[m,0]:6.1f}", f"load {us[m,1]:6.1f}"]
    for lp in range(lm):
        row.append(f"s{lp} {us[m,2+lp]:6.1f}")
    steps = [us[m, 20 + k] for k in range(10) if st[m, 20 + k] >= t0]
    row.append(f"elim {us[m,12]:6.1f} (steps " + " ".join(f"{x:.1f}" for x in steps) + ")")
    for k in (13, 14, 15, 16, 17):
        if st[m, k] >= t0:
            row.append(f"{names[k]} {us[m,k]:6.1f}")
    print("  ".join(row))
s.close()
