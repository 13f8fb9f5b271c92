"""Phase times of k_lm_solve (diagnostic build libplba_lms.so, -DPLBA_LMS_STAMPS): per workgroup,
averaged over the launches of one LBA; thread 0's s_memtime view.
usage (GPU box): python tools/lms_stamps.py C3"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
from plba import lib, synth  # noqa: E402

lib.load(os.path.join(ROOT, "pl-slam-plucker_amd", "libplba_lms.so"))
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
g = synth.generate(cfg)
s = lib.Solver()
s.upload(g)
s.lba_plucker(want_outputs=False)
buf0 = (ctypes.c_ulonglong * (17 * 8))()
assert s.L.plba_debug_stamps(s.ctx, buf0) == 0
s.reset()
s.lba_plucker(want_outputs=False)
buf1 = (ctypes.c_ulonglong * (17 * 8))()
assert s.L.plba_debug_stamps(s.ctx, buf1) == 0
d = np.array(buf1[:], dtype=np.float64).reshape(17, 8)[15] - np.array(buf0[:], dtype=np.float64).reshape(17, 8)[15]
nwg, nlast = d[5], max(d[7], 1)
print(f"{cfg}: workgroups {nwg:.0f} over {nlast:.0f} launches ({nwg / nlast:.0f} per launch), units = s_memtime")
for i, name in enumerate(["loads + u (round trips 1-2)", "solve + oplus + eval", "block sums + partials", "arrive_last"]):
    print(f"  {name:30s} {d[i] / nwg:10.1f} per workgroup")
print(f"  {'workgroup lifetime':30s} {d[6] / nwg:10.1f}")
print(f"  {'decide tail (last workgroup)':30s} {d[4] / nlast:10.1f} per launch")
