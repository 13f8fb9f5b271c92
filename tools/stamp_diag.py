"""Per-phase cycle breakdown of k_rcs_factor_band from the PLBA_STAMPS diagnostic build."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
import numpy as np  # noqa: E402

from plba import lib, synth  # noqa: E402

lib.load(os.path.join(ROOT, "pl-slam-plucker_amd", os.environ.get("PLBA_STAMPS_LIB", "libplba_stamps.so")))
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
s = lib.Solver()
g = synth.generate(cfg)
s.upload(g)
out = s.lba_plucker(want_outputs=False)
buf = (C.c_ulonglong * 136)()
rc = s.L.plba_debug_stamps(s.ctx, buf)
a = np.array(buf[:], dtype=np.float64).reshape(17, 8)
names = ["top(prefetch)", "phase1", "bar1", "ph2-end(refill|crit)", "bar2", "ph2-pairs", "ph2-b", "ph2-flush"]
ntr = int(sum(t["trials"] for t in out["trace"]))
nf = int((g.kf_fixed == 0).sum())
st = s.structure_stats()
steps_per_trial = (nf - st["bw"] + 1) // 2 if st["twisted"] else nf
print(cfg, "rc", rc, "trials", ntr, "forward steps per trial", steps_per_trial, "twisted", st["twisted"])
if st.get("column_lane"):
    names = ["A:publish", "B:gauss-jordan", "C:publish-X", "barrier", "EF:next-column", "prefetch",
             "w:rhs", "w:flush"]
    wnames = ["-", "-", "-", "barrier", "w:rowload", "w:pairs", "w:rhs", "w:flush"]
for w in range(16):
    if a[w].sum() == 0:
        continue
    per = a[w] / (ntr * steps_per_trial)
    nm = wnames if st.get("column_lane") and w > 0 else names
    print(f"wave {w:2d} cycles/step: " + " ".join(f"{n}={v:.0f}" for n, v in zip(nm, per) if n != "-"),
          f"total={per.sum():.0f}")

tw = a[16]
if st.get("column_lane") and st["twisted"]:
    n = ntr
    print(f"column-lane twisted (per launch): fwd seg0 {tw[0]/n:.0f} fwd seg1 {tw[1]/n:.0f} wait+merge {tw[2]/n:.0f} "
          f"separator steps {tw[3]/n:.0f} backward {tw[4]/n:.0f}")
elif tw[4] > 0:
    n = tw[4]
    print(f"twisted (per launch, s_memtime/readcyclecounter units): fwd seg0 {tw[0]/n:.0f} fwd seg1 {tw[1]/n:.0f} "
          f"handoff+separator {tw[2]/n:.0f} (of which hand-off + assembly {tw[5]/n:.0f}) backward {tw[3]/n:.0f}")
