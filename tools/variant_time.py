"""A/B timing of libplba builds (run on the GPU box): per-kernel µs and LBA ms for each library.

usage: python tools/variant_time.py C3 libplba.so libplba_p8.so ...
Each library runs in its own child process (one HIP library per process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pl-slam-plucker_amd")


def child(cfg: str, libname: str):
    sys.path.insert(0, PKG)
    import numpy as np
    from plba import lib, synth
    lib.load(os.path.join(PKG, libname))
    g = synth.generate(cfg)
    s = lib.Solver()
    s.upload(g)
    ms = []
    for _ in range(6):
        s.reset()
        r = s.lba_plucker(want_outputs=False)
        ms.append(r["solve_ms"])
    s.close()
    t = lib.Solver(kernel_timing=True)
    t.upload(g)
    t.lba_plucker(want_outputs=False)
    t.reset()
    t.lba_plucker(want_outputs=False)
    kt = t.kernel_times()
    print(json.dumps({"lib": libname, "lba_ms_median": float(np.median(ms[1:])),
                      "chi2": [float(x) for x in r.get("chi2", [])],
                      "kernels_us": {k: round(1e3 * v[0] / max(v[1], 1), 2) for k, v in kt.items()}}))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        sys.exit(0)
    cfg = sys.argv[1]
    for libname in sys.argv[2:]:
        r = subprocess.run([sys.executable, __file__, "--child", cfg, libname], capture_output=True, text=True,
                           timeout=300)
        print(r.stdout.strip() or r.stderr[-2000:], flush=True)
