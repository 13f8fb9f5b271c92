"""GPU box: a 1-rank RCCL-sharded window — is the step graph captured (graph flag), and what does
one LBA cost against the unsharded solve of the same window."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
from plba import synth  # noqa: E402
from plba.lib import Solver, comm_unique_id  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
g = synth.generate(cfg)
for mode in ("unsharded", "rccl-1"):
    s = Solver(device=0)
    if mode != "unsharded":
        s.comm_init_rccl(1, 0, comm_unique_id())
    s.upload(g)
    for k in range(4):
        s.reset()
        t = time.perf_counter()
        out = s.lba_plucker(want_outputs=False)
        ms = (time.perf_counter() - t) * 1e3
    print(mode, cfg, "graph", s.structure_stats()["graph"], "ms/LBA", round(ms, 2), flush=True)
    s.close()
