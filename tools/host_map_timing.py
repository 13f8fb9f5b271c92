"""Per-call cost of the host mirror's LBA on a C3 window inside a C5-sized map:
gather / upload / solve / write-back, incremental gather vs the reference's map scan.
usage: python tools/host_map_timing.py [calls]   (PLSLAM_THREADS, PLBA_TIMING honoured)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))
import bench  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
r = bench.host_mirror("C3", 0, calls=calls, background=(900, 180000, 36000), scan_calls=calls)
r.pop("note", None)
print(json.dumps(r), flush=True)
