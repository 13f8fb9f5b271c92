"""Gaps between consecutive kernels of the step graph (rocprofv3 kernel trace): how long the
device sits between the factorisation's end and the landmark solve's start, per step.
usage: python tools/trace_gaps.py <kernel_trace.csv>"""
import csv
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("plba::", "").split("<")[0]
pairs = {}
for a, b in zip(rows, rows[1:]):
    key = (short(a["Kernel_Name"]), short(b["Kernel_Name"]))
    gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if 0 <= gap < 50:
        pairs.setdefault(key, []).append(gap)
for k, v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:14]:
    print(f"{k[0]:28s} -> {k[1]:28s} n {len(v):5d} median gap {st.median(v):6.2f} us  mean {st.mean(v):6.2f}")
