"""Summarise a rocprofv3 kernel_trace.csv: per-kernel avg/min/total over the last N dispatches."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if tail:
    rows = rows[-tail:]
agg = defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"dispatches {len(rows)}  kernel-sum {tot:.1f} us  wall-span {span:.1f} us")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:58]:58s} n {len(v):5d} avg {sum(v)/len(v):8.2f} min {min(v):8.2f} tot {sum(v):9.1f} us {100*sum(v)/tot:5.1f}%")
