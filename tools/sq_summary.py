"""Summarise rocprofv3 SQ / GRBM counter passes (tools/profile_round.sh) per kernel.

Per launch (averaged over launches): waves launched (SQ_WAVES), SQ busy cycles, resident
wave-cycles, the mean number of resident waves while the SQs were busy
(SQ_WAVE_CYCLES / SQ_BUSY_CYCLES, summed over the chip's SQs), VALU / LDS / VMEM instructions,
LDS bank conflicts, and GRBM_GUI_ACTIVE (GPU-busy cycles of the launch).
Usage: python tools/sq_summary.py <prof_dir> [out.txt]"""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return acc
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("plba::", "").split("<")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    d = sys.argv[1]
    flat = os.path.join(d, "pmc_counter_collection.csv")  # (tools/pmc_sq.sh: one pass, no GRBM)
    if os.path.exists(flat):
        sq, gr = load(flat), {}
    else:
        sq = load(os.path.join(d, "sq", "bench_counter_collection.csv"))
        gr = load(os.path.join(d, "grbm", "bench_counter_collection.csv"))
    lines = ["kernel                      launches  waves  busy_cyc  wave_cyc  waves/busy  VALU/launch  LDS/launch  VMEM/launch  LDS_conf  GUI_active"]
    def avg(dct, c):
        v = dct.get(c, [])
        return sum(v) / len(v) if v else 0.0
    for k in sorted(sq, key=lambda k: -avg(sq[k], "SQ_BUSY_CYCLES") * len(sq[k].get("SQ_WAVES", []))):
        s = sq[k]
        n = len(s.get("SQ_WAVES", []))
        busy, wc = avg(s, "SQ_BUSY_CYCLES"), avg(s, "SQ_WAVE_CYCLES")
        lines.append(f"{k[:27]:27s} {n:8d} {avg(s,'SQ_WAVES'):6.0f} {busy:9.0f} {wc:9.0f} {wc/max(busy,1):10.2f} "
                     f"{avg(s,'SQ_INSTS_VALU'):12.0f} {avg(s,'SQ_INSTS_LDS'):11.0f} {avg(s,'SQ_INSTS_VMEM'):12.0f} "
                     f"{avg(s,'SQ_LDS_BANK_CONFLICT'):9.0f} {avg(gr.get(k, {}), 'GRBM_GUI_ACTIVE'):11.0f}")
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
