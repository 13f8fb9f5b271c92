"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<cfg>.json.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports both in KiB,
and on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream
(MI355X_MICROARCH.md §HBM) - our kernels mostly issue 8-byte accesses, for which the guide
calls the absolute uncalibrated, so raw values are kept beside the corrected estimate.
Infinity-Cache (256 MiB) hits are counted too: at C3 the working set is L3-resident.
Usage: python tools/pmc_summary.py <prof_dir> <cfg> [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "").replace("plba::", "")
        short = short.split("<")[0]
        acc[short].append(float(r["Counter_Value"]))
    return acc


def main():
    d, cfg = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join("profiles", f"pmc_{cfg}.json")
    f = load(os.path.join(d, "fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
    w = load(os.path.join(d, "write", "bench_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk = sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wk = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        res[k] = dict(fetch_kib_raw=fk, write_kib=wk, launches=len(f.get(k, [])),
                      hbm_bytes_per_launch=(2 * fk + wk) * 1024)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]):
        print(f"{k:28s} launches {v['launches']:5d} fetch {v['fetch_kib_raw']:10.1f} KiB write {v['write_kib']:10.1f} KiB "
              f"-> {v['hbm_bytes_per_launch']/1e6:8.3f} MB/launch")


if __name__ == "__main__":
    main()
