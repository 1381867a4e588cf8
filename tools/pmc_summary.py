"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), corrected as
MI355X_MICROARCH.md's HBM section prescribes: gfx950 FETCH_SIZE counts 64 B per 128-B request,
so it is doubled; WRITE_SIZE is taken as reported.  Values are KB per dispatch in the CSVs.
Usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR > pmc_traffic.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][-48:]


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    if not k.startswith("k_"):
        continue
    f, w = fetch.get(k, []), write.get(k, [])
    fm = sum(f) / len(f) if f else 0.0
    wm = sum(w) / len(w) if w else 0.0
    out[k] = {"dispatches": max(len(f), len(w)), "FETCH_SIZE_KB_mean": fm, "WRITE_SIZE_KB_mean": wm,
              "FETCH_SIZE_KB_sum": sum(f), "WRITE_SIZE_KB_sum": sum(w),
              "hbm_bytes_per_dispatch": (2.0 * fm + wm) * 1024.0}
out["_note"] = ("rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; hbm_bytes = (2 x FETCH_SIZE + "
                "WRITE_SIZE) KB x 1024 (gfx950 FETCH_SIZE counts 64 B per 128-B request); Infinity-Cache hits "
                "are included in FETCH_SIZE.  Workload: bench.py --steps 1 --warmup 0 (C3, 10M agents).")
json.dump(out, sys.stdout, indent=1)
print()
