"""Per-tick time of the protocol ticks (f2) by tick class: the k_tick dispatch durations of a rocprofv3
--kernel-trace run of tools/protocol_pmc.py, paired in order with the run's per-tick counts (the classes
of tools/protocol_pmc_join.py: quiet = no ACCLAIM sender the tick before, storm = more than 0.5 % of the
agents, ordinary = the rest).  Usage: python tools/protocol_time_join.py TRACE_DIR TICKS_JSON"""
import csv
import glob
import json
import os
import sys

import numpy as np

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_tick" in r["Kernel_Name"] and "pull" not in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
rows.sort()
info = json.load(open(sys.argv[2]))
c = np.array(info["counts"])
T = len(c)
us = np.array([d for _, d in rows][-T:]) / 1e3
acc_prev = np.concatenate([[0], c[:-1, 2]])
storm = acc_prev > 0.005 * info["agents"]
quiet = acc_prev == 0
ordinary = ~storm & ~quiet
out = {"ticks": T, "k_tick_ms_total": float(us.sum() / 1e3), "wall_ms": info["ms"]}
for name, m in (("quiet", quiet), ("ordinary", ordinary), ("storm", storm)):
    out[name] = {"ticks": int(m.sum()), "ms_total": float(us[m].sum() / 1e3),
                 "us_median": float(np.median(us[m])) if m.any() else None,
                 "us_max": float(us[m].max()) if m.any() else None}
out["per_tick_us"] = [round(float(v), 1) for v in us]
json.dump(out, sys.stdout, indent=1)
print()
