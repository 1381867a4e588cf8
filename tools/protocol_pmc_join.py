"""Join rocprofv3 --pmc per-dispatch counters of k_tick (FETCH_SIZE and WRITE_SIZE passes of
tools/protocol_pmc.py) with the run's per-tick counts: HBM bytes per tick (FETCH_SIZE doubled for gfx950,
as tools/pmc_summary.py) by tick class.  Usage: python tools/protocol_pmc_join.py FETCH_DIR WRITE_DIR TICKS_JSON"""
import csv
import glob
import json
import os
import sys

import numpy as np


def per_dispatch(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and "k_tick" in r["Kernel_Name"] and "pull" not in r["Kernel_Name"]:
                rows.append((int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))), float(r["Counter_Value"])))
    rows.sort()
    return np.array([v for _, v in rows])


fe = per_dispatch(sys.argv[1], "FETCH_SIZE") * 2 * 1024
wr = per_dispatch(sys.argv[2], "WRITE_SIZE") * 1024
info = json.load(open(sys.argv[3]))
c = np.array(info["counts"])
T = len(c)
fe, wr = fe[-T:], wr[-T:]
tot = fe + wr
acc_prev = np.concatenate([[0], c[:-1, 2]])  # ACCLAIM senders of the previous tick: this tick's receivers
hb_prev = np.concatenate([[0], c[:-1, 3]])
storm = acc_prev > 0.005 * info["agents"]
quiet = (acc_prev == 0)
out = {"ticks": T, "hbm_MB_per_tick_mean": float(tot.mean() / 1e6),
       "fetch_MB_per_tick_mean": float(fe.mean() / 1e6), "write_MB_per_tick_mean": float(wr.mean() / 1e6),
       "quiet_ticks": int(quiet.sum()), "quiet_MB_mean": float(tot[quiet].mean() / 1e6) if quiet.any() else None,
       "quiet_fetch_MB_mean": float(fe[quiet].mean() / 1e6) if quiet.any() else None,
       "quiet_write_MB_mean": float(wr[quiet].mean() / 1e6) if quiet.any() else None,
       "storm_ticks": int(storm.sum()), "storm_MB_mean": float(tot[storm].mean() / 1e6) if storm.any() else None,
       "storm_MB_total": float(tot[storm].sum() / 1e6), "all_MB_total": float(tot.sum() / 1e6),
       "traffic": info["traffic"], "ms": info["ms"],
       "per_tick": [[int(i), round(float(fe[i] / 1e6), 2), round(float(wr[i] / 1e6), 2), int(acc_prev[i]),
                     int(hb_prev[i])] for i in range(T)]}
json.dump(out, sys.stdout, indent=1)
print()
