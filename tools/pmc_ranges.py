"""Per-round-range hardware counters of the last election in rocprofv3 --pmc CSVs
(tools/pmc_passes_elect.sh): rounds = k_elect_dense / k_sparse_block dispatches in order.
Usage: python tools/pmc_ranges.py RUN_COUNTER_COLLECTION.csv [...]"""
import csv
import sys
from collections import defaultdict

import numpy as np

RANGES = [(1, 8), (9, 99), (100, 399), (400, 906), (907, 1364), (1365, 99999)]
per = defaultdict(dict)  # counter -> {range: values}
for path in sys.argv[1:]:
    disp = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "k_elect_dense" not in k and "k_sparse_block" not in k:
            continue
        d = int(r["Dispatch_Id"])
        disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = k
    ids = sorted(disp)
    # the last election: from the last dense dispatch that follows a sparse one (or the first)
    starts = [i for i, d in enumerate(ids) if "k_elect_dense" in names[d] and (i == 0 or "k_elect_dense" not in names[ids[i - 1]])]
    el = ids[starts[-1]:]
    for rnd, d in enumerate(el, 1):
        for lo, hi in RANGES:
            if lo <= rnd <= hi:
                for c, v in disp[d].items():
                    per[c].setdefault((lo, hi), []).append(v)
for c in sorted(per):
    print(c, "  ".join(f"{lo}-{hi}: {np.mean(v):.4g}" for (lo, hi), v in sorted(per[c].items())))
