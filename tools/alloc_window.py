"""Kernels of the allocation call(s) in a rocprofv3 kernel trace of bench.py: everything from the
election's k_state to k_alloc_binned (or its stats fold), with device time and start offsets.
Usage: python tools/alloc_window.py TRACE.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]) for r in rows)
ia = [i for i, k in enumerate(ks) if "k_alloc_binned" in k[2]]
for j in ia[-2:]:
    i0 = j
    while i0 > 0 and "k_state" not in ks[i0][2]:
        i0 -= 1
    j1 = j  # the allocation kernel, or the stats fold right after it (the deferred path)
    if j1 + 1 < len(ks) and "k_fold_stats" in ks[j1 + 1][2]:
        j1 += 1
    dev = sum(b - a for a, b, _ in ks[i0 + 1:j1 + 1]) / 1e3
    print(f"--- k_state end -> allocation end: {(ks[j1][1] - ks[i0][1]) / 1e3:.1f} us, device {dev:.1f} us")
    for a, b, nm in ks[i0 + 1:j1 + 2]:
        print(f"{(b - a) / 1e3:8.1f} us  +{(a - ks[i0][1]) / 1e3:8.1f}  {nm}")
