"""HIP API calls and kernels of the last Swarm.allocate call in a rocprofv3 --hip-trace
--kernel-trace run of tools/alloc_host_probe.py: one timeline, offsets from the first API call.
Usage: python tools/alloc_api_trace.py DIR"""
import csv
import glob
import sys

d = sys.argv[1]
api = list(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])))
ker = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
fn = "Function" if "Function" in api[0] else ("Operation" if "Operation" in api[0] else list(api[0])[0])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API " + r[fn]) for r in api]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU " + r["Kernel_Name"][:110]) for r in ker]
ev.sort()
# the last k_alloc_binned and everything from the torch fill kernel launch before it
ia = max(i for i, e in enumerate(ev) if "k_alloc_binned" in e[2])
i0 = ia
fills = 0
while i0 > 0 and fills < 2:
    i0 -= 1
    if ev[i0][2].startswith("GPU") and "FillFunc" in ev[i0][2]:
        fills += 1
while i0 > 0 and not (ev[i0][2].startswith("API") and "Launch" in ev[i0][2]):
    i0 -= 1
i1 = ia
while i1 < len(ev) - 1 and "hipStreamSynchronize" not in ev[i1][2]:
    i1 += 1
t0 = ev[i0][0]
for a, b, nm in ev[max(0, i0 - 3):i1 + 3]:
    print(f"+{(a - t0) / 1e3:8.1f}  {(b - a) / 1e3:7.1f} us  {nm}")
