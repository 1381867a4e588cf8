"""Debug aid: per-workgroup balance of one sparse election round (libswarm_phases.so): the
slowest workgroups' durations and marked-agent loads against the median.
Usage: python tools/wg_balance.py N ROUND [ROUND ...]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import _lib  # noqa: E402

_lib.load(os.path.join(_lib.HERE, "libswarm_phases.so"))
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1])
d = gen.swarm_inputs(n, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
sw.elect()
L = _lib.lib()
L.swarm_debug_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
for R in map(int, sys.argv[2:]):
    out = np.zeros(8192 * 8, np.uint64)
    sw.elect(max_rounds=R)
    L.swarm_debug_phases(out.ctypes.data_as(ctypes.c_void_p), out.size)
    ph = out.reshape(8192, 8).astype(np.int64)[:2048]
    dur = (ph[:, 1] - ph[:, 0]) * 0.01  # 100 MHz clock -> us
    start = (ph[:, 0] - ph[:, 0].min()) * 0.01
    order = np.argsort(-dur)
    print(f"round {R}: wg dur us med {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}; "
          f"start spread {start.max():.1f} us; marked sum med {np.median(ph[:, 2]):.0f} max {ph[:, 2].max()}; "
          f"max chunk {ph[:, 3].max()}")
    t0 = ph[:, 0].min()
    ok = ph[:, 4] > 0
    if not ok.any():
        continue
    rel = lambda c: (ph[ok, c] - ph[ok, 0]) * 0.01  # noqa: E731
    print(f"   phases (from each wg's start, median / max): stamps in {np.median(rel(4)):.1f} / {rel(4).max():.1f}, "
          f"list done {np.median(rel(5)):.1f} / {rel(5).max():.1f}, gathered {np.median(rel(6)):.1f} / "
          f"{rel(6).max():.1f}, end {np.median(rel(1)):.1f} / {rel(1).max():.1f}; kernel span (first start -> last "
          f"end) {(ph[:, 1].max() - t0) * 0.01:.1f} us")
    for w in order[:5]:
        print(f"   wg {w}: dur {dur[w]:.1f} us start {start[w]:.1f} marked {ph[w, 2]} max chunk {ph[w, 3]}")
