"""Debug aid: per-wave phase timestamps of one sparse election round (libswarm_phases.so,
built with -DSWARM_PHASES: make -C distributed-swarm-algorithm_amd/csrc phases).
Usage: python tools/phase_probe.py N ROUND [ROUND ...]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import torch  # noqa: E402
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
    L.swarm_debug_phases(out.ctypes.data_as(ctypes.c_void_p), out.size)  # clear via read
    sw.elect(max_rounds=R)
    out[:] = 0
    L.swarm_debug_phases(out.ctypes.data_as(ctypes.c_void_p), out.size)
    ph = out.reshape(8192, 8).astype(np.int64)
    ph = ph[ph[:, 0] > 0]
    t0 = ph[:, 0].min()
    rel = (ph - t0) / 100.0  # wall_clock64: 100 MHz -> us
    busy = (ph[:, 2] >= ph[:, 0]) & (ph[:, 3] >= ph[:, 2])
    print(f"round {R}: waves {len(ph)}, with marked agents {busy.sum()}")
    for k in (1, 4):
        c = rel[:, k]
        print(f"  P{k}: med {np.median(c):7.2f}  p90 {np.percentile(c, 90):7.2f}  max {c.max():7.2f} us")
    if busy.any():
        b = rel[busy]
        for a_, c_ in [(1, 2), (2, 3), (3, 4)]:
            dl = b[:, c_] - b[:, a_]
            print(f"  busy P{a_}->P{c_}: med {np.median(dl):6.2f}  p90 {np.percentile(dl, 90):6.2f}  max {dl.max():6.2f}")
        print(f"  busy end P4: med {np.median(b[:, 4]):6.2f} max {b[:, 4].max():6.2f}")
