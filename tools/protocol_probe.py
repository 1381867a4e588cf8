"""Time the timer-FSM ticks (swarm_protocol_run) at bench scale on the GPU.

python tools/protocol_probe.py [--agents N] [--ticks T]: builds the bench's synthetic swarm
(deg 16 radius graph), phase-shifted agents, runs T ticks with two leader kills, prints ms/tick,
agent-ticks/s and the per-tick byte estimate.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--agents", type=int, default=10_000_000)
ap.add_argument("--ticks", type=int, default=200)
ap.add_argument("--deg", type=float, default=16.0)
a = ap.parse_args()
d = gen.swarm_inputs(a.agents, 3, deg=a.deg)
s = Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
off = (np.arange(a.agents) * 7919 % 40).astype(np.int32)
res = {}
for rep in range(2):
    s.protocol_reset(tick_off=off, last_hb=-(off * 0.1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c = s.protocol_run(a.ticks, kill_ticks=(80, 150), seed=5)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
# per-chunk timing (10 ticks per call) to separate quiet ticks from election storms
s.protocol_reset(tick_off=off, last_hb=-(off * 0.1))
chunks = []
for k in range(a.ticks // 10):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    cc = s.protocol_run(10, kill_ticks=(80, 150), seed=5)
    torch.cuda.synchronize()
    chunks.append((round(1e3 * (time.perf_counter() - t1) / 10, 4), int(cc[:, 1].sum()), int(cc[:, 2].sum()),
                   int(cc[:, 3].sum())))
print(json.dumps(dict(chunk_ms_per_tick_waits_acclaims_hbs=chunks)))
res = dict(agents=a.agents, edges=s.n_edges, ticks=a.ticks, ms_per_tick=1e3 * dt / a.ticks,
           agent_ticks_per_s=a.agents * a.ticks / dt,
           bytes_per_tick_est=a.agents * 26 + 5 * s.n_edges,
           leaders_final=int(c[-1, 0]), waits=int(c[:, 1].sum()), hb=int(c[:, 3].sum()))
res["gbs_est"] = res["bytes_per_tick_est"] / (res["ms_per_tick"] * 1e-3) / 1e9
print(json.dumps(res))
