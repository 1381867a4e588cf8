"""Per-tick HBM traffic of the protocol ticks (f2): the bench's 200-tick scenario of the C3 swarm (10M
agents, leader kills at ticks 80 and 150, hybrid mode) in one swarm_protocol_run call, meant to run under
rocprofv3 --pmc (one counter per pass).  Writes the per-tick counts (leaders, waits, ACCLAIM senders,
HEARTBEAT senders) and the run's traffic counters to gpurun_out/protocol_ticks_<tag>.json;
tools/protocol_pmc_join.py pairs them with the per-dispatch counters of k_tick.
Usage: python tools/protocol_pmc.py TAG"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
sys.path.insert(0, ".")
import os  # noqa: E402

from swarm_amd import _lib, gen  # noqa: E402
if os.environ.get("PROTO_LIB"):  # A/B builds under swarm_amd/
    _lib.load(os.path.join(_lib.HERE, os.environ["PROTO_LIB"]))
from swarm_amd.swarm import Swarm  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "p"
d = gen.swarm_inputs(10_000_000, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
n = sw.n
off = (np.arange(n, dtype=np.int64) * 7919 % 40).astype(np.int32)
ticks = 200
sw.protocol_reset(tick_off=off, last_hb=-(off * 0.1))
torch.cuda.synchronize()
t0 = time.perf_counter()
c = sw.protocol_run(ticks, kill_ticks=(80, 150), seed=5, traffic=True)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3
out = {"agents": n, "ticks": ticks, "ms": ms, "counts": c.tolist(), "traffic": [int(v) for v in sw.fsm_traffic]}
json.dump(out, open(f"gpurun_out/protocol_ticks_{tag}.json", "w"))
print(json.dumps({k: out[k] for k in ("agents", "ticks", "ms", "traffic")}), flush=True)
