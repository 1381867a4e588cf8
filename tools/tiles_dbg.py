"""One C3 election with the tiled tail and SWARM_TILE_DEBUG phase clocks (printed by libswarm)."""
import os
import sys

import torch

os.environ.setdefault("SWARM_TILE_DEBUG", "1")
sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, deg=16.0)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
r = s.elect(tiles=sys.argv[2] if len(sys.argv) > 2 else True)
torch.cuda.synchronize()
print(r.rounds_exec, r.tile_from, r.tile_rounds, r.tile_launches, flush=True)
