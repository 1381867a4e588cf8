"""One 10M-agent frontier election (after one warm-up) for counter collection:
rocprofv3 --pmc ... -- python tools/elect_once.py [N]"""
import sys

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import torch  # noqa: E402
from swarm_amd import _lib, gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

_lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
r = sw.elect()
r = sw.elect()
torch.cuda.synchronize()
print("rounds", r.rounds_exec, "launched", r.rounds_launched)
