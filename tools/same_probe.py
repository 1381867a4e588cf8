"""Which part of bench.py's cpu_baseline 'same_result_as_gpu' check differs (rounds, leaders,
winners, util bits), on the bench's C3 inputs after the bench's own sequence of calls.
Usage: python tools/same_probe.py [N]"""
import sys

sys.path.insert(0, "distributed-swarm-algorithm_amd")
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from swarm_amd import _lib, gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402
from oracle import oracle  # noqa: E402

_lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, deg=16.0, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
dev = sw.device
tx, ty, tq = (torch.as_tensor(d[k], device=dev) for k in ("tx", "ty", "treq"))
for _ in range(3):
    r = sw.elect(max_rounds=1 << 16)
    a = sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
rp = sw.row_ptr.cpu().numpy().astype(np.int64)
col = sw.col.cpu().numpy()
ids = sw.ids.cpu().numpy()
x, y = sw.pos[:, 0].cpu().numpy(), sw.pos[:, 1].cpu().numpy()
caps = sw.caps.cpu().numpy().view(np.uint32)
oracle.set_threads(16)
lead, _, rounds, _ = oracle.elect_frontier(rp, col, ids)
al = oracle.allocate_binned(ids, x, y, caps, d["tx"], d["ty"], d["treq"], use_pow=False)
gl = sw.leader.cpu().numpy()
print("rounds", rounds, r.rounds_exec, "leaders equal", np.array_equal(lead, gl), "r.leader is sw.leader",
      r.leader.data_ptr() == sw.leader.data_ptr(), "n diff", int((lead != gl).sum()))
gw = a.winner.cpu().numpy()
print("winners equal", np.array_equal(al["winner"], gw), "n diff", int((al["winner"] != gw).sum()),
      "dtypes", al["winner"].dtype, gw.dtype, "shapes", al["winner"].shape, gw.shape)
print("util bits equal", np.array_equal(al["util"].view(np.uint64), a.util.cpu().numpy().view(np.uint64)))
