"""Per-round overhead of the native sharded election loop on one GPU: swarm_elect_sharded on a
1-rank RCCL communicator (no halos) against swarm_elect(FRONTIER) on the same swarm.
python tools/sharded_probe.py [N]"""
import ctypes
import sys
import time

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from swarm_amd import _lib as L  # noqa: E402
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026)
s = Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
s.elect()
torch.cuda.synchronize()
t0 = time.perf_counter()
want = s.elect()
torch.cuda.synchronize()
t_single = time.perf_counter() - t0
uid = (ctypes.c_uint8 * 128)()
L.check(L.lib().swarm_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)))
comm = ctypes.c_void_p()
L.check(L.lib().swarm_comm_create(ctypes.byref(comm), 1, 0, ctypes.cast(uid, ctypes.c_void_p)))
l0 = torch.empty(n, dtype=torch.int32, device="cuda")
l1 = torch.empty(n, dtype=torch.int32, device="cuda")
desc = L.shard_desc(n, n, s.row_ptr, s.col, s.ids, 0, 1)
rounds = ctypes.c_int32(0)
ch = np.zeros(1 << 16, np.int64)
ts = []
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.check(L.lib().swarm_elect_sharded(L.ctx(), comm, ctypes.byref(desc), L.ptr(l0), L.ptr(l1), len(ch),
                                        ctypes.byref(rounds), ch.ctypes.data_as(ctypes.c_void_p), L.stream()))
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
assert rounds.value == want.rounds_exec
print(f"n={n} rounds={want.rounds_exec} single-GPU elect {t_single * 1e3:.2f} ms; sharded loop (1 rank) "
      f"{min(ts) * 1e3:.2f} ms -> {(min(ts) - t_single) / want.rounds_exec * 1e6:.1f} us/round of loop overhead")
L.lib().swarm_comm_destroy(comm)
