"""C4 probe: the auction at N agents x N tasks on cuda:0 (time, rounds, tail share).
Usage: python tools/auction_probe.py [N] [eps]"""
import sys
import time

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import torch  # noqa: E402
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
eps = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
d = gen.swarm_inputs(n, 2026, t=n)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0")
tx, ty, tq = (torch.as_tensor(d[k], device="cuda:0") for k in ("tx", "ty", "treq"))
r = s.auction(tx, ty, tq, eps=eps)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    r = s.auction(tx, ty, tq, eps=eps)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
a = r.assigned.cpu().numpy()
print(f"n={n} eps={eps}: {min(ts) * 1e3:.2f} ms, rounds {r.rounds_exec}, tail rounds {r.stats['tail_rounds']}, "
      f"pairs {r.stats['n_pairs']}, bids {r.stats['bids_total']}, assigned {(a >= 0).sum()}")
