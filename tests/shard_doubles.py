"""Test doubles for the sharded driver (swarm_amd/dist.py).

NumpyBackend restates the frontier stepper (swarm_frontier_begin/step/ghosts/changes) and the
allocation with the oracle, on CPU tensors, so the partitioning / halo / convergence logic of
ShardedSwarm runs under gloo without a GPU.  ThreadHalo lets two shards live in one process
(two threads, one GPU) so the GPU test can exercise the real stepper kernels with ghosts.
Test infrastructure only.
"""
import queue
import threading

import numpy as np
import torch


class NumpyBackend:
    def __init__(self):
        self.device = torch.device("cpu")

    def cell_order(self, pos):
        from swarm_amd import gen
        p = pos.numpy()
        return torch.as_tensor(gen.cell_order(p[:, 0], p[:, 1], 1.0), dtype=torch.long)

    def build_graph(self, pos, radius):
        from oracle import oracle
        p = pos.numpy()
        rp, col = oracle.rgg_csr(p[:, 0], p[:, 1], radius)
        return torch.as_tensor(rp), torch.as_tensor(col)

    # leaders: two buffers, round t reads [(t-1)&1] and writes [t&1] (swarm_frontier_* contract)
    def begin(self, n_rows, init, leaders):
        leaders[0].copy_(init)
        leaders[1].copy_(init)
        self.n_rows = n_rows
        self.act = np.ones(init.numel(), np.int64)
        self.counts = {}

    def step(self, t, rp, col, leaders):
        Lr, Lw = leaders[(t - 1) & 1].numpy(), leaders[t & 1].numpy()
        rp_, col_ = rp.numpy(), col.numpy()
        Lw[: self.n_rows] = Lr[: self.n_rows]
        act = np.nonzero(self.act[: self.n_rows] == t)[0]
        changed = []
        for v in act:
            nb = col_[rp_[v]:rp_[v + 1]]
            m = Lr[nb].max() if len(nb) else Lr[v]
            if m > Lr[v]:
                changed.append((v, m))
        for v, m in changed:
            Lw[v] = m
            self.act[col_[rp_[v]:rp_[v + 1]]] = t + 1
        self.counts[t] = len(changed)

    def ghosts(self, t, begin, incoming, rp, col, leaders):
        cur = leaders[t & 1].numpy()
        rp_, col_ = rp.numpy(), col.numpy()
        for i, nv in enumerate(incoming.numpy()):
            g = begin + i
            if nv > cur[g]:
                leaders[0].numpy()[g] = nv
                leaders[1].numpy()[g] = nv
                self.act[col_[rp_[g]:rp_[g + 1]]] = t + 1

    def changes(self, t0, t1):
        return np.array([self.counts.get(t, 0) for t in range(t0, t1 + 1)], np.int64)

    def allocate(self, ids, pos, caps, tx, ty, treq, claim_thr=20.0, hysteresis=5.0, u_scale=100.0, mode="auto"):
        from oracle import oracle
        p = pos.numpy()
        r = oracle.allocate(ids.numpy(), p[:, 0], p[:, 1], caps.numpy().view(np.uint32), np.asarray(tx),
                            np.asarray(ty), np.asarray(treq), claim_thr=claim_thr, hysteresis=hysteresis,
                            u_scale=u_scale)

        class R:
            pass
        out = R()
        out.winner = torch.as_tensor(r["winner"])
        out.util = torch.as_tensor(r["util"])
        out.won = torch.as_tensor(r["won"])
        out.stats = dict(n_claims=r["n_claims"], n_conflicts=r["n_conflicts"], n_flagged=0,
                         n_candidates=len(ids) * len(tx), n_overflow=0)
        return out


class ThreadHalo:
    """In-process strip chain for shards driven by threads (one per shard)."""

    def __init__(self, world):
        self.world = world
        self.q = {(a, b): queue.Queue() for a in range(world) for b in range(world)}
        self.barrier = threading.Barrier(world)
        self.sums = {}
        self.lock = threading.Lock()

    def member(self, rank):
        hub = self

        class Member:
            group = None
            world = hub.world
            host_staged = True  # no RCCL communicator behind an in-process halo

            def __init__(self):
                self.rank = rank
                self.lo = rank - 1 if rank > 0 else None
                self.hi = rank + 1 if rank < hub.world - 1 else None

            def exchange(self, to_lo, to_hi, n_from_lo, n_from_hi, like):
                if self.lo is not None:
                    hub.q[(rank, self.lo)].put(to_lo.clone())
                if self.hi is not None:
                    hub.q[(rank, self.hi)].put(to_hi.clone())
                a = hub.q[(self.lo, rank)].get() if self.lo is not None else like[:0].clone()
                b = hub.q[(self.hi, rank)].get() if self.hi is not None else like[:0].clone()
                assert a.shape[0] == n_from_lo and b.shape[0] == n_from_hi
                return a, b

            def exchange_counts(self, n_to_lo, n_to_hi):
                t = torch.tensor([n_to_lo]), torch.tensor([n_to_hi])
                a, b = self.exchange(t[0], t[1], 1 if self.lo is not None else 0, 1 if self.hi is not None else 0, t[0])
                return (int(a[0]) if a.numel() else 0), (int(b[0]) if b.numel() else 0)

            def all_reduce_sum(self, arr):
                arr = np.asarray(arr)
                key = id(hub)
                with hub.lock:
                    hub.sums.setdefault("acc", []).append(arr)
                hub.barrier.wait()
                total = np.sum(hub.sums["acc"], axis=0)
                hub.barrier.wait()
                with hub.lock:
                    hub.sums.pop("acc", None)
                hub.barrier.wait()
                del key
                return total

        return Member()
