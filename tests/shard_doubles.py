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
    def begin(self, own_begin, n_own, init, leaders, col16=None):
        leaders[0].copy_(init)
        leaders[1].copy_(init)
        self.own = (own_begin, own_begin + n_own)
        self.act = np.ones(init.numel(), np.int64)
        self.counts = {}

    def step(self, t, rp, col, leaders):
        # every row steps (ghost rows too: deep halos); only the owned rows count
        Lr, Lw = leaders[(t - 1) & 1].numpy(), leaders[t & 1].numpy()
        rp_, col_ = rp.numpy(), col.numpy()
        Lw[:] = Lr
        act = np.nonzero(self.act == t)[0]
        changed = []
        for v in act:
            nb = col_[rp_[v]:rp_[v + 1]]
            m = Lr[nb].max() if len(nb) else Lr[v]
            if m > Lr[v]:
                changed.append((v, m))
        for v, m in changed:
            Lw[v] = m
            self.act[v] = t + 1
            self.act[col_[rp_[v]:rp_[v + 1]]] = t + 1
        self.counts[t] = sum(1 for v, _ in changed if self.own[0] <= v < self.own[1])

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
        out.nmsg = torch.as_tensor(r["nmsg"])
        out.nclaim = torch.as_tensor(r["nclaim"])
        out.stats = dict(n_claims=r["n_claims"], n_conflicts=r["n_conflicts"], n_flagged=0,
                         n_candidates=len(ids) * len(tx), n_overflow=0, n_resolved=0)
        return out


    # ---- sharded auction, restated (the per-round contract of swarm_auction_begin/_bid/_resolve)
    def auction_begin(self, ids, pos, caps, tx, ty, treq, claim_thr, u_scale, eps):
        import math
        p = pos.numpy()
        tx_, ty_, tq = tx.numpy(), ty.numpy(), treq.numpy()
        cp = caps.numpy().view(np.uint32)
        cand = []
        for a in range(ids.numel()):
            row = []
            for k in range(len(tx_)):
                dx, dy = float(p[a, 0]) - float(tx_[k]), float(p[a, 1]) - float(ty_[k])
                d = math.sqrt(dx * dx + dy * dy)
                has = 0.0 if (int(tq[k]) >= 0 and not (int(cp[a]) >> int(tq[k])) & 1) else 1.0
                U = (u_scale / (1.0 + d)) * has
                if U > claim_thr:
                    row.append((k, np.float32(U)))
            cand.append(row)
        t = len(tx_)
        return dict(cand=cand, ids=ids.numpy().astype(np.int64), eps=np.float32(eps),
                    index={int(v): i for i, v in enumerate(ids.numpy())},
                    out=np.zeros(ids.numel(), bool), owner_id=torch.full((t,), -1, dtype=torch.int32),
                    price=torch.zeros(t, dtype=torch.float32), assigned=torch.full((ids.numel(),), -1, dtype=torch.int32),
                    stats=dict(n_pairs=sum(len(c) for c in cand), n_flagged=0))

    def auction_bid(self, r, rank, world, keys, st):
        f = np.float32
        price, assigned, kv = st["price"].numpy(), st["assigned"].numpy(), keys.numpy()
        t = price.size
        nb = 0
        for a, row in enumerate(st["cand"]):
            if assigned[a] >= 0 or st["out"][a]:
                continue
            nb += 1
            best, second, bk = f(-np.inf), f(-np.inf), None
            for k, x in row:
                net = f(x - price[k])
                if net > best or (net == best and k < bk):
                    second, best, bk = max(second, best), net, k
                elif net > second:
                    second = net
            if not best > 0:
                st["out"][a] = True
                continue
            second = max(second, f(0.0))
            bid = f(f(price[bk] + f(best - second)) + st["eps"])
            key = (int(np.array(bid, np.float32).view(np.uint32)) << 32) | (0xFFFFFFFF - int(st["ids"][a]))
            kv[bk] = max(int(kv[bk]), key)
        kv[t + rank] = nb

    def auction_resolve(self, r, world, keys, st, log):
        kv, owner, price, assigned = keys.numpy(), st["owner_id"].numpy(), st["price"].numpy(), st["assigned"].numpy()
        t = price.size
        for k in np.nonzero(kv[:t])[0]:
            key = int(kv[k])
            w = 0xFFFFFFFF - (key & 0xFFFFFFFF)
            prev = int(owner[k])
            if prev >= 0 and prev in st["index"]:
                assigned[st["index"][prev]] = -1
            owner[k] = w
            if w in st["index"]:
                assigned[st["index"][w]] = k
            price[k] = np.array([key >> 32], np.uint32).view(np.float32)[0]
            kv[k] = 0
        log.numpy()[r] = int(kv[t:t + world].sum())
        kv[t:t + world] = 0


class ThreadHalo:
    """In-process point-to-point hub for shards driven by threads (one per shard)."""

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

            def exchange_peers(self, sends, recv_counts, like):
                for p, t in sends.items():
                    if t.numel():  # an empty message is never sent (the receiver expects 0 rows)
                        hub.q[(rank, p)].put(t.clone())
                out = {}
                for p, n in recv_counts.items():
                    got = hub.q[(p, rank)].get() if n else like[:0].clone()
                    assert got.shape[0] == n
                    out[p] = got
                return out

            def _gather(self, key, arr):
                with hub.lock:
                    hub.sums.setdefault(key, {})[rank] = arr
                hub.barrier.wait()
                vals = [hub.sums[key][r] for r in range(hub.world)]
                hub.barrier.wait()
                with hub.lock:
                    hub.sums.pop(key, None)
                hub.barrier.wait()
                return vals

            def count_matrix(self, counts):
                return np.stack(self._gather("counts", np.asarray(counts, np.int64)))

            def all_reduce_max_(self, t):
                t.copy_(torch.stack(self._gather("max", t.clone())).max(0).values)
                return t

            def all_reduce_sum(self, arr):
                return np.sum(self._gather("acc", np.asarray(arr)), axis=0)

        return Member()
