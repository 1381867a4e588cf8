"""Multi-GPU swarm step: agents sharded across ranks, one process per GPU.

Partition.  The global square is cut into horizontal strips, one per rank (the agent storage
order inside a shard is row-major cell order, so a strip is a contiguous range of the spatial
order).  north_star partitions agents by ID range: with strip-major IDs (gen.strip_ids,
gen.shard_inputs) each rank's contiguous ID range IS its strip, and partition(by="id") cuts by
ID and checks exactly that.  Each rank owns the agents inside its strip and keeps *ghost* copies
of the neighbouring ranks' agents within k radio radii of the shared border (k = halo depth).

Election (exact, contract E2).  Rounds run on every rank in lockstep through the frontier
stepper (include/swarm.h: swarm_frontier_*): round t gathers owned AND ghost agents over the
local graph; only owned changes are counted.  Every k-th round the owned agents within k radii
of a border send their leaders to the neighbour rank (torch.distributed P2P -- RCCL over xGMI on
GPUs, gloo in the CPU tests), where they overwrite the ghosts and activate their local
neighbours for the next round.  Between exchanges a ghost near the halo's outer edge misses
neighbours and may lag (a lower bound); that error starts one radius inside the outer edge and
moves at most one radius per round, so after j <= k rounds it has not reached the border: owned
agents are exact at every round, and so are the ghosts within one radius of the border.  Per-
round owned change counts are summed over ranks with one all-reduce every `check_every` rounds;
the first globally zero round ends the run and is rounds_exec (rounds after it are no-ops
everywhere).  Result: the same leaders, rounds and per-round change counts as a single-GPU run
on the union graph, with a halo exchange every k rounds instead of every round.

Allocation (exact, contract A-H).  Each rank resolves the tasks inside its strip.  Every
agent that can claim such a task lies within the claim radius Rp of it, so each rank first
receives the neighbour ranks' agents within Rp of the border (positions, IDs, capabilities),
runs swarm_allocate over owned + halo agents, and sends the halo agents' won counts back to
their owners.  No data-path all-gather; one small all-reduce for the global counters.

Auction (exact, config C4 on several GPUs).  Tasks are replicated, agents stay partitioned:
every round, each rank's bidders bid into the task-key array, one MAX all-reduce of the keys
(+ one bidder-count word per rank) makes them global, and every rank resolves every task the
same way (owners as agent IDs).  Same rounds, prices and owners as one GPU over all agents.

Exchanges: one per k election rounds, 2 x (k-radius band x 4 B) per neighbour (10k-20k agents
per radius of border at 10M agents per GPU and N = 2-8) -- latency-bound; the deep halo trades k
times fewer RCCL round trips for stepping k x 10k-20k ghost rows per border locally.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class Part:
    """One rank's share of a global swarm (partition()): indices into the global arrays."""
    rank: int
    world: int
    strip: tuple             # (y_lo, y_hi) of this rank's strip
    cuts: np.ndarray         # the world - 1 interior strip boundaries (the same on every rank)
    agents: np.ndarray       # int64 indices of the owned agents, ascending
    tasks: np.ndarray        # int64 indices of the tasks this rank resolves, ascending
    id_range: tuple = None   # by="id": [lo, hi) of the IDs this rank owns


def strip_cuts(y, world: int) -> np.ndarray:
    """world - 1 horizontal cuts at the y-quantiles k / world: strips of (nearly) equal agent
    counts.  Agent i belongs to strip searchsorted(cuts, y[i], 'right'): ties at a cut go up."""
    y = np.asarray(y, np.float64)
    if world <= 1 or len(y) == 0:
        return np.zeros(0, np.float64)
    ks = [(k * len(y)) // world for k in range(1, world)]
    return np.partition(y, ks)[ks].astype(np.float64)


def id_cuts(ids, world: int) -> np.ndarray:
    """world - 1 ID boundaries at the ID quantiles k / world: ranges of (nearly) equal agent
    counts.  Agent i belongs to range searchsorted(cuts, ids[i], 'right')."""
    ids = np.asarray(ids, np.int64)
    if world <= 1 or len(ids) == 0:
        return np.zeros(0, np.int64)
    ks = [(k * len(ids)) // world for k in range(1, world)]
    return np.partition(ids, ks)[ks].astype(np.int64)


def partition(x, y, world: int, rank: int, *, ty=None, min_height: float = 0.0, by: str = "y",
              ids=None) -> Part:
    """Split ONE global swarm (every rank passes the same arrays) into `world` horizontal strips
    of equal agent count; rank `rank` owns the agents of strip `rank` and the tasks whose y falls
    in it (tasks outside the agents' y-range go to the first / last strip).

    by="id" (north_star / SURVEY §8e: "agents are partitioned by ID range"): rank k owns the
    k-th of `world` contiguous ID ranges of equal agent count.  The halo machinery is a chain of
    strips, so the ranges must BE strips -- every agent of range k below every agent of range
    k + 1 in y (strip-major IDs: gen.strip_ids, gen.shard_inputs).  The strip cuts are then read
    off the ranges (the lowest y of each range above the first), and the function checks that
    cutting by those y values assigns every agent to its own ID range (ValueError otherwise:
    random or Morton IDs give ranges with up to 8 spatial neighbours, not a chain).

    Why the strips reproduce the single-swarm results: every agent is owned by
    exactly one rank, every RGG edge joins agents of the same or of adjacent strips when strips
    are taller than the radio radius (ShardedSwarm checks), and ShardedSwarm's deep halo and
    claim-radius halo give each rank every neighbour / claimant of its owned agents and tasks --
    so elect() and allocate() equal Swarm.elect() / Swarm.allocate() on the union, whatever the
    cut positions (tests/test_dist_gloo.py: one global swarm through partition())."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    id_range = None
    if by == "y":
        cuts = strip_cuts(y, world)
        who = np.searchsorted(cuts, y, side="right")
    elif by == "id":
        if ids is None:
            raise ValueError('partition(by="id") needs ids')
        ids = np.asarray(ids, np.int64)
        icut = id_cuts(ids, world)
        who = np.searchsorted(icut, ids, side="right")
        counts = np.bincount(who, minlength=world)
        if world > 1 and (counts == 0).any():
            raise ValueError(f"ID ranges of equal agent count leave rank(s) {np.nonzero(counts == 0)[0].tolist()} "
                             f"without agents ({len(ids)} agents, world {world}; repeated IDs?)")
        cuts = np.array([y[who == k].min() for k in range(1, world)], np.float64) if world > 1 else np.zeros(0)
        if not np.array_equal(np.searchsorted(cuts, y, side="right"), who):
            raise ValueError("the ID ranges are not horizontal strips (every agent of range k must lie below every "
                             "agent of range k + 1): ID-range sharding needs strip-major IDs (gen.strip_ids)")
        edges_id = np.concatenate([[ids.min() if len(ids) else 0], icut, [ids.max() + 1 if len(ids) else 0]])
        id_range = (int(edges_id[rank]), int(edges_id[rank + 1]))
    else:
        raise ValueError(f"unknown partition key {by!r}")
    agents = np.nonzero(who == rank)[0].astype(np.int64)
    lo = float(y.min()) if len(y) else 0.0
    hi = float(y.max()) if len(y) else 0.0
    edges = np.concatenate([[lo], cuts, [hi]])
    strip = (float(edges[rank]), float(edges[rank + 1]))
    if world > 1 and np.diff(edges).min() <= min_height:
        raise ValueError(f"strips of {world} equal agent counts are not taller than {min_height}: "
                         "too few agents per rank for this radius")
    tasks = np.zeros(0, np.int64)
    if ty is not None:
        tw = np.searchsorted(cuts, np.asarray(ty, np.float64), side="right")
        tasks = np.nonzero(tw == rank)[0].astype(np.int64)
    return Part(rank, world, strip, cuts, agents, tasks, id_range)


def _neighbors(rank, world):
    return (rank - 1 if rank > 0 else None), (rank + 1 if rank < world - 1 else None)


class Halo:
    """Neighbour exchange along the strip chain (rank-1 <-> rank <-> rank+1)."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.lo, self.hi = _neighbors(self.rank, self.world)
        self.device = device
        # gloo cannot move device tensors: stage through host memory (tests / 1-GPU rehearsal)
        self.host_staged = dist.get_backend(group) == "gloo"

    def _peer(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def exchange(self, to_lo, to_hi, n_from_lo, n_from_hi, like):
        """Send to_lo to rank-1 and to_hi to rank+1; receive n_from_lo / n_from_hi elements."""
        if self.host_staged and like.is_cuda:
            a, b = self._exchange(to_lo.cpu(), to_hi.cpu(), n_from_lo, n_from_hi, like.cpu()[:0])
            return a.to(like.device), b.to(like.device)
        return self._exchange(to_lo, to_hi, n_from_lo, n_from_hi, like)

    def _exchange(self, to_lo, to_hi, n_from_lo, n_from_hi, like):
        shape_tail = tuple(like.shape[1:])
        from_lo = torch.empty((n_from_lo,) + shape_tail, dtype=like.dtype, device=like.device)
        from_hi = torch.empty((n_from_hi,) + shape_tail, dtype=like.dtype, device=like.device)
        ops = []
        if self.lo is not None:
            if to_lo.numel():
                ops.append(dist.P2POp(dist.isend, to_lo.contiguous(), self._peer(self.lo), self.group))
            if n_from_lo:
                ops.append(dist.P2POp(dist.irecv, from_lo, self._peer(self.lo), self.group))
        if self.hi is not None:
            if to_hi.numel():
                ops.append(dist.P2POp(dist.isend, to_hi.contiguous(), self._peer(self.hi), self.group))
            if n_from_hi:
                ops.append(dist.P2POp(dist.irecv, from_hi, self._peer(self.hi), self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return from_lo, from_hi

    def all_reduce_sum(self, arr):
        """Element-wise sum over ranks of a small int64 vector (host array in, host array out)."""
        t = torch.as_tensor(np.asarray(arr, np.int64), device="cpu" if self.host_staged else self.device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy()

    def all_reduce_max_(self, t):
        """In-place element-wise MAX over ranks of an int64 tensor (the auction's bid keys)."""
        if self.world > 1:
            if self.host_staged and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.MAX, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def exchange_counts(self, n_to_lo, n_to_hi):
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor([n_to_lo], dtype=torch.int64, device=dev)
        u = torch.tensor([n_to_hi], dtype=torch.int64, device=dev)
        a, b = self.exchange(t if self.lo is not None else t[:0], u if self.hi is not None else u[:0],
                             1 if self.lo is not None else 0, 1 if self.hi is not None else 0, t)
        return (int(a.item()) if a.numel() else 0), (int(b.item()) if b.numel() else 0)


@dataclass
class ShardAuctionResult:
    rounds_exec: int
    bidders: np.ndarray        # GLOBAL bidders per round, rounds 1..rounds_exec
    owner_id: torch.Tensor     # per task: the owning agent's ID or -1 (replicated on every rank)
    price: torch.Tensor        # per task, f32 (replicated)
    assigned: torch.Tensor     # owned agents (storage order): task index or -1
    converged: bool
    stats: dict


@dataclass
class ShardElectResult:
    rounds_exec: int
    changes: np.ndarray        # GLOBAL per-round change counts, rounds 1..rounds_exec
    leader: torch.Tensor       # owned agents (storage order), int32
    state: torch.Tensor        # owned agents, uint8
    converged: bool


class GpuBackend:
    """libswarm.so on the rank's GPU (the product path)."""

    def __init__(self, device):
        from . import _lib
        self.L = _lib
        self.device = device
        _lib.load()
        # the shard's own ctx: the frontier stepper state between swarm_frontier_begin and the
        # last step lives in it, out of reach of other libswarm calls of this thread
        with torch.cuda.device(device):
            self.ctx = _lib.Ctx()

    def cell_order(self, pos):
        n = pos.shape[0]
        perm = torch.empty(n, dtype=torch.int32, device=self.device)
        if n:
            self.L.check(self.L.lib().swarm_cell_order(self.ctx, n, self.L.ptr(pos), 1.0,
                                                       self.L.ptr(perm), self.L.stream()))
        return perm.long()

    def build_graph(self, pos, radius):
        import ctypes
        n = pos.shape[0]
        rp = torch.empty(n + 1, dtype=torch.int32, device=self.device)
        ne = ctypes.c_int64(0)
        L = self.L
        L.check(L.lib().swarm_build_rgg(self.ctx, n, L.ptr(pos) if n else None, float(radius), L.ptr(rp), None, 0,
                                        ctypes.byref(ne), L.stream()))
        col = torch.empty(max(ne.value, 1), dtype=torch.int32, device=self.device)
        L.check(L.lib().swarm_build_rgg(self.ctx, n, L.ptr(pos) if n else None, float(radius), L.ptr(rp), L.ptr(col),
                                        col.numel(), ctypes.byref(ne), L.stream()))
        return rp, col

    def graph_compact(self, rp, col):
        """16-bit columns of the shard graph (swarm_graph_compact), or None when a delta does not fit."""
        L, n = self.L, rp.numel() - 1
        if n <= 0 or col.numel() == 0:
            return None
        c16 = torch.empty(col.numel(), dtype=torch.int16, device=self.device)
        rc = L.lib().swarm_graph_compact(self.ctx, n, L.ptr(rp), L.ptr(col), L.ptr(c16), L.stream())
        if rc == L.ERR_RANGE:
            return None
        L.check(rc)
        return c16

    def begin(self, own_begin, n_own, init, leaders, col16=None):
        L = self.L
        L.check(L.lib().swarm_frontier_begin_range(self.ctx, own_begin, n_own, init.numel(), L.ptr(init),
                                                   L.ptr(leaders[0]), L.ptr(leaders[1]), L.stream()))
        L.check(L.lib().swarm_frontier_set_compact(self.ctx, L.ptr(col16) if col16 is not None else None))

    def step(self, t, rp, col, leaders):
        L = self.L
        L.check(L.lib().swarm_frontier_step(self.ctx, t, L.ptr(rp), L.ptr(col), L.ptr(leaders[0]),
                                            L.ptr(leaders[1]), L.stream()))

    def ghosts(self, t, begin, incoming, rp, col, leaders):
        L = self.L
        if incoming.numel():
            L.check(L.lib().swarm_frontier_ghosts(self.ctx, t, begin, incoming.numel(), L.ptr(incoming),
                                                  L.ptr(rp), L.ptr(col), L.ptr(leaders[0]), L.ptr(leaders[1]),
                                                  L.stream()))

    # ---- native sharded loop (csrc/comm.hip: RCCL on the device stream, or the shared-memory transport)
    def native_comm(self, halo):
        """A libswarm communicator over the halo's group, or None.  A device (nccl) group gets an RCCL
        communicator; a host-staged (gloo) group whose ranks all run on this host gets the
        shared-memory transport (SWARM_COMM_SHM: the same C loops, every exchange staged through
        host memory -- how 2-3 processes sharing one GPU run swarm_elect_sharded).  SWARM_NATIVE_HALO=0
        disables both (the Python stepper then drives the rounds).  Every rank agrees on the outcome
        before anything collective is started, and again after the (collective) create."""
        import ctypes
        import os
        import socket
        import sys
        import zlib
        L = self.L
        if os.environ.get("SWARM_NATIVE_HALO", "1") == "0" or halo.world < 2 or not isinstance(halo, Halo):
            return None  # (test doubles that exchange in-process have no torch.distributed group)
        kind = L.COMM_SHM if halo.host_staged else L.COMM_RCCL
        dev = "cpu" if halo.host_staged else self.device
        avail = 1 if (kind == L.COMM_SHM or L.lib().swarm_comm_available()) else 0
        host = zlib.crc32(socket.gethostname().encode()) & 0x7FFFFFFF
        agree = torch.tensor([avail, host, -host], dtype=torch.int64, device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MIN, group=halo.group)
        same_host = int(agree[1]) == -int(agree[2])
        if int(agree[0]) == 0 or (kind == L.COMM_SHM and not same_host):
            return None
        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if halo.rank == 0:
            buf = (ctypes.c_uint8 * 128)()
            L.check(L.lib().swarm_comm_unique_id_kind(kind, ctypes.cast(buf, ctypes.c_void_p)))
            uid.copy_(torch.frombuffer(bytearray(buf), dtype=torch.uint8))
        dist.broadcast(uid, src=halo._peer(0), group=halo.group)
        raw = (ctypes.c_uint8 * 128)(*uid.cpu().tolist())
        comm = ctypes.c_void_p()
        rc = L.lib().swarm_comm_create_kind(ctypes.byref(comm), kind, halo.world, halo.rank,
                                           ctypes.cast(raw, ctypes.c_void_p))
        # a rank whose communicator failed makes all of them take the torch.distributed halo
        ok = torch.tensor([1 if rc == 0 else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=halo.group)
        if int(ok.item()) == 0:
            if rc == 0:
                L.lib().swarm_comm_destroy(comm)
            print(f"[swarm_amd.dist] native communicator unavailable ({L.last_error() if rc else 'a peer failed'}):"
                  " using the torch.distributed halo", file=sys.stderr, flush=True)
            return None
        self.comm_kind = "rccl" if kind == L.COMM_RCCL else "shm"
        return comm

    def elect_sharded(self, comm, sh, max_rounds):
        import ctypes
        L = self.L
        z = ctypes.c_void_p(0)
        desc = L.Shard(sh.n_own, sh.all_ids.numel(), L.ptr(sh.row_ptr), L.ptr(sh.col) if sh.col.numel() else z,
                       L.ptr(sh.all_ids), L.ptr(sh.send_lo_all) if sh.send_lo.numel() else z, sh.send_lo.numel(),
                       L.ptr(sh.send_hi_all) if sh.send_hi.numel() else z, sh.send_hi.numel(),
                       0, sh.n_glo, sh.n_glo + sh.n_own, sh.n_ghi,
                       sh.halo.lo if sh.halo.lo is not None else -1,
                       sh.halo.hi if sh.halo.hi is not None else -1, sh.halo_depth, sh.own_begin,
                       L.ptr(sh.c16) if sh.c16 is not None else z)
        rounds = ctypes.c_int32(0)
        changes = np.zeros(max_rounds, np.int64)
        rc = L.check(L.lib().swarm_elect_sharded(self.ctx, comm, ctypes.byref(desc), L.ptr(sh.leaders[0]),
                                                 L.ptr(sh.leaders[1]), max_rounds, ctypes.byref(rounds),
                                                 changes.ctypes.data_as(ctypes.c_void_p), L.stream()))
        r = rounds.value
        return r, changes[:r].copy(), rc == L.OK

    def changes(self, t0, t1):
        L = self.L
        out = np.zeros(t1 - t0 + 1, np.int64)
        L.check(L.lib().swarm_frontier_changes(self.ctx, t0, t1, out.ctypes.data_as(__import__("ctypes").c_void_p),
                                               L.stream()))
        return out

    # ---- sharded auction (swarm_auction_begin / _bid / _resolve, or the native RCCL loop)
    def auction_begin(self, ids, pos, caps, tx, ty, treq, claim_thr, u_scale, eps):
        import ctypes
        L, dev = self.L, self.device
        n, t = ids.numel(), tx.numel()
        tpos = torch.stack([tx, ty], 1).contiguous()
        st = dict(owner_id=torch.empty(t, dtype=torch.int32, device=dev),
                  price=torch.empty(t, dtype=torch.float32, device=dev),
                  assigned=torch.empty(n, dtype=torch.int32, device=dev), tpos=tpos, treq=treq)
        stats = L.AuctionStats()
        L.check(L.lib().swarm_auction_begin(
            self.ctx, n, L.ptr(ids) if n else None, L.ptr(pos) if n else None, L.ptr(caps) if n else None, t,
            L.ptr(tpos) if t else None, L.ptr(treq) if t else None, float(claim_thr), float(u_scale), float(eps),
            L.ptr(st["owner_id"]) if t else None, L.ptr(st["price"]) if t else None,
            L.ptr(st["assigned"]) if n else None, ctypes.byref(stats), L.stream()))
        st["stats"] = {k: int(getattr(stats, k)) for k, _ in L.AuctionStats._fields_}
        return st

    def auction_bid(self, r, rank, world, keys, st):
        L = self.L
        L.check(L.lib().swarm_auction_bid(self.ctx, r, rank, world, L.ptr(keys),
                                          L.ptr(st["price"]) if st["price"].numel() else None,
                                          L.ptr(st["assigned"]) if st["assigned"].numel() else None, L.stream()))

    def auction_resolve(self, r, world, keys, st, log):
        L = self.L
        L.check(L.lib().swarm_auction_resolve(self.ctx, r, world, L.ptr(keys),
                                              L.ptr(st["owner_id"]) if st["owner_id"].numel() else None,
                                              L.ptr(st["price"]) if st["price"].numel() else None,
                                              L.ptr(st["assigned"]) if st["assigned"].numel() else None,
                                              L.ptr(log), L.stream()))

    def auction_native(self, comm, ids, pos, caps, tx, ty, treq, claim_thr, u_scale, eps, max_rounds):
        import ctypes
        L, dev = self.L, self.device
        n, t = ids.numel(), tx.numel()
        tpos = torch.stack([tx, ty], 1).contiguous()
        owner = torch.empty(t, dtype=torch.int32, device=dev)
        price = torch.empty(t, dtype=torch.float32, device=dev)
        assigned = torch.empty(n, dtype=torch.int32, device=dev)
        rounds = ctypes.c_int32(0)
        bidders = np.zeros(max_rounds, np.int64)
        stats = L.AuctionStats()
        rc = L.check(L.lib().swarm_auction_sharded(
            self.ctx, comm, n, L.ptr(ids) if n else None, L.ptr(pos) if n else None, L.ptr(caps) if n else None, t,
            L.ptr(tpos) if t else None, L.ptr(treq) if t else None, float(claim_thr), float(u_scale), float(eps),
            int(max_rounds), L.ptr(owner) if t else None, L.ptr(price) if t else None,
            L.ptr(assigned) if n else None, ctypes.byref(rounds), bidders.ctypes.data_as(ctypes.c_void_p),
            ctypes.byref(stats), L.stream()))
        r = rounds.value
        return ShardAuctionResult(r, bidders[:r].copy(), owner, price, assigned, rc == L.OK,
                                  {k: int(getattr(stats, k)) for k, _ in L.AuctionStats._fields_})

    def allocate(self, ids, pos, caps, tx, ty, treq, **kw):
        from .swarm import Swarm
        s = Swarm.__new__(Swarm)  # a view over already-resident tensors (no reordering)
        s.device, s.n, s.ids, s.pos, s.caps = self.device, ids.numel(), ids, pos, caps
        s.perm, s.layout, s._id_index = None, "input", None
        s.row_ptr = s.col = None
        return s.allocate(tx, ty, treq, **kw)


class ShardedSwarm:
    """This rank's shard of a strip-partitioned swarm (see module docstring)."""

    def __init__(self, ids, x, y, caps, strip, *, radius: float = 1.0, group=None, device=None,
                 backend=None, halo=None, halo_depth: int | None = None):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.backend = backend if backend is not None else GpuBackend(self.device)
        self.halo = halo if halo is not None else Halo(group, self.device)
        self.radius = float(radius)
        self.strip = (float(strip[0]), float(strip[1]))
        if self.halo.world > 1 and self.strip[1] - self.strip[0] <= self.radius:
            raise ValueError("strips must be taller than the radio radius")
        self.halo_depth = self._agree_depth(halo_depth)
        dev = self.device
        pos = torch.stack([torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64),
                           torch.as_tensor(np.ascontiguousarray(y), dtype=torch.float64)], 1).to(dev)
        ids_t = torch.as_tensor(np.ascontiguousarray(ids, dtype=np.int32)).to(dev)
        caps_np = np.ascontiguousarray(caps if caps is not None else np.zeros(len(ids), np.uint32),
                                       dtype=np.uint32).view(np.int32)
        caps_t = torch.as_tensor(caps_np).to(dev)
        from .swarm import take_rows
        perm = self.backend.cell_order(pos) if pos.shape[0] > 1 else torch.arange(pos.shape[0], device=dev)
        self.pos, self.ids, self.caps = take_rows(pos, perm), ids_t[perm].contiguous(), caps_t[perm].contiguous()
        self.perm = perm
        self.n_own = int(self.ids.numel())
        # ghosts: neighbour ranks' agents within halo_depth radii of the shared borders
        self.send_lo, self.send_hi = self._border(self.radius * self.halo_depth)
        n_lo, n_hi = self.halo.exchange_counts(self.send_lo.numel(), self.send_hi.numel())
        gp_lo, gp_hi = self.halo.exchange(self.pos[self.send_lo], self.pos[self.send_hi], n_lo, n_hi, self.pos)
        gi_lo, gi_hi = self.halo.exchange(self.ids[self.send_lo], self.ids[self.send_hi], n_lo, n_hi, self.ids)
        self.n_glo, self.n_ghi = n_lo, n_hi
        # ghosts within one radius of the border: exact at every round (the end-of-run check)
        self.inner_lo = gp_lo[:, 1] >= self.strip[0] - self.radius - 1e-9
        self.inner_hi = gp_hi[:, 1] <= self.strip[1] + self.radius + 1e-9
        # shard graph rows: [ghosts from below | owned | ghosts from above] -- each block in its owner's
        # cell order, so the whole shard is in (near) row-major cell order and its 16-bit columns fit
        self.own_begin = self.n_glo
        self.all_pos = torch.cat([gp_lo, self.pos, gp_hi]).contiguous()
        self.all_ids = torch.cat([gi_lo, self.ids, gi_hi]).contiguous()
        self.send_lo_all = (self.send_lo + self.own_begin).contiguous()  # owned send rows as shard rows
        self.send_hi_all = (self.send_hi + self.own_begin).contiguous()
        self.row_ptr, self.col = self.backend.build_graph(self.all_pos, self.radius)
        self.c16 = self.backend.graph_compact(self.row_ptr, self.col) if hasattr(self.backend, "graph_compact") \
            else None
        self.leaders = (torch.empty(self.all_ids.numel(), dtype=torch.int32, device=dev),
                        torch.empty(self.all_ids.numel(), dtype=torch.int32, device=dev))

    @classmethod
    def from_global(cls, ids, x, y, caps=None, *, ty=None, radius: float = 1.0, group=None, device=None,
                    backend=None, halo=None, halo_depth: int | None = None, by: str = "y"):
        """This rank's shard of ONE global swarm (every rank passes the same arrays): strips of
        equal agent count (partition(); by="id": contiguous ID ranges, which must be strips).
        self.part holds the global indices of the owned agents and of the tasks this rank
        resolves (allocate_global)."""
        if halo is not None:
            rank, world = halo.rank, halo.world
        else:
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        part = partition(x, y, world, rank, ty=ty, min_height=radius, by=by, ids=ids)
        a = part.agents
        caps_a = None if caps is None else np.asarray(caps)[a]
        sh = cls(np.asarray(ids)[a], np.asarray(x)[a], np.asarray(y)[a], caps_a, part.strip, radius=radius,
                 group=group, device=device, backend=backend, halo=halo, halo_depth=halo_depth)
        sh.part = part
        return sh

    def allocate_global(self, tx, ty, treq, **kw):
        """allocate() over this rank's share (self.part.tasks) of a GLOBAL task list; the result
        rows are those tasks, in ascending global index."""
        k = self.part.tasks
        return self.allocate(np.asarray(tx)[k], np.asarray(ty)[k], np.asarray(treq)[k], **kw)

    def _agree_depth(self, want):
        """Halo depth k, the same on every rank: the requested depth (SWARM_HALO_DEPTH, default 16)
        capped so that a k-radius band stays inside the neighbour's strip."""
        import os
        k = int(want if want is not None else os.environ.get("SWARM_HALO_DEPTH", "16"))
        h = self.strip[1] - self.strip[0]
        k = max(1, min(k, int(math.floor(h / self.radius)) - 1))
        if self.halo.world > 1:
            t = torch.tensor([-k], dtype=torch.int64)
            if not getattr(self.halo, "host_staged", True):
                t = t.to(self.device)
            k = -int(self.halo.all_reduce_max_(t)[0])
        return k

    def _border(self, width):
        y = self.pos[:, 1]
        lo = torch.nonzero(y <= self.strip[0] + width + 1e-9).flatten() if self.halo.lo is not None \
            else torch.zeros(0, dtype=torch.long, device=self.device)
        hi = torch.nonzero(y >= self.strip[1] - width - 1e-9).flatten() if self.halo.hi is not None \
            else torch.zeros(0, dtype=torch.long, device=self.device)
        return lo, hi

    # ------------------------------------------------------------------ election
    def elect(self, max_rounds: int = 1 << 16, check_every: int = 64) -> ShardElectResult:
        be, h = self.backend, self.halo
        if getattr(self, "_native", "unset") == "unset":
            self._native = be.native_comm(h) if hasattr(be, "native_comm") else None
        own_sl = slice(self.own_begin, self.own_begin + self.n_own)
        if self._native is not None:
            rounds, changes, conv = be.elect_sharded(self._native, self, max_rounds)
            own = self.leaders[rounds & 1][own_sl]
            self._check_ghosts(self.leaders[rounds & 1])
            state = torch.where(own == self.ids, 3, 1).to(torch.uint8)
            return ShardElectResult(rounds, changes, own, state, conv)
        rp, col, lead = self.row_ptr, self.col, self.leaders
        be.begin(self.own_begin, self.n_own, self.all_ids, lead, self.c16)
        g_lo, g_hi = 0, self.own_begin + self.n_own
        changes = []
        t, found = 1, -1
        check_every = max(1, min(int(check_every), 256))
        while t <= max_rounds and found < 0:
            tend = min(max_rounds, t + check_every - 1)
            for r in range(t, tend + 1):
                be.step(r, rp, col, lead)
                if r % self.halo_depth:
                    continue  # ghosts stepped locally between exchanges
                cur = lead[r & 1]  # state after round r
                in_lo, in_hi = h.exchange(cur[self.send_lo_all], cur[self.send_hi_all], self.n_glo, self.n_ghi, cur)
                be.ghosts(r, g_lo, in_lo, rp, col, lead)
                be.ghosts(r, g_hi, in_hi, rp, col, lead)
            glob = h.all_reduce_sum(be.changes(t, tend))
            for i, c in enumerate(glob):
                changes.append(int(c))
                if c == 0:
                    found = t + i
                    break
            t = tend + 1
        rounds = found if found > 0 else max_rounds
        own = lead[rounds & 1][own_sl]
        state = torch.where(own == self.ids, 3, 1).to(torch.uint8)
        return ShardElectResult(rounds, np.array(changes[:rounds], np.int64), own, state, found > 0)

    def _check_ghosts(self, cur):
        """Every ghost within one radius of the border must hold its owner's final leader (cheap
        end-to-end halo check; the deeper ghosts may lag between exchanges by design)."""
        h = self.halo
        in_lo, in_hi = h.exchange(cur[self.send_lo_all], cur[self.send_hi_all], self.n_glo, self.n_ghi, cur)
        g_lo = cur[: self.n_glo]
        g_hi = cur[self.own_begin + self.n_own:self.own_begin + self.n_own + self.n_ghi]
        il, ih = self.inner_lo.to(cur.device), self.inner_hi.to(cur.device)
        if not (torch.equal(in_lo[il], g_lo[il]) and torch.equal(in_hi[ih], g_hi[ih])):
            raise RuntimeError("sharded election: ghost leaders disagree with their owners")

    # ------------------------------------------------------------------ auction (C4 sharded)
    def auction(self, tx, ty, treq, *, eps: float = 0.1, claim_thr: float = 20.0, u_scale: float = 100.0,
                max_rounds: int = 1 << 20, check_every: int = 16, native: bool | None = None) -> ShardAuctionResult:
        """Jacobi auction of this rank's agents against the SAME task set on every rank (tasks
        replicated, agents partitioned): per round, local bids -> one MAX all-reduce of the
        task keys (+ a bidder-count word per rank) -> identical resolution everywhere.  Equal
        to Swarm.auction over the union of all ranks' agents.  native (default: when an RCCL
        communicator is available) runs the whole loop in libswarm on the device stream."""
        be, h = self.backend, self.halo
        dev = self.device
        tx = torch.as_tensor(np.ascontiguousarray(tx), dtype=torch.float64).to(dev)
        ty = torch.as_tensor(np.ascontiguousarray(ty), dtype=torch.float64).to(dev)
        treq = torch.as_tensor(np.ascontiguousarray(treq), dtype=torch.int8).to(dev)
        if native is None or native:
            if getattr(self, "_native", "unset") == "unset":
                self._native = be.native_comm(h) if hasattr(be, "native_comm") else None
            if self._native is not None:
                return be.auction_native(self._native, self.ids, self.pos, self.caps, tx, ty, treq, claim_thr,
                                         u_scale, eps, max_rounds)
            if native:
                raise RuntimeError("no RCCL communicator for the native sharded auction")
        t, world, rank = tx.numel(), h.world, h.rank
        st = be.auction_begin(self.ids, self.pos, self.caps, tx, ty, treq, claim_thr, u_scale, eps)
        keys = torch.zeros(t + world, dtype=torch.int64, device=dev)
        log = torch.zeros(max_rounds + 2, dtype=torch.int64, device=dev)
        bidders = []
        r, found = 1, -1
        check_every = max(1, int(check_every))
        while r <= max_rounds and found < 0:
            rend = min(max_rounds, r + check_every - 1)
            for q in range(r, rend + 1):
                be.auction_bid(q, rank, world, keys, st)
                h.all_reduce_max_(keys)
                be.auction_resolve(q, world, keys, st, log)
            for q, nb in zip(range(r, rend + 1), log[r:rend + 1].cpu().tolist()):
                if nb == 0:
                    found = q
                    break
                bidders.append(int(nb))
            r = rend + 1
        rounds = found - 1 if found > 0 else max_rounds
        stats = dict(st.get("stats", {}), rounds_launched=min(r - 1, max_rounds), bids_total=int(sum(bidders)))
        return ShardAuctionResult(rounds, np.array(bidders[:rounds], np.int64), st["owner_id"], st["price"],
                                  st["assigned"], found > 0, stats)

    # ------------------------------------------------------------------ allocation
    def allocate(self, tx, ty, treq, *, claim_thr: float = 20.0, hysteresis: float = 5.0,
                 u_scale: float = 100.0, mode: str = "auto"):
        """Resolve this rank's tasks (inside its strip) exactly; returns (AllocResult over the
        owned tasks, won counts of the owned agents in storage order, global stats)."""
        h = self.halo
        rp_claim = (u_scale / claim_thr - 1.0) * (1 + 1e-9) + 1e-12 if claim_thr > 0 and u_scale > 0 else math.inf
        if math.isinf(rp_claim) and h.world > 1:
            raise ValueError("sharded allocation needs a finite claim radius (claim_thr > 0)")
        if h.world > 1 and self.strip[1] - self.strip[0] <= rp_claim:
            raise ValueError("strips must be taller than the claim radius")
        s_lo, s_hi = self._border(rp_claim if h.world > 1 else 0.0)
        n_lo, n_hi = h.exchange_counts(s_lo.numel(), s_hi.numel())
        hp = h.exchange(self.pos[s_lo], self.pos[s_hi], n_lo, n_hi, self.pos)
        hi_ = h.exchange(self.ids[s_lo], self.ids[s_hi], n_lo, n_hi, self.ids)
        hc = h.exchange(self.caps[s_lo], self.caps[s_hi], n_lo, n_hi, self.caps)
        ids = torch.cat([self.ids, hi_[0], hi_[1]]).contiguous()
        pos = torch.cat([self.pos, hp[0], hp[1]]).contiguous()
        caps = torch.cat([self.caps, hc[0], hc[1]]).contiguous()
        res = self.backend.allocate(ids, pos, caps, tx, ty, treq, claim_thr=claim_thr,
                                    hysteresis=hysteresis, u_scale=u_scale, mode=mode)
        won_all = res.won
        # halo agents' wins go back to their owners (reverse of the halo exchange)
        w_lo = won_all[self.n_own:self.n_own + n_lo]
        w_hi = won_all[self.n_own + n_lo:]
        back_lo, back_hi = h.exchange(w_lo, w_hi, s_lo.numel(), s_hi.numel(), won_all)
        won = won_all[: self.n_own].clone()
        if back_lo.numel():
            won.index_add_(0, s_lo, back_lo)
        if back_hi.numel():
            won.index_add_(0, s_hi, back_hi)
        keys = ("n_claims", "n_conflicts", "n_flagged", "n_candidates", "n_overflow", "n_resolved")
        st = h.all_reduce_sum([res.stats[k] for k in keys])
        gstats = dict(zip(keys, (int(v) for v in st)))
        return res, won, gstats
