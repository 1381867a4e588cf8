"""Multi-GPU swarm step: agents sharded across ranks, one process per GPU.

Partition.  Every rank owns a set of agents (north_star: a contiguous ID range) and knows, through
a Layout, which of its agents every other rank needs: the agents within a given distance of that
rank's region.  Layouts: StripChain (this rank's horizontal strip only; the neighbours are the ranks
above and below -- gen.shard_inputs, strip-major IDs), Rects (every rank's axis-aligned region:
strips cut from one global swarm, Morton blocks -- gen.shard_inputs(layout="blocks")), and Cells
(any ownership at all, e.g. ID ranges of random or Morton IDs of one global swarm: each rank's
occupied grid cells, dilated).  The agent storage order inside a shard is row-major cell order, and
the shard's rows are [ghosts of the peers ranked below | owned | ghosts of the peers ranked above].

Election (exact, contract E2).  Rounds run on every rank in lockstep through the frontier stepper
(include/swarm.h: swarm_frontier_*): round t gathers owned AND ghost agents over the local graph;
only owned changes are counted.  The ghosts are every other rank's agents within k radio radii of
this rank's region (k = halo depth), i.e. at least every agent within k hops of an owned agent.
Every k-th round each rank sends the leaders of the owned agents each peer keeps as ghosts to that
peer (torch.distributed P2P, or libswarm's native loop over RCCL / shared memory), where they
overwrite the ghosts and activate their local neighbours for the next round.  Between exchanges a
ghost k hops out misses neighbours and may lag (a lower bound); that error moves at most one hop per
round, so after j <= k rounds it has not reached an owned agent: owned agents are exact at every
round, and so are the ghosts adjacent to one.  Per-round owned change counts are summed over ranks
with one all-reduce every `check_every` rounds; the first globally zero round ends the run and is
rounds_exec.  Result: the same leaders, rounds and per-round change counts as a single-GPU run on
the union graph, with a halo exchange every k rounds instead of every round.

Allocation (exact, contract A-H).  Each rank resolves its own tasks.  Every agent that can claim a
task lies within the claim radius Rp of it, so each rank first receives every peer's agents within
Rp of its region (positions, IDs, capabilities), runs swarm_allocate over owned + halo agents, and
sends the halo agents' won counts back to their owners.  No data-path all-gather; one small
all-reduce for the global counters.

Auction (exact, config C4 on several GPUs).  Tasks are replicated, agents stay partitioned:
every round, each rank's bidders bid into the task-key array, one MAX all-reduce of the keys
(+ one bidder-count word per rank) makes them global, and every rank resolves every task the
same way (owners as agent IDs).  Same rounds, prices and owners as one GPU over all agents.

Exchanges: one per k election rounds, (agents within k radii of the border) x 4 B per peer (10k-20k
agents per radius of border at 10M agents per GPU and N = 2-8) -- latency-bound; the deep halo
trades k times fewer round trips for stepping k x 10k-20k ghost rows per border locally.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


# ------------------------------------------------------------------------------------------ layouts
class StripChain:
    """This rank's horizontal strip [y_lo, y_hi) of a chain of strips, rank k below rank k+1: the peers
    are rank - 1 (agents within `width` of the lower border) and rank + 1 (of the upper border).  Only
    the rank's own strip is known (gen.shard_inputs builds every rank's strip on its own), so a halo may
    reach one strip only: the depth is capped below the strip height."""
    kind = "strips (chain)"

    def __init__(self, strip, rank: int, world: int):
        self.strip = (float(strip[0]), float(strip[1]))
        self.rank, self.world = rank, world

    def depth_cap(self, radius):
        return max(1, int(math.floor((self.strip[1] - self.strip[0]) / radius)) - 1)

    def targets(self, x, y, width, purpose="elect"):
        out = {}
        if self.rank > 0:
            out[self.rank - 1] = y <= self.strip[0] + width + 1e-9
        if self.rank < self.world - 1:
            out[self.rank + 1] = y >= self.strip[1] - width - 1e-9
        return out

    def min_extent(self):
        return self.strip[1] - self.strip[0]


class Rects:
    """Every rank's region as axis-aligned rectangles (world x [x0, x1, y0, y1], or world x k x 4 for k
    rectangles per rank: thin strips dealt round-robin, gen.shard_inputs(pieces=k); regions may not
    overlap): rank p needs the agents within `width` (Euclidean) of any of its rectangles.  Strips cut
    from one global swarm, Morton blocks (gen.block_rects).  No depth cap: a deep halo reaches as many
    ranks as it covers."""
    kind = "rectangles"

    def __init__(self, rects, rank: int):
        r = np.asarray(rects, np.float64)
        self.rects = r.reshape(-1, 1, 4) if r.ndim <= 2 else r
        self.rank, self.world = rank, len(self.rects)

    def depth_cap(self, radius):
        return None

    def targets(self, x, y, width, purpose="elect"):
        out = {}
        w2 = (width + 1e-9) ** 2
        for p in range(self.world):
            if p == self.rank:
                continue
            m = np.zeros(len(x), bool)
            for x0, x1, y0, y1 in self.rects[p]:
                dx = np.maximum(np.maximum(x0 - x, x - x1), 0.0)
                dy = np.maximum(np.maximum(y0 - y, y - y1), 0.0)
                m |= dx * dx + dy * dy <= w2
            if m.any():
                out[p] = m
        return out

    def min_extent(self):
        r = self.rects.reshape(-1, 4)
        return float(min((r[:, 1] - r[:, 0]).min(), (r[:, 3] - r[:, 2]).min()))


def _dilate(occ: np.ndarray, k: int) -> np.ndarray:
    """Boolean grid: cells within Chebyshev distance k of an occupied cell (box sum by integral image)."""
    if k <= 0:
        return occ.copy()
    ny, nx = occ.shape
    c = np.zeros((ny + 1, nx + 1), np.int64)
    c[1:, 1:] = np.cumsum(np.cumsum(occ, 0, dtype=np.int64), 1)
    y0 = np.clip(np.arange(ny) - k, 0, ny)
    y1 = np.clip(np.arange(ny) + k + 1, 0, ny)
    x0 = np.clip(np.arange(nx) - k, 0, nx)
    x1 = np.clip(np.arange(nx) + k + 1, 0, nx)
    s = c[y1][:, x1] - c[y0][:, x1] - c[y1][:, x0] + c[y0][:, x0]
    return s > 0


class Cells:
    """Any ownership of the agents (e.g. ID ranges of random or Morton IDs of one global swarm): each
    rank's occupied cells of a grid of side `cell` over the global square, for its agents ("elect") and
    for its tasks ("alloc").  Rank p needs an agent iff the agent's cell lies within ceil(width / cell)
    cells (Chebyshev) of a cell p occupies -- a superset of the agents within `width` of p's agents or
    tasks, which is all exactness needs."""
    kind = "cells"

    def __init__(self, x, y, who, rank: int, world: int, cell: float, tx=None, ty=None, twho=None, bounds=None):
        """bounds (x0, y0, x1, y1): the grid's extent, given when the agents arrive in parts (add());
        every point added must lie inside it.  Otherwise the extent of x, y (and tx, ty)."""
        self.rank, self.world, self.cell = rank, world, float(cell)
        x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
        if bounds is not None:
            self.x0, self.y0, x1, y1 = (float(b) for b in bounds)
        else:
            pts = [x, y] + ([np.asarray(tx, np.float64), np.asarray(ty, np.float64)] if tx is not None else [])
            self.x0 = min(float(v.min()) for v in pts[0::2] if len(v)) if len(x) else 0.0
            self.y0 = min(float(v.min()) for v in pts[1::2] if len(v)) if len(x) else 0.0
            x1 = max(float(v.max()) for v in pts[0::2] if len(v)) if len(x) else 0.0
            y1 = max(float(v.max()) for v in pts[1::2] if len(v)) if len(x) else 0.0
        self.shape = (int((y1 - self.y0) // self.cell) + 1, int((x1 - self.x0) // self.cell) + 1)
        self.occ = {"elect": self._occupancy(x, y, who)}
        if tx is not None:
            self.occ["alloc"] = self._occupancy(np.asarray(tx, np.float64), np.asarray(ty, np.float64), twho)
        self._dil = {}

    def add(self, x, y, who, purpose="elect"):
        """Mark more points' cells (a swarm that arrives in parts; bounds= at construction)."""
        occ = self.occ.setdefault(purpose, np.zeros((self.world,) + self.shape, bool))
        cy, cx = self._cells(np.asarray(x, np.float64), np.asarray(y, np.float64))
        occ[np.asarray(who, np.int64), cy, cx] = True
        self._dil = {}

    def _cells(self, x, y):
        cy = np.clip(((y - self.y0) // self.cell).astype(np.int64), 0, self.shape[0] - 1)
        cx = np.clip(((x - self.x0) // self.cell).astype(np.int64), 0, self.shape[1] - 1)
        return cy, cx

    def _occupancy(self, x, y, who):
        occ = np.zeros((self.world,) + self.shape, bool)
        cy, cx = self._cells(x, y)
        occ[np.asarray(who, np.int64), cy, cx] = True
        return occ

    def depth_cap(self, radius):
        return None

    def targets(self, x, y, width, purpose="elect"):
        occ = self.occ["alloc" if purpose == "alloc" and "alloc" in self.occ else "elect"]
        k = int(math.ceil(width / self.cell - 1e-12))
        cy, cx = self._cells(np.asarray(x, np.float64), np.asarray(y, np.float64))
        out = {}
        for p in range(self.world):
            if p == self.rank:
                continue
            key = (purpose, p, k)
            if key not in self._dil:
                self._dil[key] = _dilate(occ[p], k)
            m = self._dil[key][cy, cx]
            if m.any():
                out[p] = m
        return out

    def min_extent(self):
        return math.inf


@dataclass
class Part:
    """One rank's share of a global swarm (partition()): indices into the global arrays."""
    rank: int
    world: int
    strip: tuple             # (y_lo, y_hi) of this rank's strip (strip layouts), else the agents' y-range
    cuts: np.ndarray         # the world - 1 interior strip boundaries (strip layouts), else empty
    agents: np.ndarray       # int64 indices of the owned agents, ascending
    tasks: np.ndarray        # int64 indices of the tasks this rank resolves, ascending
    id_range: tuple = None   # by="id": [lo, hi) of the IDs this rank owns
    layout: object = None    # Rects (strips) or Cells (any other ID map): what ShardedSwarm exchanges by


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


def piece_owner(ids, cuts, world: int) -> np.ndarray:
    """Owner of each ID when the IDs are cut into len(cuts) + 1 ranges (id_cuts(ids, world * pieces))
    dealt round-robin: range j goes to rank j % world.  One range per rank (pieces = 1) is the plain
    ID-range partition; more pieces spread every rank over the whole square (Morton IDs: each Morton
    block's j-th piece to rank j), which evens out the per-round work when the election's front crosses
    the square from one corner."""
    return np.searchsorted(np.asarray(cuts, np.int64), np.asarray(ids, np.int64), side="right") % world


def block_pieces(n_per: int, seed: int, world: int, rank: int, pieces: int, *, deg: float = 16.0, t: int = 0,
                 cell: float = 1.0):
    """Rank `rank`'s share of the Morton-blocks swarm (gen.shard_inputs(layout="blocks"), SURVEY §8e's C5
    shape: IDs 0 .. n_per * world - 1 along the blocks' Morton order) when its IDs are cut into
    world * pieces equal ranges dealt round-robin (piece_owner): rank q owns the ranges q, q + world, ...
    -- with pieces = world, the q-th Morton piece of every block.  Every rank generates the whole swarm
    block by block (same seeds, so the union is the blocks layout's) and keeps its own agents; its
    tasks are block `rank`'s.  Returns (inputs dict as shard_inputs', Cells layout of every rank's
    agents and tasks).  The cuts are id_cuts' on the full ID set: (j * total) // (world * pieces)."""
    from . import gen
    total = n_per * world
    cuts = np.array([(j * total) // (world * pieces) for j in range(1, world * pieces)], np.int64)
    side = gen.side_length(total, deg)
    layout = Cells(np.zeros(0), np.zeros(0), np.zeros(0, np.int64), rank, world, cell, bounds=(0.0, 0.0, side, side))
    keep = {k: [] for k in ("x", "y", "ids", "caps")}
    out = None
    for b in range(world):
        d = gen.shard_inputs(n_per, seed, world, b, deg=deg, t=t, layout="blocks")
        who = piece_owner(d["ids"], cuts, world)
        layout.add(d["x"], d["y"], who)
        if t:  # block b's tasks go to rank b
            layout.add(d["tx"], d["ty"], np.full(len(d["tx"]), b, np.int64), purpose="alloc")
        m = who == rank
        for k in keep:
            keep[k].append(d[k][m])
        if b == rank:
            out = d
        del d, who, m
    d = dict(out, **{k: np.concatenate(v) for k, v in keep.items()})
    d.update(n=int(len(d["ids"])), pieces=pieces, id_range=None)
    return d, layout


def _strip_rects(x, y, tx, ty, cuts):
    pts_x = [np.asarray(x, np.float64)] + ([np.asarray(tx, np.float64)] if tx is not None else [])
    pts_y = [np.asarray(y, np.float64)] + ([np.asarray(ty, np.float64)] if ty is not None else [])
    big = 1e300
    ylo = np.concatenate([[-big], cuts])
    yhi = np.concatenate([cuts, [big]])
    return np.stack([np.full(len(ylo), -big), np.full(len(ylo), big), ylo, yhi], 1)


def partition(x, y, world: int, rank: int, *, ty=None, tx=None, min_height: float = 0.0, by: str = "y",
              ids=None, cell: float = 1.0, pieces: int = 1) -> Part:
    """Split ONE global swarm (every rank passes the same arrays) over `world` ranks; rank `rank`
    owns part.agents and resolves part.tasks.

    by="y": horizontal strips of equal agent count; a task goes to the strip its y falls in (outside
    the agents' range: the first / last strip).  Layout Rects.
    by="id" (north_star / SURVEY §8e: "agents are partitioned by ID range"): rank k owns the k-th of
    `world` contiguous ID ranges of equal agent count, whatever the ID map.  When the ranges are
    horizontal strips (strip-major IDs: gen.strip_ids) the layout is those strips (Rects, tasks by
    strip); otherwise (random IDs, Morton IDs, ...) the layout is Cells and the tasks are dealt in
    `world` contiguous index ranges.  pieces > 1 (by="id"): world * pieces ID ranges of equal agent
    count, range j to rank j % world (piece_owner) -- layout Cells.

    Why the union of the shards reproduces the single-swarm results: every agent is owned exactly
    once, every task resolved exactly once, and ShardedSwarm's deep halo and claim-radius halo give
    each rank every agent within k hops of its owned agents and every claimant of its tasks -- so
    elect() and allocate() equal Swarm.elect() / Swarm.allocate() on the union, whatever the cut
    (tests/test_dist_gloo.py: one global swarm through partition())."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    id_range = None
    strips = True
    if by == "y":
        cuts = strip_cuts(y, world)
        who = np.searchsorted(cuts, y, side="right")
    elif by == "id":
        if ids is None:
            raise ValueError('partition(by="id") needs ids')
        ids = np.asarray(ids, np.int64)
        if pieces < 1:
            raise ValueError("pieces must be >= 1")
        icut = id_cuts(ids, world * pieces)
        who = piece_owner(ids, icut, world)
        counts = np.bincount(who, minlength=world)
        if world > 1 and (counts == 0).any():
            raise ValueError(f"ID ranges of equal agent count leave rank(s) {np.nonzero(counts == 0)[0].tolist()} "
                             f"without agents ({len(ids)} agents, world {world}; repeated IDs?)")
        cuts = np.array([y[who == k].min() for k in range(1, world)], np.float64) if world > 1 else np.zeros(0)
        # strip-major IDs: the ID ranges ARE horizontal strips (every agent of range k below range k+1)
        strips = bool(np.array_equal(np.searchsorted(cuts, y, side="right"), who))
        if pieces > 1:
            strips = False
        else:
            edges_id = np.concatenate([[ids.min() if len(ids) else 0], icut, [ids.max() + 1 if len(ids) else 0]])
            id_range = (int(edges_id[rank]), int(edges_id[rank + 1]))
    else:
        raise ValueError(f"unknown partition key {by!r}")
    agents = np.nonzero(who == rank)[0].astype(np.int64)
    lo = float(y.min()) if len(y) else 0.0
    hi = float(y.max()) if len(y) else 0.0
    tasks = np.zeros(0, np.int64)
    if strips:
        edges = np.concatenate([[lo], cuts, [hi]])
        strip = (float(edges[rank]), float(edges[rank + 1]))
        if world > 1 and np.diff(edges).min() <= min_height:
            raise ValueError(f"strips of {world} equal agent counts are not taller than {min_height}: "
                             "too few agents per rank for this radius")
        tw = None
        if ty is not None:
            tw = np.searchsorted(cuts, np.asarray(ty, np.float64), side="right")
            tasks = np.nonzero(tw == rank)[0].astype(np.int64)
        layout = Rects(_strip_rects(x, y, tx, ty, cuts), rank)
    else:
        strip, cuts = (lo, hi), np.zeros(0)
        twho = None
        if ty is not None:
            nt = len(ty)
            twho = (np.arange(nt, dtype=np.int64) * world) // max(nt, 1)
            tasks = np.nonzero(twho == rank)[0].astype(np.int64)
        if ty is not None and tx is None:
            raise ValueError('partition(by="id") with non-strip IDs needs the task x too (tx=) to place the tasks')
        layout = Cells(x, y, who, rank, world, cell, tx=tx, ty=ty, twho=twho)
    return Part(rank, world, strip, cuts, agents, tasks, id_range, layout)


class Halo:
    """Point-to-point exchange with any set of peers over a torch.distributed group."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        # gloo cannot move device tensors: stage through host memory (tests / 1-GPU rehearsal)
        self.host_staged = dist.get_backend(group) == "gloo"

    def _peer(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def exchange_peers(self, sends: dict, recv_counts: dict, like):
        """Send sends[p] to every peer p and receive recv_counts[p] elements (rows shaped like `like`)
        from it, in one batch of P2P ops.  Returns {peer: tensor}."""
        dev = like.device
        staged = self.host_staged and like.is_cuda
        tail = tuple(like.shape[1:])
        tdev = "cpu" if staged else dev
        out = {p: torch.empty((int(n),) + tail, dtype=like.dtype, device=tdev) for p, n in recv_counts.items()}
        ops = []
        for p in sorted(set(sends) | set(recv_counts)):
            t = sends.get(p)
            if t is not None and t.numel():
                t = t.contiguous().cpu() if staged else t.contiguous()
                ops.append(dist.P2POp(dist.isend, t, self._peer(p), self.group))
            if recv_counts.get(p, 0):
                ops.append(dist.P2POp(dist.irecv, out[p], self._peer(p), self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return {p: v.to(dev) for p, v in out.items()} if staged else out

    def count_matrix(self, counts):
        """counts[p] = what this rank sends to p (world int64): every rank's row, all_gather."""
        dev = "cpu" if self.host_staged else self.device
        t = torch.as_tensor(np.asarray(counts, np.int64)).to(dev)
        if self.world == 1:
            return t.cpu().numpy().reshape(1, -1)
        rows = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(rows, t, group=self.group)
        return torch.stack(rows).cpu().numpy()

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
        """16-bit columns of the shard graph (swarm_graph_compact); when a delta does not fit -- a ghost row
        stored in another peer's block -- swarm_graph_compact_escaped's, the escaped neighbours read from the
        int32 columns (self.last_escaped: their count; SWARM_C16_ESC=0: None instead, the int32 columns)."""
        import os
        L, n = self.L, rp.numel() - 1
        self.last_escaped = 0
        if n <= 0 or col.numel() == 0:
            return None
        c16 = torch.empty(col.numel(), dtype=torch.int16, device=self.device)
        rc = L.lib().swarm_graph_compact(self.ctx, n, L.ptr(rp), L.ptr(col), L.ptr(c16), L.stream())
        if rc != L.ERR_RANGE:
            L.check(rc)
            return c16
        if os.environ.get("SWARM_C16_ESC", "1") == "0" or col.numel() >= (1 << 30):
            return None
        ne = ctypes.c_int64(0)
        L.check(L.lib().swarm_graph_compact_escaped(self.ctx, n, L.ptr(rp), L.ptr(col), L.ptr(c16),
                                                    ctypes.byref(ne), L.stream()))
        self.last_escaped = int(ne.value)
        return c16

    def begin(self, own_begin, n_own, init, leaders, col16=None, escaped=False):
        L = self.L
        L.check(L.lib().swarm_frontier_begin_range(self.ctx, own_begin, n_own, init.numel(), L.ptr(init),
                                                   L.ptr(leaders[0]), L.ptr(leaders[1]), L.stream()))
        setc = L.lib().swarm_frontier_set_compact_escaped if escaped else L.lib().swarm_frontier_set_compact
        L.check(setc(self.ctx, L.ptr(col16) if col16 is not None else None))

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
        host memory -- how 2-3 processes sharing one GPU run swarm_elect_sharded).  SWARM_NATIVE_COMM=rccl
        takes the RCCL communicator on a gloo group too (with SWARM_RCCL_PATH naming the RCCL test double
        of tests/rccl_double: the RCCL branch of the native loops with peers that share one GPU, which
        real RCCL refuses).  SWARM_NATIVE_HALO=0 disables both (the Python stepper then drives the rounds).  Every rank agrees on the outcome
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
        if os.environ.get("SWARM_NATIVE_COMM", "") == "rccl":
            kind = L.COMM_RCCL
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

    def elect_sharded(self, comm, sh, max_rounds, record=False, alone=False, timed=True):
        """The native sharded loop (swarm_elect_sharded_ex).  record: also this rank's per-round counts
        (owned changes, rows and edges gathered) and per-round device times.  alone: the shard graph stepped
        by itself, no peers and no communicator (the cost model's calibration run)."""
        import ctypes
        L = self.L
        peers = [] if alone else sh.peers
        n_all = sh.all_ids.numel()
        # alone: every row counts as owned (no ghost blocks without peers)
        desc = L.shard_desc(n_all if alone else sh.n_own, n_all, sh.row_ptr, sh.col, sh.all_ids,
                            0 if alone else sh.own_begin,
                            sh.halo_depth, peers, [sh.send_count[p] for p in peers],
                            None if alone else sh.send_rows_all, [sh.ghost_count[p] for p in peers], sh.c16,
                            col16_escaped=sh.c16_escaped > 0)
        rounds = ctypes.c_int32(0)
        changes = np.zeros(max_rounds, np.int64)
        local = np.zeros((max_rounds, 3), np.int64) if record else None
        rms = np.zeros(max_rounds, np.float32) if record and timed else None
        hp = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731
        rc = L.check(L.lib().swarm_elect_sharded_ex(self.ctx, None if alone else comm, ctypes.byref(desc),
                                                    L.ptr(sh.leaders[0]), L.ptr(sh.leaders[1]), max_rounds,
                                                    ctypes.byref(rounds), hp(changes), hp(local), hp(rms),
                                                    L.stream()))
        r = rounds.value
        if record:
            return r, changes[:r].copy(), rc == L.OK, local[:r].copy(), rms[:r].copy() if rms is not None else None
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
    """This rank's shard of a partitioned swarm (see module docstring).

    region: this rank's strip (y_lo, y_hi) in a chain of strips (StripChain: gen.shard_inputs), or a
    layout (StripChain / Rects / Cells) that says which of this rank's agents every other rank needs."""

    def __init__(self, ids, x, y, caps, region, *, radius: float = 1.0, group=None, device=None,
                 backend=None, halo=None, halo_depth: int | None = None):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.backend = backend if backend is not None else GpuBackend(self.device)
        self.halo = halo if halo is not None else Halo(group, self.device)
        self.radius = float(radius)
        rank, world = self.halo.rank, self.halo.world
        self.layout = region if hasattr(region, "targets") else StripChain(region, rank, world)
        self.strip = getattr(self.layout, "strip", None)
        if world > 1 and self.layout.min_extent() <= self.radius:
            raise ValueError("regions must be wider and taller than the radio radius")
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
        hp = self.pos.cpu().numpy()
        self._hx, self._hy = np.ascontiguousarray(hp[:, 0]), np.ascontiguousarray(hp[:, 1])
        # ghosts: every peer's agents within halo_depth radii of this rank's region
        send = self._targets(self.radius * self.halo_depth, "elect")
        recv = self._recv_counts(send)
        self.peers = sorted(p for p in set(send) | set(recv) if send.get(p, np.zeros(0)).size or recv.get(p, 0))
        self.send_rows = {p: send.get(p, np.zeros(0, np.int64)) for p in self.peers}
        self.send_count = {p: int(self.send_rows[p].size) for p in self.peers}
        self.ghost_count = {p: int(recv.get(p, 0)) for p in self.peers}
        self.lower = [p for p in self.peers if p < rank]
        self.upper = [p for p in self.peers if p > rank]
        rows_dev = {p: torch.as_tensor(v, device=dev) for p, v in self.send_rows.items()}
        gp = self.halo.exchange_peers({p: self.pos[r] for p, r in rows_dev.items()}, self.ghost_count, self.pos)
        gi = self.halo.exchange_peers({p: self.ids[r] for p, r in rows_dev.items()}, self.ghost_count, self.ids)
        # shard graph rows: [ghosts of the peers below | owned | ghosts of the peers above] -- each block in
        # its owner's cell order; with strips the whole shard is in (near) row-major cell order and its
        # 16-bit columns fit
        self.own_begin = sum(self.ghost_count[p] for p in self.lower)
        self.all_pos = torch.cat([gp[p] for p in self.lower] + [self.pos] + [gp[p] for p in self.upper]).contiguous()
        self.all_ids = torch.cat([gi[p] for p in self.lower] + [self.ids] + [gi[p] for p in self.upper]).contiguous()
        self.send_rows_all = (torch.cat([rows_dev[p] for p in self.peers]) + self.own_begin).contiguous() \
            if self.peers else torch.zeros(0, dtype=torch.int64, device=dev)
        self.row_ptr, self.col = self.backend.build_graph(self.all_pos, self.radius)
        self.c16 = self.backend.graph_compact(self.row_ptr, self.col) if hasattr(self.backend, "graph_compact") \
            else None
        self.c16_escaped = int(getattr(self.backend, "last_escaped", 0)) if self.c16 is not None else 0
        self.leaders = (torch.empty(self.all_ids.numel(), dtype=torch.int32, device=dev),
                        torch.empty(self.all_ids.numel(), dtype=torch.int32, device=dev))

    # the ghost blocks below / above the owned rows (the strip chain's names)
    @property
    def n_glo(self):
        return self.own_begin

    @property
    def n_ghi(self):
        return int(self.all_ids.numel()) - self.own_begin - self.n_own

    def _targets(self, width, purpose):
        """{peer: ascending storage indices of the owned agents it needs} at halo width `width`."""
        t = self.layout.targets(self._hx, self._hy, width, purpose) if self.halo.world > 1 else {}
        return {p: np.nonzero(m)[0].astype(np.int64) for p, m in t.items() if m.any()}

    def _recv_counts(self, send):
        """What every peer sends this rank, from one all_gather of the send counts."""
        world, rank = self.halo.world, self.halo.rank
        if world == 1:
            return {}
        row = np.zeros(world, np.int64)
        for p, v in send.items():
            row[p] = v.size
        m = self.halo.count_matrix(row)
        return {q: int(m[q, rank]) for q in range(world) if q != rank and m[q, rank]}

    @classmethod
    def from_global(cls, ids, x, y, caps=None, *, ty=None, tx=None, radius: float = 1.0, group=None, device=None,
                    backend=None, halo=None, halo_depth: int | None = None, by: str = "y", pieces: int = 1):
        """This rank's shard of ONE global swarm (every rank passes the same arrays): strips of
        equal agent count, or (by="id") contiguous ID ranges of any ID map -- partition().
        self.part holds the global indices of the owned agents and of the tasks this rank
        resolves (allocate_global)."""
        if halo is not None:
            rank, world = halo.rank, halo.world
        else:
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        part = partition(x, y, world, rank, ty=ty, tx=tx, min_height=radius, by=by, ids=ids, cell=radius,
                         pieces=pieces)
        a = part.agents
        caps_a = None if caps is None else np.asarray(caps)[a]
        sh = cls(np.asarray(ids)[a], np.asarray(x)[a], np.asarray(y)[a], caps_a, part.layout, radius=radius,
                 group=group, device=device, backend=backend, halo=halo, halo_depth=halo_depth)
        sh.part = part
        return sh

    def allocate_global(self, tx, ty, treq, **kw):
        """allocate() over this rank's share (self.part.tasks) of a GLOBAL task list; the result
        rows are those tasks, in ascending global index."""
        k = self.part.tasks
        return self.allocate(np.asarray(tx)[k], np.asarray(ty)[k], np.asarray(treq)[k], **kw)

    def _agree_depth(self, want):
        """Halo depth k, the same on every rank: the requested depth (SWARM_HALO_DEPTH, default 16),
        capped (StripChain) so that a k-radius band stays inside the neighbour's strip."""
        import os
        k = int(want if want is not None else os.environ.get("SWARM_HALO_DEPTH", "16"))
        cap = self.layout.depth_cap(self.radius)
        k = max(1, k if cap is None else min(k, cap))
        if self.halo.world > 1:
            t = torch.tensor([-k], dtype=torch.int64)
            if not getattr(self.halo, "host_staged", True):
                t = t.to(self.device)
            k = -int(self.halo.all_reduce_max_(t)[0])
        return k

    def _exchange_leaders(self, cur):
        """The current leaders of the rows every peer keeps as ghosts, sent; the ghosts' owners' values
        received: (lower block, upper block) in row order."""
        sends, off = {}, 0
        for p in self.peers:
            n = self.send_count[p]
            sends[p] = cur[self.send_rows_all[off:off + n]]
            off += n
        got = self.halo.exchange_peers(sends, self.ghost_count, cur)
        empty = cur[:0]
        lo = torch.cat([got[p] for p in self.lower]) if self.lower else empty
        hi = torch.cat([got[p] for p in self.upper]) if self.upper else empty
        return lo, hi

    # ------------------------------------------------------------------ election
    def elect(self, max_rounds: int = 1 << 16, check_every: int = 64, record: bool = False) -> ShardElectResult:
        """The sharded election (contract E2).  record (native loop only): the result also carries this
        rank's per-round counts (.local: owned changes, rows gathered, edges gathered; -1 edges = a dense
        round over the whole shard graph) and per-round device times (.round_ms)."""
        be, h = self.backend, self.halo
        if getattr(self, "_native", "unset") == "unset":
            self._native = be.native_comm(h) if hasattr(be, "native_comm") else None
        own_sl = slice(self.own_begin, self.own_begin + self.n_own)
        if self._native is not None:
            out = be.elect_sharded(self._native, self, max_rounds, record=record)
            rounds, changes, conv = out[:3]
            own = self.leaders[rounds & 1][own_sl]
            self._check_ghosts(self.leaders[rounds & 1])
            state = torch.where(own == self.ids, 3, 1).to(torch.uint8)
            res = ShardElectResult(rounds, changes, own, state, conv)
            if record:
                res.local, res.round_ms = out[3], out[4]
            return res
        if record:
            raise RuntimeError("elect(record=True) needs the native sharded loop")
        rp, col, lead = self.row_ptr, self.col, self.leaders
        if self.c16_escaped:
            be.begin(self.own_begin, self.n_own, self.all_ids, lead, self.c16, escaped=True)
        else:
            be.begin(self.own_begin, self.n_own, self.all_ids, lead, self.c16)
        g_lo, g_hi = 0, self.own_begin + self.n_own
        changes = []
        t, found = 1, -1
        check_every = max(1, min(int(check_every), 256))
        while t <= max_rounds and found < 0:
            tend = min(max_rounds, t + check_every - 1)
            for r in range(t, tend + 1):
                be.step(r, rp, col, lead)
                if r % self.halo_depth or h.world == 1:
                    continue  # ghosts stepped locally between exchanges
                in_lo, in_hi = self._exchange_leaders(lead[r & 1])  # state after round r
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

    def elect_alone(self, max_rounds: int = 1 << 16, timed: bool = True):
        """This shard's graph elected by itself on this rank's GPU (no peers, no exchange): the calibration
        run of the election cost model -- (rounds, per-round local counts, per-round device ms, wall ms).
        timed=False: no per-round events (rms None), the wall time of the plain loop."""
        import time
        be = self.backend
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        r, _, _, local, rms = be.elect_sharded(None, self, max_rounds, record=True, alone=True, timed=timed)
        torch.cuda.synchronize(self.device)
        return r, local, rms, (time.perf_counter() - t0) * 1e3

    def exact_ghosts(self):
        """Ghost rows adjacent to an owned row (one hop from the owned agents): their values are exact
        at every round, so after the run they must equal their owners' final leaders."""
        if getattr(self, "_exact_ghosts", None) is None:
            rp = self.row_ptr.cpu().numpy()
            col = self.col.cpu().numpy()
            ob, oe = self.own_begin, self.own_begin + self.n_own
            c = col[int(rp[ob]):int(rp[oe])] if self.n_own else col[:0]
            m = np.zeros(int(self.all_ids.numel()), bool)
            m[c[(c < ob) | (c >= oe)]] = True
            self._exact_ghosts = torch.as_tensor(m)
        return self._exact_ghosts

    def _check_ghosts(self, cur):
        """Every ghost adjacent to an owned agent must hold its owner's final leader (cheap end-to-end
        halo check; the deeper ghosts may lag between exchanges by design)."""
        in_lo, in_hi = self._exchange_leaders(cur)
        oe = self.own_begin + self.n_own
        m = self.exact_ghosts().to(cur.device)
        if not (torch.equal(in_lo[m[:self.own_begin]], cur[:self.own_begin][m[:self.own_begin]])
                and torch.equal(in_hi[m[oe:]], cur[oe:][m[oe:]])):
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
        """Resolve this rank's tasks exactly; returns (AllocResult over the owned tasks, won counts of
        the owned agents in storage order, global stats).  The tasks must lie in this rank's region
        (StripChain / Rects) or be this rank's share of the global tasks (Cells: partition().tasks)."""
        h = self.halo
        rp_claim = (u_scale / claim_thr - 1.0) * (1 + 1e-9) + 1e-12 if claim_thr > 0 and u_scale > 0 else math.inf
        if math.isinf(rp_claim) and h.world > 1:
            raise ValueError("sharded allocation needs a finite claim radius (claim_thr > 0)")
        if h.world > 1 and isinstance(self.layout, StripChain) and self.layout.min_extent() <= rp_claim:
            raise ValueError("strips must be taller than the claim radius")
        send = self._targets(rp_claim, "alloc")
        recv = self._recv_counts(send)
        peers = sorted(set(send) | set(recv))
        rows = {p: torch.as_tensor(send[p], device=self.device) for p in send}
        cnt = {p: int(recv.get(p, 0)) for p in peers}
        hp = h.exchange_peers({p: self.pos[r] for p, r in rows.items()}, cnt, self.pos)
        hi_ = h.exchange_peers({p: self.ids[r] for p, r in rows.items()}, cnt, self.ids)
        hc = h.exchange_peers({p: self.caps[r] for p, r in rows.items()}, cnt, self.caps)
        ids = torch.cat([self.ids] + [hi_[p] for p in peers]).contiguous()
        pos = torch.cat([self.pos] + [hp[p] for p in peers]).contiguous()
        caps = torch.cat([self.caps] + [hc[p] for p in peers]).contiguous()
        res = self.backend.allocate(ids, pos, caps, tx, ty, treq, claim_thr=claim_thr,
                                    hysteresis=hysteresis, u_scale=u_scale, mode=mode)
        won_all = res.won
        # halo agents' wins go back to their owners (reverse of the halo exchange)
        back, off = {}, self.n_own
        for p in peers:
            back[p] = won_all[off:off + cnt[p]]
            off += cnt[p]
        got = h.exchange_peers(back, {p: int(rows[p].numel()) for p in rows}, won_all)
        won = won_all[: self.n_own].clone()
        for p, v in got.items():
            if v.numel():
                won.index_add_(0, rows[p], v)
        keys = ("n_claims", "n_conflicts", "n_flagged", "n_candidates", "n_overflow", "n_resolved")
        st = h.all_reduce_sum([res.stats[k] for k in keys])
        gstats = dict(zip(keys, (int(v) for v in st)))
        return res, won, gstats
