"""Batched, HBM-resident swarm: the GPU face of the reference's per-round handlers.

One ``Swarm`` holds every agent as structure-of-arrays in device memory (SURVEY §2 "SoA swarm
state"): ``ids`` int32, ``pos`` float64 (x, y) pairs, ``caps`` uint32 bitmask, the neighbour
CSR (``row_ptr`` int32, ``col`` int32) and the election outputs ``leader`` int32 / ``state``
uint8.  Agents are stored in spatial (grid-cell) order by default, so a neighbour gather and a
task's candidate scan touch nearby memory; ``perm`` maps storage index -> input index.

  elect()     all rounds of contract E2 to convergence  -> swarm_elect (libswarm.so)
              (SwarmAgent._handle_election_acclaim / _handle_heartbeat, agent.py:243-275)
  allocate()  one claim/resolve/notify round             -> swarm_allocate
              (SwarmAgent._process_tasks / _handle_task_claim / _handle_task_conflict /
               _calculate_utility, agent.py:292-347)

Every compute call goes through the HIP kernels; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib

# swarm_elect_compact's edge cap with 16-bit columns (elect.hip elect_impl: 32-bit byte offsets into
# the int16 columns, less a margin for the clamped offsets past a row's end)
_C16_EDGE_CAP = (1 << 31) - (1 << 20)


def _c16_rounds() -> bool:
    """Every round of swarm_elect_compact reads the 16-bit columns (the A/B knobs of elect.hip's
    tuning(): SWARM_C16 and SWARM_DENSE_FLAT, both on by default)."""
    return os.environ.get("SWARM_C16", "1") != "0" and os.environ.get("SWARM_DENSE_FLAT", "1") != "0"


CAP_VOCAB_DEFAULT = ("extinguisher", "sonar", "camera", "gripper")
STATUS_NAMES = ("OPEN", "TENTATIVE", "LOCKED", "ASSIGNED")
# Capability bit reserved for "a required capability no agent holds" (a task dict naming a
# capability outside the vocabulary: agent.py:344 gives every agent has_cap = 0 for it).  The
# bridge never sets it on an agent, so vocabularies hold at most 31 names.
CAP_UNHELD_BIT = 31


def _dev(device):
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError("swarm_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def _to(a, dtype, device):
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:  # torch refuses read-only buffers (np.frombuffer, np.load views)
        a = a.copy()
    return torch.as_tensor(a, dtype=dtype, device=device)


# SWARM_TRUST_C16=0 (A/B aid): every election re-checks the 16-bit columns on the device
_TRUST_C16 = _lib.ELECT_TRUST_C16 if os.environ.get("SWARM_TRUST_C16", "1") != "0" else 0


@dataclass
class ElectResult:
    rounds_exec: int
    changes: np.ndarray                 # per-round change counts, rounds 1..rounds_exec
    leader: torch.Tensor                # int32 [n], storage order
    state: torch.Tensor                 # uint8 [n], storage order (1 FOLLOWER, 3 LEADER)
    converged: bool = True
    rounds_launched: int = 0
    active_total: int = 0               # agents gathered (dense: all, sparse: marked), summed over rounds
    edges_total: int = 0                # CSR edges visited, summed over rounds
    dense_rounds: int = 0               # rounds run as a full dense sweep
    bytes_total: float = 0.0            # algorithmic HBM bytes of rounds 1..rounds_exec


@dataclass
class AuctionResult:
    owner: torch.Tensor                 # int32 [t] storage index of the task's agent (-1 = none)
    price: torch.Tensor                 # float32 [t] final prices
    assigned: torch.Tensor              # int32 [n] task index per agent (storage order, -1 = none)
    rounds_exec: int                    # rounds that had bidders
    bidders: np.ndarray                 # per-round bidder counts, rounds 1..rounds_exec
    converged: bool = True
    stats: dict = field(default_factory=dict)


@dataclass
class AllocResult:
    winner: torch.Tensor                # int32 [t] (-1 = unclaimed)
    util: torch.Tensor                  # float64 [t] winning claim value (f32-valued)
    won: torch.Tensor                   # int32 [n] tasks won per agent (storage order)
    nclaim: torch.Tensor                # int64 [t] TASK_CLAIMs per task
    nmsg: torch.Tensor                  # int64 [t] TASK_CONFLICTs per task
    stats: dict = field(default_factory=dict)


def _fast_ptr(t):
    """Device pointer of a tensor this module made or owns (contiguous, on the right device): no
    validation (allocate's per-call host cost; user tensors go through _lib.ptr)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def take_rows(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """t[idx] for a 2-D tensor, gathered one column at a time.  On this PyTorch-ROCm build the
    row gathers of an (N, 2) float64 tensor (t[idx], index_select, gather) return wrong rows
    above 2^26 rows, while 1-D gathers are right (checked on MI355X at 68M and 140M rows); the
    wrong positions piled 67M agents into one grid cell, and the graph build then never ended."""
    if t.dim() != 2:
        return t[idx].contiguous()
    return torch.stack([t[:, j].contiguous()[idx] for j in range(t.shape[1])], 1).contiguous()


class Swarm:
    """Structure-of-arrays swarm resident on one GPU."""

    def __init__(self, ids, x, y, caps=None, *, layout: str = "spatial", cell: float = 1.0,
                 device=None):
        dev = _dev(device)
        _lib.lib()
        self.device = dev
        ids_t = _to(ids, torch.int32, dev)
        n = ids_t.numel()
        pos = torch.stack([_to(x, torch.float64, dev), _to(y, torch.float64, dev)], dim=1).contiguous()
        if caps is None:
            caps = np.zeros(n, np.uint32)
        if not isinstance(caps, torch.Tensor):  # uint32 bitmask, carried bit-for-bit as int32
            caps = np.ascontiguousarray(caps, dtype=np.uint32).view(np.int32)
        caps_t = _to(caps, torch.int32, dev)
        self.n = n
        if layout == "spatial" and n > 1:
            perm = torch.empty(n, dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                _lib.check(_lib.lib().swarm_cell_order(_lib.ctx(), n, _lib.ptr(pos, torch.float64),
                                                       float(cell), _lib.ptr(perm), _lib.stream()))
            p = perm.long()
            ids_t, pos, caps_t = ids_t[p].contiguous(), take_rows(pos, p), caps_t[p].contiguous()
            self.perm = perm
        elif layout in ("spatial", "input"):
            self.perm = torch.arange(n, dtype=torch.int32, device=dev)
        else:
            raise ValueError(f"unknown layout {layout!r}")
        self.layout = layout
        self.cell = float(cell)
        self._cindex = None  # (Grid, cell_off): cell index of the spatial storage order, built lazily
        self.ids, self.pos, self.caps = ids_t, pos, caps_t
        if n and int(ids_t.min()) < 0:
            raise ValueError("agent IDs must be non-negative")
        self.row_ptr = None
        self.col = None
        self.leader = torch.empty(n, dtype=torch.int32, device=dev)
        self.state = torch.full((n,), _lib.FOLLOWER, dtype=torch.uint8, device=dev)
        self._id_index = None

    # ------------------------------------------------------------------ graph
    @property
    def n_edges(self) -> int:
        return 0 if self.col is None else int(self.col.numel())

    def build_graph(self, radius: float = 1.0):
        """Radius graph over the current storage order, built on the GPU (swarm_build_rgg)."""
        n, dev = self.n, self.device
        L = _lib.lib()
        row_ptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        ne = ctypes.c_int64(0)
        with torch.cuda.device(dev):
            _lib.check(L.swarm_build_rgg(_lib.ctx(), n, _lib.ptr(self.pos) if n else None, float(radius),
                                         _lib.ptr(row_ptr), None, 0, ctypes.byref(ne), _lib.stream()))
            col = torch.empty(max(ne.value, 1), dtype=torch.int32, device=dev)
            _lib.check(L.swarm_build_rgg(_lib.ctx(), n, _lib.ptr(self.pos) if n else None, float(radius),
                                         _lib.ptr(row_ptr), _lib.ptr(col), col.numel(), ctypes.byref(ne),
                                         _lib.stream()))
        self.row_ptr, self.col = row_ptr, col[: ne.value]
        self._hear = None  # a radius graph is symmetric: its own transpose
        return self

    def set_graph(self, row_ptr, col):
        """CSR given over INPUT indices (as the caller numbered agents); relabelled to storage."""
        rp = np.asarray(row_ptr.cpu() if isinstance(row_ptr, torch.Tensor) else row_ptr, np.int64)
        cl = np.asarray(col.cpu() if isinstance(col, torch.Tensor) else col, np.int64)
        if rp[-1] >= 2**31:
            raise ValueError("graph has >= 2^31 edges; shard it (swarm_amd.dist)")
        perm = self.perm.cpu().numpy().astype(np.int64)
        if self.layout != "input" and self.n > 1:
            inv = np.empty(self.n, np.int64)
            inv[perm] = np.arange(self.n)
            deg = np.diff(rp)[perm]
            new_rp = np.zeros(self.n + 1, np.int64)
            new_rp[1:] = np.cumsum(deg)
            flat = np.repeat(rp[:-1][perm] - new_rp[:-1], deg) + np.arange(new_rp[-1])
            cl = inv[cl[flat]]
            rp = new_rp
        self.row_ptr = torch.as_tensor(rp.astype(np.int32), device=self.device)
        self.col = torch.as_tensor(cl.astype(np.int32), device=self.device)
        # hearers (transpose) CSR for the protocol's push marks: the same arrays when symmetric
        src = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(rp))
        fwd = np.sort(src * max(self.n, 1) + cl)
        bwd = np.sort(cl * max(self.n, 1) + src)
        if np.array_equal(fwd, bwd):
            self._hear = None
        else:
            order = np.argsort(cl, kind="stable")
            trp = np.zeros(self.n + 1, np.int64)
            trp[1:] = np.cumsum(np.bincount(cl, minlength=self.n))
            self._hear = (torch.as_tensor(trp.astype(np.int32), device=self.device),
                          torch.as_tensor(src[order].astype(np.int32), device=self.device))
        return self

    # ------------------------------------------------------------------ election
    def graph_compact(self) -> torch.Tensor | None:
        """16-bit columns of the (symmetric) neighbour graph (swarm_graph_compact: each neighbour as
        a delta from its row's 64-agent base), built on first use and rebuilt whenever row_ptr / col
        are replaced or modified in place; None when a delta does not fit (the int32 columns are
        used then) or the graph is directed."""
        if self.row_ptr is None or getattr(self, "_hear", None) is not None or not 0 < self.n < (1 << 30):
            return None
        key = (self.row_ptr.data_ptr(), self.col.data_ptr(), self.row_ptr._version, self.col._version,
               self.n, self.col.numel())
        cached = getattr(self, "_c16", None)
        if cached is None or cached[0] != key:
            c16 = torch.empty(max(self.col.numel(), 1), dtype=torch.int16, device=self.device)
            with torch.cuda.device(self.device):
                rc = _lib.lib().swarm_graph_compact(_lib.ctx(), self.n, _lib.ptr(self.row_ptr, torch.int32),
                                                    _lib.ptr(self.col, torch.int32) if self.col.numel() else None,
                                                    _lib.ptr(c16), _lib.stream())
            if rc == _lib.ERR_RANGE:
                c16 = None
            else:
                _lib.check(rc)
            self._c16 = cached = (key, c16)
        return cached[1]

    def elect(self, mode: str = "frontier", max_rounds: int = 1 << 16, timed: bool = False,
              compact: bool = True, wide: bool | None = None) -> ElectResult:
        """Contract E2 to convergence on the GPU (swarm_elect_compact with the graph's 16-bit
        columns when they fit; swarm_elect_directed when the neighbour lists are not symmetric).
        timed: per-kernel HIP events.  compact=False: the int32-column entry point swarm_elect
        (same results).  wide: int64 row offsets (swarm_elect_i64) -- chosen by itself for
        graphs of >= 2^30 edges unless their 16-bit columns fit (swarm_elect_compact then takes up
        to 2^31 - 2^20 edges on 32-bit offsets: C5's 100M agents on one GPU, ~1.6e9), True forces it.
        The 16-bit columns are graph_compact's, rebuilt whenever row_ptr / col change: the call passes
        SWARM_ELECT_TRUST_C16, so the library skips its device check of them (include/swarm.h)."""
        if self.row_ptr is None:
            raise RuntimeError("no neighbour graph: call build_graph() or set_graph()")
        if wide is None:
            wide = self.n_edges >= (1 << 30) or self.n >= (1 << 30)
            if wide and self.n < (1 << 30) and self.n_edges < _C16_EDGE_CAP and compact \
                    and getattr(self, "_hear", None) is None and _c16_rounds():
                with torch.cuda.device(self.device):
                    wide = self.graph_compact() is None
        if wide:
            return self._elect_wide(mode, max_rounds, timed, compact)
        m = {"dense": _lib.ELECT_DENSE, "frontier": _lib.ELECT_FRONTIER}[mode] | (_lib.ELECT_TIMED if timed else 0)
        n = self.n
        rounds = ctypes.c_int32(0)
        cap = int(max_rounds)
        changes = np.empty(cap, np.int64)  # libswarm writes rounds 1..rounds_exec
        st = _lib.ElectStats()
        hear = getattr(self, "_hear", None)
        with torch.cuda.device(self.device):
            c16 = self.graph_compact() if (compact and hear is None) else None
            if c16 is not None:  # symmetric graph, 16-bit columns
                # graph_compact built them on this ctx from the current row_ptr / col (its cache key holds
                # their versions): the library skips its column check and edge-count read-back
                rc = _lib.check(_lib.lib().swarm_elect_compact(
                    _lib.ctx(), n, _lib.ptr(self.row_ptr, torch.int32), _lib.ptr(self.col, torch.int32),
                    _lib.ptr(c16), _lib.ptr(self.ids, torch.int32), _lib.ptr(self.leader, torch.int32),
                    _lib.ptr(self.state, torch.uint8), cap, m | _TRUST_C16, ctypes.byref(rounds),
                    changes.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), _lib.stream()))
            elif hear is None:  # symmetric graph: risers mark through their own rows
                rc = _lib.check(_lib.lib().swarm_elect(
                    _lib.ctx(), n, _lib.ptr(self.row_ptr, torch.int32), _lib.ptr(self.col, torch.int32),
                    _lib.ptr(self.ids, torch.int32), _lib.ptr(self.leader, torch.int32),
                    _lib.ptr(self.state, torch.uint8), cap, m, ctypes.byref(rounds),
                    changes.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), _lib.stream()))
            else:  # directed (from_agents / set_graph with asymmetric lists): mark the hearers
                rc = _lib.check(_lib.lib().swarm_elect_directed(
                    _lib.ctx(), n, _lib.ptr(self.row_ptr, torch.int32), _lib.ptr(self.col, torch.int32),
                    _lib.ptr(hear[0], torch.int32), _lib.ptr(hear[1], torch.int32) if hear[1].numel() else None,
                    _lib.ptr(self.ids, torch.int32), _lib.ptr(self.leader, torch.int32),
                    _lib.ptr(self.state, torch.uint8), cap, m, ctypes.byref(rounds),
                    changes.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), _lib.stream()))
        r = rounds.value
        res = ElectResult(r, changes[:r].copy(), self.leader, self.state, rc == _lib.OK,
                          st.rounds_launched, st.active_total, st.edges_total, st.dense_rounds,
                          st.bytes_total)
        res.changes_total = st.changes_total
        res.gather_ms, res.apply_ms, res.timed_launches = st.gather_ms, st.apply_ms, st.gather_launches
        res.sparse_ms, res.sparse_launches, res.sparse_bytes = st.sparse_ms, st.sparse_launches, st.sparse_bytes
        res.compact = c16 is not None  # the rounds read the 16-bit columns (2 of the 4 column bytes)
        res.wide = False               # 32-bit row offsets
        return res

    def _elect_wide(self, mode: str, max_rounds: int, timed: bool, compact: bool = True) -> ElectResult:
        """swarm_elect_compact_i64 (16-bit columns when they fit) or swarm_elect_i64 over an int64
        copy of row_ptr (kept while row_ptr is unchanged)."""
        if getattr(self, "_hear", None) is not None:
            raise ValueError("int64 row offsets: symmetric neighbour graphs only (swarm_elect_i64)")
        key = (self.row_ptr.data_ptr(), self.row_ptr._version, self.n)
        cached = getattr(self, "_rp64", None)
        if cached is None or cached[0] != key:
            self._rp64 = cached = (key, self.row_ptr.to(torch.int64))
        rp64 = cached[1]
        m = {"dense": _lib.ELECT_DENSE, "frontier": _lib.ELECT_FRONTIER}[mode] | (_lib.ELECT_TIMED if timed else 0)
        rounds = ctypes.c_int32(0)
        cap = int(max_rounds)
        changes = np.empty(cap, np.int64)
        st = _lib.ElectStats()
        with torch.cuda.device(self.device):
            c16 = self.graph_compact() if compact else None
            rc = _lib.check(_lib.lib().swarm_elect_compact_i64(
                _lib.ctx(), self.n, _lib.ptr(rp64, torch.int64), _lib.ptr(self.col, torch.int32),
                _lib.ptr(c16) if c16 is not None else None,
                _lib.ptr(self.ids, torch.int32), _lib.ptr(self.leader, torch.int32),
                _lib.ptr(self.state, torch.uint8), cap, m, ctypes.byref(rounds),
                changes.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), _lib.stream()))
        r = rounds.value
        res = ElectResult(r, changes[:r].copy(), self.leader, self.state, rc == _lib.OK,
                          st.rounds_launched, st.active_total, st.edges_total, st.dense_rounds,
                          st.bytes_total)
        res.changes_total = st.changes_total
        res.gather_ms, res.apply_ms, res.timed_launches = st.gather_ms, st.apply_ms, st.gather_launches
        res.sparse_ms, res.sparse_launches, res.sparse_bytes = st.sparse_ms, st.sparse_launches, st.sparse_bytes
        # the int64-offset DENSE rounds read the int32 columns (elect.hip launch_dense_round takes
        # col16 only with 32-bit offsets): only the frontier's sparse rounds read the 16-bit ones
        res.compact = c16 is not None and mode == "frontier"
        res.wide = True
        return res

    # ------------------------------------------------------------------ allocation
    def id_index(self) -> torch.Tensor | None:
        """id -> storage index table (None if IDs are too sparse for a dense table)."""
        if self._id_index is None and self.n:
            span = int(self.ids.max()) + 1
            if span <= 4 * self.n + 1024:
                t = torch.full((span,), -1, dtype=torch.int32, device=self.device)
                t[self.ids.long()] = torch.arange(self.n, dtype=torch.int32, device=self.device)
                self._id_index = t
        return self._id_index

    def _indexable(self, mode, claim_thr, u_scale) -> bool:
        """The binned round can use the storage order's cell index: spatial layout, a finite claim
        radius spanning <= 16 index rows (else swarm_allocate bins by hashed cells)."""
        if self.layout != "spatial" or self.n < 2 or mode == "dense" or not (claim_thr > 0 and u_scale > 0):
            return False
        rp = (u_scale / claim_thr - 1.0) * (1 + 1e-9) + 1e-12
        return rp > 0 and np.floor(2.0 * rp / self.cell) + 2 <= 16  # index cells are >= self.cell

    def _cell_index(self):
        """(Grid, cell_off) of the storage order (swarm_cell_index), built once; the allocation
        verifies it on the device every call and drops it when positions have moved.  None when
        the current positions are no longer in cell order (after physics_step moved agents across
        cells): allocate() then bins by hashed cells, and the index is tried again only after
        the positions change again (self._cindex = False marks 'not indexable' for the position
        tensor and version in self._cindex_bad)."""
        if self._cindex is False:
            if self._indexed_pos("_cindex_bad"):
                return None
            self._cindex = None
        if self._cindex is None:
            L, g, nc = _lib.lib(), _lib.Grid(), ctypes.c_int64(0)
            _lib.check(L.swarm_cell_index(_lib.ctx(), self.n, _lib.ptr(self.pos), self.cell, ctypes.byref(g), None, 0,
                                          ctypes.byref(nc), _lib.stream()))
            off = torch.empty(nc.value + 1, dtype=torch.int32, device=self.device)
            rc = L.swarm_cell_index(_lib.ctx(), self.n, _lib.ptr(self.pos), self.cell, ctypes.byref(g),
                                    _lib.ptr(off), off.numel(), ctypes.byref(nc), _lib.stream())
            if rc == _lib.ERR_ARG and "not in cell order" in _lib.last_error():
                self._cindex, self._cindex_bad = False, (self.pos, self.pos._version)
                return None
            _lib.check(rc)
            self._cindex = (g, off)
            # the positions it indexed: the tensor object itself (held, so its storage cannot be handed to
            # another tensor) and its version; allocate trusts the index while both are unchanged
            self._cindex_key = (self.pos, self.pos._version)
        return self._cindex

    def _indexed_pos(self, attr="_cindex_key") -> bool:
        """self.pos is the very tensor, at the same version, that the key `attr` recorded."""
        k = getattr(self, attr, None)
        return k is not None and k[0] is self.pos and k[1] == self.pos._version

    def allocate(self, tx, ty, treq, *, winner=None, util=None, claim_thr: float = 20.0,
                 hysteresis: float = 5.0, u_scale: float = 100.0, mode: str = "auto") -> AllocResult:
        """One allocation round over t tasks (swarm_allocate).  winner/util = existing claims."""
        if winner is None and util is None and mode == "auto":
            r = self._allocate_again(tx, ty, treq, claim_thr, hysteresis, u_scale)
            if r is not None:
                return r
        dev = self.device
        tpos = self._task_pos(tx, ty)
        tq = _to(treq, torch.int8, dev)
        t = tq.numel()
        # no claim table: winner / util are outputs only (the indexed call initialises them on the device)
        fresh = winner is None and util is None
        w = (torch.empty(t, dtype=torch.int32, device=dev) if winner is None
             else _to(winner, torch.int32, dev).clone())
        u = (torch.empty(t, dtype=torch.float64, device=dev) if util is None
             else _to(util, torch.float64, dev).clone())
        # libswarm zeroes won and writes nclaim / nmsg for every task (one buffer for both)
        won = torch.empty(self.n, dtype=torch.int32, device=dev)
        nc_nm = torch.empty((2, t), dtype=torch.int64, device=dev)
        nclaim, nmsg = nc_nm[0], nc_nm[1]
        idx = self.id_index()
        st = _lib.AllocStats()
        m = {"auto": _lib.ALLOC_AUTO, "binned": _lib.ALLOC_BINNED, "dense": _lib.ALLOC_DENSE}[mode]
        L = _lib.lib()
        # every tensor below is this call's or the Swarm's own (contiguous, on dev): raw pointers
        p = _fast_ptr
        with torch.cuda.device(dev):
            ci = self._cell_index() if self._indexable(mode, claim_thr, u_scale) else None
            rc = _lib.ERR_STALE
            if ci is not None:  # spatial storage order: no binning pass (swarm_allocate_indexed_ex)
                # the index is trusted while self.pos is the tensor and version it was built from (the
                # device staleness check runs otherwise); the claim table is updated in place: keep
                # the caller's for a stale-index retry
                trusted = self._indexed_pos()
                flags = (_lib.ALLOC_TRUST_INDEX if trusted else 0) | (_lib.ALLOC_FRESH_CLAIMS if fresh else 0)
                w0 = None if winner is None or trusted else w.clone()
                u0 = None if util is None or trusted else u.clone()
                rc = L.swarm_allocate_indexed_ex(
                    _lib.ctx(), self.n, p(self.ids), p(self.pos), p(self.caps),
                    ctypes.byref(ci[0]), p(ci[1]), t, p(tpos), p(tq), float(claim_thr),
                    float(hysteresis), float(u_scale), flags, p(w), p(u), p(won), p(idx),
                    0 if idx is None else idx.numel(), p(nclaim), p(nmsg), ctypes.byref(st),
                    _lib.stream())
                if rc == _lib.OK and trusted and fresh and mode == "auto" and isinstance(treq, torch.Tensor) \
                        and tq is treq:
                    # the same call again (same task tensors and versions, same trusted index, same
                    # swarm arrays) needs none of the above: _allocate_again replays it from here
                    self._again = ((tx, ty, treq, (tx._version, ty._version, treq._version), self.pos,
                                    self.pos._version, self.ids, self.caps, (claim_thr, hysteresis, u_scale),
                                    torch.cuda.current_device()),
                                   (self.n, self.ids.data_ptr(), self.pos.data_ptr(), self.caps.data_ptr(),
                                    ctypes.byref(ci[0]), ci[1].data_ptr(), t, tpos.data_ptr(), tq.data_ptr(),
                                    float(claim_thr), float(hysteresis), float(u_scale), flags),
                                   (idx.data_ptr() if idx is not None else None, 0 if idx is None else idx.numel()),
                                   (ci, tpos, idx))
                if rc == _lib.ERR_STALE:  # positions moved since the index: bin them this call
                    self._cindex = None  # rebuilt next call if they are still in cell order
                    w.copy_(w0) if w0 is not None else w.fill_(-1)
                    u.copy_(u0) if u0 is not None else u.zero_()
                else:
                    _lib.check(rc)
            if rc == _lib.ERR_STALE:
                if ci is None and fresh:
                    w.fill_(-1)
                    u.zero_()
                _lib.check(L.swarm_allocate(
                    _lib.ctx(), self.n, p(self.ids), p(self.pos), p(self.caps), t,
                    p(tpos), p(tq), float(claim_thr), float(hysteresis), float(u_scale), m,
                    p(w), p(u), p(won), p(idx),
                    0 if idx is None else idx.numel(), p(nclaim), p(nmsg),
                    ctypes.byref(st), _lib.stream()))
        stats = {k: getattr(st, k) for k, _ in _lib.AllocStats._fields_}
        return AllocResult(w, u, won, nclaim, nmsg, stats)

    def _allocate_again(self, tx, ty, treq, claim_thr, hysteresis, u_scale):
        """The previous fresh, trusted-index allocation repeated (the same task tensors at the same
        versions, the same swarm arrays and position version, the same thresholds, on the same device):
        one libswarm call with its arguments kept from that call -- none of allocate()'s per-call Python
        (task stacking, index checks, device context, pointer validation).  None when anything differs."""
        c = getattr(self, "_again", None)
        if c is None:
            return None
        k = c[0]
        if not (k[0] is tx and k[1] is ty and k[2] is treq and k[4] is self.pos and k[6] is self.ids
                and k[7] is self.caps and k[3] == (tx._version, ty._version, treq._version)
                and k[5] == self.pos._version and k[8] == (claim_thr, hysteresis, u_scale)
                and k[9] == torch.cuda.current_device() and c[3][0] is self._cindex
                and c[3][2] is self._id_index):
            return None
        a = c[1]
        t, n = a[6], self.n
        # the four outputs carved from ONE allocation (one caching-allocator call instead of four):
        # util (f64), nclaim + nmsg (i64), winner (i32), won (i32), each 8-byte aligned
        buf = torch.empty(24 * t + 4 * t + 4 * n + 8, dtype=torch.uint8, device=self.device)
        b0 = buf.data_ptr()
        u = buf[:8 * t].view(torch.float64)
        nc_nm = buf[8 * t:24 * t].view(torch.int64).view(2, t)
        w = buf[24 * t:28 * t].view(torch.int32)
        o_won = (28 * t + 7) & ~7
        won = buf[o_won:o_won + 4 * n].view(torch.int32)
        st = _lib.AllocStats()
        _lib.check(_lib.lib().swarm_allocate_indexed_ex(_lib.ctx(), *a, b0 + 24 * t, b0, b0 + o_won, *c[2],
                                                        b0 + 8 * t, b0 + 16 * t, ctypes.byref(st), _lib.stream()))
        return AllocResult(w, u, won, nc_nm[0], nc_nm[1], {k_: getattr(st, k_) for k_, _ in _lib.AllocStats._fields_})

    def _task_pos(self, tx, ty) -> torch.Tensor:
        """(t, 2) float64 task positions on the device.  When tx / ty are float64 device tensors the
        stacked copy is kept and reused while both are unchanged (the same tensor objects at the
        same version counters): a caller that allocates over the same tasks every step pays no
        stacking kernel."""
        dev = self.device
        if isinstance(tx, torch.Tensor) and isinstance(ty, torch.Tensor) and tx.dtype == ty.dtype == torch.float64 \
                and tx.device == ty.device == dev:
            # the SAME tensor objects (held by the cache, so their storage cannot be recycled) at
            # the same version counters
            c = getattr(self, "_tpos_cache", None)
            if c is not None and c[0] is tx and c[1] is ty and c[2] == (tx._version, ty._version):
                return c[3]
            tpos = torch.stack([tx, ty], 1).contiguous()
            self._tpos_cache = (tx, ty, (tx._version, ty._version), tpos)
            return tpos
        return torch.stack([_to(tx, torch.float64, dev), _to(ty, torch.float64, dev)], 1).contiguous()

    def auction(self, tx, ty, treq, *, eps: float = 0.1, claim_thr: float = 20.0, u_scale: float = 100.0,
                max_rounds: int = 1 << 20) -> AuctionResult:
        """Auction allocation over the admissible pairs (swarm_auction; SURVEY §8f f4, the north
        star's auction price update): one task per agent, highest bid wins, ties to the lowest
        ID.  No reference counterpart; parity against oracle.auction."""
        dev = self.device
        tpos = torch.stack([_to(tx, torch.float64, dev), _to(ty, torch.float64, dev)], 1).contiguous()
        tq = _to(treq, torch.int8, dev)
        t = tq.numel()
        owner = torch.empty(max(t, 1), dtype=torch.int32, device=dev)
        price = torch.empty(max(t, 1), dtype=torch.float32, device=dev)
        assigned = torch.empty(max(self.n, 1), dtype=torch.int32, device=dev)
        rounds = ctypes.c_int32(0)
        bidders = np.zeros(int(max_rounds), np.int64)
        st = _lib.AuctionStats()
        with torch.cuda.device(dev):
            rc = _lib.check(_lib.lib().swarm_auction(
                _lib.ctx(), self.n, _lib.ptr(self.ids), _lib.ptr(self.pos), _lib.ptr(self.caps), t,
                _lib.ptr(tpos), _lib.ptr(tq), float(claim_thr), float(u_scale), float(eps), int(max_rounds),
                _lib.ptr(owner), _lib.ptr(price), _lib.ptr(assigned), ctypes.byref(rounds),
                bidders.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), _lib.stream()))
        r = rounds.value
        stats = {k: getattr(st, k) for k, _ in _lib.AuctionStats._fields_}
        return AuctionResult(owner[:t], price[:t], assigned[: self.n], r, bidders[:r].copy(), rc == _lib.OK, stats)

    # ------------------------------------------------------------------ physics
    def leader_index(self, leader: torch.Tensor | None = None) -> torch.Tensor:
        """Storage index of each FOLLOWER's leader (-1 for leaders / unknown IDs), from the
        election's leader IDs (self.leader after elect())."""
        leader = self.leader if leader is None else _to(leader, torch.int32, self.device)
        out = torch.full((self.n,), -1, dtype=torch.int32, device=self.device)
        idx = self.id_index()
        if idx is None or self.n == 0:
            srt, order = torch.sort(self.ids.long())
            pos = torch.searchsorted(srt, leader.long()).clamp(max=max(self.n - 1, 0))
            hit = srt[pos] == leader.long()
            cand = torch.where(hit, order[pos].int(), out)
        else:
            ok = (leader >= 0) & (leader < idx.numel())
            cand = torch.where(ok, idx[leader.clamp(0, idx.numel() - 1).long()], out)
        return torch.where(self.state == _lib.FOLLOWER, cand, out).contiguous()

    def physics_step(self, obstacles=None, *, sensors=None, leader_index=None, dt: float = 0.1,
                     max_speed: float = 5.0, steps: int = 1) -> dict:
        """`steps` synchronous _update_physics steps (agent.py:94-181) of every agent, in place on
        self.pos (contract P1; swarm_physics_step).  obstacles: (m, 3) [x, y, r]; sensors:
        (row_ptr, col) over storage indices (default: the neighbour graph); leader_index:
        default self.leader_index().  Velocity / target state lives on the Swarm."""
        dev, n = self.device, self.n
        if not hasattr(self, "vel"):
            self.vel = torch.zeros((n, 2), dtype=torch.float64, device=dev)
            self.target = torch.zeros((n, 2), dtype=torch.float64, device=dev)
            self.has_target = torch.zeros(n, dtype=torch.uint8, device=dev)
        obs = torch.zeros((0, 3), dtype=torch.float64, device=dev) if obstacles is None else \
            _to(obstacles, torch.float64, dev).reshape(-1, 3).contiguous()
        rp, col = sensors if sensors is not None else (self.row_ptr, self.col)
        if rp is None:
            raise RuntimeError("no sensor graph: pass sensors=(row_ptr, col) or build_graph()")
        rp, col = _to(rp, torch.int32, dev), _to(col, torch.int32, dev)
        li = self.leader_index() if leader_index is None else _to(leader_index, torch.int32, dev)
        other = torch.empty_like(self.pos)
        sing = ctypes.c_int64(0)
        total = 0
        with torch.cuda.device(dev):
            for _ in range(int(steps)):
                _lib.check(_lib.lib().swarm_physics_step(
                    _lib.ctx(), n, _lib.ptr(self.ids), _lib.ptr(self.state), _lib.ptr(li), _lib.ptr(self.pos),
                    _lib.ptr(other), _lib.ptr(self.vel), _lib.ptr(self.target), _lib.ptr(self.has_target),
                    obs.shape[0], _lib.ptr(obs) if obs.numel() else None, _lib.ptr(rp), _lib.ptr(col) if col.numel() else None,
                    float(dt), float(max_speed), ctypes.byref(sing), _lib.stream()))
                total += sing.value
                self.pos, other = other, self.pos
                self._cindex = None  # agents moved: the storage order is no longer their cell order
        return {"singular": total}

    # ------------------------------------------------------------------ timer FSM (f2)
    def _storage(self, a, dtype):
        """Per-agent array in INPUT order -> storage order on the device."""
        t = _to(a, dtype, self.device)
        if t.numel() != self.n:
            raise ValueError(f"expected {self.n} values, got {t.numel()}")
        return t[self.perm.long()].contiguous() if self.layout != "input" else t

    def protocol_reset(self, tick_off=None, last_hb=None):
        """Every agent as SwarmAgent.__init__ leaves it (agent.py:31-39): FOLLOWER, no leader,
        no leader position, alive, nothing in flight; last_heartbeat_time = last_hb (input
        order, default 0.0 = the clock at tick 0); tick_off: each agent's tick-counter phase
        (input order, default 0 = lock-step).  Tick counter restarts at 0."""
        n, dev = self.n, self.device
        z = lambda dt: torch.zeros(n, dtype=dt, device=dev)  # noqa: E731
        self.state.fill_(_lib.FOLLOWER)
        self.leader.fill_(-1)
        self.fsm = dict(last_hb=z(torch.float64) if last_hb is None else self._storage(last_hb, torch.float64),
                        wait_start=z(torch.float64), delay=z(torch.float64),
                        leader_pos=torch.zeros((n, 2), dtype=torch.float32, device=dev),
                        has_leader_pos=z(torch.uint8), alive=torch.ones(n, dtype=torch.uint8, device=dev),
                        outbox=torch.zeros(2 * n, dtype=torch.uint8, device=dev))
        self.tick_off = z(torch.int32) if tick_off is None else self._storage(tick_off, torch.int32)
        self.fsm_tick = 0
        return self

    def protocol_run(self, ticks: int, *, kill_ticks=(), dt: float = 0.1, timeout: float = 3.0,
                     jitter: float = 0.2, seed: int = 0, mode: str = "hybrid", pull_frac: float = 0.125,
                     traffic: bool = False) -> np.ndarray:
        """Advance the timer FSM + election handlers `ticks` ticks under contract T1
        (swarm_protocol_run; agent.py:66-80, 217-289), messages along the neighbour graph.
        kill_ticks: absolute ticks at whose start every alive LEADER dies.  Returns counts
        (ticks x 4): alive LEADERs, alive ELECTION_WAITs, ACCLAIM senders, HEARTBEAT senders.
        mode "push": senders mark their hearers and only marked agents scan their row; "pull":
        every agent scans its row every tick; "hybrid": push, but a tick in which a workgroup's
        senders exceed pull_frac x its share of the agents (a timeout wave) has the next tick pull
        (swarm_protocol_run_ex).  Same results.
        traffic: count what the ticks touched (self.fsm_traffic: 8 int64, see include/swarm.h)."""
        if self.row_ptr is None:
            raise RuntimeError("no neighbour graph: call build_graph() or set_graph()")
        if not hasattr(self, "fsm"):
            self.protocol_reset()
        f = self.fsm
        fs = _lib.Fsm(*[_lib.ptr(t) if self.n else None for t in
                        (self.state, self.leader, f["last_hb"], f["wait_start"], f["delay"], f["leader_pos"],
                         f["has_leader_pos"], f["alive"], f["outbox"])])
        kt = np.ascontiguousarray(np.asarray(kill_ticks, np.int64))
        if mode not in ("push", "pull", "hybrid"):
            raise ValueError(f"unknown mode {mode!r}")
        h = getattr(self, "_hear", None) or (self.row_ptr, self.col)
        hear = (None, None) if mode == "pull" or self.n == 0 else \
            (_lib.ptr(h[0], torch.int32), _lib.ptr(h[1], torch.int32) if h[1].numel() else None)
        counts = np.zeros((int(ticks), 4), np.int64)
        tr = np.zeros(8, np.int64)
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().swarm_protocol_run_ex(
                _lib.ctx(), self.n, _lib.ptr(self.ids) if self.n else None, _lib.ptr(self.pos) if self.n else None,
                _lib.ptr(self.row_ptr, torch.int32), _lib.ptr(self.col, torch.int32) if self.n_edges else None,
                *hear, _lib.ptr(self.tick_off) if self.n else None, ctypes.byref(fs), self.fsm_tick, int(ticks),
                float(dt), float(timeout), float(jitter), ctypes.c_uint64(int(seed)),
                kt.ctypes.data_as(ctypes.c_void_p) if kt.size else None, kt.size,
                float(pull_frac) if mode == "hybrid" else -1.0, counts.ctypes.data_as(ctypes.c_void_p),
                tr.ctypes.data_as(ctypes.c_void_p) if traffic else None, _lib.stream()))
        if traffic:
            self.fsm_traffic = tr
        self.fsm_tick += int(ticks)
        return counts

    # ------------------------------------------------------------------ views / bridge
    def to_input_order(self, storage_tensor) -> np.ndarray:
        """Host copy of a per-agent tensor re-ordered to the caller's input numbering."""
        a = storage_tensor.cpu().numpy()
        out = np.empty_like(a)
        out[self.perm.cpu().numpy()] = a
        return out

    @classmethod
    def from_agents(cls, agents, neighbors=None, cap_vocab=CAP_VOCAB_DEFAULT, device=None, layout="spatial"):
        """Batch a population of agent.SwarmAgent objects (drop-in bridge).

        neighbors: list of neighbour-index lists (who agent i hears), or None to build the
        radius-1 graph from positions on the GPU."""
        if len(cap_vocab) > CAP_UNHELD_BIT:
            raise ValueError(f"at most {CAP_UNHELD_BIT} capability names (bit {CAP_UNHELD_BIT} is reserved for "
                             f"capabilities no agent holds), got {len(cap_vocab)}")
        vocab = {c: k for k, c in enumerate(cap_vocab)}
        ids = np.array([a.agent_id for a in agents], np.int32)
        x = np.array([a.position[0] for a in agents], np.float64)
        y = np.array([a.position[1] for a in agents], np.float64)
        caps = np.zeros(len(agents), np.uint32)
        for i, a in enumerate(agents):
            for c in a.capabilities:
                if c not in vocab:
                    raise ValueError(f"capability {c!r} not in the vocabulary {cap_vocab}")
                caps[i] |= np.uint32(1 << vocab[c])
        sw = cls(ids, x, y, caps, device=device, layout=layout)
        sw.cap_vocab = tuple(cap_vocab)
        if neighbors is None:
            sw.build_graph(1.0)
        else:
            rp = np.zeros(len(agents) + 1, np.int64)
            rp[1:] = np.cumsum([len(nb) for nb in neighbors])
            col = np.array([j for nb in neighbors for j in nb], np.int64)
            sw.set_graph(rp, col)
        return sw

    def write_back_election(self, agents, result: ElectResult):
        """Set leader_id / state on the agent objects as the E2 rounds leave them."""
        from agent import AgentState  # the drop-in scalar module
        lead = self.to_input_order(result.leader)
        st = self.to_input_order(result.state)
        for i, a in enumerate(agents):
            a.leader_id = int(lead[i])
            a.state = AgentState(int(st[i]))

    def tasks_from_dict(self, tasks: dict):
        """(task_ids, tx, ty, treq) arrays from a reference-style task dict."""
        vocab = {c: k for k, c in enumerate(getattr(self, "cap_vocab", CAP_VOCAB_DEFAULT))}
        tid = np.array(list(tasks.keys()), np.int64)
        tx = np.array([tasks[k]["pos"][0] for k in tid], np.float64)
        ty = np.array([tasks[k]["pos"][1] for k in tid], np.float64)
        # a required cap outside the vocabulary blocks every agent: the reserved bit no agent holds
        treq = np.array([vocab.get(tasks[k]["required_cap"], CAP_UNHELD_BIT) if "required_cap" in tasks[k] else -1
                         for k in tid], np.int8)
        return tid, tx, ty, treq

    def write_back_allocation(self, agents, task_ids, res: AllocResult, resolver=None):
        """Statuses every agent holds after full TASK_CONFLICT delivery, and the resolver's
        task_claims table (agent.py:320)."""
        winner = res.winner.cpu().numpy()
        util = res.util.cpu().numpy()
        nmsg = res.nmsg.cpu().numpy()
        nclaim = res.nclaim.cpu().numpy()
        for a in agents:
            for k, tid in enumerate(task_ids):
                task = a.tasks.get(int(tid))
                if task is None:
                    continue
                if nmsg[k] > 0:
                    task["status"] = "ASSIGNED" if a.agent_id == winner[k] else "LOCKED"
                elif nclaim[k] > 0 and a.agent_id == winner[k]:
                    task["status"] = "TENTATIVE"  # lone rejected claim of the incumbent
        if resolver is not None:
            for k, tid in enumerate(task_ids):
                if winner[k] >= 0:
                    resolver.task_claims[int(tid)] = {"winner": int(winner[k]), "utility": float(util[k])}
