"""The batched election and allocation as registered PyTorch custom ops (torch.library).

    torch.ops.swarm_amd.elect(row_ptr, col, ids, col16, max_rounds, dense)
        -> (leader int32[n], state uint8[n], info int64[max_rounds + 2] on the host)
       contract E2 to convergence: SwarmAgent._handle_election_acclaim / _handle_heartbeat
       (agent.py:243-275) applied round by round; info = [rounds_exec, converged, changes of rounds
       1..rounds_exec, 0...].  Calls swarm_elect_compact (col16: swarm_graph_compact's columns of the same
       graph, or None for the int32 columns).
    torch.ops.swarm_amd.allocate(ids, pos, caps, tpos, treq, id_index, claim_thr, hysteresis, u_scale)
        -> (winner int32[t], util float64[t], won int32[n], nclaim int64[t], nmsg int64[t],
            stats int64[7] on the host)
       one claim/resolve round from fresh claims (contract A-H: _process_tasks / _handle_task_claim /
       _handle_task_conflict / _calculate_utility, agent.py:292-347); calls swarm_allocate.  stats =
       n_claims, n_conflicts, n_flagged, n_candidates, n_overflow, mode_used, n_resolved.

Both run on torch's current stream (the C-ABI takes it), so they order like any other op; their fake
(meta) implementations give the output shapes, so a caller's function that uses them traces under
torch.compile(fullgraph=True) with the op as one opaque node.  Same C-ABI calls and results as
Swarm.elect / Swarm.allocate (which add the storage-order bookkeeping and the cell-index fast path).
There is no CPU implementation: the ops are registered for the "cuda" device only.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

_STATS = ("n_claims", "n_conflicts", "n_flagged", "n_candidates", "n_overflow", "mode_used", "n_resolved")


@torch.library.custom_op("swarm_amd::elect", mutates_args=(), device_types="cuda")
def elect(row_ptr: torch.Tensor, col: torch.Tensor, ids: torch.Tensor, col16: Optional[torch.Tensor],
          max_rounds: int, dense: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    n = ids.numel()
    dev = ids.device
    leader = torch.empty(n, dtype=torch.int32, device=dev)
    state = torch.empty(n, dtype=torch.uint8, device=dev)
    info = torch.zeros(max_rounds + 2, dtype=torch.int64)
    rounds = ctypes.c_int32(0)
    P = _lib.ptr
    with torch.cuda.device(dev):
        rc = _lib.check(_lib.lib().swarm_elect_compact(
            _lib.ctx(), n, P(row_ptr, torch.int32, n + 1, "row_ptr"),
            P(col, torch.int32, name="col") if col.numel() else None,
            P(col16, torch.int16, name="col16") if col16 is not None and col16.numel() else None,
            P(ids, torch.int32, n, "ids") if n else None, P(leader) if n else None, P(state) if n else None,
            int(max_rounds), _lib.ELECT_DENSE if dense else _lib.ELECT_FRONTIER, ctypes.byref(rounds),
            ctypes.c_void_p(info.data_ptr() + 16), None, _lib.stream()))
    info[0] = rounds.value
    info[1] = 1 if rc == _lib.OK else 0
    return leader, state, info


@elect.register_fake
def _elect_fake(row_ptr, col, ids, col16, max_rounds, dense):
    n = ids.shape[0]
    return (torch.empty(n, dtype=torch.int32, device=ids.device), torch.empty(n, dtype=torch.uint8, device=ids.device),
            torch.empty(max_rounds + 2, dtype=torch.int64, device="cpu"))


@torch.library.custom_op("swarm_amd::allocate", mutates_args=(), device_types="cuda")
def allocate(ids: torch.Tensor, pos: torch.Tensor, caps: torch.Tensor, tpos: torch.Tensor, treq: torch.Tensor,
             id_index: Optional[torch.Tensor], claim_thr: float, hysteresis: float,
             u_scale: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor,
                                      torch.Tensor]:
    n, t = ids.numel(), treq.numel()
    dev = ids.device
    winner = torch.full((t,), -1, dtype=torch.int32, device=dev)
    util = torch.zeros(t, dtype=torch.float64, device=dev)
    won = torch.empty(n, dtype=torch.int32, device=dev)
    nclaim = torch.empty(t, dtype=torch.int64, device=dev)
    nmsg = torch.empty(t, dtype=torch.int64, device=dev)
    st = _lib.AllocStats()
    P = _lib.ptr
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().swarm_allocate(
            _lib.ctx(), n, P(ids, torch.int32, n, "ids") if n else None, P(pos, torch.float64, 2 * n, "pos") if n else None,
            P(caps, torch.int32, n, "caps") if n else None, t, P(tpos, torch.float64, 2 * t, "tpos") if t else None,
            P(treq, torch.int8, t, "treq") if t else None, float(claim_thr), float(hysteresis), float(u_scale),
            _lib.ALLOC_AUTO, P(winner) if t else None, P(util) if t else None, P(won) if n else None,
            P(id_index, torch.int32, name="id_index") if id_index is not None else None,
            0 if id_index is None else id_index.numel(), P(nclaim) if t else None, P(nmsg) if t else None,
            ctypes.byref(st), _lib.stream()))
    stats = torch.tensor([int(getattr(st, k)) for k in _STATS], dtype=torch.int64)
    return winner, util, won, nclaim, nmsg, stats


@allocate.register_fake
def _allocate_fake(ids, pos, caps, tpos, treq, id_index, claim_thr, hysteresis, u_scale):
    n, t, dev = ids.shape[0], treq.shape[0], ids.device
    return (torch.empty(t, dtype=torch.int32, device=dev), torch.empty(t, dtype=torch.float64, device=dev),
            torch.empty(n, dtype=torch.int32, device=dev), torch.empty(t, dtype=torch.int64, device=dev),
            torch.empty(t, dtype=torch.int64, device=dev), torch.empty(len(_STATS), dtype=torch.int64, device="cpu"))


def stats_dict(stats: torch.Tensor) -> dict:
    """The allocate op's stats tensor as Swarm.allocate's stats dict."""
    return dict(zip(_STATS, (int(v) for v in stats.tolist())))
