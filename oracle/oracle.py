"""CPU oracle for the swarm step -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module.  It is the checker, never the thing measured or shipped: the product path
(``swarm_amd``) never imports it.

Two restatements of the reference (``agent.py``, see swarm_oracle.c's header for the
file:line map):
  * ``liboracle.so`` (swarm_oracle.c, OpenMP) for every size the tests use;
  * pure-Python loops (``*_py``) for tiny cases, written straight from the handlers.
Both are pinned against tests/golden/ (generated from the reference's own handlers by
tools/gen_golden.py) in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import math
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OPEN, TENTATIVE, LOCKED, ASSIGNED = 0, 1, 2, 3
FOLLOWER, ELECTION_WAIT, LEADER = 1, 2, 3

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        l, d, i = ctypes.c_long, ctypes.c_double, ctypes.c_int
        L.orc_elect.restype = l
        L.orc_elect.argtypes = [l, P, P, P, P, P, l, P]
        L.orc_elect_frontier.restype = l
        L.orc_elect_frontier.argtypes = [l, P, P, P, P, P, P, P, l, P, P]
        L.orc_allocate_binned.restype = l
        L.orc_allocate_binned.argtypes = [l, P, P, P, P, l, P, P, P, d, d, d, i, P, P, P, P, P]
        L.orc_utility.restype = None
        L.orc_utility.argtypes = [l, P, P, P, P, P, P, d, i, P]
        L.orc_allocate.restype = l
        L.orc_allocate.argtypes = [l, P, P, P, P, l, P, P, P, d, d, d, i, P, P, P, P, P]
        L.orc_task_claims.restype = l
        L.orc_task_claims.argtypes = [l, P, P, P, P, d, d, ctypes.c_int8, d, d, i, P, P, l]
        L.orc_protocol.restype = None
        L.orc_protocol.argtypes = [l, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, l, l, d, d, d,
                                   ctypes.c_uint64, P, l, P]
        L.orc_rgg_csr.restype = l
        L.orc_rgg_csr.argtypes = [l, P, P, d, P, P]
        L.orc_auction.restype = l
        L.orc_auction.argtypes = [l, P, P, P, P, l, P, P, P, d, d, i, ctypes.c_float, l, P, P, P, P, P]
        L.orc_physics.restype = l
        L.orc_physics.argtypes = [l, P, P, P, P, P, P, P, P, P, P, l, P, P, P, d, d, l, i]
        L.orc_num_threads.restype = i
        L.orc_set_threads.argtypes = [i]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def set_threads(n: int):
    lib().orc_set_threads(int(n))


def num_threads() -> int:
    return int(lib().orc_num_threads())


def elect(row_ptr, col, ids, max_rounds=1 << 20):
    """E2 election to convergence -> (leader int32, state uint8, rounds_exec, changes int64)."""
    ids = _c(ids, np.int32)
    n = len(ids)
    rp = _c(row_ptr, np.int64)
    cl = _c(col, np.int32)
    leader = np.empty(n, np.int32)
    state = np.empty(n, np.uint8)
    changes = np.zeros(max(1, min(max_rounds, 1 << 20)), np.int64)
    r = lib().orc_elect(n, _p(rp), _p(cl), _p(ids), _p(leader), _p(state), len(changes), _p(changes))
    return leader, state, int(r), changes[: max(r, 0)].copy()


def elect_frontier(row_ptr, col, ids, hear=None, max_rounds=1 << 20, with_active=False):
    """E2 election by the frontier restatement (orc_elect_frontier): same outputs as elect();
    hear = (row_ptr, col) of the transpose graph (who hears each agent), None when symmetric.
    with_active: also return the agents recomputed per round."""
    ids = _c(ids, np.int32)
    n = len(ids)
    rp = _c(row_ptr, np.int64)
    cl = _c(col, np.int32)
    hp, hc = (None, None) if hear is None else (_c(hear[0], np.int64), _c(hear[1], np.int32))
    leader = np.empty(n, np.int32)
    state = np.empty(n, np.uint8)
    cap = max(1, min(max_rounds, 1 << 20))
    changes = np.zeros(cap, np.int64)
    active = np.zeros(cap, np.int64)
    r = lib().orc_elect_frontier(n, _p(rp), _p(cl), None if hp is None else _p(hp), None if hc is None else _p(hc),
                                 _p(ids), _p(leader), _p(state), cap, _p(changes), _p(active))
    k = r if r > 0 else cap
    out = (leader, state, int(r), changes[:max(r, 0)].copy())
    return out + (active[:k].copy(),) if with_active else out


def transpose_csr(row_ptr, col, n=None):
    """(row_ptr, col) of the transpose graph, rows ascending (who hears each agent)."""
    rp = np.asarray(row_ptr, np.int64)
    cl = np.asarray(col, np.int64)
    n = len(rp) - 1 if n is None else n
    src = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    o = np.lexsort((src, cl))
    trp = np.zeros(n + 1, np.int64)
    trp[1:] = np.cumsum(np.bincount(cl, minlength=n))
    return trp, src[o].astype(np.int32)


def utility(ax, ay, caps, tx, ty, treq, use_pow=True, u_scale=100.0):
    """Elementwise utility of (agent_i, task_i) pairs (agent.py:338-347), fp64."""
    arrs = [_c(ax, np.float64), _c(ay, np.float64), _c(caps, np.uint32), _c(tx, np.float64),
            _c(ty, np.float64), _c(treq, np.int8)]
    out = np.empty(len(arrs[0]), np.float64)
    lib().orc_utility(len(out), *[_p(a) for a in arrs], u_scale, int(use_pow), _p(out))
    return out


def allocate(ids, ax, ay, caps, tx, ty, treq, winner=None, util=None, claim_thr=20.0,
             hysteresis=5.0, u_scale=100.0, use_pow=True):
    """A-H allocation -> dict(winner, util, nclaim, nmsg, won, n_claims, n_conflicts)."""
    ids = _c(ids, np.int32)
    n, t = len(ids), len(tx)
    w = np.full(t, -1, np.int32) if winner is None else _c(winner, np.int32).copy()
    u = np.zeros(t, np.float64) if util is None else _c(util, np.float64).copy()
    nclaim = np.zeros(t, np.int64)
    nmsg = np.zeros(t, np.int64)
    won = np.zeros(n, np.int32)
    arrs = [_c(ax, np.float64), _c(ay, np.float64), _c(caps, np.uint32)]
    tarr = [_c(tx, np.float64), _c(ty, np.float64), _c(treq, np.int8)]
    total = lib().orc_allocate(n, _p(ids), *[_p(a) for a in arrs], t, *[_p(a) for a in tarr],
                               claim_thr, hysteresis, u_scale, int(use_pow), _p(w), _p(u),
                               _p(nclaim), _p(nmsg), _p(won))
    return dict(winner=w, util=u, nclaim=nclaim, nmsg=nmsg, won=won, n_claims=int(total),
                n_conflicts=int(nmsg.sum()))


def allocate_binned(ids, ax, ay, caps, tx, ty, treq, winner=None, util=None, claim_thr=20.0,
                    hysteresis=5.0, u_scale=100.0, use_pow=True):
    """allocate() evaluating only the agents inside the claim radius (orc_allocate_binned):
    same outputs, the CPU counterpart of the GPU's binned strategy."""
    ids = _c(ids, np.int32)
    n, t = len(ids), len(tx)
    w = np.full(t, -1, np.int32) if winner is None else _c(winner, np.int32).copy()
    u = np.zeros(t, np.float64) if util is None else _c(util, np.float64).copy()
    nclaim = np.zeros(t, np.int64)
    nmsg = np.zeros(t, np.int64)
    won = np.zeros(n, np.int32)
    arrs = [_c(ax, np.float64), _c(ay, np.float64), _c(caps, np.uint32)]
    tarr = [_c(tx, np.float64), _c(ty, np.float64), _c(treq, np.int8)]
    total = lib().orc_allocate_binned(n, _p(ids), *[_p(a) for a in arrs], t, *[_p(a) for a in tarr],
                                      claim_thr, hysteresis, u_scale, int(use_pow), _p(w), _p(u),
                                      _p(nclaim), _p(nmsg), _p(won))
    return dict(winner=w, util=u, nclaim=nclaim, nmsg=nmsg, won=won, n_claims=int(total),
                n_conflicts=int(nmsg.sum()))


def auction(ids, ax, ay, caps, tx, ty, treq, eps=0.1, claim_thr=20.0, u_scale=100.0, use_pow=False,
            max_rounds=1 << 20):
    """Jacobi auction over the admissible pairs (swarm_oracle.c orc_auction) -> dict(owner, price,
    assigned, rounds, bidders, n_pairs).  use_pow=False: the GPU's x*x utility arithmetic."""
    ids = _c(ids, np.int32)
    n, t = len(ids), len(tx)
    owner = np.empty(t, np.int32)
    price = np.empty(t, np.float32)
    assigned = np.empty(n, np.int32)
    bidders = np.zeros(max(1, min(max_rounds, 1 << 20)), np.int64)
    npairs = np.zeros(1, np.int64)
    arrs = [_c(ax, np.float64), _c(ay, np.float64), _c(caps, np.uint32)]
    tarr = [_c(tx, np.float64), _c(ty, np.float64), _c(treq, np.int8)]
    r = lib().orc_auction(n, _p(ids), *[_p(a) for a in arrs], t, *[_p(a) for a in tarr], claim_thr,
                          u_scale, int(use_pow), float(eps), len(bidders), _p(owner), _p(price),
                          _p(assigned), _p(bidders), _p(npairs))
    return dict(owner=owner, price=price, assigned=assigned, rounds=int(r),
                bidders=bidders[: max(r, 0)].copy(), n_pairs=int(npairs[0]))


def physics(ids, state, leader, x, y, vx, vy, tx, ty, has_t, obs, row_ptr, col, dt=0.1, max_speed=5.0,
            steps=1, use_pow=True):
    """Physics steps under contract P1 (swarm_oracle.c orc_physics) -> dict of the new state
    (x, y, vx, vy, tx, ty, has_t) and `singular` (reference ZeroDivisionError cases)."""
    o = dict(x=_c(x, np.float64).copy(), y=_c(y, np.float64).copy(), vx=_c(vx, np.float64).copy(),
             vy=_c(vy, np.float64).copy(), tx=_c(tx, np.float64).copy(), ty=_c(ty, np.float64).copy(),
             has_t=_c(has_t, np.uint8).copy())
    ids = _c(ids, np.int32)
    obs = _c(np.asarray(obs, np.float64).reshape(-1, 3), np.float64)
    sing = lib().orc_physics(len(ids), _p(ids), _p(_c(state, np.uint8)), _p(_c(leader, np.int32)), _p(o["x"]),
                             _p(o["y"]), _p(o["vx"]), _p(o["vy"]), _p(o["tx"]), _p(o["ty"]), _p(o["has_t"]),
                             len(obs), _p(obs), _p(_c(row_ptr, np.int64)), _p(_c(col, np.int32)), float(dt),
                             float(max_speed), int(steps), int(use_pow))
    o["singular"] = int(sing)
    return o


def protocol(ids, x, y, row_ptr, col, tick_off, ticks, *, state=None, leader=None, last_hb=None,
             wait_start=None, delay=None, lpos=None, has_lpos=None, alive=None, outbox=None, t0=0, dt=0.1,
             timeout=3.0, jitter=0.2, seed=0, kill_ticks=()):
    """Timer FSM ticks t0+1 .. t0+ticks under contract T1 (swarm_oracle.c orc_protocol) -> dict
    of the state after the last tick and counts (ticks x 4).  Defaults: the reference's initial
    agent (FOLLOWER, no leader, last_heartbeat_time 0, alive)."""
    n = len(ids)
    o = dict(state=np.full(n, FOLLOWER, np.uint8) if state is None else _c(state, np.uint8).copy(),
             leader=np.full(n, -1, np.int32) if leader is None else _c(leader, np.int32).copy(),
             last_hb=np.zeros(n) if last_hb is None else _c(last_hb, np.float64).copy(),
             wait_start=np.zeros(n) if wait_start is None else _c(wait_start, np.float64).copy(),
             delay=np.zeros(n) if delay is None else _c(delay, np.float64).copy(),
             lpos=np.zeros((n, 2), np.float32) if lpos is None else _c(lpos, np.float32).reshape(n, 2).copy(),
             has_lpos=np.zeros(n, np.uint8) if has_lpos is None else _c(has_lpos, np.uint8).copy(),
             alive=np.ones(n, np.uint8) if alive is None else _c(alive, np.uint8).copy(),
             outbox=np.zeros(2 * n, np.uint8) if outbox is None else _c(outbox, np.uint8).copy())
    kt = _c(np.asarray(kill_ticks, np.int64), np.int64)
    counts = np.zeros((int(ticks), 4), np.int64)
    lib().orc_protocol(n, _p(_c(ids, np.int32)), _p(_c(x, np.float64)), _p(_c(y, np.float64)),
                       _p(_c(row_ptr, np.int64)), _p(_c(col, np.int32)), _p(_c(tick_off, np.int32)),
                       _p(o["state"]), _p(o["leader"]), _p(o["last_hb"]), _p(o["wait_start"]), _p(o["delay"]),
                       _p(o["lpos"]), _p(o["has_lpos"]), _p(o["alive"]), _p(o["outbox"]), int(t0), int(ticks),
                       float(dt), float(timeout), float(jitter), ctypes.c_uint64(int(seed)), _p(kt), len(kt),
                       _p(counts))
    o["counts"] = counts
    return o


def task_claims(ids, ax, ay, caps, tx, ty, treq, claim_thr=20.0, u_scale=100.0, use_pow=True):
    """Claims on one task in ascending-ID order -> (ids int32, f32 values)."""
    ids = _c(ids, np.int32)
    n = len(ids)
    oid = np.empty(n, np.int32)
    ox = np.empty(n, np.float32)
    m = lib().orc_task_claims(n, _p(ids), _p(_c(ax, np.float64)), _p(_c(ay, np.float64)),
                              _p(_c(caps, np.uint32)), float(tx), float(ty), int(treq), claim_thr,
                              u_scale, int(use_pow), _p(oid), _p(ox), n)
    return oid[:m].copy(), ox[:m].copy()


def rgg_csr(x, y, radius=1.0):
    """Radius graph over storage indices (rows ascending) -> (row_ptr int64, col int32)."""
    x = _c(x, np.float64)
    y = _c(y, np.float64)
    n = len(x)
    rp = np.zeros(n + 1, np.int64)
    e = lib().orc_rgg_csr(n, _p(x), _p(y), radius, _p(rp), None)
    col = np.empty(max(e, 1), np.int32)
    lib().orc_rgg_csr(n, _p(x), _p(y), radius, _p(rp), _p(col))
    return rp, col[:e].copy()


def statuses(ids, winner, nmsg, claimed=None):
    """Per-agent task status after full TASK_CONFLICT delivery (agent.py:327-336).

    A task with >= 1 conflict message ends ASSIGNED for the final winner and LOCKED for every
    other agent (the last message names the final winner); with none it stays as the claim
    phase left it: TENTATIVE where the agent claimed (``claimed[i, k]``), else OPEN."""
    ids = np.asarray(ids)
    n, t = len(ids), len(winner)
    st = np.zeros((n, t), np.uint8)
    if claimed is not None:
        st[claimed] = TENTATIVE
    has = np.asarray(nmsg) > 0
    st[:, has] = LOCKED
    win = (ids[:, None] == np.asarray(winner)[None, :]) & has[None, :]
    st[win] = ASSIGNED
    return st


# ------------------------------------------------------------------ pure-Python restatements

def elect_py(row_ptr, col, ids, max_rounds=100000):
    """Straight restatement of the E2 rounds (tiny inputs only)."""
    n = len(ids)
    leader = [int(i) for i in ids]
    changes = []
    for _ in range(max_rounds):
        snap = list(leader)
        for v in range(n):
            for u in col[row_ptr[v]:row_ptr[v + 1]]:
                if snap[u] > leader[v]:
                    leader[v] = snap[u]
        c = sum(1 for v in range(n) if leader[v] != snap[v])
        changes.append(c)
        if c == 0:
            break
    state = [LEADER if leader[v] == ids[v] else FOLLOWER for v in range(n)]
    return np.array(leader, np.int32), np.array(state, np.uint8), len(changes), np.array(changes)


def utility_py(ax, ay, caps, tx, ty, treq, u_scale=100.0):
    dist = math.sqrt((ax - tx) ** 2 + (ay - ty) ** 2)
    has = 0.0 if (treq >= 0 and not (int(caps) >> int(treq)) & 1) else 1.0
    return (u_scale / (1.0 + dist)) * has


def f32(x: float) -> float:
    return struct.unpack("!f", struct.pack("!f", x))[0]


def allocate_py(ids, ax, ay, caps, tx, ty, treq, claim_thr=20.0, hysteresis=5.0):
    """Straight restatement of claim -> resolve (tiny inputs only)."""
    order = sorted(range(len(ids)), key=lambda i: int(ids[i]))
    winner, util, nmsg = [], [], []
    for k in range(len(tx)):
        w, u, m = -1, 0.0, 0
        for i in order:
            U = utility_py(float(ax[i]), float(ay[i]), caps[i], float(tx[k]), float(ty[k]), int(treq[k]))
            if U > claim_thr:
                x = f32(U)
                if w < 0 or x > u + hysteresis:
                    w, u, m = int(ids[i]), x, m + 1
                elif w != int(ids[i]):
                    m += 1
        winner.append(w)
        util.append(u)
        nmsg.append(m)
    return np.array(winner, np.int32), np.array(util), np.array(nmsg)


def auction_py(ids, ax, ay, caps, tx, ty, treq, eps=0.1, claim_thr=20.0, max_rounds=100000):
    """Straight restatement of the Jacobi auction (tiny inputs only): numpy float32 scalars
    carry the f32 arithmetic, the x*x utility as on the GPU."""
    n, t = len(ids), len(tx)
    f = np.float32
    cand = []
    for a in range(n):
        row = []
        for k in range(t):
            dx, dy = float(ax[a]) - float(tx[k]), float(ay[a]) - float(ty[k])
            d = math.sqrt(dx * dx + dy * dy)
            has = 0.0 if (int(treq[k]) >= 0 and not (int(caps[a]) >> int(treq[k])) & 1) else 1.0
            U = (100.0 / (1.0 + d)) * has
            if U > claim_thr:
                row.append((k, f(U)))
        cand.append(row)
    price = [f(0.0)] * t
    owner = [-1] * t
    assigned = [-1] * n
    out = [False] * n
    rounds, bidders = 0, []
    while rounds < max_rounds:
        bids = {}
        nb = 0
        for a in range(n):
            if assigned[a] >= 0 or out[a]:
                continue
            nb += 1
            best, second, bk = f(-np.inf), f(-np.inf), None
            for k, x in cand[a]:
                net = f(x - price[k])
                if net > best or (net == best and k < bk):
                    second, best, bk = max(second, best), net, k
                elif net > second:
                    second = net
            if not best > 0:
                out[a] = True
                continue
            second = max(second, f(0.0))
            bid = f(f(price[bk] + f(best - second)) + f(eps))
            key = (bid, -int(ids[a]))
            if bk not in bids or key > bids[bk][0]:
                bids[bk] = (key, a)
        if nb == 0:
            break
        bidders.append(nb)
        rounds += 1
        for k, (key, a) in bids.items():
            if owner[k] >= 0:
                assigned[owner[k]] = -1
            owner[k], assigned[a], price[k] = a, k, key[0]
    return dict(owner=np.array(owner, np.int32), price=np.array(price, np.float32),
                assigned=np.array(assigned, np.int32), rounds=rounds, bidders=np.array(bidders, np.int64))


# ----------------------------------------------------------------------------- wire codec (f3)
# Restatement of the transport framing: SwarmAgent._pack_header / _send_msg (agent.py:184-194),
# the senders' payloads (heartbeat '!ff' agent.py:283-289, acclaim '!B' 240, coordinator 241,
# claim '!If' 302, conflict '!IB' 322/325) and on_message_received's dispatch (agent.py:197-214)
# with the handlers' first unpack (256-258, 305, 328).  Pinned by tests/golden/codec_kat.npz.
HB, ACCLAIM, COORD, CLAIM, CONFLICT = 1, 2, 3, 4, 5


def codec_encode_py(typ, sender, tick, a, b, task, winner, wide=False):
    """Per message: status (0 ok, 1 struct.error, 2 OverflowError, 3 unknown type) and packet
    bytes (b"" on error).  Payload packed before the header, as the senders do."""
    idf = "I" if wide else "B"
    out_st, out_pk = [], []
    for ty, s, tk, x, y, t, w in zip(typ, sender, tick, a, b, task, winner):
        ty, s, tk, t, w = int(ty), int(s), int(tk), int(t), int(w)
        try:
            if ty == HB:
                pl = struct.pack("!ff", float(x), float(y))
            elif ty == ACCLAIM:
                pl = struct.pack("!" + idf, s)
            elif ty == COORD:
                pl = b""
            elif ty == CLAIM:
                pl = struct.pack("!If", t, float(x))
            elif ty == CONFLICT:
                pl = struct.pack("!I" + idf, t, w)
            else:
                out_st.append(3)
                out_pk.append(b"")
                continue
            pk = struct.pack("!B" + idf + "I", ty, s, tk) + pl
            out_st.append(0)
            out_pk.append(pk)
        except struct.error:
            out_st.append(1)
            out_pk.append(b"")
        except OverflowError:
            out_st.append(2)
            out_pk.append(b"")
    return np.array(out_st, np.int8), out_pk


def codec_decode_py(packets, wide=False):
    """Per packet: the receiver's dispatch.  status 0 handled, 1 dropped (< header), 2 unknown
    type, 3 the handler's unpack raises; fields as the handler sees them (0 where absent)."""
    hdr, idf = (9, "I") if wide else (6, "B")
    keys = ("status", "type", "sender", "tick", "task", "winner", "has_pos")
    rows = {k: [] for k in keys + ("a", "b")}
    for pk in packets:
        r = dict(status=1, type=0, sender=0, tick=0, task=0, winner=0, has_pos=0, a=0.0, b=0.0)
        if len(pk) >= hdr:
            r["type"], r["sender"], r["tick"] = struct.unpack("!B" + idf + "I", pk[:hdr])
            pl = pk[hdr:]
            r["status"] = 0
            if r["type"] == HB:
                if len(pl) == 8:
                    r["a"], r["b"] = struct.unpack("!ff", pl)
                    r["has_pos"] = 1
            elif r["type"] in (ACCLAIM, COORD):
                pass
            elif r["type"] == CLAIM:
                try:
                    r["task"], r["a"] = struct.unpack("!If", pl)
                except struct.error:
                    r["status"] = 3
            elif r["type"] == CONFLICT:
                try:
                    r["task"], r["winner"] = struct.unpack("!I" + idf, pl)
                except struct.error:
                    r["status"] = 3
            else:
                r["status"] = 2
        for k in rows:
            rows[k].append(r[k])
    out = {k: np.array(rows[k], np.int64) for k in keys}
    out["a"] = np.array(rows["a"], np.float32)
    out["b"] = np.array(rows["b"], np.float32)
    return out


def split_packets(buf, lens):
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    raw = bytes(np.asarray(buf, np.uint8))
    return [raw[off[i]:off[i + 1]] for i in range(len(lens))], off
