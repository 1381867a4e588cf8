"""The HIP sharded path across PROCESSES on one GPU.

Two (or three) processes share cuda:0 over gloo: each is one rank with the product backend
(GpuBackend: libswarm's frontier stepper, ghost and allocation kernels).  RCCL refuses two ranks on
one device, so the ranks talk through host memory, in two ways:
  transport "shm"     libswarm's NATIVE sharded C loops (swarm_elect_sharded, swarm_auction_sharded)
                      over its shared-memory transport (SWARM_COMM_SHM): the batching, the counter
                      all-reduce, the ghost application order and the convergence decision of the
                      code that runs over RCCL on a multi-GPU node;
  transport "shm-agent"  the same, with the tail's agent-order stamp layout forced from the second
                      batch of rounds on (SWARM_IL_MIN_CHANGES): the layout switch of the native loop;
  transport "rccl-double"  the native loops' RCCL branch (SWARM_NATIVE_COMM=rccl) over the RCCL test
                      double (tests/rccl_double via SWARM_RCCL_PATH): the ncclSend/ncclRecv groups, the
                      per-peer counts and datatypes, the ncclSum counter all-reduce and the auction's
                      MAX all-reduce / all-gather, with real peers on one GPU;
  transport "python"  SWARM_NATIVE_HALO=0: ShardedSwarm's Python stepper, halo over gloo.
Every rank's leaders, rounds and per-round global change counts, the sharded allocation (winners,
claim values, conflicts, won counts) and -- native -- the sharded auction (owners, prices, per-round
bidders) must equal the oracle over the union swarm.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(kind, world):
    from swarm_amd import gen
    if kind == "shards":  # weak-scaling inputs: rank k's strip holds the ID range [k n, (k+1) n)
        return [gen.shard_inputs(6_000, 41, world, r, t=120) for r in range(world)]
    if kind == "blocks":  # C5's shape: Morton blocks, Morton IDs, rank k's block = the ID range [k n, (k+1) n)
        return [gen.shard_inputs(6_000, 47, world, r, t=120, layout="blocks") for r in range(world)]
    # one global swarm, cut by ID range: strip-major IDs (strips), Morton IDs or random IDs (cells)
    ids = {"global": "random", "global-morton": "morton", "global-random": "random"}[kind]
    d = gen.swarm_inputs(12_000, 43, t=300, ids=ids)
    if kind == "global":
        d["ids"] = gen.strip_ids(d["y"], world, 43)
    return d


def _auction_tasks(kind, world):
    """The task list every rank passes to the sharded auction (tasks are replicated): all of them."""
    d = _inputs(kind, world)
    if kind in ("shards", "blocks"):
        return tuple(np.concatenate([e[k] for e in d]) for k in ("tx", "ty", "treq"))
    return d["tx"], d["ty"], d["treq"]


def _worker(rank, world, port, out_q, kind, depth, transport, dbl):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      SWARM_NATIVE_HALO="0" if transport == "python" else "1")
    if transport == "rccl-double":
        os.environ.update(SWARM_NATIVE_COMM="rccl", SWARM_RCCL_PATH=dbl, RCCL_DOUBLE_TIMEOUT_S="60")
    if transport == "shm-agent":  # the tail's agent-order stamp layout from the second batch on
        os.environ["SWARM_IL_MIN_CHANGES"] = str(1 << 40)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from swarm_amd.dist import GpuBackend, Rects, ShardedSwarm
        dev = torch.device("cuda", 0)
        if kind in ("shards", "blocks"):
            d = _inputs(kind, world)[rank]
            region = Rects(d["rects"], rank) if kind == "blocks" else d["strip"]
            sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], region, device=dev, halo_depth=depth)
            tx, ty, tq = d["tx"], d["ty"], d["treq"]
            tasks = None
        else:
            d = _inputs(kind, world)
            sh = ShardedSwarm.from_global(d["ids"], d["x"], d["y"], d["caps"], tx=d["tx"], ty=d["ty"], device=dev,
                                          halo_depth=depth, by="id")
            k = sh.part.tasks
            tx, ty, tq = d["tx"][k], d["ty"][k], d["treq"][k]
            tasks = k
        assert isinstance(sh.backend, GpuBackend) and sh.halo.host_staged
        r = sh.elect(check_every=16)
        native = getattr(sh, "_native", None) is not None
        want_kind = {"rccl-double": "rccl", "python": None}.get(transport, "shm")
        assert native == (transport != "python") and (not native or sh.backend.comm_kind == want_kind)
        sh._check_ghosts(sh.leaders[r.rounds_exec & 1])
        res, won, gst = sh.allocate(tx, ty, tq)
        auc = None
        if native:  # the native sharded auction over the same transport: agents sharded, tasks replicated
            a = sh.auction(*_auction_tasks(kind, world), native=True)
            auc = dict(owner=a.owner_id.cpu().numpy(), price=a.price.cpu().numpy(), bidders=a.bidders,
                       rounds=a.rounds_exec, ids=sh.ids.cpu().numpy(), assigned=a.assigned.cpu().numpy())
        torch.cuda.synchronize()
        dstats = None
        if transport == "rccl-double":  # what the double executed in this process (the RCCL branch ran)
            import ctypes
            D = ctypes.CDLL(dbl)
            st = (ctypes.c_longlong * 6)()
            D.rccl_double_stats(ctypes.cast(st, ctypes.c_void_p))
            dstats = list(st)
        out_q.put(dict(rank=rank, dstats=dstats, rounds=r.rounds_exec, changes=r.changes, ids=sh.ids.cpu().numpy(),
                       leader=r.leader.cpu().numpy(), state=r.state.cpu().numpy(), winner=res.winner.cpu().numpy(),
                       util=res.util.cpu().numpy(), nmsg=res.nmsg.cpu().numpy(), won=won.cpu().numpy(),
                       gstats=gst, tasks=tasks, converged=r.converged, ghosts=sh.n_glo + sh.n_ghi, native=native,
                       auc=auc, peers=list(sh.peers)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,depth,transport", [(2, "shards", 16, "python"), (2, "global", 4, "python"),
                                                         (3, "global", 16, "python"), (2, "shards", 16, "shm"),
                                                         (2, "global", 1, "shm"), (3, "global", 16, "shm"),
                                                         (3, "shards", 4, "shm"), (2, "global", 16, "shm-agent"),
                                                         (3, "shards", 1, "shm-agent"), (4, "blocks", 16, "shm"),
                                                         (3, "blocks", 5, "shm"), (2, "blocks", 8, "python"),
                                                         (3, "global-morton", 6, "shm"), (4, "global-morton", 16, "shm"),
                                                         (2, "global-random", 2, "shm"), (4, "global-random", 3, "shm"),
                                                         (3, "global-random", 2, "python"),
                                                         (2, "shards", 16, "rccl-double"),
                                                         (3, "global", 1, "rccl-double"),
                                                         (4, "blocks", 16, "rccl-double"),
                                                         (3, "global-morton", 6, "rccl-double"),
                                                         (4, "global-random", 3, "rccl-double")])
def test_hip_sharded_processes_match_union_oracle(world, kind, depth, transport, oracle_mod, rccl_double):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind, depth, transport, rccl_double))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = sorted([q.get(timeout=100) for _ in range(world)], key=lambda o: o["rank"])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    d = _inputs(kind, world)
    if kind in ("shards", "blocks"):
        cat = lambda k: np.concatenate([e[k] for e in d])  # noqa: E731
        ids, x, y, caps, tx, ty, tq = (cat(k) for k in ("ids", "x", "y", "caps", "tx", "ty", "treq"))
    else:
        ids, x, y, caps, tx, ty, tq = (d[k] for k in ("ids", "x", "y", "caps", "tx", "ty", "treq"))
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, ids)
    want = dict(zip(ids.tolist(), lead.tolist()))
    if transport == "rccl-double":  # groups, sends, recvs, all-reduces, all-gathers, bytes
        for o in outs:
            g, sd, rv, ar, ag, _ = o["dstats"]
            assert g > 0 and ar > 0 and ag > 0 and (sd > 0 and rv > 0) == bool(o["peers"]), o["dstats"]
    for o in outs:
        assert o["native"] == (transport != "python")
        assert o["converged"] and o["rounds"] == rounds and o["ghosts"] > 0
        np.testing.assert_array_equal(o["changes"], changes)
        assert all(want[int(i)] == int(v) for i, v in zip(o["ids"], o["leader"]))
        assert ((o["state"] == 3) == (o["leader"] == o["ids"])).all()
    assert sum(len(o["ids"]) for o in outs) == len(ids)
    wa = oracle_mod.allocate(ids, x, y, caps, tx, ty, tq)
    if (kind == "blocks" and world == 4) or kind == "global-random":
        assert all(len(o["peers"]) == world - 1 for o in outs)  # multi-peer halos: a 2 x 2 block grid / random IDs
    for key in ("winner", "util", "nmsg"):
        if kind in ("shards", "blocks"):
            got = np.concatenate([o[key] for o in outs])
        else:
            got = np.empty_like(wa[key])
            for o in outs:
                got[o["tasks"]] = o[key]
        np.testing.assert_array_equal(got, wa[key], err_msg=key)
    won_want = dict(zip(ids.tolist(), wa["won"].tolist()))
    for o in outs:
        assert all(won_want[int(i)] == int(w) for i, w in zip(o["ids"], o["won"]))
        assert o["gstats"]["n_claims"] == wa["n_claims"] and o["gstats"]["n_conflicts"] == wa["n_conflicts"]
    if transport != "python":  # the native sharded auction equals the one-GPU auction over the union
        atx, aty, atq = _auction_tasks(kind, world)
        w = oracle_mod.auction(ids, x, y, caps, atx, aty, atq)
        own_w = np.where(w["owner"] >= 0, ids[np.maximum(w["owner"], 0)], -1)
        for o in outs:
            au = o["auc"]
            assert au["rounds"] == w["rounds"]
            np.testing.assert_array_equal(au["bidders"], w["bidders"][: w["rounds"]])
            np.testing.assert_array_equal(au["owner"], own_w)
            np.testing.assert_array_equal(au["price"].view(np.uint32), np.asarray(w["price"], np.float32).view(np.uint32))
            by_id = dict(zip(ids.tolist(), w["assigned"].tolist()))
            assert all(by_id[int(i)] == int(a) for i, a in zip(au["ids"], au["assigned"]))
