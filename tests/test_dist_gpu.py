"""The HIP sharded path across PROCESSES on one GPU.

Two (or three) processes share cuda:0 over gloo: each is one rank with the product backend
(GpuBackend: libswarm's frontier stepper, ghost and allocation kernels), the halo staged through
host memory (gloo cannot move device tensors; RCCL refuses two ranks on one device, so the native
RCCL loop is covered by tests/test_native_halo_multigpu.py where >= 2 GPUs exist).  Every rank's
leaders, rounds and per-round global change counts, and the sharded allocation (winners, claim
values, conflicts, won counts), must equal the oracle over the union swarm.
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
    d = gen.swarm_inputs(12_000, 43, t=300)  # one global swarm, cut by ID range (strip-major IDs)
    d["ids"] = gen.strip_ids(d["y"], world, 43)
    return d


def _worker(rank, world, port, out_q, kind, depth):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from swarm_amd.dist import GpuBackend, ShardedSwarm
        dev = torch.device("cuda", 0)
        if kind == "shards":
            d = _inputs(kind, world)[rank]
            sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device=dev, halo_depth=depth)
            tx, ty, tq = d["tx"], d["ty"], d["treq"]
            tasks = None
        else:
            d = _inputs(kind, world)
            sh = ShardedSwarm.from_global(d["ids"], d["x"], d["y"], d["caps"], ty=d["ty"], device=dev,
                                          halo_depth=depth, by="id")
            k = sh.part.tasks
            tx, ty, tq = d["tx"][k], d["ty"][k], d["treq"][k]
            tasks = k
        assert isinstance(sh.backend, GpuBackend) and sh.halo.host_staged
        r = sh.elect(check_every=16)
        sh._check_ghosts(sh.leaders[r.rounds_exec & 1])
        res, won, gst = sh.allocate(tx, ty, tq)
        torch.cuda.synchronize()
        out_q.put(dict(rank=rank, rounds=r.rounds_exec, changes=r.changes, ids=sh.ids.cpu().numpy(),
                       leader=r.leader.cpu().numpy(), state=r.state.cpu().numpy(), winner=res.winner.cpu().numpy(),
                       util=res.util.cpu().numpy(), nmsg=res.nmsg.cpu().numpy(), won=won.cpu().numpy(),
                       gstats=gst, tasks=tasks, converged=r.converged, ghosts=sh.n_glo + sh.n_ghi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,depth", [(2, "shards", 16), (2, "global", 4), (3, "global", 16)])
def test_hip_sharded_processes_match_union_oracle(world, kind, depth, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind, depth)) for r in range(world)]
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
    if kind == "shards":
        cat = lambda k: np.concatenate([e[k] for e in d])  # noqa: E731
        ids, x, y, caps, tx, ty, tq = (cat(k) for k in ("ids", "x", "y", "caps", "tx", "ty", "treq"))
    else:
        ids, x, y, caps, tx, ty, tq = (d[k] for k in ("ids", "x", "y", "caps", "tx", "ty", "treq"))
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, ids)
    want = dict(zip(ids.tolist(), lead.tolist()))
    for o in outs:
        assert o["converged"] and o["rounds"] == rounds and o["ghosts"] > 0
        np.testing.assert_array_equal(o["changes"], changes)
        assert all(want[int(i)] == int(v) for i, v in zip(o["ids"], o["leader"]))
        assert ((o["state"] == 3) == (o["leader"] == o["ids"])).all()
    assert sum(len(o["ids"]) for o in outs) == len(ids)
    wa = oracle_mod.allocate(ids, x, y, caps, tx, ty, tq)
    for key in ("winner", "util", "nmsg"):
        if kind == "shards":
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
