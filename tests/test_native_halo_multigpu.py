"""The native RCCL sharded election loop (swarm_elect_sharded, csrc/comm.hip) with real peers:
one rank per GPU over nccl (RCCL), halo depths 1 and 16, against the single-swarm oracle on the
union graph (leaders, rounds, per-round change counts).  Needs >= 2 GPUs (RCCL does not run two
ranks of one communicator on one device); skipped otherwise -- the 1-GPU box of the round-end
test run skips it, the multi-GPU node runs it."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

N, SEED = 200_000, 11


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, depth, out_q):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    try:
        from swarm_amd import gen
        from swarm_amd.dist import ShardedSwarm
        d = gen.swarm_inputs(N, SEED)
        sh = ShardedSwarm.from_global(d["ids"], d["x"], d["y"], d["caps"], device=f"cuda:{rank}", halo_depth=depth)
        r = sh.elect(check_every=32)
        out_q.put(dict(rank=rank, native=getattr(sh, "_native", None) is not None, rounds=r.rounds_exec,
                       changes=r.changes, ids=sh.ids.cpu().numpy(), leader=r.leader.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one RCCL rank per device)")
@pytest.mark.parametrize("depth", [1, 16])
def test_native_rccl_halo_matches_union_oracle(depth, oracle_mod):
    import torch.multiprocessing as mp
    world = min(torch.cuda.device_count(), 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from swarm_amd import gen
    d = gen.swarm_inputs(N, SEED)
    rp, col = oracle_mod.rgg_csr(d["x"], d["y"], 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, d["ids"])
    want = dict(zip(d["ids"].tolist(), lead.tolist()))
    for o in outs:
        assert o["native"], "the native RCCL loop did not run"
        assert o["rounds"] == rounds
        np.testing.assert_array_equal(o["changes"], changes)
        assert all(want[int(i)] == int(v) for i, v in zip(o["ids"], o["leader"]))
