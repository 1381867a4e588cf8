"""Sharded (multi-rank) swarm step on CPU: world_size 2 and 3 over gloo, numpy stepper double.

Checks that strip partitioning + ghost halos + per-round halo exchange + batched global change
counts reproduce, exactly, the single-graph election of the union swarm (leaders per agent ID,
rounds_exec, per-round change counts), and that the halo-based sharded allocation reproduces
the single-resolver allocation (winners, claim values, won per agent)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

N_PER, SEED, T_PER = 1500, 5, 60


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q, n_per, deg, check_every, halo_depth, layout="strips"):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_doubles import NumpyBackend
        from swarm_amd import gen
        from swarm_amd.dist import Rects, ShardedSwarm
        layout, _, pk = layout.partition(":")  # "strips:3": 3 thin strips per rank, dealt round-robin
        d = gen.shard_inputs(n_per, SEED, world, rank, deg=deg, t=T_PER, layout=layout, pieces=int(pk or 1))
        region = Rects(d["rects"], rank) if (layout == "blocks" or pk) else d["strip"]
        sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], region, device="cpu", backend=NumpyBackend(),
                          halo_depth=halo_depth)
        r = sh.elect(check_every=check_every)
        sh._check_ghosts(sh.leaders[r.rounds_exec & 1])
        res, won, gst = sh.allocate(d["tx"], d["ty"], d["treq"])
        res0, won0, _ = sh.allocate(d["tx"], d["ty"], d["treq"], hysteresis=0.0)  # argmax (h = 0) mode
        out_q.put(dict(rank=rank, rounds=r.rounds_exec, changes=r.changes, ids=sh.ids.numpy(),
                       leader=r.leader.numpy(), state=r.state.numpy(), winner=res.winner.numpy(),
                       util=res.util.numpy(), won=won.numpy(), gstats=gst,
                       winner0=res0.winner.numpy(), won0=won0.numpy(),
                       n_ghost=(sh.n_glo, sh.n_ghi), depth=sh.halo_depth, peers=list(sh.peers)))
    finally:
        dist.destroy_process_group()


def _run(world, n_per=N_PER, deg=16.0, check_every=7, halo_depth=1, layout="strips"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, n_per, deg, check_every, halo_depth, layout))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(outs, key=lambda o: o["rank"])


def _union(world, n_per=N_PER, deg=16.0, layout="strips"):
    from swarm_amd import gen
    layout, _, pk = layout.partition(":")
    ds = [gen.shard_inputs(n_per, SEED, world, r, deg=deg, t=T_PER, layout=layout, pieces=int(pk or 1))
          for r in range(world)]
    cat = lambda k: np.concatenate([d[k] for d in ds])  # noqa: E731
    return ds, cat


@pytest.mark.parametrize("world,depth,layout", [(2, 1, "strips"), (2, 4, "strips"), (3, 16, "strips"),
                                                (2, 4, "blocks"), (3, 3, "blocks"), (4, 6, "blocks"),
                                                (2, 2, "strips:3"), (3, 4, "strips:2")])
def test_sharded_election_and_allocation_match_single_graph(world, depth, layout, oracle_mod):
    """depth: halo depth k (ghosts k radii deep, exchanged every k rounds); with strips 16 is capped by
    the strip height (the same cap on every rank).  layout "blocks": Morton-ordered blocks with Morton
    IDs (SURVEY §8e's C5 partition) -- up to 8 peers per rank, halos deeper than a block reach further.
    "strips:k": world x k thin strips dealt round-robin (k ID ranges per rank, Rects with k rectangles)."""
    outs = _run(world, halo_depth=depth, layout=layout)
    ds, cat = _union(world, layout=layout)
    x, y, ids, caps = cat("x"), cat("y"), cat("ids"), cat("caps")
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    lead, state, rounds, changes = oracle_mod.elect(rp, col, ids)
    want = dict(zip(ids.tolist(), lead.tolist()))
    for o in outs:
        assert o["rounds"] == rounds
        np.testing.assert_array_equal(o["changes"], changes)
        got = dict(zip(o["ids"].tolist(), o["leader"].tolist()))
        assert all(got[k] == want[k] for k in got)
        assert ((o["state"] == 3) == (o["leader"] == o["ids"])).all()
        assert sum(o["n_ghost"]) > 0
        assert o["depth"] == outs[0]["depth"] and 1 <= o["depth"] <= depth
        if layout != "strips":
            assert o["depth"] == depth  # no cap: the peer set grows instead
    if layout == "blocks" and world == 4:
        assert all(len(o["peers"]) == 3 for o in outs)  # a 2 x 2 grid: every block touches the other three
    assert sum(len(o["ids"]) for o in outs) == len(ids)
    # allocation: every rank resolves its own tasks; the union resolver must agree
    wa = oracle_mod.allocate(ids, x, y, caps, cat("tx"), cat("ty"), cat("treq"))
    np.testing.assert_array_equal(np.concatenate([o["winner"] for o in outs]), wa["winner"])
    np.testing.assert_array_equal(np.concatenate([o["util"] for o in outs]), wa["util"])
    won_want = dict(zip(ids.tolist(), wa["won"].tolist()))
    for o in outs:
        assert all(won_want[int(i)] == int(w) for i, w in zip(o["ids"], o["won"]))
        assert o["gstats"]["n_claims"] == wa["n_claims"]
        assert o["gstats"]["n_conflicts"] == wa["n_conflicts"]
    # hysteresis 0: the argmax (lowest-ID tie-break) resolution through the same sharded path
    w0 = oracle_mod.allocate(ids, x, y, caps, cat("tx"), cat("ty"), cat("treq"), hysteresis=0.0)
    np.testing.assert_array_equal(np.concatenate([o["winner0"] for o in outs]), w0["winner"])
    won0 = dict(zip(ids.tolist(), w0["won"].tolist()))
    for o in outs:
        assert all(won0[int(i)] == int(w) for i, w in zip(o["ids"], o["won0"]))


def test_shard_ids_are_a_global_permutation():
    from swarm_amd import gen
    ids = np.concatenate([gen.shard_inputs(777, 3, 5, r)["ids"] for r in range(5)])
    assert (np.sort(ids) == np.arange(777 * 5)).all()
    for r in range(5):  # ids="range": rank r owns exactly the ID range [777 r, 777 (r + 1)) -- its strip
        d = gen.shard_inputs(777, 3, 5, r)
        assert (np.sort(d["ids"]) == np.arange(*d["id_range"])).all() and d["id_range"] == (777 * r, 777 * (r + 1))
        assert (d["y"] >= d["strip"][0]).all() and (d["y"] < d["strip"][1]).all()
    ids = np.concatenate([gen.shard_inputs(777, 3, 5, r, ids="global")["ids"] for r in range(5)])
    assert (np.sort(ids) == np.arange(777 * 5)).all()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_partition_by_id_range_is_the_strip_partition(world):
    """north_star's ID-range partition: with strip-major IDs each rank's contiguous ID range is
    exactly its y-strip (the same owned agents and tasks as partition(by='y')); IDs that are not
    strip-major are refused."""
    from swarm_amd import gen
    from swarm_amd.dist import partition
    d = gen.swarm_inputs(6_000, 17, t=300)
    ids = gen.strip_ids(d["y"], world, 17)
    assert np.array_equal(np.sort(ids), np.arange(6_000))
    covered = []
    for r in range(world):
        pi = partition(d["x"], d["y"], world, r, ty=d["ty"], by="id", ids=ids)
        py = partition(d["x"], d["y"], world, r, ty=d["ty"])
        np.testing.assert_array_equal(pi.agents, py.agents)
        np.testing.assert_array_equal(pi.tasks, py.tasks)
        lo, hi = pi.id_range
        assert np.array_equal(np.sort(ids[pi.agents]), np.arange(lo, hi))
        covered.append((lo, hi))
    assert covered[0][0] == 0 and covered[-1][1] == 6_000
    assert all(covered[k][1] == covered[k + 1][0] for k in range(world - 1))
    assert type(pi.layout).__name__ == "Rects"
    # any other ID map: the ranges are not strips -> the cell layout, tasks dealt by index ranges
    parts = [partition(d["x"], d["y"], world, r, tx=d["tx"], ty=d["ty"], by="id", ids=d["ids"]) for r in range(world)]
    assert all(type(q.layout).__name__ == "Cells" for q in parts)
    assert np.array_equal(np.sort(np.concatenate([q.agents for q in parts])), np.arange(6_000))
    assert np.array_equal(np.sort(np.concatenate([q.tasks for q in parts])), np.arange(300))
    for q in parts:
        lo, hi = q.id_range
        assert np.array_equal(np.sort(d["ids"][q.agents]), np.arange(lo, hi))


@pytest.mark.parametrize("world,pieces", [(4, 4), (8, 8), (2, 3)])
def test_block_pieces_are_the_round_robin_id_partition(world, pieces):
    """dist.block_pieces (the C5 rehearsal's --pieces inputs, generated rank by rank): every rank owns
    exactly what partition(by='id', pieces=) gives on the union of the Morton blocks, n_per agents each,
    and its Cells layout marks every rank's agents and every block's tasks (block b's tasks: rank b)."""
    from swarm_amd import gen
    from swarm_amd.dist import block_pieces, partition
    n_per, t = 3_000, 40
    ds = [gen.shard_inputs(n_per, 11, world, b, t=t, layout="blocks") for b in range(world)]
    x, y = np.concatenate([d["x"] for d in ds]), np.concatenate([d["y"] for d in ds])
    ids = np.concatenate([d["ids"] for d in ds])
    for q in range(world):
        dq, lay = block_pieces(n_per, 11, world, q, pieces, t=t)
        assert len(dq["ids"]) == n_per
        pt = partition(x, y, world, q, by="id", ids=ids, pieces=pieces)
        np.testing.assert_array_equal(np.sort(ids[pt.agents]), np.sort(dq["ids"]))
        np.testing.assert_array_equal(dq["tx"], ds[q]["tx"])
        cy, cx = lay._cells(dq["x"], dq["y"])
        assert lay.occ["elect"][q, cy, cx].all() and lay.occ["alloc"].sum() > 0
        assert type(pt.layout).__name__ == "Cells"


# ----------------------------------------------------------------------------- sharded auction
A_PER, A_T = 300, 60


def _auction_worker(rank, world, port, out_q, check_every):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_doubles import NumpyBackend
        from swarm_amd import gen
        from swarm_amd.dist import ShardedSwarm
        ds = [gen.shard_inputs(A_PER, SEED + 1, world, r, t=A_T) for r in range(world)]
        d = ds[rank]
        tx, ty, tq = (np.concatenate([e[k] for e in ds]) for k in ("tx", "ty", "treq"))  # replicated tasks
        sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device="cpu", backend=NumpyBackend())
        r = sh.auction(tx, ty, tq, check_every=check_every)
        out_q.put(dict(rank=rank, rounds=r.rounds_exec, bidders=r.bidders, owner=r.owner_id.numpy().copy(),
                       price=r.price.numpy().copy(), assigned=r.assigned.numpy().copy(), ids=sh.ids.numpy().copy(),
                       converged=r.converged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,check_every", [(2, 5), (3, 16)])
def test_sharded_auction_matches_single_auction(world, check_every, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_auction_worker, args=(r, world, port, q, check_every)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from swarm_amd import gen
    ds = [gen.shard_inputs(A_PER, SEED + 1, world, r, t=A_T) for r in range(world)]
    cat = lambda k: np.concatenate([d[k] for d in ds])  # noqa: E731
    ids = cat("ids")
    want = oracle_mod.auction(ids, cat("x"), cat("y"), cat("caps"), cat("tx"), cat("ty"), cat("treq"))
    owner_id = np.where(want["owner"] >= 0, ids[np.maximum(want["owner"], 0)], -1)
    assert want["rounds"] > 3 and (want["owner"] >= 0).sum() > 0
    by_id = dict(zip(ids.tolist(), want["assigned"].tolist()))
    for o in outs:
        assert o["converged"] and o["rounds"] == want["rounds"]
        np.testing.assert_array_equal(o["bidders"], want["bidders"])
        np.testing.assert_array_equal(o["owner"], owner_id)
        np.testing.assert_array_equal(o["price"], want["price"])
        assert all(by_id[int(i)] == int(a) for i, a in zip(o["ids"], o["assigned"]))


# ------------------------------------------------------------------ one global swarm, partitioned
G_N, G_T = 4000, 150


def _global_inputs(world, by, ids="strip"):
    from swarm_amd import gen
    d = gen.swarm_inputs(G_N, SEED + 3, t=G_T, ids="morton" if ids == "morton" else "random")
    if by == "id" and ids == "strip":
        d["ids"] = gen.strip_ids(d["y"], world, SEED + 3)
    return d


def _global_worker(rank, world, port, out_q, depth, by="y", ids="strip", pieces=1):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_doubles import NumpyBackend
        from swarm_amd import gen
        from swarm_amd.dist import ShardedSwarm
        d = _global_inputs(world, by, ids)
        sh = ShardedSwarm.from_global(d["ids"], d["x"], d["y"], d["caps"], tx=d["tx"], ty=d["ty"], device="cpu",
                                      backend=NumpyBackend(), halo_depth=depth, by=by, pieces=pieces)
        r = sh.elect(check_every=5)
        res, won, gst = sh.allocate_global(d["tx"], d["ty"], d["treq"])
        out_q.put(dict(rank=rank, rounds=r.rounds_exec, changes=r.changes, ids=sh.ids.numpy(),
                       leader=r.leader.numpy(), tasks=sh.part.tasks, agents=sh.part.agents,
                       winner=res.winner.numpy(), util=res.util.numpy(), nmsg=res.nmsg.numpy(),
                       won=won.numpy(), gstats=gst))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,depth,by,ids,pieces", [
    (2, 4, "y", "strip", 1), (3, 16, "y", "strip", 1), (2, 4, "id", "strip", 1), (3, 16, "id", "strip", 1),
    (2, 3, "id", "morton", 1), (3, 5, "id", "morton", 1), (4, 4, "id", "morton", 1), (2, 2, "id", "random", 1),
    (3, 1, "id", "random", 1), (4, 3, "id", "random", 1), (2, 3, "id", "morton", 2), (3, 4, "id", "morton", 3)])
def test_partitioned_global_swarm_matches_single_swarm(world, depth, by, ids, pieces, oracle_mod):
    """ShardedSwarm.from_global: one global input (tasks anywhere) cut on every rank -- by y into strips
    with random IDs, or by contiguous ID range (north_star's ID-range partition) of strip-major IDs
    (strips), of Morton IDs (compact regions with several neighbouring ranks) or of random IDs (every
    rank a peer of every other), or world x pieces ID ranges of Morton IDs dealt round-robin (every rank a
    piece of every region: dist.piece_owner); the union of the shards' results equals the single-swarm
    oracle (leaders, rounds, per-round changes, winners, claim values, conflicts, won counts)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_worker, args=(r, world, port, q, depth, by, ids, pieces)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = _global_inputs(world, by, ids)
    # every agent and every task owned exactly once, parts of near-equal size
    agents = np.concatenate([o["agents"] for o in outs])
    assert np.array_equal(np.sort(agents), np.arange(G_N))
    assert max(len(o["agents"]) for o in outs) - min(len(o["agents"]) for o in outs) <= 2
    tasks = np.concatenate([o["tasks"] for o in outs])
    assert np.array_equal(np.sort(tasks), np.arange(G_T))
    rp, col = oracle_mod.rgg_csr(d["x"], d["y"], 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, d["ids"])
    want = dict(zip(d["ids"].tolist(), lead.tolist()))
    for o in outs:
        assert o["rounds"] == rounds
        np.testing.assert_array_equal(o["changes"], changes)
        assert all(want[int(i)] == int(v) for i, v in zip(o["ids"], o["leader"]))
    wa = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    for key in ("winner", "util", "nmsg"):
        got = np.empty_like(wa[key])
        for o in outs:
            got[o["tasks"]] = o[key]
        np.testing.assert_array_equal(got, wa[key])
    won_want = dict(zip(d["ids"].tolist(), wa["won"].tolist()))
    for o in outs:
        assert all(won_want[int(i)] == int(w) for i, w in zip(o["ids"], o["won"]))
        assert o["gstats"]["n_claims"] == wa["n_claims"]


def test_partition_cuts():
    from swarm_amd.dist import partition, strip_cuts
    g = np.random.default_rng(0)
    y = g.uniform(0, 100, 10_001)
    cuts = strip_cuts(y, 4)
    parts = [partition(np.zeros_like(y), y, 4, r, ty=y[:50]) for r in range(4)]
    assert np.array_equal(np.sort(np.concatenate([p.agents for p in parts])), np.arange(len(y)))
    assert [len(p.agents) for p in parts] == [2500, 2500, 2500, 2501]
    assert all(np.array_equal(p.cuts, cuts) for p in parts)
    for p in parts:  # owned agents lie inside the strip
        assert (y[p.agents] >= p.strip[0]).all() and (y[p.agents] <= p.strip[1]).all()
    with pytest.raises(ValueError):
        partition(np.zeros(8), np.arange(8.0), 4, 0, min_height=5.0)


def test_partition_by_id_empty_range_is_a_clear_error():
    """More ranks than distinct IDs leaves an ID range empty: a ValueError that says so,
    not numpy's bare 'zero-size array' error."""
    from swarm_amd.dist import partition
    ids = np.array([5, 5, 5, 5, 9, 9], np.int64)
    y = np.array([0.0, 0.1, 0.2, 0.3, 5.0, 5.1])
    with pytest.raises(ValueError, match="without agents"):
        partition(np.zeros_like(y), y, 3, 0, by="id", ids=ids)


def _auction_check_worker(rank, world, port, out_q):
    import sys
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from shard_doubles import NumpyBackend
        from swarm_amd import gen
        from swarm_amd.dist import ShardedSwarm
        ds = [gen.shard_inputs(A_PER, SEED + 2, world, r, t=A_T) for r in range(world)]
        d = ds[rank]
        tx, ty, tq = (np.concatenate([e[k] for e in ds]) for k in ("tx", "ty", "treq"))
        sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device="cpu", backend=NumpyBackend())
        r = sh.auction(tx, ty, tq)
        good = bench.auction_union_check(sh, r, ds, tx, ty, tq, rank, world)
        r.assigned[0] = -2 if r.assigned.numel() else 0  # one agent's assignment spoiled on every rank
        bad = bench.auction_union_check(sh, r, ds, tx, ty, tq, rank, world)
        out_q.put(dict(rank=rank, good=good, bad=bad))
    finally:
        dist.destroy_process_group()


def test_bench_auction_union_check():
    """bench.py's union-oracle check of the sharded auction (the N > 1 line's rows.C4_auction_sharded):
    equal on a correct run, and it notices one wrong assignment."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_auction_check_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in range(2)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g, b = outs[0]["good"], outs[0]["bad"]
    assert g["equal"] and g["rounds"] and g["owner"] and g["price_bits"] and g["assigned"]
    assert not b["equal"] and not b["assigned"]
    assert outs[1]["good"] is None
