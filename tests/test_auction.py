"""Auction allocation (BASELINE config C4).

No reference counterpart exists (the reference allocates by greedy claims + leader hysteresis),
so parity is "parity unpinned" against the reference and bit-exact against the build's own CPU
restatement: oracle.auction (C) is first checked against the straight pure-Python restatement
(oracle.auction_py) and against the auction's defining properties; the GPU path (libswarm
swarm_auction through the C-ABI) is then checked bit-exactly against oracle.auction --
assignments, f32 prices, per-round bidder counts and the round count.
"""
import os

import numpy as np
import pytest

from swarm_amd import gen


def _inputs(n, seed, t=None):
    d = gen.swarm_inputs(n, seed, t=max(1, n if t is None else t))
    if t == 0:
        for k in ("tx", "ty", "treq"):
            d[k] = d[k][:0]
    return d


def _check_properties(d, res, eps=0.1, thr=20.0):
    """Matching consistency, prices, and eps-complementary slackness at termination."""
    from oracle import oracle
    owner, price, assigned = res["owner"], res["price"], res["assigned"]
    n, t = len(d["ids"]), len(d["tx"])
    for k in range(t):
        if owner[k] >= 0:
            assert assigned[owner[k]] == k
    for a in range(n):
        if assigned[a] >= 0:
            assert owner[assigned[a]] == a
    assert (price >= 0).all()
    assert ((price > 0) == (owner >= 0)).all()  # a task's price rises exactly when it is taken
    # eps-CS: an assigned agent's net value is within eps of its best alternative (incl. 0)
    rng = np.random.default_rng(0)
    for a in rng.choice(n, size=min(n, 50), replace=False):
        if assigned[a] < 0:
            continue
        U = oracle.utility(np.full(t, d["x"][a]), np.full(t, d["y"][a]), np.full(t, d["caps"][a], np.uint32),
                           d["tx"], d["ty"], d["treq"], use_pow=False)
        adm = U > thr
        net = np.where(adm, U.astype(np.float32) - price, -np.inf)
        mine = np.float32(U[assigned[a]]) - price[assigned[a]]
        assert mine >= max(net.max(), 0.0) - eps - 1e-4


@pytest.mark.parametrize("n,seed", [(1, 11), (60, 1), (300, 2), (700, 3)])
def test_oracle_c_matches_python_restatement(oracle_mod, n, seed):
    d = _inputs(n, seed)
    a = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    b = oracle_mod.auction_py(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    assert a["rounds"] == b["rounds"] >= 0
    for k in ("owner", "price", "assigned", "bidders"):
        np.testing.assert_array_equal(a[k], b[k])
    _check_properties(d, a)


def test_oracle_edge_cases(oracle_mod):
    # no tasks, no agents, unreachable tasks, more tasks than agents
    d = _inputs(50, 7, t=0)
    r = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    assert r["rounds"] == 1 and (r["assigned"] == -1).all()  # round 1: everyone drops out
    np.testing.assert_array_equal(r["bidders"], [50])
    d = _inputs(40, 8, t=200)
    r = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"] + 1e6, d["ty"], d["treq"])
    assert r["rounds"] == 1 and (r["assigned"] == -1).all()  # everyone bids once and drops out
    r = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    p = oracle_mod.auction_py(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    np.testing.assert_array_equal(r["assigned"], p["assigned"])
    _check_properties(d, r)


def test_oracle_eps_trades_rounds_for_value(oracle_mod):
    d = _inputs(500, 9)
    vals = {}
    for eps in (1.0, 0.1):
        r = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"], eps=eps)
        U = oracle_mod.utility(d["x"], d["y"], d["caps"], d["tx"][np.maximum(r["assigned"], 0)],
                               d["ty"][np.maximum(r["assigned"], 0)], d["treq"][np.maximum(r["assigned"], 0)],
                               use_pow=False)
        vals[eps] = (float(np.sum(np.where(r["assigned"] >= 0, U.astype(np.float32), 0.0))), r["rounds"])
        _check_properties(d, r, eps=eps)
    assert vals[0.1][1] > vals[1.0][1]          # smaller eps: more rounds ...
    assert vals[0.1][0] >= vals[1.0][0] - 1e-3  # ... and no worse total value


# ----------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("tail", ["0", "512", "2048"])
@pytest.mark.parametrize("n,seed", [(60, 1), (2000, 4), (20000, 5)])
def test_gpu_auction_matches_oracle(oracle_mod, n, seed, tail):
    from swarm_amd.swarm import Swarm
    d = _inputs(n, seed)
    want = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    os.environ["SWARM_AUCTION_TAIL"] = tail
    try:
        s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
        r = s.auction(d["tx"], d["ty"], d["treq"])
    finally:
        del os.environ["SWARM_AUCTION_TAIL"]
    assert r.converged and r.rounds_exec == want["rounds"]
    np.testing.assert_array_equal(r.bidders, want["bidders"])
    np.testing.assert_array_equal(r.price.cpu().numpy(), want["price"])
    perm = s.perm.cpu().numpy()
    own = r.owner.cpu().numpy()
    np.testing.assert_array_equal(np.where(own >= 0, perm[np.maximum(own, 0)], -1), want["owner"])
    np.testing.assert_array_equal(s.to_input_order(r.assigned), want["assigned"])
    # n_flagged: pairs a libm-pow utility (the reference's arithmetic) might round differently;
    # the auction has no reference counterpart, so it is reported, not required to be 0
    assert r.stats["n_pairs"] > 0 and r.stats["n_flagged"] <= r.stats["n_pairs"] // 100000 + 2
    if tail == "0":
        assert r.stats["tail_rounds"] == 0
    elif n >= 2000:
        assert r.stats["tail_rounds"] > 0


@pytest.mark.gpu
def test_gpu_auction_edge_cases(oracle_mod):
    from swarm_amd.swarm import Swarm
    d = _inputs(40, 8, t=200)
    s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    r = s.auction(d["tx"] + 1e6, d["ty"], d["treq"])  # unreachable: one round, everyone drops out
    assert r.rounds_exec == 1 and (r.assigned.cpu().numpy() == -1).all() and r.stats["n_pairs"] == 0
    r = s.auction(d["tx"][:0], d["ty"][:0], d["treq"][:0])  # no tasks: round 1, all drop out
    assert r.rounds_exec == 1 and list(r.bidders) == [40] and (r.assigned.cpu().numpy() == -1).all()
    r = s.auction(d["tx"], d["ty"], d["treq"], max_rounds=2)  # not converged in 2 rounds
    want = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    assert want["rounds"] > 2 and not r.converged and r.rounds_exec == 2


# ----------------------------------------------------------------------------- sharded (C4 on N GPUs)

@pytest.mark.gpu
def test_gpu_sharded_auction_two_shards_on_one_gpu(oracle_mod):
    """swarm_auction_begin/_bid/_resolve through ShardedSwarm.auction: two shards (two threads,
    one GPU, in-process MAX reduce of the keys), tasks replicated; the union auction is the
    reference (oracle.auction over all agents)."""
    import threading

    import torch
    from shard_doubles import ThreadHalo
    from swarm_amd import gen
    from swarm_amd.dist import ShardedSwarm
    world, n_per, t_per = 2, 6000, 3000
    ds = [gen.shard_inputs(n_per, 12, world, k, t=t_per) for k in range(world)]
    cat = lambda k: np.concatenate([d[k] for d in ds])  # noqa: E731
    tx, ty, tq = cat("tx"), cat("ty"), cat("treq")
    hub = ThreadHalo(world)
    outs, errs = {}, []

    def run(rank):
        try:
            torch.cuda.set_device(0)
            d = ds[rank]
            sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device="cuda:0",
                              halo=hub.member(rank))
            r = sh.auction(tx, ty, tq, check_every=32)
            torch.cuda.synchronize()
            outs[rank] = dict(r=r, ids=sh.ids.cpu().numpy(), owner=r.owner_id.cpu().numpy(),
                              price=r.price.cpu().numpy(), assigned=r.assigned.cpu().numpy())
        except Exception as e:  # surfaced below
            errs.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    ids = cat("ids")
    want = oracle_mod.auction(ids, cat("x"), cat("y"), cat("caps"), tx, ty, tq)
    owner_id = np.where(want["owner"] >= 0, ids[np.maximum(want["owner"], 0)], -1)
    by_id = dict(zip(ids.tolist(), want["assigned"].tolist()))
    for k in range(world):
        o = outs[k]
        assert o["r"].converged and o["r"].rounds_exec == want["rounds"]
        np.testing.assert_array_equal(o["r"].bidders, want["bidders"])
        np.testing.assert_array_equal(o["owner"], owner_id)
        np.testing.assert_array_equal(o["price"], want["price"])
        assert all(by_id[int(i)] == int(a) for i, a in zip(o["ids"], o["assigned"]))


@pytest.mark.gpu
def test_gpu_native_sharded_auction_single_rank_rccl():
    """swarm_auction_sharded (RCCL all-reduce per round) on a 1-rank communicator equals
    swarm_auction on the same agents: rounds, bidders, prices, owners (as IDs), assignments."""
    import ctypes

    import torch
    from swarm_amd import _lib as L
    from swarm_amd.swarm import Swarm
    if not L.lib().swarm_comm_available():
        pytest.skip("RCCL not resolvable in this process")
    d = _inputs(20000, 5)
    s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    want = s.auction(d["tx"], d["ty"], d["treq"])
    uid = (ctypes.c_uint8 * 128)()
    L.check(L.lib().swarm_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)))
    comm = ctypes.c_void_p()
    L.check(L.lib().swarm_comm_create(ctypes.byref(comm), 1, 0, ctypes.cast(uid, ctypes.c_void_p)))
    try:
        t = len(d["tx"])
        tpos = torch.as_tensor(np.stack([d["tx"], d["ty"]], 1), device="cuda").contiguous()
        treq = torch.as_tensor(d["treq"], device="cuda")
        owner = torch.empty(t, dtype=torch.int32, device="cuda")
        price = torch.empty(t, dtype=torch.float32, device="cuda")
        assigned = torch.empty(s.n, dtype=torch.int32, device="cuda")
        rounds = ctypes.c_int32(0)
        bid = np.zeros(1 << 16, np.int64)
        L.check(L.lib().swarm_auction_sharded(
            L.ctx(), comm, s.n, L.ptr(s.ids), L.ptr(s.pos), L.ptr(s.caps), t, L.ptr(tpos), L.ptr(treq), 20.0, 100.0,
            0.1, len(bid), L.ptr(owner), L.ptr(price), L.ptr(assigned), ctypes.byref(rounds),
            bid.ctypes.data_as(ctypes.c_void_p), None, L.stream()))
        r = rounds.value
        assert r == want.rounds_exec
        np.testing.assert_array_equal(bid[:r], want.bidders)
        np.testing.assert_array_equal(price.cpu().numpy(), want.price.cpu().numpy())
        ids = s.ids.cpu().numpy()
        wo = want.owner.cpu().numpy()
        np.testing.assert_array_equal(owner.cpu().numpy(), np.where(wo >= 0, ids[np.maximum(wo, 0)], -1))
        np.testing.assert_array_equal(assigned.cpu().numpy(), want.assigned.cpu().numpy())
    finally:
        L.lib().swarm_comm_destroy(comm)


@pytest.mark.gpu
def test_gpu_auction_large_ids(oracle_mod):
    """IDs at the top of the int32 range: the packed key's ~id tie-break and the ID index."""
    from swarm_amd.swarm import Swarm
    d = _inputs(3000, 13)
    d["ids"] = (np.int64(2**31 - 1) - np.random.default_rng(1).permutation(len(d["ids"])) * 7).astype(np.int32)
    want = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    r = s.auction(d["tx"], d["ty"], d["treq"])
    assert r.rounds_exec == want["rounds"]
    np.testing.assert_array_equal(r.price.cpu().numpy(), want["price"])
    np.testing.assert_array_equal(s.to_input_order(r.assigned), want["assigned"])


@pytest.mark.gpu
@pytest.mark.parametrize("fused,tail", [("1000000000", "0"), ("1000000000", "128"), ("0", "128"), ("4096", "0")])
@pytest.mark.parametrize("n,seed", [(2000, 14), (20000, 15)])
def test_gpu_auction_fused_rounds_match_oracle(oracle_mod, n, seed, fused, tail):
    """Fused rounds (resolve round q-1 and bid round q in one kernel, keys over three buffers,
    a fresh list per batch) against the oracle, alone, beside the list-driven rounds and before
    the one-workgroup tail."""
    from swarm_amd.swarm import Swarm
    d = _inputs(n, seed)
    want = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    os.environ["SWARM_AUCTION_TAIL"] = tail
    os.environ["SWARM_AUCTION_FUSED"] = fused
    try:
        s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
        r = s.auction(d["tx"], d["ty"], d["treq"])
        cut = {}
        for m in (1, 2, 9, 10, 25, 57, want["rounds"] - 1):
            if 1 <= m < want["rounds"]:
                cut[m] = s.auction(d["tx"], d["ty"], d["treq"], max_rounds=m)
    finally:
        del os.environ["SWARM_AUCTION_TAIL"]
        del os.environ["SWARM_AUCTION_FUSED"]
    assert r.converged and r.rounds_exec == want["rounds"]
    np.testing.assert_array_equal(r.bidders, want["bidders"])
    np.testing.assert_array_equal(r.price.cpu().numpy(), want["price"])
    np.testing.assert_array_equal(s.to_input_order(r.assigned), want["assigned"])
    for m, rc in cut.items():  # the state after exactly m rounds (every bid of round m resolved)
        w = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"], max_rounds=m)
        assert not rc.converged and rc.rounds_exec == m, m
        np.testing.assert_array_equal(rc.bidders, want["bidders"][:m])
        np.testing.assert_array_equal(rc.price.cpu().numpy(), w["price"])
        np.testing.assert_array_equal(s.to_input_order(rc.assigned), w["assigned"])
