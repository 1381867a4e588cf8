"""GPU parity: the HIP path (libswarm.so through the C-ABI) against the reference's golden
vectors and, at larger sizes, against the CPU oracle on identical seeded inputs.

Bars (north star): leaders, states, round counts, per-round change counts, task winners,
claim/message counts and per-agent won counts bit-exact; winning claim values bit-exact (they
are f32 values); fp64 utilities within 1e-15 relative of the reference's libm-pow bits (the
north star allows 1e-6) and bit-exact against the oracle's x*x restatement.
"""
import numpy as np
import pytest
import torch

from conftest import golden_index, golden_names, load_golden

pytestmark = pytest.mark.gpu

ELECT = golden_names("elect_")
ALLOC = golden_names("alloc_")


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


def _swarm(sw, g, layout):
    n = len(g["ids"])
    x = g["x"] if "x" in g else np.arange(n, dtype=np.float64)
    y = g["y"] if "y" in g else np.zeros(n)
    caps = g["caps"] if "caps" in g else None
    return sw.Swarm(g["ids"], x, y, caps, layout=layout, device="cuda")


# ----------------------------------------------------------------------------- election

@pytest.mark.parametrize("mode", ["dense", "frontier"])
@pytest.mark.parametrize("layout", ["input", "spatial"])
@pytest.mark.parametrize("name", ELECT)
def test_elect_matches_reference(sw, name, mode, layout):
    g = load_golden(name)
    s = _swarm(sw, g, layout).set_graph(g["row_ptr"], g["col"])
    r = s.elect(mode=mode)
    assert r.converged
    assert r.rounds_exec == int(g["rounds_exec"])
    np.testing.assert_array_equal(r.changes, g["changes"])
    np.testing.assert_array_equal(s.to_input_order(r.leader), g["leader"])
    np.testing.assert_array_equal(s.to_input_order(r.state), g["state"])


def test_gpu_rgg_builder_matches_oracle(sw, oracle_mod):
    from swarm_amd import gen
    for n, seed in [(1, 1), (7, 2), (20000, 3), (150000, 4)]:
        d = gen.swarm_inputs(n, seed)
        s = sw.Swarm(d["ids"], d["x"], d["y"], layout="input", device="cuda").build_graph(1.0)
        rp, col = oracle_mod.rgg_csr(d["x"], d["y"], 1.0)
        np.testing.assert_array_equal(s.row_ptr.cpu().numpy(), rp)
        np.testing.assert_array_equal(s.col.cpu().numpy(), col)


def test_take_rows_above_2_26_rows(sw):
    """The Swarm's position permutation (swarm.take_rows) above 2^26 rows, where this PyTorch-ROCm
    build's row gathers of an (N, 2) float64 tensor return wrong rows (seen at 68M: the graph
    build then never ended).  Checked against the CPU gather of the same rows."""
    import torch
    n = (1 << 26) + 4099
    g = torch.Generator(device="cuda").manual_seed(3)
    t = torch.rand(n, 2, dtype=torch.float64, device="cuda", generator=g)
    p = torch.randperm(n, device="cuda", generator=g)
    out = sw.take_rows(t, p)
    k = torch.randint(0, n, (4096,), generator=torch.Generator().manual_seed(4))
    k = torch.cat([k, torch.arange(n - 64, n)])
    want = t.cpu()[p.cpu()[k]]
    assert torch.equal(out.cpu()[k], want)
    assert out.is_contiguous() and out.shape == (n, 2)


@pytest.mark.parametrize("n,seed,deg", [(300000, 41, 16.0), (200000, 42, 6.0)])
def test_elect_large_vs_oracle(sw, oracle_mod, n, seed, deg):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, deg=deg)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    rp = s.row_ptr.cpu().numpy().astype(np.int64)
    col = s.col.cpu().numpy()
    ids = s.ids.cpu().numpy()
    lead, state, rounds, changes = oracle_mod.elect(rp, col, ids)
    for mode in ("frontier", "dense"):
        r = s.elect(mode=mode)
        assert r.rounds_exec == rounds, mode
        np.testing.assert_array_equal(r.changes, changes)
        np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
        np.testing.assert_array_equal(r.state.cpu().numpy(), state)


def test_elect_not_converged_reports(sw):
    g = load_golden("elect_path_n300")
    s = _swarm(sw, g, "input").set_graph(g["row_ptr"], g["col"])
    for mode in ("dense", "frontier"):
        r = s.elect(mode=mode, max_rounds=50)
        assert not r.converged and r.rounds_exec == 50
        np.testing.assert_array_equal(r.changes, g["changes"][:50])
        # the state after exactly 50 rounds: leader = max id within 50 hops on the path
        ids = g["ids"]
        want = np.array([ids[max(0, i - 50):i + 51].max() for i in range(len(ids))])
        np.testing.assert_array_equal(r.leader.cpu().numpy(), want)


def test_elect_round_primitive(sw, oracle_mod):
    """swarm_elect_round (the sharded building block) = one dense E2 round."""
    import ctypes
    from swarm_amd import _lib
    g = load_golden("elect_n2000")
    rp = torch.as_tensor(g["row_ptr"].astype(np.int32), device="cuda")
    col = torch.as_tensor(g["col"], device="cuda")
    lin = torch.as_tensor(g["ids"], device="cuda")
    lout = torch.empty_like(lin)
    changed = torch.zeros(1, dtype=torch.int64, device="cuda")
    _lib.check(_lib.lib().swarm_elect_round(_lib.ctx(), len(lin), _lib.ptr(rp), _lib.ptr(col), _lib.ptr(lin),
                                            _lib.ptr(lout), _lib.ptr(changed), _lib.stream()))
    torch.cuda.synchronize()
    assert int(changed.item()) == int(g["changes"][0])
    lead, _, _, _ = oracle_mod.elect(g["row_ptr"], g["col"], g["ids"], max_rounds=1)
    np.testing.assert_array_equal(lout.cpu().numpy(), lead)
    del ctypes


# ---------------------------------------------------------------------------- allocation

def _alloc(sw, g, mode, layout, hysteresis=5.0):
    s = _swarm(sw, g, layout)
    r = s.allocate(g["tx"], g["ty"], g["treq"], winner=g.get("pre_w"), util=g.get("pre_u"),
                   mode=mode, hysteresis=hysteresis)
    return s, r


@pytest.mark.parametrize("mode", ["binned", "dense"])
@pytest.mark.parametrize("layout", ["input", "spatial"])
@pytest.mark.parametrize("name", ALLOC)
def test_allocate_matches_reference(sw, oracle_mod, name, mode, layout):
    g = load_golden(name)
    s, r = _alloc(sw, g, mode, layout)
    assert r.stats["n_flagged"] == 0 or name == "alloc_edge_n60_t40"
    np.testing.assert_array_equal(r.winner.cpu().numpy(), g["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy().view(np.uint64), g["util"].view(np.uint64))
    np.testing.assert_array_equal(s.to_input_order(r.won), g["won"])
    assert r.stats["n_claims"] == int(g["n_claims"])
    assert r.stats["n_conflicts"] == int(g["n_conflicts"])
    assert int(r.nclaim.sum()) == int(g["n_claims"])
    # per-agent statuses derived from (winner, nmsg) equal the reference's after delivery
    claimed = np.zeros((len(g["ids"]), len(g["tx"])), bool)
    pos = {int(a): i for i, a in enumerate(g["ids"])}
    claimed[[pos[int(x)] for x in g["claim_sender"]], g["claim_task"]] = True
    st = oracle_mod.statuses(g["ids"], r.winner.cpu().numpy(), r.nmsg.cpu().numpy(), claimed)
    if "status" in g:
        np.testing.assert_array_equal(st, g["status"])
    else:
        np.testing.assert_array_equal(np.stack([(st == k).sum(0) for k in range(4)]), g["status_counts"])


def test_utility_kat(sw, oracle_mod):
    import swarm_amd._lib as L
    k = load_golden("utility_kat")
    m = len(k["util"])
    dev = "cuda"
    apos = torch.as_tensor(np.stack([k["ax"], k["ay"]], 1), device=dev).contiguous()
    tpos = torch.as_tensor(np.stack([k["tx"], k["ty"]], 1), device=dev).contiguous()
    caps = torch.as_tensor(k["caps"].view(np.int32), device=dev)
    treq = torch.as_tensor(k["treq"], device=dev)
    out = torch.empty(m, dtype=torch.float64, device=dev)
    L.check(L.lib().swarm_utility(L.ctx(), m, L.ptr(apos), L.ptr(caps), L.ptr(tpos), L.ptr(treq), 100.0,
                                  L.ptr(out), L.stream()))
    u = out.cpu().numpy()
    # bit-exact vs the same arithmetic on the host (IEEE sqrt and division on gfx950)
    uxx = oracle_mod.utility(k["ax"], k["ay"], k["caps"], k["tx"], k["ty"], k["treq"], use_pow=False)
    np.testing.assert_array_equal(u.view(np.uint64), uxx.view(np.uint64))
    # reference (libm pow) semantics: tolerance, identical claim decisions and f32 claim values
    np.testing.assert_allclose(u, k["util"], rtol=1e-15, atol=0)
    np.testing.assert_array_equal(u > 20.0, k["claim"])
    np.testing.assert_array_equal(u.astype(np.float32).view(np.uint32), k["util_f32"].view(np.uint32))


@pytest.mark.parametrize("n,t,seed", [(200000, 3000, 51), (60000, 20000, 52)])
def test_allocate_large_vs_oracle(sw, oracle_mod, n, t, seed):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, t=t)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    want = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    for mode in ("binned", "dense"):
        r = s.allocate(d["tx"], d["ty"], d["treq"], mode=mode)
        assert r.stats["n_flagged"] == 0
        np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
        np.testing.assert_array_equal(r.util.cpu().numpy(), want["util"])
        np.testing.assert_array_equal(s.to_input_order(r.won), want["won"])
        np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
        np.testing.assert_array_equal(r.nclaim.cpu().numpy(), want["nclaim"])


def test_allocate_argmax_mode_h0(sw, oracle_mod):
    """hysteresis 0 = argmax of the claim value, lowest ID on ties (north-star argmin mode)."""
    from swarm_amd import gen
    d = gen.swarm_inputs(20000, 61, t=500)
    x, y = d["x"].copy(), d["y"].copy()
    x[1::7], y[1::7] = x[0::7][: len(x[1::7])], y[0::7][: len(y[1::7])]  # exact ties
    s = sw.Swarm(d["ids"], x, y, d["caps"], device="cuda")
    want = oracle_mod.allocate(d["ids"], x, y, d["caps"], d["tx"], d["ty"], d["treq"], hysteresis=0.0)
    for mode in ("binned", "dense"):
        r = s.allocate(d["tx"], d["ty"], d["treq"], hysteresis=0.0, mode=mode)
        np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    # independent argmax restatement
    for k in range(0, 500, 37):
        cid, cx = oracle_mod.task_claims(d["ids"], x, y, d["caps"], d["tx"][k], d["ty"][k], d["treq"][k])
        if len(cid):
            best = cx.max()
            assert want["winner"][k] == cid[cx == best].min()


def test_allocate_overflow_path_exact(sw, oracle_mod):
    """> 2048 claimants on one task (co-located agents) takes the recompute path; still exact."""
    from swarm_amd import gen
    n = 6000
    d = gen.swarm_inputs(n, 71, t=40)
    x, y = d["x"].copy(), d["y"].copy()
    x[:3000] = 5.0 + (np.arange(3000) % 50) * 1e-3
    y[:3000] = 5.0
    tx, ty = d["tx"].copy(), d["ty"].copy()
    tx[:5], ty[:5] = 5.01, 5.0
    caps = np.full(n, 0xF, np.uint32)
    s = sw.Swarm(d["ids"], x, y, caps, device="cuda")
    want = oracle_mod.allocate(d["ids"], x, y, caps, tx, ty, d["treq"], hysteresis=0.25)
    for mode in ("binned", "dense"):
        r = s.allocate(tx, ty, d["treq"], hysteresis=0.25, mode=mode)
        if mode == "binned":
            assert r.stats["n_overflow"] >= 5
        np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
        np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
        np.testing.assert_array_equal(s.to_input_order(r.won), want["won"])


def test_allocate_edge_shapes(sw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(500, 81, t=30)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    # no tasks
    r = s.allocate(np.zeros(0), np.zeros(0), np.zeros(0, np.int8))
    assert r.winner.numel() == 0 and int(r.won.sum()) == 0
    # threshold above the utility scale: nobody can claim, preloaded winners keep their task
    pre = np.where(np.arange(30) % 3 == 0, d["ids"][:30], -1).astype(np.int32)
    r = s.allocate(d["tx"], d["ty"], d["treq"], winner=pre, util=np.full(30, 42.0), claim_thr=150.0)
    np.testing.assert_array_equal(r.winner.cpu().numpy(), pre)
    assert r.stats["n_claims"] == 0 and int(r.won.sum()) == int((pre >= 0).sum())
    # negative threshold: everybody claims (cap-less agents claim with U = 0) -> dense path
    want = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"],
                               claim_thr=-1.0)
    r = s.allocate(d["tx"], d["ty"], d["treq"], claim_thr=-1.0)
    assert r.stats["mode_used"] == 2
    np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
    # tasks far outside the swarm
    r = s.allocate(np.full(4, 1e7), np.full(4, -1e7), np.full(4, -1, np.int8))
    assert (r.winner.cpu().numpy() == -1).all() and r.stats["n_claims"] == 0


def test_empty_and_single_swarms(sw):
    for n in (0, 1):
        s = sw.Swarm(np.arange(n, dtype=np.int32) + 5, np.zeros(n), np.zeros(n), device="cuda")
        s.build_graph(1.0)
        r = s.elect()
        assert r.rounds_exec == 1 and list(r.changes) == [0]
        a = s.allocate(np.array([0.5]), np.array([0.0]), np.array([-1], np.int8))
        assert int(a.winner.item()) == (5 if n else -1)


def test_dropin_bridge_round_trip(sw, oracle_mod):
    """Reference-style SwarmAgent objects -> GPU round -> written back onto the objects."""
    import agent
    g = load_golden("alloc_wire_n200_t50")
    agents = []
    for i in range(len(g["ids"])):
        names = [sw.CAP_VOCAB_DEFAULT[k] for k in range(4) if (int(g["caps"][i]) >> k) & 1]
        a = agent.SwarmAgent(int(g["ids"][i]), len(g["ids"]), capabilities=names)
        a.position = [float(g["x"][i]), float(g["y"][i])]
        a.tasks = {k: ({"status": "OPEN", "pos": (float(g["tx"][k]), float(g["ty"][k]))} |
                       ({"required_cap": sw.CAP_VOCAB_DEFAULT[int(g["treq"][k])]} if g["treq"][k] >= 0 else {}))
                   for k in range(len(g["tx"]))}
        agents.append(a)
    s = sw.Swarm.from_agents(agents)
    e = s.elect()
    s.write_back_election(agents, e)
    lead = max(agents, key=lambda a: a.agent_id)
    tids, tx, ty, treq = s.tasks_from_dict(agents[0].tasks)
    r = s.allocate(tx, ty, treq)
    s.write_back_allocation(agents, tids, r, resolver=lead)
    codes = {"OPEN": 0, "TENTATIVE": 1, "LOCKED": 2, "ASSIGNED": 3}
    st = np.array([[codes[a.tasks[k]["status"]] for k in range(len(g["tx"]))] for a in agents])
    np.testing.assert_array_equal(st, g["status"])
    assert {k: v["winner"] for k, v in lead.task_claims.items()} == \
        {k: int(w) for k, w in enumerate(g["winner"]) if w >= 0}
    # election write-back is consistent with the oracle on the radius-1 graph
    for a in agents:
        assert a.state in (agent.AgentState.LEADER, agent.AgentState.FOLLOWER)
        assert (a.state == agent.AgentState.LEADER) == (a.leader_id == a.agent_id)


def test_sharded_stepper_two_shards_on_one_gpu(sw, oracle_mod):
    """The frontier stepper + ghost kernels through ShardedSwarm: two shards driven by two
    threads on cuda:0 with an in-process halo; union-graph oracle as the reference."""
    import threading
    from shard_doubles import ThreadHalo
    from swarm_amd import gen
    from swarm_amd.dist import ShardedSwarm
    world, n_per = 2, 40000
    hub = ThreadHalo(world)
    outs, errs = {}, []

    def run(rank):
        try:
            torch.cuda.set_device(0)
            d = gen.shard_inputs(n_per, 9, world, rank, t=400)
            sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device="cuda:0",
                              halo=hub.member(rank))
            r = sh.elect(check_every=32)
            res, won, gst = sh.allocate(d["tx"], d["ty"], d["treq"])
            torch.cuda.synchronize()
            outs[rank] = dict(r=r, ids=sh.ids.cpu().numpy(), leader=r.leader.cpu().numpy(),
                              winner=res.winner.cpu().numpy(), won=won.cpu().numpy(), gst=gst)
        except Exception as e:  # surfaced below
            errs.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    ds = [gen.shard_inputs(n_per, 9, world, k, t=400) for k in range(world)]
    cat = lambda k: np.concatenate([d[k] for d in ds])  # noqa: E731
    x, y, ids = cat("x"), cat("y"), cat("ids")
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, ids)
    want = dict(zip(ids.tolist(), lead.tolist()))
    for k in range(world):
        o = outs[k]
        assert o["r"].rounds_exec == rounds
        np.testing.assert_array_equal(o["r"].changes, changes)
        assert all(want[int(i)] == int(v) for i, v in zip(o["ids"], o["leader"]))
    wa = oracle_mod.allocate(ids, x, y, cat("caps"), cat("tx"), cat("ty"), cat("treq"))
    np.testing.assert_array_equal(np.concatenate([outs[k]["winner"] for k in range(world)]), wa["winner"])
    won_want = dict(zip(ids.tolist(), wa["won"].tolist()))
    for k in range(world):
        assert all(won_want[int(i)] == int(w) for i, w in zip(outs[k]["ids"], outs[k]["won"]))


def test_elect_timed_stats(sw, oracle_mod):
    g = load_golden("elect_n10000")
    s = _swarm(sw, g, "spatial").set_graph(g["row_ptr"], g["col"])
    r = s.elect(mode="frontier", timed=True)
    assert r.rounds_exec == int(g["rounds_exec"])
    assert r.changes_total == int(g["changes"].sum())
    assert r.timed_launches == r.rounds_launched >= r.rounds_exec and r.gather_ms > 0 and r.apply_ms >= 0
    assert r.sparse_launches == r.rounds_launched - r.dense_rounds and r.sparse_ms > 0 and r.sparse_bytes > 0
    r2 = s.elect(mode="dense", timed=True)
    assert r2.rounds_exec == int(g["rounds_exec"]) and r2.gather_ms > 0


def test_native_sharded_loop_single_rank_rccl(sw, oracle_mod):
    """swarm_elect_sharded (the RCCL round loop) on a 1-rank communicator: same rounds, changes
    and leaders as the single-GPU frontier election (no halos; exercises the loop, the batched
    RCCL all-reduce and the convergence test)."""
    import ctypes
    from swarm_amd import _lib as L
    from swarm_amd import gen
    if not L.lib().swarm_comm_available():
        pytest.skip("RCCL not resolvable in this process")
    d = gen.swarm_inputs(120000, 77)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    want = s.elect(mode="frontier")
    uid = (ctypes.c_uint8 * 128)()
    L.check(L.lib().swarm_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)))
    comm = ctypes.c_void_p()
    L.check(L.lib().swarm_comm_create(ctypes.byref(comm), 1, 0, ctypes.cast(uid, ctypes.c_void_p)))
    try:
        n = s.n
        l0 = torch.empty(n, dtype=torch.int32, device="cuda")
        l1 = torch.empty(n, dtype=torch.int32, device="cuda")
        desc = L.shard_desc(n, n, s.row_ptr, s.col, s.ids, 0, 1)
        rounds = ctypes.c_int32(0)
        ch = np.zeros(1 << 12, np.int64)
        L.check(L.lib().swarm_elect_sharded(L.ctx(), comm, ctypes.byref(desc), L.ptr(l0), L.ptr(l1), len(ch),
                                            ctypes.byref(rounds), ch.ctypes.data_as(ctypes.c_void_p), L.stream()))
        r = rounds.value
        assert r == want.rounds_exec
        np.testing.assert_array_equal(ch[:r], want.changes)
        final = (l1 if r & 1 else l0).cpu().numpy()
        np.testing.assert_array_equal(final, want.leader.cpu().numpy())
    finally:
        L.lib().swarm_comm_destroy(comm)
