"""Parity at the configured scales (BASELINE.json configs C3 and C4) and past the election's
counter-ring / stamp cycles.

* C3, the headline workload: 10M agents (seed 2026, deg 16, random IDs), 10 000 tasks -- the
  exact swarm bench.py times.  Election (1 364 rounds) in both strategies against the oracle's
  frontier restatement (leaders, states, rounds_exec, every per-round change count); the
  allocation against the binned oracle on all 10 000 tasks and against the dense oracle (the
  reference algorithm, every agent x task) on 48 of them.  agent.py:263-275, 292-325.
* Long elections (> 1 024 rounds): the per-round counters live in a 512-round ring and the
  frontier stamps cycle through 255 values per buffer parity; these cases wrap both several
  times, one-GPU and through the sharded stepper.
* Directed neighbour graphs (agent.py:59-65: sensed neighbour lists need not be symmetric).
* C4: 100k agents x 100k tasks auction against oracle.auction, and the hysteresis-0 (argmax)
  allocation on 100k x 100k against the dense oracle on a task sample.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


# ------------------------------------------------------------------------------------- C3
@pytest.fixture(scope="module")
def c3(sw):
    from swarm_amd import gen
    d = gen.swarm_inputs(10_000_000, 2026, deg=16.0, t=10_000)  # bench.py's C3 inputs
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    host = dict(rp=s.row_ptr.cpu().numpy().astype(np.int64), col=s.col.cpu().numpy(), ids=s.ids.cpu().numpy(),
                x=s.pos[:, 0].cpu().numpy(), y=s.pos[:, 1].cpu().numpy(),
                caps=s.caps.cpu().numpy().view(np.uint32))
    yield d, s, host
    del s
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c3_elect(c3, oracle_mod):
    _, _, h = c3
    return oracle_mod.elect_frontier(h["rp"], h["col"], h["ids"])


def test_c3_election_full_scale(c3, c3_elect):
    d, s, h = c3
    lead, state, rounds, changes = c3_elect
    assert rounds > 1024  # the headline election wraps the 512-round counter ring
    for mode in ("frontier", "dense"):
        r = s.elect(mode=mode, max_rounds=1 << 16)
        assert r.converged and r.rounds_exec == rounds, (mode, r.rounds_exec, rounds)
        np.testing.assert_array_equal(r.changes, changes)
        np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
        np.testing.assert_array_equal(r.state.cpu().numpy(), state)


def test_c3_election_int64_offsets(c3, c3_elect):
    """The int64-row-offset instantiation (swarm_elect_i64, what a >= 2^30-edge graph such as C5's
    100M agents on one GPU runs) on the headline swarm."""
    d, s, h = c3
    lead, state, rounds, changes = c3_elect
    for compact in (True, False):
        r = s.elect(wide=True, compact=compact)
        assert r.converged and r.rounds_exec == rounds and r.compact == compact
        np.testing.assert_array_equal(r.changes, changes)
        np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
        np.testing.assert_array_equal(r.state.cpu().numpy(), state)


def test_c3_allocation_full_scale(c3, oracle_mod):
    d, s, h = c3
    r = s.allocate(d["tx"], d["ty"], d["treq"])
    assert r.stats["mode_used"] == 1 and r.stats["n_flagged"] == 0
    # all 10 000 tasks against the binned restatement (pinned to the dense one on CPU)
    want = oracle_mod.allocate_binned(h["ids"], h["x"], h["y"], h["caps"], d["tx"], d["ty"], d["treq"], use_pow=False)
    np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy().view(np.uint64), want["util"].view(np.uint64))
    np.testing.assert_array_equal(r.nclaim.cpu().numpy(), want["nclaim"])
    np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
    np.testing.assert_array_equal(r.won.cpu().numpy(), want["won"])
    assert r.stats["n_claims"] == want["n_claims"] and r.stats["n_conflicts"] == want["n_conflicts"]
    # a seeded sample of tasks against the reference algorithm itself: every agent x task, libm
    # pow squares (agent.py:340); task chains are independent with an empty claim table
    k = np.sort(np.random.default_rng(7).choice(len(d["tx"]), 48, replace=False))
    dense = oracle_mod.allocate(h["ids"], h["x"], h["y"], h["caps"], d["tx"][k], d["ty"][k], d["treq"][k])
    np.testing.assert_array_equal(r.winner.cpu().numpy()[k], dense["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy()[k], dense["util"])
    np.testing.assert_array_equal(r.nclaim.cpu().numpy()[k], dense["nclaim"])
    np.testing.assert_array_equal(r.nmsg.cpu().numpy()[k], dense["nmsg"])


# ---------------------------------------------------------------------- long elections
def _path(n):
    """Path graph 0 - 1 - ... - n-1 as CSR (rows ascending)."""
    rp = np.zeros(n + 1, np.int64)
    deg = np.full(n, 2)
    deg[0] = deg[-1] = 1
    rp[1:] = np.cumsum(deg)
    col = [u for v in range(n) for u in (v - 1, v + 1) if 0 <= u < n]
    return rp, np.array(col, np.int32)


@pytest.mark.parametrize("layout", ["input", "spatial"])
def test_long_path_wraps_ring_and_stamps(sw, oracle_mod, layout):
    """1 500 agents on a path with IDs rising along it: 1 500 rounds, each changing one agent
    fewer -- the 512-round counter ring wraps twice and each stamp parity cycles ~3 times."""
    n = 1500
    rp, col = _path(n)
    ids = np.arange(n, dtype=np.int32)
    x = np.arange(n, dtype=np.float64) * 0.9
    s = sw.Swarm(ids, x, np.zeros(n), layout=layout, device="cuda").set_graph(rp, col)
    want = oracle_mod.elect(rp, col, ids)
    assert want[2] == n
    for mode in ("dense", "frontier"):
        r = s.elect(mode=mode)
        assert r.converged and r.rounds_exec == n, mode
        np.testing.assert_array_equal(r.changes, want[3])
        np.testing.assert_array_equal(s.to_input_order(r.leader), want[0])
        np.testing.assert_array_equal(s.to_input_order(r.state), want[1])


@pytest.mark.parametrize("n_len,seed", [(1400, 3), (2600, 4)])
def test_long_strip_rgg_random_ids(sw, oracle_mod, n_len, seed):
    """A thin strip (length n_len radii, width 2, 10 agents per unit area: connected) of an RGG
    with random IDs: more than n_len / 2 rounds (> 1 024 for the longer strip) of sparse fronts,
    through the small-swarm (512-agent chunk) kernel."""
    from swarm_amd import gen
    g = np.random.default_rng(seed)
    n = int(n_len * 2 * 10)
    x, y = g.uniform(0, n_len, n), g.uniform(0, 2.0, n)
    ids = gen.random_ids(n, seed)
    s = sw.Swarm(ids, x, y, device="cuda").build_graph(1.0)
    rp, col = s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy()
    want = oracle_mod.elect(rp, col, s.ids.cpu().numpy())
    assert want[2] > n_len // 2
    for mode in ("frontier", "dense"):
        r = s.elect(mode=mode)
        assert r.rounds_exec == want[2], mode
        np.testing.assert_array_equal(r.changes, want[3])
        np.testing.assert_array_equal(r.leader.cpu().numpy(), want[0])


def test_long_election_sharded_stepper(sw, oracle_mod):
    """The frontier stepper + ghost kernels (two shards on one GPU, in-process halo) on a
    1 300-round path crossing the strip border: ring and stamps wrap in the sharded loop too."""
    import threading
    from shard_doubles import ThreadHalo
    from swarm_amd.dist import ShardedSwarm
    world, n = 2, 1300
    y = np.arange(n, dtype=np.float64) * 0.9  # a vertical path: the strips cut it once
    x = np.full(n, 0.5)
    ids = np.arange(n, dtype=np.int32)[::-1].copy()  # max ID at the bottom
    h = (y[-1] + 0.45) / world
    hub = ThreadHalo(world)
    outs, errs = {}, []

    def run(rank):
        try:
            torch.cuda.set_device(0)
            sel = (y >= rank * h) & (y < (rank + 1) * h)
            sh = ShardedSwarm(ids[sel], x[sel], y[sel], None, (rank * h, (rank + 1) * h), device="cuda:0",
                              halo=hub.member(rank), halo_depth=8)
            r = sh.elect(check_every=64)
            outs[rank] = dict(r=r, ids=sh.ids.cpu().numpy(), leader=r.leader.cpu().numpy())
        except Exception as e:  # surfaced below
            errs.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    lead, _, rounds, changes = oracle_mod.elect(rp, col, ids)
    assert rounds == n
    for k in range(world):
        assert outs[k]["r"].rounds_exec == rounds
        np.testing.assert_array_equal(outs[k]["r"].changes, changes)
        np.testing.assert_array_equal(outs[k]["leader"], np.full(len(outs[k]["ids"]), n - 1))


# ----------------------------------------------------------------------- directed graphs
def _digraph(n, out_deg, seed):
    g = np.random.default_rng(seed)
    src = np.repeat(np.arange(n), out_deg)
    dst = g.integers(0, n - 1, n * out_deg)
    dst = dst + (dst >= src)
    key = np.unique(src.astype(np.int64) * n + dst)
    src, dst = key // n, key % n
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(src, minlength=n))
    return rp, dst.astype(np.int32)


@pytest.mark.parametrize("n,deg,layout", [(3000, 2, "input"), (300_000, 3, "spatial"), (1_500_000, 3, "input")])
def test_directed_graph_election(sw, oracle_mod, n, deg, layout):
    """Asymmetric neighbour lists: FRONTIER marks through the transpose (swarm_elect_directed);
    both strategies equal the dense oracle.  300k / 1.5M agents take the 2 048-agent-chunk kernel."""
    from swarm_amd import gen
    rp, col = _digraph(n, deg, n)
    ids = gen.random_ids(n, n + 1)
    d = gen.swarm_inputs(n, 5)
    s = sw.Swarm(ids, d["x"], d["y"], layout=layout, device="cuda").set_graph(rp, col)
    assert s._hear is not None  # detected as directed
    want = oracle_mod.elect(rp, col, ids)
    for mode in ("frontier", "dense"):
        r = s.elect(mode=mode)
        assert r.rounds_exec == want[2], mode
        np.testing.assert_array_equal(r.changes, want[3])
        np.testing.assert_array_equal(s.to_input_order(r.leader), want[0])
        np.testing.assert_array_equal(s.to_input_order(r.state), want[1])


def test_directed_from_agents_bridge(sw, oracle_mod):
    """SwarmAgent objects with asymmetric sensed neighbours (update_sensors, agent.py:59-65)."""
    import agent
    n = 400
    rp, col = _digraph(n, 2, 9)
    g = np.random.default_rng(9)
    ids = g.permutation(n).astype(np.int32)
    agents = []
    for i in range(n):
        a = agent.SwarmAgent(int(ids[i]), n)
        a.position = [float(g.uniform(0, 20)), float(g.uniform(0, 20))]
        agents.append(a)
    nbrs = [list(col[rp[i]:rp[i + 1]]) for i in range(n)]
    s = sw.Swarm.from_agents(agents, neighbors=nbrs)
    r = s.elect()
    want = oracle_mod.elect(rp, col, ids)
    assert r.rounds_exec == want[2]
    s.write_back_election(agents, r)
    assert [a.leader_id for a in agents] == want[0].tolist()


# ------------------------------------------------------------------------------------ C4
@pytest.fixture(scope="module")
def c4(sw):
    from swarm_amd import gen
    d = gen.swarm_inputs(100_000, 2026 + 2, t=100_000)  # bench.py's C4 row
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    return d, s


def test_c4_auction_full_scale(c4, oracle_mod):
    d, s = c4
    want = oracle_mod.auction(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    r = s.auction(d["tx"], d["ty"], d["treq"])
    assert r.converged and r.rounds_exec == want["rounds"]
    np.testing.assert_array_equal(r.bidders, want["bidders"])
    assert r.stats["n_pairs"] == want["n_pairs"]
    np.testing.assert_array_equal(r.price.cpu().numpy().view(np.uint32), want["price"].view(np.uint32))
    perm = s.perm.cpu().numpy()
    owner = r.owner.cpu().numpy()
    np.testing.assert_array_equal(np.where(owner >= 0, perm[np.maximum(owner, 0)], -1), want["owner"])
    np.testing.assert_array_equal(s.to_input_order(r.assigned), want["assigned"])


def test_c4_argmax_allocation_full_scale(c4, oracle_mod):
    """hysteresis 0 (the north star's argmin/argmax mode, agent.py:297, 302): 100k x 100k in
    both strategies (dense = all 10^10 pairs in ID-ordered tiles), a task sample against the
    dense oracle."""
    d, s = c4
    k = np.sort(np.random.default_rng(11).choice(len(d["tx"]), 600, replace=False))
    want = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"][k], d["ty"][k], d["treq"][k],
                               hysteresis=0.0)
    res = {}
    for mode in ("binned", "dense"):
        r = s.allocate(d["tx"], d["ty"], d["treq"], hysteresis=0.0, mode=mode)
        res[mode] = r.winner.cpu().numpy()
        np.testing.assert_array_equal(res[mode][k], want["winner"])
        np.testing.assert_array_equal(r.util.cpu().numpy()[k], want["util"])
        np.testing.assert_array_equal(r.nmsg.cpu().numpy()[k], want["nmsg"])
    np.testing.assert_array_equal(res["binned"], res["dense"])


# ------------------------------------------------------------------------ input checks
def test_treq_outside_mask_rejected(sw):
    from swarm_amd import _lib, gen
    d = gen.swarm_inputs(2000, 3, t=20)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    bad = d["treq"].copy()
    bad[5] = 40
    for mode in ("binned", "dense"):
        with pytest.raises(_lib.SwarmError, match="treq outside"):
            s.allocate(d["tx"], d["ty"], bad, mode=mode)
    with pytest.raises(_lib.SwarmError, match="treq outside"):
        s.auction(d["tx"], d["ty"], bad)
    ok = d["treq"].copy()
    ok[5] = 31  # bit 31: a capability name nobody holds in this vocabulary -> no claims on it
    r = s.allocate(d["tx"], d["ty"], ok)
    assert int(r.nclaim[5]) == 0


def test_provenance_of_loaded_library(sw):
    from swarm_amd import _lib
    p = _lib.provenance()
    assert p["matches_tree"], p
