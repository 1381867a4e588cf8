"""The oracle's frontier election and binned allocation restatements, pinned against the dense
restatements (themselves pinned to the reference's golden vectors in test_oracle_golden.py) and
against the golden vectors directly.  These two are the checkers the GPU tests use at full
scale (C3: 10M agents, 1 364 rounds), where the dense oracle would take minutes.  CPU only."""
import numpy as np
import pytest

from conftest import golden_names, load_golden

ELECT = golden_names("elect_")
ALLOC = golden_names("alloc_")


@pytest.mark.parametrize("name", ELECT)
def test_frontier_oracle_matches_reference(name, oracle_mod):
    g = load_golden(name)
    leader, state, rounds, changes, active = oracle_mod.elect_frontier(g["row_ptr"], g["col"], g["ids"],
                                                                       with_active=True)
    assert rounds == int(g["rounds_exec"])
    np.testing.assert_array_equal(changes, g["changes"])
    np.testing.assert_array_equal(leader, g["leader"])
    np.testing.assert_array_equal(state, g["state"])
    assert active[0] == len(g["ids"]) and (active[1:] <= len(g["ids"])).all()


@pytest.mark.parametrize("n,seed,deg", [(200_000, 5, 16.0), (150_000, 6, 5.0), (50_000, 7, 2.0)])
def test_frontier_oracle_equals_dense_rgg(n, seed, deg, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, deg=deg)
    rp, col = oracle_mod.rgg_csr(d["x"], d["y"], 1.0)
    want = oracle_mod.elect(rp, col, d["ids"])
    got = oracle_mod.elect_frontier(rp, col, d["ids"])
    assert got[2] == want[2]
    for a, b in zip(got[:2] + got[3:], want[:2] + want[3:]):
        np.testing.assert_array_equal(a, b)


def random_digraph(n, out_deg, seed):
    """Directed graph: each agent hears out_deg random others (no self-loops, rows ascending)."""
    g = np.random.default_rng(seed)
    src = np.repeat(np.arange(n), out_deg)
    dst = g.integers(0, n - 1, n * out_deg)
    dst = dst + (dst >= src)  # skip self
    key = np.unique(src.astype(np.int64) * n + dst)
    src, dst = key // n, key % n
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(src, minlength=n))
    return rp, dst.astype(np.int32)


@pytest.mark.parametrize("n,deg,seed", [(300, 2, 1), (5000, 3, 2), (100_000, 4, 3)])
def test_frontier_oracle_directed(n, deg, seed, oracle_mod):
    """Asymmetric neighbourhoods (agent.py:59-65 sensed lists need not be symmetric): risers must
    mark the agents that HEAR them (the transpose), not the agents they hear."""
    rp, col = random_digraph(n, deg, seed)
    ids = np.random.default_rng(seed + 100).permutation(n).astype(np.int32)
    want = oracle_mod.elect(rp, col, ids)
    got = oracle_mod.elect_frontier(rp, col, ids, hear=oracle_mod.transpose_csr(rp, col))
    assert got[2] == want[2]
    np.testing.assert_array_equal(got[3], want[3])
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
    if n <= 300:
        py = oracle_mod.elect_py(rp, col, ids)
        assert py[2] == want[2]
        np.testing.assert_array_equal(py[0], want[0])
    # marking through the graph itself instead of the transpose is wrong on a directed graph
    bad = oracle_mod.elect_frontier(rp, col, ids)
    assert not (bad[2] == want[2] and np.array_equal(bad[0], want[0]) and np.array_equal(bad[3], want[3]))


def path_graph(n):
    rp = np.zeros(n + 1, np.int64)
    deg = np.full(n, 2)
    deg[0] = deg[-1] = 1
    rp[1:] = np.cumsum(deg)
    col = np.empty(rp[-1], np.int32)
    for v in range(n):
        nb = [u for u in (v - 1, v + 1) if 0 <= u < n]
        col[rp[v]:rp[v + 1]] = nb
    return rp, col


def test_frontier_oracle_long_path_and_cut(oracle_mod):
    n = 1500
    rp, col = path_graph(n)
    ids = np.arange(n, dtype=np.int32)  # max ID at one end: n - 1 change rounds + the quiet one
    want = oracle_mod.elect(rp, col, ids)
    got = oracle_mod.elect_frontier(rp, col, ids)
    assert want[2] == got[2] == n
    np.testing.assert_array_equal(got[3], want[3])
    np.testing.assert_array_equal(got[0], np.full(n, n - 1))
    # cut at max_rounds: not converged, same intermediate state
    w50 = oracle_mod.elect(rp, col, ids, max_rounds=50)
    g50 = oracle_mod.elect_frontier(rp, col, ids, max_rounds=50)
    assert w50[2] == g50[2] == -1
    np.testing.assert_array_equal(g50[0], w50[0])


@pytest.mark.parametrize("name", ALLOC)
def test_binned_allocation_oracle_matches_reference(name, oracle_mod):
    g = load_golden(name)
    r = oracle_mod.allocate_binned(g["ids"], g["x"], g["y"], g["caps"], g["tx"], g["ty"], g["treq"],
                                   winner=g.get("pre_w"), util=g.get("pre_u"))
    np.testing.assert_array_equal(r["winner"], g["winner"])
    np.testing.assert_array_equal(r["util"].view(np.uint64), g["util"].view(np.uint64))
    np.testing.assert_array_equal(r["won"], g["won"])
    assert r["n_claims"] == int(g["n_claims"]) and r["n_conflicts"] == int(g["n_conflicts"])


@pytest.mark.parametrize("kw", [{}, {"hysteresis": 0.0}, {"claim_thr": 150.0}, {"claim_thr": -1.0},
                                {"claim_thr": 35.0, "hysteresis": 1.5}])
def test_binned_allocation_oracle_equals_dense(kw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(30_000, 11, t=300)
    pre = np.where(np.arange(300) % 4 == 0, d["ids"][:300], -1).astype(np.int32)
    args = (d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    for w0, u0 in ((None, None), (pre, np.full(300, 41.5))):
        want = oracle_mod.allocate(*args, winner=w0, util=u0, **kw)
        got = oracle_mod.allocate_binned(*args, winner=w0, util=u0, **kw)
        for k in ("winner", "util", "nclaim", "nmsg", "won"):
            np.testing.assert_array_equal(got[k], want[k])


def test_utility_capability_index_outside_mask(oracle_mod):
    """A required capability index >= 32 is a name no agent holds (agent.py:343-345): U = 0,
    never the shifted-mod-32 bit (the C restatement must not shift by >= 32)."""
    caps = np.array([0xFFFFFFFF, 0x2, 0x0], np.uint32)
    for rq in (32, 33, 63, 127):
        u = oracle_mod.utility(np.zeros(3), np.zeros(3), caps, np.ones(3), np.zeros(3), np.full(3, rq, np.int8))
        np.testing.assert_array_equal(u, 0.0)
        assert oracle_mod.utility_py(0.0, 0.0, 0xFFFFFFFF, 1.0, 0.0, rq) == 0.0
    u = oracle_mod.utility(np.zeros(3), np.zeros(3), caps, np.ones(3), np.zeros(3), np.full(3, 31, np.int8))
    np.testing.assert_array_equal(u, [50.0, 0.0, 0.0])
