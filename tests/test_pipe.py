"""The pipelined election tail (k_pipe_rounds, DESIGN.md §4 "pipelined tail") against the oracle's
frontier restatement of contract E2 (agent.py:263-275): leaders, states, rounds_exec and every
per-round change count, bit for bit.

The pipelined rounds run many rounds in one launch, each chunk of agents waiting only for the
chunks within the graph's reach to finish the previous round, with agent-scope (sc1) hand-offs of
leaders and stamps.  pipe="early" makes the marks agent-ordered from the first sparse round, so the
pipeline runs nearly the whole election; these cases cover both chunk sizes (512-agent chunks below
2^20 agents, 2 048 above), int32 and int64 row offsets, tiny grids (fewer chunks than the reach),
long elections that wrap the counter ring and the stamp values, max_rounds cuts inside a launch,
back-to-back calls, and graphs whose reach is too long for the pipeline (it must stay off).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


def _check(r, want, m=None):
    lead, state, rounds, changes = want
    if m is None:
        assert r.converged and r.rounds_exec == rounds, (r.rounds_exec, rounds)
        np.testing.assert_array_equal(r.changes, changes)
        np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
        np.testing.assert_array_equal(r.state.cpu().numpy(), state)
    else:
        assert not r.converged and r.rounds_exec == m
        np.testing.assert_array_equal(r.changes, changes[:m])


@pytest.mark.parametrize("n,deg,seed", [(3, 16.0, 1), (700, 3.0, 2), (5_000, 16.0, 3), (120_000, 16.0, 4),
                                        (300_000, 6.0, 5), (1_048_577, 16.0, 6), (2_100_000, 16.0, 7)])
def test_pipe_early_matches_oracle(sw, oracle_mod, n, deg, seed):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, deg=deg)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    rp = s.row_ptr.cpu().numpy().astype(np.int64)
    want = oracle_mod.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy())
    for pipe in ("early", True, False):
        r = s.elect(pipe=pipe)
        _check(r, want)
        if pipe == "early" and want[2] > 12 and s.n_edges:
            assert r.pipe_from > 0 and r.pipe_rounds > 0 and r.pipe_grid >= 1
        if pipe is False:
            assert r.pipe_from == 0


def test_pipe_int64_offsets(sw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(1_100_000, 11, deg=16.0)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    want = oracle_mod.elect_frontier(s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy(),
                                     s.ids.cpu().numpy())
    r = s.elect(wide=True, pipe="early")
    _check(r, want)
    assert r.pipe_from > 0


def test_pipe_long_path_wraps_ring_and_stamps(sw, oracle_mod):
    """2 000 agents on a path, IDs rising along it: 2 000 rounds (the 512-round counter ring wraps,
    every stamp value recurs), almost all of them pipelined, on a grid of 4 chunks (reach 1)."""
    n = 2000
    rp = np.zeros(n + 1, np.int64)
    deg = np.full(n, 2)
    deg[0] = deg[-1] = 1
    rp[1:] = np.cumsum(deg)
    col = np.array([u for v in range(n) for u in (v - 1, v + 1) if 0 <= u < n], np.int32)
    ids = np.arange(n, dtype=np.int32)
    s = sw.Swarm(ids, np.arange(n) * 0.9, np.zeros(n), layout="input", device="cuda").set_graph(rp, col)
    want = oracle_mod.elect_frontier(rp, col, ids)
    assert want[2] == n
    r = s.elect(pipe="early")
    _check(r, want)
    assert r.pipe_rounds > n - 40


@pytest.mark.parametrize("pipe", ["early", True])
def test_pipe_cuts_and_repeats(sw, oracle_mod, pipe):
    """max_rounds cuts inside pipelined launches, and back-to-back calls on one swarm (stamps and
    counter slots left by a cut run must not leak into the next)."""
    from swarm_amd import gen
    d = gen.swarm_inputs(200_000, 21, deg=12.0)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    rp, col, ids = s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy(), s.ids.cpu().numpy()
    want = oracle_mod.elect_frontier(rp, col, ids)
    rounds = want[2]
    for m in (rounds // 3, 57, rounds - 1, 1 << 16, 30, 1 << 16):
        r = s.elect(pipe=pipe, max_rounds=m)
        if m >= rounds:
            _check(r, want)
        else:
            _check(r, want, m)
            cut = oracle_mod.elect_frontier(rp, col, ids, max_rounds=m)
            np.testing.assert_array_equal(r.leader.cpu().numpy(), cut[0])


def test_pipe_off_when_reach_too_long(sw, oracle_mod):
    """A graph whose edges span more than 31 chunks (16-bit columns still fit): the election keeps
    its per-round launches (pipe_from 0) and stays exact."""
    n = 100_000
    g = np.random.default_rng(5)
    ids = g.permutation(n).astype(np.int32)
    src = np.arange(n - 20_000)
    pairs = np.concatenate([np.stack([src, src + 20_000], 1), np.stack([src[:-1], src[:-1] + 1], 1)])
    u = np.concatenate([pairs[:, 0], pairs[:, 1]])
    v = np.concatenate([pairs[:, 1], pairs[:, 0]])
    order = np.lexsort((v, u))
    u, v = u[order], v[order]
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(u, minlength=n))
    col = v.astype(np.int32)
    s = sw.Swarm(ids, np.arange(n, dtype=np.float64), np.zeros(n), layout="input", device="cuda").set_graph(rp, col)
    assert s.graph_compact() is not None
    want = oracle_mod.elect_frontier(rp, col, ids)
    r = s.elect(pipe="early")
    _check(r, want)
    assert r.pipe_from == 0
