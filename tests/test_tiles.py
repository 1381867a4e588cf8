"""Tiled tail rounds of the election (swarm_elect_tiled, DESIGN.md §4 'tiled rounds').

A swarm in cell order whose edges join cells at most one apart runs its late E2 rounds
(agent.py:263-275 under contract E2) as launches of 4 rounds over 16 x 16-cell tiles held in LDS.
The results must equal the oracle's exactly: leaders, states, rounds_exec, every per-round change
count -- with the tiles from the first sparse round on ('early') and with the default switch, at
max_rounds cuts inside a launch, on sparse / disconnected graphs and next to the fallbacks (a
non-local graph, a directed one)."""
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


def _oracle(oracle_mod, s, max_rounds=1 << 16):
    rp = s.row_ptr.cpu().numpy().astype(np.int64)
    return oracle_mod.elect(rp, s.col.cpu().numpy(), s.ids.cpu().numpy(), max_rounds=max_rounds)


def _check(r, want):
    lead, state, rounds, changes = want
    assert r.rounds_exec == rounds, (r.rounds_exec, rounds)
    np.testing.assert_array_equal(r.changes, changes)
    np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
    np.testing.assert_array_equal(r.state.cpu().numpy(), state)


@pytest.mark.parametrize("n,deg,seed", [(30_000, 16.0, 1), (200_000, 16.0, 2), (120_000, 6.0, 3), (60_000, 3.0, 4),
                                        (1_000_000, 16.0, 5)])
def test_tiled_rounds_match_oracle(sw, oracle_mod, n, deg, seed):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, deg=deg)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    assert s.tile_index() is not None
    want = _oracle(oracle_mod, s)
    for tiles in ("early", True, False):
        r = s.elect(tiles=tiles)
        _check(r, want)
        if tiles == "early" and want[2] > 40:
            assert r.tile_rounds > 0 and r.tile_launches > 0
        if tiles != "early":  # the default threshold never switches
            assert r.tile_rounds == 0


@pytest.mark.parametrize("cut", [27, 30, 31, 33, 64, 101])
def test_tiled_rounds_max_rounds_cuts(sw, oracle_mod, cut):
    """Cuts inside and at the end of a 4-round launch: the state after exactly `cut` rounds."""
    from swarm_amd import gen
    d = gen.swarm_inputs(150_000, 11)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    full = _oracle(oracle_mod, s)
    assert full[2] > cut
    # the state after `cut` Jacobi rounds, by numpy (the max ID within `cut` hops)
    rp, col, ids = s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy(), s.ids.cpu().numpy()
    lead = ids.astype(np.int64)
    starts = rp[:-1]
    nonempty = np.diff(rp) > 0
    for _ in range(cut):
        m = np.maximum.reduceat(lead[col], starts[nonempty]) if col.size else np.zeros(0, np.int64)
        nxt = lead.copy()
        nxt[nonempty] = np.maximum(lead[nonempty], m)
        lead = nxt
    r = s.elect(tiles="early", max_rounds=cut)
    assert not r.converged and r.rounds_exec == cut
    np.testing.assert_array_equal(r.changes, full[3][:cut])
    np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
    np.testing.assert_array_equal(r.state.cpu().numpy(), np.where(lead == ids, 3, 1))


def test_tiled_rounds_repeat_and_ids_at_int32_top(sw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(80_000, 13)
    ids = (np.int64(2**31 - 1) - d["ids"].astype(np.int64) * 7).astype(np.int32)  # distinct, near INT32_MAX
    s = sw.Swarm(ids, d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    want = _oracle(oracle_mod, s)
    for _ in range(2):
        _check(s.elect(tiles="early"), want)


def test_non_local_graph_falls_back(sw, oracle_mod):
    """A long edge (agents far apart): no tile index, the plain frontier path, same results."""
    from swarm_amd import gen
    d = gen.swarm_inputs(40_000, 17)
    rp, col = gen.rgg_csr(d["x"], d["y"], 1.0)
    # add the edge 0 <-> 1 (far apart, symmetric)
    rows = [list(col[rp[i]:rp[i + 1]]) for i in range(len(d["x"]))]
    a, b = 0, int(np.argmax((d["x"] - d["x"][0]) ** 2 + (d["y"] - d["y"][0]) ** 2))
    rows[a].append(b)
    rows[b].append(a)
    rows = [sorted(set(r)) for r in rows]
    rp2 = np.zeros(len(rows) + 1, np.int64)
    rp2[1:] = np.cumsum([len(r) for r in rows])
    col2 = np.array([c for r in rows for c in r], np.int64)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").set_graph(rp2, col2)
    assert s.tile_index() is None
    want = _oracle(oracle_mod, s)
    _check(s.elect(tiles="early"), want)


def test_tile_index_after_physics_rebuilds(sw, oracle_mod):
    """Positions move (physics_step), the graph is rebuilt: the tile index follows the new cell
    order, or is refused when the storage order is no longer cell order."""
    from swarm_amd import gen
    d = gen.swarm_inputs(50_000, 19)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    s.elect()
    s.physics_step(np.array([[20.0, 20.0, 2.0]]), steps=4)
    s.build_graph(1.0)
    want = _oracle(oracle_mod, s)
    _check(s.elect(tiles="early"), want)
