"""Record-list tail of the election (swarm_elect_records, DESIGN.md §4 'record tail').

The late E2 rounds (agent.py:263-275 under contract E2) are computed as per-agent pareto lists of
records (round offset, value) over 8 x 8-cell tiles held on chip, ~8 rounds per launch, and the
per-round changes and leaders are read off the lists.  The results must equal the oracle's exactly:
leaders, states, rounds_exec, every per-round change count -- with the tail from the first sparse
round on ('early', where long lists may overflow and hand the election back to the frontier rounds)
and with the default switch, at max_rounds cuts inside the tail, on sparse / disconnected graphs,
with IDs at the top of the int32 range, repeated calls (list generations), and next to the
fallbacks (a non-local graph)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


def _oracle(oracle_mod, s, max_rounds=1 << 16):
    rp = s.row_ptr.cpu().numpy().astype(np.int64)
    return oracle_mod.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy(), max_rounds=max_rounds)[:4]


def _check(r, want):
    lead, state, rounds, changes = want
    assert r.rounds_exec == rounds, (r.rounds_exec, rounds)
    np.testing.assert_array_equal(r.changes, changes)
    np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
    np.testing.assert_array_equal(r.state.cpu().numpy(), state)


@pytest.mark.parametrize("n,deg,seed", [(30_000, 16.0, 1), (200_000, 16.0, 2), (120_000, 6.0, 3), (60_000, 3.0, 4),
                                        (1_000_000, 16.0, 5)])
def test_record_tail_matches_oracle(sw, oracle_mod, n, deg, seed):
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed, deg=deg)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    assert s.record_index() is not None
    want = _oracle(oracle_mod, s)
    for records in ("early", True, False):
        r = s.elect(records=records)
        _check(r, want)
        if records == "early" and want[2] > 40:
            assert r.record_from > 0 or r.record_fallback != 0, (r.record_from, r.record_fallback)
        if not records:
            assert r.record_from == 0


@pytest.mark.parametrize("cut", [12, 19, 33, 64, 101, 170])
def test_record_tail_max_rounds_cuts(sw, oracle_mod, cut):
    """Cuts inside the tail (inside a launch's window and at its end): the state after exactly
    `cut` rounds, not converged."""
    from swarm_amd import gen
    d = gen.swarm_inputs(150_000, 11)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    full = _oracle(oracle_mod, s)
    assert full[2] > cut
    want = _oracle(oracle_mod, s, max_rounds=cut)
    r = s.elect(records="early", max_rounds=cut)
    assert not r.converged and r.rounds_exec == cut
    np.testing.assert_array_equal(r.changes, full[3][:cut])
    np.testing.assert_array_equal(r.leader.cpu().numpy(), want[0])
    np.testing.assert_array_equal(r.state.cpu().numpy(), want[1])


def test_record_tail_cut_at_last_change(sw, oracle_mod):
    """max_rounds = the last round with a change: every round changed something -> not converged;
    max_rounds = one more: converged."""
    from swarm_amd import gen
    d = gen.swarm_inputs(90_000, 23)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    full = _oracle(oracle_mod, s)
    last = full[2] - 1
    r = s.elect(records="early", max_rounds=last)
    assert not r.converged and r.rounds_exec == last
    np.testing.assert_array_equal(r.leader.cpu().numpy(), full[0])
    r = s.elect(records="early", max_rounds=last + 1)
    assert r.converged
    _check(r, full)


def test_record_tail_repeat_and_ids_at_int32_top(sw, oracle_mod):
    """IDs near INT32_MAX; repeated calls on one ctx reuse the list buffers (generations)."""
    from swarm_amd import gen
    d = gen.swarm_inputs(80_000, 13)
    ids = (np.int64(2**31 - 1) - d["ids"].astype(np.int64) * 7).astype(np.int32)  # distinct, near INT32_MAX
    s = sw.Swarm(ids, d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    want = _oracle(oracle_mod, s)
    for _ in range(3):
        _check(s.elect(records="early"), want)
        _check(s.elect(records=True), want)


def test_record_tail_after_other_swarm(sw, oracle_mod):
    """A larger swarm's lists in the ctx buffers, then a smaller one: stale entries never count."""
    from swarm_amd import gen
    big = gen.swarm_inputs(300_000, 29)
    small = gen.swarm_inputs(50_000, 31)
    sb = sw.Swarm(big["ids"], big["x"], big["y"], big["caps"], device="cuda").build_graph(1.0)
    ss = sw.Swarm(small["ids"], small["x"], small["y"], small["caps"], device="cuda").build_graph(1.0)
    wb, ws = _oracle(oracle_mod, sb), _oracle(oracle_mod, ss)
    _check(sb.elect(records="early"), wb)
    _check(ss.elect(records="early"), ws)
    _check(sb.elect(records=True), wb)


def test_record_index_refuses_non_local_graph(sw, oracle_mod):
    """A long edge (agents far apart): no record index, the plain frontier path, same results."""
    from swarm_amd import gen
    d = gen.swarm_inputs(40_000, 17)
    rp, col = gen.rgg_csr(d["x"], d["y"], 1.0)
    rows = [list(col[rp[i]:rp[i + 1]]) for i in range(len(d["x"]))]
    a, b = 0, int(np.argmax((d["x"] - d["x"][0]) ** 2 + (d["y"] - d["y"][0]) ** 2))
    rows[a].append(b)
    rows[b].append(a)
    rows = [sorted(set(r)) for r in rows]
    rp2 = np.zeros(len(rows) + 1, np.int64)
    rp2[1:] = np.cumsum([len(r) for r in rows])
    col2 = np.array([c for r in rows for c in r], np.int64)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").set_graph(rp2, col2)
    assert s.record_index() is None
    want = _oracle(oracle_mod, s)
    _check(s.elect(records="early"), want)


def test_record_tail_after_physics_rebuild(sw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(50_000, 19)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    s.elect(records=True)
    s.physics_step(np.array([[20.0, 20.0, 2.0]]), steps=4)
    s.build_graph(1.0)
    want = _oracle(oracle_mod, s)
    _check(s.elect(records="early"), want)
