"""16-bit column deltas for the election (swarm_graph_compact / swarm_elect_compact).

The compact columns are an MI355X layout with no reference counterpart: the bar is that the
election through them returns exactly what the int32-column path and the oracle return (leaders,
states, rounds, every per-round change count; reference semantics agent.py:263-275), in both
modes and at both sparse chunk sizes, and that a graph whose deltas do not fit is refused
(SWARM_ERR_RANGE) and elected through the int32 columns instead.
"""
import ctypes

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


def c16_np(rp, col):
    """numpy restatement of the documented layout (include/swarm.h, swarm_graph_compact)."""
    src = np.repeat(np.arange(len(rp) - 1, dtype=np.int64), np.diff(rp))
    return (np.asarray(col, np.int64) - (src & ~63)).astype(np.int16)


def far_graph(sw, n=150_000, seed=41):
    """A swarm graph whose first 4 096 agents are stored at the end: their neighbours' 16-bit deltas
    do not fit (swarm_graph_compact refuses it; the escaped build marks those columns)."""
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    n = s.n
    perm = np.concatenate([np.arange(4096, n), np.arange(4096)])
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    rp = s.row_ptr.cpu().numpy().astype(np.int64)
    col = s.col.cpu().numpy().astype(np.int64)
    deg = np.diff(rp)[perm]
    rp2 = np.concatenate([[0], np.cumsum(deg)])
    flat = np.repeat(rp[:-1][perm] - rp2[:-1], deg) + np.arange(rp2[-1])
    col2 = inv[col[flat]]
    ids2 = s.ids.cpu().numpy()[perm]
    rp_t = torch.as_tensor(rp2.astype(np.int32), device="cuda")
    col_t = torch.as_tensor(col2.astype(np.int32), device="cuda")
    return n, deg, rp_t, col_t, ids2, col2


def test_graph_compact_layout(sw):
    from swarm_amd import gen
    d = gen.swarm_inputs(200000, 31)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    c = s.graph_compact()
    assert c is not None and c.numel() == s.n_edges
    np.testing.assert_array_equal(c.cpu().numpy(), c16_np(s.row_ptr.cpu().numpy(), s.col.cpu().numpy()))


@pytest.mark.parametrize("n,seed", [(120000, 51), (1_200_000, 52)])
def test_elect_compact_vs_int32_vs_oracle(sw, oracle_mod, n, seed):
    # 120k agents: 512-stamp chunks; 1.2M: 2 048-stamp chunks
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    assert s.graph_compact() is not None
    lead, state, rounds, changes = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    for mode in ("frontier", "dense"):
        for compact in (True, False):
            r = s.elect(mode=mode, compact=compact)
            assert r.converged and r.rounds_exec == rounds, (mode, compact)
            np.testing.assert_array_equal(r.changes, changes)
            np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)
            np.testing.assert_array_equal(r.state.cpu().numpy(), state)


def test_far_neighbours_refused_and_elected_with_int32(sw, oracle_mod):
    """Input storage order of a random swarm: neighbours lie anywhere, deltas overflow int16."""
    from swarm_amd import _lib, gen
    d = gen.swarm_inputs(100000, 61)
    s = sw.Swarm(d["ids"], d["x"], d["y"], layout="input", device="cuda").build_graph(1.0)
    c16 = torch.empty(s.n_edges, dtype=torch.int16, device="cuda")
    rc = _lib.lib().swarm_graph_compact(_lib.ctx(), s.n, _lib.ptr(s.row_ptr), _lib.ptr(s.col), _lib.ptr(c16),
                                        _lib.stream())
    assert rc == _lib.ERR_RANGE
    assert s.graph_compact() is None
    r = s.elect()
    lead, state, rounds, changes = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    assert r.rounds_exec == rounds
    np.testing.assert_array_equal(r.changes, changes)
    np.testing.assert_array_equal(r.leader.cpu().numpy(), lead)


def test_compact_rebuilt_after_graph_change(sw, oracle_mod):
    from swarm_amd import gen
    d = gen.swarm_inputs(50000, 12)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    r1 = s.elect()
    c1 = s.graph_compact()
    assert s.graph_compact() is c1  # cached while the graph is unchanged
    # in place: every edge now points at its own agent (no propagation at all)
    s.col.copy_(torch.repeat_interleave(torch.arange(s.n, dtype=torch.int32, device="cuda"),
                                        s.row_ptr.diff().long()))
    r2 = s.elect()
    assert s.graph_compact() is not c1
    assert r1.rounds_exec > 1 and r2.rounds_exec == 1
    np.testing.assert_array_equal(r2.leader.cpu().numpy(), s.ids.cpu().numpy())


def test_elect_compact_null_is_int32_path(sw, oracle_mod):
    """swarm_elect_compact with col16 = NULL is swarm_elect."""
    from swarm_amd import _lib, gen
    d = gen.swarm_inputs(30000, 21)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    lead = torch.empty(s.n, dtype=torch.int32, device="cuda")
    state = torch.empty(s.n, dtype=torch.uint8, device="cuda")
    rounds = ctypes.c_int32(0)
    _lib.check(_lib.lib().swarm_elect_compact(_lib.ctx(), s.n, _lib.ptr(s.row_ptr), _lib.ptr(s.col), None,
                                              _lib.ptr(s.ids), _lib.ptr(lead), _lib.ptr(state), 1 << 16,
                                              _lib.ELECT_FRONTIER, ctypes.byref(rounds), None, None, _lib.stream()))
    o_lead, o_state, o_rounds, _ = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    assert rounds.value == o_rounds
    np.testing.assert_array_equal(lead.cpu().numpy(), o_lead)
    np.testing.assert_array_equal(state.cpu().numpy(), o_state)


@pytest.mark.parametrize("offset", [0, 1, 4, 8])
def test_elect_compact_any_column_alignment(sw, oracle_mod, offset):
    """The dense rounds read 16-byte aligned 16-bit columns 8 per lane (Col16A); a column array
    that is not 16-byte aligned (a view 2, 8 or 16 bytes into a buffer) takes the 2-byte loads.
    Both through the C-ABI, same results as the oracle (including the array's last rows, whose
    16-byte groups run past the end and are read one column at a time)."""
    from swarm_amd import _lib, gen
    d = gen.swarm_inputs(150_000, 61 + offset)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    c = s.graph_compact()
    assert c is not None
    buf = torch.empty(c.numel() + 16, dtype=torch.int16, device=c.device)
    view = buf[offset:offset + c.numel()]
    view.copy_(c)
    lead, state, rounds, changes = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    n = s.n
    leader = torch.empty(n, dtype=torch.int32, device=c.device)
    st = torch.empty(n, dtype=torch.uint8, device=c.device)
    got = np.zeros(1 << 16, np.int64)
    rx = ctypes.c_int32(0)
    for mode in (_lib.ELECT_FRONTIER, _lib.ELECT_DENSE):
        _lib.check(_lib.lib().swarm_elect_compact(
            _lib.ctx(), n, _lib.ptr(s.row_ptr), _lib.ptr(s.col), _lib.ptr(view), _lib.ptr(s.ids),
            _lib.ptr(leader), _lib.ptr(st), 1 << 16, mode, ctypes.byref(rx),
            got.ctypes.data_as(ctypes.c_void_p), None, _lib.stream()))
        torch.cuda.synchronize()
        assert rx.value == rounds
        np.testing.assert_array_equal(got[:rounds], changes)
        np.testing.assert_array_equal(leader.cpu().numpy(), lead)
        np.testing.assert_array_equal(st.cpu().numpy(), state)


def test_graph_compact_escaped_layout_and_sharded_election(sw):
    """swarm_graph_compact_escaped: deltas outside [-32767, 32767] become -32768 (escapes, read from the
    int32 columns), counted; then the frontier stepper over those columns (swarm_frontier_set_compact_escaped)
    returns the int32-column stepper's leaders and per-round counts exactly."""
    from swarm_amd import _lib
    n, deg, rp_t, col_t, ids2, col2 = far_graph(sw)
    c16 = torch.empty(col_t.numel(), dtype=torch.int16, device="cuda")
    L = _lib.lib()
    assert L.swarm_graph_compact(_lib.ctx(), n, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(c16), _lib.stream()) \
        == _lib.ERR_RANGE
    ne = ctypes.c_int64(0)
    _lib.check(L.swarm_graph_compact_escaped(_lib.ctx(), n, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(c16),
                                             ctypes.byref(ne), _lib.stream()))
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    delta = col2 - (src & ~63)
    fits = (delta >= -32767) & (delta <= 32767)
    assert ne.value == int((~fits).sum()) > 0
    want = np.where(fits, delta, -32768).astype(np.int16)
    np.testing.assert_array_equal(c16.cpu().numpy(), want)
    # the frontier stepper over all rows: int32 columns vs escaped 16-bit columns
    from swarm_amd.dist import GpuBackend
    ids_t = torch.as_tensor(ids2.astype(np.int32), device="cuda")
    res = []
    for cc, esc in ((None, False), (c16, True)):
        be = GpuBackend(torch.device("cuda"))
        lead = (torch.empty_like(ids_t), torch.empty_like(ids_t))
        be.begin(0, n, ids_t, lead, cc, escaped=esc)
        ch = []
        for t in range(1, 100_000):
            be.step(t, rp_t, col_t, lead)
            c = int(be.changes(t, t)[0])
            ch.append(c)
            if c == 0:
                break
        res.append((ch, lead[len(ch) & 1].cpu().numpy()))
    assert res[0][0] == res[1][0] and res[0][0][-1] == 0
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_escaped_columns_refused_by_plain_readers(sw, oracle_mod):
    """swarm_graph_compact_escaped's columns hold -32768 sentinels that the plain 16-bit readers would
    decode as a delta 32 768 below the row base (round 5: an illegal address in k_sparse_block).  Every
    entry point that reads plain 16-bit columns refuses them with SWARM_ERR_ARG before any round runs:
    the buffer this ctx built (remembered), a copy of it (the device column check), the int64-offset
    election, the stepper (at set time, or at its first step for the copy), the sharded loop on its own,
    and a buffer of out-of-range deltas.  The ctx then still elects exactly (agent.py:263-275)."""
    import ctypes
    from swarm_amd import _lib
    n, deg, rp_t, col_t, ids2, col2 = far_graph(sw)
    L, cx, st = _lib.lib(), _lib.ctx(), _lib.stream()
    c16 = torch.empty(col_t.numel(), dtype=torch.int16, device="cuda")
    ne = ctypes.c_int64(0)
    _lib.check(L.swarm_graph_compact_escaped(cx, n, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(c16),
                                             ctypes.byref(ne), st))
    assert ne.value > 0
    copy = c16.clone()
    garbage = torch.full_like(c16, 32767)  # every row base + 32767: past the end for the last rows
    ids_t = torch.as_tensor(ids2.astype(np.int32), device="cuda")
    rp64 = rp_t.to(torch.int64)
    lead = torch.empty(n, dtype=torch.int32, device="cuda")
    state = torch.empty(n, dtype=torch.uint8, device="cuda")
    rx = ctypes.c_int32(0)
    for buf in (c16, copy, garbage):
        for fn, rp in ((L.swarm_elect_compact, rp_t), (L.swarm_elect_compact_i64, rp64)):
            # (SWARM_ELECT_TRUST_C16 vouches only for buffers swarm_graph_compact wrote: none of these)
            for mode in (_lib.ELECT_FRONTIER, _lib.ELECT_DENSE, _lib.ELECT_FRONTIER | _lib.ELECT_TRUST_C16):
                rc = fn(cx, n, _lib.ptr(rp), _lib.ptr(col_t), _lib.ptr(buf), _lib.ptr(ids_t), _lib.ptr(lead),
                        _lib.ptr(state), 1 << 16, mode, ctypes.byref(rx), None, None, st)
                assert rc == _lib.ERR_ARG, (fn, rc, _lib.last_error())
    # the stepper: the remembered buffer at set time, the copy and the garbage at the first step
    L0, L1 = torch.empty_like(ids_t), torch.empty_like(ids_t)
    _lib.check(L.swarm_frontier_begin(cx, n, n, _lib.ptr(ids_t), _lib.ptr(L0), _lib.ptr(L1), st))
    assert L.swarm_frontier_set_compact(cx, _lib.ptr(c16)) == _lib.ERR_ARG
    assert "escaped" in _lib.last_error()
    for buf in (copy, garbage):
        _lib.check(L.swarm_frontier_begin(cx, n, n, _lib.ptr(ids_t), _lib.ptr(L0), _lib.ptr(L1), st))
        _lib.check(L.swarm_frontier_set_compact(cx, _lib.ptr(buf)))
        assert L.swarm_frontier_step(cx, 1, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(L0), _lib.ptr(L1), st) \
            == _lib.ERR_ARG
    # escaped reading of an out-of-range buffer is refused too
    _lib.check(L.swarm_frontier_begin(cx, n, n, _lib.ptr(ids_t), _lib.ptr(L0), _lib.ptr(L1), st))
    _lib.check(L.swarm_frontier_set_compact_escaped(cx, _lib.ptr(garbage)))
    assert L.swarm_frontier_step(cx, 1, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(L0), _lib.ptr(L1), st) \
        == _lib.ERR_ARG
    # the sharded loop (one rank, no communicator) with the escaped columns declared plain
    for buf in (c16, copy):
        sh = _lib.shard_desc(n, n, rp_t, col_t, ids_t, 0, 1, col16=buf, col16_escaped=False)
        rc = L.swarm_elect_sharded(cx, None, ctypes.byref(sh), _lib.ptr(L0), _lib.ptr(L1), 1 << 16,
                                   ctypes.byref(rx), None, st)
        assert rc == _lib.ERR_ARG, _lib.last_error()
    # the same ctx, the same columns declared escaped: exact against the oracle
    o_lead, o_state, o_rounds, o_changes = oracle_mod.elect(rp_t.cpu().numpy(), col2.astype(np.int32), ids2)
    sh = _lib.shard_desc(n, n, rp_t, col_t, ids_t, 0, 1, col16=c16, col16_escaped=True)
    _lib.check(L.swarm_elect_sharded(cx, None, ctypes.byref(sh), _lib.ptr(L0), _lib.ptr(L1), 1 << 16,
                                     ctypes.byref(rx), None, st))
    assert rx.value == o_rounds
    np.testing.assert_array_equal((L0 if o_rounds % 2 == 0 else L1).cpu().numpy(), o_lead)
    _lib.check(L.swarm_elect(cx, n, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(ids_t), _lib.ptr(lead),
                             _lib.ptr(state), 1 << 16, _lib.ELECT_FRONTIER, ctypes.byref(rx), None, None, st))
    torch.cuda.synchronize()
    assert rx.value == o_rounds
    np.testing.assert_array_equal(lead.cpu().numpy(), o_lead)
    np.testing.assert_array_equal(state.cpu().numpy(), o_state)


def test_trusted_columns_need_the_ctx_record(sw, oracle_mod):
    """SWARM_ELECT_TRUST_C16 (Swarm.elect passes it for the columns its graph_compact built) skips the
    column check only for a buffer this ctx's swarm_graph_compact wrote from the same row_ptr / col / n:
    exact there; a call with another row_ptr is checked as usual; and once swarm_graph_compact_escaped
    rewrites the buffer its record is gone (refused).  Reference semantics agent.py:263-275."""
    from swarm_amd import _lib, gen
    L, cx, st = _lib.lib(), _lib.ctx(), _lib.stream()
    n, deg, rp_t, col_t, ids2, col2 = far_graph(sw)
    d = gen.swarm_inputs(30_000, 5, deg=12.0)
    s2 = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    buf = torch.empty(max(s2.n_edges, col_t.numel()), dtype=torch.int16, device="cuda")
    _lib.check(L.swarm_graph_compact(cx, s2.n, _lib.ptr(s2.row_ptr), _lib.ptr(s2.col), _lib.ptr(buf), st))
    m = _lib.ELECT_FRONTIER | _lib.ELECT_TRUST_C16
    lead2, st2 = torch.empty_like(s2.leader), torch.empty_like(s2.state)
    rx = ctypes.c_int32(0)
    ch = np.zeros(1 << 12, np.int64)
    want = oracle_mod.elect(s2.row_ptr.cpu().numpy(), s2.col.cpu().numpy(), s2.ids.cpu().numpy())
    for rp in (s2.row_ptr, s2.row_ptr.clone()):  # the recorded row_ptr (trusted), a copy (checked)
        _lib.check(L.swarm_elect_compact(cx, s2.n, _lib.ptr(rp), _lib.ptr(s2.col), _lib.ptr(buf), _lib.ptr(s2.ids),
                                         _lib.ptr(lead2), _lib.ptr(st2), 1 << 12, m, ctypes.byref(rx),
                                         ch.ctypes.data_as(ctypes.c_void_p), None, st))
        assert rx.value == want[2]
        np.testing.assert_array_equal(ch[:rx.value], want[3])
        np.testing.assert_array_equal(lead2.cpu().numpy(), want[0])
    ne = ctypes.c_int64(0)
    _lib.check(L.swarm_graph_compact_escaped(cx, n, _lib.ptr(rp_t), _lib.ptr(col_t), _lib.ptr(buf), ctypes.byref(ne),
                                             st))
    assert ne.value > 0
    rc = L.swarm_elect_compact(cx, s2.n, _lib.ptr(s2.row_ptr), _lib.ptr(s2.col), _lib.ptr(buf), _lib.ptr(s2.ids),
                               _lib.ptr(lead2), _lib.ptr(st2), 1 << 12, m, ctypes.byref(rx), None, None, st)
    assert rc == _lib.ERR_ARG
