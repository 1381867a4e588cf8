"""ELL rows for the sparse election rounds (swarm_graph_ell / swarm_elect_ell).

The ELL rows are an MI355X layout with no reference counterpart: 32 16-bit deltas per agent in
one 64-byte row, so that a sparse round gathers a marked agent's neighbours without a row_ptr
load.  The bar: the layout is exactly the documented one (include/swarm.h), and the election
through it returns what the CSR paths and the oracle return -- leaders, states, rounds, every
per-round change count, the marked-agent and edge totals (reference semantics agent.py:263-275)
-- at both sparse chunk sizes and with rows longer than 32 neighbours (walked through the CSR).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PAD, LONG = -32768, -32767


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


def ell_np(rp, c16):
    """numpy restatement of the layout: slot s of row v holds edge (s % 8) * 4 + s // 8."""
    n = len(rp) - 1
    out = np.full((n, 32), PAD, np.int16)
    deg = np.diff(rp)
    s = np.arange(32)
    k = (s % 8) * 4 + s // 8
    for v in range(n):
        if deg[v] > 32:
            out[v, :] = LONG
        else:
            m = k < deg[v]
            out[v, m] = c16[rp[v] + k[m]]
    return out.reshape(-1)


def test_graph_ell_layout(sw):
    from swarm_amd import gen
    d = gen.swarm_inputs(20000, 41)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.6)  # some rows > 32
    rp = s.row_ptr.cpu().numpy()
    assert np.diff(rp).max() > 32
    e = s.graph_ell()
    assert e is not None and e.numel() == 32 * s.n
    np.testing.assert_array_equal(e.cpu().numpy(), ell_np(rp, s.graph_compact().cpu().numpy()))


def _elect_both(s, mode="frontier"):
    r_ell = s.elect(mode=mode)
    ell_stats = (r_ell.rounds_exec, r_ell.changes.copy(), r_ell.leader.cpu().numpy().copy(),
                 r_ell.state.cpu().numpy().copy(), r_ell.active_total, r_ell.edges_total)
    s._ell = (s._c16[0], None)  # the cached rows dropped: swarm_elect_compact
    r_csr = s.elect(mode=mode)
    s._ell = None
    return ell_stats, r_csr


@pytest.mark.parametrize("n,seed,radius", [(120000, 71, 1.0), (1_200_000, 72, 1.0), (300000, 73, 1.7),
                                           (3000, 74, 1.0)])
def test_elect_ell_vs_csr_vs_oracle(sw, oracle_mod, n, seed, radius):
    # 120k / 3k agents: 512-stamp chunks; 1.2M / 300k: 2 048-stamp chunks; radius 1.7: many rows of
    # more than 32 neighbours
    from swarm_amd import gen
    d = gen.swarm_inputs(n, seed)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(radius)
    assert s.graph_ell() is not None
    if radius > 1.5:
        assert (s.row_ptr.diff() > 32).sum().item() > 100
    lead, state, rounds, changes = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    (r_rounds, r_changes, r_lead, r_state, r_act, r_edges), csr = _elect_both(s)
    assert r_rounds == rounds and csr.rounds_exec == rounds
    np.testing.assert_array_equal(r_changes, changes)
    np.testing.assert_array_equal(r_lead, lead)
    np.testing.assert_array_equal(r_state, state)
    # the per-round marked agents and edges the counters add up are the CSR path's
    assert (r_act, r_edges) == (csr.active_total, csr.edges_total)


def test_elect_ell_null_is_compact(sw, oracle_mod):
    from swarm_amd import _lib, gen
    d = gen.swarm_inputs(30000, 81)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    c16 = s.graph_compact()
    lead = torch.empty(s.n, dtype=torch.int32, device="cuda")
    state = torch.empty(s.n, dtype=torch.uint8, device="cuda")
    rounds = ctypes.c_int32(0)
    o_lead, o_state, o_rounds, _ = oracle_mod.elect(s.row_ptr.cpu().numpy(), s.col.cpu().numpy(),
                                                    s.ids.cpu().numpy())
    for ell in (None, s.graph_ell()):
        _lib.check(_lib.lib().swarm_elect_ell(_lib.ctx(), s.n, _lib.ptr(s.row_ptr), _lib.ptr(s.col), _lib.ptr(c16),
                                              _lib.ptr(ell) if ell is not None else None, _lib.ptr(s.ids),
                                              _lib.ptr(lead), _lib.ptr(state), 1 << 16, _lib.ELECT_FRONTIER,
                                              ctypes.byref(rounds), None, None, _lib.stream()))
        torch.cuda.synchronize()
        assert rounds.value == o_rounds
        np.testing.assert_array_equal(lead.cpu().numpy(), o_lead)
        np.testing.assert_array_equal(state.cpu().numpy(), o_state)


def test_reserved_delta_refused(sw):
    from swarm_amd import _lib
    rp = torch.tensor([0, 1, 2], dtype=torch.int32, device="cuda")
    ell = torch.empty(64, dtype=torch.int16, device="cuda")
    for bad in (PAD, LONG):
        c16 = torch.tensor([1, bad], dtype=torch.int16, device="cuda")
        rc = _lib.lib().swarm_graph_ell(_lib.ctx(), 2, _lib.ptr(rp), _lib.ptr(c16), _lib.ptr(ell), _lib.stream())
        assert rc == _lib.ERR_RANGE
    c16 = torch.tensor([1, -1], dtype=torch.int16, device="cuda")
    _lib.check(_lib.lib().swarm_graph_ell(_lib.ctx(), 2, _lib.ptr(rp), _lib.ptr(c16), _lib.ptr(ell), _lib.stream()))
    got = ell.cpu().numpy().reshape(2, 32)
    assert got[0, 0] == 1 and got[1, 0] == -1 and (got[:, 1:] == PAD).all()


def test_ell_rebuilt_after_graph_change(sw):
    from swarm_amd import gen
    d = gen.swarm_inputs(50000, 12)
    s = sw.Swarm(d["ids"], d["x"], d["y"], device="cuda").build_graph(1.0)
    r1 = s.elect()
    e1 = s.graph_ell()
    assert s.graph_ell() is e1
    s.col.copy_(torch.repeat_interleave(torch.arange(s.n, dtype=torch.int32, device="cuda"),
                                        s.row_ptr.diff().long()))
    r2 = s.elect()
    assert s.graph_ell() is not e1
    assert r1.rounds_exec > 1 and r2.rounds_exec == 1
    np.testing.assert_array_equal(r2.leader.cpu().numpy(), s.ids.cpu().numpy())
