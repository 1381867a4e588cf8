"""swarm_allocate_indexed (the binned allocation over the spatial storage order's cell index, no
binning pass) against swarm_allocate's hashed binning and the oracle; staleness detection when
positions move after the index was built (agent.py:292-325, contract A-H)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib, gen
    _lib.load()
    return swm, _lib, gen


def _both(s, d, **kw):
    """Swarm.allocate through the index (default for the spatial layout) and through hashed
    binning (the same swarm with the index path disabled)."""
    a = s.allocate(d["tx"], d["ty"], d["treq"], **kw)
    assert s._cindex is not None  # the indexed path ran
    saved = s._indexable
    s._indexable = lambda *a_, **k_: False
    try:
        b = s.allocate(d["tx"], d["ty"], d["treq"], **kw)
    finally:
        s._indexable = saved
    return a, b


@pytest.mark.parametrize("n,t,seed,h", [(300_000, 3_000, 1, 5.0), (60_000, 20_000, 2, 0.0), (5_000, 800, 3, 5.0)])
def test_indexed_equals_hashed_and_oracle(mods, oracle_mod, n, t, seed, h):
    swm, _lib, gen = mods
    d = gen.swarm_inputs(n, seed, t=t)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    a, b = _both(s, d, hysteresis=h)
    for k in ("winner", "nclaim", "nmsg", "won"):
        np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy(), err_msg=k)
    np.testing.assert_array_equal(a.util.cpu().numpy().view(np.uint64), b.util.cpu().numpy().view(np.uint64))
    for k in ("n_claims", "n_conflicts", "n_flagged", "n_candidates", "n_overflow"):
        assert a.stats[k] == b.stats[k], k
    ids, x, y = s.ids.cpu().numpy(), s.pos[:, 0].cpu().numpy(), s.pos[:, 1].cpu().numpy()
    want = oracle_mod.allocate_binned(ids, x, y, s.caps.cpu().numpy().view(np.uint32), d["tx"], d["ty"], d["treq"],
                                      hysteresis=h, use_pow=False)
    np.testing.assert_array_equal(a.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(a.won.cpu().numpy(), want["won"])


def test_prior_claims_and_tasks_outside(mods, oracle_mod):
    """Pre-loaded claim table and tasks far outside the agents' bounding box (empty windows)."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(20_000, 7, t=500)
    d["tx"][:50] += 1e4  # no agent within reach
    g = np.random.default_rng(7)
    w = np.where(g.random(500) < 0.3, g.integers(0, 20_000, 500), -1).astype(np.int32)
    u = np.where(w >= 0, g.uniform(20, 100, 500), 0.0)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    a, b = _both(s, d, winner=w, util=u)
    np.testing.assert_array_equal(a.winner.cpu().numpy(), b.winner.cpu().numpy())
    np.testing.assert_array_equal(a.util.cpu().numpy(), b.util.cpu().numpy())
    np.testing.assert_array_equal(a.won.cpu().numpy(), b.won.cpu().numpy())
    assert (a.nclaim.cpu().numpy()[:50] == 0).all()


def test_stale_index_detected_and_recovered(mods, oracle_mod):
    swm, _lib, gen = mods
    d = gen.swarm_inputs(50_000, 9, t=2_000)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    s.allocate(d["tx"], d["ty"], d["treq"])
    g, off = s._cindex
    # move agents behind the Swarm's back: the next call must notice and rebin
    s.pos[:, 0] = s.pos[:, 0].flip(0)
    L = _lib.lib()
    t = len(d["tx"])
    tpos = torch.stack([torch.as_tensor(d["tx"]), torch.as_tensor(d["ty"])], 1).cuda().contiguous()
    tq = torch.as_tensor(d["treq"]).cuda()
    w = torch.full((t,), -1, dtype=torch.int32, device="cuda")
    u = torch.zeros(t, dtype=torch.float64, device="cuda")
    rc = L.swarm_allocate_indexed(_lib.ctx(), s.n, _lib.ptr(s.ids), _lib.ptr(s.pos), _lib.ptr(s.caps),
                                  ctypes.byref(g), _lib.ptr(off), t, _lib.ptr(tpos), _lib.ptr(tq), 20.0, 5.0, 100.0,
                                  _lib.ptr(w), _lib.ptr(u), None, None, 0, None, None, None, _lib.stream())
    assert rc == _lib.ERR_STALE
    a = s.allocate(d["tx"], d["ty"], d["treq"])  # falls back to hashed binning
    ids, x, y = s.ids.cpu().numpy(), s.pos[:, 0].cpu().numpy(), s.pos[:, 1].cpu().numpy()
    want = oracle_mod.allocate_binned(ids, x, y, s.caps.cpu().numpy().view(np.uint32), d["tx"], d["ty"], d["treq"],
                                      use_pow=False)
    np.testing.assert_array_equal(a.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(a.won.cpu().numpy(), want["won"])


def test_cell_index_rejects_unsorted(mods):
    swm, _lib, gen = mods
    d = gen.swarm_inputs(10_000, 4)
    pos = torch.stack([torch.as_tensor(d["x"]), torch.as_tensor(d["y"])], 1).cuda().contiguous()  # input order
    g, nc = _lib.Grid(), ctypes.c_int64(0)
    L = _lib.lib()
    _lib.check(L.swarm_cell_index(_lib.ctx(), 10_000, _lib.ptr(pos), 1.0, ctypes.byref(g), None, 0, ctypes.byref(nc),
                                  _lib.stream()))
    off = torch.empty(nc.value + 1, dtype=torch.int32, device="cuda")
    with pytest.raises(_lib.SwarmError, match="not in cell order"):
        _lib.check(L.swarm_cell_index(_lib.ctx(), 10_000, _lib.ptr(pos), 1.0, ctypes.byref(g), _lib.ptr(off),
                                      off.numel(), ctypes.byref(nc), _lib.stream()))


def _oracle_now(oracle_mod, s, tx, ty, tq, **kw):
    """The oracle over the Swarm's CURRENT storage-order state (x*x arithmetic, as the GPU)."""
    ids, x, y = s.ids.cpu().numpy(), s.pos[:, 0].cpu().numpy(), s.pos[:, 1].cpu().numpy()
    return oracle_mod.allocate_binned(ids, x, y, s.caps.cpu().numpy().view(np.uint32), tx, ty, tq, use_pow=False,
                                      **kw)


def test_physics_then_allocate(mods, oracle_mod):
    """physics_step moves agents across cells, so the storage order is no longer cell order: the
    next allocate() must bin by hashed cells (not fail building the index), and so must the one
    after it (both used to raise SwarmError)."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(30_000, 21, t=1_500)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
    s.allocate(d["tx"], d["ty"], d["treq"])
    assert s._cindex not in (None, False)
    s.elect()
    obs = np.array([[30.0, 30.0, 2.0], [60.0, 20.0, 1.0]])
    s.physics_step(obs, steps=6)
    moved = int((s.to_input_order(s.pos) != np.stack([d["x"], d["y"]], 1)).any(1).sum())
    assert moved > 1000
    for _ in range(2):
        a = s.allocate(d["tx"], d["ty"], d["treq"])
        want = _oracle_now(oracle_mod, s, d["tx"], d["ty"], d["treq"])
        for k in ("winner", "nclaim", "nmsg", "won"):
            np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), want[k], err_msg=k)
        np.testing.assert_array_equal(a.util.cpu().numpy(), want["util"])
    assert s._cindex is False  # not indexable until the positions change again


def test_edge_agent_moved_past_bbox(mods, oracle_mod):
    """An edge-cell agent moved just past the indexed bounding box maps (clamped) to its old cell;
    the index must report itself stale instead of dropping that agent's claims."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(20_000, 23, t=200)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    xmax = float(d["x"].max())
    tx = np.concatenate([d["tx"], [xmax + 5.0]])
    ty = np.concatenate([d["ty"], [float(d["y"][np.argmax(d["x"])])]])
    tq = np.concatenate([d["treq"], [-1]]).astype(np.int8)
    s.allocate(tx, ty, tq)
    assert s._cindex not in (None, False)
    i = int(torch.argmax(s.pos[:, 0]))
    s.pos[i, 0] = xmax + 3.0  # in place, behind the Swarm's back: 2.0 from the last task
    a = s.allocate(tx, ty, tq)
    want = _oracle_now(oracle_mod, s, tx, ty, tq)
    assert want["nclaim"][-1] >= 1
    for k in ("winner", "nclaim", "won"):
        np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), want[k], err_msg=k)


def test_task_positions_cache_follows_in_place_writes(mods, oracle_mod):
    """Swarm.allocate reuses its stacked task positions only for the same, unmodified tensors."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(20_000, 29, t=400)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    tx, ty = torch.as_tensor(d["tx"], device="cuda"), torch.as_tensor(d["ty"], device="cuda")
    tq = torch.as_tensor(d["treq"], device="cuda")
    a = s.allocate(tx, ty, tq)
    tx[:200] += 3.0  # in place: the version counter moves, the cache must not serve the old copy
    b = s.allocate(tx, ty, tq)
    want = _oracle_now(oracle_mod, s, tx.cpu().numpy(), d["ty"], d["treq"])
    np.testing.assert_array_equal(b.winner.cpu().numpy(), want["winner"])
    assert not np.array_equal(a.winner.cpu().numpy(), b.winner.cpu().numpy())


def test_trusted_index_and_fresh_claims_flags(mods, oracle_mod):
    """swarm_allocate_indexed_ex: SWARM_ALLOC_TRUST_INDEX (no device staleness check) and
    SWARM_ALLOC_FRESH_CLAIMS (winner / util initialised on the device, whatever the buffers held)
    give the results of the plain indexed call, and of the oracle; Swarm.allocate trusts its index
    only while self.pos is the tensor and version it was built from."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(60_000, 31, t=3_000)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    a0 = s.allocate(d["tx"], d["ty"], d["treq"])  # builds the index
    assert s._indexed_pos() and s._cindex_key[0] is s.pos
    g, off = s._cindex
    L = _lib.lib()
    t = len(d["tx"])
    tpos = torch.stack([torch.as_tensor(d["tx"]), torch.as_tensor(d["ty"])], 1).cuda().contiguous()
    tq = torch.as_tensor(d["treq"]).cuda()
    outs = {}
    for flags in (0, _lib.ALLOC_TRUST_INDEX, _lib.ALLOC_FRESH_CLAIMS, _lib.ALLOC_TRUST_INDEX | _lib.ALLOC_FRESH_CLAIMS):
        if flags & _lib.ALLOC_FRESH_CLAIMS:  # garbage the device must overwrite
            w = torch.randint(-5, 1000, (t,), dtype=torch.int32, device="cuda")
            u = torch.rand(t, dtype=torch.float64, device="cuda") * 1e3
        else:
            w = torch.full((t,), -1, dtype=torch.int32, device="cuda")
            u = torch.zeros(t, dtype=torch.float64, device="cuda")
        won = torch.empty(s.n, dtype=torch.int32, device="cuda")
        nc = torch.empty((2, t), dtype=torch.int64, device="cuda")
        st = _lib.AllocStats()
        _lib.check(L.swarm_allocate_indexed_ex(
            _lib.ctx(), s.n, _lib.ptr(s.ids), _lib.ptr(s.pos), _lib.ptr(s.caps), ctypes.byref(g), _lib.ptr(off), t,
            _lib.ptr(tpos), _lib.ptr(tq), 20.0, 5.0, 100.0, flags, _lib.ptr(w), _lib.ptr(u), _lib.ptr(won), None, 0,
            _lib.ptr(nc[0]), _lib.ptr(nc[1]), ctypes.byref(st), _lib.stream()))
        outs[flags] = (w.cpu().numpy(), u.cpu().numpy(), won.cpu().numpy(), nc.cpu().numpy(), st.n_claims)
    for flags, o in outs.items():
        for a, b in zip(o[:4], outs[0][:4]):
            np.testing.assert_array_equal(a, b, err_msg=str(flags))
        assert o[4] == outs[0][4]
    want = _oracle_now(oracle_mod, s, d["tx"], d["ty"], d["treq"])
    np.testing.assert_array_equal(outs[0][0], want["winner"])
    np.testing.assert_array_equal(a0.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(a0.util.cpu().numpy(), want["util"])
    # an in-place write moves the version: the next call checks on the device and rebins
    i = int(torch.argmax(s.pos[:, 1]))
    s.pos[i, 1] += 50.0
    assert not s._indexed_pos()
    b = s.allocate(d["tx"], d["ty"], d["treq"])
    want = _oracle_now(oracle_mod, s, d["tx"], d["ty"], d["treq"])
    np.testing.assert_array_equal(b.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(b.won.cpu().numpy(), want["won"])


def test_reassigned_positions_are_not_trusted(mods, oracle_mod):
    """a NEW position tensor of the same shape (possibly at a recycled address, version 0) must
    not inherit the trust of the index built for the old one: the allocation checks on the device and
    gives the oracle's result for the new positions."""
    swm, _lib, gen = mods
    d = gen.swarm_inputs(40_000, 37, t=2_000)
    s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    s.allocate(d["tx"], d["ty"], d["treq"])  # builds and trusts the index
    assert s._indexed_pos()
    new = s.pos.clone()
    i = int(torch.argmax(new[:, 1]))
    new[i, 1] += 60.0  # one agent leaves its cell: the old index is wrong for these positions
    del_ptr = s.pos.data_ptr()
    s.pos = new
    assert not s._indexed_pos()
    b = s.allocate(d["tx"], d["ty"], d["treq"])
    want = _oracle_now(oracle_mod, s, d["tx"], d["ty"], d["treq"])
    np.testing.assert_array_equal(b.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(b.won.cpu().numpy(), want["won"])
    # the same holds when the new tensor reuses the old storage address
    s.pos = s.pos.clone()
    assert not s._indexed_pos() and del_ptr is not None
