"""Guard-band resolution of claims (VERDICT r2 'Resolve flagged claims').

The reference squares with libm pow (agent.py:340: CPython float ** 2); the device squares with
x*x.  For the pairs guard_cases constructs -- an agent at the claim threshold (agent.py:297) or at
an f32 rounding midpoint of its claim value (agent.py:302) where this host's pow and x*x round
apart -- the x*x arithmetic gives a different claim, claim value, winner or won count.  libswarm
defers every task with a guard-band pair, decides those pairs with the host's libm pow and
resolves the task once more; the results must equal the oracle's pow arithmetic bit for bit.
"""
import math

import numpy as np
import pytest

import guard_cases


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


@pytest.fixture(scope="module")
def case():
    return guard_cases.swarm_case(seed=0)


def test_case_is_meaningful_on_this_host(case, oracle_mod):
    """CPU: the constructed pairs do flip between the two arithmetics, the oracle's pow arithmetic
    is CPython's `**` (the reference's own expression, agent.py:340, evaluated here), and the
    pow- and x*x-oracles disagree on winners, claim values and claim counts."""
    d = case
    k = d["n_flips"]
    assert k >= 8 and {"decision", "f32"} <= set(d["kinds"])
    # the flipped agents are listed first (with companions interleaved): pick them by slot
    rows = guard_cases.find_flips(0)
    ax, ay, tx, ty = (np.array([r[i] for r in rows]) for i in range(4))
    ref = np.array([(100.0 / (1.0 + math.sqrt((a - c) ** 2 + (b - e) ** 2))) * 1.0
                    for a, b, c, e in zip(ax, ay, tx, ty)])
    u_pow = oracle_mod.utility(ax, ay, np.full(k, 15, np.uint32), tx, ty, np.full(k, -1, np.int8), use_pow=True)
    u_mul = oracle_mod.utility(ax, ay, np.full(k, 15, np.uint32), tx, ty, np.full(k, -1, np.int8), use_pow=False)
    np.testing.assert_array_equal(u_pow.view(np.uint64), ref.view(np.uint64))
    flips = ((u_pow > 20.0) != (u_mul > 20.0)) | (u_pow.astype(np.float32) != u_mul.astype(np.float32))
    assert flips.all()
    args = (d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"])
    a = oracle_mod.allocate(*args, use_pow=True)
    b = oracle_mod.allocate(*args, use_pow=False)
    assert (a["winner"] != b["winner"]).any() and (a["util"] != b["util"]).any()
    assert (a["nclaim"] != b["nclaim"]).any()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["spatial", "input"])
@pytest.mark.parametrize("mode", ["auto", "binned", "dense"])
@pytest.mark.parametrize("h", [5.0, 0.0])
def test_flagged_claims_resolved_with_libm(case, oracle_mod, sw, layout, mode, h):
    d = case
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], layout=layout, device="cuda")
    r = s.allocate(d["tx"], d["ty"], d["treq"], mode=mode, hysteresis=h)
    want = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"], hysteresis=h,
                               use_pow=True)
    assert r.stats["n_flagged"] > 0 and r.stats["n_resolved"] > 0, r.stats
    np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy().view(np.uint64), want["util"].view(np.uint64))
    np.testing.assert_array_equal(r.nclaim.cpu().numpy(), want["nclaim"])
    np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
    np.testing.assert_array_equal(s.to_input_order(r.won), want["won"])
    assert r.stats["n_claims"] == want["n_claims"] and r.stats["n_conflicts"] == want["n_conflicts"]


@pytest.mark.gpu
def test_flagged_claims_with_prior_claim_table(case, oracle_mod, sw):
    """A pre-loaded claim table (the resolver's task_claims, agent.py:309) on the deferred tasks."""
    d = case
    t = len(d["tx"])
    g = np.random.default_rng(3)
    w = np.where(g.random(t) < 0.4, d["ids"][g.integers(0, len(d["ids"]), t)], -1).astype(np.int32)
    u = np.where(w >= 0, g.uniform(20.5, 60.0, t), 0.0)
    s = sw.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda")
    r = s.allocate(d["tx"], d["ty"], d["treq"], winner=w, util=u)
    want = oracle_mod.allocate(d["ids"], d["x"], d["y"], d["caps"], d["tx"], d["ty"], d["treq"], winner=w, util=u,
                               use_pow=True)
    assert r.stats["n_resolved"] > 0
    np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy().view(np.uint64), want["util"].view(np.uint64))
    np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
    np.testing.assert_array_equal(s.to_input_order(r.won), want["won"])


@pytest.mark.gpu
@pytest.mark.parametrize("h", [5.0, 0.0])
def test_dense_deferred_tasks_with_crowded_claims(case, oracle_mod, sw, h):
    """Dense strategy, deferred tasks whose claims overflow the per-task LDS list (> 512 claimants):
    700 extra agents inside the claim radius of every task.  The deferred tasks are resolved by the
    chain walk over the dense tile summaries with the host's decisions patched in (the
    per-task wave pass rescanned every agent per chain link there)."""
    d = case
    g = np.random.default_rng(11)
    tx, ty = np.asarray(d["tx"]), np.asarray(d["ty"])
    m = 700
    r_ = 3.5 * np.sqrt(g.random((len(tx), m)))
    th = g.uniform(0, 2 * np.pi, (len(tx), m))
    ex = (tx[:, None] + r_ * np.cos(th)).ravel()
    ey = (ty[:, None] + r_ * np.sin(th)).ravel()
    ids = np.concatenate([d["ids"], int(np.max(d["ids"])) + 1 + g.permutation(ex.size)]).astype(np.int32)
    x = np.concatenate([d["x"], ex])
    y = np.concatenate([d["y"], ey])
    caps = np.concatenate([d["caps"], np.full(ex.size, 15, np.uint32)]).astype(np.uint32)
    s = sw.Swarm(ids, x, y, caps, device="cuda")
    r = s.allocate(tx, ty, d["treq"], mode="dense", hysteresis=h)
    want = oracle_mod.allocate(ids, x, y, caps, tx, ty, d["treq"], hysteresis=h, use_pow=True)
    assert r.stats["mode_used"] == 2 and r.stats["n_resolved"] > 0, r.stats
    assert want["nclaim"].max() > 512
    np.testing.assert_array_equal(r.winner.cpu().numpy(), want["winner"])
    np.testing.assert_array_equal(r.util.cpu().numpy().view(np.uint64), want["util"].view(np.uint64))
    np.testing.assert_array_equal(r.nclaim.cpu().numpy(), want["nclaim"])
    np.testing.assert_array_equal(r.nmsg.cpu().numpy(), want["nmsg"])
    np.testing.assert_array_equal(s.to_input_order(r.won), want["won"])
