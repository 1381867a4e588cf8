"""Timer FSM / protocol ticks: _check_election_timeout (agent.py:217-241),
_send_heartbeat (283-289) and the election handlers (243-281) ticking under contract T1.

Parity is pinned by the reference itself: tests/golden/fsm_*.npz were produced by ticking real
SwarmAgent objects (their clock and jitter draw patched to the contract's, packets framed by
_pack_header and delivered through on_message_received; tools/gen_golden.py ref_fsm), with
phase-shifted agents and leader kills (fsm_n200, fsm_wide_n800) and in lock-step
(fsm_lockstep_n150, where the optimistic COORDINATOR takeover makes simultaneous winners
depose each other).  The C oracle must reproduce them exactly, and the GPU
(swarm_protocol_run) must match both bit for bit.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden

FSM = golden_names("fsm_")
OUT = ("state", "leader", "last_hb", "wait_start", "delay", "has_lpos", "lpos", "alive")
F, W, L = 1, 2, 3


def _run_oracle(oracle_mod, g, **kw):
    return oracle_mod.protocol(g["ids"], g["x"], g["y"], g["row_ptr"], g["col"], g["tick_off"], int(g["ticks"]),
                               last_hb=g["last_hb0"], dt=float(g["dt"]), seed=int(g["seed"]),
                               kill_ticks=g["kill_ticks"], **kw)


@pytest.mark.parametrize("name", FSM)
def test_oracle_matches_reference_fixture(oracle_mod, name):
    g = load_golden(name)
    o = _run_oracle(oracle_mod, g)
    for k in OUT:
        np.testing.assert_array_equal(o[k], g[k + "_out"], err_msg=k)
    np.testing.assert_array_equal(o["counts"], g["counts"])


def test_fixtures_exercise_the_fsm():
    g = load_golden("fsm_n200")
    c = g["counts"]
    assert c[:, 0].max() > 0 and c[:, 1].sum() > 0 and c[:, 2].sum() > 0 and c[:, 3].sum() > 0
    assert g["alive_out"].sum() < len(g["ids"])           # the kills removed leaders
    k = int(g["kill_ticks"][0])
    assert c[k - 1, 0] < c[k - 2, 0]                       # ... and leadership dropped at the kill
    assert c[k - 1 + 28:, 0].max() > 0                     # ... and re-election follows the timeout
    lock = load_golden("fsm_lockstep_n150")["counts"]
    assert lock[:, 2].sum() > 0 and lock[-20:, 0].max() == 0  # winners depose each other


def test_oracle_chunked_equals_one_run(oracle_mod):
    g = load_golden("fsm_wide_n800")
    full = _run_oracle(oracle_mod, g)
    a = oracle_mod.protocol(g["ids"], g["x"], g["y"], g["row_ptr"], g["col"], g["tick_off"], 77,
                            last_hb=g["last_hb0"], dt=float(g["dt"]), seed=int(g["seed"]), kill_ticks=g["kill_ticks"])
    b = oracle_mod.protocol(g["ids"], g["x"], g["y"], g["row_ptr"], g["col"], g["tick_off"], int(g["ticks"]) - 77,
                            t0=77, dt=float(g["dt"]), seed=int(g["seed"]), kill_ticks=g["kill_ticks"],
                            **{k: a[k] for k in OUT + ("outbox",) if k in a})
    for k in OUT:
        np.testing.assert_array_equal(b[k], full[k], err_msg=k)
    np.testing.assert_array_equal(np.concatenate([a["counts"], b["counts"]]), full["counts"])


def test_oracle_reference_unit_scenarios(oracle_mod):
    """test_election.py's FSM cases (22-71) restated as ticks of one / two agents."""
    empty = np.zeros(2, np.int64), np.zeros(0, np.int32)
    # timeout trigger (22-30): 5 s of silence > 3 s -> ELECTION_WAIT, wait started
    o = oracle_mod.protocol([1], [0.0], [0.0], *empty, [1], 1, last_hb=[-4.9], dt=0.1)
    assert o["state"][0] == W and o["wait_start"][0] == 0.1 and 0.0 <= o["delay"][0] < 0.2
    # victory after the wait (32-45): LEADER, leader_id = self, ACCLAIM (+ COORDINATOR) sent
    o = oracle_mod.protocol([1], [0.0], [0.0], *empty, [1], 1, state=[W], wait_start=[-1.0], delay=[0.1], dt=0.1)
    assert o["state"][0] == L and o["leader"][0] == 1 and o["counts"][0, 2] == 1
    # submission to a higher acclaim (47-56) and bullying a lower one (58-71): agents 1 and 2,
    # both LEADER; 2 has just sent ACCLAIM, 1 hears it and backs down ...
    rp, col = np.array([0, 1, 2]), np.array([1, 0], np.int32)
    ob = np.zeros(4, np.uint8)
    ob[1] = 1  # tick-0 outbox (parity 0): agent index 1 (ID 2) acclaimed
    o = oracle_mod.protocol([1, 2], [0.0, 1.0], [0.0, 0.0], rp, col, [0, 0], 1, state=[L, L], leader=[1, 2],
                            outbox=ob, dt=0.1)
    assert o["state"][0] == F and o["leader"][0] == 2
    # ... while 2, hearing 1's acclaim on a heartbeat tick (own tick % 10 == 0), bullies back
    ob = np.zeros(4, np.uint8)
    ob[0] = 1
    o = oracle_mod.protocol([1, 2], [0.0, 1.0], [0.0, 0.0], rp, col, [0, 9], 1, state=[L, L], leader=[1, 2],
                            outbox=ob, dt=0.1)
    assert o["outbox"][2 + 1] & 2  # heartbeat sent by ID 2 (the COORDINATOR then takes it over)


# ----------------------------------------------------------------------------- GPU

def _gpu_swarm(g, layout="spatial"):
    from swarm_amd.swarm import Swarm
    s = Swarm(g["ids"], g["x"], g["y"], layout=layout, device="cuda")
    s.set_graph(g["row_ptr"], g["col"])
    s.protocol_reset(tick_off=g["tick_off"], last_hb=g["last_hb0"])
    return s


def _gpu_state(s):
    f = s.fsm
    out = dict(state=s.state, leader=s.leader, last_hb=f["last_hb"], wait_start=f["wait_start"], delay=f["delay"],
               has_lpos=f["has_leader_pos"], lpos=f["leader_pos"], alive=f["alive"])
    return {k: s.to_input_order(v) for k, v in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("name", FSM)
@pytest.mark.parametrize("layout,mode", [("spatial", "push"), ("input", "push"), ("spatial", "pull"),
                                         ("spatial", "hybrid")])
def test_gpu_matches_reference_fixture(name, layout, mode):
    g = load_golden(name)
    s = _gpu_swarm(g, layout)
    counts = s.protocol_run(int(g["ticks"]), kill_ticks=g["kill_ticks"], dt=float(g["dt"]), seed=int(g["seed"]),
                            mode=mode)
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], g[k + "_out"], err_msg=k)
    np.testing.assert_array_equal(counts, g["counts"])


def _random_case(n, seed, side):
    from swarm_amd import gen
    rng = np.random.default_rng(seed)
    x, y = rng.uniform(0, side, n), rng.uniform(0, side, n)
    ids = rng.permutation(n).astype(np.int32)
    rp, col = gen.rgg_csr(x, y, 1.0)
    off = rng.integers(0, 40, n).astype(np.int32)
    return dict(ids=ids, x=x, y=y, row_ptr=np.asarray(rp, np.int64), col=np.asarray(col, np.int32), tick_off=off,
                last_hb0=-(off * 0.1), dt=np.float64(0.1), seed=np.uint64(seed))


def _directed(g, seed):
    """Drop a third of the edges one way: agent i may hear j while j does not hear i."""
    rng = np.random.default_rng(seed)
    rp, col = g["row_ptr"], g["col"]
    keep = rng.uniform(size=col.size) > 0.33
    deg = np.add.reduceat(keep, rp[:-1]) if col.size else np.zeros(len(rp) - 1, np.int64)
    deg[np.diff(rp) == 0] = 0
    g = dict(g)
    g["row_ptr"] = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    g["col"] = col[keep]
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,side,mode,directed", [(20000, 1, 50.0, "push", False),
                                                       (20000, 3, 50.0, "push", True),
                                                       (20000, 4, 50.0, "pull", True),
                                                       (300000, 2, 180.0, "push", False)])
def test_gpu_matches_oracle_random(oracle_mod, n, seed, side, mode, directed):
    g = _random_case(n, seed, side)
    if directed:
        g = _directed(g, seed)
    g["ticks"], g["kill_ticks"] = np.int64(150), np.array([60, 61, 110], np.int64)
    want = _run_oracle(oracle_mod, g)
    s = _gpu_swarm(g)
    assert (s._hear is not None) == directed
    c1 = s.protocol_run(64, kill_ticks=g["kill_ticks"], seed=seed, mode=mode)  # in two chunks: the state
    c2 = s.protocol_run(86, kill_ticks=g["kill_ticks"], seed=seed, mode=mode)  # and in-flight sends carry over
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_array_equal(np.concatenate([c1, c2]), want["counts"])
    assert want["counts"][:, 0].max() > 0 and want["alive"].sum() < n


@pytest.mark.gpu
@pytest.mark.parametrize("dt,t0", [(0.1, 0), (0.07, 1234), (-0.05, 3)])
def test_gpu_timer_encodings_match_oracle(oracle_mod, dt, t0):
    """A run keeps a FOLLOWER's last_heartbeat_time as a tick of the run and an ELECTION_WAIT's end as the
    first tick its test holds (protocol.hip, the per-agent record); values no tick represents, and waits
    when dt <= 0, stay in the f64 arrays.  Mixed initial states -- FOLLOWERs with tick-exact and arbitrary
    last_hb, ELECTION_WAITs with arbitrary wait_start / delay, LEADERs, dead agents, leader positions --
    at other dt and a nonzero start tick, in two chunks: every state, timer, leader position and count
    equals the oracle's (agent.py:217-241)."""
    import torch
    from swarm_amd.swarm import Swarm
    n = 20000
    g = _random_case(n, 11, 50.0)
    rng = np.random.default_rng(7)
    st = rng.choice([F, W, L], n, p=[0.6, 0.3, 0.1]).astype(np.uint8)
    lhb = np.where(rng.uniform(size=n) < 0.5, (t0 - rng.integers(0, 40, n)).astype(np.float64) * dt,
                   t0 * dt - rng.uniform(0, 4, n))
    ws, dl = t0 * dt - rng.uniform(0, 0.3, n), rng.uniform(0, 0.2, n)
    leader = np.where(st == L, g["ids"], rng.choice(g["ids"], n)).astype(np.int32)
    alive = (rng.uniform(size=n) > 0.02).astype(np.uint8)
    lpos = rng.uniform(-5, 5, (n, 2)).astype(np.float32)
    has = (rng.uniform(size=n) < 0.5).astype(np.uint8)
    kills = np.array([t0 + 50, t0 + 100], np.int64)
    want = oracle_mod.protocol(g["ids"], g["x"], g["y"], g["row_ptr"], g["col"], g["tick_off"], 130, state=st,
                               leader=leader, last_hb=lhb, wait_start=ws, delay=dl, lpos=lpos, has_lpos=has,
                               alive=alive, t0=t0, dt=dt, seed=11, kill_ticks=kills)
    s = Swarm(g["ids"], g["x"], g["y"], device="cuda")
    s.set_graph(g["row_ptr"], g["col"])
    s.protocol_reset(tick_off=g["tick_off"], last_hb=lhb)
    s.state.copy_(s._storage(st, torch.uint8))
    s.leader.copy_(s._storage(leader, torch.int32))
    s.fsm["wait_start"], s.fsm["delay"] = s._storage(ws, torch.float64), s._storage(dl, torch.float64)
    s.fsm["alive"], s.fsm["has_leader_pos"] = s._storage(alive, torch.uint8), s._storage(has, torch.uint8)
    s.fsm["leader_pos"] = torch.as_tensor(lpos, device="cuda")[s.perm.long()].contiguous()
    s.fsm_tick = t0
    c1 = s.protocol_run(60, kill_ticks=kills, dt=dt, seed=11)
    c2 = s.protocol_run(70, kill_ticks=kills, dt=dt, seed=11)
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_array_equal(np.concatenate([c1, c2]), want["counts"])
    if dt > 0:
        assert want["counts"][:, 1].sum() > 0 and want["counts"][:, 0].max() > 0


@pytest.mark.gpu
def test_gpu_empty_and_isolated():
    from swarm_amd.swarm import Swarm
    s = Swarm(np.zeros(0, np.int32), [], [], device="cuda")
    s.set_graph(np.zeros(1, np.int64), np.zeros(0, np.int32))
    assert s.protocol_run(5).shape == (5, 4)
    s = Swarm(np.arange(3, dtype=np.int32), [0.0, 10.0, 20.0], [0.0, 0.0, 0.0], device="cuda")
    s.set_graph(np.zeros(4, np.int64), np.zeros(0, np.int32))  # nobody hears anybody
    c = s.protocol_run(40)
    assert c[30, 1] == 3 and c[-1, 0] == 3  # all time out at t=31 (3.1 s > 3.0 s), then all lead


@pytest.mark.gpu
def test_gpu_large_ids_match_oracle(oracle_mod):
    """IDs at the top of the int32 range (jitter hash, ID comparisons, leader IDs)."""
    g = _random_case(20000, 9, 50.0)
    g["ids"] = (np.int64(2**31 - 1) - np.random.default_rng(2).permutation(20000) * 3).astype(np.int32)
    g["ticks"], g["kill_ticks"] = np.int64(120), np.array([70], np.int64)
    want = _run_oracle(oracle_mod, g)
    s = _gpu_swarm(g)
    c = s.protocol_run(120, kill_ticks=g["kill_ticks"], seed=int(g["seed"]))
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_array_equal(c, want["counts"])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [20001, 20000])
def test_gpu_sweep_unaligned_arrays_match_oracle(oracle_mod, n):
    """k_sweep reads 4 agents per thread with word loads when every per-agent array is aligned;
    arrays one byte / one element off force its scalar path (and odd n the word path's tail):
    both must give the oracle's states, timers and counts."""
    import torch
    g = _random_case(n, 9, 50.0)
    g["ticks"], g["kill_ticks"] = np.int64(120), np.array([50, 90], np.int64)
    want = _run_oracle(oracle_mod, g)
    s = _gpu_swarm(g)

    def shifted(t):  # same values, storage one element past an aligned allocation
        buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=t.device)
        v = buf[1:].view(t.shape)
        v.copy_(t)
        return v

    for k in ("alive", "outbox", "last_hb"):
        s.fsm[k] = shifted(s.fsm[k])
    s.tick_off = shifted(s.tick_off)
    counts = s.protocol_run(120, kill_ticks=g["kill_ticks"], seed=9)
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_array_equal(counts, want["counts"])


@pytest.mark.gpu
@pytest.mark.parametrize("pull_frac", [0.0, 0.02, 0.125])
def test_gpu_hybrid_storm_ticks_match_oracle(oracle_mod, pull_frac):
    """Hybrid mode (swarm_protocol_run_ex): a tick in which a workgroup's senders exceed pull_frac x
    its share of the agents has the next tick pull (every alive agent walks its row); pull_frac 0
    pulls after every tick with a sender, and nothing is mailed.  States, timers, leader positions and per-tick counts equal the oracle's, in two chunks
    (a pulled tick at a chunk boundary), and the traffic counters add up."""
    g = _random_case(20000, 5, 50.0)
    g["ticks"], g["kill_ticks"] = np.int64(150), np.array([60, 110], np.int64)
    want = _run_oracle(oracle_mod, g)
    s = _gpu_swarm(g)
    c1 = s.protocol_run(64, kill_ticks=g["kill_ticks"], seed=5, mode="hybrid", pull_frac=pull_frac, traffic=True)
    t1 = s.fsm_traffic.copy()
    c2 = s.protocol_run(86, kill_ticks=g["kill_ticks"], seed=5, mode="hybrid", pull_frac=pull_frac, traffic=True)
    tr = t1 + s.fsm_traffic
    got = _gpu_state(s)
    for k in OUT:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    np.testing.assert_array_equal(np.concatenate([c1, c2]), want["counts"])
    if pull_frac == 0.0:  # every tick after one with a sender pulled: nothing was mailed
        assert tr[7] > 0 and tr[6] > 0 and tr[3] == 0 and tr[0] == 0
    senders = int((want["counts"][:, 2] + want["counts"][:, 3]).sum())
    assert tr[3] <= senders


@pytest.mark.gpu
@pytest.mark.parametrize("recv_wgs", ["1", "3"])
def test_gpu_few_receive_workgroups_match_oracle(recv_wgs):
    """k_tick's receive role with 1 or 3 workgroups (SWARM_FSM_RECV_WGS), each serving many
    4 096-agent units one after the other, beside the sweep role: the oracle's states, timers and
    counts.  The tuning is read once per process: a child process."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    p = subprocess.run([sys.executable, "-u", os.path.join(here, "protocol_env_case.py")],
                       env=dict(os.environ, SWARM_FSM_RECV_WGS=recv_wgs), capture_output=True, text=True,
                       timeout=300)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    res = json.loads(lines[-1])
    assert res["ok"], (res["error"], [c for c in res["cases"] if c["bad"]])
