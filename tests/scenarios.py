"""The ten shipped single-agent scenarios (test_election.py, test_allocation.py), restated as
data-producing functions so the same code can drive either the reference module (only in
tools/gen_golden.py, in the build container) or this repo's drop-in ``agent`` module.

Each scenario takes an ``agent`` *module* and returns a JSON-able dict of everything the
reference test observes: the positional ``_send_msg`` call log (type, payload hex) and the
attributes the test asserts on.
"""
from __future__ import annotations

import struct
import time


class Recorder:
    """Stand-in for the tests' ``MagicMock`` on the instance attribute ``_send_msg``
    (test_election.py:16, test_allocation.py:14): records positional (type, payload)."""

    def __init__(self):
        self.calls = []

    def __call__(self, *args, **kwargs):
        self.calls.append((args, kwargs))

    def log(self):
        out = []
        for args, kwargs in self.calls:
            mt = int(args[0]) if args else int(kwargs["msg_type"])
            pl = args[1] if len(args) > 1 else kwargs.get("payload", b"")
            out.append([mt, pl.hex(), len(args)])
        return out


def _state_name(s):
    return None if s is None else s.name


def _mk(mod, **kw):
    a = mod.SwarmAgent(**kw)
    a._send_msg = Recorder()
    return a


def s_initial_state(mod):  # test_election.py:18-20
    a = _mk(mod, agent_id=1, total_agents=3)
    return dict(state=_state_name(a.state), leader_id=a.leader_id, log=a._send_msg.log())


def s_election_timeout_trigger(mod):  # test_election.py:22-30
    a = _mk(mod, agent_id=1, total_agents=3)
    a.last_heartbeat_time = time.time() - 5.0
    a._check_election_timeout()
    return dict(state=_state_name(a.state), leader_id=a.leader_id,
                wait_start_set=a.election_wait_start is not None, log=a._send_msg.log())


def s_election_victory_after_wait(mod):  # test_election.py:32-46
    a = _mk(mod, agent_id=1, total_agents=3)
    a.state = mod.AgentState.ELECTION_WAIT
    a.election_wait_start = time.time() - 1.0
    a.election_delay = 0.1
    a._check_election_timeout()
    return dict(state=_state_name(a.state), leader_id=a.leader_id, log=a._send_msg.log())


def s_submission_to_higher_id(mod):  # test_election.py:48-57
    a = _mk(mod, agent_id=1, total_agents=3)
    a.state = mod.AgentState.LEADER
    a.agent_id = 1
    a._handle_election_acclaim(sender=2)
    return dict(state=_state_name(a.state), leader_id=a.leader_id, log=a._send_msg.log())


def s_bullying_lower_id(mod):  # test_election.py:59-71
    a = _mk(mod, agent_id=1, total_agents=3)
    a.state = mod.AgentState.LEADER
    a.agent_id = 2
    a._handle_election_acclaim(sender=1)
    return dict(state=_state_name(a.state), leader_id=a.leader_id, log=a._send_msg.log())


def s_utility_with_capability(mod):  # test_allocation.py:16-23
    a = _mk(mod, agent_id=1, total_agents=3, capabilities=["extinguisher"])
    task = {"status": "OPEN", "pos": (1.0, 0.0), "required_cap": "extinguisher"}
    a.position = [0.0, 0.0]
    return dict(util=a._calculate_utility(task).hex(), log=a._send_msg.log())


def s_utility_missing_capability(mod):  # test_allocation.py:25-32
    a = _mk(mod, agent_id=1, total_agents=3, capabilities=["extinguisher"])
    task = {"status": "OPEN", "pos": (1.0, 0.0), "required_cap": "sonar"}
    a.position = [0.0, 0.0]
    return dict(util=a._calculate_utility(task).hex(), log=a._send_msg.log())


def s_greedy_claim(mod):  # test_allocation.py:34-50
    a = _mk(mod, agent_id=1, total_agents=3, capabilities=["extinguisher"])
    a.tasks = {101: {"status": "OPEN", "pos": (1.0, 0.0), "required_cap": "extinguisher"}}
    a.position = [0.0, 0.0]
    a._process_tasks()
    return dict(status=a.tasks[101]["status"], log=a._send_msg.log())


def s_leader_conflict_resolution_win(mod):  # test_allocation.py:52-68
    a = _mk(mod, agent_id=1, total_agents=3, capabilities=["extinguisher"])
    a.state = mod.AgentState.LEADER
    a.task_claims = {}
    a._handle_task_claim(sender=2, payload=struct.pack("!If", 101, 50.0))
    return dict(claims={str(k): [v["winner"], float(v["utility"]).hex()] for k, v in a.task_claims.items()},
                log=a._send_msg.log())


def s_leader_hysteresis(mod):  # test_allocation.py:70-96
    a = _mk(mod, agent_id=1, total_agents=3, capabilities=["extinguisher"])
    a.state = mod.AgentState.LEADER
    a.task_claims = {101: {"winner": 2, "utility": 50.0}}
    a._handle_task_claim(sender=3, payload=struct.pack("!If", 101, 52.0))
    mid = a.task_claims[101]["winner"]
    log1 = a._send_msg.log()
    a._send_msg = Recorder()
    a._handle_task_claim(sender=3, payload=struct.pack("!If", 101, 60.0))
    return dict(mid_winner=mid, log1=log1, final_winner=a.task_claims[101]["winner"],
                log2=a._send_msg.log())


# Extra single-agent edge scenarios beyond the shipped ten (handler corners the batch
# kernels must also honour).

def s_heartbeat_paths(mod):  # agent.py:243-261
    out = []
    for state, me, sender in [("LEADER", 5, 3), ("LEADER", 5, 9), ("FOLLOWER", 5, 3),
                              ("ELECTION_WAIT", 5, 3), ("ELECTION_WAIT", 5, 9)]:
        a = _mk(mod, agent_id=me, total_agents=10)
        a.state = getattr(mod.AgentState, state)
        a.position = [1.5, -2.25]
        a._handle_heartbeat(sender, struct.pack("!ff", 3.5, 4.25))
        out.append(dict(state=_state_name(a.state), leader_id=a.leader_id,
                        leader_pos=list(a.leader_pos) if a.leader_pos else None,
                        log=a._send_msg.log()))
    return dict(cases=out)


def s_acclaim_paths(mod):  # agent.py:263-275
    out = []
    for state, me, sender, tick in [("ELECTION_WAIT", 5, 3, 0), ("ELECTION_WAIT", 5, 3, 7),
                                    ("FOLLOWER", 5, 3, 0), ("LEADER", 5, 5, 0),
                                    ("FOLLOWER", 5, 8, 0)]:
        a = _mk(mod, agent_id=me, total_agents=10)
        a.state = getattr(mod.AgentState, state)
        a.tick = tick
        a._handle_election_acclaim(sender)
        out.append(dict(state=_state_name(a.state), leader_id=a.leader_id, log=a._send_msg.log()))
    return dict(cases=out)


def s_coordinator_and_wire(mod):  # agent.py:197-214, 277-281
    a = _mk(mod, agent_id=7, total_agents=10, capabilities=["sonar"])
    a.state = mod.AgentState.LEADER
    a.on_message_received(b"\x03\x02")                              # short: dropped
    a.on_message_received(struct.pack("!BBI", 9, 2, 0))             # unknown type: ignored
    s1 = [_state_name(a.state), a.leader_id]
    a.on_message_received(struct.pack("!BBI", 3, 2, 0))             # coordinator
    s2 = [_state_name(a.state), a.leader_id]
    a.tasks = {4: {"status": "OPEN", "pos": (0.0, 0.0)}, 6: {"status": "OPEN", "pos": (0.0, 0.0)}}
    a.on_message_received(struct.pack("!BBI", 5, 9, 0) + struct.pack("!IB", 4, 7))
    a.on_message_received(struct.pack("!BBI", 5, 9, 0) + struct.pack("!IB", 6, 3))
    a.on_message_received(struct.pack("!BBI", 5, 9, 0) + struct.pack("!IB", 8, 7))
    a.state = mod.AgentState.LEADER
    a.on_message_received(struct.pack("!BBI", 4, 3, 0) + struct.pack("!If", 11, 33.25))
    a.on_message_received(struct.pack("!BBI", 1, 200, 0) + struct.pack("!ff", 1.0, 2.0))
    return dict(s1=s1, s2=s2, statuses={str(k): v["status"] for k, v in a.tasks.items()},
                claims={str(k): [v["winner"], float(v["utility"]).hex()] for k, v in a.task_claims.items()},
                final=[_state_name(a.state), a.leader_id, list(a.leader_pos) if a.leader_pos else None],
                log=a._send_msg.log())


def s_claim_loop(mod):  # agent.py:292-302 over several tasks, statuses and the 20.0 edge
    a = _mk(mod, agent_id=3, total_agents=10, capabilities=["camera", "sonar"])
    a.position = [0.5, -0.25]
    a.tasks = {
        1: {"status": "OPEN", "pos": (4.5, -0.25)},                        # d = 4 -> U = 20 (no claim)
        2: {"status": "OPEN", "pos": (1.0, 1.0), "required_cap": "sonar"},
        3: {"status": "LOCKED", "pos": (0.5, -0.25)},
        4: {"status": "OPEN", "pos": (0.5, -0.25), "required_cap": "gripper"},
        5: {"status": "OPEN", "pos": (0.5, -0.25)},                        # d = 0 -> U = 100
        6: {"status": "OPEN", "pos": (3.0, 2.0), "required_cap": "camera"},
    }
    a._process_tasks()
    return dict(statuses={str(k): v["status"] for k, v in a.tasks.items()}, log=a._send_msg.log())


SHIPPED = [s_initial_state, s_election_timeout_trigger, s_election_victory_after_wait,
           s_submission_to_higher_id, s_bullying_lower_id, s_utility_with_capability,
           s_utility_missing_capability, s_greedy_claim, s_leader_conflict_resolution_win,
           s_leader_hysteresis]
EXTRA = [s_heartbeat_paths, s_acclaim_paths, s_coordinator_and_wire, s_claim_loop]
ALL = SHIPPED + EXTRA
