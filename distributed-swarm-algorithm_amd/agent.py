"""Drop-in ``agent`` module: the reference's scalar SwarmAgent surface.

``from agent import SwarmAgent, AgentState, MsgType`` works as it does against the reference
(test_election.py:10, test_allocation.py:9).  Every handler keeps its name, argument order,
wire format, side effects and the positional ``self._send_msg(type, payload)`` egress that
the reference tests mock per instance (test_election.py:16).

This module is the *single-agent* (config 1, CPU plumbing) face of the framework.  The
batched, HBM-resident round -- thousands to hundreds of millions of agents per call -- is
``swarm_amd.Swarm`` (HIP kernels behind the C-ABI in include/swarm.h); ``Swarm.from_agents``
/ ``Swarm.write_back`` move a population of these objects onto and off the GPU.

Reference map (agent.py in the reference):
  MsgType/AgentState 12-22 | __init__ 25-54 | loop 67-92 | physics 94-181 | codec 184-214 |
  election 216-289 | allocation 291-347 | CLI 349-360
"""
from __future__ import annotations

import argparse
import enum
import logging
import math
import random
import struct
import time

__all__ = ["MsgType", "AgentState", "SwarmAgent"]


class MsgType(enum.IntEnum):
    HEARTBEAT = 1
    ELECTION_ACCLAIM = 2
    COORDINATOR = 3
    TASK_CLAIM = 4
    TASK_CONFLICT = 5


class AgentState(enum.Enum):
    FOLLOWER = 1
    ELECTION_WAIT = 2
    LEADER = 3


# Wire layouts (network byte order).  The u8 sender / winner fields cap IDs at 255, exactly
# as the reference's formats do; the batched Swarm path uses int32 IDs and no packets.
HEADER = "!BBI"          # type, sender, tick           (agent.py:186)
HEADER_LEN = 6
ACCLAIM_BODY = "!B"      # acclaimed id                 (agent.py:240)
POS_BODY = "!ff"         # leader position              (agent.py:286)
CLAIM_BODY = "!If"       # task id, f32 utility         (agent.py:302)
CONFLICT_BODY = "!IB"    # task id, winner id           (agent.py:322)

# Protocol constants (agent.py:222, 229, 288, 297, 316, 347)
HB_TIMEOUT_S = 3.0
JITTER_MAX_S = 0.2
HB_EVERY_TICKS = 10
CLAIM_THRESHOLD = 20.0
HYSTERESIS = 5.0
UTILITY_SCALE = 100.0

# Motion constants (agent.py:49, 68, 118-129, 149-153)
TICK_HZ = 10.0
ARRIVE_TOL = 0.5
K_ATTRACT = 1.0
K_OBSTACLE = 50.0
OBSTACLE_RANGE = 5.0
K_SEPARATE = 20.0
PERSONAL_SPACE = 2.0
MIN_DIST = 0.001

_log = logging.getLogger


class SwarmAgent:
    """One robot: quiet-bully election, greedy claims with leader arbitration, APF motion."""

    def __init__(self, agent_id, total_agents, capabilities=None):
        self.agent_id = agent_id
        self.total_agents = total_agents
        self.logger = _log(str(agent_id))
        # election
        self.state = AgentState.FOLLOWER
        self.leader_id = None
        self.leader_pos = None
        self.last_heartbeat_time = time.time()
        self.tick = 0
        self.election_wait_start = 0.0
        self.election_delay = 0.0
        # allocation: tasks {id: {'status', 'pos', ['required_cap']}}, claims {id: {'winner', 'utility'}}
        self.tasks = {}
        self.task_claims = {}
        # motion
        self.position = [0.0, 0.0]
        self.velocity = [0.0, 0.0]
        self.max_speed = 5.0
        self.sensors = {"obstacles": [], "neighbors": []}
        self.target = None
        self.capabilities = capabilities or []
        # optional egress: callable(packet: bytes); None keeps the reference's stub behaviour
        self.transport = None
        self.logger.info("Agent initialized. State: %s Caps: %s", self.state.name, self.capabilities)

    # ------------------------------------------------------------------ sensors / targets
    def set_target(self, x, y):
        self.target = (x, y)

    def update_sensors(self, obstacles, neighbors):
        """obstacles: [(x, y, radius)], neighbors: [(id, x, y)]."""
        self.sensors["obstacles"] = obstacles
        self.sensors["neighbors"] = neighbors

    # ------------------------------------------------------------------ control loop
    def update_loop(self):
        period = 1.0 / TICK_HZ
        while True:
            t0 = time.time()
            self.tick += 1
            self._process_logic()
            self._update_physics(period)
            slack = period - (time.time() - t0)
            if slack > 0:
                time.sleep(slack)

    def _process_logic(self):
        self._check_election_timeout()
        if self.state == AgentState.LEADER:
            self._send_heartbeat()
        self._process_tasks()

    # ------------------------------------------------------------------ codec / transport
    def _pack_header(self, msg_type):
        return struct.pack(HEADER, msg_type, self.agent_id, self.tick)

    def _send_msg(self, msg_type, payload=b""):
        packet = self._pack_header(msg_type) + payload
        if self.transport is not None:
            self.transport(packet)

    def on_message_received(self, data):
        if len(data) < HEADER_LEN:
            return
        msg_type, sender, _tick = struct.unpack(HEADER, data[:HEADER_LEN])
        body = data[HEADER_LEN:]
        route = self._ROUTES.get(msg_type)
        if route is not None:
            route(self, sender, body)

    _ROUTES = {
        MsgType.HEARTBEAT: lambda self, s, b: self._handle_heartbeat(s, b),
        MsgType.ELECTION_ACCLAIM: lambda self, s, b: self._handle_election_acclaim(s),
        MsgType.COORDINATOR: lambda self, s, b: self._handle_coordinator(s),
        MsgType.TASK_CLAIM: lambda self, s, b: self._handle_task_claim(s, b),
        MsgType.TASK_CONFLICT: lambda self, s, b: self._handle_task_conflict(s, b),
    }

    # ------------------------------------------------------------------ election
    def _check_election_timeout(self):
        st = self.state
        if st == AgentState.LEADER:
            return
        silent_for = time.time() - self.last_heartbeat_time
        if st == AgentState.FOLLOWER and silent_for > HB_TIMEOUT_S:
            self.logger.warning("Leader timeout (%.1fs). Entering ELECTION_WAIT.", silent_for)
            self.state = AgentState.ELECTION_WAIT
            self.election_wait_start = time.time()
            self.election_delay = random.uniform(0.0, JITTER_MAX_S)
            self.leader_id = None
            self.leader_pos = None
        if self.state == AgentState.ELECTION_WAIT and \
                time.time() - self.election_wait_start > self.election_delay:
            self.logger.info("Election wait ended. Acclaiming Leadership.")
            self.state = AgentState.LEADER
            self.leader_id = self.agent_id
            self._send_msg(MsgType.ELECTION_ACCLAIM, struct.pack(ACCLAIM_BODY, self.agent_id))
            self._send_msg(MsgType.COORDINATOR)

    def _handle_heartbeat(self, sender, payload):
        leading = self.state == AgentState.LEADER
        if leading and sender < self.agent_id:
            self._send_heartbeat()          # out-rank the sender: answer with our own beat
            return
        if leading and sender > self.agent_id:
            self.logger.info("Yielding to higher leader %s", sender)
            self.state = AgentState.FOLLOWER
        self.leader_id = sender
        self.last_heartbeat_time = time.time()
        if len(payload) == struct.calcsize(POS_BODY):
            self.leader_pos = struct.unpack(POS_BODY, payload)
        if self.state == AgentState.ELECTION_WAIT:
            self.state = AgentState.FOLLOWER

    def _handle_election_acclaim(self, sender):
        me = self.agent_id
        if sender > me:
            self.logger.info("Saw acclaim from higher node %s. Backing down.", sender)
            self.state = AgentState.FOLLOWER
            self.leader_id = sender
            self.last_heartbeat_time = time.time()
            return
        if sender < me and self.state in (AgentState.LEADER, AgentState.ELECTION_WAIT):
            if self.state == AgentState.ELECTION_WAIT:
                self.state = AgentState.LEADER
                self.leader_id = me
            self._send_heartbeat()

    def _handle_coordinator(self, sender):
        self.leader_id = sender
        self.state = AgentState.FOLLOWER
        self.last_heartbeat_time = time.time()
        self.logger.info("New Coordinator: %s", sender)

    def _send_heartbeat(self):
        body = struct.pack(POS_BODY, self.position[0], self.position[1])
        if self.tick % HB_EVERY_TICKS == 0:
            self._send_msg(MsgType.HEARTBEAT, body)

    # ------------------------------------------------------------------ allocation
    def _process_tasks(self):
        for task_id, task in self.tasks.items():
            if task["status"] != "OPEN":
                continue
            u = self._calculate_utility(task)
            if u > CLAIM_THRESHOLD:
                self.logger.info("Claiming task %s with U=%.1f", task_id, u)
                task["status"] = "TENTATIVE"
                self._send_msg(MsgType.TASK_CLAIM, struct.pack(CLAIM_BODY, task_id, u))

    def _handle_task_claim(self, sender, payload):
        task_id, offered = struct.unpack(CLAIM_BODY, payload)
        if self.state != AgentState.LEADER:
            return
        held = self.task_claims.get(task_id)
        if not held or offered > held["utility"] + HYSTERESIS:
            self.task_claims[task_id] = {"winner": sender, "utility": offered}
            self._send_msg(MsgType.TASK_CONFLICT, struct.pack(CONFLICT_BODY, task_id, sender))
        elif held["winner"] != sender:
            self._send_msg(MsgType.TASK_CONFLICT, struct.pack(CONFLICT_BODY, task_id, held["winner"]))

    def _handle_task_conflict(self, sender, payload):
        task_id, winner_id = struct.unpack(CONFLICT_BODY, payload)
        mine = winner_id == self.agent_id
        if mine:
            self.logger.info("Won task %s!", task_id)
        if task_id in self.tasks:
            self.tasks[task_id]["status"] = "ASSIGNED" if mine else "LOCKED"

    def _calculate_utility(self, task):
        # ``** 2`` (CPython float_pow -> libm pow), not x*x: keeps the reference's bits.
        tx, ty = task["pos"][0], task["pos"][1]
        dist = math.sqrt((self.position[0] - tx) ** 2 + (self.position[1] - ty) ** 2)
        capable = not ("required_cap" in task and task["required_cap"] not in self.capabilities)
        return (UTILITY_SCALE / (1.0 + dist)) * (1.0 if capable else 0.0)

    # ------------------------------------------------------------------ motion (APF)
    def _update_physics(self, dt):
        px, py = self.position[0], self.position[1]
        if self.state == AgentState.FOLLOWER and self.leader_pos:
            rank = self.agent_id                       # V formation behind the leader
            side = 2.0 * rank if rank % 2 == 0 else -2.0 * rank
            self.target = (self.leader_pos[0] - 2.0 * rank, self.leader_pos[1] + side)
        if not self.target:
            return
        fx = fy = 0.0
        gx, gy = self.target[0] - px, self.target[1] - py
        if math.sqrt(gx ** 2 + gy ** 2) > ARRIVE_TOL:
            fx, fy = K_ATTRACT * gx, K_ATTRACT * gy
        rx = ry = 0.0
        for ox, oy, rad in self.sensors["obstacles"]:
            gap = math.sqrt((px - ox) ** 2 + (py - oy) ** 2) - rad
            if gap <= MIN_DIST:
                gap = MIN_DIST
            if gap < OBSTACLE_RANGE:
                push = K_OBSTACLE * (1.0 / gap - 1.0 / OBSTACLE_RANGE) / (gap ** 2)
                ux, uy = px - ox, py - oy
                norm = math.sqrt(ux ** 2 + uy ** 2)
                rx += (ux / norm) * push
                ry += (uy / norm) * push
        sx = sy = 0.0
        for _nid, nx, ny in self.sensors["neighbors"]:
            gap = math.sqrt((px - nx) ** 2 + (py - ny) ** 2)
            if gap < PERSONAL_SPACE:
                gap = MIN_DIST if gap <= MIN_DIST else gap
                push = K_SEPARATE / (gap ** 2)
                ux, uy = px - nx, py - ny
                norm = math.sqrt(ux ** 2 + uy ** 2)
                sx += (ux / norm) * push
                sy += (uy / norm) * push
        tx_, ty_ = fx + rx + sx, fy + ry + sy
        speed = math.sqrt(tx_ ** 2 + ty_ ** 2)
        if speed > self.max_speed:
            k = self.max_speed / speed
            self.velocity = [tx_ * k, ty_ * k]
        else:
            self.velocity = [tx_, ty_]
        self.position[0] += self.velocity[0] * dt
        self.position[1] += self.velocity[1] * dt
        if self.tick % HB_EVERY_TICKS == 0:
            self.logger.info("Pos: (%.2f, %.2f) V: (%.2f, %.2f)", self.position[0], self.position[1],
                             self.velocity[0], self.velocity[1])


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--id", type=int, required=True, help="Agent ID")
    ap.add_argument("--count", type=int, default=1, help="Total Agents")
    ap.add_argument("--caps", type=str, nargs="+", default=[], help="Agent Capabilities")
    a = ap.parse_args(argv)
    bot = SwarmAgent(a.id, a.count, capabilities=a.caps)
    try:
        bot.update_loop()
    except KeyboardInterrupt:
        print("Shutting down.")


if __name__ == "__main__":
    main()
