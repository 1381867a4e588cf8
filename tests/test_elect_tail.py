"""The one-workgroup tail (SWARM_TAIL_WG, elect.hip k_tail_wg; opt-in, an experiment of VERDICT r5 #4): the
election with the tail forced early (a large cap) returns exactly the oracle's leaders, states, rounds and
per-round change counts (agent.py:263-275 under contract E2) -- 16-bit and int32 columns, hand-backs when the
marked set outgrows the list, runs cut by max_rounds inside the tail.  The tunable is read once per process,
so the cases run in a subprocess."""
import json
import os
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [%r, %r]
from swarm_amd import gen
from swarm_amd.swarm import Swarm
from oracle import oracle
out = []
for n, seed, deg, compact, cap_rounds in [(30_000, 3, 16.0, True, None), (120_000, 5, 16.0, True, None),
                                          (120_000, 5, 16.0, False, None), (200_000, 7, 6.0, True, None),
                                          (120_000, 5, 16.0, True, -3)]:
    d = gen.swarm_inputs(n, seed, deg=deg)
    s = Swarm(d["ids"], d["x"], d["y"], device="cuda:0").build_graph(1.0)
    lead, state, rounds, changes = oracle.elect(s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy(),
                                                s.ids.cpu().numpy())
    mr = rounds + cap_rounds if cap_rounds else 1 << 16
    r = s.elect(max_rounds=mr, compact=compact)
    if cap_rounds:  # cut inside the tail: the state after mr rounds
        lead_c, _, _, _ = oracle.elect(s.row_ptr.cpu().numpy().astype(np.int64), s.col.cpu().numpy(),
                                       s.ids.cpu().numpy(), max_rounds=mr)
        ok = (not r.converged and r.rounds_exec == mr and np.array_equal(r.changes, changes[:mr])
              and np.array_equal(r.leader.cpu().numpy(), lead_c))
    else:
        ok = (r.converged and r.rounds_exec == rounds and np.array_equal(r.changes, changes)
              and np.array_equal(r.leader.cpu().numpy(), lead) and np.array_equal(r.state.cpu().numpy(), state))
    out.append(dict(n=n, seed=seed, compact=compact, cut=cap_rounds, ok=bool(ok), rounds=int(r.rounds_exec)))
print(json.dumps(out))
"""


@pytest.mark.parametrize("cap", ["2048", "64"])
def test_tail_exact_against_oracle(cap):
    env = dict(os.environ, SWARM_TAIL_WG=cap)
    p = subprocess.run([sys.executable, "-c", _CHILD % (PKG, ROOT)], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert all(c["ok"] for c in res), res
