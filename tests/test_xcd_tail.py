"""Single-XCD tail rounds (k_tail_xcd) forced from round 10 on small swarms, against
the oracle's frontier restatement (agent.py:263-275): leaders, states, rounds_exec, every per-round
change count, and cut runs (max_rounds) inside and across the tail kernel's launches.  The tuning is
read once per process, so the cases run in one child process with the environment set."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("min_changes", ["1000000000", "-1"])
def test_forced_xcd_tail_matches_oracle(min_changes):
    env = dict(os.environ, SWARM_SMALL_CHUNKS="0", SWARM_XCD_TAIL="1", SWARM_XCD_MIN_CHANGES=min_changes)
    if min_changes != "-1":  # agent-order stamps from the first sparse round: the tail starts at round 10
        env["SWARM_IL_MIN_CHANGES"] = min_changes
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "xcd_tail_case.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    res = json.loads(lines[-1])
    assert res["ok"], (res["error"], [c for c in res["cases"] if not c["ok"]])
