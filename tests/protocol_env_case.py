"""Subprocess body of test_protocol.py's environment-forced cases: protocol ticks with k_tick's
receive-role grid forced by the environment (SWARM_FSM_RECV_WGS, read once per process), checked
against the oracle (agent.py:217-289 as contract T1).  Prints one JSON line."""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "distributed-swarm-algorithm_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    from oracle import oracle
    from swarm_amd import _lib
    from test_protocol import OUT, _directed, _gpu_state, _gpu_swarm, _random_case, _run_oracle
    oracle.lib()
    _lib.load()
    cases = []
    for n, seed, side, mode, directed in ((20000, 1, 50.0, "push", False), (20000, 3, 50.0, "push", True),
                                          (20000, 5, 50.0, "hybrid", False), (300000, 2, 180.0, "push", False)):
        g = _random_case(n, seed, side)
        if directed:
            g = _directed(g, seed)
        g["ticks"], g["kill_ticks"] = np.int64(150), np.array([60, 61, 110], np.int64)
        want = _run_oracle(oracle, g)
        s = _gpu_swarm(g)
        c1 = s.protocol_run(64, kill_ticks=g["kill_ticks"], seed=seed, mode=mode)
        c2 = s.protocol_run(86, kill_ticks=g["kill_ticks"], seed=seed, mode=mode)
        got = _gpu_state(s)
        bad = [k for k in OUT if not np.array_equal(got[k], want[k])]
        if not np.array_equal(np.concatenate([c1, c2]), want["counts"]):
            bad.append("counts")
        cases.append({"n": n, "seed": seed, "mode": mode, "directed": directed, "bad": bad})
    return cases


if __name__ == "__main__":
    try:
        cases = main()
        print(json.dumps({"ok": all(not c["bad"] for c in cases), "cases": cases, "error": ""}))
    except Exception:  # noqa: BLE001 -- reported to the parent test
        print(json.dumps({"ok": False, "cases": [], "error": traceback.format_exc()}))
