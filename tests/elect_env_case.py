"""Subprocess body of test_elect_sizes.py's environment-forced cases: elections with the tuning read
once per process from the environment (SWARM_XCD_MAX_N: which swarms run their sparse rounds on one
XCD; SWARM_SMALL_CHUNKS: the chunk size), checked against the oracle's frontier restatement
(agent.py:263-275): leaders, states, rounds, every per-round count, and cut runs.  Prints one JSON
line."""
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
    from swarm_amd import _lib, gen
    import swarm_amd.swarm as swm
    oracle.lib()
    _lib.load()
    cases = []
    for n, deg, seed in ((2, 16.0, 1), (2049, 3.0, 2), (65_537, 16.0, 3), (100_000, 16.0, 4), (300_000, 3.0, 5),
                         (1_048_577, 16.0, 6)):
        d = gen.swarm_inputs(n, 500 + seed, deg=deg)
        s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
        rp = s.row_ptr.cpu().numpy().astype(np.int64)
        lead, state, rounds, changes = oracle.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy())
        for compact in (True, False):
            r = s.elect(compact=compact, max_rounds=1 << 16)
            ok = (r.converged and r.rounds_exec == rounds and np.array_equal(r.changes, changes)
                  and np.array_equal(r.leader.cpu().numpy(), lead) and np.array_equal(r.state.cpu().numpy(), state))
            cases.append({"n": n, "deg": deg, "compact": compact, "ok": bool(ok)})
        if rounds > 12:
            m = rounds // 2
            want = oracle.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy(), max_rounds=m)
            r = s.elect(max_rounds=m)
            ok = (not r.converged and r.rounds_exec == m and np.array_equal(r.leader.cpu().numpy(), want[0])
                  and np.array_equal(r.changes, changes[:m]))
            cases.append({"n": n, "deg": deg, "cut": m, "ok": bool(ok)})
    # a path: ~1 500 rounds, several 248-round launches, cut runs on and around their boundaries
    n = 1500
    rng = np.random.default_rng(12)
    ids = rng.permutation(n).astype(np.int32)
    rp = np.concatenate([[0], np.cumsum([1] + [2] * (n - 2) + [1])]).astype(np.int64)
    col = np.concatenate([[1]] + [[i - 1, i + 1] for i in range(1, n - 1)] + [[n - 2]]).astype(np.int32)
    s = swm.Swarm(ids, np.arange(float(n)), np.zeros(n), layout="input", device="cuda").set_graph(rp, col)
    full = s.elect(max_rounds=1 << 16)
    lead, _, rounds, changes = oracle.elect_frontier(rp, col, ids)
    cases.append({"n": n, "graph": "path", "ok": bool(full.converged and full.rounds_exec == rounds
                                                      and np.array_equal(full.changes, changes)
                                                      and np.array_equal(full.leader.cpu().numpy(), lead))})
    for m in (9, 10, 11, 257, 258, 259, 505, 506, 507, 1000):
        if m >= full.rounds_exec:
            continue
        r = s.elect(max_rounds=m)
        want = np.array([ids[max(0, i - m):i + m + 1].max() for i in range(n)])
        cases.append({"n": n, "graph": "path", "cut": m,
                      "ok": bool(not r.converged and r.rounds_exec == m and np.array_equal(r.changes, changes[:m])
                                 and np.array_equal(r.leader.cpu().numpy(), want))})
    return cases


if __name__ == "__main__":
    try:
        cases = main()
        print(json.dumps({"ok": all(c["ok"] for c in cases), "cases": cases, "error": ""}))
    except Exception:  # noqa: BLE001 -- reported to the parent test
        print(json.dumps({"ok": False, "cases": [], "error": traceback.format_exc()}))
