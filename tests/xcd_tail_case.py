"""Subprocess body of test_xcd_tail.py: elections with the single-XCD tail forced (the tuning is read
once per process from the environment), checked against the oracle's frontier restatement
(agent.py:263-275).  Prints one JSON line: {"ok": bool, "cases": [...], "error": str}."""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-swarm-algorithm_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def path_graph(n, seed):
    rng = np.random.default_rng(seed)
    ids = rng.permutation(n).astype(np.int32)
    rp = np.concatenate([[0], np.cumsum([1] + [2] * (n - 2) + [1])]).astype(np.int64)
    col = np.concatenate([[1]] + [[i - 1, i + 1] for i in range(1, n - 1)] + [[n - 2]]).astype(np.int32)
    return ids, rp, col


def main():
    from oracle import oracle
    from swarm_amd import _lib, gen
    import swarm_amd.swarm as swm
    oracle.lib()
    _lib.load()
    cases = []
    # random geometric swarms (dense and sparse graphs), then a long path (hundreds of tail rounds:
    # several launches, the 256-round stamp clears) with cut runs around them
    for n, deg, seed in ((5_000, 16.0, 1), (70_000, 3.0, 2), (300_000, 16.0, 3)):
        d = gen.swarm_inputs(n, seed, deg=deg)
        s = swm.Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
        rp = s.row_ptr.cpu().numpy().astype(np.int64)
        lead, state, rounds, changes = oracle.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy())
        for compact in (True, False):
            r = s.elect(compact=compact)
            ok = (r.converged and r.rounds_exec == rounds and np.array_equal(r.changes, changes)
                  and np.array_equal(r.leader.cpu().numpy(), lead) and np.array_equal(r.state.cpu().numpy(), state))
            cases.append({"n": n, "deg": deg, "compact": compact, "rounds": int(rounds), "ok": bool(ok)})
        m = max(1, rounds // 2)
        want = oracle.elect_frontier(rp, s.col.cpu().numpy(), s.ids.cpu().numpy(), max_rounds=m)
        r = s.elect(max_rounds=m)
        ok = (not r.converged and r.rounds_exec == m and np.array_equal(r.leader.cpu().numpy(), want[0])
              and np.array_equal(r.changes, changes[:m]))
        cases.append({"n": n, "deg": deg, "cut": m, "ok": bool(ok)})
    n = 3000
    ids, rp, col = path_graph(n, 12)
    s = swm.Swarm(ids, np.arange(float(n)), np.zeros(n), layout="input", device="cuda").set_graph(rp, col)
    full = s.elect()
    lead, state, rounds, changes = oracle.elect_frontier(rp, col, ids)
    ok = (full.converged and full.rounds_exec == rounds and np.array_equal(full.changes, changes)
          and np.array_equal(full.leader.cpu().numpy(), lead))
    cases.append({"n": n, "graph": "path", "rounds": int(rounds), "ok": bool(ok)})
    for m in (11, 255, 256, 257, 258, 300, 511, 512, 513, 1000):
        if m >= full.rounds_exec:
            continue
        r = s.elect(max_rounds=m)
        want = np.array([ids[max(0, i - m):i + m + 1].max() for i in range(n)])
        ok = (not r.converged and r.rounds_exec == m and np.array_equal(r.changes, full.changes[:m])
              and np.array_equal(r.leader.cpu().numpy(), want))
        cases.append({"n": n, "graph": "path", "cut": m, "ok": bool(ok)})
    return cases


if __name__ == "__main__":
    try:
        cases = main()
        print(json.dumps({"ok": all(c["ok"] for c in cases), "cases": cases, "error": ""}))
    except Exception:  # noqa: BLE001 -- reported to the parent test
        print(json.dumps({"ok": False, "cases": [], "error": traceback.format_exc()}))
