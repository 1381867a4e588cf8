"""PCIe-inclusive election rate at C3 (10M agents): the graph and IDs start in pinned host memory,
are copied into the swarm's device buffers, the election runs, and leaders + states come back to
pinned host memory.  bench.py's `value` starts with inputs resident in HBM (the C-ABI takes device
pointers); this probe prices the host hand-over a caller with host-side buffers would pay.
Usage: python tools/pcie_probe.py [--agents N] [--reps K]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2026)
    args = ap.parse_args()
    import torch
    from swarm_amd import gen
    from swarm_amd.swarm import Swarm

    dev = torch.device("cuda", 0)
    d = gen.swarm_inputs(args.agents, args.seed, deg=16.0, t=16)
    sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device=dev).build_graph(1.0)
    h_rp = sw.row_ptr.cpu().pin_memory()
    h_col = sw.col.cpu().pin_memory()
    h_ids = sw.ids.cpu().pin_memory()
    h_leader = torch.empty_like(sw.leader, device="cpu").pin_memory()
    h_state = torch.empty_like(sw.state, device="cpu").pin_memory()
    h2d = h_rp.numel() * 4 + h_col.numel() * 4 + h_ids.numel() * 4
    d2h = h_leader.numel() * 4 + h_state.numel()
    sw.elect()  # warm-up
    torch.cuda.synchronize()
    out = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sw.row_ptr.copy_(h_rp, non_blocking=True)
        sw.col.copy_(h_col, non_blocking=True)
        sw.ids.copy_(h_ids, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r = sw.elect()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        h_leader.copy_(sw.leader, non_blocking=True)
        h_state.copy_(sw.state, non_blocking=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out.append((t1 - t0, t2 - t1, t3 - t2, r.rounds_exec))
    h, e, b, rounds = min(out, key=lambda q: q[0] + q[1] + q[2])
    tot = h + e + b
    print(json.dumps({"agents": sw.n, "edges": sw.n_edges, "rounds_exec": rounds,
                      "h2d_bytes": h2d, "d2h_bytes": d2h, "h2d_ms": h * 1e3, "elect_ms": e * 1e3,
                      "d2h_ms": b * 1e3, "h2d_GBps": h2d / h / 1e9, "d2h_GBps": d2h / b / 1e9,
                      "resident_agent_rounds_per_s": sw.n * rounds / e,
                      "pcie_inclusive_agent_rounds_per_s": sw.n * rounds / tot}))


if __name__ == "__main__":
    main()
