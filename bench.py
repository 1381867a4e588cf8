#!/usr/bin/env python3
"""Headline benchmark: agent-rounds/sec of the swarm step (election to convergence + one
10k-task allocation round) at 10M agents on MI355X (BASELINE.json config C3).

A step = one full election (contract E2, all rounds to convergence) + one allocation round,
over inputs already resident in HBM.  value = agents x rounds_exec x steps / elapsed, summed
over ranks (weak scaling: every rank owns `--agents` agents).  Rank 0 prints ONE JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--agents 10000000] [--tasks 10000]
  multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
REF_PYTHON_RATE = 65_355.0  # agent-rounds/s, SURVEY.md §6 (reference Python, 1 core)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--agents", type=int, default=None,
                    help="agents per GPU (default: 10M for C3; C5 splits 100M over the GPUs)")
    ap.add_argument("--config", choices=["C3", "C5"], default="C3",
                    help="C3: 10M agents per GPU (weak scaling); C5: 100M agents in all, split over the GPUs "
                         "by contiguous ID range (12.5M per GPU at N = 8; strong scaling)")
    ap.add_argument("--tasks", type=int, default=10_000)
    ap.add_argument("--deg", type=float, default=16.0)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--elect-mode", choices=["frontier", "dense"], default="frontier")
    ap.add_argument("--roofline-rounds", type=int, default=20)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the oracle timing")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--rows", type=int, default=1,
                    help="0 to skip the other SURVEY §8 rows (C2, C4 auction, physics, protocol, codec)")
    ap.add_argument("--partition", choices=["strips", "blocks"], default="strips",
                    help="N > 1: strips (strip-major IDs: 2 peers per rank, 16-bit columns) or blocks "
                         "(SURVEY §8e's Morton IDs: Morton-ordered blocks, up to 8 peers per rank)")
    ap.add_argument("--pieces", type=int, default=None,
                    help="cut the IDs into N x PIECES equal ranges dealt round-robin (rank q owns ranges q, q + N, "
                         "...) -- evens out the election's per-round work across ranks (DESIGN §6).  blocks: Morton "
                         "pieces of every block (dist.block_pieces); strips: N x PIECES thin strips, strip-major IDs "
                         "at that grain (gen.shard_inputs pieces=)).  Default: 16 for --config C5 --partition "
                         "blocks (with --halo-depth 4: the model's 6.3x at 8 GPUs), else 1")
    ap.add_argument("--halo-depth", type=int, default=None,
                    help="N > 1: rounds between halo exchanges = ghost depth in radio radii (default: "
                         "SWARM_HALO_DEPTH or 16; C5 blocks with --pieces 16: 4, DESIGN §6)")
    ap.add_argument("--union-gpu", type=int, default=1,
                    help="with --oracle-check: also elect the union swarm on rank 0's GPU (the model's N = 1 time)")
    ap.add_argument("--model", type=int, default=1,
                    help="N > 1: the election cost model (DESIGN §6) from this run's per-rank round counts and a "
                         "calibration election of rank 0's shard alone")
    ap.add_argument("--oracle-check", type=int, default=None,
                    help="N > 1: compare every rank's leaders, rounds and per-round global changes with the C "
                         "oracle (orc_elect_frontier) over the union swarm on rank 0's host (default: on for C5)")
    a = ap.parse_args()
    a.world_hint = int(os.environ.get("WORLD_SIZE", "1"))
    if a.agents is None:
        a.agents = 100_000_000 // a.world_hint if a.config == "C5" else 10_000_000
    if a.config == "C5":
        a.rows = 0  # the other §8 rows keep their own (C2 / C3-sized) workloads: not re-run at C5
    if a.pieces is None:
        a.pieces = 16 if (a.config == "C5" and a.partition == "blocks") else 1
        if a.pieces > 1 and a.halo_depth is None and "SWARM_HALO_DEPTH" not in os.environ:
            a.halo_depth = 4
    if a.oracle_check is None:
        a.oracle_check = 1 if a.config == "C5" else 0
    return a


def _spin_until_idle():
    """Wait for torch's current stream (libswarm launches on it) by polling, the thread kept awake."""
    import torch
    st = torch.cuda.current_stream()
    while not st.query():
        pass


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel_prefix):
    """HBM bytes per dispatch of a kernel from the newest committed rocprofv3 --pmc summary
    (profiles/*/pmc_traffic.json, written by tools/gpu_pmc.sh + tools/pmc_summary.py: FETCH_SIZE
    and WRITE_SIZE in separate passes, FETCH_SIZE doubled for gfx950).  bench.py cannot collect
    PMC counters itself (that needs rocprofv3 around the process), so it reports the measured
    figure of the same command with its source, or None."""
    import glob
    best = None
    paths = glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json"))
    latest = os.path.join(ROOT, "profiles", "LATEST")  # names the round directory to prefer
    if os.path.exists(latest):
        pref = os.path.join(ROOT, "profiles", open(latest).read().strip(), "pmc_traffic.json")
        paths = [pref] + [q for q in paths if q != pref] if os.path.exists(pref) else paths
    for path in paths:
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if k.startswith(kernel_prefix) and isinstance(v, dict):
                # profiles/LATEST's directory first, else the last in name order
                m = (path == paths[0] and os.path.exists(latest), path)
                if best is None or m > best[2]:
                    best = (v["hbm_bytes_per_dispatch"], os.path.relpath(path, ROOT), m)
    return None if best is None else (best[0], f"rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, {best[1]}")


def pmc_traffic_sum(names):
    """Summed HBM bytes per dispatch of several kernels (exact names, e.g. the launches of one
    protocol tick) from profiles/LATEST's PMC summary, or None when one of them is missing."""
    latest = os.path.join(ROOT, "profiles", "LATEST")
    if not os.path.exists(latest):
        return None
    path = os.path.join(ROOT, "profiles", open(latest).read().strip(), "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if not all(isinstance(d.get(k), dict) for k in names):
        return None
    return (sum(d[k]["hbm_bytes_per_dispatch"] for k in names),
            f"rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, {os.path.relpath(path, ROOT)} ({' + '.join(names)})")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SWARM_DIST_BACKEND=gloo: rehearse N ranks on fewer GPUs (halo staged through the host);
    # the default and the measured configuration is nccl (RCCL over xGMI), one GPU per rank
    backend = os.environ.get("SWARM_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from swarm_amd import _lib, gen
    from swarm_amd.swarm import Swarm

    dev = torch.device("cuda", local)
    if world > 1:
        return sharded(args, rank, world, dev)
    t0 = time.time()
    d = gen.swarm_inputs(args.agents, args.seed + 7919 * rank, deg=args.deg, t=args.tasks)
    sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device=dev).build_graph(1.0)
    tpos_x = torch.as_tensor(d["tx"], device=dev)
    tpos_y = torch.as_tensor(d["ty"], device=dev)
    treq = torch.as_tensor(d["treq"], device=dev)
    torch.cuda.synchronize()
    n, e = sw.n, sw.n_edges
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s: n={n} E={e} tasks={args.tasks}")

    def step():
        r = sw.elect(mode=args.elect_mode, max_rounds=1 << 16)
        a = sw.allocate(tpos_x, tpos_y, treq)
        return r, a

    for _ in range(args.warmup):
        r, a = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    rounds_total = 0
    for _ in range(args.steps):
        r, a = step()
        rounds_total += r.rounds_exec
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    # a non-converged election would report max_rounds rounds: refuse to print such a number
    assert r.converged, f"election did not converge in {r.rounds_exec} rounds"
    assert a.stats["mode_used"] in (_lib.ALLOC_BINNED, _lib.ALLOC_DENSE), a.stats
    check = final_state_check(sw, r)

    agent_rounds = float(n) * rounds_total
    if world > 1:
        t = torch.tensor([elapsed, agent_rounds], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, agent_rounds = float(mx[0]), float(t[1])

    # ---- split timing of a step (untimed replays, median of 3): election vs allocation
    splits = []
    for _ in range(3):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        r = sw.elect(mode=args.elect_mode, max_rounds=1 << 16)
        # elect() returns with its last kernels queued and then builds its result on the host:
        # wait, so that host tail counts as election time, not as the allocation's.  Spin on the stream
        # rather than block in a synchronize: in the timed step the allocation is launched by a thread
        # that never slept (libswarm's own waits spin), and a woken thread's first launches are slower
        # by up to ~0.1 ms on some boxes -- host wake-up, not allocation time
        _spin_until_idle()
        ev[1].record()
        a = sw.allocate(tpos_x, tpos_y, treq)
        ev[2].record()
        torch.cuda.synchronize()
        splits.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    t_elect_ms = float(np.median([x[0] for x in splits]))
    t_alloc_ms = float(np.median([x[1] for x in splits]))
    # the allocation's cell index (swarm_cell_index over the spatial storage order): built once per
    # position set, before the timed region -- the positions are static over the bench's steps
    idx_ms = []
    for _ in range(3):
        sw._cindex, sw._again = None, None
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sw._cell_index()
        torch.cuda.synchronize()
        idx_ms.append((time.perf_counter() - t1) * 1e3)
    sw.allocate(tpos_x, tpos_y, treq)  # trusted again (the index above is the current one)

    # ---- per-kernel device time of the election (HIP events recorded by libswarm around every
    # launch on the stream it launches on), one instrumented replay.  The dominant kernel is the
    # sparse round (k_sparse_block); like rocprof, its average covers every launch, including the
    # no-op rounds a batch issues after convergence.
    rt = sw.elect(mode=args.elect_mode, max_rounds=1 << 16, timed=True)
    if args.elect_mode == "frontier" and rt.sparse_launches:
        pmc = pmc_traffic("k_sparse_block<int, 8,")  # the 2 048-agent-chunk variant (10M agents)
        dom = {"kernel": "k_sparse_block (sparse E2 round: marked agents gather)",
               **sparse_round_bytes(rt.active_total, rt.edges_total, rt.dense_rounds, rt.rounds_exec, n, e,
                                    rt.sparse_launches, getattr(rt, "compact", False)),
               "avg_launch_ms": rt.sparse_ms / rt.sparse_launches, "launches": rt.sparse_launches,
               "traffic": pmc[0] if pmc else None, "traffic_source": pmc[1] if pmc else None,
               "all_rounds": {"bytes_per_launch": rt.bytes_total / max(rt.timed_launches, 1),
                              "avg_launch_ms": rt.gather_ms / max(rt.timed_launches, 1),
                              "launches": rt.timed_launches, "dense_rounds": rt.dense_rounds}}
    else:
        dom = None

    # ---- roofline of the dense election round (the north-star kernel), HIP events on the
    # stream libswarm launches on (torch's current stream)
    import ctypes
    rp, col, lin = sw.row_ptr, sw.col, sw.ids
    lout = torch.empty_like(lin)
    changed = torch.zeros(1, dtype=torch.int64, device=dev)
    L = _lib.lib()
    for _ in range(3):
        _lib.check(L.swarm_elect_round(_lib.ctx(), n, _lib.ptr(rp), _lib.ptr(col), _lib.ptr(lin),
                                       _lib.ptr(lout), _lib.ptr(changed), _lib.stream()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.roofline_rounds):
        _lib.check(L.swarm_elect_round(_lib.ctx(), n, _lib.ptr(rp), _lib.ptr(col), _lib.ptr(lin),
                                       _lib.ptr(lout), _lib.ptr(changed), _lib.stream()))
    e1.record()
    torch.cuda.synchronize()
    dense_round_ms = e0.elapsed_time(e1) / args.roofline_rounds
    bytes_round = 12 * n + 8 * e + 4
    achieved = bytes_round / (dense_round_ms * 1e-3) / 1e9
    del ctypes

    out = None
    if rank == 0:
        value = agent_rounds / elapsed
        out = {
            "metric": "agent-rounds/sec (election+allocation) at 10M agents; % of HBM roofline",
            "value": value,
            "unit": "agent-rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.config == "C5" else "weak",
            "vs_baseline": None,
            "dtype": "int32+f64",
            "data": "synthetic (seeded RGG, SplitMix64)",
            "config": {"workload": "%s: %d agents/GPU, deg %g RGG, election to convergence + %d-task allocation"
                       % (args.config, n, args.deg, args.tasks),
                       "agents_per_gpu": n, "edges_per_gpu": e, "tasks": args.tasks,
                       "elect_mode": args.elect_mode, "alloc_mode": a.stats.get("mode_used"),
                       "rounds_exec": r.rounds_exec, "parallelism": f"agents sharded x{world}",
                       "alloc_index": "the cell index of the static positions is built once, outside the timed "
                                      "steps (alloc_index_build_ms); a step that moves agents rebuilds it"},
            "breakdown_ms": {"elect": t_elect_ms, "alloc": t_alloc_ms},
            "alloc_index_build_ms": float(np.median(idx_ms)),
            # the step's algorithmic bytes (the frontier's per-round counters, DESIGN §4, + the
            # allocation's compulsory 24 B/agent + 36 B/task) over its time
            "hbm_frac_step": (r.bytes_total + 24 * n + 36 * args.tasks)
            / ((t_elect_ms + t_alloc_ms) * 1e-3) / (HBM_PEAK_GBS * 1e9),
            # the same over SURVEY §8(d)'s per-unit bytes only (12 B per gathered agent + 8 B per edge in
            # every executed round, dense rounds 12N + 8E + 4; no stamp scan, no second row offset):
            # the step-level fraction of the north-star target
            "hbm_frac_step_survey": survey_step_bytes(r, n, e, args.tasks)
            / ((t_elect_ms + t_alloc_ms) * 1e-3) / (HBM_PEAK_GBS * 1e9),
            # SURVEY §8d's formula, which prices every executed round as a dense round
            # (12N + 8E + 4 bytes): > 1 because the frontier reads only the changing neighbourhoods
            "hbm_frac_step_dense_equivalent": (r.rounds_exec * bytes_round + 24 * n + 36 * args.tasks)
            / ((t_elect_ms + t_alloc_ms) * 1e-3) / (HBM_PEAK_GBS * 1e9),
            "roofline": ({"kernel": dom["kernel"], "bound": "hbm",
                          "achieved": dom["bytes_per_launch"] / (dom["avg_launch_ms"] * 1e-3) / 1e9,
                          "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": dom["bytes_per_launch"] / (dom["avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          **{k: v for k, v in dom.items() if k != "kernel"}}
                         if dom else
                         {"kernel": "k_elect_dense (one E2 round)", "bound": "hbm",
                          "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                          "bytes_per_launch": bytes_round, "avg_launch_ms": dense_round_ms}),
            "roofline_dense_round": {"kernel": "k_elect_dense (one E2 round, the north-star kernel)",
                                     "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                                     "bytes_per_launch": bytes_round, "avg_launch_ms": dense_round_ms,
                                     "agent_rounds_per_s": n / (dense_round_ms * 1e-3)},
            # the reference Python CPU path (agent.py:263-275 driven as contract E2, one core), as
            # SURVEY §6 measured it in the build container: the reference does not ship to the GPU box
            "reference_python": {"value": REF_PYTHON_RATE, "unit": "agent-rounds/s", "cores": 1,
                                 "source": "SURVEY.md §6: reference election, N=100k RGG deg 15.9, 183 rounds, "
                                           "280 s on 1 core of the build container (Xeon KVM)",
                                 "gpu_over_reference_python": value / REF_PYTHON_RATE},
            "build": _lib.provenance(),
            "result_check": check,
            "elect_stats": {"rounds_launched": r.rounds_launched, "active_total": r.active_total,
                            "edges_total": r.edges_total,
                            "dense_rounds": r.dense_rounds, "changes_total": rt.changes_total},
            "alloc_stats": a.stats,
        }
    # ---- the other §8 rows, each timed once at its own scale (informational; not `value`);
    # some of them step this swarm (physics, timers): the CPU baseline below compares against a
    # host snapshot of the timed step, and runs last (its OpenMP threads would share the host
    # with the rows' launches)
    snap = host_snapshot(sw, a) if rank == 0 and args.cpu_baseline else None
    if rank == 0 and args.rows:
        out["rows"] = rows_bench(sw, dev, args)
    # ---- CPU baseline: the oracle's restatement of the same algorithm (frontier election +
    # binned allocation) on the host cores -- the whole C3 step on every thread, and a bounded
    # sample on one thread
    if rank == 0 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_step(snap, d, r, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def final_state_check(sw, r):
    """Cheap end-to-end check of the timed election's output (the full comparison against the
    oracle is tests/test_scale.py): one more E2 round over the final leaders changes nothing
    (every agent's leader is at least each neighbour's), and state == LEADER iff leader == id."""
    import torch
    from swarm_amd import _lib
    lout = torch.empty_like(sw.leader)
    changed = torch.zeros(1, dtype=torch.int64, device=sw.leader.device)
    _lib.check(_lib.lib().swarm_elect_round(_lib.ctx(), sw.n, _lib.ptr(sw.row_ptr), _lib.ptr(sw.col),
                                            _lib.ptr(sw.leader), _lib.ptr(lout), _lib.ptr(changed), _lib.stream()))
    fixed_point = int(changed.item()) == 0 and bool(torch.equal(lout, sw.leader))
    state_ok = bool(torch.equal(sw.state == _lib.LEADER, sw.leader == sw.ids))
    assert fixed_point and state_ok, ("final election state is not a fixed point", fixed_point, state_ok)
    return {"fixed_point": fixed_point, "state_consistent": state_ok, "rounds_exec": r.rounds_exec,
            "converged": r.converged, "leaders": int((sw.state == _lib.LEADER).sum())}


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def host_snapshot(sw, a):
    """Host copies of what cpu_baseline_step needs from the timed step: the graph, the swarm and
    the GPU's results (taken before the rows step the same swarm)."""
    return {"rp": sw.row_ptr.cpu().numpy().astype(np.int64), "col": sw.col.cpu().numpy(),
            "ids": sw.ids.cpu().numpy(), "x": sw.pos[:, 0].cpu().numpy(), "y": sw.pos[:, 1].cpu().numpy(),
            "caps": sw.caps.cpu().numpy().view(np.uint32), "leader": sw.leader.cpu().numpy(),
            "winner": a.winner.cpu().numpy()}


def cpu_baseline_step(h, d, r, args):
    """The C3 step on the host: the oracle's frontier election (orc_elect_frontier) and binned
    allocation (orc_allocate_binned) -- the same algorithms the GPU runs, restated in C with
    OpenMP -- over the same swarm (storage order), all host threads, measured whole (no
    extrapolation), then again on one thread (round 4's one-thread figure was extrapolated from
    the first 40 rounds and 1 000 tasks)."""
    from oracle import oracle
    threads = _threads()
    rp, col, ids, x, y, caps = h["rp"], h["col"], h["ids"], h["x"], h["y"], h["caps"]
    n = len(ids)
    oracle.set_threads(threads)
    t1 = time.perf_counter()
    lead, _, rounds, _ = oracle.elect_frontier(rp, col, ids)
    t_el = time.perf_counter() - t1
    t1 = time.perf_counter()
    al = oracle.allocate_binned(ids, x, y, caps, d["tx"], d["ty"], d["treq"], use_pow=False)
    t_al = time.perf_counter() - t1
    same = (rounds == r.rounds_exec and bool(np.array_equal(lead, h["leader"]))
            and bool(np.array_equal(al["winner"], h["winner"])))
    # one thread: the same step again, whole (~20 s on the GPU box's host)
    oracle.set_threads(1)
    t1 = time.perf_counter()
    lead1, _, rounds1, _ = oracle.elect_frontier(rp, col, ids)
    t_el1 = time.perf_counter() - t1
    t1 = time.perf_counter()
    al1 = oracle.allocate_binned(ids, x, y, caps, d["tx"], d["ty"], d["treq"], use_pow=False)
    t_al1 = time.perf_counter() - t1
    oracle.set_threads(threads)
    same1 = rounds1 == rounds and bool(np.array_equal(lead1, lead)) and bool(np.array_equal(al1["winner"], al["winner"]))
    return {"value": n * rounds / (t_el + t_al), "unit": "agent-rounds/s", "cores": threads, "kind": "port",
            "value_1core": n * rounds / (t_el1 + t_al1),
            "value_1core_kind": "measured: the whole step on one host thread",
            "elect_s": t_el, "alloc_s": t_al, "elect_s_1core": t_el1, "alloc_s_1core": t_al1,
            "same_result_as_gpu": same and same1,
            "sample": f"C oracle, the GPU's algorithms (orc_elect_frontier + orc_allocate_binned), the whole C3 step "
                      f"on the same {n}-agent swarm: election {rounds} rounds {t_el:.2f} s + {len(d['tx'])}-task "
                      f"allocation {t_al:.2f} s on {threads} threads; on 1 thread {t_el1:.1f} s + {t_al1:.1f} s "
                      f"(both measured whole, not extrapolated)"}


def _timed(fn, reps=1):
    """Wall time of fn() (device work included) in ms, best of reps, after one warm call."""
    import torch
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        res = fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        best = ms if best is None or ms < best else best
    return best, res


def _roof(alg_bytes, ms, kernel, pmc_kernel=None, note=None):
    """Row roofline: algorithmic bytes of one unit of work over its measured time (device work
    of the unit, wall-clock around a synchronised call), traffic from the committed PMC summary."""
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    if isinstance(pmc_kernel, (list, tuple)):
        t = pmc_traffic_sum(pmc_kernel)
    else:
        t = pmc_traffic(pmc_kernel) if pmc_kernel else None
    out = {"bound": "hbm", "kernel": kernel, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes": alg_bytes, "ms": ms,
           "traffic_per_dispatch": t[0] if t else None, "traffic_source": t[1] if t else None}
    if note:
        out["note"] = note
    return out


def _codec_abi_ms(f, enc, m, pk, dev):
    """Best-of-5 wall ms of swarm_codec_encode and swarm_codec_decode through the C-ABI, outputs
    preallocated; both results checked against the wrapper's."""
    import ctypes

    import torch
    from swarm_amd import _lib
    L, P = _lib.lib(), _lib.ptr
    off = torch.empty(m + 1, dtype=torch.int64, device=dev)
    st = torch.empty(m, dtype=torch.int8, device=dev)
    buf = torch.empty(pk, dtype=torch.uint8, device=dev)
    tot = ctypes.c_int64()
    with torch.cuda.device(dev):
        ms_e, _ = _timed(lambda: _lib.check(L.swarm_codec_encode(
            _lib.ctx(), m, *[P(t) for t in f], 0, P(buf), pk, P(off), P(st), ctypes.byref(tot), _lib.stream())),
            reps=5)
        assert tot.value == pk and torch.equal(buf, enc.buf) and torch.equal(off, enc.offsets)
        cols = {k: torch.empty(m, dtype=dt, device=dev) for k, dt in (
            ("status", torch.int8), ("type", torch.int64), ("sender", torch.int64), ("tick", torch.int64),
            ("a", torch.float32), ("b", torch.float32), ("task", torch.int64), ("winner", torch.int64),
            ("has_pos", torch.uint8))}
        ms_d, _ = _timed(lambda: _lib.check(L.swarm_codec_decode(
            _lib.ctx(), m, P(buf), pk, P(off), 0, *[P(cols[k]) for k in (
                "status", "type", "sender", "tick", "a", "b", "task", "winner", "has_pos")], _lib.stream())), reps=5)
        assert torch.equal(cols["type"][st == 0], f[0][st == 0])
    return ms_e, ms_d


def _enc_kernels():
    """The encode's kernels (label, PMC names): the one-pass form, or the three-launch form when
    SWARM_ENC_PASSES=3 selects it."""
    if os.environ.get("SWARM_ENC_PASSES") == "3":
        return "k_enc_tile + k_enc_base + k_enc_place", ["k_enc_tile", "k_enc_base", "k_enc_place"]
    return "k_enc_one (one pass, tile bases by decoupled look-back)", ["k_enc_one<2>"]


def rows_bench(sw, dev, args):
    """One measurement per SURVEY §8 row beside the headline (C3): C2 election, C4 auction,
    f1 physics, f2 timer FSM ticks, f3 codec -- each with its roofline figure and its CPU
    restatement (oracle/) timed on a bounded sample of the host cores.  Synthetic seeded inputs,
    resident in HBM."""
    import torch
    from swarm_amd import codec, gen
    from swarm_amd.swarm import Swarm
    cpu = bool(args.cpu_baseline)
    if cpu:
        from oracle import oracle
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        oracle.set_threads(threads)

    rows = {}
    # C2: 100k-agent RGG, election to convergence
    d2 = gen.swarm_inputs(100_000, args.seed + 1, deg=args.deg)
    s2 = Swarm(d2["ids"], d2["x"], d2["y"], device=dev).build_graph(1.0)
    ms, r2 = _timed(lambda: s2.elect(max_rounds=1 << 16), reps=3)
    rows["C2_elect_100k"] = {"ms": ms, "rounds_exec": r2.rounds_exec,
                             "agent_rounds_per_s": s2.n * r2.rounds_exec / (ms * 1e-3),
                             "roofline": _roof(float(r2.bytes_total), ms, "k_elect_dense + k_sparse_block",
                                               note="all rounds' algorithmic bytes (DESIGN §4) over the election")}
    if cpu:
        rp2 = s2.row_ptr.cpu().numpy().astype(np.int64)
        t1 = time.perf_counter()
        oracle.elect(rp2, s2.col.cpu().numpy(), s2.ids.cpu().numpy())
        cms = (time.perf_counter() - t1) * 1e3
        rows["C2_elect_100k"]["cpu_baseline"] = {
            "value": s2.n * r2.rounds_exec / (cms * 1e-3), "unit": "agent-rounds/s", "cores": threads,
            "kind": "port", "sample": f"the whole C2 election, C oracle (OpenMP x{threads}): {cms:.0f} ms"}
    # C4: 100k agents x 100k tasks auction (eps 0.1)
    d4 = gen.swarm_inputs(100_000, args.seed + 2, t=100_000)
    s4 = Swarm(d4["ids"], d4["x"], d4["y"], d4["caps"], device=dev)
    tq = [torch.as_tensor(d4[k], device=dev) for k in ("tx", "ty", "treq")]
    ms, r4 = _timed(lambda: s4.auction(*tq), reps=2)
    rows["C4_auction_100k_x_100k"] = {"ms": ms, "rounds": r4.rounds_exec, "pairs": r4.stats["n_pairs"],
                                      "bids": r4.stats["bids_total"], "us_per_round": ms * 1e3 / max(r4.rounds_exec, 1),
                                      "assigned": int((r4.assigned >= 0).sum()),
                                      "roofline": {"bound": "latency", "note": "rounds are dependent; a round is a "
                                                   "few dependent memory steps and <= 2 launches (DESIGN §4b)"}}
    if cpu:  # bounded sample: 20k x 20k, GPU timed on the same sample
        ds = gen.swarm_inputs(20_000, args.seed + 5, t=20_000)
        t1 = time.perf_counter()
        rs = oracle.auction(ds["ids"], ds["x"], ds["y"], ds["caps"], ds["tx"], ds["ty"], ds["treq"])
        cms = (time.perf_counter() - t1) * 1e3
        ss = Swarm(ds["ids"], ds["x"], ds["y"], ds["caps"], device=dev)
        tqs = [torch.as_tensor(ds[k], device=dev) for k in ("tx", "ty", "treq")]
        gms, rg = _timed(lambda: ss.auction(*tqs), reps=2)
        assert rg.rounds_exec == rs["rounds"]
        rows["C4_auction_100k_x_100k"]["cpu_baseline"] = {
            "value": cms, "unit": "ms (20k x 20k sample)", "cores": 1, "kind": "port",
            "sample": f"C oracle orc_auction on 20k agents x 20k tasks ({rs['rounds']} rounds): {cms:.0f} ms; "
                      f"the GPU on the same sample: {gms:.1f} ms"}
        del ss
    del s2, s4
    # f1: synchronous physics steps of the C3 swarm (formation behind the elected leaders,
    # 16 obstacles, separation over the sensor graph)
    g = np.random.default_rng(args.seed + 3)
    side = float(sw.pos[:, 0].max())
    obs = np.stack([g.uniform(0, side, 16), g.uniform(0, side, 16), g.uniform(0.2, 1.5, 16)], 1)
    li = sw.leader_index()
    n_fol = int((li >= 0).sum())
    steps = 5
    ms, _ = _timed(lambda: sw.physics_step(obs, leader_index=li, steps=steps), reps=1)
    n, e = sw.n, sw.n_edges
    rows["f1_physics_step"] = {"agents": n, "ms_per_step": ms / steps,
                               "agent_steps_per_s": n * steps / (ms * 1e-3),
                               "roofline": _roof(82.0 * n + 20.0 * e + 16.0 * n_fol, ms / steps,
                                                 "k_physics", "k_physics",
                                                 note="82 B/agent + 20 B/edge + 16 B per follower's leader gather")}
    if cpu:
        dp = gen.swarm_inputs(1_000_000, args.seed + 6)
        rpp, colp = oracle.rgg_csr(dp["x"], dp["y"], 1.0)
        m1 = len(dp["ids"])
        t1 = time.perf_counter()
        oracle.physics(dp["ids"], np.full(m1, 1, np.uint8), np.full(m1, -1, np.int32), dp["x"], dp["y"], np.zeros(m1),
                       np.zeros(m1), dp["x"] + 1.0, dp["y"], np.ones(m1, np.uint8), obs, rpp, colp, use_pow=False)
        cs = time.perf_counter() - t1
        rows["f1_physics_step"]["cpu_baseline"] = {
            "value": m1 / cs, "unit": "agent-steps/s", "cores": threads, "kind": "port",
            "sample": f"C oracle orc_physics (OpenMP x{threads}), 1 step of 1M agents: {cs * 1e3:.0f} ms"}
    # f3: codec, 10M messages of every type (encode: fields -> packets; decode: packets -> fields)
    m = 10_000_000
    g = np.random.default_rng(args.seed + 4)
    fields = (g.integers(1, 6, m), g.integers(0, 256, m), g.integers(0, 2**32, m), g.normal(0, 1e3, m),
              g.normal(0, 1e3, m), g.integers(0, 2**32, m), g.integers(0, 256, m))
    f = [torch.as_tensor(v, device=dev) for v in fields]
    ms_e, enc = _timed(lambda: codec.encode(*f, device=dev), reps=3)
    ms_d, _ = _timed(lambda: codec.decode(enc.buf, enc.offsets, device=dev), reps=3)
    pk = enc.total_bytes
    # the C-ABI calls themselves (swarm_codec_encode / _decode into preallocated outputs: what a caller
    # that keeps its buffers pays; the Python wrappers above add their allocations and argument checks)
    ms_ec, ms_dc = _codec_abi_ms(f, enc, m, pk, dev)
    rows["f3_codec"] = {"messages": m, "bytes": pk, "encode_ms": ms_ec, "decode_ms": ms_dc,
                        "encode_ms_python": ms_e, "decode_ms_python": ms_d,
                        "encode_msgs_per_s": m / (ms_ec * 1e-3), "decode_msgs_per_s": m / (ms_dc * 1e-3),
                        "timing": "wall clock per synchronised C-ABI call into preallocated buffers, best of 5 "
                                  "(*_ms_python: the swarm_amd.codec wrappers, which allocate their outputs)",
                        "roofline_encode": _roof(65.0 * m + 8.0 + pk, ms_ec, *_enc_kernels(),
                                                 note="compulsory bytes only: the 7 fields read once (56 B), status 1 B "
                                                      "and the int64 offsets 8 B written per message, the packet "
                                                      "bytes written; the call's final host sync included"),
                        "roofline_decode": _roof(66.0 * m + pk, ms_dc, "k_decode", "k_decode",
                                                 note="offsets 16 B + fields written 50 B per packet + packet bytes")}
    if cpu:
        mc = 200_000
        sub = [v[:mc] for v in fields]
        t1 = time.perf_counter()
        _, pks = oracle.codec_encode_py(*sub)
        t2 = time.perf_counter()
        oracle.codec_decode_py(pks)
        t3 = time.perf_counter()
        rows["f3_codec"]["cpu_baseline"] = {
            "value": mc / (t2 - t1), "unit": "encoded msgs/s", "cores": 1, "kind": "port",
            "decode_msgs_per_s": mc / (t3 - t2),
            "sample": f"struct-based restatement (the reference's own struct calls), {mc} messages: encode "
                      f"{(t2 - t1) * 1e3:.0f} ms, decode {(t3 - t2) * 1e3:.0f} ms"}
    # f2: timer FSM ticks of the C3 swarm (phase-shifted agents, a leader kill at tick 80)
    off = (np.arange(n, dtype=np.int64) * 7919 % 40).astype(np.int32)
    ticks = 200

    def run_fsm(traffic=False):
        sw.protocol_reset(tick_off=off, last_hb=-(off * 0.1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c = sw.protocol_run(ticks, kill_ticks=(80, 150), seed=5, traffic=traffic)  # hybrid: storm ticks pull
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, c
    run_fsm()
    ms, c = run_fsm()
    run_fsm(traffic=True)  # what the ticks touched (an untimed replay: the counters add atomics)
    fb = fsm_bytes(sw.fsm_traffic, n, ticks)
    rows["f2_protocol_ticks"] = {"agents": n, "ticks": ticks, "ms_per_tick": ms / ticks,
                                 "agent_ticks_per_s": n * ticks / (ms * 1e-3),
                                 "leaders_final": int(c[-1, 0]), "heartbeats": int(c[:, 3].sum()),
                                 "traffic": [int(v) for v in sw.fsm_traffic],
                                 "roofline": _roof(fb / ticks, ms / ticks, "k_tick", ["k_tick"],
                                                   note="every tick's algorithmic bytes (fsm_bytes: the sweep's 15 B "
                                                        "per agent, the mail bitmap read and cleared, each receiver's "
                                                        "fields, 5 B per row edge walked, 8 B per sender + 6 B per "
                                                        "hearer mailed), from the run's traffic counters; storm "
                                                        "ticks pulled")}
    if cpu:
        dq = gen.swarm_inputs(1_000_000, args.seed + 7)
        rpq, colq = oracle.rgg_csr(dq["x"], dq["y"], 1.0)
        m2 = len(dq["ids"])
        offq = (np.arange(m2) * 7919 % 40).astype(np.int32)
        t1 = time.perf_counter()
        oracle.protocol(dq["ids"], dq["x"], dq["y"], rpq, colq, offq, 20, last_hb=-(offq * 0.1), seed=5)
        cs = time.perf_counter() - t1
        rows["f2_protocol_ticks"]["cpu_baseline"] = {
            "value": m2 * 20 / cs, "unit": "agent-ticks/s", "cores": 1, "kind": "port",
            "sample": f"C oracle orc_protocol (1 thread), 20 ticks of 1M agents: {cs * 1e3:.0f} ms"}
    return rows


def sharded(args, rank, world, dev):
    """N > 1: one strip of a world-wide swarm per GPU -- rank k owns the contiguous ID range
    [k n, (k+1) n) (north_star: agents partitioned by ID range) -- (C3: args.agents per GPU, weak
    scaling; C5: 100M in all),
    exact sharded election (deep RCCL halo every k rounds + batched all-reduce) and allocation."""
    import torch
    import torch.distributed as dist

    from swarm_amd import gen
    from swarm_amd.dist import ShardedSwarm

    from swarm_amd.dist import Rects
    t0 = time.time()
    if args.partition == "blocks" and args.pieces > 1:
        from swarm_amd.dist import block_pieces
        d, region = block_pieces(args.agents, args.seed, world, rank, args.pieces, deg=args.deg, t=args.tasks)
    else:
        d = gen.shard_inputs(args.agents, args.seed, world, rank, deg=args.deg, t=args.tasks, layout=args.partition,
                             pieces=args.pieces)
        region = Rects(d["rects"], rank) if (args.partition == "blocks" or args.pieces > 1) else d["strip"]
    sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], region, device=dev, halo_depth=args.halo_depth)
    tx = torch.as_tensor(d["tx"], device=dev)
    ty = torch.as_tensor(d["ty"], device=dev)
    tq = torch.as_tensor(d["treq"], device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s: own={sh.n_own} ghosts={sh.n_glo + sh.n_ghi} "
        f"peers={sh.peers} E_local={sh.col.numel()} col16={sh.c16 is not None} escaped={sh.c16_escaped}")

    def step():
        r = sh.elect(check_every=128)
        a = sh.allocate(tx, ty, tq)
        return r, a

    for _ in range(args.warmup):
        r, a = step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    rounds_total = 0
    for _ in range(args.steps):
        r, a = step()
        rounds_total += r.rounds_exec
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    cdev = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    total_agents = args.agents * world
    check = sharded_state_check(sh, r)
    if args.oracle_check:
        check["union_oracle"] = union_oracle_check(args, sh, r, rank, world)
    # dominant kernel on every rank: k_sparse_block timed with HIP events over one instrumented
    # election of this rank's shard graph (owned + ghost rows) -- the kernel the sharded loop
    # launches every round, on the same graph; rank 0 reports its own, and the spread over ranks
    dom = shard_roofline(sh, dev)
    fr = torch.tensor([dom["frac"], -dom["frac"]], dtype=torch.float64, device=cdev)
    dist.all_reduce(fr, op=dist.ReduceOp.MAX)
    model = sharded_model(args, sh, rank, world, check) if args.model and getattr(sh, "_native", None) else None
    path = _shard_path(sh)
    staged = dist.get_backend() != "nccl"
    if rank == 0:
        out = {
            "metric": "agent-rounds/sec (election+allocation) at 10M agents; % of HBM roofline",
            "value": total_agents * rounds_total / elapsed,
            "unit": "agent-rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if args.config == "C5" else "weak",
            "vs_baseline": None,
            "dtype": "int32+f64",
            "data": ("synthetic (seeded RGG, SplitMix64; rank k owns the contiguous ID range [k n, (k+1) n): "
                     + ("its horizontal strip, random order inside it)" if args.partition == "strips" else
                        "its Morton-ordered block, Morton order inside it)")
                     if args.pieces == 1 else
                     "synthetic (seeded RGG, SplitMix64; the Morton-blocks swarm, its IDs cut into %d ranges dealt "
                     "round-robin: rank k owns the k-th Morton pieces of every block)" % (world * args.pieces)
                     if args.partition == "blocks" else
                     "synthetic (seeded RGG, SplitMix64; %d thin horizontal strips, thin strip j holding the ID range "
                     "[j n/%d, (j+1) n/%d) in random order, dealt round-robin: rank k owns thin strips k, k+%d, ...)"
                     % (world * args.pieces, args.pieces, args.pieces, world)),
            "config": {"workload": ("C5: %d agents sharded by ID range over %d GPUs (%d per GPU)"
                                    % (total_agents, world, args.agents) if args.config == "C5" else
                                    "C3 per GPU x %d GPUs (weak scaling): %d agents/GPU" % (world, args.agents))
                       + ", deg %g, election to convergence + %d tasks/GPU allocation" % (args.deg, args.tasks),
                       "agents_total": total_agents, "tasks_total": args.tasks * world,
                       "partition": (("contiguous ID ranges = horizontal strips (gen.shard_inputs ids='range': "
                                      "strip-major IDs, not a global random permutation)" if args.pieces == 1 else
                                      "%d ID ranges per rank = thin horizontal strips dealt round-robin (layout Rects, "
                                      "%d rectangles per rank)" % (args.pieces, args.pieces))
                                     if args.partition == "strips" else
                                     ("contiguous ID ranges of Morton IDs = Morton-ordered blocks "
                                      "(gen.shard_inputs layout='blocks')" if args.pieces == 1 else
                                      "%d ID ranges of Morton IDs per rank, dealt round-robin over the ranks "
                                      "(dist.block_pieces; layout Cells)" % args.pieces)),
                       "pieces": args.pieces,
                       "peers_rank0": list(sh.peers), "ghosts_rank0": int(sh.n_glo + sh.n_ghi),
                       "columns_rank0": ("int16 deltas" + (" (%d escaped to int32)" % sh.c16_escaped
                                                           if sh.c16_escaped else "")) if sh.c16 is not None
                       else "int32",
                       "rounds_exec": r.rounds_exec,
                       "halo_depth": sh.halo_depth,
                       "parallelism": f"strip-sharded x{world}: {path}; halo exchanged every {sh.halo_depth} "
                                      "rounds (ghosts that deep, stepped locally)",
                       # the cost model's transport constants (out["model"]): assumed, never measured
                       "transport_model_assumed": transport_assumed()},
            "alloc_stats": a[2],
            "result_check": check,
            "model": model,
            **({"rehearsal": f"REHEARSAL, not a scaling figure: {world} ranks over the host-staged "
                             f"{dist.get_backend()} group ({path}) on "
                             f"{torch.cuda.device_count()} GPU(s); every exchange goes through host memory"}
               if staged else {}),
            **({"rccl_double": rccl_double_stats()} if os.environ.get("SWARM_RCCL_PATH") else {}),
            "reference_python": {"value": REF_PYTHON_RATE, "unit": "agent-rounds/s", "cores": 1,
                                 "source": "SURVEY.md §6 (reference election on 1 core of the build container)"},
            "roofline": dict(dom, frac_max_over_ranks=float(fr[0]), frac_min_over_ranks=-float(fr[1]),
                             note="rank 0's k_sparse_block over its shard graph (owned + ghost rows), HIP events "
                                  "on libswarm's stream, one instrumented election of that graph"),
            "cpu_baseline": None,
        }
        if args.cpu_baseline:
            out["cpu_baseline"] = shard_cpu_baseline(sh, tx, ty, tq)
    # C4 on N GPUs beside the headline: 100k agents split over the ranks, 100k tasks replicated,
    # the native sharded auction (the round's bids exchanged by one all-gather per round)
    if args.rows:
        c4 = sharded_auction_row(args, rank, world, dev)
        if rank == 0:
            out["rows"] = {"C4_auction_sharded": c4}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def sharded_state_check(sh, r):
    """End-to-end check of a sharded election on this rank: one more E2 round over the owned rows
    of the shard graph changes nothing (their neighbours are owned agents or ghosts within one
    radius of the border, which hold their owners' final leaders: ShardedSwarm._check_ghosts),
    and state == LEADER iff leader == id.  Raises on failure."""
    import torch
    import torch.distributed as dist
    from swarm_amd import _lib
    L = sh.leaders[r.rounds_exec & 1]
    lout = torch.empty_like(L)
    changed = torch.zeros(1, dtype=torch.int64, device=L.device)
    # one round over every shard row (owned rows sit between the two ghost blocks); the outermost
    # ghosts may still move, so only the owned slice is compared
    own = slice(sh.own_begin, sh.own_begin + sh.n_own)
    with torch.cuda.device(L.device):
        _lib.check(_lib.lib().swarm_elect_round(_lib.ctx(), L.numel(), _lib.ptr(sh.row_ptr), _lib.ptr(sh.col),
                                                _lib.ptr(L), _lib.ptr(lout), _lib.ptr(changed), _lib.stream()))
    ok = torch.tensor([int(torch.equal(lout[own], L[own])),
                       int(torch.equal(r.state == _lib.LEADER, r.leader == sh.ids))], dtype=torch.int64,
                      device=L.device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    fixed_point, state_ok = bool(ok[0]), bool(ok[1])
    assert fixed_point and state_ok, ("sharded election state is not a fixed point", fixed_point, state_ok)
    return {"fixed_point_all_ranks": fixed_point, "state_consistent_all_ranks": state_ok,
            "rounds_exec": r.rounds_exec, "converged": r.converged}


# ---- election cost model at N GPUs.  Assumed transport latencies (the pool's boxes have one
# GPU: RCCL over xGMI was never measured here): one send/recv group to the peers, one small all-reduce
# with its host read-back, and the per-peer xGMI bandwidth a halo message sees.
ALPHA_P2P_US = 10.0
ALPHA_AR_US = 20.0
LINK_GBS = 100.0
STAMP_US_PER_MB = 0.23  # the sparse round's stamp scan: 10 MB in ~2.3 us (per-workgroup clocks)
EXCH_LAUNCH_US = 4.0    # the pack and ghost-apply kernels of an exchange


def transport_assumed():
    """The model's three transport constants, ASSUMED (no multi-GPU box in the pool: never measured)."""
    return {"alpha_p2p_us": ALPHA_P2P_US, "alpha_allreduce_us": ALPHA_AR_US, "link_GBps": LINK_GBS,
            "status": "assumed, not measured (one-GPU boxes only)"}


def batch_schedule(changes, max_batch=256):
    """The host batches of the sharded C loop (comm.hip + swarm_common.h next_round_batch) over the GLOBAL
    per-round changes: how many counter all-reduces (host round trips) the election takes."""
    hist, t, batch, n, R = [], 1, 8, 0, len(changes)
    while t <= R:
        tend = min(R, t + batch - 1)
        n += 1
        hist.extend(int(c) for c in changes[t - 1:tend])
        t = tend + 1
        b = min(batch * 2, max_batch)
        if len(hist) >= 32:
            slope = (hist[-32] - hist[-1]) / 31.0
            if slope > 0:
                rem = 1.25 * hist[-1] / slope + 4.0
                p = 8 if rem < 8 else (max_batch if rem > max_batch else int(rem + 0.5))
                b = min(b, p)
        batch = b
    return n


def fit_round_cost(local, round_ms, n_rows, n_edges):
    """Per-round device time of the frontier round on one rank as a function of its work, fitted on a
    calibration election (round_ms from HIP events, local = per-round (changes, rows, edges)): sparse
    rounds t = a + b * rows + c * edges (non-negative least squares), dense rounds t = d * (rows + edges)."""
    from scipy.optimize import nnls
    local = np.asarray(local, np.float64)
    t = np.asarray(round_ms, np.float64) * 1e3  # us
    dense = local[:, 2] < 0
    sp = ~dense
    A = np.stack([np.ones(sp.sum()), local[sp, 1], local[sp, 2]], 1)
    coef, _ = nnls(A, t[sp])
    pred = A @ coef
    d = float(np.mean(t[dense] / (n_rows + n_edges))) if dense.any() else 0.0
    return {"a_us": float(coef[0]), "b_us_per_row": float(coef[1]), "c_us_per_edge": float(coef[2]),
            "dense_us_per_row_or_edge": d, "calib_rows": int(n_rows), "calib_edges": int(n_edges),
            "sparse_rounds_fitted": int(sp.sum()), "fit_r2": float(1 - ((t[sp] - pred) ** 2).sum()
                                                                   / max(((t[sp] - t[sp].mean()) ** 2).sum(), 1e-30)),
            "fit_sum_ms": float(pred.sum() / 1e3 + t[dense].sum() / 1e3), "measured_sum_ms": float(t.sum() / 1e3)}


def election_model(per_rank, shard_rows, shard_edges, send_bytes, changes, depth, cal, merge=1):
    """Predicted time of one sharded election on N = len(per_rank) / merge GPUs: every merge consecutive
    ranks of the run taken as one (Morton blocks and strips both merge into the N/2-rank partition; their
    ghost rows are counted as owned work), per-round cost from the calibration fit, the ranks meeting at
    every halo exchange (each window costs its slowest rank), plus the exchanges (alpha + kernels + the
    largest per-peer message over one xGMI link) and the per-batch counter all-reduce."""
    R = len(changes)
    k = len(per_rank) // merge
    rows = np.zeros((k, R))
    edges = np.zeros((k, R))
    n_all = np.zeros(k)
    e_all = np.zeros(k)
    for g in range(k):
        for q in range(g * merge, (g + 1) * merge):
            loc = np.asarray(per_rank[q], np.float64)[:R]
            dense = loc[:, 2] < 0
            rows[g] += loc[:, 1]
            edges[g] += np.where(dense, shard_edges[q], loc[:, 2])
            n_all[g] += shard_rows[q]
            e_all[g] += shard_edges[q]
    dense = np.asarray(per_rank[0], np.float64)[:R, 2] < 0
    a0 = cal["a_us"] - STAMP_US_PER_MB * cal["calib_rows"] / 1e6
    t = np.where(dense[None, :], cal["dense_us_per_row_or_edge"] * (n_all[:, None] + e_all[:, None]),
                 a0 + STAMP_US_PER_MB * n_all[:, None] / 1e6 + cal["b_us_per_row"] * rows
                 + cal["c_us_per_edge"] * edges)
    if k == 1:
        return {"n_gpus": 1, "ms": float(t.sum() / 1e3), "rounds": R, "exchanges": 0, "batches": 0}
    d = max(1, int(depth))
    wins = [np.arange(i, min(i + d, R)) for i in range(0, R, d)]
    compute = sum(float(t[:, w].sum(1).max()) for w in wins)
    n_exch = R // d
    msg_us = max(send_bytes) * merge ** 0.5 / (LINK_GBS * 1e3)  # a merged region's border grows ~ sqrt
    nb = batch_schedule(changes)
    exch = n_exch * (ALPHA_P2P_US + EXCH_LAUNCH_US + msg_us)
    ar = nb * ALPHA_AR_US
    return {"n_gpus": k, "ms": (compute + exch + ar) / 1e3, "compute_ms": compute / 1e3, "exchange_ms": exch / 1e3,
            "allreduce_ms": ar / 1e3, "rounds": R, "exchanges": n_exch, "batches": nb,
            "imbalance": float(compute / max(t.sum(0).sum() / k, 1e-9))}


# The 100M-agent C5 swarm with RANDOM IDs elected on one GPU (DESIGN §7, round 5, 32-bit offsets with
# 16-bit columns): the comparison C5's Morton-ID model rates are stated against.
C5_RANDOM_IDS_1GPU = {"agent_rounds_per_s": 1.54e12, "ms": 328.0, "agents": 100_000_000,
                      "source": "profiles/r5 (DESIGN §7): swarm_elect_compact at 100M agents, random IDs"}


def annotate_model(table, agents_total, rounds):
    """Every model row gets its absolute predicted rate (agent-rounds/s of the whole job: agents_total x
    rounds over the predicted election time) and its speedup over the model's own N = 1 row, so that no
    ratio is printed without the rate it comes from."""
    t1 = next((e["ms"] for e in table if e["n_gpus"] == 1), None)
    for e in table:
        e["agent_rounds_per_s"] = agents_total * rounds / (e["ms"] * 1e-3)
        e["speedup_vs_model_n1"] = (t1 / e["ms"]) if t1 else None
    return table


def sharded_model(args, sh, rank, world, check):
    """DESIGN §6's election cost model for this run: one more (untimed, identical) sharded election records
    every rank's per-round work; rank 0 then elects its shard graph alone (the other ranks wait, the GPU is
    rank 0's) with per-round HIP events, fits the per-round cost, and predicts the election on N, N/2, ...,
    1 real GPUs (RCCL over xGMI, the ALPHA_* latencies assumed)."""
    import torch.distributed as dist
    rec = sh.elect(check_every=128, record=True)
    info = dict(local=rec.local, rows=int(sh.all_ids.numel()), edges=int(sh.col.numel()),
                send=4 * max([0] + list(sh.send_count.values())), changes=rec.changes, rounds=rec.rounds_exec)
    allinfo = [None] * world
    dist.all_gather_object(allinfo, info)
    dist.barrier()
    out = None
    if rank == 0:
        ra, loc, rms, wall = sh.elect_alone()
        sh.elect_alone(timed=False)  # warm
        _, _, _, wall_plain = sh.elect_alone(timed=False)
        cal = fit_round_cost(loc, rms, info["rows"], info["edges"])
        # the per-round events of the calibration run cost time of their own: take it out of the per-round
        # constant (the production loop records none)
        ev_us = max(0.0, (wall - wall_plain) * 1e3 / max(1, int(ra)))
        cal["event_overhead_us_per_round"] = ev_us
        cal["wall_ms_without_events"] = wall_plain
        cal["a_us_with_events"] = cal["a_us"]
        cal["a_us"] = max(0.0, cal["a_us"] - ev_us)
        per_rank = [i["local"] for i in allinfo]
        rows, edges, send = [i["rows"] for i in allinfo], [i["edges"] for i in allinfo], [i["send"] for i in allinfo]
        table, m = [], 1
        while m <= world:
            if world % m == 0:
                table.append(election_model(per_rank, rows, edges, send, rec.changes, sh.halo_depth, cal, merge=m))
            m *= 2
        annotate_model(table, args.agents * world, int(rec.rounds_exec))
        by_n = {e["n_gpus"]: e for e in table}
        out = {"calibration": dict(cal, rounds=int(ra), wall_ms=wall, shard_rows=info["rows"]),
               "assumed": dict(transport_assumed(), stamp_us_per_MB=STAMP_US_PER_MB,
                               exchange_launch_us=EXCH_LAUNCH_US),
               "table": table,
               "note": "per-round work = this run's per-rank counts (exact, timing-free); N/2 ... 1 merge adjacent "
                       "ranks; the election only (the allocation is ~0.2 ms)"}
        t1 = (check.get("union_oracle") or {}).get("t1_gpu_ms")
        out["model_agent_rounds_per_s"] = {str(e["n_gpus"]): e["agent_rounds_per_s"] for e in table}
        if args.config == "C5":  # strong scaling: the union's election on one GPU against the model at N
            if t1:
                out["t1_measured_ms"] = t1
                out["t1_measured_agent_rounds_per_s"] = args.agents * world * int(rec.rounds_exec) / (t1 * 1e-3)
                out["model_vs_measured_n1"] = by_n[1]["ms"] / t1
            out["model_speedup"] = (t1 or by_n[1]["ms"]) / by_n[world]["ms"]
            out["model_speedup_basis"] = ("the union elected on one GPU (measured)" if t1 else
                                          "the model's own N = 1") + " / the model at N"
            out["comparison"] = dict(C5_RANDOM_IDS_1GPU, note=(
                "the same 100M-agent swarm with random IDs elected on ONE GPU (measured, DESIGN §7): Morton IDs "
                "make C5's election dense-like (about half the agents change every round for ~7.4k rounds), so "
                "every predicted Morton rate above is set against this 1-GPU figure"))
        else:  # weak scaling: agent-rounds/s at N (model) against one GPU electing one rank's shard (measured)
            v1 = info["rows"] * int(ra) / (wall * 1e-3)
            vn = args.agents * world * int(rec.rounds_exec) / (by_n[world]["ms"] * 1e-3)
            out.update(model_value=vn, value_1gpu_shard_alone=v1, model_speedup=vn / v1,
                       model_speedup_basis="agent-rounds/s: the N-GPU model against rank 0's shard elected alone on "
                                           "one GPU (measured, calibration run)")
            if t1:
                out["t1_measured_ms"] = t1
                out["model_vs_measured_n1"] = by_n[1]["ms"] / t1
    dist.barrier()
    return out


def union_oracle_check(args, sh, r, rank, world):
    """The sharded election against the C oracle over the UNION swarm (rank 0's host): every rank's
    owned leaders (by agent ID), rounds_exec and every per-round GLOBAL change count must equal
    orc_elect_frontier's on the union graph (regenerated from the same seeds, cell-ordered, radius-1
    RGG by orc_rgg_csr).  The oracle is the checker here, never the measured path.  Prints progress
    while it runs (one C call per stage)."""
    import threading

    import torch
    import torch.distributed as dist
    from swarm_amd import gen
    cpu = torch.device("cpu")
    ids_t = sh.ids.to(cpu).to(torch.int64)
    lead_t = r.leader.to(cpu).to(torch.int64)
    n_t = torch.tensor([ids_t.numel()], dtype=torch.int64)
    counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    staged = dist.get_backend() != "nccl"
    if staged:
        dist.all_gather(counts, n_t)
    else:  # nccl groups carry device tensors only
        cd = [c.to(sh.device) for c in counts]
        dist.all_gather(cd, n_t.to(sh.device))
        counts = [c.cpu() for c in cd]
    mx = int(max(int(c) for c in counts))
    pad = lambda t: torch.cat([t, torch.full((mx - t.numel(),), -1, dtype=torch.int64)])  # noqa: E731
    g_ids = [torch.empty(mx, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
    g_lead = [torch.empty(mx, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
    if staged:
        dist.gather(pad(ids_t), g_ids, dst=0)
        dist.gather(pad(lead_t), g_lead, dst=0)
    else:
        gi = [torch.empty(mx, dtype=torch.int64, device=sh.device) for _ in range(world)]
        gl = [torch.empty(mx, dtype=torch.int64, device=sh.device) for _ in range(world)]
        dist.all_gather(gi, pad(ids_t).to(sh.device))
        dist.all_gather(gl, pad(lead_t).to(sh.device))
        g_ids, g_lead = ([t.cpu() for t in gi], [t.cpu() for t in gl]) if rank == 0 else (None, None)
    res = None
    if rank == 0:
        from oracle import oracle as orc
        t0 = time.time()
        ds = [gen.shard_inputs(args.agents, args.seed, world, q, deg=args.deg, layout=args.partition,
                               pieces=args.pieces if args.partition == "strips" else 1)
              for q in range(world)]
        x = np.concatenate([e["x"] for e in ds])
        y = np.concatenate([e["y"] for e in ds])
        ids = np.concatenate([e["ids"] for e in ds]).astype(np.int32)
        del ds
        perm = gen.cell_order(x, y, 1.0)  # locality for the oracle's gathers (results are order-free)
        x, y, ids = x[perm], y[perm], ids[perm]
        del perm
        box = {}

        def work():
            orc.set_threads(_threads())
            t1 = time.time()
            rp, col = orc.rgg_csr(x, y, 1.0)
            box["graph_s"] = time.time() - t1
            box["edges"] = int(rp[-1])
            t1 = time.time()
            box["elect"] = orc.elect_frontier(rp, col, ids)
            box["elect_s"] = time.time() - t1

        th = threading.Thread(target=work)
        th.start()
        while th.is_alive():
            th.join(30)
            log(f"[rank 0] union oracle running {time.time() - t0:.0f}s")
        lead, _, rounds, changes = box["elect"]
        # the union on ONE GPU (this rank's; the others wait): the N = 1 time the model's speedup divides
        t1_ms, gpu_equal = None, None
        if args.union_gpu:
            import torch
            from swarm_amd.swarm import Swarm
            su = Swarm(ids, x, y, device=sh.device).build_graph(1.0)
            ru = su.elect()
            ts = []
            for _ in range(2):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                ru = su.elect()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t1) * 1e3)
            t1_ms = min(ts)
            gpu_equal = ru.rounds_exec == int(rounds) and bool(np.array_equal(np.asarray(ru.changes), np.asarray(changes)))
            log(f"[rank 0] union on one GPU: {su.n} agents, {ru.rounds_exec} rounds, {t1_ms:.1f} ms")
            del su, ru
            torch.cuda.empty_cache()
        want = np.full(int(ids.max()) + 1, -1, np.int64)
        want[ids] = lead
        ok_lead, n_checked = True, 0
        for q in range(world):
            k = int(counts[q])
            gi, gl = g_ids[q][:k].numpy(), g_lead[q][:k].numpy()
            ok_lead &= bool(np.array_equal(want[gi], gl))
            n_checked += k
        res = {"agents_union": int(len(ids)), "edges_union": box["edges"], "agents_checked": n_checked,
               "rounds_oracle": int(rounds), "rounds_sharded": int(r.rounds_exec),
               "rounds_equal": int(rounds) == int(r.rounds_exec),
               "changes_equal": bool(np.array_equal(np.asarray(changes), r.changes)),
               "leaders_equal": ok_lead and n_checked == len(ids),
               "oracle": f"orc_elect_frontier over the {len(ids)}-agent union (orc_rgg_csr {box['graph_s']:.0f} s, "
                         f"election {box['elect_s']:.0f} s, {_threads()} threads)"}
        if t1_ms is not None:
            res.update(t1_gpu_ms=t1_ms, t1_gpu_rounds_changes_equal=gpu_equal)
        res["all_equal"] = res["rounds_equal"] and res["changes_equal"] and res["leaders_equal"]
        log(f"[rank 0] union oracle: {res}")
    dist.barrier()
    if rank == 0:
        assert res["all_equal"], ("sharded election differs from the union oracle", res)
    return res


def survey_step_bytes(r, n, e, tasks):
    """SURVEY §8(d)'s algorithmic bytes of one step: every executed election round at 12 B per
    gathered agent + 8 B per edge (a dense round gathers all n agents and E edges, + 4 B), and the
    allocation's compulsory 24 B per agent + 36 B per task."""
    return (12.0 * r.active_total + 8.0 * r.edges_total + 4.0 * r.dense_rounds + 24.0 * n + 36.0 * tasks)


def fsm_bytes(tr, n, ticks):
    """Algorithmic bytes of `ticks` protocol ticks from swarm_protocol_run_ex's traffic counters
    (DESIGN.md §4e): the sweep reads 15 B per agent per tick (alive, outbox, state, tick phase, 8-B
    timer); a mailed tick reads the 1-bit mail map and clears it; a receiver served by its single
    sender reads / writes ~36 B of fields, one that walks its row ~31 B plus 5 B per row edge
    (column, sender's outbox); a sender mails for 8 B (row offsets) + 6 B per hearer (column, the
    64-bit mail word per few hearers).  (Round 4 counted a 4-B receiver list entry written and read,
    8 B per receiver: the list was the implementation's, k_tick has none.)"""
    single, multi, edges, senders, hear, _, pulled_agents, pulled_ticks = (float(v) for v in tr)
    return (15.0 * n * ticks + (ticks - pulled_ticks) * n / 4.0 + 36.0 * single
            + 31.0 * (multi + pulled_agents) + 5.0 * edges + 8.0 * senders + 6.0 * hear)


def sparse_round_bytes(active_total, edges_total, dense_rounds, rounds_exec, n, e, launches, compact):
    """Algorithmic bytes per sparse-round launch on SURVEY §8(d)'s per-unit figure -- 12 B per
    gathered agent (row offset, own leader, leader write) + 8 B per edge (column, neighbour
    leader) -- over the executed sparse rounds, spread over every launched sparse round (as
    rocprof's per-dispatch average is).  The frontier's own bookkeeping (the n-byte stamp scan of
    every sparse round and the second row offset a lone agent reads) is reported beside it, not in
    it; so are the bytes as read with 16-bit columns (2 of the 4 column bytes)."""
    sp_active = active_total - dense_rounds * n
    sp_edges = edges_total - dense_rounds * e
    sp_rounds = rounds_exec - dense_rounds
    b8d = 12.0 * sp_active + 8.0 * sp_edges
    keep = float(n) * sp_rounds + 4.0 * sp_active
    return {"bytes_per_launch": b8d / launches,
            "bytes_source": "SURVEY 8(d): 12 B per gathered agent + 8 B per edge, sparse rounds",
            "bookkeeping_bytes_per_launch": keep / launches,
            "bookkeeping": "n-byte stamp scan per sparse round + 4 B second row offset per gathered agent",
            "columns": "int16 deltas (swarm_elect_compact)" if compact else "int32",
            "bytes_per_launch_columns_as_read": (b8d - (2.0 if compact else 0.0) * sp_edges) / launches,
            "sparse_rounds_exec": int(sp_rounds), "gathered_agents": int(sp_active), "gathered_edges": int(sp_edges)}


def shard_roofline(sh, dev):
    """k_sparse_block's algorithmic bytes per launch over its HIP-event time, from one instrumented
    single-GPU election of this rank's shard graph (ELECT_TIMED)."""
    import ctypes

    import torch
    from swarm_amd import _lib
    n = sh.all_ids.numel()
    lead = torch.empty(n, dtype=torch.int32, device=dev)
    state = torch.empty(n, dtype=torch.uint8, device=dev)
    rounds = ctypes.c_int32(0)
    st = _lib.ElectStats()
    # the shard's rows are in cell order ([ghosts-lo | owned | ghosts-hi]), so its 16-bit columns
    # (sh.c16) normally exist and the election reads them, as the sharded run does; ESCAPED columns
    # (swarm_graph_compact_escaped: multi-peer shards) are the frontier stepper's only, so this single-GPU
    # election of the shard graph reads its int32 columns then
    c16 = sh.c16 if sh.c16 is not None and not getattr(sh, "c16_escaped", 0) else None
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().swarm_elect_compact(_lib.ctx(), n, _lib.ptr(sh.row_ptr), _lib.ptr(sh.col),
                                                  _lib.ptr(c16) if c16 is not None else None,
                                                  _lib.ptr(sh.all_ids), _lib.ptr(lead), _lib.ptr(state), 1 << 16,
                                                  _lib.ELECT_FRONTIER | _lib.ELECT_TIMED, ctypes.byref(rounds), None,
                                                  ctypes.byref(st), _lib.stream()))
    torch.cuda.synchronize()
    sb = sparse_round_bytes(st.active_total, st.edges_total, st.dense_rounds, rounds.value, n,
                            int(sh.row_ptr[-1].item()), max(st.sparse_launches, 1), c16 is not None)
    bpl = sb["bytes_per_launch"]
    ms = st.sparse_ms / max(st.sparse_launches, 1)
    # the committed PMC figure is the N = 1 C3 bench's (10M agents): it stands for shards of about
    # that size only
    pmc = pmc_traffic("k_sparse_block<int, 8,") if 0.8e7 <= n <= 1.25e7 else None
    ach = bpl / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"kernel": "k_sparse_block (sparse E2 round: marked agents gather)", "bound": "hbm", "achieved": ach,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": pmc[0] if pmc else None,
            "traffic_source": pmc[1] if pmc else None, **sb, "avg_launch_ms": ms,
            "launches": int(st.sparse_launches), "shard_rows": int(n), "shard_rounds": int(rounds.value)}


def shard_cpu_baseline(sh, tx, ty, tq):
    """Rank 0's share on the host: the oracle's frontier election over its shard graph (owned +
    ghost rows, as one graph) and the binned allocation of its tasks over its owned agents, all
    host threads -- the same per-GPU work as the N = 1 line's CPU sample."""
    from oracle import oracle
    threads = _threads()
    oracle.set_threads(threads)
    rp = sh.row_ptr.cpu().numpy().astype(np.int64)
    col = sh.col.cpu().numpy()
    ids = sh.all_ids.cpu().numpy()
    t1 = time.perf_counter()
    _, _, rounds, _ = oracle.elect_frontier(rp, col, ids)
    t_el = time.perf_counter() - t1
    pos = sh.pos.cpu().numpy()
    t1 = time.perf_counter()
    oracle.allocate_binned(sh.ids.cpu().numpy(), pos[:, 0].copy(), pos[:, 1].copy(),
                           sh.caps.cpu().numpy().view(np.uint32), tx.cpu().numpy(), ty.cpu().numpy(),
                           tq.cpu().numpy(), use_pow=False)
    t_al = time.perf_counter() - t1
    n = len(ids)
    return {"value": n * rounds / (t_el + t_al), "unit": "agent-rounds/s", "cores": threads, "kind": "port",
            "elect_s": t_el, "alloc_s": t_al,
            "sample": f"rank 0's share on the host: C oracle orc_elect_frontier over its {n}-row shard graph "
                      f"({rounds} rounds, {t_el:.2f} s) + orc_allocate_binned of its {tx.numel()} tasks "
                      f"({t_al:.2f} s), {threads} threads"}


def sharded_auction_row(args, rank, world, dev):
    import torch
    import torch.distributed as dist

    from swarm_amd import gen
    from swarm_amd.dist import ShardedSwarm
    n_tot = 100_000
    ds = [gen.shard_inputs(n_tot // world, args.seed + 2, world, r, t=n_tot // world) for r in range(world)]
    d = ds[rank]
    tx, ty, tq = (np.concatenate([e[k] for e in ds]) for k in ("tx", "ty", "treq"))
    sh = ShardedSwarm(d["ids"], d["x"], d["y"], d["caps"], d["strip"], device=dev)
    sh.auction(tx, ty, tq)  # warm-up (communicator, scratch)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    r = sh.auction(tx, ty, tq)
    torch.cuda.synchronize()
    dist.barrier()
    ms = torch.tensor([(time.perf_counter() - t0) * 1e3], dtype=torch.float64,
                      device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    out = {"ms": float(ms[0]), "agents": n_tot, "tasks": len(tx), "gpus": world, "rounds": r.rounds_exec,
           "bids": int(r.bidders.sum()), "converged": r.converged,
           "path": _shard_path(sh, "auction")}
    if args.oracle_check:
        out["union_oracle"] = auction_union_check(sh, r, ds, tx, ty, tq, rank, world)
    if dist.get_backend() != "nccl":
        out["rehearsal"] = ("REHEARSAL, not a scaling figure: the ranks exchange every round through host memory "
                            f"(gloo group; {_shard_path(sh, 'auction')}); C4's rounds are latency-bound and do not shard "
                            "(DESIGN §4b)")
    return out


def _gather_rows(t, rank, world, dev):
    """Every rank's 1-D int64 tensor (any lengths) -> the list on rank 0 (None elsewhere); host-staged
    groups gather host tensors, nccl groups device ones."""
    import torch
    import torch.distributed as dist
    staged = dist.get_backend() != "nccl"
    on = (lambda v: v) if staged else (lambda v: v.to(dev))  # noqa: E731
    n_t = torch.tensor([t.numel()], dtype=torch.int64)
    counts = [on(torch.zeros(1, dtype=torch.int64)) for _ in range(world)]
    dist.all_gather(counts, on(n_t))
    counts = [int(c) for c in counts]
    mx = max(counts)
    padded = on(torch.cat([t.cpu().to(torch.int64), torch.full((mx - t.numel(),), -1, dtype=torch.int64)]))
    if staged:
        g = [torch.empty(mx, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
        dist.gather(padded, g, dst=0)
    else:
        g = [torch.empty(mx, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(g, padded)
    return [g[q][:counts[q]].cpu() for q in range(world)] if rank == 0 else None


def auction_union_check(sh, r, ds, tx, ty, tq, rank, world):
    """The sharded auction against the C oracle's auction over the UNION (rank 0's host): rounds, bidders
    per round, every task's owner (by agent ID) and price bits, every agent's assigned task.  The oracle
    is the checker here, never the measured path."""
    ids_l = _gather_rows(sh.ids, rank, world, sh.device)
    asg_l = _gather_rows(r.assigned, rank, world, sh.device)
    if rank != 0:
        return None
    from oracle import oracle as orc
    t0 = time.time()
    orc.set_threads(_threads())
    ids = np.concatenate([e["ids"] for e in ds]).astype(np.int32)
    w = orc.auction(ids, np.concatenate([e["x"] for e in ds]), np.concatenate([e["y"] for e in ds]),
                    np.concatenate([e["caps"] for e in ds]), tx, ty, tq)
    own_w = np.where(w["owner"] >= 0, ids[np.maximum(w["owner"], 0)], -1)
    by_id = dict(zip(ids.tolist(), w["assigned"].tolist()))
    got_ids = torch_cat_np(ids_l)
    got_asg = torch_cat_np(asg_l)
    rounds = int(w["rounds"])
    ok = {"rounds": r.rounds_exec == rounds,
          "bidders": r.rounds_exec == rounds and bool(np.array_equal(r.bidders, w["bidders"][:rounds])),
          "owner": bool(np.array_equal(r.owner_id.cpu().numpy(), own_w)),
          "price_bits": bool(np.array_equal(r.price.cpu().numpy().view(np.uint32),
                                            np.asarray(w["price"], np.float32).view(np.uint32))),
          "assigned": len(got_ids) == len(ids) and all(by_id[int(i)] == int(a) for i, a in zip(got_ids, got_asg))}
    return {"equal": all(ok.values()), **ok, "oracle_rounds": rounds, "oracle_s": time.time() - t0,
            "oracle": "C oracle orc_auction over the union (checker only)"}


def torch_cat_np(ts):
    return np.concatenate([t.numpy() for t in ts]) if ts else np.zeros(0, np.int64)


def _shard_path(sh, what="elect"):
    """Which halo path the sharded run took: libswarm's native C loop over RCCL or over the shared-memory
    transport (gloo rehearsal: processes of one host), or the Python stepper over torch.distributed.
    what: "elect" (swarm_elect_sharded) or "auction" (swarm_auction_sharded)."""
    import torch.distributed as dist
    if getattr(sh, "_native", None) is not None:
        if getattr(sh.backend, "comm_kind", "rccl") == "shm":
            return ("native C loop over the shared-memory transport (" +
                    ("host-staged halo + all-reduce per batch)" if what == "elect" else
                     "host-staged all-gather of each round's bids)"))
        dbl = os.environ.get("SWARM_RCCL_PATH", "")
        return (("native RCCL loop (swarm_elect_sharded: ncclSend/ncclRecv halo + ncclAllReduce per batch)"
                 if what == "elect" else
                 "native RCCL loop (swarm_auction_sharded: ncclAllGather of each round's bids + ncclAllReduce)") +
                (f" through the RCCL test double {os.path.basename(dbl)} (SWARM_RCCL_PATH)" if dbl else ""))
    return f"torch.distributed {dist.get_backend()} halo" + (" (host-staged)" if sh.halo.host_staged else "")


def rccl_double_stats():
    """What the RCCL test double (tests/rccl_double, loaded by libswarm through SWARM_RCCL_PATH) executed in
    this process: P2P groups, sends, recvs, all-reduces, all-gathers, bytes -- proof that the native loop's
    RCCL branch ran."""
    import ctypes
    L = ctypes.CDLL(os.environ["SWARM_RCCL_PATH"])
    st = (ctypes.c_longlong * 6)()
    L.rccl_double_stats(ctypes.cast(st, ctypes.c_void_p))
    return dict(zip(("groups", "sends", "recvs", "allreduce", "allgather", "bytes"), list(st)))


if __name__ == "__main__":
    main()
