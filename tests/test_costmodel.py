"""The election cost model of DESIGN §6 (bench.py: fit_round_cost, election_model, batch_schedule) on
synthetic per-round counts: host logic only, no GPU."""
import numpy as np

import bench


def _counts(world, R, seed=0, dense=9):
    g = np.random.default_rng(seed)
    out = []
    for q in range(world):
        loc = np.zeros((R, 3), np.int64)
        loc[:, 1] = g.integers(0, 20_000, R)
        loc[:, 2] = loc[:, 1] * 16
        loc[:dense, 1] = 1000
        loc[:dense, 2] = -1
        out.append(loc)
    return out


def test_fit_recovers_a_linear_cost():
    R = 400
    loc = _counts(1, R)[0]
    rows, edges = 1000, 16_000
    t_us = np.where(loc[:, 2] < 0, 0.01 * (rows + edges), 6.0 + 0.002 * loc[:, 1] + 0.0001 * loc[:, 2])
    cal = bench.fit_round_cost(loc, t_us / 1e3, rows, edges)
    assert abs(cal["a_us"] - 6.0) < 1e-6 and cal["fit_r2"] > 0.999
    assert abs(cal["dense_us_per_row_or_edge"] - 0.01) < 1e-9
    pred = cal["b_us_per_row"] * 10_000 + cal["c_us_per_edge"] * 160_000
    assert abs(pred - (0.002 * 10_000 + 0.0001 * 160_000)) < 1e-6  # rows and edges are collinear here


def test_model_merges_and_synchronises():
    world, R = 8, 600
    per = _counts(world, R, seed=3)
    changes = np.maximum(1, np.linspace(10_000, 1, R)).astype(np.int64)
    changes[-1] = 0
    cal = {"a_us": 7.0, "b_us_per_row": 0.002, "c_us_per_edge": 0.0, "dense_us_per_row_or_edge": 0.001,
           "calib_rows": 1_000_000, "calib_edges": 16_000_000}
    rows, edges, send = [1_000_000] * world, [16_000_000] * world, [400_000] * world
    t = {m: bench.election_model(per, rows, edges, send, changes, 16, cal, merge=m) for m in (1, 2, 4, 8)}
    assert [t[m]["n_gpus"] for m in (1, 2, 4, 8)] == [8, 4, 2, 1]
    assert t[8]["exchanges"] == 0 and t[1]["exchanges"] == R // 16
    # more GPUs: less compute per GPU, but never below the per-round floor
    assert t[1]["compute_ms"] < t[2]["compute_ms"] < t[4]["compute_ms"] < t[8]["ms"]
    assert t[1]["compute_ms"] * 1e3 >= R * (7.0 - bench.STAMP_US_PER_MB + bench.STAMP_US_PER_MB)
    assert t[1]["imbalance"] >= 1.0
    assert t[1]["batches"] == bench.batch_schedule(changes) > 0


def test_batch_schedule_grows_then_caps():
    flat = np.full(5000, 1000, np.int64)
    n = bench.batch_schedule(flat)
    # 8, 16, ..., 256 then 256 per batch
    assert n == 6 + int(np.ceil((5000 - (8 + 16 + 32 + 64 + 128 + 256)) / 256))


def test_model_rows_carry_absolute_rates_and_assumed_constants():
    """Every model row prints its predicted agent-rounds/s beside its speedup, and the line carries the
    transport constants marked assumed."""
    world, R = 8, 600
    per = _counts(world, R, seed=5)
    changes = np.maximum(1, np.linspace(10_000, 1, R)).astype(np.int64)
    changes[-1] = 0
    cal = {"a_us": 7.0, "b_us_per_row": 0.002, "c_us_per_edge": 0.0, "dense_us_per_row_or_edge": 0.001,
           "calib_rows": 1_000_000, "calib_edges": 16_000_000}
    rows, edges, send = [1_000_000] * world, [16_000_000] * world, [400_000] * world
    table = [bench.election_model(per, rows, edges, send, changes, 16, cal, merge=m) for m in (1, 2, 4, 8)]
    bench.annotate_model(table, 8 * 1_000_000, R)
    by_n = {e["n_gpus"]: e for e in table}
    assert set(by_n) == {1, 2, 4, 8}
    for k, e in by_n.items():
        assert e["agent_rounds_per_s"] == 8e6 * R / (e["ms"] * 1e-3)
        assert abs(e["speedup_vs_model_n1"] - by_n[1]["ms"] / e["ms"]) < 1e-12
    a = bench.transport_assumed()
    assert {"alpha_p2p_us", "alpha_allreduce_us", "link_GBps"} <= set(a) and "assumed" in a["status"]
    assert bench.C5_RANDOM_IDS_1GPU["agent_rounds_per_s"] == 1.54e12
