"""bench.py's host-side contract (no GPU): default flags give the N=1 run the driver expects, and
the roofline `traffic` of the headline names the 2 048-agent-chunk sparse kernel's PMC entry (the
512-agent-chunk variant, used by small swarms only, shares the name prefix)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.agents, a.tasks, a.elect_mode) == (1, 10_000_000, 10_000, "frontier")
    assert a.steps >= 1 and a.warmup >= 0


def test_headline_pmc_entry():
    latest = open(os.path.join(ROOT, "profiles", "LATEST")).read().strip()
    path = os.path.join(ROOT, "profiles", latest, "pmc_traffic.json")
    d = json.load(open(path))
    keys = [k for k in d if k.startswith("k_sparse_block<int, 8,")]
    assert len(keys) == 1
    got = bench.pmc_traffic("k_sparse_block<int, 8,")
    assert got is not None
    assert got[0] == d[keys[0]]["hbm_bytes_per_dispatch"]
    assert latest in got[1]


def test_c5_defaults(monkeypatch):
    """C5: 100M agents split over the ranks, the union-oracle check on by default (a rehearsal or a real
    N-GPU run prints whether every rank's result equals the oracle's), the other rows off; C3 leaves the
    (slow) union check off."""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--config", "C5"])
    monkeypatch.setenv("WORLD_SIZE", "8")
    a = bench.parse()
    assert a.agents == 12_500_000 and a.oracle_check == 1 and a.rows == 0 and a.model == 1
    assert a.partition == "strips"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--config", "C5", "--partition", "blocks"])
    assert bench.parse().partition == "blocks"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    a = bench.parse()
    assert a.agents == 10_000_000 and a.oracle_check == 0 and a.rows == 1
