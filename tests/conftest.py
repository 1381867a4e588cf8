import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-swarm-algorithm_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


def golden_index():
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)["fixtures"]


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(kind_prefix):
    return sorted(k for k in golden_index() if k.startswith(kind_prefix))


RCCL_DOUBLE_DIR = os.path.join(ROOT, "tests", "rccl_double")
RCCL_DOUBLE = os.path.join(RCCL_DOUBLE_DIR, "librccl_double.so")


def build_rccl_double():
    """tests/rccl_double/librccl_double.so (make: rebuilt only when its source changed; g++, host code)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", RCCL_DOUBLE_DIR], check=True, capture_output=True)
    return RCCL_DOUBLE


@pytest.fixture(scope="session")
def rccl_double():
    """Path of the RCCL test double (SWARM_RCCL_PATH): libswarm's RCCL branch with peers on one GPU."""
    return build_rccl_double()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle
