"""The radius-graph builder's work bound ('Bound the graph build's work').

swarm_build_rgg scans each agent's 3 x 3 cell window and insertion-sorts its row, one thread per
agent: co-located agents would make that quadratic scan run for hours on the device (the 68M-agent
stall of round 2 was this, after a wrong gather piled 67M agents into one cell).  The builder now
prices the scan from the cell occupancies first and refuses with SWARM_ERR_RANGE above its
limits; legitimately dense but bounded inputs still build, exactly.
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw():
    import swarm_amd.swarm as swm
    from swarm_amd import _lib
    _lib.load()
    return swm


def test_colocated_million_refused_promptly(sw):
    from swarm_amd import _lib
    n = 1_200_000
    g = np.random.default_rng(1)
    x = 5.0 + g.uniform(0, 1e-3, n)  # every agent inside one cell
    y = 5.0 + g.uniform(0, 1e-3, n)
    s = sw.Swarm(np.arange(n, dtype=np.int32), x, y, device="cuda")
    t0 = time.time()
    with pytest.raises(_lib.SwarmError, match="too dense") as e:
        s.build_graph(1.0)
    assert e.value.code == _lib.ERR_RANGE
    assert time.time() - t0 < 20.0


def test_dense_cluster_builds_exactly(sw, oracle_mod):
    """3 000 agents within one cell plus a sparse background: rows of ~3 000 neighbours."""
    g = np.random.default_rng(2)
    bx, by = g.uniform(0, 300, 20_000), g.uniform(0, 300, 20_000)
    cx, cy = 150.0 + g.uniform(0, 0.5, 3_000), 150.0 + g.uniform(0, 0.5, 3_000)
    x, y = np.concatenate([bx, cx]), np.concatenate([by, cy])
    n = len(x)
    s = sw.Swarm(g.permutation(n).astype(np.int32), x, y, layout="input", device="cuda").build_graph(1.0)
    rp, col = oracle_mod.rgg_csr(x, y, 1.0)
    np.testing.assert_array_equal(s.row_ptr.cpu().numpy(), rp)
    np.testing.assert_array_equal(s.col.cpu().numpy(), col)
