"""Partition layouts of the sharded swarm (swarm_amd/dist.py): which of a rank's agents every peer needs.
Host logic only.  Exactness needs every agent within the halo width of a peer's agents (or region) in
that peer's set -- a superset is allowed; the tests check the superset property by brute force."""
import numpy as np

from swarm_amd import gen
from swarm_amd.dist import Cells, Rects, StripChain, _dilate, partition


def test_dilate_is_a_chebyshev_box():
    g = np.random.default_rng(1)
    occ = g.uniform(size=(23, 31)) < 0.05
    for k in (0, 1, 3):
        want = np.zeros_like(occ)
        for y, x in zip(*np.nonzero(occ)):
            want[max(0, y - k):y + k + 1, max(0, x - k):x + k + 1] = True
        np.testing.assert_array_equal(_dilate(occ, k), want)


def _brute_need(px, py, qx, qy, width):
    """Points p within `width` of any q (brute force)."""
    d2 = (px[:, None] - qx[None, :]) ** 2 + (py[:, None] - qy[None, :]) ** 2
    return (d2 <= width * width).any(1)


def test_cells_targets_cover_every_agent_within_the_width():
    d = gen.swarm_inputs(3000, 7)
    world = 3
    who = np.random.default_rng(2).integers(0, world, 3000)  # any ownership at all
    for rank in range(world):
        lay = Cells(d["x"], d["y"], who, rank, world, 1.0)
        mine = who == rank
        for width in (1.0, 2.5):
            t = lay.targets(d["x"][mine], d["y"][mine], width)
            for p in range(world):
                if p == rank:
                    continue
                need = _brute_need(d["x"][mine], d["y"][mine], d["x"][who == p], d["y"][who == p], width)
                got = t.get(p, np.zeros(mine.sum(), bool))
                assert not (need & ~got).any()


def test_morton_blocks_are_the_id_ranges_and_rects_cover_the_halo():
    world, n_per = 8, 2000
    ds = [gen.shard_inputs(n_per, 3, world, r, layout="blocks") for r in range(world)]
    rects = ds[0]["rects"]
    side = ds[0]["side"]
    assert np.isclose((rects[:, 1] - rects[:, 0]) @ (rects[:, 3] - rects[:, 2]), side * side)  # a tiling
    ids = np.concatenate([e["ids"] for e in ds])
    assert np.array_equal(np.sort(ids), np.arange(world * n_per))
    for r, e in enumerate(ds):  # rank r owns exactly the ID range [r n, (r+1) n), inside its block
        assert np.array_equal(np.sort(e["ids"]), np.arange(r * n_per, (r + 1) * n_per))
        x0, x1, y0, y1 = rects[r]
        assert ((e["x"] >= x0) & (e["x"] < x1) & (e["y"] >= y0) & (e["y"] < y1)).all()
    peers = []
    for r, e in enumerate(ds):
        t = Rects(rects, r).targets(e["x"], e["y"], 4.0)
        peers.append(sorted(t))
        for p in range(world):
            if p == r:
                continue
            need = _brute_need(e["x"], e["y"], ds[p]["x"], ds[p]["y"], 4.0)
            got = t.get(p, np.zeros(n_per, bool))
            assert not (need & ~got).any()
    assert max(len(p) for p in peers) >= 3  # compact blocks: more than the two neighbours of a strip


def test_strip_chain_peers_are_the_neighbouring_strips():
    lay = StripChain((10.0, 20.0), 1, 3)
    y = np.array([10.5, 15.0, 19.5])
    t = lay.targets(np.zeros(3), y, 1.0)
    assert sorted(t) == [0, 2]
    assert t[0].tolist() == [True, False, False] and t[2].tolist() == [False, False, True]
    assert lay.depth_cap(1.0) == 9


def test_partition_by_id_with_morton_ids_is_cells():
    d = gen.swarm_inputs(5000, 11, t=200, ids="morton")
    parts = [partition(d["x"], d["y"], 4, r, tx=d["tx"], ty=d["ty"], by="id", ids=d["ids"]) for r in range(4)]
    assert all(type(p.layout).__name__ == "Cells" for p in parts)
    assert np.array_equal(np.sort(np.concatenate([p.agents for p in parts])), np.arange(5000))
    # Morton ranges are compact: each part's agents span about a quarter of the square, not all of it
    for p in parts:
        xs, ys = d["x"][p.agents], d["y"][p.agents]
        assert (xs.max() - xs.min()) * (ys.max() - ys.min()) < 0.6 * d["side"] ** 2
