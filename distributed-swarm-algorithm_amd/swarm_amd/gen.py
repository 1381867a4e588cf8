"""Deterministic synthetic swarm inputs.

Everything here is host-side input *creation* (numpy, SplitMix64-seeded) and
is never inside a timed region.  The same seeds give the same bytes on every
host, so golden fixtures only need to record (seed, n, deg, ...).

Layout conventions shared with the C-ABI (include/swarm.h):
  * agents are addressed by a storage index i in [0, n); ``ids[i]`` is the
    agent's protocol ID (``SwarmAgent.agent_id``, agent.py:26), int32;
  * positions are float64 ``x[i], y[i]`` (agent.py:47 ``self.position``);
  * capabilities are a uint32 bitmask, bit k = capability name ``CAP_NAMES[k]``
    (agent.py:52 ``self.capabilities`` list);
  * tasks: float64 ``tx, ty`` (agent.py:41 ``task['pos']``) and int8 ``treq``,
    -1 = no ``'required_cap'`` key (agent.py:344), else the capability bit.
"""
from __future__ import annotations

import math

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
CAP_NAMES = ("extinguisher", "sonar", "camera", "gripper")

# stream tags (one independent SplitMix64 stream per quantity)
TAG_X, TAG_Y, TAG_ID, TAG_CAP, TAG_TX, TAG_TY, TAG_TREQ, TAG_TREQ2 = range(1, 9)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def stream(seed: int, tag: int, n: int) -> np.ndarray:
    """n SplitMix64 outputs of stream (seed, tag) as uint64."""
    with np.errstate(over="ignore"):
        base = _mix(np.array([(seed * 0x100000001B3 + tag * 0x51ED27) & 0xFFFFFFFFFFFFFFFF],
                             dtype=np.uint64))[0]
        i = np.arange(1, n + 1, dtype=np.uint64)
        return _mix(base + i * GOLDEN)


def uniform(seed: int, tag: int, n: int) -> np.ndarray:
    """float64 uniform in [0, 1) from the top 53 bits."""
    return (stream(seed, tag, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def side_length(n: int, deg: float = 16.0, radius: float = 1.0) -> float:
    """Square side L with expected degree ``deg`` for a radius-r RGG: n*pi*r^2/L^2 = deg."""
    return math.sqrt(max(n, 1) * math.pi * radius * radius / deg)


def positions(n: int, seed: int, side: float) -> tuple[np.ndarray, np.ndarray]:
    return uniform(seed, TAG_X, n) * side, uniform(seed, TAG_Y, n) * side


def random_ids(n: int, seed: int) -> np.ndarray:
    """Seeded random permutation of 0..n-1 (int32): argsort of SplitMix64 keys."""
    return np.argsort(stream(seed, TAG_ID, n), kind="stable").astype(np.int32)


def feistel_ids(index: np.ndarray, total: int, seed: int, rounds: int = 4) -> np.ndarray:
    """Seeded pseudo-random bijection of [0, total) evaluated at `index` (int64 array):
    a balanced Feistel network on the next even power of two, with cycle walking.  Lets every
    shard draw globally unique random IDs without materialising a global permutation."""
    bits = max(2, int(total - 1).bit_length())
    bits += bits & 1
    half = bits // 2
    mask = np.uint64((1 << half) - 1)
    keys = [_mix(np.array([(seed * 0x2545F4914F6CDD1D + 977 * (k + 1)) & 0xFFFFFFFFFFFFFFFF],
                          dtype=np.uint64))[0] for k in range(rounds)]

    def perm(v):
        lo = v & mask
        hi = (v >> np.uint64(half)) & mask
        with np.errstate(over="ignore"):
            for k in keys:
                f = _mix(lo ^ k) & mask
                lo, hi = hi ^ f, lo
        return (hi << np.uint64(half)) | lo

    v = np.asarray(index, dtype=np.uint64).copy()
    out = perm(v)
    bad = out >= np.uint64(total)
    while bad.any():  # cycle walking: stays inside [0, total), still a bijection
        out[bad] = perm(out[bad])
        bad = out >= np.uint64(total)
    return out.astype(np.int64)


def _morton2(bx: np.ndarray, by: np.ndarray) -> np.ndarray:
    """Interleaved bits of small non-negative integers (x in the even bits)."""
    code = np.zeros(len(bx), np.int64)
    for b in range(16):
        code |= ((np.asarray(bx, np.int64) >> b) & 1) << (2 * b)
        code |= ((np.asarray(by, np.int64) >> b) & 1) << (2 * b + 1)
    return code


def block_rects(world: int, side: float) -> np.ndarray:
    """`world` equal rectangles tiling the square [0, side)^2, a gx x gy grid (gx the largest divisor of
    world <= sqrt(world)), numbered along a Morton curve over the block grid: rank k's block is row k,
    [x0, x1, y0, y1].  With Morton IDs inside each block (shard_inputs(layout="blocks")), the contiguous
    ID ranges of equal size ARE these blocks -- SURVEY §8e's C5 partition."""
    gx = max(d for d in range(1, int(math.isqrt(world)) + 1) if world % d == 0)
    gy = world // gx
    bx, by = np.meshgrid(np.arange(gx), np.arange(gy), indexing="xy")
    bx, by = bx.ravel(), by.ravel()
    o = np.argsort(_morton2(bx, by), kind="stable")
    bx, by = bx[o], by[o]
    w, h = side / gx, side / gy
    return np.stack([bx * w, (bx + 1) * w, by * h, (by + 1) * h], 1).astype(np.float64)


def shard_inputs(n_per: int, seed: int, world: int, rank: int, deg: float = 16.0, t: int = 0,
                 ids: str = "range", layout: str = "strips", pieces: int = 1):
    """Rank `rank`'s part of a world-wide synthetic swarm of n_per*world agents: uniform
    positions inside the rank's region of the global square, tasks inside the region.
    layout="strips": horizontal strips.  ids="range" (north_star: agents partitioned by ID range): rank k
    owns exactly the contiguous ID range [k n_per, (k+1) n_per), in a seeded random order inside its
    strip -- the ID range IS the strip.  ids="global": one global seeded bijection (IDs unrelated to ranks).
    layout="blocks" (SURVEY §8e's C5 shape): rank k's Morton-ordered block (block_rects), IDs
    k n_per + the Morton rank of the agent inside its block -- Morton IDs whose contiguous ranges are
    the blocks, each with up to 8 neighbouring ranks."""
    total = n_per * world
    side = side_length(total, deg)
    h = side / world
    sseed = seed * 1000003 + rank
    if layout == "blocks":
        rects = block_rects(world, side)
        x0, x1, y0, y1 = rects[rank]
        x = x0 + uniform(sseed, TAG_X, n_per) * (x1 - x0)
        y = y0 + uniform(sseed, TAG_Y, n_per) * (y1 - y0)
        loc = morton_rank(x - x0, y - y0, max(x1 - x0, y1 - y0))
        out = dict(n=n_per, total=total, seed=seed, deg=deg, side=side, rects=rects, rect=tuple(rects[rank]),
                   strip=(y0, y1), x=x, y=y, ids=(loc.astype(np.int64) + np.int64(rank) * n_per).astype(np.int32),
                   id_range=(rank * n_per, (rank + 1) * n_per), caps=capabilities(n_per, sseed))
        if t:
            tx, ty, treq = tasks(t, sseed, side)
            out["tx"], out["ty"], out["treq"] = x0 + tx / side * (x1 - x0), y0 + ty / side * (y1 - y0), treq
        return out
    if layout != "strips":
        raise ValueError(f"unknown layout {layout!r}")
    if pieces > 1:
        return _strip_pieces(n_per, seed, world, rank, deg, t, pieces, side, sseed)
    x = uniform(sseed, TAG_X, n_per) * side
    y = rank * h + uniform(sseed, TAG_Y, n_per) * h
    if ids == "range":
        loc = feistel_ids(np.arange(n_per, dtype=np.int64), n_per, seed * 7919 + rank)
        idv = (loc + np.int64(rank) * n_per).astype(np.int32)
    elif ids == "global":
        gidx = np.arange(n_per, dtype=np.int64) + np.int64(rank) * n_per
        idv = feistel_ids(gidx, total, seed).astype(np.int32)
    else:
        raise ValueError(f"unknown ids {ids!r}")
    out = dict(n=n_per, total=total, seed=seed, deg=deg, side=side, strip=(rank * h, (rank + 1) * h),
               x=x, y=y, ids=idv, id_range=(rank * n_per, (rank + 1) * n_per), caps=capabilities(n_per, sseed))
    if t:
        tx, ty, treq = tasks(t, sseed, side)
        out["tx"], out["ty"], out["treq"] = tx, rank * h + ty / side * h, treq
    return out


def _strip_pieces(n_per, seed, world, rank, deg, t, k, side, sseed):
    """shard_inputs(layout="strips", pieces=k): the square cut into world * k thin horizontal strips of
    n_per / k agents each, thin strip j holding the ID range [j n_per / k, (j + 1) n_per / k) in a seeded
    random order (strip-major IDs at the thin strips' grain), dealt round-robin: rank q owns the thin
    strips q, q + world, ... -- so every rank has agents at every height, and the election's front, which
    starts from the top strip's maximum, loads all ranks alike.  Each rank's region is its k
    thin strips (rects: world x k x 4)."""
    if n_per % k:
        raise ValueError("pieces must divide the agents per rank")
    m, S = n_per // k, world * k
    hs = side / S
    xs, ys, idv = [], [], []
    for i in range(k):
        j = i * world + rank
        js = seed * 1000003 + 7_777_777 + j
        xs.append(uniform(js, TAG_X, m) * side)
        ys.append(j * hs + uniform(js, TAG_Y, m) * hs)
        idv.append(feistel_ids(np.arange(m, dtype=np.int64), m, seed * 7919 + 104_729 + j) + np.int64(j) * m)
    rects = np.array([[[0.0, side, (i * world + q) * hs, (i * world + q + 1) * hs] for i in range(k)]
                      for q in range(world)], np.float64)
    out = dict(n=n_per, total=n_per * world, seed=seed, deg=deg, side=side, rects=rects, pieces=k,
               strip=(float(rects[rank, :, 2].min()), float(rects[rank, :, 3].max())),
               x=np.concatenate(xs), y=np.concatenate(ys), ids=np.concatenate(idv).astype(np.int32),
               id_range=None, caps=capabilities(n_per, sseed))
    if t:
        tx, ty, treq = tasks(t, sseed, side)
        f = ty / side * k  # task height -> one of the rank's thin strips, same relative place inside it
        i = np.minimum(f.astype(np.int64), k - 1)
        out["tx"], out["ty"], out["treq"] = tx, (i * world + rank + (f - i)) * hs, treq
    return out


def strip_ids(y: np.ndarray, world: int, seed: int) -> np.ndarray:
    """IDs 0..n-1 for one global swarm such that the `world` contiguous ID ranges of equal size
    are the `world` horizontal strips of equal agent count (y-quantile cuts, as
    dist.strip_cuts): strip k holds IDs [sum of the strips below, + its count), in a seeded
    random order.  dist.partition(by="id") then cuts exactly the strips ("agents are
    partitioned by ID range"; strip-major ranks instead of Morton ranks keep each range's
    neighbours to the two adjacent ranges -- the chain halo of dist.py)."""
    y = np.asarray(y, np.float64)
    n = len(y)
    if world <= 1 or n == 0:
        who = np.zeros(n, np.int64)
    else:
        ks = [(k * n) // world for k in range(1, world)]
        cuts = np.partition(y, ks)[ks]
        who = np.searchsorted(cuts, y, side="right")
    out = np.empty(n, np.int64)
    base = 0
    for k in range(max(world, 1)):
        idx = np.nonzero(who == k)[0]
        out[idx] = base + feistel_ids(np.arange(len(idx), dtype=np.int64), max(len(idx), 1), seed * 31 + k)
        base += len(idx)
    return out.astype(np.int32)


def capabilities(n: int, seed: int, ncaps: int = 4, p: float = 0.5) -> np.ndarray:
    """uint32 bitmask, each of ``ncaps`` bits set independently with probability p."""
    out = np.zeros(n, dtype=np.uint32)
    for k in range(ncaps):
        u = uniform(seed, TAG_CAP + 16 * (k + 1), n)
        out |= (u < p).astype(np.uint32) << np.uint32(k)
    return out


def tasks(t: int, seed: int, side: float, ncaps: int = 4, p_req: float = 0.7):
    """Task positions uniform in [0, side)^2; required cap present w.p. p_req."""
    tx = uniform(seed, TAG_TX, t) * side
    ty = uniform(seed, TAG_TY, t) * side
    has = uniform(seed, TAG_TREQ, t) < p_req
    which = np.minimum((uniform(seed, TAG_TREQ2, t) * ncaps).astype(np.int64), ncaps - 1)
    treq = np.where(has, which, -1).astype(np.int8)
    return tx, ty, treq


def morton_rank(x: np.ndarray, y: np.ndarray, side: float, bits: int = 16) -> np.ndarray:
    """Rank of each point along a Morton (Z-order) curve: C5's spatially compact IDs."""
    q = np.uint64((1 << bits) - 1)
    s = ((1 << bits) - 1) / max(side, 1e-300)
    qx = np.minimum((x * s).astype(np.uint64), q)
    qy = np.minimum((y * s).astype(np.uint64), q)

    def spread(v):
        v = v & np.uint64(0xFFFFFFFF)
        v = (v | (v << np.uint64(16))) & np.uint64(0x0000FFFF0000FFFF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x00FF00FF00FF00FF)
        v = (v | (v << np.uint64(4))) & np.uint64(0x0F0F0F0F0F0F0F0F)
        v = (v | (v << np.uint64(2))) & np.uint64(0x3333333333333333)
        v = (v | (v << np.uint64(1))) & np.uint64(0x5555555555555555)
        return v

    code = spread(qx) | (spread(qy) << np.uint64(1))
    rank = np.empty(len(x), dtype=np.int32)
    rank[np.argsort(code, kind="stable")] = np.arange(len(x), dtype=np.int32)
    return rank


def cell_order(x: np.ndarray, y: np.ndarray, cell: float = 1.0) -> np.ndarray:
    """Storage permutation that groups agents by row-major grid cell (stable)."""
    cx = np.floor(x / cell).astype(np.int64)
    cy = np.floor(y / cell).astype(np.int64)
    ncx = int(cx.max()) + 1 if len(x) else 1
    return np.argsort(cy * ncx + cx, kind="stable")


def rgg_csr(x: np.ndarray, y: np.ndarray, radius: float = 1.0, chunk: int = 1 << 20):
    """Random geometric graph as CSR over storage indices (host numpy; tests/fixtures only).

    Edge i~j (i != j) iff (xi-xj)*(xi-xj) + (yi-yj)*(yi-yj) <= radius*radius in float64
    (plain products, no FMA).  Rows are sorted ascending.  Returns (row_ptr int64, col int32).
    """
    n = len(x)
    if n == 0:
        return np.zeros(1, np.int64), np.zeros(0, np.int32)
    r2 = radius * radius
    cx = np.floor(x / radius).astype(np.int64)
    cy = np.floor(y / radius).astype(np.int64)
    ncx = int(cx.max()) + 3
    key = (cy + 1) * ncx + (cx + 1)
    order = np.argsort(key, kind="stable")
    skey = key[order]
    srcs, dsts = [], []
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        ii = np.arange(lo, hi, dtype=np.int64)
        for oy in (-1, 0, 1):
            for ox in (-1, 0, 1):
                nk = key[ii] + oy * ncx + ox
                a = np.searchsorted(skey, nk, "left")
                b = np.searchsorted(skey, nk, "right")
                cnt = b - a
                rep_i = np.repeat(ii, cnt)
                offs = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
                jj = order[np.repeat(a, cnt) + offs]
                dx = x[rep_i] - x[jj]
                dy = y[rep_i] - y[jj]
                keep = (dx * dx + dy * dy <= r2) & (rep_i != jj)
                srcs.append(rep_i[keep])
                dsts.append(jj[keep])
    src = np.concatenate(srcs)
    dst = np.concatenate(dsts)
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    row_ptr = np.zeros(n + 1, np.int64)
    np.add.at(row_ptr, src + 1, 1)
    row_ptr = np.cumsum(row_ptr)
    return row_ptr, dst.astype(np.int32)


def permute_csr(row_ptr, col, perm):
    """Relabel a CSR so new index k is old index perm[k]; rows re-sorted ascending."""
    n = len(perm)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    deg = np.diff(row_ptr)[perm]
    new_ptr = np.zeros(n + 1, np.int64)
    new_ptr[1:] = np.cumsum(deg)
    src = np.repeat(np.arange(n), deg)
    flat = np.repeat(row_ptr[perm] - new_ptr[:-1], deg) + np.arange(new_ptr[-1])
    new_col = inv[col[flat]]
    o = np.lexsort((new_col, src))
    return new_ptr, new_col[o].astype(np.int32)


def swarm_inputs(n: int, seed: int, deg: float = 16.0, t: int = 0, ids: str = "random"):
    """One synthetic swarm: positions, ids, caps, and optionally t tasks."""
    side = side_length(n, deg)
    x, y = positions(n, seed, side)
    if ids == "random":
        aid = random_ids(n, seed)
    elif ids == "morton":
        aid = morton_rank(x, y, side)
    else:
        aid = np.arange(n, dtype=np.int32)
    out = dict(n=n, seed=seed, deg=deg, side=side, x=x, y=y, ids=aid,
               caps=capabilities(n, seed))
    if t:
        out["tx"], out["ty"], out["treq"] = tasks(t, seed, side)
    return out
