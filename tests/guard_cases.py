"""Agent/task pairs that sit in the libm guard band, constructed on THIS host.

The reference squares with libm pow (CPython float ** 2 -> pow(|x|, 2.0), agent.py:340); the GPU
squares with x*x.  The two differ by an ulp on ~0.1 % of inputs, and for a pair sitting right at
the claim threshold (d ~ 4, agent.py:297) or at an f32 rounding midpoint of U (the claim payload,
agent.py:302) that ulp flips the claim decision or the claim value.  find_flips() searches task
positions ulp by ulp around such points and keeps the pairs where the two arithmetics disagree,
evaluated exactly as the device and the reference do (dx = ax - tx in float64), with this host's
libm -- so the cases are valid for whatever libm the GPU box's host has.
"""
import math

import numpy as np


def _u_mul(ax, ay, tx, ty):
    dx, dy = ax - tx, ay - ty
    return 100.0 / (1.0 + np.sqrt(dx * dx + dy * dy))


def _u_pow1(ax, ay, tx, ty):
    dx, dy = ax - tx, ay - ty
    return 100.0 / (1.0 + math.sqrt(math.pow(abs(dx), 2.0) + math.pow(abs(dy), 2.0)))


def find_flips(seed=0, want=6, max_trials=20000, span=25):
    """Returns [(ax, ay, tx, ty, kind)]: pairs whose claim decision ('decision') or f32 claim value
    ('f32') differs between pow and x*x arithmetic on this host.  Pair k's task sits at (~0, 10 k)
    (slots 10 apart: no agent reaches another slot's task).  The x coordinates stay small (ulps
    <= 9e-16), so stepping the agent one ulp in x moves dx*dx + dy*dy by a few of its own ulps --
    with coordinates in the hundreds a step jumps hundreds of them and the few s values where the
    two arithmetics round apart are never hit."""
    rng = np.random.default_rng(seed)
    out = {"decision": [], "f32": []}
    steps = np.arange(-span, span + 1, dtype=np.float64)
    slot = 0
    for trial in range(max_trials):
        if all(len(v) >= want for v in out.values()):
            break
        kind = "decision" if len(out["decision"]) <= len(out["f32"]) else "f32"
        k = (slot + 1) // 2 * (1 if slot % 2 else -1)  # 0, 1, -1, 2, -2, ...
        tx, ty = rng.uniform(-0.25, 0.25), 10.0 * k + rng.uniform(-0.25, 0.25)
        if kind == "decision":
            target = 20.0
        else:
            lo = np.float32(rng.uniform(21.0, 99.0))
            target = (float(lo) + float(np.nextafter(lo, np.float32(np.inf)))) / 2.0  # an f32 midpoint
        d = 100.0 / target - 1.0
        th = rng.uniform(0, 2 * math.pi)
        ax0, ay0 = tx + d * math.cos(th), ty + d * math.sin(th)
        ax = ax0 + steps[:, None] * np.spacing(ax0)
        ay = ay0 + steps[None, :] * np.spacing(ay0)
        ax, ay = np.broadcast_arrays(ax, ay)
        um = _u_mul(ax, ay, tx, ty)
        near = np.argwhere(np.abs(um - target) <= 6 * np.spacing(target))
        for i, j in near:
            a, b = float(ax[i, j]), float(ay[i, j])
            m, p = float(um[i, j]), _u_pow1(a, b, tx, ty)
            if kind == "decision":
                hit = (m > 20.0) != (p > 20.0)
            else:
                hit = m > 20.0 and p > 20.0 and np.float32(m) != np.float32(p)
            if hit:
                out[kind].append((a, b, float(tx), float(ty)))
                slot += 1
                break
    return [(a, b, c, e, k) for k in out for (a, b, c, e) in out[k]]


def swarm_case(seed=0, want=6, n_background=3000):
    """A swarm holding every flipped (agent, task) pair in its own slot, a lower-ID companion 1.5
    from every second flipped task (it claims first: the flipped claim must then beat its value
    + 5), and background agents / tasks with ordinary claims far away.  The slot agents hold every
    capability; the slot tasks require none."""
    rows = find_flips(seed, want)
    rng = np.random.default_rng(seed + 1)
    ax, ay, tx, ty, companion = [], [], [], [], []
    for k, (a, b, c, e, _) in enumerate(rows):
        ax.append(a), ay.append(b), tx.append(c), ty.append(e), companion.append(False)
        if k % 2:
            ax.append(c + 1.5), ay.append(e), companion.append(True)
    near = len(ax)
    bx, by = rng.uniform(30.0, 900.0, n_background), rng.uniform(-40.0, 40.0, n_background)
    ax = np.concatenate([ax, bx])
    ay = np.concatenate([ay, by])
    n = len(ax)
    ids = rng.permutation(4 * n)[:n].astype(np.int32)
    for i in range(near):  # a companion claims before the flipped agent listed just before it
        if companion[i] and ids[i] > ids[i - 1]:
            ids[i], ids[i - 1] = ids[i - 1], ids[i]
    t_bg = 400
    tx = np.concatenate([tx, rng.uniform(30.0, 900.0, t_bg)])
    ty = np.concatenate([ty, rng.uniform(-40.0, 40.0, t_bg)])
    caps = rng.integers(0, 16, n).astype(np.uint32)
    caps[:near] = 0xF
    treq = np.concatenate([np.full(len(rows), -1), rng.integers(-1, 4, t_bg)]).astype(np.int8)
    return dict(ids=ids, x=ax, y=ay, caps=caps, tx=tx, ty=ty, treq=treq, n_flips=len(rows),
                kinds=[r[4] for r in rows])
