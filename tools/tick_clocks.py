"""Where a protocol tick's time goes: runs the bench's 200-tick scenario (10M agents, hybrid 0.125) with a
libswarm build made with -DSWARM_TICK_CLOCKS=1 (tools/build_variant.sh clk "-DSWARM_TICK_CLOCKS=1"
protocol.hip), then summarises the per-workgroup wall clocks (100 MHz) per tick: the tick's span, when
workgroups start (dispatch), how long each role's work takes, the mailing phase.
Usage: python tools/tick_clocks.py [--lib libswarm_clk.so] [--out gpurun_out/tick_clocks.json]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="libswarm_clk.so")
ap.add_argument("--out", default="gpurun_out/tick_clocks.json")
ap.add_argument("--agents", type=int, default=10_000_000)
a = ap.parse_args()
raw = os.path.join(ROOT, "gpurun_out", "tick_clocks.bin")
os.makedirs(os.path.dirname(raw), exist_ok=True)
os.environ["SWARM_TICK_CLOCKS_FILE"] = raw

import torch  # noqa: E402

from swarm_amd import _lib, gen  # noqa: E402
_lib.load(os.path.join(_lib.HERE, a.lib))
from swarm_amd.swarm import Swarm  # noqa: E402

d = gen.swarm_inputs(a.agents, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
off = (np.arange(sw.n, dtype=np.int64) * 7919 % 40).astype(np.int32)
sw.protocol_reset(tick_off=off, last_hb=-(off * 0.1))
c = sw.protocol_run(200, kill_ticks=(80, 150), seed=5)
torch.cuda.synchronize()

hdr = np.fromfile(raw, dtype=np.int64, count=3)
ticks, grid, g_recv = (int(v) for v in hdr)
rec = np.fromfile(raw, dtype=np.uint64, offset=24).reshape(ticks, grid, 5)
us = lambda v: v.astype(np.float64) / 100.0  # noqa: E731  (100 MHz ticks -> µs)
out = []
senders_prev = np.concatenate([[0], c[:-1, 2] + c[:-1, 3]])
for t in range(ticks):
    r = rec[t]
    t0 = r[:, 0].min()
    st, work, dec, end = (us(r[:, k] - t0) for k in range(4))
    ns = (r[:, 4] & ((1 << 40) - 1)).astype(np.int64)
    is_recv = ((r[:, 4] >> 40) & 1).astype(bool)
    pulled = bool(((r[:, 4] >> 41) & 1).any())
    sw_ = ~is_recv
    mail = end - dec
    out.append(dict(tick=t + 1, senders_prev=int(senders_prev[t]), pulled=pulled, span=float(end.max()),
                    start_p50=float(np.median(st)), start_p90=float(np.percentile(st, 90)), start_max=float(st.max()),
                    recv_work_p50=float(np.median((work - st)[is_recv])) if is_recv.any() else None,
                    recv_work_max=float((work - st)[is_recv].max()) if is_recv.any() else None,
                    recv_end_max=float(end[is_recv].max()) if is_recv.any() else None,
                    sweep_work_p50=float(np.median((work - st)[sw_])), sweep_work_max=float((work - st)[sw_].max()),
                    mail_p50=float(np.median(mail[ns > 0])) if (ns > 0).any() else 0.0,
                    mail_max=float(mail.max()), wgs_mailing=int((ns > 0).sum()), senders=int(ns.sum()),
                    last_end_role="recv" if is_recv[np.argmax(end)] else "sweep"))
json.dump(dict(ticks=ticks, grid=grid, g_recv=g_recv, per_tick=out), open(a.out, "w"))
spans = np.array([o["span"] for o in out])
print(json.dumps(dict(ticks=ticks, grid=grid, g_recv=g_recv, span_sum_ms=float(spans.sum() / 1e3))))
for lo, hi in ((0, 1000), (1000, 30000), (30000, 100000), (100000, 10**9)):
    sel = [o for o in out if lo <= o["senders_prev"] < hi and not o["pulled"]]
    if not sel:
        continue
    med = {k: float(np.median([o[k] for o in sel if o[k] is not None])) for k in
           ("span", "start_p50", "start_p90", "start_max", "recv_work_p50", "recv_work_max", "recv_end_max",
            "sweep_work_p50", "sweep_work_max", "mail_p50", "mail_max", "wgs_mailing", "senders")}
    print(json.dumps(dict(senders_prev=[lo, hi], ticks=len(sel), **{k: round(v, 1) for k, v in med.items()})))
