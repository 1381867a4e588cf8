"""Batched wire codec: the reference's transport framing for many messages at once.

SURVEY.md §8f row f3.  The reference frames each message with SwarmAgent._pack_header /
_send_msg ('!BBI' type, sender, tick + a type-specific payload; agent.py:184-194) and parses
inbound packets in on_message_received (agent.py:197-214).  ``encode`` / ``decode`` do that for
a whole batch on the GPU (libswarm swarm_codec_encode / swarm_codec_decode): packets are laid
out back to back in one byte buffer with an int64 offset array (packet i =
buf[offsets[i]:offsets[i+1]]).

Message types (agent.py MsgType): 1 HEARTBEAT (a, b = leader x, y as '!ff'), 2 ELECTION_ACCLAIM
(sender as '!B'), 3 COORDINATOR, 4 TASK_CLAIM (task '!I', a = utility '!f'), 5 TASK_CONFLICT
(task '!I', winner '!B').  Errors are per message, as the reference raises them: status 1
struct.error (a field out of range, e.g. an ID > 255), 2 OverflowError (a finite value beyond
f32), 3 unknown type; decode status 1 dropped (short packet), 2 unknown type, 3 the handler's
unpack raises, 4 offsets outside the buffer (not read).  ``wide=True`` widens the u8 ID fields to u32 (IDs > 255; not in the reference).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from .swarm import _dev, _to

HEARTBEAT, ELECTION_ACCLAIM, COORDINATOR, TASK_CLAIM, TASK_CONFLICT = 1, 2, 3, 4, 5
MAX_PACKET, MAX_PACKET_WIDE = 14, 17   # '!BBI' + '!ff' / '!If';  '!BII' + '!II'
WORST_CASE_LIMIT = 1 << 31              # bytes: above it, size the buffer with a first call


@dataclass
class Encoded:
    buf: torch.Tensor       # uint8 packets back to back
    offsets: torch.Tensor   # int64 (m+1)
    status: torch.Tensor    # int8 per message
    total_bytes: int


@dataclass
class Decoded:
    status: torch.Tensor
    type: torch.Tensor
    sender: torch.Tensor
    tick: torch.Tensor
    a: torch.Tensor         # float32: heartbeat x / claim utility
    b: torch.Tensor         # float32: heartbeat y
    task: torch.Tensor
    winner: torch.Tensor
    has_pos: torch.Tensor   # uint8: heartbeat carried a position


def encode(type, sender, tick, a=None, b=None, task=None, winner=None, *, wide=False, device=None) -> Encoded:
    """Frame m messages.  Integer fields as int64 (out-of-range values report status 1)."""
    dev = _dev(device)
    ty = _to(type, torch.int64, dev)
    m = ty.numel()

    def col(v, dt):
        return torch.zeros(m, dtype=dt, device=dev) if v is None else _to(v, dt, dev)

    snd, tk = col(sender, torch.int64), col(tick, torch.int64)
    fa, fb = col(a, torch.float64), col(b, torch.float64)
    tsk, win = col(task, torch.int64), col(winner, torch.int64)
    for name, t in (("sender", snd), ("tick", tk), ("a", fa), ("b", fb), ("task", tsk), ("winner", win)):
        if t.numel() != m:
            raise ValueError(f"{name}: {t.numel()} values for {m} messages")
    offsets = torch.empty(m + 1, dtype=torch.int64, device=dev)
    status = torch.empty(m, dtype=torch.int8, device=dev)
    total = ctypes.c_int64(0)
    L = _lib.lib()
    args = [ty, snd, tk, fa, fb, tsk, win]
    worst = m * (MAX_PACKET_WIDE if wide else MAX_PACKET)
    with torch.cuda.device(dev):
        p = [_lib.ptr(t) if m else None for t in args]
        if worst <= WORST_CASE_LIMIT:  # one call into a worst-case buffer
            buf = torch.empty(max(worst, 1), dtype=torch.uint8, device=dev)
        else:  # a sizing call first
            _lib.check(L.swarm_codec_encode(_lib.ctx(), m, *p, int(bool(wide)), None, 0, _lib.ptr(offsets),
                                            _lib.ptr(status) if m else None, ctypes.byref(total), _lib.stream()))
            buf = torch.empty(max(total.value, 1), dtype=torch.uint8, device=dev)
        _lib.check(L.swarm_codec_encode(_lib.ctx(), m, *p, int(bool(wide)), _lib.ptr(buf), buf.numel(),
                                        _lib.ptr(offsets), _lib.ptr(status) if m else None, ctypes.byref(total),
                                        _lib.stream()))
    return Encoded(buf[:total.value], offsets, status, total.value)


def decode(buf, offsets, *, wide=False, device=None) -> Decoded:
    """Parse packets buf[offsets[i]:offsets[i+1]]; a packet whose offsets leave buf or run
    backwards gets status 4 and is not read."""
    dev = _dev(device)
    raw = _to(buf, torch.uint8, dev)
    off = _to(offsets, torch.int64, dev)
    m = max(off.numel() - 1, 0)
    e = lambda dt: torch.empty(m, dtype=dt, device=dev)  # noqa: E731  (k_decode writes every field)
    out = Decoded(e(torch.int8), e(torch.int64), e(torch.int64), e(torch.int64), e(torch.float32),
                  e(torch.float32), e(torch.int64), e(torch.int64), e(torch.uint8))
    if m:
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().swarm_codec_decode(
                _lib.ctx(), m, _lib.ptr(raw) if raw.numel() else None, raw.numel(), _lib.ptr(off), int(bool(wide)),
                *[_lib.ptr(t) for t in (out.status, out.type, out.sender, out.tick, out.a, out.b, out.task,
                                        out.winner, out.has_pos)], _lib.stream()))
    return out
