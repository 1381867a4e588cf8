"""Batched wire codec: the transport framing of agent.py:184-214.

Parity is pinned by the reference itself: tests/golden/codec_kat.npz holds messages framed by
the real senders (_send_heartbeat, _check_election_timeout, _process_tasks,
_handle_task_claim -> _pack_header) with the exception each raised, and packets (the encoded
ones plus malformed ones) parsed by the real on_message_received (tools/gen_golden.py
ref_codec).  The struct-based restatement (oracle.codec_*_py) must reproduce it exactly; the GPU
(libswarm swarm_codec_encode / swarm_codec_decode) must reproduce both bit-exactly, and at
large sizes an encode -> decode round trip must return every field (f32-rounded floats).
"""
import numpy as np
import pytest

from conftest import load_golden

DEC_KEYS = ("status", "type", "sender", "tick", "task", "winner", "has_pos", "a", "b")


@pytest.fixture(scope="module")
def kat():
    return load_golden("codec_kat")


def _fields(g):
    return [g["enc_" + k] for k in ("type", "sender", "tick", "a", "b", "task", "winner")]


def test_kat_covers_every_outcome(kat):
    assert set(np.unique(kat["enc_status"])) == {0, 1, 2}
    assert set(np.unique(kat["dec_status"])) == {0, 1, 2, 3}
    assert set(np.unique(kat["enc_type"])) == {1, 2, 3, 4, 5}
    assert kat["dec_has_pos"].any() and not kat["dec_has_pos"].all()


def test_oracle_encode_matches_reference(oracle_mod, kat):
    st, pk = oracle_mod.codec_encode_py(*_fields(kat))
    np.testing.assert_array_equal(st, kat["enc_status"])
    np.testing.assert_array_equal([len(p) for p in pk], kat["enc_len"])
    np.testing.assert_array_equal(np.frombuffer(b"".join(pk), np.uint8), kat["enc_bytes"])


def test_oracle_decode_matches_reference(oracle_mod, kat):
    pk, _ = oracle_mod.split_packets(kat["dec_bytes"], kat["dec_len"])
    d = oracle_mod.codec_decode_py(pk)
    for k in DEC_KEYS:
        np.testing.assert_array_equal(d[k], kat["dec_" + k], err_msg=k)


def _random_msgs(m, seed, wide=False, bad=True):
    rng = np.random.default_rng(seed)
    id_max = 2**32 if wide else 256
    ty = rng.integers(1, 6, m)
    if bad:
        ty[rng.uniform(size=m) < 0.01] = rng.integers(6, 9)
    snd = rng.integers(0, id_max, m)
    tick = rng.integers(0, 2**32, m)
    task = rng.integers(0, 2**32, m)
    win = rng.integers(0, id_max, m)
    a = rng.normal(0, 1e3, m)
    b = rng.normal(0, 1e3, m)
    if bad:
        for arr, hi in ((snd, id_max), (tick, 2**32), (task, 2**32), (win, id_max)):
            sel = rng.uniform(size=m) < 0.01
            arr[sel] = np.where(rng.uniform(size=sel.sum()) < 0.5, -1 - rng.integers(0, 5, sel.sum()),
                                hi + rng.integers(0, 5, sel.sum()))
        a[rng.uniform(size=m) < 0.01] = 3.5e38 * np.sign(rng.normal())
        b[rng.uniform(size=m) < 0.005] = np.inf
        a[rng.uniform(size=m) < 0.005] = np.nan
        a[rng.uniform(size=m) < 0.005] = 3.4028235677973366e38  # rounds to FLT_MAX, no overflow
    return [ty, snd, tick, a, b, task, win]


@pytest.mark.parametrize("wide", [False, True])
def test_oracle_round_trip(oracle_mod, wide):
    f = _random_msgs(3000, 3, wide=wide)
    st, pk = oracle_mod.codec_encode_py(*f, wide=wide)
    assert {0, 1, 2, 3} <= set(np.unique(st))
    ok = st == 0
    d = oracle_mod.codec_decode_py([p for p in pk if p], wide=wide)
    assert (d["status"] == 0).all()
    for k, v in zip(("type", "sender", "tick"), f[:3]):
        np.testing.assert_array_equal(d[k], v[ok])


# ----------------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_gpu_encode_matches_reference(kat):
    from swarm_amd import codec
    e = codec.encode(*_fields(kat), device="cuda")
    np.testing.assert_array_equal(e.status.cpu().numpy(), kat["enc_status"])
    np.testing.assert_array_equal(np.diff(e.offsets.cpu().numpy()), kat["enc_len"])
    assert e.total_bytes == kat["enc_bytes"].size
    np.testing.assert_array_equal(e.buf.cpu().numpy(), kat["enc_bytes"])


@pytest.mark.gpu
def test_gpu_decode_matches_reference(kat):
    from swarm_amd import codec
    off = np.concatenate([[0], np.cumsum(kat["dec_len"])])
    d = codec.decode(kat["dec_bytes"], off, device="cuda")
    for k in DEC_KEYS:
        np.testing.assert_array_equal(getattr(d, k).cpu().numpy(), kat["dec_" + k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
def test_gpu_matches_oracle_random(oracle_mod, wide):
    from swarm_amd import codec
    f = _random_msgs(20000, 11 + wide, wide=wide)
    st, pk = oracle_mod.codec_encode_py(*f, wide=wide)
    e = codec.encode(*f, wide=wide, device="cuda")
    np.testing.assert_array_equal(e.status.cpu().numpy(), st)
    np.testing.assert_array_equal(e.buf.cpu().numpy(), np.frombuffer(b"".join(pk), np.uint8))
    np.testing.assert_array_equal(e.offsets.cpu().numpy(), np.concatenate([[0], np.cumsum([len(p) for p in pk])]))
    # decode: the encoded packets with malformed ones spliced in
    rng = np.random.default_rng(5)
    pk = [p for p in pk if p]
    for i in rng.choice(len(pk), 400, replace=False):
        pk[i] = pk[i][:int(rng.integers(0, len(pk[i])))]
    want = oracle_mod.codec_decode_py(pk, wide=wide)
    buf, off = oracle_mod.split_packets(np.frombuffer(b"".join(pk), np.uint8), [len(p) for p in pk])
    d = codec.decode(np.frombuffer(b"".join(pk), np.uint8), off, wide=wide, device="cuda")
    assert {0, 1, 3} <= set(np.unique(want["status"]))
    for k in DEC_KEYS:
        np.testing.assert_array_equal(getattr(d, k).cpu().numpy(), want[k], err_msg=k)


@pytest.mark.gpu
def test_gpu_round_trip_large():
    """4M messages: encode -> decode returns every field (size-independent property)."""
    import torch
    from swarm_amd import codec
    m = 1 << 22
    f = _random_msgs(m, 21, bad=False)
    e = codec.encode(*f, device="cuda")
    assert int((e.status != 0).sum()) == 0
    d = codec.decode(e.buf, e.offsets, device="cuda")
    assert int((d.status != 0).sum()) == 0
    ty = torch.as_tensor(f[0], device="cuda")
    for k, v in zip(("type", "sender", "tick"), f[:3]):
        assert torch.equal(getattr(d, k), torch.as_tensor(v, device="cuda")), k
    a32 = torch.as_tensor(f[3], device="cuda").float()
    b32 = torch.as_tensor(f[4], device="cuda").float()
    hb, cl, cf = ty == 1, ty == 4, ty == 5
    assert torch.equal(d.a[hb], a32[hb]) and torch.equal(d.b[hb], b32[hb]) and bool(d.has_pos[hb].all())
    assert torch.equal(d.a[cl], a32[cl])
    task = torch.as_tensor(f[5], device="cuda")
    assert torch.equal(d.task[cl | cf], task[cl | cf])
    assert torch.equal(d.winner[cf], torch.as_tensor(f[6], device="cuda")[cf])


@pytest.mark.gpu
def test_gpu_empty_and_errors():
    import torch
    from swarm_amd import _lib, codec
    e = codec.encode(np.zeros(0, np.int64), [], [], device="cuda")
    assert e.total_bytes == 0 and e.offsets.cpu().tolist() == [0]
    d = codec.decode(np.zeros(0, np.uint8), [0], device="cuda")
    assert d.status.numel() == 0
    d = codec.decode(np.zeros(12, np.uint8), [0, 6, 20, 3, 9], device="cuda")  # ok, past the end, backwards
    assert d.status.cpu().tolist() == [2, 4, 4, 2]  # type 0 is unknown; bad offsets are not read
    # undersized output buffer: SWARM_ERR_RANGE, not a write past the end
    ty = torch.ones(4, dtype=torch.int64, device="cuda")
    z = torch.zeros(4, dtype=torch.int64, device="cuda")
    zf = torch.zeros(4, dtype=torch.float64, device="cuda")
    off = torch.empty(5, dtype=torch.int64, device="cuda")
    st = torch.empty(4, dtype=torch.int8, device="cuda")
    buf = torch.empty(10, dtype=torch.uint8, device="cuda")
    import ctypes
    tot = ctypes.c_int64()
    rc = _lib.lib().swarm_codec_encode(_lib.ctx(), 4, *[_lib.ptr(t) for t in (ty, z, z, zf, zf, z, z)], 0,
                                       _lib.ptr(buf), 10, _lib.ptr(off), _lib.ptr(st), ctypes.byref(tot),
                                       _lib.stream())
    assert rc == _lib.ERR_RANGE and tot.value == 56


@pytest.mark.gpu
def test_gpu_encode_sizing_call_and_tile_edges(oracle_mod):
    """swarm_codec_encode with out = NULL returns the byte count; message counts around the encode tile
    (2 048 messages: 8 waves x 256, slabs of 128) give the oracle's bytes and offsets."""
    import ctypes

    import torch
    from swarm_amd import _lib, codec
    for m in (1, 127, 255, 257, 1024, 2047, 2048, 2049, 4096 + 17, 70_001):
        f = _random_msgs(m, 100 + m)
        st, pk = oracle_mod.codec_encode_py(*f)
        want = np.frombuffer(b"".join(pk), np.uint8)
        e = codec.encode(*f, device="cuda")
        np.testing.assert_array_equal(e.status.cpu().numpy(), st)
        np.testing.assert_array_equal(e.buf.cpu().numpy(), want)
        np.testing.assert_array_equal(e.offsets.cpu().numpy(), np.concatenate([[0], np.cumsum([len(p) for p in pk])]))
        cols = [torch.as_tensor(np.asarray(v), device="cuda") for v in f]
        cols = [c.double() if k in (3, 4) else c.long() for k, c in enumerate(cols)]
        off = torch.empty(m + 1, dtype=torch.int64, device="cuda")
        stt = torch.empty(m, dtype=torch.int8, device="cuda")
        tot = ctypes.c_int64(-1)
        _lib.check(_lib.lib().swarm_codec_encode(_lib.ctx(), m, *[_lib.ptr(c) for c in cols], 0, None, 0,
                                                 _lib.ptr(off), _lib.ptr(stt), ctypes.byref(tot), _lib.stream()))
        assert tot.value == len(want)


@pytest.mark.gpu
def test_gpu_encode_unaligned_columns_and_sizing_offsets(oracle_mod):
    """Columns that are views at an odd element offset (8-byte, not 16-byte aligned) take the one-message-
    per-lane form of the one-pass encode; the result is the same, and the sizing call (out = NULL) fills
    status and offsets too."""
    import ctypes

    import torch
    from swarm_amd import _lib
    for m in (3, 1025, 5000):
        f = _random_msgs(m, 7 + m)
        st, pk = oracle_mod.codec_encode_py(*f)
        want = np.frombuffer(b"".join(pk), np.uint8)
        want_off = np.concatenate([[0], np.cumsum([len(p) for p in pk])])
        cols = []
        for k, v in enumerate(f):
            dt = torch.float64 if k in (3, 4) else torch.int64
            big = torch.zeros(m + 1, dtype=dt, device="cuda")
            big[1:] = torch.as_tensor(np.asarray(v), dtype=dt, device="cuda")
            cols.append(big[1:])  # data_ptr % 16 == 8
        assert all(c.data_ptr() % 16 == 8 for c in cols)
        off_big = torch.full((m + 2,), -1, dtype=torch.int64, device="cuda")
        off = off_big[1:]
        stt = torch.full((m,), -1, dtype=torch.int8, device="cuda")
        buf = torch.zeros(max(len(want), 1), dtype=torch.uint8, device="cuda")
        tot = ctypes.c_int64(-1)
        _lib.check(_lib.lib().swarm_codec_encode(_lib.ctx(), m, *[_lib.ptr(c) for c in cols], 0, _lib.ptr(buf),
                                                 buf.numel(), _lib.ptr(off), _lib.ptr(stt), ctypes.byref(tot),
                                                 _lib.stream()))
        assert tot.value == len(want)
        np.testing.assert_array_equal(buf.cpu().numpy()[:len(want)], want)
        np.testing.assert_array_equal(off.cpu().numpy(), want_off)
        np.testing.assert_array_equal(stt.cpu().numpy(), st)
        off.fill_(-1)
        stt.fill_(-1)
        _lib.check(_lib.lib().swarm_codec_encode(_lib.ctx(), m, *[_lib.ptr(c) for c in cols], 0, None, 0,
                                                 _lib.ptr(off), _lib.ptr(stt), ctypes.byref(tot), _lib.stream()))
        np.testing.assert_array_equal(off.cpu().numpy(), want_off)
        np.testing.assert_array_equal(stt.cpu().numpy(), st)


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
def test_gpu_encode_large_matches_oracle_on_a_sample(oracle_mod, wide):
    """6M messages with errors mixed in (~3 000 encode tiles, so the tile offsets come out of long
    look-back walks): every packet length follows from its status and type, the offsets are their
    running sum, and 30 000 sampled messages' statuses and packet bytes equal the oracle's."""
    from swarm_amd import codec
    m = 6_000_000
    f = _random_msgs(m, 31 + wide, wide=wide)
    e = codec.encode(*f, wide=wide, device="cuda")
    st = e.status.cpu().numpy()
    off = e.offsets.cpu().numpy()
    buf = e.buf.cpu().numpy()
    hdr = 9 if wide else 6
    lut = np.zeros(16, np.int64)
    lut[[1, 2, 3, 4, 5]] = [8, 4 if wide else 1, 0, 8, 8 if wide else 5]  # payload bytes by type
    ty = np.asarray(f[0])
    want_len = np.where(st == 0, hdr + lut[np.clip(ty, 0, 15)], 0)
    np.testing.assert_array_equal(np.diff(off), want_len)
    assert off[0] == 0 and off[-1] == e.total_bytes == len(buf)
    assert {0, 1, 3} <= set(np.unique(st))
    idx = np.sort(np.random.default_rng(3).choice(m, 30_000, replace=False))
    sub = [np.asarray(v)[idx] for v in f]
    ost, opk = oracle_mod.codec_encode_py(*sub, wide=wide)
    np.testing.assert_array_equal(st[idx], ost)
    for k, i in enumerate(idx):
        assert bytes(buf[off[i]:off[i + 1]]) == opk[k], int(i)


@pytest.mark.gpu
def test_gpu_encode_recovers_after_a_failed_call(oracle_mod, monkeypatch):
    """A one-pass encode that fails (here: a tile ticket left over, as a failed or overlapping call would
    leave it -- SWARM_ENC_TEST_POISON) reports SWARM_ERR_HIP, and the NEXT call on the same ctx zeroes the
    ticket and the look-back words again and encodes exactly (the ctx no longer trusts a
    buffer a failure left behind)."""
    from swarm_amd import _lib, codec
    m = 200_000
    f = _random_msgs(m, 77)
    good = codec.encode(*f, device="cuda")
    monkeypatch.setenv("SWARM_ENC_TEST_POISON", "1")
    with pytest.raises(_lib.SwarmError) as ei:
        codec.encode(*f, device="cuda")
    assert ei.value.code == _lib.ERR_HIP and "ticket" in str(ei.value)
    monkeypatch.delenv("SWARM_ENC_TEST_POISON")
    for _ in range(2):
        e = codec.encode(*f, device="cuda")
        assert e.total_bytes == good.total_bytes
        np.testing.assert_array_equal(e.offsets.cpu().numpy(), good.offsets.cpu().numpy())
        np.testing.assert_array_equal(e.buf.cpu().numpy(), good.buf.cpu().numpy())
        np.testing.assert_array_equal(e.status.cpu().numpy(), good.status.cpu().numpy())
