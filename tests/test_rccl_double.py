"""The RCCL test double itself (tests/rccl_double), on the CPU: host buffers (RCCL_DOUBLE_HOST=1), ranks
as processes.  The GPU suite loads the same library into libswarm through SWARM_RCCL_PATH to execute the
native loops' RCCL branch with real peers on one GPU (tests/test_dist_gpu.py, tests/test_c5_rehearsal.py);
these checks pin the double's own semantics first: P2P groups deliver what RCCL would, the collectives
reduce and gather like RCCL, and every pattern under which RCCL would hang -- an unmatched or
mis-sized send/recv, mismatched collectives -- fails on every rank instead.  No reference counterpart
(agent.py:188-194's transport is a stub)."""
import ctypes
import multiprocessing as mp

import numpy as np
import pytest

NCCL_INT32, NCCL_UINT64, NCCL_FLOAT64 = 2, 5, 8
NCCL_SUM, NCCL_MAX, NCCL_MIN = 0, 2, 3
NCCL_INVALID_USAGE = 5


class UniqueId(ctypes.Structure):  # ncclUniqueId: passed BY VALUE to ncclCommInitRank
    _fields_ = [("internal", ctypes.c_char * 128)]


def _load(path):
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    L.ncclGetUniqueId.argtypes = [P]
    L.ncclCommInitRank.argtypes = [ctypes.POINTER(P), ctypes.c_int, UniqueId, ctypes.c_int]
    L.ncclSend.argtypes = [P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, P, P]
    L.ncclRecv.argtypes = [P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, P, P]
    L.ncclAllReduce.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, P, P]
    L.ncclAllGather.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int, P, P]
    L.ncclCommDestroy.argtypes = [P]
    L.rccl_double_stats.argtypes = [P]
    L.rccl_double_stats.restype = None
    return L


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _rank(path, uid, rank, world, case, q):
    import os
    os.environ["RCCL_DOUBLE_HOST"] = "1"
    os.environ["RCCL_DOUBLE_TIMEOUT_S"] = "3"
    L = _load(path)
    comm = ctypes.c_void_p()
    rc = L.ncclCommInitRank(ctypes.byref(comm), world, UniqueId.from_buffer_copy(uid), rank)
    assert rc == 0
    out = {"rank": rank}
    if case == "ring":
        # every rank sends rank * 100 + i (i < 5 + rank) to rank + 1 and receives from rank - 1, plus a
        # second message to rank + 2 in the same group (two sends to different peers, two receives)
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        n2, p2 = (rank + 2) % world, (rank - 2) % world
        a = (rank * 100 + np.arange(5 + rank)).astype(np.int32)
        b = np.full(3, rank, np.int32)
        ra = np.zeros(5 + prv, np.int32)
        rb = np.zeros(3, np.int32)
        L.ncclGroupStart()
        assert L.ncclSend(_ptr(a), a.size, NCCL_INT32, nxt, comm, None) == 0
        assert L.ncclRecv(_ptr(ra), ra.size, NCCL_INT32, prv, comm, None) == 0
        assert L.ncclSend(_ptr(b), b.size, NCCL_INT32, n2, comm, None) == 0
        assert L.ncclRecv(_ptr(rb), rb.size, NCCL_INT32, p2, comm, None) == 0
        assert L.ncclGroupEnd() == 0
        out["ra"], out["rb"] = ra, rb
        # an empty group on every rank (the native loops' ranks without peers still take part)
        L.ncclGroupStart()
        assert L.ncclGroupEnd() == 0
        s = np.array([rank + 1, 10 * rank, 7], np.uint64)
        assert L.ncclAllReduce(_ptr(s), _ptr(s), 3, NCCL_UINT64, NCCL_SUM, comm, None) == 0
        out["sum"] = s.copy()
        m = np.array([rank, -rank], np.float64)
        assert L.ncclAllReduce(_ptr(m), _ptr(m), 2, NCCL_FLOAT64, NCCL_MAX, comm, None) == 0
        out["max"] = m.copy()
        g = np.array([rank, rank * rank], np.uint64)
        gout = np.zeros(2 * world, np.uint64)
        assert L.ncclAllGather(_ptr(g), _ptr(gout), 2, NCCL_UINT64, comm, None) == 0
        out["gather"] = gout
    elif case == "count_mismatch":
        # rank 1 sends 4 ints to rank 0, which expects 5: RCCL would hang; the double fails everywhere
        buf = np.zeros(5, np.int32)
        L.ncclGroupStart()
        if rank == 0:
            L.ncclRecv(_ptr(buf), 5, NCCL_INT32, 1, comm, None)
        elif rank == 1:
            L.ncclSend(_ptr(buf), 4, NCCL_INT32, 0, comm, None)
        out["rc"] = L.ncclGroupEnd()
    elif case == "unmatched_send":
        buf = np.zeros(4, np.int32)
        L.ncclGroupStart()
        if rank == 1:
            L.ncclSend(_ptr(buf), 4, NCCL_INT32, 0, comm, None)
        out["rc"] = L.ncclGroupEnd()
    elif case == "collective_mismatch":
        s = np.zeros(4, np.uint64)
        out["rc"] = L.ncclAllReduce(_ptr(s), _ptr(s), 4 if rank else 3, NCCL_UINT64, NCCL_SUM, comm, None)
    st = (ctypes.c_longlong * 6)()
    L.rccl_double_stats(ctypes.cast(st, ctypes.c_void_p))
    out["stats"] = list(st)
    L.ncclCommDestroy(comm)
    q.put(out)


def _run(path, world, case):
    L = _load(path)
    uid = (ctypes.c_char * 128)()
    assert L.ncclGetUniqueId(ctypes.cast(uid, ctypes.c_void_p)) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(path, bytes(uid), r, world, case, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = sorted([q.get(timeout=60) for _ in ps], key=lambda o: o["rank"])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    return outs


def test_p2p_groups_and_collectives(rccl_double):
    world = 4
    outs = _run(rccl_double, world, "ring")
    for o in outs:
        r = o["rank"]
        prv, p2 = (r - 1) % world, (r - 2) % world
        np.testing.assert_array_equal(o["ra"], prv * 100 + np.arange(5 + prv))
        np.testing.assert_array_equal(o["rb"], np.full(3, p2))
        np.testing.assert_array_equal(o["sum"], [sum(q + 1 for q in range(world)), 10 * sum(range(world)), 7 * world])
        np.testing.assert_array_equal(o["max"], [world - 1, 0.0])
        np.testing.assert_array_equal(o["gather"].reshape(world, 2), [[q, q * q] for q in range(world)])
        groups, sends, recvs, ar, ag, _ = o["stats"]
        assert (groups, sends, recvs, ar, ag) == (1, 2, 2, 2, 1)  # the empty group involves no rank


@pytest.mark.parametrize("case,involved", [("count_mismatch", (0, 1)), ("unmatched_send", (1,)),
                                           ("collective_mismatch", (0, 1, 2))])
def test_patterns_rccl_would_hang_on_fail(rccl_double, case, involved):
    """The ranks RCCL would leave hanging fail instead (one of them with ncclInvalidUsage); a rank outside
    a point-to-point pair is not involved, as with RCCL."""
    outs = _run(rccl_double, 3, case)
    assert all(o["rc"] != 0 for o in outs if o["rank"] in involved), outs
    assert all(o["rc"] == 0 for o in outs if o["rank"] not in involved), outs
    assert any(o["rc"] == NCCL_INVALID_USAGE for o in outs)
