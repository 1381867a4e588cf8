// A test double of the ten RCCL entry points libswarm resolves at run time (csrc/comm.hip, rccl()),
// loaded through SWARM_RCCL_PATH.  It lets the native sharded loops take their RCCL branch --
// ncclSend/ncclRecv pairs inside ncclGroupStart/End, the counter all-reduce, the auction's MAX
// all-reduce and all-gather -- with real peers that share ONE GPU (real RCCL refuses two ranks on one
// device), so that the pairing, the per-peer counts, the datatypes and the reduction ops of that code
// are executed and checked, not only compiled.
//
// Transport: a POSIX shared-memory segment named by the unique id.  Synchronous on the host: the
// caller's stream is synchronised before any payload is read from the device.
//   P2P     RCCL's semantics: pairwise, FIFO per (sender, receiver) pair, no rank outside the pair
//           involved.  One channel per ordered pair with a ring of kSlots message slots; at
//           ncclGroupEnd a rank posts all its sends (device -> slot), then takes its recvs in order
//           (slot -> device, ack), then waits until its own sends are acked.
//   collectives  one mailbox per rank and a process-shared barrier: all ranks post, meet, combine,
//           meet again; every rank must have passed the same count, datatype and reduction op.
// Where RCCL would hang, the double fails (ncclInvalidUsage, or ncclSystemError after
// RCCL_DOUBLE_TIMEOUT_S, default 60 s): a recv whose matching send has a different count or datatype,
// a recv that no send ever meets, a send that no recv takes, mismatched collectives.  A failing rank
// raises the segment's abort flag, so the peers waiting on it fail at once.
// rccl_double_stats() reports what was executed (the tests assert that the RCCL branch really ran).
// Test infrastructure only: built by tests/rccl_double/Makefile (tests/conftest.py,
// __graft_entry__.build()), never linked into libswarm.so.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <random>
#include <vector>

namespace {

constexpr uint32_t kMagic = 0x52434344u;  // "RCCD"
constexpr size_t kHeader = 4096;

constexpr int kSlots = 2;  // messages in flight per (sender, receiver) pair

struct Seg {
    std::atomic<uint32_t> magic;
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> gen;
    std::atomic<uint32_t> abort;
    uint32_t nranks;
    uint64_t cap;       // bytes per collective mailbox
    uint64_t slot_cap;  // payload bytes per P2P slot
};

// A collective mailbox: a Box, then the payload at kPayload.
enum OpKind : uint32_t { OP_ALLREDUCE = 2, OP_ALLGATHER = 3 };
struct Box {
    uint32_t kind;
    uint32_t pad;
    uint64_t seq;  // the collective's index in the communicator's sequence of collectives
    uint64_t count;
    int32_t dtype, op;
};
constexpr size_t kPayload = 64;

// A P2P channel (sender -> receiver): message k lives in slot k % kSlots.
struct Chan {
    std::atomic<uint64_t> posted;  // messages the sender has written
    std::atomic<uint64_t> acked;   // messages the receiver has taken
    uint64_t count[kSlots];
    int32_t dtype[kSlots];
};
constexpr size_t kChanHdr = 128;
static_assert(sizeof(Chan) <= kChanHdr, "channel header");

struct Pending {
    bool send;
    void *buf;
    size_t count;
    ncclDataType_t dtype;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};

thread_local int g_depth = 0;
thread_local std::vector<Pending> g_pending;

std::atomic<long long> g_groups{0}, g_sends{0}, g_recvs{0}, g_allreduce{0}, g_allgather{0}, g_bytes{0};

size_t dsize(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

void say(const char *fmt, ...) {
    char m[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(m, sizeof(m), fmt, ap);
    va_end(ap);
    fprintf(stderr, "[rccl_double] %s\n", m);
}

}  // namespace

struct ncclComm {
    int rank = 0, nranks = 1;
    void *base = nullptr;
    size_t bytes = 0;
    Seg *seg = nullptr;
    uint64_t seq = 0;
    double timeout_s = 60.0;
};

namespace {

char *box_of(ncclComm *c, int r) { return static_cast<char *>(c->base) + kHeader + size_t(r) * c->seg->cap; }

size_t chan_bytes(const Seg *s) { return kChanHdr + kSlots * s->slot_cap; }

Chan *chan_of(ncclComm *c, int from, int to) {
    char *p = static_cast<char *>(c->base) + kHeader + size_t(c->nranks) * c->seg->cap +
              (size_t(from) * c->nranks + to) * chan_bytes(c->seg);
    return reinterpret_cast<Chan *>(p);
}

char *slot_of(ncclComm *c, Chan *ch, uint64_t k) {
    return reinterpret_cast<char *>(ch) + kChanHdr + (k % kSlots) * c->seg->slot_cap;
}

ncclResult_t fail(ncclComm *c, ncclResult_t rc) {
    if (c && c->seg) c->seg->abort.store(1);
    return rc;
}

ncclResult_t barrier(ncclComm *c) {
    Seg *s = c->seg;
    const uint32_t g = s->gen.load(std::memory_order_acquire);
    if (s->arrived.fetch_add(1, std::memory_order_acq_rel) == uint32_t(c->nranks) - 1) {
        s->arrived.store(0, std::memory_order_relaxed);
        s->gen.fetch_add(1, std::memory_order_release);
        return ncclSuccess;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; s->gen.load(std::memory_order_acquire) == g; ++spin) {
        if (s->abort.load()) {
            say("rank %d: a peer failed", c->rank);
            return ncclSystemError;
        }
        if ((spin & 255) == 255) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                say("rank %d: barrier timed out (a peer issued a different operation sequence?)", c->rank);
                return fail(c, ncclSystemError);
            }
            sched_yield();
        }
    }
    return ncclSuccess;
}

// Spin until pred() holds; fails on the abort flag or after the timeout (what: the message then).
template <typename Pred>
ncclResult_t wait_for(ncclComm *c, Pred pred, const char *what, int peer) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; !pred(); ++spin) {
        if (c->seg->abort.load()) {
            say("rank %d: a peer failed (while waiting: %s rank %d)", c->rank, what, peer);
            return ncclSystemError;
        }
        if ((spin & 255) == 255) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                say("rank %d: %s rank %d: timed out (RCCL would hang)", c->rank, what, peer);
                return fail(c, ncclInvalidUsage);
            }
            sched_yield();
        }
    }
    return ncclSuccess;
}

ncclResult_t hip_ok(ncclComm *c, hipError_t e, const char *what) {
    if (e == hipSuccess) return ncclSuccess;
    say("rank %d: %s -> %s", c->rank, what, hipGetErrorString(e));
    return fail(c, ncclUnhandledCudaError);
}

// RCCL_DOUBLE_HOST=1: the buffers are host memory (the double's own CPU tests, no GPU): plain copies,
// no stream synchronisation.
bool host_mode() {
    static const bool h = [] {
        const char *e = getenv("RCCL_DOUBLE_HOST");
        return e && e[0] == '1';
    }();
    return h;
}

ncclResult_t copy(ncclComm *c, void *dst, const void *src, size_t n, hipMemcpyKind k, const char *what) {
    if (host_mode()) {
        memcpy(dst, src, n);
        return ncclSuccess;
    }
    return hip_ok(c, hipMemcpy(dst, src, n, k), what);
}

ncclResult_t sync(ncclComm *c, hipStream_t s) {
    return host_mode() ? ncclSuccess : hip_ok(c, hipStreamSynchronize(s), "hipStreamSynchronize");
}

#define DB_TRY(x)                         \
    do {                                  \
        ncclResult_t r_ = (x);            \
        if (r_ != ncclSuccess) return r_; \
    } while (0)

// The peers' mailboxes must hold the same operation as this rank's (kind and sequence number).
ncclResult_t same_op(ncclComm *c, const Box *mine) {
    for (int r = 0; r < c->nranks; ++r) {
        const Box *o = reinterpret_cast<const Box *>(box_of(c, r));
        if (o->kind != mine->kind || o->seq != mine->seq) {
            say("rank %d: operation %llu is kind %u here but kind %u (operation %llu) on rank %d", c->rank,
                (unsigned long long)mine->seq, mine->kind, o->kind, (unsigned long long)o->seq, r);
            return fail(c, ncclInvalidUsage);
        }
        if ((o->count != mine->count || o->dtype != mine->dtype || o->op != mine->op)) {
            say("rank %d: collective %llu: count/datatype/op %llu/%d/%d here, %llu/%d/%d on rank %d", c->rank,
                (unsigned long long)mine->seq, (unsigned long long)mine->count, mine->dtype, mine->op,
                (unsigned long long)o->count, o->dtype, o->op, r);
            return fail(c, ncclInvalidUsage);
        }
    }
    return ncclSuccess;
}

// One P2P group of one communicator: post every send of this rank, take its recvs in order, then wait
// until its sends are taken.  Only the ranks of each pair are involved (RCCL's point-to-point semantics).
ncclResult_t run_p2p(ncclComm *c, const std::vector<Pending> &ops) {
    for (const auto &p : ops) DB_TRY(sync(c, p.stream));
    std::vector<std::pair<Chan *, uint64_t>> mine;  // channel, message index of each send
    for (const auto &p : ops) {
        if (!p.send) continue;
        const size_t nb = p.count * dsize(p.dtype);
        if (nb > c->seg->slot_cap) {
            say("rank %d: a send of %zu bytes is larger than a slot (RCCL_DOUBLE_P2P_MB)", c->rank, nb);
            return fail(c, ncclInvalidUsage);
        }
        Chan *ch = chan_of(c, c->rank, p.peer);
        const uint64_t k = ch->posted.load(std::memory_order_relaxed);
        DB_TRY(wait_for(c, [&] { return ch->acked.load(std::memory_order_acquire) + kSlots > k; },
                        "a free slot towards", p.peer));
        if (nb) DB_TRY(copy(c, slot_of(c, ch, k), p.buf, nb, hipMemcpyDeviceToHost, "send copy"));
        ch->count[k % kSlots] = p.count;
        ch->dtype[k % kSlots] = int32_t(p.dtype);
        ch->posted.store(k + 1, std::memory_order_release);
        mine.emplace_back(ch, k);
        g_sends++;
        g_bytes += (long long)nb;
    }
    for (const auto &p : ops) {
        if (p.send) continue;
        Chan *ch = chan_of(c, p.peer, c->rank);
        const uint64_t k = ch->acked.load(std::memory_order_relaxed);
        DB_TRY(wait_for(c, [&] { return ch->posted.load(std::memory_order_acquire) > k; },
                        "a recv that no send meets, from", p.peer));
        if (ch->count[k % kSlots] != p.count || ch->dtype[k % kSlots] != int32_t(p.dtype)) {
            say("rank %d: recv of %zu x dtype %d from rank %d, which sends %llu x dtype %d (RCCL would hang)",
                c->rank, p.count, int(p.dtype), p.peer, (unsigned long long)ch->count[k % kSlots],
                ch->dtype[k % kSlots]);
            return fail(c, ncclInvalidUsage);
        }
        const size_t nb = p.count * dsize(p.dtype);
        if (nb) DB_TRY(copy(c, p.buf, slot_of(c, ch, k), nb, hipMemcpyHostToDevice, "recv copy"));
        ch->acked.store(k + 1, std::memory_order_release);
        g_recvs++;
    }
    for (size_t i = 0; i < mine.size(); ++i) {
        Chan *ch = mine[i].first;
        const uint64_t k = mine[i].second;
        const int peer = int(((reinterpret_cast<char *>(ch) - static_cast<char *>(c->base) - kHeader -
                               size_t(c->nranks) * c->seg->cap) / chan_bytes(c->seg)) % size_t(c->nranks));
        DB_TRY(wait_for(c, [&] { return ch->acked.load(std::memory_order_acquire) > k; },
                        "a send that no recv takes, to", peer));
    }
    g_groups++;
    return ncclSuccess;
}

template <typename T>
void reduce_into(T *acc, const T *x, size_t n, ncclRedOp_t op) {
    for (size_t i = 0; i < n; ++i) {
        switch (op) {
        case ncclSum: acc[i] = T(acc[i] + x[i]); break;
        case ncclProd: acc[i] = T(acc[i] * x[i]); break;
        case ncclMax: acc[i] = std::max(acc[i], x[i]); break;
        case ncclMin: acc[i] = std::min(acc[i], x[i]); break;
        default: break;
        }
    }
}

bool reduce_typed(void *acc, const void *x, size_t n, ncclDataType_t t, ncclRedOp_t op) {
    switch (t) {
    case ncclInt8: reduce_into(static_cast<int8_t *>(acc), static_cast<const int8_t *>(x), n, op); return true;
    case ncclUint8: reduce_into(static_cast<uint8_t *>(acc), static_cast<const uint8_t *>(x), n, op); return true;
    case ncclInt32: reduce_into(static_cast<int32_t *>(acc), static_cast<const int32_t *>(x), n, op); return true;
    case ncclUint32: reduce_into(static_cast<uint32_t *>(acc), static_cast<const uint32_t *>(x), n, op); return true;
    case ncclInt64: reduce_into(static_cast<int64_t *>(acc), static_cast<const int64_t *>(x), n, op); return true;
    case ncclUint64: reduce_into(static_cast<uint64_t *>(acc), static_cast<const uint64_t *>(x), n, op); return true;
    case ncclFloat32: reduce_into(static_cast<float *>(acc), static_cast<const float *>(x), n, op); return true;
    case ncclFloat64: reduce_into(static_cast<double *>(acc), static_cast<const double *>(x), n, op); return true;
    default: return false;
    }
}

ncclResult_t collective(ncclComm *c, OpKind kind, const void *send, void *recv, size_t count, ncclDataType_t t,
                        ncclRedOp_t op, hipStream_t s) {
    if (g_depth > 0) {
        say("rank %d: collectives inside a group are not supported by the double", c->rank);
        return fail(c, ncclInvalidUsage);
    }
    const size_t es = dsize(t);
    if (es == 0 || (kind == OP_ALLREDUCE && op != ncclSum && op != ncclProd && op != ncclMax && op != ncclMin)) {
        say("rank %d: unsupported datatype %d / op %d", c->rank, int(t), int(op));
        return fail(c, ncclInvalidArgument);
    }
    const size_t nb = count * es;
    if (kPayload + nb > c->seg->cap) {
        say("rank %d: collective larger than the mailbox (RCCL_DOUBLE_MB)", c->rank);
        return fail(c, ncclInvalidUsage);
    }
    DB_TRY(sync(c, s));
    char *mine = box_of(c, c->rank);
    Box *b = reinterpret_cast<Box *>(mine);
    if (nb) DB_TRY(copy(c, mine + kPayload, send, nb, hipMemcpyDeviceToHost, "collective send copy"));
    b->kind = kind;
    b->pad = 0;
    b->seq = c->seq;
    b->count = count;
    b->dtype = int32_t(t);
    b->op = kind == OP_ALLREDUCE ? int32_t(op) : 0;
    DB_TRY(barrier(c));
    DB_TRY(same_op(c, b));
    if (kind == OP_ALLREDUCE) {
        std::vector<char> acc(nb);
        memcpy(acc.data(), box_of(c, 0) + kPayload, nb);
        for (int r = 1; r < c->nranks; ++r) reduce_typed(acc.data(), box_of(c, r) + kPayload, count, t, op);
        if (nb) DB_TRY(copy(c, recv, acc.data(), nb, hipMemcpyHostToDevice, "all-reduce result copy"));
        g_allreduce++;
    } else {
        for (int r = 0; r < c->nranks; ++r)
            if (nb)
                DB_TRY(copy(c, static_cast<char *>(recv) + size_t(r) * nb, box_of(c, r) + kPayload, nb,
                            hipMemcpyHostToDevice, "all-gather copy"));
        g_allgather++;
    }
    g_bytes += (long long)nb;
    DB_TRY(barrier(c));
    ++c->seq;
    return ncclSuccess;
}

ncclResult_t flush_pending() {
    std::vector<Pending> ops;
    ops.swap(g_pending);
    // one group per communicator, in the order the communicators first appear
    std::vector<ncclComm_t> comms;
    for (const auto &p : ops)
        if (std::find(comms.begin(), comms.end(), p.comm) == comms.end()) comms.push_back(p.comm);
    for (ncclComm_t c : comms) {
        std::vector<Pending> mine;
        for (const auto &p : ops)
            if (p.comm == c) mine.push_back(p);
        DB_TRY(run_p2p(c, mine));
    }
    return ncclSuccess;
}

ncclResult_t enqueue(bool send, void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    if (!c || peer < 0 || peer >= c->nranks || peer == c->rank || dsize(t) == 0) {
        say("rank %d: bad %s (peer %d, dtype %d)", c ? c->rank : -1, send ? "send" : "recv", peer, int(t));
        return fail(c, ncclInvalidArgument);
    }
    g_pending.push_back(Pending{send, buf, count, t, peer, c, s});
    if (g_depth == 0) return flush_pending();  // outside a group: the op is its own group
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    std::random_device rd;
    memset(id, 0, sizeof(*id));
    snprintf(id->internal, sizeof(id->internal), "/rccl-double-%d-%08x%08x", int(getpid()), unsigned(rd()),
             unsigned(rd()));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || id.internal[0] != '/') return ncclInvalidArgument;
    auto *c = new (std::nothrow) ncclComm();
    if (!c) return ncclSystemError;
    c->rank = rank;
    c->nranks = nranks;
    if (const char *to = getenv("RCCL_DOUBLE_TIMEOUT_S")) c->timeout_s = atof(to);
    char name[NCCL_UNIQUE_ID_BYTES + 1] = {};
    memcpy(name, id.internal, NCCL_UNIQUE_ID_BYTES);
    int fd = -1;
    const auto t0 = std::chrono::steady_clock::now();
    const char *mb = getenv("RCCL_DOUBLE_MB");
    const char *pmb = getenv("RCCL_DOUBLE_P2P_MB");
    const uint64_t cap = (mb ? uint64_t(atoll(mb)) : 4ull) << 20;   // rank 0's choice holds for all
    const uint64_t slot = (pmb ? uint64_t(atoll(pmb)) : 4ull) << 20;
    if (rank == 0) {
        c->bytes = kHeader + size_t(nranks) * cap + size_t(nranks) * nranks * (kChanHdr + kSlots * slot);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, off_t(c->bytes)) != 0) {
            say("rank 0: shared-memory segment %s: %s", name, strerror(errno));
            if (fd >= 0) {
                close(fd);
                shm_unlink(name);
            }
            delete c;
            return ncclSystemError;
        }
    } else {
        for (;;) {
            fd = shm_open(name, O_RDWR, 0600);
            struct stat st {};
            if (fd >= 0 && fstat(fd, &st) == 0 && st.st_size > off_t(kHeader)) {
                c->bytes = size_t(st.st_size);
                break;
            }
            if (fd >= 0) close(fd);
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                say("rank %d: segment %s never appeared", rank, name);
                delete c;
                return ncclSystemError;
            }
            usleep(1000);
        }
    }
    c->base = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (c->base == MAP_FAILED) {
        if (rank == 0) shm_unlink(name);
        delete c;
        return ncclSystemError;
    }
    c->seg = static_cast<Seg *>(c->base);
    if (rank == 0) {
        new (c->seg) Seg();
        c->seg->arrived.store(0);
        c->seg->gen.store(0);
        c->seg->abort.store(0);
        c->seg->nranks = uint32_t(nranks);
        c->seg->cap = cap;
        c->seg->slot_cap = slot;
        c->seg->magic.store(kMagic, std::memory_order_release);
    } else {
        while (c->seg->magic.load(std::memory_order_acquire) != kMagic) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                munmap(c->base, c->bytes);
                delete c;
                return ncclSystemError;
            }
            usleep(1000);
        }
        if (c->seg->nranks != uint32_t(nranks)) {
            say("rank %d: segment is for %u ranks, not %d", rank, c->seg->nranks, nranks);
            munmap(c->base, c->bytes);
            delete c;
            return ncclInvalidArgument;
        }
    }
    const ncclResult_t rc = barrier(c);  // every rank has mapped it: the name can go
    if (rank == 0) shm_unlink(name);
    if (rc != ncclSuccess) {
        munmap(c->base, c->bytes);
        delete c;
        return rc;
    }
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclSuccess;
    if (c->base) munmap(c->base, c->bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    return flush_pending();
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    return enqueue(true, const_cast<void *>(buf), count, t, peer, c, s);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    return enqueue(false, buf, count, t, peer, c, s);
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t t, ncclRedOp_t op, ncclComm_t c,
                           hipStream_t s) {
    if (!c) return ncclInvalidArgument;
    return collective(c, OP_ALLREDUCE, send, recv, count, t, op, s);
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t c, hipStream_t s) {
    if (!c) return ncclInvalidArgument;
    return collective(c, OP_ALLGATHER, send, recv, count, t, ncclSum, s);
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (rccl double)";
    case ncclUnhandledCudaError: return "HIP call failed (rccl double)";
    case ncclSystemError: return "system error: barrier timeout, a peer failed, or shared memory (rccl double)";
    case ncclInvalidArgument: return "invalid argument (rccl double)";
    case ncclInvalidUsage: return "invalid usage: unmatched send/recv or mismatched collective (rccl double)";
    default: return "error (rccl double)";
    }
}

// Counters of what this process executed: groups, sends, recvs, all-reduces, all-gathers, bytes.
void rccl_double_stats(long long *out6) {
    out6[0] = g_groups.load();
    out6[1] = g_sends.load();
    out6[2] = g_recvs.load();
    out6[3] = g_allreduce.load();
    out6[4] = g_allgather.load();
    out6[5] = g_bytes.load();
}

}  // extern "C"
