// Multi-GPU election driver: the whole sharded round loop on the device stream, with the halo
// exchange as RCCL point-to-point calls over xGMI and the convergence test as one RCCL
// all-reduce per batch of rounds.  No host synchronisation inside a batch.
//
// RCCL is resolved at run time (dlopen/dlsym) from the instance already loaded in the process
// (torch's, SONAME librccl.so.1) so that libswarm.so never links a second copy; only the
// header types come from /opt/rocm/include/rccl.
//
// A second transport runs the same C loops between processes of ONE host whatever their GPUs
// (RCCL refuses two ranks on one device): SWARM_COMM_SHM, a POSIX shared-memory segment with one
// mailbox per rank and op parity and a process-shared barrier.  Each exchange copies the send
// buffers device -> mailbox, meets the barrier, and copies the peers' mailboxes -> device; an
// all-reduce combines every rank's mailbox on the host.  Host-staged and synchronous per op: a
// test and rehearsal transport for the native loops, not a fast one.
#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <cstdlib>
#include <random>
#include <vector>

#include "swarm_common.h"

namespace swarm {
struct ShmHeader {
    std::atomic<uint32_t> magic;    // kShmMagic once rank 0 has initialised the segment
    std::atomic<uint32_t> arrived;  // barrier arrivals in the current generation
    std::atomic<uint32_t> gen;      // barrier generation
    std::atomic<uint32_t> abort;    // a rank gave up waiting: every later barrier fails
    uint32_t nranks;
    uint64_t cap;                   // bytes per mailbox (one per rank and op parity)
};
constexpr uint32_t kShmMagic = 0x5357524Du;  // "SWRM"
constexpr size_t kShmHeader = 4096;
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics must be lock-free");
}  // namespace swarm

struct swarm_comm {
    int kind = SWARM_COMM_RCCL;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    // SWARM_COMM_SHM
    void *base = nullptr;
    size_t bytes = 0;
    swarm::ShmHeader *hdr = nullptr;
    uint64_t ops = 0;                // ops issued (every rank issues the same sequence): parity
    double timeout_s = 120.0;
};

namespace swarm {
namespace {

struct Rccl {
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char *(*errorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl &rccl() {
    static Rccl r = [] {
        Rccl x;
        void *h = nullptr;
        if (const char *p = getenv("SWARM_RCCL_PATH")) h = dlopen(p, RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's, already mapped
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
#define SW_SYM(field, name) x.field = reinterpret_cast<decltype(x.field)>(dlsym(h, name))
        SW_SYM(getUniqueId, "ncclGetUniqueId");
        SW_SYM(commInitRank, "ncclCommInitRank");
        SW_SYM(commDestroy, "ncclCommDestroy");
        SW_SYM(send, "ncclSend");
        SW_SYM(recv, "ncclRecv");
        SW_SYM(allReduce, "ncclAllReduce");
        SW_SYM(allGather, "ncclAllGather");
        SW_SYM(groupStart, "ncclGroupStart");
        SW_SYM(groupEnd, "ncclGroupEnd");
        SW_SYM(errorString, "ncclGetErrorString");
#undef SW_SYM
        x.ok = x.getUniqueId && x.commInitRank && x.commDestroy && x.send && x.recv && x.allReduce && x.allGather &&
               x.groupStart && x.groupEnd && x.errorString;
        return x;
    }();
    return r;
}

#define SW_NCCL(call)                                                                        \
    do {                                                                                     \
        ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess) {                                                             \
            swarm::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,                   \
                             rccl().errorString(r_));                                        \
            return SWARM_ERR_HIP;                                                            \
        }                                                                                    \
    } while (0)

// send buffer <- current leaders of the rows every peer keeps as ghosts (one index list, peer after peer)
__global__ __launch_bounds__(kBlock) void k_pack(const int32_t *__restrict__ L, const int64_t *__restrict__ rows,
                                                int64_t n, int32_t *__restrict__ buf) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        buf[i] = L[rows[i]];
}

// ---- shared-memory transport
char *shm_box(swarm_comm *c, int rank, uint64_t parity) {
    return static_cast<char *>(c->base) + kShmHeader + (size_t(rank) * 2 + parity) * c->hdr->cap;
}

// Process-shared generation barrier with a deadline (a peer that died must not hang the rest).
int shm_barrier(swarm_comm *c) {
    ShmHeader *h = c->hdr;
    const uint32_t g = h->gen.load(std::memory_order_acquire);
    if (h->arrived.fetch_add(1, std::memory_order_acq_rel) == uint32_t(c->nranks) - 1) {
        h->arrived.store(0, std::memory_order_relaxed);
        h->gen.fetch_add(1, std::memory_order_release);
        return SWARM_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; h->gen.load(std::memory_order_acquire) == g; ++spin) {
        if (h->abort.load(std::memory_order_relaxed)) {
            set_error("shared-memory transport: a peer gave up");
            return SWARM_ERR_HIP;
        }
        if ((spin & 255) == 255) {
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt > c->timeout_s) {
                h->abort.store(1, std::memory_order_relaxed);
                set_error("shared-memory transport: barrier timed out after %.0f s (a peer is gone?)", dt);
                return SWARM_ERR_HIP;
            }
            sched_yield();
        }
    }
    return SWARM_OK;
}

// A local error inside a shared-memory op: the peers' next barrier fails at once instead of timing out.
int shm_fail(swarm_comm *c, int rc) {
    if (c->hdr) c->hdr->abort.store(1, std::memory_order_relaxed);
    return rc;
}

// A HIP call inside a shared-memory op: on failure the peers are told (abort) before this rank returns.
#define SW_SHM_HIP(c, call)                                                                  \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) {                                                              \
            swarm::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return shm_fail(c, SWARM_ERR_HIP);                                               \
        }                                                                                    \
    } while (0)

// Halo exchange over the mailboxes.  This rank's mailbox of the op's parity holds a table of
// (offset, count) per destination rank, then its whole send buffer (the segments for its peers back to
// back); a rank reads its ghosts from each peer's mailbox at the offset that peer's table gives it.
// One device -> host copy of the send buffer, one host -> device copy per peer.
int shm_halo(swarm_comm *c, const int32_t *send, const int64_t *soff, const int32_t *peers, int n_peers,
             int32_t *recv, const int64_t *roff, hipStream_t s) {
    const uint64_t par = c->ops++ & 1;
    const size_t tab = size_t(c->nranks) * 2 * 8;
    char *mine = shm_box(c, c->rank, par);
    int64_t *t = reinterpret_cast<int64_t *>(mine);
    for (int q = 0; q < 2 * c->nranks; ++q) t[q] = 0;
    for (int j = 0; j < n_peers; ++j) {
        t[2 * peers[j]] = soff[j];
        t[2 * peers[j] + 1] = soff[j + 1] - soff[j];
    }
    if (soff[n_peers]) SW_SHM_HIP(c, hipMemcpyAsync(mine + tab, send, size_t(soff[n_peers]) * 4, hipMemcpyDeviceToHost, s));
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    if (int rc = shm_barrier(c)) return rc;
    for (int j = 0; j < n_peers; ++j) {
        const char *box = shm_box(c, peers[j], par);
        const int64_t *pt = reinterpret_cast<const int64_t *>(box);
        const int64_t off = pt[2 * c->rank], cnt = pt[2 * c->rank + 1];
        if (cnt != roff[j + 1] - roff[j]) {
            set_error("halo exchange: rank %d sends %lld ghosts to rank %d, which expects %lld", peers[j],
                      (long long)cnt, c->rank, (long long)(roff[j + 1] - roff[j]));
            return shm_fail(c, SWARM_ERR_ARG);
        }
        if (cnt) SW_SHM_HIP(c, hipMemcpyAsync(recv + roff[j], box + tab + size_t(off) * 4, size_t(cnt) * 4,
                                       hipMemcpyHostToDevice, s));
    }
    // the mailboxes of this parity are rewritten two ops later, after every rank has passed the
    // next op's barrier -- which this rank reaches only once its reads here are done
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    return SWARM_OK;
}

int shm_allreduce_u64(swarm_comm *c, unsigned long long *buf, size_t count, bool is_max, hipStream_t s) {
    const uint64_t par = c->ops++ & 1;
    if (uint64_t(count) * 8 > c->hdr->cap) {
        set_error("all-reduce larger than the shared-memory mailboxes (raise SWARM_SHM_MB)");
        return shm_fail(c, SWARM_ERR_ARG);
    }
    SW_SHM_HIP(c, hipMemcpyAsync(shm_box(c, c->rank, par), buf, count * 8, hipMemcpyDeviceToHost, s));
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    if (int rc = shm_barrier(c)) return rc;
    std::vector<unsigned long long> acc(count);
    memcpy(acc.data(), shm_box(c, 0, par), count * 8);
    for (int r = 1; r < c->nranks; ++r) {
        const unsigned long long *q = reinterpret_cast<const unsigned long long *>(shm_box(c, r, par));
        for (size_t i = 0; i < count; ++i) acc[i] = is_max ? std::max(acc[i], q[i]) : acc[i] + q[i];
    }
    SW_SHM_HIP(c, hipMemcpyAsync(buf, acc.data(), count * 8, hipMemcpyHostToDevice, s));
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    return SWARM_OK;
}

int shm_allgather_u64(swarm_comm *c, const unsigned long long *send, size_t count, unsigned long long *recv,
                      hipStream_t s) {
    const uint64_t par = c->ops++ & 1;
    if (uint64_t(count) * 8 > c->hdr->cap) {
        set_error("all-gather larger than the shared-memory mailboxes (raise SWARM_SHM_MB)");
        return shm_fail(c, SWARM_ERR_ARG);
    }
    SW_SHM_HIP(c, hipMemcpyAsync(shm_box(c, c->rank, par), send, count * 8, hipMemcpyDeviceToHost, s));
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    if (int rc = shm_barrier(c)) return rc;
    for (int r = 0; r < c->nranks; ++r)
        SW_SHM_HIP(c, hipMemcpyAsync(recv + size_t(r) * count, shm_box(c, r, par), count * 8, hipMemcpyHostToDevice, s));
    SW_SHM_HIP(c, hipStreamSynchronize(s));
    return SWARM_OK;
}

int shm_create(swarm_comm *c, const char *name) {
    const char *mb = getenv("SWARM_SHM_MB");
    const char *to = getenv("SWARM_SHM_TIMEOUT_S");
    if (to) c->timeout_s = atof(to);
    int fd = -1;
    if (c->rank == 0) {
        const uint64_t cap = (mb ? uint64_t(atoll(mb)) : 16ull) << 20;
        c->bytes = kShmHeader + size_t(c->nranks) * 2 * cap;
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) {
            set_error("shm_open(%s, O_CREAT) failed: %s", name, strerror(errno));
            return SWARM_ERR_HIP;
        }
        if (ftruncate(fd, off_t(c->bytes)) != 0) {
            set_error("ftruncate(%zu) of the shared-memory segment failed: %s", c->bytes, strerror(errno));
            close(fd);
            shm_unlink(name);
            return SWARM_ERR_OOM;
        }
    } else {  // wait for rank 0 to create and size it
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            fd = shm_open(name, O_RDWR, 0600);
            struct stat st{};
            if (fd >= 0 && fstat(fd, &st) == 0 && st.st_size >= off_t(kShmHeader)) {
                c->bytes = size_t(st.st_size);
                break;
            }
            if (fd >= 0) close(fd);
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                set_error("shared-memory segment %s never appeared (rank 0 failed?)", name);
                return SWARM_ERR_HIP;
            }
            usleep(1000);
        }
    }
    c->base = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (c->base == MAP_FAILED) {
        c->base = nullptr;
        set_error("mmap of the shared-memory segment failed: %s", strerror(errno));
        if (c->rank == 0) shm_unlink(name);
        return SWARM_ERR_OOM;
    }
    c->hdr = static_cast<ShmHeader *>(c->base);
    if (c->rank == 0) {
        new (c->hdr) ShmHeader();
        c->hdr->arrived.store(0);
        c->hdr->gen.store(0);
        c->hdr->abort.store(0);
        c->hdr->nranks = uint32_t(c->nranks);
        c->hdr->cap = (c->bytes - kShmHeader) / (size_t(c->nranks) * 2);
        c->hdr->magic.store(kShmMagic, std::memory_order_release);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while (c->hdr->magic.load(std::memory_order_acquire) != kShmMagic) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                set_error("shared-memory segment %s never initialised", name);
                return SWARM_ERR_HIP;
            }
            usleep(1000);
        }
        if (c->hdr->nranks != uint32_t(c->nranks)) {
            set_error("shared-memory segment %s is for %u ranks, not %d", name, c->hdr->nranks, c->nranks);
            return SWARM_ERR_ARG;
        }
    }
    int rc = shm_barrier(c);  // everyone has mapped it: the name can go
    if (c->rank == 0) shm_unlink(name);
    return rc;
}

}  // namespace

// Element-wise MAX all-reduce of u64 words in place on the device stream (the auction's
// per-round bid keys, csrc/auction.hip).  comm->nranks == 1 is a no-op.
int comm_allreduce_max_u64(swarm_comm *comm, unsigned long long *buf, size_t count, hipStream_t s) {
    if (comm == nullptr) {
        set_error("NULL communicator");
        return SWARM_ERR_ARG;
    }
    if (comm->nranks <= 1 || count == 0) return SWARM_OK;
    if (comm->kind == SWARM_COMM_SHM) return shm_allreduce_u64(comm, buf, count, true, s);
    SW_NCCL(rccl().allReduce(buf, buf, count, ncclUint64, ncclMax, comm->comm, s));
    return SWARM_OK;
}

// recv[r * count ...] <- rank r's send buffer of count u64 words, for every rank r (device stream).
int comm_allgather_u64(swarm_comm *comm, const unsigned long long *send, size_t count, unsigned long long *recv,
                       hipStream_t s) {
    if (comm == nullptr) {
        set_error("NULL communicator");
        return SWARM_ERR_ARG;
    }
    if (count == 0) return SWARM_OK;
    if (comm->nranks <= 1) {
        SW_HIP(hipMemcpyAsync(recv, send, count * 8, hipMemcpyDeviceToDevice, s));
        return SWARM_OK;
    }
    if (comm->kind == SWARM_COMM_SHM) return shm_allgather_u64(comm, send, count, recv, s);
    SW_NCCL(rccl().allGather(send, recv, count, ncclUint64, comm->comm, s));
    return SWARM_OK;
}

int comm_rank(const swarm_comm *comm, int *rank, int *nranks) {
    if (comm == nullptr) {
        set_error("NULL communicator");
        return SWARM_ERR_ARG;
    }
    *rank = comm->rank;
    *nranks = comm->nranks;
    return SWARM_OK;
}

}  // namespace swarm

// the frontier round launcher lives in elect.hip
namespace swarm {
int frontier_round_stepper(swarm_ctx *ctx, int t, const int32_t *rp, const int32_t *col, int32_t *L0,
                           int32_t *L1, hipStream_t s);
int frontier_ghosts_both(swarm_ctx *ctx, int t, const int32_t *rp, const int32_t *col, int64_t b_lo, int64_t n_lo,
                         const int32_t *in_lo, int64_t b_hi, int64_t n_hi, const int32_t *in_hi, int32_t *L0,
                         int32_t *L1, hipStream_t s);
int frontier_round_totals(swarm_ctx *ctx, int t0, int t1, unsigned long long *dtot, hipStream_t s);
int frontier_check_compact(swarm_ctx *ctx, const int32_t *rp, const int32_t *col, hipStream_t s);
int64_t frontier_il_min(int64_t n);
bool frontier_round_dense(int t);
}  // namespace swarm

extern "C" {

int swarm_comm_available(void) { return swarm::rccl().ok ? 1 : 0; }

int swarm_comm_unique_id_kind(int kind, void *out128) {
    using namespace swarm;
    SW_ARG(out128 != nullptr, "out is NULL");
    SW_ARG(kind == SWARM_COMM_RCCL || kind == SWARM_COMM_SHM, "unknown transport kind");
    if (kind == SWARM_COMM_RCCL) return swarm_comm_unique_id(out128);
    std::random_device rd;
    char name[128] = {};
    snprintf(name, sizeof(name), "/swarm-shm-%d-%08x%08x", int(getpid()), unsigned(rd()), unsigned(rd()));
    memcpy(out128, name, sizeof(name));
    return SWARM_OK;
}

int swarm_comm_unique_id(void *out128) {
    using namespace swarm;
    SW_ARG(out128 != nullptr, "out is NULL");
    if (!rccl().ok) {
        set_error("RCCL not found in the process (import torch with a ROCm build, or set SWARM_RCCL_PATH)");
        return SWARM_ERR_ARG;
    }
    ncclUniqueId id;
    SW_NCCL(rccl().getUniqueId(&id));
    memcpy(out128, &id, sizeof(id));
    return SWARM_OK;
}

int swarm_comm_create_kind(swarm_comm **out, int kind, int nranks, int rank, const void *id128) {
    using namespace swarm;
    SW_ARG(out && id128, "NULL argument");
    SW_ARG(kind == SWARM_COMM_RCCL || kind == SWARM_COMM_SHM, "unknown transport kind");
    SW_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "rank / nranks out of range");
    if (kind == SWARM_COMM_RCCL) return swarm_comm_create(out, nranks, rank, id128);
    char name[129] = {};
    memcpy(name, id128, 128);
    SW_ARG(name[0] == '/' && strlen(name) > 1, "not a shared-memory transport id (swarm_comm_unique_id_kind)");
    auto *c = new swarm_comm();
    c->kind = SWARM_COMM_SHM;
    c->rank = rank;
    c->nranks = nranks;
    if (int rc = shm_create(c, name)) {
        swarm_comm_destroy(c);
        return rc;
    }
    *out = c;
    return SWARM_OK;
}

int swarm_comm_kind(const swarm_comm *comm) { return comm ? comm->kind : -1; }

int swarm_comm_create(swarm_comm **out, int nranks, int rank, const void *id128) {
    using namespace swarm;
    SW_ARG(out && id128, "NULL argument");
    SW_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "rank / nranks out of range");
    if (!rccl().ok) {
        set_error("RCCL not found in the process");
        return SWARM_ERR_ARG;
    }
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    auto *c = new swarm_comm();
    c->rank = rank;
    c->nranks = nranks;
    ncclResult_t r = rccl().commInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank -> %s", rccl().errorString(r));
        delete c;
        return SWARM_ERR_HIP;
    }
    *out = c;
    return SWARM_OK;
}

int swarm_comm_destroy(swarm_comm *c) {
    if (!c) return SWARM_OK;
    if (c->base) munmap(c->base, c->bytes);
    if (c->comm && swarm::rccl().ok) (void)swarm::rccl().commDestroy(c->comm);
    delete c;
    return SWARM_OK;
}

int swarm_elect_sharded(swarm_ctx *ctx, swarm_comm *comm, const swarm_shard *sh, int32_t *leader0,
                        int32_t *leader1, int32_t max_rounds, int32_t *rounds_exec, int64_t *changes_host,
                        void *stream) {
    return swarm_elect_sharded_ex(ctx, comm, sh, leader0, leader1, max_rounds, rounds_exec, changes_host, nullptr,
                                  nullptr, stream);
}

int swarm_elect_sharded_ex(swarm_ctx *ctx, swarm_comm *comm, const swarm_shard *sh, int32_t *leader0,
                           int32_t *leader1, int32_t max_rounds, int32_t *rounds_exec, int64_t *changes_host,
                           int64_t *local_counts, float *round_ms, void *stream) {
    using namespace swarm;
    SW_ARG(ctx && sh && rounds_exec, "NULL argument");
    swarm_comm solo;  // comm NULL: one rank, no peers (a shard graph stepped alone)
    if (!comm) {
        SW_ARG(sh->n_peers == 0, "a shard with peers needs a communicator");
        solo.kind = SWARM_COMM_RCCL;
        comm = &solo;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool shm = comm->kind == SWARM_COMM_SHM;
    const Rccl &R = rccl();
    if (!shm && comm->nranks > 1 && !R.ok) {
        set_error("RCCL not found in the process");
        return SWARM_ERR_ARG;
    }
    // Every check that one rank alone could fail is made here and agreed on by all ranks (one MAX
    // all-reduce) before the round loop: a rank that left early would keep its peers waiting in their
    // next exchange.
    char why[256] = {};
    const int np = sh->n_peers;
    std::vector<int64_t> soff(size_t(std::max(np, 0)) + 1, 0), roff(size_t(std::max(np, 0)) + 1, 0);
    int64_t below = 0;
    {
        auto bad = [&](const char *m) { if (!why[0]) snprintf(why, sizeof(why), "%s", m); };
        if (max_rounds < 1) bad("max_rounds < 1");
        if (sh->n_rows < 0 || sh->n_all < sh->n_rows) bad("shard sizes");
        if (sh->own_begin < 0 || sh->own_begin + sh->n_rows > sh->n_all) bad("owned range out of [0, n_all)");
        if (np < 0 || (np > 0 && (!sh->peers || !sh->send_count || !sh->ghost_count))) bad("peer list");
        for (int j = 0; j < np && !why[0]; ++j) {
            const int p = sh->peers[j];
            if (p < 0 || p >= comm->nranks || p == comm->rank || (j && p <= sh->peers[j - 1]))
                bad("peers must be ascending ranks of the communicator, other than this rank");
            if (sh->send_count[j] < 0 || sh->ghost_count[j] < 0) bad("negative halo count");
            soff[j + 1] = soff[j] + sh->send_count[j];
            roff[j + 1] = roff[j] + sh->ghost_count[j];
            if (p < comm->rank) below += sh->ghost_count[j];
        }
        if (!why[0] && soff[np] && !sh->send_rows) bad("send_rows is NULL");
        // the ghosts of the peers below fill [0, own_begin), those of the peers above the rows after the owned
        if (!why[0] && (below != sh->own_begin || roff[np] != sh->n_all - sh->n_rows))
            bad("ghost rows must be [peers below | owned | peers above], ghost_count peer by peer");
        if (!why[0] && shm && uint64_t(comm->nranks) * 16 + uint64_t(soff[np]) * 4 > comm->hdr->cap)
            bad("halo larger than the shared-memory mailboxes (raise SWARM_SHM_MB)");
    }
    const size_t nsend = size_t(soff[np]), nrecv = size_t(roff[np]);
    constexpr int kMaxBatch = 256;
    constexpr int kC = kElectCounters;
    const int nr_all = comm->nranks;
    // agreement row of one rank: [failed, depth, send count to each rank, ghosts from each rank]
    const size_t aw = 2 + 2 * size_t(nr_all);
    unsigned long long *dtot;
    SW_ALLOC(dtot, ctx, S_ESTATS, std::max(size_t(kC) * 8 * kMaxBatch, (aw + aw * size_t(nr_all)) * 8));
    // pinned read-back: the batch's global counters, then (local_counts) this rank's own
    unsigned long long *h = static_cast<unsigned long long *>(
        pinned(ctx, std::max(size_t(kC) * 16 * kMaxBatch, aw * size_t(nr_all) * 8)));
    if (!h) return SWARM_ERR_OOM;
    unsigned long long *hl = h + size_t(kC) * kMaxBatch;
    const int depth = sh->halo_depth > 1 ? sh->halo_depth : 1;
    // Everything else that one rank alone could fail -- the stepper's scratch, the 16-bit column check,
    // the loop's buffers and events -- is done before the agreement, so a failure here is agreed on too.
    int local_rc = SWARM_OK;
    int32_t *sbuf = nullptr;
    unsigned long long *lcnt = nullptr;  // this rank's counters of the batch, before the all-reduce
    // per-round device time of this rank's round launches (round_ms): an event before every round of a
    // batch and one after its last (round r's time runs from its start to the next round's)
    std::vector<hipEvent_t> ev;
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() { for (auto e : v) (void)hipEventDestroy(e); }
    } ev_free{ev};
    if (!why[0]) {
        int rc = swarm_frontier_begin_range(ctx, sh->own_begin, sh->n_rows, sh->n_all, sh->init, leader0, leader1,
                                            stream);
        if (!rc)
            rc = sh->col16_escaped ? swarm_frontier_set_compact_escaped(ctx, sh->col16)
                                   : swarm_frontier_set_compact(ctx, sh->col16);
        if (!rc) rc = frontier_check_compact(ctx, sh->row_ptr, sh->col, s);
        if (!rc && !(sbuf = static_cast<int32_t *>(scratch(ctx, S_TMP0, (nsend + nrecv + 4) * 4)))) rc = scratch_code();
        if (!rc && local_counts &&
            !(lcnt = static_cast<unsigned long long *>(scratch(ctx, S_TMP1, size_t(kC) * 8 * kMaxBatch))))
            rc = scratch_code();
        if (!rc && round_ms) {
            ev.assign(kMaxBatch + 1, nullptr);
            for (auto &e : ev)
                if (!rc && hipEventCreate(&e) != hipSuccess) {
                    set_error("hipEventCreate failed");
                    rc = SWARM_ERR_HIP;
                }
        }
        if (rc) {
            local_rc = rc;
            snprintf(why, sizeof(why), "%s", swarm_last_error());
        }
    }
    {
        // one all-gather of every rank's row: every rank then checks the same matrix and reaches the same
        // verdict (a count mismatch would otherwise hang an RCCL send/recv pair)
        std::vector<unsigned long long> row(aw, 0);
        row[0] = why[0] ? 1ull : 0ull;
        row[1] = (unsigned long long)depth;
        for (int j = 0; j < np && !why[0]; ++j) {
            row[2 + sh->peers[j]] = (unsigned long long)sh->send_count[j];
            row[2 + nr_all + sh->peers[j]] = (unsigned long long)sh->ghost_count[j];
        }
        SW_HIP(hipMemcpyAsync(dtot, row.data(), aw * 8, hipMemcpyHostToDevice, s));
        if (int rc = comm_allgather_u64(comm, dtot, aw, dtot + aw, s)) return rc;
        SW_HIP(hipMemcpyAsync(h, dtot + aw, aw * size_t(nr_all) * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        if (why[0]) {
            if (local_rc) return local_rc;  // the error of the failed step is already set
            set_error("swarm_elect_sharded: %s", why);
            return SWARM_ERR_ARG;
        }
        const auto M = [&](int r, size_t k) { return h[size_t(r) * aw + k]; };
        for (int r = 0; r < nr_all; ++r) {
            if (M(r, 0)) {
                set_error("swarm_elect_sharded: rank %d rejected its shard (see its error)", r);
                return SWARM_ERR_ARG;
            }
            if (int(M(r, 1)) != depth) {
                set_error("swarm_elect_sharded: halo_depth differs between ranks (%d here, %d on rank %d)", depth,
                          int(M(r, 1)), r);
                return SWARM_ERR_ARG;
            }
        }
        for (int a = 0; a < nr_all; ++a)
            for (int b = 0; b < nr_all; ++b)
                if (a != b && M(a, 2 + b) != M(b, 2 + nr_all + a)) {
                    set_error("swarm_elect_sharded: rank %d sends %llu halo rows to rank %d, which expects %llu "
                              "(send_count / ghost_count / peers disagree)",
                              a, M(a, 2 + b), b, M(b, 2 + nr_all + a));
                    return SWARM_ERR_ARG;
                }
    }
    int rc = SWARM_OK;
    int32_t *rbuf = sbuf + nsend;
    const int64_t own_end = sh->own_begin + sh->n_rows;
    int found = -1, t = 1, batch = 8;
    std::vector<int64_t> hist;
    // the stamp layout: interleaved while rounds are busy, agent order in the tail (as swarm_elect),
    // switched on the GLOBAL changes against the threshold for the global agent count
    const int64_t il_min = frontier_il_min(sh->n_rows * int64_t(comm->nranks));
    while (t <= max_rounds && found < 0) {
        const int tend = std::min(max_rounds, t + batch - 1);
        ctx->step_wr_agent = (!hist.empty() && hist.back() < il_min) ? 1 : 0;
        for (int r = t; r <= tend; ++r) {
            if (round_ms) SW_HIP(hipEventRecord(ev[r - t], s));
            if ((rc = frontier_round_stepper(ctx, r, sh->row_ptr, sh->col, leader0, leader1, s))) return rc;
            if (r % depth || comm->nranks == 1) continue;  // deep halo: ghosts are stepped locally between exchanges
            // every rank takes part in every exchange, peers or not (the shared-memory ops are barriers)
            int32_t *Lcur = (r & 1) ? leader1 : leader0;
            if (nsend) {
                hipLaunchKernelGGL(k_pack, dim3(grid_for(int64_t(nsend), kBlock, 1024)), dim3(kBlock), 0, s, Lcur,
                                   sh->send_rows, int64_t(nsend), sbuf);
                SW_LAUNCHED();
            }
            if (shm) {
                if ((rc = shm_halo(comm, sbuf, soff.data(), sh->peers, np, rbuf, roff.data(), s))) return rc;
            } else {
                SW_NCCL(R.groupStart());
                for (int j = 0; j < np; ++j) {
                    if (sh->send_count[j])
                        SW_NCCL(R.send(sbuf + soff[j], size_t(sh->send_count[j]), ncclInt32, sh->peers[j], comm->comm, s));
                    if (sh->ghost_count[j])
                        SW_NCCL(R.recv(rbuf + roff[j], size_t(sh->ghost_count[j]), ncclInt32, sh->peers[j], comm->comm, s));
                }
                SW_NCCL(R.groupEnd());
            }
            // the receive buffer is in row order: the lower ghost block, then the upper one
            if (nrecv && (rc = frontier_ghosts_both(ctx, r, sh->row_ptr, sh->col, 0, sh->own_begin, rbuf, own_end,
                                           sh->n_all - own_end, rbuf + sh->own_begin, leader0, leader1, s)))
                return rc;
        }
        const int nr = tend - t + 1;
        if (round_ms) SW_HIP(hipEventRecord(ev[nr], s));
        if ((rc = frontier_round_totals(ctx, t, tend, dtot, s))) return rc;
        if (lcnt) {
            SW_HIP(hipMemcpyAsync(lcnt, dtot, size_t(nr) * kC * 8, hipMemcpyDeviceToDevice, s));
            SW_HIP(hipMemcpyAsync(hl, lcnt, size_t(nr) * kC * 8, hipMemcpyDeviceToHost, s));
        }
        if (shm) {
            if (comm->nranks > 1 && (rc = shm_allreduce_u64(comm, dtot, size_t(nr) * kC, false, s))) return rc;
        } else if (comm->nranks > 1 || comm->comm) {
            SW_NCCL(R.allReduce(dtot, dtot, size_t(nr) * kC, ncclUint64, ncclSum, comm->comm, s));
        }
        SW_HIP(hipMemcpyAsync(h, dtot, size_t(nr) * kC * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        for (int r = t; r <= tend; ++r) {
            if (local_counts) {  // owned changes, gathered rows, gathered edges (a dense round: every row)
                const unsigned long long *q = hl + size_t(r - t) * kC;
                const bool dn = frontier_round_dense(r);
                local_counts[size_t(r - 1) * 3 + 0] = int64_t(q[0]);
                local_counts[size_t(r - 1) * 3 + 1] = dn ? sh->n_all : int64_t(q[1]);
                local_counts[size_t(r - 1) * 3 + 2] = dn ? -1 : int64_t(q[2]);  // -1: all the shard's edges
            }
            if (round_ms) SW_HIP(hipEventElapsedTime(&round_ms[r - 1], ev[r - t], ev[r - t + 1]));
            const unsigned long long c = h[size_t(r - t) * kC];  // C_CHG: owned changes
            hist.push_back(int64_t(c));
            if (changes_host) changes_host[r - 1] = int64_t(c);
            if (c == 0) {
                found = r;
                break;
            }
        }
        t = tend + 1;
        batch = next_round_batch(hist.data(), hist.size(), batch, kMaxBatch);
    }
    *rounds_exec = found > 0 ? found : max_rounds;
    return found > 0 ? SWARM_OK : SWARM_NOT_CONVERGED;
}

}  // extern "C"
