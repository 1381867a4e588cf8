// Multi-GPU election driver: the whole sharded round loop on the device stream, with the halo
// exchange as RCCL point-to-point calls over xGMI and the convergence test as one RCCL
// all-reduce per batch of rounds.  No host synchronisation inside a batch.
//
// RCCL is resolved at run time (dlopen/dlsym) from the instance already loaded in the process
// (torch's, SONAME librccl.so.1) so that libswarm.so never links a second copy; only the
// header types come from /opt/rocm/include/rccl.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "swarm_common.h"

struct swarm_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
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
        SW_SYM(groupStart, "ncclGroupStart");
        SW_SYM(groupEnd, "ncclGroupEnd");
        SW_SYM(errorString, "ncclGetErrorString");
#undef SW_SYM
        x.ok = x.getUniqueId && x.commInitRank && x.commDestroy && x.send && x.recv && x.allReduce &&
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

// send buffers <- current leaders of the boundary agents (both borders in one launch)
__global__ __launch_bounds__(kBlock) void k_pack(const int32_t *__restrict__ L, const int64_t *__restrict__ lo_idx,
                                                int64_t n_lo, const int64_t *__restrict__ hi_idx, int64_t n_hi,
                                                int32_t *__restrict__ lo_buf, int32_t *__restrict__ hi_buf) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n_lo + n_hi; i += int64_t(gridDim.x) * kBlock) {
        if (i < n_lo) lo_buf[i] = L[lo_idx[i]];
        else hi_buf[i - n_lo] = L[hi_idx[i - n_lo]];
    }
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
    SW_NCCL(rccl().allReduce(buf, buf, count, ncclUint64, ncclMax, comm->comm, s));
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
}  // namespace swarm

extern "C" {

int swarm_comm_available(void) { return swarm::rccl().ok ? 1 : 0; }

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
    if (c->comm && swarm::rccl().ok) (void)swarm::rccl().commDestroy(c->comm);
    delete c;
    return SWARM_OK;
}

int swarm_elect_sharded(swarm_ctx *ctx, swarm_comm *comm, const swarm_shard *sh, int32_t *leader0,
                        int32_t *leader1, int32_t max_rounds, int32_t *rounds_exec, int64_t *changes_host,
                        void *stream) {
    using namespace swarm;
    SW_ARG(ctx && comm && sh && rounds_exec, "NULL argument");
    SW_ARG(max_rounds >= 1, "max_rounds < 1");
    SW_ARG(sh->n_rows >= 0 && sh->n_all >= sh->n_rows, "shard sizes");
    SW_ARG(sh->own_begin >= 0 && sh->own_begin + sh->n_rows <= sh->n_all, "owned range out of [0, n_all)");
    SW_ARG((sh->peer_lo >= 0 || (sh->n_send_lo == 0 && sh->n_ghost_lo == 0)) &&
           (sh->peer_hi >= 0 || (sh->n_send_hi == 0 && sh->n_ghost_hi == 0)), "halo without a peer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = swarm_frontier_begin_range(ctx, sh->own_begin, sh->n_rows, sh->n_all, sh->init, leader0, leader1, stream);
    if (rc) return rc;
    if ((rc = swarm_frontier_set_compact(ctx, sh->col16))) return rc;
    int32_t *bufs;
    const size_t nb = size_t(sh->n_send_lo + sh->n_send_hi + sh->n_ghost_lo + sh->n_ghost_hi) + 4;
    SW_ALLOC(bufs, ctx, S_TMP0, nb * 4);
    int32_t *s_lo = bufs, *s_hi = s_lo + sh->n_send_lo, *r_lo = s_hi + sh->n_send_hi, *r_hi = r_lo + sh->n_ghost_lo;
    constexpr int kMaxBatch = 256;
    unsigned long long *dtot;
    constexpr int kC = kElectCounters;
    SW_ALLOC(dtot, ctx, S_ESTATS, size_t(kC) * 8 * kMaxBatch);
    unsigned long long *h = static_cast<unsigned long long *>(pinned(ctx, size_t(kC) * 8 * kMaxBatch));
    if (!h) return SWARM_ERR_OOM;
    const Rccl &R = rccl();
    const int depth = sh->halo_depth > 1 ? sh->halo_depth : 1;
    int found = -1, t = 1, batch = 8;
    std::vector<int64_t> hist;
    while (t <= max_rounds && found < 0) {
        const int tend = std::min(max_rounds, t + batch - 1);
        for (int r = t; r <= tend; ++r) {
            if ((rc = frontier_round_stepper(ctx, r, sh->row_ptr, sh->col, leader0, leader1, s))) return rc;
            if (r % depth) continue;  // deep halo: ghosts are stepped locally between exchanges
            int32_t *Lcur = (r & 1) ? leader1 : leader0;
            const int64_t ns = sh->n_send_lo + sh->n_send_hi;
            if (ns) {
                hipLaunchKernelGGL(k_pack, dim3(grid_for(ns, kBlock, 1024)), dim3(kBlock), 0, s, Lcur, sh->send_lo,
                                   sh->n_send_lo, sh->send_hi, sh->n_send_hi, s_lo, s_hi);
                SW_LAUNCHED();
            }
            SW_NCCL(R.groupStart());
            if (sh->peer_lo >= 0) {
                if (sh->n_send_lo) SW_NCCL(R.send(s_lo, size_t(sh->n_send_lo), ncclInt32, sh->peer_lo, comm->comm, s));
                if (sh->n_ghost_lo) SW_NCCL(R.recv(r_lo, size_t(sh->n_ghost_lo), ncclInt32, sh->peer_lo, comm->comm, s));
            }
            if (sh->peer_hi >= 0) {
                if (sh->n_send_hi) SW_NCCL(R.send(s_hi, size_t(sh->n_send_hi), ncclInt32, sh->peer_hi, comm->comm, s));
                if (sh->n_ghost_hi) SW_NCCL(R.recv(r_hi, size_t(sh->n_ghost_hi), ncclInt32, sh->peer_hi, comm->comm, s));
            }
            SW_NCCL(R.groupEnd());
            if ((rc = frontier_ghosts_both(ctx, r, sh->row_ptr, sh->col, sh->ghost_lo_begin, sh->n_ghost_lo, r_lo,
                                           sh->ghost_hi_begin, sh->n_ghost_hi, r_hi, leader0, leader1, s)))
                return rc;
        }
        const int nr = tend - t + 1;
        if ((rc = frontier_round_totals(ctx, t, tend, dtot, s))) return rc;
        SW_NCCL(R.allReduce(dtot, dtot, size_t(nr) * kC, ncclUint64, ncclSum, comm->comm, s));
        SW_HIP(hipMemcpyAsync(h, dtot, size_t(nr) * kC * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        for (int r = t; r <= tend; ++r) {
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
