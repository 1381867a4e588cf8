// Shared host/device plumbing for libswarm.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/swarm.h"

namespace swarm {

constexpr int kBlock = 256;   // threads per workgroup: 4 waves of 64
constexpr int kWave = 64;
constexpr int kElectCounters = 4;  // per-round election counters (elect.hip C_CHG..C_GHOST)

void set_error(const char *fmt, ...);

// Scratch slots owned by a ctx; each grows on demand (never shrinks until destroy).
enum Slot {
    S_LEADER_B = 0,   // election: second leader buffer (dense)
    S_ACT,            // election: per-agent append stamp (frontier)
    S_LIST,           // election: change lists, both round parities (frontier)
    S_CHANGES,        // election: per-round change counters (device)
    S_ESTATS,         // election: per-round active/edge counters (device)
    S_KEYS_IN,        // binning: cell keys
    S_KEYS_OUT,
    S_VALS_IN,        // binning: agent indices
    S_VALS_OUT,
    S_CELL_START,
    S_CELL_END,
    S_CUB_TMP,        // hipcub temporary storage
    S_BBOX,           // bounding box (device)
    S_ASTATS,         // allocation counters (device)
    S_DEG,            // graph builder: degrees
    S_TILEMAX,        // dense allocation: per (task, agent tile) max claim
    S_ORDER,          // dense allocation: agents in ascending ID order
    S_TMP0,
    S_TMP1,
    S_AUC_OFF,        // auction: candidate-list offsets (int64, n + 1)
    S_AUC_K,          // auction: candidate tasks
    S_AUC_V,          // auction: candidate values (f32)
    S_AUC_OUT,        // auction: dropped-out flags
    S_AUC_KEY,        // auction: per-task bid keys (u64)
    S_AUC_LIST,       // auction: bidder lists, targets, keys, counters, per-round log
    S_FSM_MAIL,       // protocol: mail bitmap (1 bit per agent) + list counters
    S_FSM_LIST,       // protocol: receivers of the current tick
    S_FSM_FROM,       // protocol: each receiver's sender when it has exactly one
    S_FSM_SEND,       // protocol: per-workgroup sender segments + counts
    S_DEFER,          // allocation: guard-band tasks deferred to the libm pass (list + per-task flags)
    S_FPAIRS,         // allocation: the deferred tasks' guard-band pairs (device -> host)
    S_OVR,            // allocation: host libm decisions for those pairs (host -> device)
    S_ENC_FLAGS,      // codec: tile ticket + per-tile look-back words (kept across calls, tagged by epoch)
    S_CHECK,          // election: the 16-bit column check's verdict word
    S_FSM_FLAGS,      // protocol: per-agent records of a run (flag word + timer tick; leader + leader position)
    S_NUM
};

}  // namespace swarm

namespace swarm {
// Sharded auction state kept between swarm_auction_begin and the per-round calls (pointers into
// this ctx's scratch slots; see auction.hip).
struct AucPersist {
    int64_t n = 0, t = 0, npairs = 0;
    float eps = 0.f;
    const int32_t *ids = nullptr;
    int64_t *off = nullptr;
    int32_t *ck = nullptr;
    float *cv = nullptr;
    uint32_t *sorted_ids = nullptr;
    int32_t *order = nullptr;
    uint8_t *out = nullptr;
    unsigned long long *ring = nullptr;
    bool ready = false;
};
}  // namespace swarm

struct swarm_ctx {
    swarm::AucPersist auc;         // sharded auction between begin and the round calls
    int device = 0;
    void *slot[swarm::S_NUM] = {};
    size_t cap[swarm::S_NUM] = {};
    void *host_pinned = nullptr;   // small pinned staging buffer for scalar/array readback
    size_t host_cap = 0;
    void *host_mapped = nullptr;   // coherent mapped host buffer the device writes (election read-back)
    void *mapped_dev = nullptr;
    size_t mapped_cap = 0;
    int64_t step_rows = 0;         // frontier stepper: owned rows / agents (rows + ghosts)
    int64_t step_all = 0;
    int64_t step_lo = 0;           // frontier stepper: the owned rows are [step_lo, step_lo + step_rows)
    const int16_t *step_c16 = nullptr;  // frontier stepper: 16-bit columns of the shard graph, or NULL
    bool step_c16_esc = false;          // step_c16 holds escapes (read through the int32 columns)
    bool step_c16_checked = false;      // step_c16 passed the column check against the stepped graph
    std::vector<const int16_t *> esc_built;  // column buffers swarm_graph_compact_escaped last wrote
    struct C16Built {                        // column buffers swarm_graph_compact last wrote (all deltas fit)
        const int16_t *c16;
        const void *rp;
        const int32_t *col;
        int64_t n, e_total;
    };
    std::vector<C16Built> c16_built;
    int step_rd_agent = 0;         // frontier stepper: the marks the next round reads are in agent order
    int step_wr_agent = 0;         // ... and the next round writes its marks in agent order (the tail)
    hipStream_t side = nullptr;    // a second stream for work that overlaps the caller's (side_stream)
    hipEvent_t side_ev[2] = {};    // fork / join events
    void *enc_flags = nullptr;     // codec one-pass encode: the S_ENC_FLAGS buffer last zeroed ...
    size_t enc_cap = 0;            // ... and its size
    uint32_t enc_epoch = 0;        // ... the epoch tag of the last call (look-back words carry it)
    unsigned long long fold_epoch = 0;  // allocation: the last epoch k_fold_stats wrote to mapped memory
};

namespace swarm {

int comm_allreduce_max_u64(swarm_comm *comm, unsigned long long *buf, size_t count, hipStream_t s);
int comm_allgather_u64(swarm_comm *comm, const unsigned long long *send, size_t count, unsigned long long *recv,
                       hipStream_t s);
int comm_rank(const swarm_comm *comm, int *rank, int *nranks);

// Returns a device buffer of at least `bytes` for `s` (nullptr + error on failure: the ctx
// belongs to another device -> scratch_code() SWARM_ERR_ARG, else SWARM_ERR_OOM).
void *scratch(swarm_ctx *ctx, Slot s, size_t bytes);
int scratch_code();
bool ctx_on_current_device(const swarm_ctx *ctx);
void *pinned(swarm_ctx *ctx, size_t bytes);
// The ctx's side stream and a fork / join event pair (created on first use, on the ctx's device):
// record fork on the caller's stream, wait for it on *side, launch there, record join on *side,
// wait for join on the caller's stream.
int side_stream(swarm_ctx *ctx, hipStream_t *side, hipEvent_t *fork, hipEvent_t *join);
void *mapped(swarm_ctx *ctx, size_t bytes, void **dev);
// Host wait for a device-written word of mapped memory to equal v (a spin: a waiting host thread stays
// on its core, where a stream / event synchronisation may yield it -- and the next call's launches then
// start from a cold core); hipStreamQuery every 256 spins reports a failed stream, and a stream that
// finished without the write is an error.
int wait_mapped_word(const unsigned long long *w, unsigned long long v, hipStream_t s, const char *what);

}  // namespace swarm

#define SW_HIP(call)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            swarm::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,                \
                             hipGetErrorString(e_));                                     \
            return SWARM_ERR_HIP;                                                        \
        }                                                                                \
    } while (0)

#define SW_ARG(cond, msg)                                                                \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            swarm::set_error("invalid argument: %s", msg);                               \
            return SWARM_ERR_ARG;                                                        \
        }                                                                                \
    } while (0)

#define SW_ALLOC(ptr, ctx, slot, bytes)                                                  \
    do {                                                                                 \
        (ptr) = static_cast<std::remove_reference_t<decltype(ptr)>>(swarm::scratch((ctx), (slot), (bytes)));      \
        if (!(ptr)) return swarm::scratch_code();                                        \
    } while (0)

// Launch-error check after a kernel launch.
#define SW_LAUNCHED() SW_HIP(hipGetLastError())

namespace swarm {

// Rounds in the next batch of an election loop (launched before the host reads their counts):
// double up to max_batch, but no more than ~1.5x the rounds a linear extrapolation of the last
// 32 per-round change counts leaves before zero -- rounds launched past convergence are wasted
// no-op launches (~8 us each at 10M agents; 164 of them at C3, 106 at C2 with pure doubling).
inline int next_round_batch(const int64_t *hist, size_t nh, int batch, int max_batch) {
    int b = batch * 2 < max_batch ? batch * 2 : max_batch;
    constexpr size_t k = 32;
    static const bool doubling_only = [] {  // SWARM_BATCH_DOUBLING=1: plain doubling (A/B aid)
        const char *e = getenv("SWARM_BATCH_DOUBLING");
        return e && e[0] == '1';
    }();
    if (nh >= k && !doubling_only) {
        const double slope = double(hist[nh - k] - hist[nh - 1]) / double(k - 1);
        if (slope > 0) {
            // rounds left on the linear trend, + 25 % and 4 rounds of margin: an overshoot costs one
            // no-op launch per round (~6 µs), an undershoot one more host round trip
            const double rem = 1.25 * double(hist[nh - 1]) / slope + 4.0;
            const int p = rem < 8.0 ? 8 : (rem > double(max_batch) ? max_batch : int(rem + 0.5));
            if (p < b) b = p;
        }
    }
    return b;
}

// Grid for a grid-stride kernel over `work` items with `per_block` items per block pass.
inline unsigned grid_for(int64_t work, int64_t per_block, unsigned cap = 8192) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<unsigned>(g);
}

}  // namespace swarm
