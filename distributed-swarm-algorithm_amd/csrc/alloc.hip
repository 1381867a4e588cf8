// Task allocation round (contract A-H) on gfx950.
//
// Replaces, batched over every agent and task:
//   _process_tasks + _calculate_utility (agent.py:292-302, 338-347): claim iff U > 20.0 (fp64),
//       claim value x = f32(U) (struct '!If', round-to-nearest-even);
//   _handle_task_claim (agent.py:304-325) at the resolver, claims in ascending sender ID:
//       first claim wins, a later one wins iff x > u_cur + 5.0; every accepted claim and every
//       rejected claim from a non-incumbent emits one TASK_CONFLICT;
//   _handle_task_conflict (agent.py:327-336): winner ASSIGNED, everyone else LOCKED (derived
//       from winner / nmsg, never materialised as an N x T matrix).
//
// The chain is NOT argmax: with hysteresis h the winner is the end of the "record chain"
//   c1 = min-ID claim (or min-ID claim with x > u0 + h if the task already had a winner),
//   c_{k+1} = min-ID claim with ID > id(c_k) and x > x(c_k) + h.
// Each link is one workgroup-wide min-ID reduction over the task's claims held in LDS; with
// x in (thr, u_scale] and h = 5 there are at most 17 links.  h = 0 gives argmax with the
// lowest-ID tie-break (the north star's "wavefront argmin" mode) through the same code.
//
// BINNED (exact): U > thr <=> d < Rc = u_scale/thr - 1 (has_cap), so only agents inside a
// slightly larger radius Rp can claim.  Agents are bucketed in a uniform grid (hipCUB radix
// sort); one workgroup per task walks the 2-3 grid rows its Rp-disc covers, evaluates U in
// fp64 (no FMA contraction: matches the reference's separately rounded squares), appends
// claims to LDS, then walks the chain.  Per task ~pi*Rp^2*density candidates instead of N.
// DENSE: agents in ascending-ID tiles of 256; each workgroup stages 64 tasks in LDS and
// records, per (task, tile), the max claim value and claim count; the chain then walks
// tiles (ballot over tile maxima) and re-evaluates only the one tile a link lands in.
#include "binning.h"
#include "utility.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

namespace swarm {
namespace {

__device__ __forceinline__ long long block_sum_ll(long long v, long long *s_red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    long long m = 0;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) m += s_red[w];
    return m;
}

// Guard-band resolution.  The reference squares with libm pow (agent.py:340);
// the device squares with x*x.  A task with ANY candidate pair inside the guard band (guard_flag)
// is not finished by the main pass: it is appended to a deferred list, its guard-band pairs are
// collected (PASS_COLLECT) and handed to the host, which decides them with the host's libm pow
// exactly as agent.py:340/297/302 do, and the deferred tasks are then resolved once (PASS_RESOLVE)
// with those decisions in place of the device's for exactly those pairs.
struct FlagPair {            // device -> host
    double ax, ay, tx, ty;
    int32_t j;               // position of the task in the deferred list
    int32_t agent;           // storage index
    int32_t has;             // has_cap (agent.py:343-345)
    int32_t pad;
};
struct Override {            // host -> device, sorted by (j, agent)
    int32_t agent;
    float x;                 // f32(U_ref): the claim payload (agent.py:302)
    int32_t claim;           // U_ref > claim_thr (agent.py:297)
    int32_t pad;
};
struct Defer {
    int32_t *list = nullptr;               // deferred task indices
    unsigned long long *count = nullptr;   // [0] deferred tasks, [1] guard-band pairs collected
    uint8_t *tflag = nullptr;              // dense strategy: tasks with a guard-band pair
    FlagPair *pairs = nullptr;
    int64_t pair_cap = 0;
    const uint32_t *ov_off = nullptr;      // deferred task j: overrides [ov_off[j], ov_off[j + 1])
    const Override *ov = nullptr;
};

struct Params {
    double thr, h, u_scale, rp2;
    int32_t *winner;
    double *util;
    int32_t *won;
    const int32_t *id_to_index;
    int64_t id_span;
    int64_t *nclaim;
    int64_t *nmsg;
    unsigned long long *stats;  // kStatShards x 16 u64: [claims, conflicts, flagged, candidates, overflow, bad treq]
    Defer D;
};

// candidate sources of the per-task wave kernel
constexpr int SRC_HASH = 0;  // hashed cell buckets (swarm_allocate, BINNED)
constexpr int SRC_ROWS = 1;  // the caller's cell index over the storage order (swarm_allocate_indexed)
constexpr int SRC_ALL = 2;   // every agent (the dense strategy's deferred tasks)
// passes
constexpr int PASS_MAIN = 0;     // every task; guard-band tasks deferred when P.D.list is set
constexpr int PASS_COLLECT = 1;  // deferred tasks: append their guard-band pairs
constexpr int PASS_RESOLVE = 2;  // deferred tasks: claims with the host's decisions, chain, finish

__device__ __forceinline__ void apply_override(const Params &P, uint32_t a, uint32_t b, int32_t agent, bool &claim,
                                               float &x) {
    for (uint32_t q = a; q < b; ++q) {
        const Override o = P.D.ov[q];
        if (o.agent == agent) {
            claim = o.claim != 0;
            x = o.x;
            return;
        }
    }
}

constexpr int kStatShards = 64;   // each shard on its own 128-B line
constexpr int kStatStride = 16;

// Per-workgroup totals, flushed once per workgroup into one of 64 shards (a single
// contended counter costs ~12 ns per arrival: MI355X_MICROARCH.md 'fanin').
struct BlockStats {
    unsigned long long claims = 0, msgs = 0, overflow = 0, bad = 0;
};
// + [6]: agents with a non-finite position (hashed binning), [7]: agents outside their cell's range
// (swarm_allocate_indexed: the index is stale)
constexpr int kNumStats = 8;

__device__ __forceinline__ void flush_stats(const Params &P, unsigned long long claims, unsigned long long msgs,
                                            unsigned long long flagged, unsigned long long cand,
                                            unsigned long long overflow, unsigned long long bad = 0) {
    unsigned long long *sh = P.stats + size_t(blockIdx.x & (kStatShards - 1)) * kStatStride;
    if (bad) atomicAdd(sh + 5, bad);
    if (claims) atomicAdd(sh + 0, claims);
    if (msgs) atomicAdd(sh + 1, msgs);
    if (flagged) atomicAdd(sh + 2, flagged);
    if (cand) atomicAdd(sh + 3, cand);
    if (overflow) atomicAdd(sh + 4, overflow);
}

// One launch before a round: the stat shards, the deferred counters and won zeroed; with a fresh
// claim table (SWARM_ALLOC_FRESH_CLAIMS, winner != NULL here) every task's winner / util too.
__global__ __launch_bounds__(kBlock) void k_alloc_init(unsigned long long *__restrict__ stats,
                                                      unsigned long long *__restrict__ dcount,
                                                      int32_t *__restrict__ won, int64_t n,
                                                      int32_t *__restrict__ winner, double *__restrict__ util,
                                                      int64_t t) {
    const int64_t i0 = int64_t(blockIdx.x) * kBlock + threadIdx.x, stride = int64_t(gridDim.x) * kBlock;
    for (int64_t i = i0; i < int64_t(kStatShards) * kStatStride; i += stride) stats[i] = 0;
    if (i0 == 0) dcount[0] = dcount[1] = 0;
    if (won)
        for (int64_t i = i0; i < n; i += stride) won[i] = 0;
    if (winner)
        for (int64_t i = i0; i < t; i += stride) {
            winner[i] = -1;
            util[i] = 0.0;
        }
}

// out[0, kNumStats): the shard sums; out[kNumStats] = *dcount (the deferred tasks) when given.  out may
// be host-mapped memory (the round's stats reach the host without a copy).
// done / epoch: the host's wait word (mapped host memory) -- written last, after a system-scope fence,
// so that a host that sees the epoch sees every folded value.
__global__ void k_fold_stats(const unsigned long long *__restrict__ sh, unsigned long long *__restrict__ out,
                             const unsigned long long *__restrict__ dcount = nullptr,
                             unsigned long long *__restrict__ done = nullptr, unsigned long long epoch = 0) {
    for (int c = 0; c < kNumStats; ++c) {
        unsigned long long v = sh[size_t(threadIdx.x) * kStatStride + c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) out[c] = v;
    }
    if (dcount && threadIdx.x == 0) out[kNumStats] = *dcount;
    if (done && threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(done, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Per-task epilogue shared by both strategies.
__device__ __forceinline__ void finish_task(const Params &P, int64_t k, int w0, double u0, bool w0_claimed,
                                            int accepted, int first_id, int cur_id, double cur_u,
                                            int cur_idx, long long nclaims, BlockStats &bs) {
    const long long msgs = nclaims - ((w0 >= 0 && w0_claimed && (accepted == 0 || w0 < first_id)) ? 1 : 0);
    if (accepted > 0) {
        P.winner[k] = cur_id;
        P.util[k] = cur_u;
        if (P.won) atomicAdd(&P.won[cur_idx], 1);
    } else if (w0 >= 0 && P.won && P.id_to_index && w0 < P.id_span) {
        const int ix = P.id_to_index[w0];
        if (ix >= 0) atomicAdd(&P.won[ix], 1);
    }
    if (P.nclaim) P.nclaim[k] = nclaims;
    if (P.nmsg) P.nmsg[k] = msgs;
    bs.claims += (unsigned long long)nclaims;
    bs.msgs += (unsigned long long)msgs;
}

// ------------------------------------------------------------------------ hashed cells
// BINNED candidates: agents bucketed by grid cell of side Rp, cells hashed into 2^k buckets (no
// bounding box, so no device -> host round trip before the launch).  A task's Rp-disc covers at
// most 3 x 3 cells; an agent is visited under its own cell only (its cell is recomputed and
// compared), so cells sharing a bucket are never double counted.  Bucket = counting sort: one
// wave-aggregated atomic per (wave, bucket) for the counts and in-bucket ranks, a hipCUB scan,
// one scatter.  Order inside a bucket is arbitrary: the claims are collected in LDS and the
// record chain picks by ID.
struct HashGrid {
    double inv_cell;
    uint32_t mask;  // buckets - 1 (power of two)
};

constexpr double kCellClamp = 1e15;  // cells beyond +-1e15 merge (the distance test still decides)

__device__ __forceinline__ int64_t hcell(double v, double inv) {
    double f = floor(v * inv);
    if (!(f >= -kCellClamp)) f = -kCellClamp;  // also NaN
    if (f > kCellClamp) f = kCellClamp;
    return int64_t(f);
}

__device__ __forceinline__ uint32_t hbucket(int64_t cx, int64_t cy, uint32_t mask) {
    uint64_t h = uint64_t(cx) * 0x9E3779B97F4A7C15ull ^ (uint64_t(cy) + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= h >> 32;
    h *= 0xD6E8FEB86659FD93ull;
    return uint32_t(h >> 32) & mask;
}

// Counts per bucket and each agent's rank in its bucket.  Agents in spatial storage order put a
// wave's 64 lanes in a few cells: one atomic per distinct bucket of the wave.
__global__ __launch_bounds__(kBlock) void k_hash_count(const double2 *__restrict__ apos, int64_t n, HashGrid hg,
                                                      uint32_t *__restrict__ cnt, uint32_t *__restrict__ key,
                                                      uint32_t *__restrict__ rank,
                                                      unsigned long long *__restrict__ nonfinite) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = int64_t(gridDim.x) * kBlock;
    unsigned long long bad = 0;
    for (int64_t base = int64_t(blockIdx.x) * kBlock + (threadIdx.x & ~63); base < n; base += stride) {
        const int64_t i = base + lane;
        const bool valid = i < n;
        uint32_t k = 0;
        if (valid) {
            const double2 p = apos[i];
            bad += (isfinite(p.x) && isfinite(p.y)) ? 0 : 1;
            k = hbucket(hcell(p.x, hg.inv_cell), hcell(p.y, hg.inv_cell), hg.mask);
        }
        // group the wave's lanes by bucket (no memory traffic), then ONE atomic instruction: every
        // group's first lane adds its group size, and each lane's rank = group base + lanes of its
        // group below it
        uint32_t lead = 0, gsize = 0, below = 0;
        unsigned long long todo = __ballot(valid);
        while (todo) {
            const int l = __ffsll((long long)todo) - 1;
            const uint32_t lk = __shfl(k, l, 64);
            const unsigned long long same = __ballot(valid && k == lk) & todo;
            if ((same >> lane) & 1ull) {
                lead = uint32_t(l);
                gsize = uint32_t(__popcll(same));
                below = uint32_t(__popcll(same & ((1ull << lane) - 1ull)));
            }
            todo &= ~same;
        }
        uint32_t b = 0;
        if (valid && lead == uint32_t(lane)) b = atomicAdd(&cnt[k], gsize);
        const uint32_t r = __shfl(b, int(lead), 64) + below;
        if (valid) {
            key[i] = k;
            rank[i] = r;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) bad += __shfl_xor(bad, off, 64);
    if (lane == 0 && bad) atomicAdd(nonfinite, bad);
}

__global__ __launch_bounds__(kBlock) void k_hash_scatter(int64_t n, const uint32_t *__restrict__ key,
                                                        const uint32_t *__restrict__ rank,
                                                        const uint32_t *__restrict__ off,
                                                        int32_t *__restrict__ sorted) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        sorted[off[key[i]] + rank[i]] = int32_t(i);
}

// A task's cell window (at most 4 x 4 cells; 3 x 3 in practice: the window is 2 Rp wide with
// cells of side Rp) as one flat candidate range: cell j holds bucket entries
// [a[j], a[j] + pre[j+1] - pre[j]), its coordinates are (cx[j], cy[j]).  Built by the task's wave.
constexpr int kMaxCells = 16;
struct CellWindow {
    uint32_t a[kMaxCells], pre[kMaxCells + 1];
    int64_t cx[kMaxCells], cy[kMaxCells];
    int ncell;
};

__device__ __forceinline__ void window_setup(double2 tp, double rp, const HashGrid &hg,
                                             const uint32_t *__restrict__ off, CellWindow &w, int lane) {
    const int64_t x0 = hcell(tp.x - rp, hg.inv_cell), y0 = hcell(tp.y - rp, hg.inv_cell);
    int64_t x1 = hcell(tp.x + rp, hg.inv_cell), y1 = hcell(tp.y + rp, hg.inv_cell);
    if (x1 > x0 + 3) x1 = x0 + 3;  // never taken (see above): a guard on the table size
    if (y1 > y0 + 3) y1 = y0 + 3;
    const int wx = int(x1 - x0 + 1), nc = wx * int(y1 - y0 + 1);
    uint32_t len = 0;
    if (lane < nc) {
        const int64_t cx = x0 + lane % wx, cy = y0 + lane / wx;
        const uint32_t b = hbucket(cx, cy, hg.mask);
        const uint32_t a = off[b];
        len = off[b + 1] - a;
        w.a[lane] = a;
        w.cx[lane] = cx;
        w.cy[lane] = cy;
    }
    uint32_t incl = len;  // inclusive prefix of the lengths
#pragma unroll
    for (int o = 1; o < kMaxCells; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, 64);
        if (lane >= o) incl += x;
    }
    if (lane < kMaxCells) w.pre[lane + 1] = incl;
    if (lane == 0) {
        w.pre[0] = 0;
        w.ncell = nc;
    }
    __builtin_amdgcn_wave_barrier();
}

// The same window over a caller's cell index (swarm_cell_index: agents stored in row-major cell
// order, cell side <= the claim radius allows): one entry per grid ROW the window covers, the
// contiguous storage range of its cells x0..x1 -- no binning pass, no per-candidate cell test.
__device__ __forceinline__ void window_setup_rows(double2 tp, double rp, const Grid &g,
                                                  const uint32_t *__restrict__ off, CellWindow &w, int lane) {
    const bool miss = tp.x + rp < g.xmin || tp.x - rp > g.xmax || tp.y + rp < g.ymin || tp.y - rp > g.ymax;
    const int64_t x0 = cell_coord(tp.x - rp, g.xmin, g.inv_cell, g.ncx);
    const int64_t x1 = cell_coord(tp.x + rp, g.xmin, g.inv_cell, g.ncx);
    const int64_t y0 = cell_coord(tp.y - rp, g.ymin, g.inv_cell, g.ncy);
    int64_t y1 = cell_coord(tp.y + rp, g.ymin, g.inv_cell, g.ncy);
    if (y1 > y0 + kMaxCells - 1) y1 = y0 + kMaxCells - 1;  // the host checks rows <= kMaxCells
    const int nc = miss ? 0 : int(y1 - y0 + 1);
    uint32_t len = 0;
    if (lane < nc) {
        const int64_t row = (y0 + lane) * g.ncx;
        const uint32_t a = off[row + x0];
        len = off[row + x1 + 1] - a;
        w.a[lane] = a;
    }
    uint32_t incl = len;
#pragma unroll
    for (int o = 1; o < kMaxCells; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, 64);
        if (lane >= o) incl += x;
    }
    if (lane < kMaxCells) w.pre[lane + 1] = incl;
    if (lane == 0) {
        w.pre[0] = 0;
        w.ncell = nc;
    }
    __builtin_amdgcn_wave_barrier();
}

// Every agent as one candidate range (the dense strategy's deferred tasks).
__device__ __forceinline__ void window_setup_all(int64_t n, CellWindow &w, int lane) {
    if (lane == 0) {
        w.a[0] = 0;
        w.pre[0] = 0;
        w.pre[1] = uint32_t(n);
        w.ncell = 1;
    }
    __builtin_amdgcn_wave_barrier();
}

constexpr int kCheckPer = 4;  // agents per thread in flight (k_check_index)

// Staleness test of a cell index: every agent must lie in its cell's range AND inside the indexed
// bounding box.  cell_coord clamps, so an edge-cell agent that moved past [xmin, xmax] x [ymin,
// ymax] still maps to its old cell; window_setup_rows skips every task whose disc misses that box,
// so such an agent would lose its claims silently.  k_check_index runs on the ctx's side stream,
// concurrently with the indexed allocation (it streams the positions while the task waves wait on
// their dependent loads); the host reads the count with the folded stats and reports
// SWARM_ERR_STALE (outputs undefined) instead of the results.
__global__ __launch_bounds__(kBlock) void k_check_index(const double2 *__restrict__ apos, int64_t n, Grid g,
                                                       const uint32_t *__restrict__ off,
                                                       unsigned long long *__restrict__ bad_out) {
    unsigned long long bad = 0;
    const int64_t stride = int64_t(gridDim.x) * kBlock * kCheckPer;
    for (int64_t i0 = int64_t(blockIdx.x) * kBlock * kCheckPer + threadIdx.x; i0 < n; i0 += stride) {
        double2 p[kCheckPer];
#pragma unroll
        for (int j = 0; j < kCheckPer; ++j) {
            const int64_t i = i0 + int64_t(j) * kBlock;
            p[j] = apos[i < n ? i : n - 1];
        }
        uint32_t lo[kCheckPer], hi[kCheckPer];
        bool inside[kCheckPer];
#pragma unroll
        for (int j = 0; j < kCheckPer; ++j) {
            const int64_t c = cell_coord(p[j].y, g.ymin, g.inv_cell, g.ncy) * g.ncx +
                              cell_coord(p[j].x, g.xmin, g.inv_cell, g.ncx);
            inside[j] = p[j].x >= g.xmin && p[j].x <= g.xmax && p[j].y >= g.ymin && p[j].y <= g.ymax;  // false for NaN
            lo[j] = off[c];
            hi[j] = off[c + 1];
        }
#pragma unroll
        for (int j = 0; j < kCheckPer; ++j) {
            const int64_t i = i0 + int64_t(j) * kBlock;
            if (i < n) bad += (inside[j] && lo[j] <= uint32_t(i) && uint32_t(i) < hi[j]) ? 0 : 1;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(bad_out, bad);
}

// ------------------------------------------------------------------------------ binned
// One WAVE per task (4 tasks per workgroup): pass 1 evaluates the window's candidates, kWU per
// lane with all their loads in flight, and keeps the claims in the wave's LDS list (ballot
// slots, no atomics); pass 2 walks the record chain with wave-wide min-ID reductions.  A task is
// latency-bound (dependent loads, then the chain), so the point is tasks in flight: 32 per CU.
#ifndef SWARM_ALLOC_WCAP  // A/B builds (tools/build_variant_alloc.sh) override these two
#define SWARM_ALLOC_WCAP 512
#endif
#ifndef SWARM_ALLOC_WU
#define SWARM_ALLOC_WU 4
#endif
constexpr int kWCap = SWARM_ALLOC_WCAP;  // claims per task kept in LDS (beyond: exact recompute path; C3 max ~350)
constexpr int kWU = SWARM_ALLOC_WU;      // candidates in flight per lane

__device__ __forceinline__ int wave_min_int(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    return v;
}

// SRC: where a task's candidates come from (SRC_HASH: the hashed buckets sorted_idx / bucket_off /
// hg; SRC_ROWS: a cell index over the storage order, bucket_off = cell_off over grid g; SRC_ALL:
// every agent).  PASS: see PASS_MAIN / PASS_COLLECT / PASS_RESOLVE.  In the COLLECT and RESOLVE
// passes the wave's task is P.D.list[kk] (kk < t_count = the deferred count).
template <int SRC, int PASS>
__global__ __launch_bounds__(kBlock) void k_alloc_binned(
    int64_t t_count, const double2 *__restrict__ tpos, const int8_t *__restrict__ treq,
    const int32_t *__restrict__ ids, const double2 *__restrict__ apos,
    const uint32_t *__restrict__ caps, const int32_t *__restrict__ sorted_idx,
    const uint32_t *__restrict__ bucket_off, HashGrid hg, Grid g, double rp, int64_t n_all, Params P) {
    constexpr int kW = kBlock / kWave;
    constexpr bool HASH = SRC == SRC_HASH;
    __shared__ int s_id[kW][kWCap];
    __shared__ float s_x[kW][kWCap];
    __shared__ int s_ix[kW][kWCap];
    __shared__ CellWindow s_win[kW];
    __shared__ long long s_red64[kW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int *cid = s_id[wid], *cix = s_ix[wid];
    float *cxv = s_x[wid];
    CellWindow &w = s_win[wid];
    const unsigned long long below = (1ull << lane) - 1ull;
    long long my_cand = 0, my_flag = 0;
    BlockStats bs;
    const int64_t nw = int64_t(gridDim.x) * kW;
    for (int64_t kk = int64_t(blockIdx.x) * kW + wid; kk < t_count; kk += nw) {
        const int64_t k = PASS == PASS_MAIN ? kk : int64_t(P.D.list[kk]);
        const double2 tp = tpos[k];
        const int rq = treq[k];
        const int w0 = P.winner[k];
        const double u0 = P.util[k];
        uint32_t ov_a = 0, ov_b = 0;
        if (PASS == PASS_RESOLVE) {
            ov_a = P.D.ov_off[kk];
            ov_b = P.D.ov_off[kk + 1];
        }
        int nclaims = 0;
        bool w0c = false, tflag = false;
        uint32_t total = 0;
        if (P.rp2 >= 0.0) {
            if (SRC == SRC_HASH)
                window_setup(tp, rp, hg, bucket_off, w, lane);
            else if (SRC == SRC_ROWS)
                window_setup_rows(tp, rp, g, bucket_off, w, lane);
            else
                window_setup_all(n_all, w, lane);
            total = w.pre[w.ncell];
        }
        // pass 1: evaluate candidates, keep claims in LDS
        for (uint32_t q0 = 0; q0 < total; q0 += 64 * kWU) {
            int32_t ii[kWU];
            int jj[kWU];
#pragma unroll
            for (int u = 0; u < kWU; ++u) {
                const uint32_t q = q0 + u * 64 + lane;
                int j = 0;
                while (j + 1 < w.ncell && w.pre[j + 1] <= q) ++j;
                jj[u] = q < total ? j : -1;
                const uint32_t e = q < total ? w.a[j] + (q - w.pre[j]) : 0;
                ii[u] = HASH ? sorted_idx[e] : int32_t(e);
            }
            double2 p[kWU];
            uint32_t cp[kWU];
            int32_t idv[kWU];
#pragma unroll
            for (int u = 0; u < kWU; ++u) {
                p[u] = apos[ii[u]];
                cp[u] = caps[ii[u]];
                idv[u] = ids[ii[u]];
            }
#pragma unroll
            for (int u = 0; u < kWU; ++u) {
                bool claim = false, fl = false;
                float x = 0.f;
                const int j = jj[u];
                if (j >= 0 && (!HASH || (hcell(p[u].x, hg.inv_cell) == w.cx[j] &&
                                         hcell(p[u].y, hg.inv_cell) == w.cy[j]))) {
                    const double dx = p[u].x - tp.x, dy = p[u].y - tp.y;
                    if (dx * dx + dy * dy <= P.rp2) {
                        if (PASS == PASS_MAIN) ++my_cand;
                        const double U = utility(p[u].x, p[u].y, cp[u], tp.x, tp.y, rq, P.u_scale);
                        fl = guard_flag(U, P.thr);
                        if (PASS == PASS_MAIN) my_flag += fl;
                        claim = U > P.thr;
                        x = float(U);
                        if (PASS == PASS_RESOLVE && fl) apply_override(P, ov_a, ov_b, ii[u], claim, x);
                        if (PASS == PASS_COLLECT && fl) {
                            const unsigned long long slot = atomicAdd(P.D.count + 1, 1ull);
                            if (slot < (unsigned long long)P.D.pair_cap) {
                                const bool has = rq < 0 || (rq < 32 && ((cp[u] >> rq) & 1u));
                                P.D.pairs[slot] = FlagPair{p[u].x, p[u].y, tp.x, tp.y, int32_t(kk), ii[u],
                                                           has ? 1 : 0, 0};
                            }
                        }
                    }
                }
                if (PASS == PASS_COLLECT) continue;
                if (PASS == PASS_MAIN) tflag = tflag || __ballot(fl) != 0ull;
                const unsigned long long bm = __ballot(claim);
                if (claim) {
                    const int slot = nclaims + __popcll(bm & below);
                    if (slot < kWCap) {
                        cid[slot] = idv[u];
                        cxv[slot] = x;
                        cix[slot] = ii[u];
                    }
                }
                w0c = w0c || __ballot(claim && idv[u] == w0) != 0ull;
                nclaims += __popcll(bm);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (PASS == PASS_COLLECT) continue;
        if (PASS == PASS_MAIN && tflag && P.D.list) {  // the libm pass decides this task
            if (lane == 0) {
                const unsigned long long slot = atomicAdd(P.D.count, 1ull);
                P.D.list[slot] = int32_t(k);
                bs.bad += bad_req(rq) ? 1 : 0;
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        const bool overflow = nclaims > kWCap;
        // pass 2: the record chain
        int prev = -1, cur_id = w0, cur_idx = -1, accepted = 0, first_id = -1;
        bool has = w0 >= 0;
        double cur_u = u0;
        for (;;) {
            int best = INT_MAX, best_ix = -1;
            float best_x = 0.f;
            if (!overflow) {
                for (int j = lane; j < nclaims; j += 64) {
                    const int id = cid[j];
                    if (id > prev && id < best && (!has || double(cxv[j]) > cur_u + P.h)) {
                        best = id;
                        best_x = cxv[j];
                        best_ix = cix[j];
                    }
                }
            } else {  // exact recompute over the candidates (rare: > kWCap claims on one task)
                for (uint32_t q = lane; q < total; q += 64) {
                    int j = 0;
                    while (j + 1 < w.ncell && w.pre[j + 1] <= q) ++j;
                    const uint32_t e = w.a[j] + (q - w.pre[j]);
                    const int32_t i = HASH ? sorted_idx[e] : int32_t(e);
                    const double2 pp = apos[i];
                    if (HASH && (hcell(pp.x, hg.inv_cell) != w.cx[j] || hcell(pp.y, hg.inv_cell) != w.cy[j]))
                        continue;
                    const double dx = pp.x - tp.x, dy = pp.y - tp.y;
                    if (dx * dx + dy * dy > P.rp2) continue;
                    const double U = utility(pp.x, pp.y, caps[i], tp.x, tp.y, rq, P.u_scale);
                    bool claim = U > P.thr;
                    float x = float(U);
                    if (PASS == PASS_RESOLVE && guard_flag(U, P.thr)) apply_override(P, ov_a, ov_b, i, claim, x);
                    const int id = ids[i];
                    if (claim && id > prev && id < best && (!has || double(x) > cur_u + P.h)) {
                        best = id;
                        best_x = x;
                        best_ix = i;
                    }
                }
            }
            const int win = wave_min_int(best);
            if (win == INT_MAX) break;
            const int src = __ffsll((long long)__ballot(best == win)) - 1;
            cur_u = double(__shfl(best_x, src, 64));
            cur_idx = __shfl(best_ix, src, 64);
            cur_id = win;
            has = true;
            prev = win;
            if (++accepted == 1) first_id = win;
        }
        if (lane == 0) {
            finish_task(P, k, w0, u0, w0c, accepted, first_id, cur_id, cur_u, cur_idx, nclaims, bs);
            bs.overflow += overflow ? 1 : 0;
            if (PASS == PASS_MAIN) bs.bad += bad_req(rq) ? 1 : 0;
        }
        __builtin_amdgcn_wave_barrier();  // the wave's window and claim list are reused
    }
    const long long c = block_sum_ll(my_cand, s_red64);
    const long long f = block_sum_ll(my_flag, s_red64);
    const long long cl = block_sum_ll((long long)bs.claims, s_red64);
    const long long ms = block_sum_ll((long long)bs.msgs, s_red64);
    const long long ov = block_sum_ll((long long)bs.overflow, s_red64);
    const long long bd = block_sum_ll((long long)bs.bad, s_red64);
    if (threadIdx.x == 0)
        flush_stats(P, (unsigned long long)cl, (unsigned long long)ms, (unsigned long long)f, (unsigned long long)c,
                    (unsigned long long)ov, (unsigned long long)bd);
}

// ------------------------------------------------------------------------------- dense
constexpr int kTileA = 256;  // agents per tile (one per thread)
constexpr int kTileT = 64;   // tasks staged in LDS per workgroup

// Agents in ascending-ID order: order[j] = storage index of the j-th smallest ID.
// Per (task k, agent tile a): tmax[k * ntiles + a] = max claim value in the tile (or -inf),
// tcnt likewise the number of claims.
__global__ __launch_bounds__(kBlock) void k_alloc_dense_tiles(
    int64_t n, int64_t t_count, const double2 *__restrict__ tpos, const int8_t *__restrict__ treq,
    const double2 *__restrict__ apos, const uint32_t *__restrict__ caps,
    const int32_t *__restrict__ order, int64_t ntiles, float *__restrict__ tmax,
    int *__restrict__ tcnt, Params P) {
    __shared__ double s_tx[kTileT], s_ty[kTileT];
    __shared__ int s_rq[kTileT];
    __shared__ float s_max[kTileT][kBlock / kWave];
    __shared__ int s_cnt[kTileT][kBlock / kWave];
    __shared__ long long s_red64[kBlock / kWave];
    const int64_t ttiles = (t_count + kTileT - 1) / kTileT;
    long long my_flag = 0;
    for (int64_t blk = blockIdx.x; blk < ntiles * ttiles; blk += gridDim.x) {
        const int64_t at = blk % ntiles, tt = blk / ntiles;
        __syncthreads();
        if (threadIdx.x < kTileT) {
            const int64_t k = tt * kTileT + threadIdx.x;
            const bool ok = k < t_count;
            s_tx[threadIdx.x] = ok ? tpos[k].x : 0.0;
            s_ty[threadIdx.x] = ok ? tpos[k].y : 0.0;
            s_rq[threadIdx.x] = ok ? int(treq[k]) : -1;
        }
        __syncthreads();
        const int64_t j = at * kTileA + threadIdx.x;
        const bool valid = j < n;
        double ax = 0, ay = 0;
        uint32_t c = 0;
        if (valid) {
            const int32_t i = order[j];
            const double2 p = apos[i];
            ax = p.x; ay = p.y; c = caps[i];
        }
        for (int q = 0; q < kTileT; ++q) {
            float x = -INFINITY;
            int claim = 0;
            bool fl = false;
            if (valid) {
                const double U = utility(ax, ay, c, s_tx[q], s_ty[q], s_rq[q], P.u_scale);
                fl = guard_flag(U, P.thr);
                my_flag += fl;
                if (U > P.thr) { x = float(U); claim = 1; }
            }
            // the task has a guard-band pair: the libm pass decides it (idempotent byte store)
            if (P.D.tflag && __ballot(fl) != 0ull && (threadIdx.x & 63) == 0) P.D.tflag[tt * kTileT + q] = 1;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                x = fmaxf(x, __shfl_xor(x, off, 64));
                claim += __shfl_xor(claim, off, 64);
            }
            if ((threadIdx.x & 63) == 0) { s_max[q][threadIdx.x >> 6] = x; s_cnt[q][threadIdx.x >> 6] = claim; }
        }
        __syncthreads();
        if (threadIdx.x < kTileT) {
            const int64_t k = tt * kTileT + threadIdx.x;
            if (k < t_count) {
                float m = s_max[threadIdx.x][0];
                int cc = s_cnt[threadIdx.x][0];
                for (int w = 1; w < kBlock / kWave; ++w) { m = fmaxf(m, s_max[threadIdx.x][w]); cc += s_cnt[threadIdx.x][w]; }
                tmax[k * ntiles + at] = m;
                tcnt[k * ntiles + at] = cc;
            }
        }
    }
    const long long f = block_sum_ll(my_flag, s_red64);
    if (threadIdx.x == 0 && f) flush_stats(P, 0, 0, (unsigned long long)f, 0, 0);
}

// One wave per task: walk the record chain over the tile summaries.  RESOLVE: the deferred tasks
// (P.D.list[0, t_count)) with the host's libm decisions for their guard-band pairs (P.D.ov): the
// claim count corrected by each override, tiles holding an overridden agent always scanned (their
// summary was computed with the device's decision), the override applied inside them.  The chain
// stays a walk over tile summaries, where the per-task wave pass over every agent (k_alloc_binned
// SRC_ALL) would rescan all n agents per chain link once a task's claims overflow its LDS list.
template <bool RESOLVE>
__global__ __launch_bounds__(kBlock) void k_alloc_dense_chain(
    int64_t n, int64_t t_count, const double2 *__restrict__ tpos, const int8_t *__restrict__ treq,
    const int32_t *__restrict__ ids, const double2 *__restrict__ apos,
    const uint32_t *__restrict__ caps, const int32_t *__restrict__ order,
    const uint32_t *__restrict__ sorted_ids, int64_t ntiles, const float *__restrict__ tmax,
    const int *__restrict__ tcnt, Params P) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
    BlockStats bs;
    __shared__ unsigned long long s_c[kBlock / kWave], s_m[kBlock / kWave], s_b[kBlock / kWave];
    for (int64_t kk = wave; kk < t_count; kk += nwaves) {
        const int64_t k = RESOLVE ? int64_t(P.D.list[kk]) : kk;
        const int rq = treq[k];
        if (!RESOLVE && P.D.list && P.D.tflag[k]) {  // a guard-band pair: deferred to the libm pass
            if (lane == 0) {
                P.D.list[atomicAdd(P.D.count, 1ull)] = int32_t(k);
                bs.bad += bad_req(rq) ? 1 : 0;
            }
            continue;
        }
        const double2 tp = tpos[k];
        const int w0 = P.winner[k];
        const double u0 = P.util[k];
        const float *mk = tmax + k * ntiles;
        const int *ck = tcnt + k * ntiles;
        long long nclaims = 0;
        for (int64_t a = lane; a < ntiles; a += 64) nclaims += ck[a];
        uint32_t ov_a = 0, ov_b = 0;
        int64_t ov_tile = -1;  // RESOLVE: the ID-order tile of override ov_a + lane (lanes < nov)
        int nov = 0;
        if (RESOLVE) {
            ov_a = P.D.ov_off[kk];
            ov_b = P.D.ov_off[kk + 1];
            nov = int(ov_b - ov_a);
            for (uint32_t q = ov_a + lane; q < ov_b; q += 64) {
                const Override o = P.D.ov[q];
                const double2 p = apos[o.agent];
                const bool dev = utility(p.x, p.y, caps[o.agent], tp.x, tp.y, rq, P.u_scale) > P.thr;
                nclaims += (o.claim ? 1 : 0) - (dev ? 1 : 0);
                if (q == ov_a + lane) {  // its position in ID order: binary search of its ID
                    const uint32_t id = uint32_t(ids[o.agent]);
                    int64_t lo = 0, hi = n - 1;
                    while (lo < hi) {
                        const int64_t mid = (lo + hi) >> 1;
                        if (sorted_ids[mid] < id) lo = mid + 1; else hi = mid;
                    }
                    ov_tile = lo / kTileA;
                }
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) nclaims += __shfl_xor(nclaims, off, 64);
        // did the incumbent claim?  (binary search of w0 in the ID-sorted keys)
        bool w0_claimed = false;
        if (w0 >= 0 && nclaims > 0) {
            int64_t lo = 0, hi = n - 1;
            while (lo <= hi) {
                const int64_t mid = (lo + hi) >> 1;
                const uint32_t v = sorted_ids[mid];
                if (v == uint32_t(w0)) {
                    const int32_t i = order[mid];
                    const double2 p = apos[i];
                    const double U = utility(p.x, p.y, caps[i], tp.x, tp.y, rq, P.u_scale);
                    bool cl = U > P.thr;
                    float xw = float(U);
                    if (RESOLVE && guard_flag(U, P.thr)) apply_override(P, ov_a, ov_b, i, cl, xw);
                    w0_claimed = cl;
                    break;
                }
                if (v < uint32_t(w0)) lo = mid + 1; else hi = mid - 1;
            }
        }
        // chain: position pos (in ID order) of the current winner; -1 before the first link
        int64_t pos = -1;
        bool has = w0 >= 0;
        double cur_u = u0;
        int cur_id = w0, cur_idx = -1, accepted = 0, first_id = -1;
        for (;;) {
            // first tile after pos whose max could host a link
            const int64_t tstart = (pos + 1) / kTileA;
            int64_t found_tile = -1;
            for (int64_t a0 = tstart; a0 < ntiles && found_tile < 0; a0 += 64) {
                const int64_t a = a0 + lane;
                const float m = a < ntiles ? mk[a] : -INFINITY;
                bool forced = false;  // RESOLVE: a tile with an overridden agent (more than 64: every tile)
                if (RESOLVE && nov > 0) {
                    if (nov > 64) {
                        forced = true;
                    } else {
                        for (int q = 0; q < nov; ++q) forced = forced || __shfl(ov_tile, q, 64) == a;
                    }
                }
                const bool ok = a < ntiles && ((m != -INFINITY && (!has || double(m) > cur_u + P.h)) || forced);
                const unsigned long long b = __ballot(ok);
                if (b) found_tile = a0 + __ffsll((long long)b) - 1;
            }
            if (found_tile < 0) break;
            // inside the tile: first agent j > pos with a qualifying claim (4 sub-chunks of 64)
            int64_t hitj = -1;
            float hitx = 0.f;
            int hit_ix = -1;
            for (int64_t j0 = found_tile * kTileA; j0 < (found_tile + 1) * kTileA && hitj < 0; j0 += 64) {
                const int64_t j = j0 + lane;
                bool ok = false;
                float x = 0.f;
                int32_t i = -1;
                if (j < n && j > pos) {
                    i = order[j];
                    const double2 p = apos[i];
                    const double U = utility(p.x, p.y, caps[i], tp.x, tp.y, rq, P.u_scale);
                    x = float(U);
                    bool cl = U > P.thr;
                    if (RESOLVE && guard_flag(U, P.thr)) apply_override(P, ov_a, ov_b, i, cl, x);
                    ok = cl && (!has || double(x) > cur_u + P.h);
                }
                const unsigned long long b = __ballot(ok);
                if (b) {
                    const int src = __ffsll((long long)b) - 1;
                    hitj = j0 + src;
                    hitx = __shfl(x, src, 64);
                    hit_ix = __shfl(i, src, 64);
                }
            }
            if (hitj < 0) {  // tile max qualified but every qualifying claim sits at or before pos
                pos = (found_tile + 1) * kTileA - 1;
                continue;
            }
            pos = hitj;
            cur_idx = hit_ix;
            cur_id = ids[hit_ix];
            cur_u = double(hitx);
            has = true;
            if (++accepted == 1) first_id = cur_id;
        }
        if (lane == 0) {
            finish_task(P, k, w0, u0, w0_claimed, accepted, first_id, cur_id, cur_u, cur_idx, nclaims, bs);
            bs.bad += bad_req(rq) ? 1 : 0;
        }
    }
    if (lane == 0) { s_c[threadIdx.x >> 6] = bs.claims; s_m[threadIdx.x >> 6] = bs.msgs; s_b[threadIdx.x >> 6] = bs.bad; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0, m = 0, b = 0;
        for (int w = 0; w < kBlock / kWave; ++w) { c += s_c[w]; m += s_m[w]; b += s_b[w]; }
        flush_stats(P, c, m, 0, 0, 0, b);
    }
}

// Ascending-ID order of agents (dense mode): radix sort of (id, index).
__global__ __launch_bounds__(kBlock) void k_iota_ids(const int32_t *__restrict__ ids, int64_t n,
                                                    uint32_t *__restrict__ keys, int32_t *__restrict__ vals) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        keys[i] = uint32_t(ids[i]);
        vals[i] = int32_t(i);
    }
}

__global__ __launch_bounds__(kBlock) void k_utility(int64_t m, const double2 *__restrict__ apos,
                                                   const uint32_t *__restrict__ caps,
                                                   const double2 *__restrict__ tpos,
                                                   const int8_t *__restrict__ treq, double u_scale,
                                                   double *__restrict__ out) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < m; i += int64_t(gridDim.x) * kBlock) {
        const double2 a = apos[i], t = tpos[i];
        out[i] = utility(a.x, a.y, caps[i], t.x, t.y, treq[i], u_scale);
    }
}

}  // namespace
static_assert(sizeof(swarm_grid) == sizeof(Grid), "swarm_grid mirrors the internal Grid");

#define SW_TRY(call)                 \
    do {                             \
        const int rc_ = (call);      \
        if (rc_ != SWARM_OK) return rc_; \
    } while (0)

namespace {

// The dense strategy's ID order and tile summaries (the deferred tasks' chains walk them too).
struct DenseChain {
    const int32_t *order = nullptr;
    const uint32_t *sorted_ids = nullptr;
    int64_t ntiles = 0;
    const float *tmax = nullptr;
    const int *tcnt = nullptr;
};

// A per-task pass's candidate source (SRC_* and what it reads).
struct Cand {
    int src = SRC_ALL;
    const int32_t *sorted = nullptr;
    const uint32_t *off = nullptr;
    HashGrid hg{1.0, 0};
    Grid g{};
    double rp = 0.0;
    DenseChain dense;  // SRC_ALL from the dense strategy: resolve through k_alloc_dense_chain<true>
};

template <int SRC, int PASS>
int launch_one(const Cand &c, int64_t count, int64_t n, const double *tpos, const int8_t *treq, const int32_t *ids,
               const double *apos, const uint32_t *acaps, const Params &P, hipStream_t s) {
    hipLaunchKernelGGL((k_alloc_binned<SRC, PASS>), dim3(grid_for(count, kBlock / kWave, 4096)), dim3(kBlock), 0, s,
                       count, reinterpret_cast<const double2 *>(tpos), treq, ids,
                       reinterpret_cast<const double2 *>(apos), acaps, c.sorted, c.off, c.hg, c.g, c.rp, n, P);
    SW_LAUNCHED();
    return SWARM_OK;
}

template <int PASS>
int launch_tasks(const Cand &c, int64_t count, int64_t n, const double *tpos, const int8_t *treq, const int32_t *ids,
                 const double *apos, const uint32_t *acaps, const Params &P, hipStream_t s) {
    if (count <= 0) return SWARM_OK;
    switch (c.src) {
        case SRC_HASH: return launch_one<SRC_HASH, PASS>(c, count, n, tpos, treq, ids, apos, acaps, P, s);
        case SRC_ROWS: return launch_one<SRC_ROWS, PASS>(c, count, n, tpos, treq, ids, apos, acaps, P, s);
        default: return launch_one<SRC_ALL, PASS>(c, count, n, tpos, treq, ids, apos, acaps, P, s);
    }
}

// The reference's utility on the HOST, for guard-band pairs only (agent.py:338-347).  `**2` is
// CPython's float_pow, which calls libm pow(|x|, 2.0) (it strips a negative base's sign before the
// call).  Called through a volatile pointer: a compiler folds pow(x, 2.0) into x*x -- the device's
// arithmetic, not the reference's.
double (*volatile g_libm_pow)(double, double) = static_cast<double (*)(double, double)>(std::pow);

double ref_utility(const FlagPair &q, double u_scale) {
    const double dx = q.ax - q.tx, dy = q.ay - q.ty;
    const double d = std::sqrt(g_libm_pow(std::fabs(dx), 2.0) + g_libm_pow(std::fabs(dy), 2.0));
    return (u_scale / (1.0 + d)) * (q.has ? 1.0 : 0.0);
}

// Deferred tasks (P.D.list[0, deferred)): collect their guard-band pairs, decide each on the host
// with libm pow, resolve the tasks once with those decisions.  One host sync per step; only runs
// when some pair fell inside the guard band.
int resolve_deferred(swarm_ctx *ctx, Params P, const Cand &cand, int64_t deferred, int64_t n, const double *tpos,
                     const int8_t *treq, const int32_t *ids, const double *apos, const uint32_t *acaps,
                     double claim_thr, double u_scale, hipStream_t s) {
    unsigned long long *hc = static_cast<unsigned long long *>(pinned(ctx, 128));
    if (!hc) return SWARM_ERR_OOM;
    int64_t cap = deferred * 32 > 4096 ? deferred * 32 : 4096;
    unsigned long long npairs = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        SW_ALLOC(P.D.pairs, ctx, S_FPAIRS, size_t(cap) * sizeof(FlagPair));
        P.D.pair_cap = cap;
        SW_HIP(hipMemsetAsync(P.D.count + 1, 0, 8, s));
        SW_TRY(launch_tasks<PASS_COLLECT>(cand, deferred, n, tpos, treq, ids, apos, acaps, P, s));
        SW_HIP(hipMemcpyAsync(hc, P.D.count + 1, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        npairs = hc[0];
        if (int64_t(npairs) <= cap) break;
        cap = int64_t(npairs);  // the second attempt holds every pair (the same ones are flagged)
    }
    if (int64_t(npairs) > cap) {
        set_error("guard-band pair list overflow (%llu > %lld)", npairs, (long long)cap);
        return SWARM_ERR_HIP;
    }
    std::vector<FlagPair> pairs(npairs);
    if (npairs) {
        SW_HIP(hipMemcpyAsync(pairs.data(), P.D.pairs, npairs * sizeof(FlagPair), hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
    }
    std::sort(pairs.begin(), pairs.end(), [](const FlagPair &a, const FlagPair &b) {
        return a.j != b.j ? a.j < b.j : a.agent < b.agent;
    });
    std::vector<uint32_t> ov_off(size_t(deferred) + 1, 0);
    std::vector<Override> ov(npairs);
    for (size_t q = 0; q < pairs.size(); ++q) {
        const double U = ref_utility(pairs[q], u_scale);
        ov[q] = Override{pairs[q].agent, float(U), U > claim_thr ? 1 : 0, 0};
        ov_off[size_t(pairs[q].j) + 1] += 1;
    }
    for (size_t j = 0; j < size_t(deferred); ++j) ov_off[j + 1] += ov_off[j];
    const size_t off_bytes = ((ov_off.size() * 4) + 63) & ~size_t(63);
    uint8_t *ob;
    SW_ALLOC(ob, ctx, S_OVR, off_bytes + ov.size() * sizeof(Override) + 64);
    SW_HIP(hipMemcpyAsync(ob, ov_off.data(), ov_off.size() * 4, hipMemcpyHostToDevice, s));
    if (!ov.empty())
        SW_HIP(hipMemcpyAsync(ob + off_bytes, ov.data(), ov.size() * sizeof(Override), hipMemcpyHostToDevice, s));
    P.D.ov_off = reinterpret_cast<const uint32_t *>(ob);
    P.D.ov = reinterpret_cast<const Override *>(ob + off_bytes);
    if (cand.dense.tmax) {
        hipLaunchKernelGGL((k_alloc_dense_chain<true>), dim3(grid_for(deferred, kBlock / kWave, 1u << 20)), dim3(kBlock),
                           0, s, n, deferred, reinterpret_cast<const double2 *>(tpos), treq, ids,
                           reinterpret_cast<const double2 *>(apos), acaps, cand.dense.order, cand.dense.sorted_ids,
                           cand.dense.ntiles, cand.dense.tmax, cand.dense.tcnt, P);
        SW_LAUNCHED();
    } else {
        SW_TRY(launch_tasks<PASS_RESOLVE>(cand, deferred, n, tpos, treq, ids, apos, acaps, P, s));
    }
    SW_HIP(hipStreamSynchronize(s));  // the host vectors above are the copies' sources
    return SWARM_OK;
}

}  // namespace

// ix / ix_off: a cell index (swarm_cell_index) of the agents' storage order, or NULL.
int alloc_impl(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps,
               int64_t t, const double *tpos, const int8_t *treq, double claim_thr, double hysteresis,
               double u_scale, int32_t mode, int32_t *winner, double *util, int32_t *won,
               const int32_t *id_to_index, int64_t id_span, int64_t *nclaim, int64_t *nmsg,
               swarm_alloc_stats *stats, void *stream, const Grid *ix, const uint32_t *ix_off, int32_t flags = 0) {
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31), "n out of range");
    SW_ARG(t >= 0 && t < (int64_t(1) << 31), "t out of range");
    SW_ARG(std::isfinite(claim_thr) && std::isfinite(hysteresis) && std::isfinite(u_scale),
           "claim_thr / hysteresis / u_scale must be finite");
    SW_ARG(mode == SWARM_ALLOC_AUTO || mode == SWARM_ALLOC_BINNED || mode == SWARM_ALLOC_DENSE,
           "unknown mode");
    SW_ARG(n == 0 || (ids && apos && acaps), "NULL agent array");
    SW_ARG(t == 0 || (tpos && treq && winner && util), "NULL task array");
    SW_ARG((flags & ~(SWARM_ALLOC_TRUST_INDEX | SWARM_ALLOC_FRESH_CLAIMS)) == 0, "unknown flags");
    const bool fresh = (flags & SWARM_ALLOC_FRESH_CLAIMS) != 0 && t > 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *dstats;  // the shards, then the folded stats
    SW_ALLOC(dstats, ctx, S_ASTATS, (size_t(kStatShards) * kStatStride + 8) * 8);

    // claim radius: U > thr  <=>  d < u_scale / thr - 1  (thr > 0, u_scale > 0, has_cap)
    const bool finite_r = claim_thr > 0 && u_scale > 0;
    const double rc = finite_r ? u_scale / claim_thr - 1.0 : 0.0;
    int used = mode;
    if (mode == SWARM_ALLOC_AUTO) used = finite_r ? SWARM_ALLOC_BINNED : SWARM_ALLOC_DENSE;
    SW_ARG(!(used == SWARM_ALLOC_BINNED && !finite_r),
           "binned mode needs claim_thr > 0 and u_scale > 0 (finite claim radius)");
    Params P;
    P.thr = claim_thr; P.h = hysteresis; P.u_scale = u_scale;
    P.winner = winner; P.util = util; P.won = won; P.id_to_index = id_to_index;
    P.id_span = id_span; P.nclaim = nclaim; P.nmsg = nmsg; P.stats = dstats;

    // guard-band deferral (FlagPair / Override above): list + counters + per-task flags
    const size_t defer_list_off = 64, defer_flag_off = 64 + ((size_t(t) * 4 + 63) & ~size_t(63));
    uint8_t *dbase;
    SW_ALLOC(dbase, ctx, S_DEFER, defer_flag_off + size_t(t) + 64);
    P.D.count = reinterpret_cast<unsigned long long *>(dbase);
    P.D.list = reinterpret_cast<int32_t *>(dbase + defer_list_off);
    hipLaunchKernelGGL(k_alloc_init, dim3(grid_for(std::max(n, fresh ? t : 0), kBlock, 2048)), dim3(kBlock), 0, s,
                       dstats, P.D.count, won, n, fresh ? winner : nullptr, fresh ? util : nullptr, t);
    SW_LAUNCHED();

    const bool nothing = (n == 0) || (used == SWARM_ALLOC_BINNED && rc <= 0.0);
    Cand cand;  // the main pass's candidate source, reused by the deferred passes
    if (t > 0 && nothing) {
        // no agent can claim: every task keeps its current claim (won credited via id_to_index)
        uint32_t *off;
        SW_ALLOC(off, ctx, S_CELL_START, 16);
        SW_HIP(hipMemsetAsync(off, 0, 16, s));
        P.rp2 = -1.0;
        cand = Cand{SRC_HASH, nullptr, off, HashGrid{1.0, 0}, Grid{}, 0.0};
        SW_TRY(launch_tasks<PASS_MAIN>(cand, t, n, tpos, treq, ids, apos, acaps, P, s));
    } else if (t > 0 && used == SWARM_ALLOC_BINNED && ix) {
        // the caller's cell index: the window's grid rows are contiguous storage ranges
        const double rp = rc * (1.0 + 1e-9) + 1e-12;
        P.rp2 = rp * rp;
        SW_ARG(std::floor(2.0 * rp * ix->inv_cell) + 2.0 <= double(kMaxCells),
               "claim radius spans more than 16 rows of the index's cells (use swarm_allocate)");
        // the staleness check on the side stream, concurrent with the allocation (joined before the
        // counters are folded) -- skipped when the caller vouches that the positions are the ones the
        // index was built from (SWARM_ALLOC_TRUST_INDEX: 160 MB of positions not streamed at 10M
        // agents).  Measured and rejected: the check as extra workgroups of the allocation's grid,
        // with the stats folded by the last workgroup through a ticket counter (one launch and no
        // side stream): 245 us for the grid against ~90 us for the pair.
        const bool check = (flags & SWARM_ALLOC_TRUST_INDEX) == 0;
        hipStream_t s2 = nullptr;
        hipEvent_t fork = nullptr, join = nullptr;
        if (check) {
            SW_TRY(side_stream(ctx, &s2, &fork, &join));
            SW_HIP(hipEventRecord(fork, s));
            SW_HIP(hipStreamWaitEvent(s2, fork, 0));
            hipLaunchKernelGGL(k_check_index, dim3(grid_for(n, kBlock * kCheckPer, 4096)), dim3(kBlock), 0, s2,
                               reinterpret_cast<const double2 *>(apos), n, *ix, ix_off, dstats + 7);
            SW_LAUNCHED();
            SW_HIP(hipEventRecord(join, s2));
        }
        cand = Cand{SRC_ROWS, nullptr, ix_off, HashGrid{1.0, 0}, *ix, rp};
        SW_TRY(launch_tasks<PASS_MAIN>(cand, t, n, tpos, treq, ids, apos, acaps, P, s));
        if (check) SW_HIP(hipStreamWaitEvent(s, join, 0));
    } else if (t > 0 && used == SWARM_ALLOC_BINNED) {
        // agents bucketed by hashed cell of side Rp (counting sort, no host round trip)
        const double rp = rc * (1.0 + 1e-9) + 1e-12;
        P.rp2 = rp * rp;
        uint32_t nb = 1024;
        while (nb < uint32_t(1) << 30 && int64_t(nb) * 8 < n) nb <<= 1;
        const HashGrid hg{1.0 / rp, nb - 1};
        uint32_t *cnt, *off, *key, *rank;
        int32_t *sorted;
        SW_ALLOC(cnt, ctx, S_KEYS_IN, size_t(nb + 1) * 4);
        SW_ALLOC(off, ctx, S_CELL_START, size_t(nb + 1) * 4);
        SW_ALLOC(key, ctx, S_KEYS_OUT, size_t(n) * 4);
        SW_ALLOC(rank, ctx, S_VALS_IN, size_t(n) * 4);
        SW_ALLOC(sorted, ctx, S_VALS_OUT, size_t(n) * 4);
        SW_HIP(hipMemsetAsync(cnt, 0, size_t(nb + 1) * 4, s));
        hipLaunchKernelGGL(k_hash_count, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s,
                           reinterpret_cast<const double2 *>(apos), n, hg, cnt, key, rank, dstats + 6);
        SW_LAUNCHED();
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, int(nb + 1), s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, int(nb + 1), s));
        hipLaunchKernelGGL(k_hash_scatter, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, n, key, rank, off,
                           sorted);
        SW_LAUNCHED();
        cand = Cand{SRC_HASH, sorted, off, hg, Grid{}, rp};
        SW_TRY(launch_tasks<PASS_MAIN>(cand, t, n, tpos, treq, ids, apos, acaps, P, s));
    } else if (t > 0) {
        P.rp2 = 0;
        P.D.tflag = dbase + defer_flag_off;
        SW_HIP(hipMemsetAsync(P.D.tflag, 0, size_t(t), s));
        const int64_t ntiles = (n + kTileA - 1) / kTileA;
        uint32_t *kin, *kout;
        int32_t *vin, *order;
        SW_ALLOC(kin, ctx, S_KEYS_IN, size_t(n) * 4);
        SW_ALLOC(kout, ctx, S_KEYS_OUT, size_t(n) * 4);
        SW_ALLOC(vin, ctx, S_VALS_IN, size_t(n) * 4);
        SW_ALLOC(order, ctx, S_ORDER, size_t(n) * 4);
        hipLaunchKernelGGL(k_iota_ids, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, ids, n, kin, vin);
        SW_LAUNCHED();
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, order, int(n), 0, 32, s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, order, int(n), 0, 32, s));
        float *tmax;
        int *tcnt;
        SW_ALLOC(tmax, ctx, S_TILEMAX, size_t(t) * size_t(ntiles) * 4);
        SW_ALLOC(tcnt, ctx, S_TMP1, size_t(t) * size_t(ntiles) * 4);
        const int64_t blocks = ntiles * ((t + kTileT - 1) / kTileT);
        hipLaunchKernelGGL(k_alloc_dense_tiles, dim3(grid_for(blocks, 1, 1u << 20)), dim3(kBlock), 0, s, n, t,
                           reinterpret_cast<const double2 *>(tpos), treq,
                           reinterpret_cast<const double2 *>(apos), acaps, order, ntiles, tmax, tcnt, P);
        SW_LAUNCHED();
        hipLaunchKernelGGL((k_alloc_dense_chain<false>), dim3(grid_for(t, kBlock / kWave, 1u << 20)), dim3(kBlock), 0,
                           s, n, t, reinterpret_cast<const double2 *>(tpos), treq, ids,
                           reinterpret_cast<const double2 *>(apos), acaps, order, kout, ntiles, tmax,
                           tcnt, P);
        SW_LAUNCHED();
        // deferred tasks: their guard-band pairs collected over every agent (no radius: rp2 = +inf
        // keeps all finite ones, the tile kernel's NaN utilities never claim either), then resolved
        // by the chain kernel over the same tile summaries (k_alloc_dense_chain<true>)
        P.rp2 = INFINITY;
        cand = Cand{SRC_ALL, nullptr, nullptr, HashGrid{1.0, 0}, Grid{}, 0.0};
        cand.dense = DenseChain{order, kout, ntiles, tmax, tcnt};
    }
    unsigned long long *hs = static_cast<unsigned long long *>(pinned(ctx, 128));
    if (!hs) return SWARM_ERR_OOM;
    unsigned long long *folded = dstats + size_t(kStatShards) * kStatStride;
    {  // the stats and the deferred count folded straight into host-mapped memory: no copies
        void *fold_dev = nullptr;
        unsigned long long *hfold = static_cast<unsigned long long *>(mapped(ctx, 16 * 8, &fold_dev));
        if (!hfold) return SWARM_ERR_OOM;
        // The host waits for the fold's epoch word in that memory instead of a stream synchronisation
        // (the results stay stream-ordered for the caller; only the counters are needed here):
        // wait_mapped_word spins on it.
        // (the mapped buffer is shared with other calls of this ctx, whose device writes have all been
        // waited for: the word is cleared here, and the epoch carries a tag no counter reaches)
        const unsigned long long ep = (0xA110Cull << 40) | (++ctx->fold_epoch & ((1ull << 40) - 1));
        __atomic_store_n(&hfold[15], 0ull, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(k_fold_stats, dim3(1), dim3(kWave), 0, s, dstats,
                           static_cast<unsigned long long *>(fold_dev), P.D.count,
                           static_cast<unsigned long long *>(fold_dev) + 15, ep);
        SW_LAUNCHED();
        SW_TRY(wait_mapped_word(&hfold[15], ep, s, "allocation"));
        for (int c = 0; c <= kNumStats; ++c) hs[c] = __atomic_load_n(&hfold[c], __ATOMIC_RELAXED);
    }
    if (hs[7]) {
        set_error("stale cell index: %llu agent(s) outside their cell's range (positions moved since "
                  "swarm_cell_index)", (unsigned long long)hs[7]);
        return SWARM_ERR_STALE;
    }
    if (hs[6]) {
        set_error("invalid argument: %llu agent position(s) are not finite", (unsigned long long)hs[6]);
        return SWARM_ERR_ARG;
    }
    if (hs[5]) {  // outputs were computed treating those capability indices as absent
        set_error("invalid argument: %llu task(s) with treq outside [-1, 31]", (unsigned long long)hs[5]);
        return SWARM_ERR_ARG;
    }
    const int64_t deferred = int64_t(hs[kNumStats]);
    if (deferred > 0) {
        SW_TRY(resolve_deferred(ctx, P, cand, deferred, n, tpos, treq, ids, apos, acaps, claim_thr, u_scale, s));
        hipLaunchKernelGGL(k_fold_stats, dim3(1), dim3(kWave), 0, s, dstats, folded);
        SW_LAUNCHED();
        SW_HIP(hipMemcpyAsync(hs, folded, 8 * kNumStats, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
    }
    if (stats) {
        stats->n_claims = int64_t(hs[0]);
        stats->n_conflicts = int64_t(hs[1]);
        stats->n_flagged = int64_t(hs[2]);
        stats->n_candidates = used == SWARM_ALLOC_DENSE ? n * t : int64_t(hs[3]);
        stats->n_overflow = int64_t(hs[4]);
        stats->mode_used = used;
        stats->n_resolved = deferred;
    }
    return SWARM_OK;
}

// keys[i] < keys[i-1] anywhere -> *bad += 1 per such i
__global__ __launch_bounds__(kBlock) void k_count_unsorted(const uint32_t *__restrict__ keys, int64_t n,
                                                          unsigned long long *__restrict__ bad_out) {
    unsigned long long bad = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x + 1; i < n; i += int64_t(gridDim.x) * kBlock)
        bad += keys[i] < keys[i - 1] ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(bad_out, bad);
}

}  // namespace swarm

extern "C" {

int swarm_allocate(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                   const uint32_t *acaps, int64_t t, const double *tpos, const int8_t *treq,
                   double claim_thr, double hysteresis, double u_scale, int32_t mode,
                   int32_t *winner, double *util, int32_t *won, const int32_t *id_to_index,
                   int64_t id_span, int64_t *nclaim, int64_t *nmsg, swarm_alloc_stats *stats,
                   void *stream) {
    return swarm::alloc_impl(ctx, n, ids, apos, acaps, t, tpos, treq, claim_thr, hysteresis, u_scale, mode, winner,
                             util, won, id_to_index, id_span, nclaim, nmsg, stats, stream, nullptr, nullptr);
}

int swarm_cell_index(swarm_ctx *ctx, int64_t n, const double *pos, double cell, swarm_grid *grid,
                     uint32_t *cell_off, int64_t cell_off_capacity, int64_t *ncells, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && grid != nullptr && ncells != nullptr, "NULL argument");
    SW_ARG(n >= 1 && n < (int64_t(1) << 31), "n out of range (need at least one agent)");
    SW_ARG(cell > 0 && std::isfinite(cell), "cell must be positive and finite");
    SW_ARG(pos != nullptr, "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    Grid g;
    int rc = make_grid(ctx, n, pos, cell, 4 * n + 1024, &g, s);  // swarm_cell_order's grid
    if (rc) return rc;
    memcpy(grid, &g, sizeof(g));
    *ncells = g.ncx * g.ncy;
    if (cell_off == nullptr) return SWARM_OK;
    SW_ARG(cell_off_capacity >= *ncells + 1, "cell_off capacity < ncells + 1");
    uint32_t *keys;
    int32_t *vals;
    unsigned long long *bad;
    SW_ALLOC(keys, ctx, S_KEYS_IN, size_t(n) * 4);
    SW_ALLOC(vals, ctx, S_VALS_IN, size_t(n) * 4);
    SW_ALLOC(bad, ctx, S_TMP0, 8);
    SW_HIP(hipMemsetAsync(bad, 0, 8, s));
    hipLaunchKernelGGL(k_cell_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s,
                       reinterpret_cast<const double2 *>(pos), n, g, keys, vals);
    SW_LAUNCHED();
    hipLaunchKernelGGL(k_count_unsorted, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, keys, n, bad);
    SW_LAUNCHED();
    hipLaunchKernelGGL(k_cell_offsets, dim3(grid_for(n + 1, kBlock, 8192)), dim3(kBlock), 0, s, keys, n, *ncells,
                       cell_off);
    SW_LAUNCHED();
    unsigned long long *hb = static_cast<unsigned long long *>(pinned(ctx, 64));
    if (!hb) return SWARM_ERR_OOM;
    SW_HIP(hipMemcpyAsync(hb, bad, 8, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    SW_ARG(hb[0] == 0, "positions are not in cell order (swarm_cell_order's layout with this cell)");
    return SWARM_OK;
}

int swarm_allocate_indexed_ex(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                              const uint32_t *acaps, const swarm_grid *grid, const uint32_t *cell_off, int64_t t,
                              const double *tpos, const int8_t *treq, double claim_thr, double hysteresis,
                              double u_scale, int32_t flags, int32_t *winner, double *util, int32_t *won,
                              const int32_t *id_to_index, int64_t id_span, int64_t *nclaim, int64_t *nmsg,
                              swarm_alloc_stats *stats, void *stream) {
    using namespace swarm;
    SW_ARG(grid != nullptr && cell_off != nullptr, "NULL index");
    SW_ARG(grid->ncx >= 1 && grid->ncy >= 1 && grid->inv_cell > 0, "bad grid");
    Grid g;
    memcpy(&g, grid, sizeof(g));
    return alloc_impl(ctx, n, ids, apos, acaps, t, tpos, treq, claim_thr, hysteresis, u_scale, SWARM_ALLOC_BINNED,
                      winner, util, won, id_to_index, id_span, nclaim, nmsg, stats, stream, &g, cell_off, flags);
}

int swarm_allocate_indexed(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos,
                           const uint32_t *acaps, const swarm_grid *grid, const uint32_t *cell_off, int64_t t,
                           const double *tpos, const int8_t *treq, double claim_thr, double hysteresis,
                           double u_scale, int32_t *winner, double *util, int32_t *won,
                           const int32_t *id_to_index, int64_t id_span, int64_t *nclaim, int64_t *nmsg,
                           swarm_alloc_stats *stats, void *stream) {
    return swarm_allocate_indexed_ex(ctx, n, ids, apos, acaps, grid, cell_off, t, tpos, treq, claim_thr, hysteresis,
                                     u_scale, 0, winner, util, won, id_to_index, id_span, nclaim, nmsg, stats, stream);
}

int swarm_utility(swarm_ctx *ctx, int64_t m, const double *apos, const uint32_t *acaps,
                  const double *tpos, const int8_t *treq, double u_scale, double *out, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(m >= 0, "m < 0");
    if (m == 0) return SWARM_OK;
    SW_ARG(apos && acaps && tpos && treq && out, "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_utility, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, m,
                       reinterpret_cast<const double2 *>(apos), acaps,
                       reinterpret_cast<const double2 *>(tpos), treq, u_scale, out);
    SW_LAUNCHED();
    return SWARM_OK;
}

}  // extern "C"
