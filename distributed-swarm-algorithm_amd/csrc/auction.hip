// Auction allocation on gfx950 (BASELINE config C4).
//
// The north star's "auction price update as a conflict-free bid kernel".  The reference has no
// auction (its allocation is greedy claim + leader hysteresis, agent.py:292-325), so parity is
// against the build's own CPU restatement (oracle/swarm_oracle.c orc_auction), bit-exact:
// assignments, prices, per-round bidder counts and the round count.
//
// Problem: agents x tasks with value x(a,k) = f32(U(a,k)) for the admissible pairs U > claim_thr
// -- the reference's claim rule (agent.py:297) and claim payload (agent.py:302) -- one task per
// agent, one agent per task, maximise total value.  Jacobi Bertsekas auction: every round every
// unassigned, active agent bids on its best task (net = x - price, ties -> lowest task index)
// price + (best - second) + eps, the opt-out option (net 0) counting as a competitor; an agent
// whose best net is <= 0 drops out for good.  Each task takes its highest bid, ties -> lowest
// agent ID; the previous owner becomes unassigned.  Stops after the first round without bidders.
//
// Kernels:
//   candidates   tasks binned in a uniform grid (cell >= claim radius); one thread per agent
//                walks the cells its claim disc covers, fp64 utilities, and writes its
//                admissible (task, f32 value) list (count pass, hipCUB scan, fill pass).
//   k_auc_bid_list  one wave per listed bidder (the unassigned, active agents; the list never
//                grows): lanes sweep its candidate list (price gathers), a wave reduction of
//                (best, task, second); the bid is ONE 64-bit atomicMax per bidder on a packed
//                key f32bits(bid) << 32 | ~id -- highest bid, then lowest ID, no conflicts.
//   k_auc_resolve_list  one thread per list entry: the standing key's bidder takes the task;
//                losers and displaced owners form the next round's list.
//   (k_auc_bid / k_auc_resolve_ids: every agent / task per round, for the sharded rounds.)
//   k_auc_tail   once few agents still bid (prices rising on a handful of contested tasks, the
//                auction's long tail), ONE workgroup runs all remaining rounds with its bidder
//                list in LDS, workgroup barriers between the phases and workgroup-scoped key
//                atomics: no kernel boundary per round.  Same rounds, same results.
// Per-round bidder counts: 64-way sharded counters in a ring (multi-workgroup rounds), a log
// written by the tail kernel; the host reads them every batch of rounds.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "binning.h"
#include "utility.h"

namespace swarm {
namespace {

constexpr int kAShards = 64;
constexpr int kAStride = 16;       // u64 per shard: one 128-B line
constexpr int kARing = 512;        // rounds of counter slots
constexpr int kTailBlock = 1024;   // k_auc_tail: threads (16 waves)
constexpr int kTailCap = 2048;     // k_auc_tail: bidder list capacity (LDS)
constexpr int kBidU = 4;           // wave_bid: list entries per lane per pass

__device__ __forceinline__ unsigned long long *aslot(unsigned long long *ring, int64_t r, int shard) {
    return ring + size_t(r % kARing) * kAShards * kAStride + size_t(shard) * kAStride;
}

// ---------------------------------------------------------------- candidate lists
struct CandIn {
    const double2 *apos;
    const uint32_t *acaps;
    const double2 *tpos;
    const int8_t *treq;
    const int32_t *sorted;     // task indices, cell by cell
    const uint32_t *cell_off;  // per-cell exclusive prefix into sorted
    Grid g;
    double rp, rp2, thr, u_scale;
};

// Walk agent a's admissible tasks: f(k, U) for every task with U > thr.
template <typename F>
__device__ __forceinline__ void for_admissible(const CandIn &c, int64_t a, unsigned long long &flagged, F f) {
    const double2 p = c.apos[a];
    const uint32_t caps = c.acaps[a];
    const Grid &g = c.g;
    if (p.x + c.rp < g.xmin || p.x - c.rp > g.xmax || p.y + c.rp < g.ymin || p.y - c.rp > g.ymax) return;
    const int64_t x0 = cell_coord(p.x - c.rp, g.xmin, g.inv_cell, g.ncx);
    const int64_t x1 = cell_coord(p.x + c.rp, g.xmin, g.inv_cell, g.ncx);
    const int64_t y0 = cell_coord(p.y - c.rp, g.ymin, g.inv_cell, g.ncy);
    const int64_t y1 = cell_coord(p.y + c.rp, g.ymin, g.inv_cell, g.ncy);
    for (int64_t yy = y0; yy <= y1; ++yy) {
        const uint32_t q0 = c.cell_off[yy * g.ncx + x0], q1 = c.cell_off[yy * g.ncx + x1 + 1];
        for (uint32_t q = q0; q < q1; ++q) {
            const int32_t k = c.sorted[q];
            const double2 tp = c.tpos[k];
            const double dx = p.x - tp.x, dy = p.y - tp.y;
            if (dx * dx + dy * dy > c.rp2) continue;
            const double U = utility(p.x, p.y, caps, tp.x, tp.y, c.treq[k], c.u_scale);
            flagged += guard_flag(U, c.thr);
            if (U > c.thr) f(k, U);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_auc_count(CandIn c, int64_t n, int64_t *__restrict__ cnt,
                                                     unsigned long long *__restrict__ flagged_out) {
    unsigned long long fl = 0;
    for (int64_t a = int64_t(blockIdx.x) * kBlock + threadIdx.x; a < n; a += int64_t(gridDim.x) * kBlock) {
        int64_t m = 0;
        for_admissible(c, a, fl, [&](int32_t, double) { ++m; });
        cnt[a] = m;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fl += __shfl_xor(fl, off, 64);
    if ((threadIdx.x & 63) == 0 && fl) atomicAdd(flagged_out + (blockIdx.x & (kAShards - 1)) * kAStride, fl);
}

__global__ __launch_bounds__(kBlock) void k_auc_fill(CandIn c, int64_t n, const int64_t *__restrict__ off,
                                                    int32_t *__restrict__ ck, float *__restrict__ cv) {
    unsigned long long fl = 0;
    for (int64_t a = int64_t(blockIdx.x) * kBlock + threadIdx.x; a < n; a += int64_t(gridDim.x) * kBlock) {
        int64_t p = off[a];
        for_admissible(c, a, fl, [&](int32_t k, double U) {
            ck[p] = k;
            cv[p] = float(U);
            ++p;
        });
    }
}

// ---------------------------------------------------------------- bidding
struct AucState {
    const int64_t *off;
    const int32_t *ck;
    const float *cv;
    const int32_t *ids;
    const uint32_t *sorted_ids;  // ascending IDs ...
    const int32_t *order;        // ... and their storage indices
    float *price;
    int32_t *owner;
    int32_t *assigned;
    uint8_t *out;
    unsigned long long *key;
    unsigned long long *ring;
    int64_t n, t;
    float eps;
};

// Best (ties -> lower task index) and second-best net over the lanes; bp: the best task's price
// as the lane loaded it (saves re-reading it after the reduction).
struct Best {
    float best, second, bp;
    int32_t bk;
};

__device__ __forceinline__ Best combine(Best x, Best y) {
    Best r;
    if (x.best > y.best || (x.best == y.best && x.bk < y.bk)) {
        r.best = x.best;
        r.bk = x.bk;
        r.bp = x.bp;
        r.second = fmaxf(x.second, y.best);
    } else {
        r.best = y.best;
        r.bk = y.bk;
        r.bp = y.bp;
        r.second = fmaxf(y.second, x.best);
    }
    return r;
}

// The whole wave evaluates agent a (wave-uniform call).  Returns the bid key (0: drop out) and
// the task in *bk.
// W lanes (a power of two <= 64, aligned within the wave) evaluate agent a together, U list
// entries per lane per pass.
template <int W, int U>
__device__ __forceinline__ unsigned long long group_bid(const AucState &s, int64_t a, int32_t *bk_out,
                                                        const unsigned long long *kprev = nullptr) {
    const int lane = threadIdx.x & (W - 1);
    Best m{-INFINITY, -INFINITY, 0.0f, INT_MAX};
    const int64_t b = s.off[a], e = s.off[a + 1];
    const uint32_t id = static_cast<uint32_t>(s.ids[a]);  // loaded beside the list bounds
    // kBidU list entries per lane per pass, all loads of a pass in flight (the result does not
    // depend on the combine order: ties go to the lower task index, second is a max)
    for (int64_t p0 = b + lane; p0 < e; p0 += W * U) {
        int32_t kk[U];
        float vv[U], pr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t p = p0 + W * u;
            kk[u] = p < e ? s.ck[p] : -1;
            vv[u] = p < e ? s.cv[p] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) pr[u] = kk[u] >= 0 ? s.price[kk[u]] : 0.0f;
        if (kprev) {  // fused rounds: the price after the previous round = max(price, its winning bid)
            unsigned long long kp[U];
#pragma unroll
            for (int u = 0; u < U; ++u) kp[u] = kk[u] >= 0 ? kprev[kk[u]] : 0ull;
#pragma unroll
            for (int u = 0; u < U; ++u) pr[u] = fmaxf(pr[u], __uint_as_float(static_cast<uint32_t>(kp[u] >> 32)));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (kk[u] >= 0) m = combine(m, Best{vv[u] - pr[u], -INFINITY, pr[u], kk[u]});
    }
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) {
        Best y;
        y.best = __shfl_xor(m.best, o, 64);
        y.second = __shfl_xor(m.second, o, 64);
        y.bp = __shfl_xor(m.bp, o, 64);
        y.bk = __shfl_xor(m.bk, o, 64);
        m = combine(m, y);
    }
    *bk_out = m.bk;
    if (!(m.best > 0.0f)) return 0ull;
    const float second = m.second < 0.0f ? 0.0f : m.second;
    const float inc = m.best - second;
    float bid = m.bp + inc;
    bid = bid + s.eps;
    return (static_cast<unsigned long long>(__float_as_uint(bid)) << 32) |
           static_cast<unsigned long long>(0xFFFFFFFFu - id);
}

__device__ __forceinline__ unsigned long long wave_bid(const AucState &s, int64_t a, int32_t *bk_out) {
    return group_bid<64, kBidU>(s, a, bk_out);
}

__device__ __forceinline__ int32_t index_of_id(const AucState &s, uint32_t id) {
    int64_t lo = 0, hi = s.n - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (s.sorted_ids[mid] < id) lo = mid + 1; else hi = mid;
    }
    return s.order[lo];
}

__global__ __launch_bounds__(kBlock) void k_auc_bid(AucState s, int64_t r) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = int64_t(gridDim.x) * (kBlock / kWave);
    unsigned long long nb = 0;
    for (int64_t a = int64_t(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6); a < s.n; a += nw) {
        if (s.assigned[a] >= 0 || s.out[a]) continue;  // wave-uniform
        ++nb;
        int32_t bk;
        const unsigned long long kk = wave_bid(s, a, &bk);
        if (lane == 0) {
            if (kk == 0) s.out[a] = 1;
            else atomicMax(&s.key[bk], kk);
        }
    }
    __shared__ unsigned long long s_nb[kBlock / kWave];
    if (lane == 0) s_nb[threadIdx.x >> 6] = nb;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long v = 0;
        for (int w = 0; w < kBlock / kWave; ++w) v += s_nb[w];
        if (v) atomicAdd(aslot(s.ring, r, blockIdx.x & (kAShards - 1)), v);
    }
}

// ---------------------------------------------------------------- list-driven rounds
// The multi-workgroup rounds keep the bidder list (the unassigned, active agents: it never grows)
// instead of scanning every agent and every task: round r's list -> bids (a wave per bidder) ->
// resolution per list entry (the standing key's bidder wins; losers and displaced owners form
// round r+1's list, appended with one global atomic per workgroup).  Task keys alternate
// halves by round parity; round r's resolution clears the keys round r-1 left.
struct AucList {
    int32_t *L[2];               // bidder lists by round parity
    int32_t *tgt[2];             // per entry: the task bid on (-1: dropped out)
    unsigned long long *mykey;   // per entry: this round's bid key
    unsigned *cnt;               // [2] list lengths by round parity
    int64_t *log;                // bidders per round, indexed by round
};

__global__ __launch_bounds__(kBlock) void k_auc_iota(int32_t *__restrict__ L, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        L[i] = int32_t(i);
}

__global__ __launch_bounds__(kBlock) void k_auc_bid_list(AucState s, AucList l, int64_t r) {
    const unsigned m = l.cnt[r & 1];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        l.log[r] = m;
        l.cnt[(r + 1) & 1] = 0;  // round r+1's list is appended by this round's resolution
    }
    unsigned long long *key = s.key + ((r & 1) ? s.t : 0);
    const int lane = threadIdx.x & 63;
    const int32_t *L = l.L[r & 1];
    int32_t *tgt = l.tgt[r & 1];
    const int64_t nw = int64_t(gridDim.x) * (kBlock / kWave);
    for (int64_t i = int64_t(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6); i < m; i += nw) {
        const int32_t a = L[i];
        int32_t bk;
        const unsigned long long kk = wave_bid(s, a, &bk);
        if (lane == 0) {
            tgt[i] = kk ? bk : -1;
            l.mykey[i] = kk;
            if (kk) atomicMax(&key[bk], kk);
            else s.out[a] = 1;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_auc_resolve_list(AucState s, AucList l, int64_t r) {
    __shared__ int s_n;
    __shared__ unsigned s_base;
    const int64_t m = l.log[r], mprev = r > 1 ? l.log[r - 1] : 0;
    unsigned long long *key = s.key + ((r & 1) ? s.t : 0), *key_prev = s.key + ((r & 1) ? 0 : s.t);
    const int32_t *L = l.L[r & 1], *tgt = l.tgt[r & 1], *tgt_prev = l.tgt[(r + 1) & 1];
    int32_t *Lnext = l.L[(r + 1) & 1];
    const int64_t span = m > mprev ? m : mprev;
    for (int64_t base = int64_t(blockIdx.x) * kBlock; base < span; base += int64_t(gridDim.x) * kBlock) {
        const int64_t i = base + threadIdx.x;
        if (i < mprev) {
            const int32_t k = tgt_prev[i];
            if (k >= 0) key_prev[k] = 0;
        }
        int32_t app = -1;
        if (i < m) {
            const int32_t k = tgt[i];
            if (k >= 0) {
                const int32_t a = L[i];
                const unsigned long long top = key[k];
                const int32_t prev = s.owner[k];
                if (top == l.mykey[i]) {
                    s.owner[k] = a;
                    s.assigned[a] = k;
                    s.price[k] = __uint_as_float(static_cast<uint32_t>(top >> 32));
                    if (prev >= 0) {
                        s.assigned[prev] = -1;
                        app = prev;
                    }
                } else {
                    app = a;
                }
            }
        }
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        const int pos = app >= 0 ? atomicAdd(&s_n, 1) : -1;
        __syncthreads();
        if (threadIdx.x == 0 && s_n) s_base = atomicAdd(&l.cnt[(r + 1) & 1], unsigned(s_n));
        __syncthreads();
        if (pos >= 0) Lnext[s_base + pos] = app;
        __syncthreads();
    }
}

// Before the tail kernel takes over at round r: clear the keys round r-1 left.
__global__ __launch_bounds__(kBlock) void k_auc_clear_keys(AucState s, AucList l, int64_t r) {
    const int64_t m = l.log[r - 1];
    unsigned long long *key = s.key + (((r - 1) & 1) ? s.t : 0);
    const int32_t *tgt = l.tgt[(r - 1) & 1];
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < m; i += int64_t(gridDim.x) * kBlock)
        if (tgt[i] >= 0) key[tgt[i]] = 0;
}

// ---------------------------------------------------------------- fused rounds
// Once the bidders are few enough that a round is launch- and latency-bound (<= fused_max), round q
// is ONE kernel: list entry i (one wave) first resolves entry i's bid of round q-1 -- it won iff its
// key still stands on its task -- and the agent that entry yields for round q (the loser itself, or
// the owner the winner displaced; at most one) bids right away in the same wave.  Its prices are
// those after round q-1: max(price, the task's winning bid of q-1), consistent whether or not that
// task's resolver has written the price yet (a bid always exceeds the price it was made at).  Task
// keys rotate over three buffers: round q bids into buf(q), resolves against buf(q-1) and clears
// what round q-2 left in buf(q-2) = buf(q+1).  Entries keep their index from round to round (holes
// where an entry yields no bidder); every batch starts from a fresh compact list (k_auc_rebuild).
struct AucFused {
    int32_t *L;                  // per entry: the agent bidding this round (-1: none)
    int32_t *tgt;                // per entry: the task it bid on (-1: none / dropped out)
    int32_t *tclr;               // per entry: the task its bid of the round before landed on
    unsigned long long *mykey;   // per entry: its bid key
    unsigned *cnt;               // list length (device)
};
enum AucFusedMode { AF_FIRST = 0, AF_NORMAL = 1, AF_RESOLVE_ONLY = 2 };

__device__ __forceinline__ unsigned long long *auc_kbuf(const AucState &s, int64_t q) {
    return s.key + size_t(q % 3) * size_t(s.t);
}

__global__ __launch_bounds__(kBlock) void k_auc_fused(AucState s, AucFused f, int64_t q, int mode) {
    const unsigned m = *f.cnt;
    if (blockIdx.x == 0)  // recycle the counter slot round q + kARing/2 will use
        for (int i = threadIdx.x; i < kAShards; i += kBlock) *aslot(s.ring, q + kARing / 2, i) = 0;
    const int lane = threadIdx.x & 63;
    unsigned long long *kcur = auc_kbuf(s, q), *kprev = auc_kbuf(s, q - 1), *kold = auc_kbuf(s, q + 1);
    const int64_t nw = int64_t(gridDim.x) * (kBlock / kWave);
    unsigned long long nb = 0;
    for (int64_t i = int64_t(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6); i < m; i += nw) {
        int32_t app = -1;
        if (lane == 0) {
            const int32_t a = f.L[i];
            if (mode == AF_FIRST) {
                app = a;
            } else {
                const int32_t c2 = f.tclr[i], k1 = f.tgt[i];
                if (c2 >= 0) kold[c2] = 0ull;  // round q-2's bid: nobody reads buf(q-2) this round
                if (a >= 0 && k1 >= 0) {
                    const unsigned long long top = kprev[k1];
                    const int32_t prev = s.owner[k1];
                    if (top == f.mykey[i]) {
                        s.owner[k1] = a;
                        s.assigned[a] = k1;
                        s.price[k1] = __uint_as_float(static_cast<uint32_t>(top >> 32));
                        if (prev >= 0) s.assigned[prev] = -1;
                        app = prev;
                    } else {
                        app = a;
                    }
                }
                f.tclr[i] = k1;
            }
        }
        app = __shfl(app, 0, 64);
        if (mode == AF_RESOLVE_ONLY || app < 0) {
            if (lane == 0) {
                f.L[i] = -1;
                f.tgt[i] = -1;
            }
            continue;
        }
        ++nb;
        int32_t bk;
        const unsigned long long kk = group_bid<64, kBidU>(s, app, &bk, mode == AF_FIRST ? nullptr : kprev);
        if (lane == 0) {
            f.L[i] = app;
            f.tgt[i] = kk ? bk : -1;
            f.mykey[i] = kk;
            if (kk) atomicMax(&kcur[bk], kk);
            else s.out[app] = 1;
        }
    }
    __shared__ unsigned long long s_nb[kBlock / kWave];
    if (lane == 0) s_nb[threadIdx.x >> 6] = nb;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long v = 0;
        for (int w = 0; w < kBlock / kWave; ++w) v += s_nb[w];
        if (v) atomicAdd(aslot(s.ring, q, blockIdx.x & (kAShards - 1)), v);
    }
}

// A fresh, compact list of the unassigned, active agents (every resolution done, keys zeroed).
__global__ __launch_bounds__(kBlock) void k_auc_rebuild(AucState s, AucFused f) {
    const int lane = threadIdx.x & 63;
    for (int64_t base = int64_t(blockIdx.x) * kBlock; base < s.n; base += int64_t(gridDim.x) * kBlock) {
        const int64_t a = base + threadIdx.x;
        const bool want = a < s.n && s.assigned[a] < 0 && !s.out[a];
        const unsigned long long bal = __ballot(want);
        unsigned pos0 = 0;
        if (lane == 0 && bal) pos0 = atomicAdd(f.cnt, unsigned(__popcll(bal)));
        pos0 = __shfl(pos0, 0, 64);
        if (want) {
            const unsigned p = pos0 + unsigned(__popcll(bal & ((1ull << lane) - 1)));
            f.L[p] = int32_t(a);
            f.tgt[p] = -1;
            f.tclr[p] = -1;
        }
    }
}

// Per-round bidder totals of rounds q0 .. q0 + gridDim.x - 1 (the ring's shards) -> out.
__global__ void k_auc_round_totals(unsigned long long *ring, int64_t q0, unsigned long long *out) {
    unsigned long long v = *aslot(ring, q0 + blockIdx.x, threadIdx.x);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// ---------------------------------------------------------------- the long tail, one workgroup
// Rounds r0, r0+1, ... until no agent bids or max_rounds: bidder list in LDS (the unassigned,
// active agents; it never grows: a round removes its winners and drop-outs and adds at most one
// displaced owner per winner).  Per round, two phases separated by workgroup barriers: bid (a
// wave per listed agent, atomicMax on the task key) and resolve (the bidder whose key stands
// wins; losers and displaced owners form the next list).  Keys are double-buffered by round
// parity, so the resolve phase also clears the previous round's keys -- no third phase.  The
// kernel is one workgroup on one XCD: its key atomics and loads are workgroup-scoped and stay
// in that XCD's L2 instead of travelling to the device-coherence point.
__global__ __launch_bounds__(kTailBlock) void k_auc_tail(AucState s, int64_t r0, int64_t max_rounds,
                                                        int64_t *__restrict__ log, int64_t *__restrict__ done) {
    __shared__ int32_t s_list[2][kTailCap];
    __shared__ int32_t s_tgt[2][kTailCap];
    __shared__ unsigned long long s_key[kTailCap];
    __shared__ int s_cnt[2];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int kWaves = kTailBlock / kWave;
    if (threadIdx.x == 0) s_cnt[0] = s_cnt[1] = 0;
    __syncthreads();
    for (int64_t a = threadIdx.x; a < s.n; a += kTailBlock)
        if (s.assigned[a] < 0 && !s.out[a]) {
            const int p = atomicAdd(&s_cnt[0], 1);
            if (p < kTailCap) s_list[0][p] = int32_t(a);
        }
    __syncthreads();
    int cur = 0, m_prev = 0;
    int64_t r = r0;
    for (; r <= max_rounds; ++r) {
        const int m = min(s_cnt[cur], kTailCap);
        if (m == 0) break;
        unsigned long long *key = s.key + ((r & 1) ? s.t : 0), *key_prev = s.key + ((r & 1) ? 0 : s.t);
        if (threadIdx.x == 0) log[r - r0] = m;
        // bid: a wave per bidder while there are at most as many bidders as waves, else 16-lane
        // groups (4 bidders per wave at once: fewer bidders in sequence per wave)
        auto post = [&](int i, int32_t a, unsigned long long kk, int32_t bk) {
            s_tgt[cur][i] = kk ? bk : -1;
            s_key[i] = kk;
            if (kk) __hip_atomic_fetch_max(&key[bk], kk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else s.out[a] = 1;
        };
        if (m <= kWaves) {
            for (int i = wid; i < m; i += kWaves) {
                const int32_t a = s_list[cur][i];
                int32_t bk;
                const unsigned long long kk = wave_bid(s, a, &bk);
                if (lane == 0) post(i, a, kk, bk);
            }
        } else {
            constexpr int kGl = 16;
            for (int i = threadIdx.x / kGl; i < m; i += kTailBlock / kGl) {
                const int32_t a = s_list[cur][i];
                int32_t bk;
                const unsigned long long kk = group_bid<kGl, 8>(s, a, &bk);
                if ((threadIdx.x & (kGl - 1)) == 0) post(i, a, kk, bk);
            }
        }
        if (threadIdx.x == 0) s_cnt[cur ^ 1] = 0;
        __syncthreads();
        // resolve: the standing key's bidder takes the task; losers bid again, the displaced
        // owner joins them.  Then clear the keys the previous round left.
        for (int i = threadIdx.x; i < m; i += kTailBlock) {
            const int32_t k = s_tgt[cur][i];
            if (k < 0) continue;
            const int32_t a = s_list[cur][i];
            const unsigned long long top = __hip_atomic_load(&key[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int32_t prev = s.owner[k];  // issued beside the key load
            if (top == s_key[i]) {
                s.owner[k] = a;
                s.assigned[a] = k;
                s.price[k] = __uint_as_float(static_cast<uint32_t>(top >> 32));
                if (prev >= 0) {
                    s.assigned[prev] = -1;
                    s_list[cur ^ 1][atomicAdd(&s_cnt[cur ^ 1], 1)] = prev;
                }
            } else {
                s_list[cur ^ 1][atomicAdd(&s_cnt[cur ^ 1], 1)] = a;
            }
        }
        for (int i = threadIdx.x; i < m_prev; i += kTailBlock) {
            const int32_t k = s_tgt[cur ^ 1][i];
            if (k >= 0) __hip_atomic_store(&key_prev[k], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        m_prev = m;
        cur ^= 1;
        __syncthreads();
    }
    // the last round's keys
    unsigned long long *key_last = s.key + (((r - 1) & 1) ? s.t : 0);
    for (int i = threadIdx.x; i < m_prev; i += kTailBlock) {
        const int32_t k = s_tgt[cur ^ 1][i];
        if (k >= 0) key_last[k] = 0;
    }
    if (threadIdx.x == 0) *done = r - r0;  // rounds this kernel ran (all had bidders)
}

// Fused rounds (one kernel per round) once a round had <= this many bidders (SWARM_AUCTION_FUSED,
// read per call; 0 = never, tests use it to exercise both paths).
int64_t auc_fused_threshold() {
    int64_t f = 8192;  // C4 sweep (tail 32): 2048..32768 all within 0.3 ms
    if (const char *e = getenv("SWARM_AUCTION_FUSED")) f = atoll(e);
    return f < 0 ? 0 : f;
}

// Hand the rounds to k_auc_tail once a round had <= this many bidders (SWARM_AUCTION_TAIL,
// read per call; 0 = never, tests use it to exercise both paths).
int auc_tail_threshold() {
    int tail = 32;  // C4 sweep after the fused rounds: 24..48 best
    if (const char *e = getenv("SWARM_AUCTION_TAIL")) tail = atoi(e);
    return tail < 0 ? 0 : (tail > kTailCap ? kTailCap : tail);
}

__global__ __launch_bounds__(kBlock) void k_count_bad_req(const int8_t *__restrict__ treq, int64_t t,
                                                         unsigned long long *__restrict__ out) {
    unsigned long long c = 0;
    for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < t; k += int64_t(gridDim.x) * kBlock)
        c += bad_req(treq[k]) ? 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// SWARM_ERR_ARG if any treq lies outside [-1, 31] (a capability index beyond the 32-bit mask).
int check_treq(swarm_ctx *ctx, int64_t t, const int8_t *treq, hipStream_t s) {
    if (t == 0) return SWARM_OK;
    unsigned long long *d;
    SW_ALLOC(d, ctx, S_TMP0, 64);
    SW_HIP(hipMemsetAsync(d, 0, 8, s));
    hipLaunchKernelGGL(k_count_bad_req, dim3(grid_for(t, kBlock, 256)), dim3(kBlock), 0, s, treq, t, d);
    SW_LAUNCHED();
    unsigned long long *h = static_cast<unsigned long long *>(pinned(ctx, 64));
    if (!h) return SWARM_ERR_OOM;
    SW_HIP(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    if (h[0]) {
        set_error("invalid argument: %llu task(s) with treq outside [-1, 31]", h[0]);
        return SWARM_ERR_ARG;
    }
    return SWARM_OK;
}

// Candidate lists, ascending-ID index, drop-out flags and round counters for n agents against t
// tasks (n, t > 0): everything but the task keys and the price / owner / assigned arrays.
int auc_prepare(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps, int64_t t,
                const double *tpos, const int8_t *treq, double claim_thr, double u_scale, float eps, AucState *out_st,
                int64_t *npairs_out, unsigned long long **flag_out, hipStream_t s) {
    // ---- candidate lists
    const double rc = u_scale / claim_thr - 1.0;  // U > thr  <=>  d < rc (has_cap)
    int64_t *off;
    unsigned long long *flag;
    SW_ALLOC(off, ctx, S_AUC_OFF, size_t(n + 1) * 8);
    SW_ALLOC(flag, ctx, S_ASTATS, size_t(kAShards) * kAStride * 8);
    SW_HIP(hipMemsetAsync(flag, 0, size_t(kAShards) * kAStride * 8, s));
    CandIn c{};
    c.apos = reinterpret_cast<const double2 *>(apos);
    c.acaps = acaps;
    c.tpos = reinterpret_cast<const double2 *>(tpos);
    c.treq = treq;
    c.thr = claim_thr;
    c.u_scale = u_scale;
    int64_t npairs = 0;
    if (rc > 0.0) {
        c.rp = rc * (1.0 + 1e-9) + 1e-12;
        c.rp2 = c.rp * c.rp;
        int rcode = make_grid(ctx, t, tpos, c.rp, 2 * t + 1024, &c.g, s);
        if (rcode) return rcode;
        int32_t *sorted;
        uint32_t *coff;
        if ((rcode = bin_agents(ctx, t, tpos, c.g, &sorted, &coff, s))) return rcode;
        c.sorted = sorted;
        c.cell_off = coff;
        const unsigned grid = grid_for(n, kBlock, 4096);
        SW_HIP(hipMemsetAsync(off, 0, 8, s));
        hipLaunchKernelGGL(k_auc_count, dim3(grid), dim3(kBlock), 0, s, c, n, off + 1, flag);
        SW_LAUNCHED();
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, off + 1, off + 1, int(n), s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, off + 1, off + 1, int(n), s));
        SW_HIP(hipMemcpyAsync(&npairs, off + n, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
    } else {
        SW_HIP(hipMemsetAsync(off, 0, size_t(n + 1) * 8, s));
    }
    int32_t *ck;
    float *cv;
    SW_ALLOC(ck, ctx, S_AUC_K, size_t(npairs + 1) * 4);
    SW_ALLOC(cv, ctx, S_AUC_V, size_t(npairs + 1) * 4);
    if (npairs) {
        hipLaunchKernelGGL(k_auc_fill, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, c, n, off, ck, cv);
        SW_LAUNCHED();
    }
    // ---- id -> storage index (ascending IDs), bid keys, flags, counters
    uint32_t *kin, *kout;
    int32_t *vin, *order;
    SW_ALLOC(kin, ctx, S_KEYS_IN, size_t(n) * 4);
    SW_ALLOC(kout, ctx, S_KEYS_OUT, size_t(n) * 4);
    SW_ALLOC(vin, ctx, S_VALS_IN, size_t(n) * 4);
    SW_ALLOC(order, ctx, S_ORDER, size_t(n) * 4);
    {
        SW_HIP(hipMemcpyAsync(kin, ids, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
        std::vector<int32_t> io(static_cast<size_t>(n));
        for (int64_t i = 0; i < n; ++i) io[size_t(i)] = int32_t(i);
        SW_HIP(hipMemcpyAsync(vin, io.data(), size_t(n) * 4, hipMemcpyHostToDevice, s));
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, order, int(n), 0, 32, s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, order, int(n), 0, 32, s));
        SW_HIP(hipStreamSynchronize(s));  // io leaves scope
    }
    AucState &st = *out_st;
    st = AucState{};
    st.off = off;
    st.ck = ck;
    st.cv = cv;
    st.ids = ids;
    st.sorted_ids = kout;
    st.order = order;
    st.n = n;
    st.t = t;
    st.eps = eps;
    SW_ALLOC(st.out, ctx, S_AUC_OUT, size_t(n));
    SW_ALLOC(st.ring, ctx, S_CHANGES, size_t(kARing) * kAShards * kAStride * 8);
    SW_HIP(hipMemsetAsync(st.out, 0, size_t(n), s));
    SW_HIP(hipMemsetAsync(st.ring, 0, size_t(kARing) * kAShards * kAStride * 8, s));
    *npairs_out = npairs;
    *flag_out = flag;
    return SWARM_OK;
}

// ---------------------------------------------------------------- sharded rounds
// Agents partitioned over ranks, tasks replicated.  Round r on every rank: its bidders bid into
// the key array (t task keys + one bidder-count word per rank), one element-wise MAX all-reduce
// makes the keys global, and every rank resolves all tasks identically (owners are agent IDs;
// each rank updates `assigned` of its own agents only).  Same rounds, bidder counts, prices and
// assignments as the single-GPU auction over the union of the agents.

// Storage index of agent ID `id` among this rank's agents, or -1.
__device__ __forceinline__ int32_t local_index(const AucState &s, uint32_t id) {
    if (s.n == 0) return -1;
    int64_t lo = 0, hi = s.n - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (s.sorted_ids[mid] < id) lo = mid + 1; else hi = mid;
    }
    return s.sorted_ids[lo] == id ? s.order[lo] : -1;
}

// This rank's bidders of round r (the ring slot's shards) -> *slot; the ring slot is recycled.
__global__ void k_auc_post_count(unsigned long long *ring, int64_t r, unsigned long long *slot) {
    unsigned long long *p = aslot(ring, r, threadIdx.x);
    unsigned long long v = *p;
    *p = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) *slot = v;
}

// All tasks, after the all-reduce: keys[0..t) task keys, keys[t..t+world) bidder counts.
__global__ __launch_bounds__(kBlock) void k_auc_resolve_ids(AucState s, int world, int64_t r,
                                                           int64_t *__restrict__ log) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int q = 0; q < world; ++q) {
            tot += s.key[s.t + q];
            s.key[s.t + q] = 0;
        }
        log[r] = int64_t(tot);
    }
    for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < s.t; k += int64_t(gridDim.x) * kBlock) {
        const unsigned long long kk = s.key[k];
        if (!kk) continue;
        const uint32_t w = 0xFFFFFFFFu - static_cast<uint32_t>(kk & 0xFFFFFFFFull);
        const int32_t prev = s.owner[k];
        if (prev >= 0) {
            const int32_t pi = local_index(s, uint32_t(prev));
            if (pi >= 0) s.assigned[pi] = -1;
        }
        s.owner[k] = int32_t(w);
        const int32_t wi = local_index(s, w);
        if (wi >= 0) s.assigned[wi] = int32_t(k);
        s.price[k] = __uint_as_float(static_cast<uint32_t>(kk >> 32));
        s.key[k] = 0;
    }
}

// ---- sparse bid exchange of the sharded rounds (round 4).  Each rank's bids of a round travel as
// a list, not as a dense t-key array: send buffer (u64 words) [0] = this rank's bidders (every
// unassigned, active agent: the per-round log), [1] = its bids, then cap entries {key, task}.  One
// all-gather of the (2 + 2 cap)-word buffers; every rank applies every rank's bids to its (zeroed)
// key array and resolves exactly the tasks that were bid on -- the same keys, owners and prices
// everywhere, as the dense MAX all-reduce gave.  cap (the host's bound on any rank's bids in a
// round) is the global bidder count of the last round it read: the global count never grows (a
// winner displaces at most the owner it replaces), so no rank can bid more.
constexpr int kBidHdr = 2;

__global__ __launch_bounds__(kBlock) void k_auc_bid_sparse(AucState s, int64_t r, unsigned long long *__restrict__ send,
                                                          int64_t cap) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = int64_t(gridDim.x) * (kBlock / kWave);
    unsigned long long nb = 0;
    for (int64_t a = int64_t(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6); a < s.n; a += nw) {
        if (s.assigned[a] >= 0 || s.out[a]) continue;  // wave-uniform
        ++nb;
        int32_t bk;
        const unsigned long long kk = wave_bid(s, a, &bk);
        if (lane == 0) {
            if (kk == 0) {
                s.out[a] = 1;
            } else {
                const unsigned long long slot = atomicAdd(send + 1, 1ull);
                if (slot < (unsigned long long)cap) {
                    send[kBidHdr + 2 * slot] = kk;
                    send[kBidHdr + 2 * slot + 1] = (unsigned long long)uint32_t(bk);
                }
            }
        }
    }
    __shared__ unsigned long long s_nb[kBlock / kWave];
    if (lane == 0) s_nb[threadIdx.x >> 6] = nb;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long v = 0;
        for (int w = 0; w < kBlock / kWave; ++w) v += s_nb[w];
        if (v) atomicAdd(aslot(s.ring, r, blockIdx.x & (kAShards - 1)), v);
    }
}

// send[0] <- this rank's bidders of round r (the ring slot, recycled)
__global__ void k_auc_post_sparse(unsigned long long *ring, int64_t r, unsigned long long *send) {
    unsigned long long *p = aslot(ring, r, threadIdx.x);
    unsigned long long v = *p;
    *p = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) send[0] = v;
}

// Every rank's bids (recv: world buffers of `words` u64) onto the key array; log[r] = global bidders.
__global__ __launch_bounds__(kBlock) void k_auc_apply_bids(AucState s, const unsigned long long *__restrict__ recv,
                                                          int world, int64_t words, int64_t cap, int64_t r,
                                                          int64_t *__restrict__ log, unsigned *__restrict__ err) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int q = 0; q < world; ++q) tot += recv[q * words];
        log[r] = int64_t(tot);
    }
    for (int q = 0; q < world; ++q) {
        const unsigned long long *b = recv + q * words;
        const unsigned long long nb = b[1];
        if (nb > (unsigned long long)cap) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 1u);
            continue;
        }
        for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < int64_t(nb); i += int64_t(gridDim.x) * kBlock)
            atomicMax(&s.key[b[kBidHdr + 2 * i + 1]], b[kBidHdr + 2 * i]);
    }
}

// Resolve exactly the tasks bid on: the first entry of a task to take its key (atomicExch) resolves
// it, as k_auc_resolve_ids does for every task; the key array is left zeroed.
__global__ __launch_bounds__(kBlock) void k_auc_resolve_bids(AucState s, const unsigned long long *__restrict__ recv,
                                                            int world, int64_t words, int64_t cap) {
    for (int q = 0; q < world; ++q) {
        const unsigned long long *b = recv + q * words;
        const int64_t nb = int64_t(b[1] < (unsigned long long)cap ? b[1] : (unsigned long long)cap);
        for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nb; i += int64_t(gridDim.x) * kBlock) {
            const int64_t k = int64_t(b[kBidHdr + 2 * i + 1]);
            const unsigned long long kk = atomicExch(&s.key[k], 0ull);
            if (!kk) continue;
            const uint32_t w = 0xFFFFFFFFu - static_cast<uint32_t>(kk & 0xFFFFFFFFull);
            const int32_t prev = s.owner[k];
            if (prev >= 0) {
                const int32_t pi = local_index(s, uint32_t(prev));
                if (pi >= 0) s.assigned[pi] = -1;
            }
            s.owner[k] = int32_t(w);
            const int32_t wi = local_index(s, w);
            if (wi >= 0) s.assigned[wi] = int32_t(k);
            s.price[k] = __uint_as_float(static_cast<uint32_t>(kk >> 32));
        }
    }
}

AucState auc_from_ctx(const swarm_ctx *ctx) {
    const AucPersist &p = ctx->auc;
    AucState st{};
    st.off = p.off;
    st.ck = p.ck;
    st.cv = p.cv;
    st.ids = p.ids;
    st.sorted_ids = p.sorted_ids;
    st.order = p.order;
    st.out = p.out;
    st.ring = p.ring;
    st.n = p.n;
    st.t = p.t;
    st.eps = p.eps;
    return st;
}

}  // namespace
}  // namespace swarm

extern "C" {

int swarm_auction(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps,
                  int64_t t, const double *tpos, const int8_t *treq, double claim_thr, double u_scale, float eps,
                  int32_t max_rounds, int32_t *owner, float *price, int32_t *assigned, int32_t *rounds_exec,
                  int64_t *bidders_per_round, swarm_auction_stats *stats, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && rounds_exec != nullptr, "NULL argument");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) && t >= 0 && t < (int64_t(1) << 31), "sizes out of range");
    SW_ARG(max_rounds >= 1, "max_rounds < 1");
    SW_ARG(std::isfinite(eps) && eps > 0.0f, "eps must be finite and > 0");
    SW_ARG(std::isfinite(claim_thr) && claim_thr > 0.0 && std::isfinite(u_scale) && u_scale > 0.0,
           "claim_thr and u_scale must be finite and > 0 (finite claim radius)");
    SW_ARG(n == 0 || (ids && apos && acaps && assigned), "NULL agent array");
    SW_ARG(t == 0 || (tpos && treq && owner && price), "NULL task array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int rc0 = check_treq(ctx, t, treq, s)) return rc0;
    if (stats) *stats = swarm_auction_stats{};
    if (n) SW_HIP(hipMemsetAsync(assigned, 0xFF, size_t(n) * 4, s));  // -1
    if (t) {
        SW_HIP(hipMemsetAsync(owner, 0xFF, size_t(t) * 4, s));
        SW_HIP(hipMemsetAsync(price, 0, size_t(t) * 4, s));
    }
    *rounds_exec = 0;
    if (n == 0 || t == 0) {  // no tasks: round 1's bidders (every agent) all drop out
        *rounds_exec = n ? 1 : 0;
        if (n && bidders_per_round) bidders_per_round[0] = n;
        if (stats) {
            stats->rounds_launched = n ? 2 : 1;
            stats->bids_total = n;
        }
        return SWARM_OK;
    }
    AucState st{};
    int64_t npairs = 0;
    unsigned long long *flag = nullptr;
    if (int rc = auc_prepare(ctx, n, ids, apos, acaps, t, tpos, treq, claim_thr, u_scale, eps, &st, &npairs, &flag, s))
        return rc;
    st.price = price;
    st.owner = owner;
    st.assigned = assigned;
    // three buffers: the fused rounds rotate over all of them, k_auc_tail double-buffers the first two
    SW_ALLOC(st.key, ctx, S_AUC_KEY, size_t(t) * 24);
    SW_HIP(hipMemsetAsync(st.key, 0, size_t(t) * 24, s));
    constexpr int kMaxBatch = 256;
    int64_t *dlog;
    SW_ALLOC(dlog, ctx, S_TMP1, (size_t(max_rounds) + 2) * 8);
    unsigned long long *h = static_cast<unsigned long long *>(pinned(ctx, size_t(kMaxBatch) * 8 + 64));
    if (!h) return SWARM_ERR_OOM;

    // bidder lists (round parity), per-entry targets and keys, list counters, per-round log
    AucList al{};
    AucFused af{};
    {
        char *p;
        const size_t nb = size_t(n) * 4;
        const size_t lsz = 4 * nb + size_t(n) * 8 + 64 + (size_t(max_rounds) + 2) * 8;
        SW_ALLOC(p, ctx, S_AUC_LIST, ((lsz + 63) & ~size_t(63)) + 3 * nb + size_t(n) * 8 + 64);
        {  // the fused rounds' entry arrays, behind the list-driven rounds' ones
            char *q = p + ((lsz + 63) & ~size_t(63));
            af.mykey = reinterpret_cast<unsigned long long *>(q);
            af.L = reinterpret_cast<int32_t *>(q + size_t(n) * 8);
            af.tgt = af.L + n;
            af.tclr = af.tgt + n;
            af.cnt = reinterpret_cast<unsigned *>(af.tclr + n);
        }
        al.L[0] = reinterpret_cast<int32_t *>(p);
        al.L[1] = reinterpret_cast<int32_t *>(p + nb);
        al.tgt[0] = reinterpret_cast<int32_t *>(p + 2 * nb);
        al.tgt[1] = reinterpret_cast<int32_t *>(p + 3 * nb);
        al.mykey = reinterpret_cast<unsigned long long *>(p + 4 * nb);
        al.cnt = reinterpret_cast<unsigned *>(p + 4 * nb + size_t(n) * 8);
        al.log = reinterpret_cast<int64_t *>(p + 4 * nb + size_t(n) * 8 + 64);
        const unsigned c0[2] = {0u, unsigned(n)};  // round 1 reads parity 1: every agent bids
        SW_HIP(hipMemcpyAsync(al.cnt, c0, 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_auc_iota, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, al.L[1], n);
        SW_LAUNCHED();
        SW_HIP(hipMemsetAsync(al.log, 0, (size_t(max_rounds) + 2) * 8, s));
        SW_HIP(hipStreamSynchronize(s));  // c0 leaves scope
    }
    const int64_t tail_thr = auc_tail_threshold();
    const int64_t fused_max = auc_fused_threshold();
    int64_t r = 1, found = -1, last_nb = n, launched = 0, tail_rounds = 0, total_bids = 0;
    int batch = 8;
    bool fused_mode = false;  // fused rounds have run (keys in three buffers, entries in af)
    bool pending = false;     // the last fused round's bids are not resolved yet
    // resolve what the last fused round left (a resolve-only round q) and zero every key buffer
    auto fused_flush = [&](int64_t q) -> int {
        if (pending) {
            hipLaunchKernelGGL(k_auc_fused, dim3(grid_for(last_nb, kBlock / kWave, 8192)), dim3(kBlock), 0, s, st, af, q,
                               int(AF_RESOLVE_ONLY));
            SW_LAUNCHED();
            pending = false;
        }
        SW_HIP(hipMemsetAsync(st.key, 0, size_t(t) * 24, s));
        return SWARM_OK;
    };
    while (r <= max_rounds && found < 0) {
        if (last_nb <= tail_thr) {  // the long tail: one workgroup runs every remaining round
            if (fused_mode) {
                if (int rc = fused_flush(r)) return rc;
            } else if (r > 1) {
                hipLaunchKernelGGL(k_auc_clear_keys, dim3(grid_for(last_nb, kBlock, 1024)), dim3(kBlock), 0, s, st, al,
                                   r);
                SW_LAUNCHED();
            }
            int64_t *ddone = dlog + max_rounds;
            hipLaunchKernelGGL(k_auc_tail, dim3(1), dim3(kTailBlock), 0, s, st, r, int64_t(max_rounds), dlog, ddone);
            SW_LAUNCHED();
            int64_t done = 0;
            SW_HIP(hipMemcpyAsync(&done, ddone, 8, hipMemcpyDeviceToHost, s));
            SW_HIP(hipStreamSynchronize(s));
            std::vector<int64_t> lg(static_cast<size_t>(done) + 1);
            if (done) SW_HIP(hipMemcpy(lg.data(), dlog, size_t(done) * 8, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < done; ++i) {
                if (bidders_per_round) bidders_per_round[r - 1 + i] = lg[size_t(i)];
                total_bids += lg[size_t(i)];
            }
            tail_rounds = done;
            launched = r + done;  // the round that found no bidder ran inside the kernel too
            r += done;
            if (r <= max_rounds) found = r;  // round r had no bidder
            break;
        }
        const int64_t rend = (max_rounds - r + 1 < batch) ? max_rounds : r + batch - 1;
        if (r > 1 && last_nb <= fused_max) {  // fused rounds: one kernel per round
            if (fused_mode) {
                if (int rc = fused_flush(r)) return rc;
            } else {
                SW_HIP(hipMemsetAsync(st.key, 0, size_t(t) * 24, s));  // the list-driven rounds' keys
                fused_mode = true;
            }
            SW_HIP(hipMemsetAsync(af.cnt, 0, sizeof(unsigned), s));
            hipLaunchKernelGGL(k_auc_rebuild, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, st, af);
            SW_LAUNCHED();
            const unsigned fgrid = grid_for(last_nb, kBlock / kWave, 8192);  // an upper bound: lists never grow
            for (int64_t q = r; q <= rend; ++q) {
                hipLaunchKernelGGL(k_auc_fused, dim3(fgrid), dim3(kBlock), 0, s, st, af, q,
                                   int(q == r ? AF_FIRST : AF_NORMAL));
                SW_LAUNCHED();
            }
            pending = true;
            launched = rend;
            hipLaunchKernelGGL(k_auc_round_totals, dim3(rend - r + 1), dim3(kWave), 0, s, st.ring, r,
                               reinterpret_cast<unsigned long long *>(dlog));
            SW_LAUNCHED();
            SW_HIP(hipMemcpyAsync(h, dlog, size_t(rend - r + 1) * 8, hipMemcpyDeviceToHost, s));
            SW_HIP(hipStreamSynchronize(s));
            for (int64_t q = r; q <= rend; ++q) {
                const int64_t nb = int64_t(h[q - r]);
                if (nb == 0) {
                    found = q;
                    pending = false;  // round q resolved round q-1 and placed no bid
                    break;
                }
                if (bidders_per_round) bidders_per_round[q - 1] = nb;
                total_bids += nb;
                last_nb = nb;
            }
            r = rend + 1;
            batch = batch < kMaxBatch ? batch * 2 : kMaxBatch;
            continue;
        }
        // grids sized by the last known bidder count: an upper bound (lists never grow)
        const unsigned bgrid = grid_for(last_nb, kBlock / kWave, 8192), rgrid = grid_for(last_nb, kBlock, 4096);
        for (int64_t q = r; q <= rend; ++q) {
            hipLaunchKernelGGL(k_auc_bid_list, dim3(bgrid), dim3(kBlock), 0, s, st, al, q);
            SW_LAUNCHED();
            hipLaunchKernelGGL(k_auc_resolve_list, dim3(rgrid), dim3(kBlock), 0, s, st, al, q);
            SW_LAUNCHED();
        }
        launched = rend;
        SW_HIP(hipMemcpyAsync(h, al.log + r, size_t(rend - r + 1) * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        for (int64_t q = r; q <= rend; ++q) {
            const int64_t nb = int64_t(h[q - r]);
            if (nb == 0) {
                found = q;
                break;
            }
            if (bidders_per_round) bidders_per_round[q - 1] = nb;
            total_bids += nb;
            last_nb = nb;
        }
        r = rend + 1;
        batch = batch < kMaxBatch ? batch * 2 : kMaxBatch;
    }
    if (pending && (fused_flush(r) != SWARM_OK)) return SWARM_ERR_HIP;  // max_rounds ended on a fused round
    *rounds_exec = int32_t(found > 0 ? found - 1 : max_rounds);
    if (stats) {
        unsigned long long fl[kAShards * kAStride];
        SW_HIP(hipMemcpyAsync(fl, flag, sizeof(fl), hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        int64_t nf = 0;
        for (int i = 0; i < kAShards; ++i) nf += int64_t(fl[i * kAStride]);
        stats->n_pairs = npairs;
        stats->n_flagged = nf;
        stats->rounds_launched = launched;
        stats->tail_rounds = tail_rounds;
        stats->bids_total = total_bids;
    }
    return found > 0 ? SWARM_OK : SWARM_NOT_CONVERGED;
}

int swarm_auction_begin(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *apos, const uint32_t *acaps,
                        int64_t t, const double *tpos, const int8_t *treq, double claim_thr, double u_scale, float eps,
                        int32_t *owner_id, float *price, int32_t *assigned, swarm_auction_stats *stats,
                        void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) && t >= 0 && t < (int64_t(1) << 31), "sizes out of range");
    SW_ARG(std::isfinite(eps) && eps > 0.0f, "eps must be finite and > 0");
    SW_ARG(std::isfinite(claim_thr) && claim_thr > 0.0 && std::isfinite(u_scale) && u_scale > 0.0,
           "claim_thr and u_scale must be finite and > 0 (finite claim radius)");
    SW_ARG(n == 0 || (ids && apos && acaps && assigned), "NULL agent array");
    SW_ARG(t == 0 || (tpos && treq && owner_id && price), "NULL task array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    ctx->auc = AucPersist{};
    if (int rc0 = check_treq(ctx, t, treq, s)) return rc0;
    if (stats) *stats = swarm_auction_stats{};
    if (n) SW_HIP(hipMemsetAsync(assigned, 0xFF, size_t(n) * 4, s));
    if (t) {
        SW_HIP(hipMemsetAsync(owner_id, 0xFF, size_t(t) * 4, s));
        SW_HIP(hipMemsetAsync(price, 0, size_t(t) * 4, s));
    }
    AucState st{};
    int64_t npairs = 0;
    unsigned long long *flag = nullptr;
    if (n > 0 && t > 0) {
        if (int rc = auc_prepare(ctx, n, ids, apos, acaps, t, tpos, treq, claim_thr, u_scale, eps, &st, &npairs, &flag,
                                 s))
            return rc;
    } else {  // nothing admissible: empty lists, every agent drops out in round 1
        int64_t *off0;
        SW_ALLOC(off0, ctx, S_AUC_OFF, size_t(n + 1) * 8);
        SW_HIP(hipMemsetAsync(off0, 0, size_t(n + 1) * 8, s));
        st.off = off0;
        SW_ALLOC(st.out, ctx, S_AUC_OUT, size_t(n) + 1);
        SW_HIP(hipMemsetAsync(st.out, 0, size_t(n) + 1, s));
        SW_ALLOC(st.ring, ctx, S_CHANGES, size_t(kARing) * kAShards * kAStride * 8);
        SW_HIP(hipMemsetAsync(st.ring, 0, size_t(kARing) * kAShards * kAStride * 8, s));
        st.ids = ids;
        st.n = n;
        st.t = t;
        st.eps = eps;
    }
    AucPersist &p = ctx->auc;
    p.n = n;
    p.t = t;
    p.npairs = npairs;
    p.eps = eps;
    p.ids = ids;
    p.off = const_cast<int64_t *>(st.off);
    p.ck = const_cast<int32_t *>(st.ck);
    p.cv = const_cast<float *>(st.cv);
    p.sorted_ids = const_cast<uint32_t *>(st.sorted_ids);
    p.order = const_cast<int32_t *>(st.order);
    p.out = st.out;
    p.ring = st.ring;
    p.ready = true;
    if (stats) {
        stats->n_pairs = npairs;
        if (flag) {
            unsigned long long fl[kAShards * kAStride];
            SW_HIP(hipMemcpyAsync(fl, flag, sizeof(fl), hipMemcpyDeviceToHost, s));
            SW_HIP(hipStreamSynchronize(s));
            for (int i = 0; i < kAShards; ++i) stats->n_flagged += int64_t(fl[i * kAStride]);
        }
    }
    return SWARM_OK;
}

int swarm_auction_bid(swarm_ctx *ctx, int64_t r, int32_t rank, int32_t world, uint64_t *keys, const float *price,
                      int32_t *assigned, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && ctx->auc.ready, "no swarm_auction_begin on this ctx");
    SW_ARG(r >= 1 && world >= 1 && rank >= 0 && rank < world && keys != nullptr, "bad round / rank / keys");
    hipStream_t s = static_cast<hipStream_t>(stream);
    AucState st = auc_from_ctx(ctx);
    st.key = reinterpret_cast<unsigned long long *>(keys);
    st.price = const_cast<float *>(price);
    st.assigned = assigned;
    hipLaunchKernelGGL(k_auc_bid, dim3(grid_for(st.n, kBlock / kWave, 8192)), dim3(kBlock), 0, s, st, r);
    SW_LAUNCHED();
    hipLaunchKernelGGL(k_auc_post_count, dim3(1), dim3(kWave), 0, s, st.ring, r, st.key + st.t + rank);
    SW_LAUNCHED();
    return SWARM_OK;
}

int swarm_auction_resolve(swarm_ctx *ctx, int64_t r, int32_t world, uint64_t *keys, int32_t *owner_id, float *price,
                          int32_t *assigned, int64_t *log, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && ctx->auc.ready, "no swarm_auction_begin on this ctx");
    SW_ARG(r >= 1 && world >= 1 && keys != nullptr && log != nullptr, "bad round / keys / log");
    hipStream_t s = static_cast<hipStream_t>(stream);
    AucState st = auc_from_ctx(ctx);
    st.key = reinterpret_cast<unsigned long long *>(keys);
    st.owner = owner_id;
    st.price = price;
    st.assigned = assigned;
    hipLaunchKernelGGL(k_auc_resolve_ids, dim3(grid_for(st.t, kBlock, 4096)), dim3(kBlock), 0, s, st, int(world), r,
                       log);
    SW_LAUNCHED();
    return SWARM_OK;
}

int swarm_auction_sharded(swarm_ctx *ctx, swarm_comm *comm, int64_t n, const int32_t *ids, const double *apos,
                          const uint32_t *acaps, int64_t t, const double *tpos, const int8_t *treq, double claim_thr,
                          double u_scale, float eps, int32_t max_rounds, int32_t *owner_id, float *price,
                          int32_t *assigned, int32_t *rounds_exec, int64_t *bidders_per_round,
                          swarm_auction_stats *stats, void *stream) {
    using namespace swarm;
    SW_ARG(rounds_exec != nullptr && max_rounds >= 1, "rounds_exec NULL or max_rounds < 1");
    int rank = 0, world = 1;
    if (int rc = comm_rank(comm, &rank, &world)) return rc;
    if (int rc = swarm_auction_begin(ctx, n, ids, apos, acaps, t, tpos, treq, claim_thr, u_scale, eps, owner_id, price,
                                     assigned, stats, stream))
        return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *keys;
    int64_t *dlog;
    SW_ALLOC(keys, ctx, S_AUC_KEY, size_t(t + world) * 8);
    SW_ALLOC(dlog, ctx, S_TMP1, (size_t(max_rounds) + 2) * 8);
    SW_HIP(hipMemsetAsync(keys, 0, size_t(t + world) * 8, s));
    constexpr int kMaxBatch = 256;
    int64_t *h = static_cast<int64_t *>(pinned(ctx, size_t(kMaxBatch) * 8 + 64));
    if (!h) return SWARM_ERR_OOM;
    // SWARM_AUCTION_EXCHANGE=dense: the round-3 exchange (one MAX all-reduce of all t task keys per
    // round); default: the round's bids as lists (k_auc_bid_sparse, one all-gather; see above)
    static const bool dense_x = [] {
        const char *e = getenv("SWARM_AUCTION_EXCHANGE");
        return e && strcmp(e, "dense") == 0;
    }();
    unsigned long long *send = nullptr, *recv = nullptr;
    unsigned *xerr = nullptr;
    int64_t cap = 0, cap0 = 0;
    AucState xs{};
    if (!dense_x) {
        // the first rounds' bound: the largest shard (a rank bids at most once per agent)
        unsigned long long *w;
        SW_ALLOC(w, ctx, S_TMP0, 64);
        const unsigned long long nn = (unsigned long long)n;
        SW_HIP(hipMemcpyAsync(w, &nn, 8, hipMemcpyHostToDevice, s));
        if (int rc = comm_allreduce_max_u64(comm, w, 1, s)) return rc;
        SW_HIP(hipMemcpyAsync(h, w, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        cap0 = cap = std::max<int64_t>(1, h[0]);
        // a round whose bound gives lists longer than the dense key array (2 cap + 2 >= t + world words)
        // takes the dense MAX all-reduce instead: the lists are only ever cap_list long
        const int64_t cap_list = std::max<int64_t>(1, std::min<int64_t>(cap0, (t + world - kBidHdr - 1) / 2));
        const size_t words0 = size_t(kBidHdr + 2 * cap_list);
        uint8_t *xb;
        SW_ALLOC(xb, ctx, S_AUC_LIST, (words0 * size_t(world + 1)) * 8 + 64);
        send = reinterpret_cast<unsigned long long *>(xb);
        recv = send + words0;
        xerr = reinterpret_cast<unsigned *>(recv + words0 * size_t(world));
        SW_HIP(hipMemsetAsync(xerr, 0, 4, s));
        xs = auc_from_ctx(ctx);
        xs.key = keys;
        xs.owner = owner_id;
        xs.price = price;
        xs.assigned = assigned;
    }
    int64_t r = 1, found = -1, launched = 0, total_bids = 0;
    int batch = 8;
    *rounds_exec = 0;
    while (r <= max_rounds && found < 0) {
        const int64_t rend = (max_rounds - r + 1 < batch) ? max_rounds : r + batch - 1;
        const int64_t words = kBidHdr + 2 * cap;
        const bool dense_batch = dense_x || words >= t + world;
        for (int64_t q = r; q <= rend; ++q) {
            if (dense_batch) {
                if (int rc = swarm_auction_bid(ctx, q, rank, world, reinterpret_cast<uint64_t *>(keys), price,
                                               assigned, stream))
                    return rc;
                if (int rc = comm_allreduce_max_u64(comm, keys, size_t(t + world), s)) return rc;
                if (int rc = swarm_auction_resolve(ctx, q, world, reinterpret_cast<uint64_t *>(keys), owner_id, price,
                                                   assigned, dlog, stream))
                    return rc;
                continue;
            }
            SW_HIP(hipMemsetAsync(send + 1, 0, 8, s));
            hipLaunchKernelGGL(k_auc_bid_sparse, dim3(grid_for(xs.n, kBlock / kWave, 8192)), dim3(kBlock), 0, s, xs, q,
                               send, cap);
            SW_LAUNCHED();
            hipLaunchKernelGGL(k_auc_post_sparse, dim3(1), dim3(kWave), 0, s, xs.ring, q, send);
            SW_LAUNCHED();
            if (int rc = comm_allgather_u64(comm, send, size_t(words), recv, s)) return rc;
            const unsigned g = grid_for(cap, kBlock, 1024);
            hipLaunchKernelGGL(k_auc_apply_bids, dim3(g), dim3(kBlock), 0, s, xs, recv, world, words, cap, q, dlog, xerr);
            SW_LAUNCHED();
            hipLaunchKernelGGL(k_auc_resolve_bids, dim3(g), dim3(kBlock), 0, s, xs, recv, world, words, cap);
            SW_LAUNCHED();
        }
        launched = rend;
        SW_HIP(hipMemcpyAsync(h, dlog + r, size_t(rend - r + 1) * 8, hipMemcpyDeviceToHost, s));
        if (xerr) SW_HIP(hipMemcpyAsync(h + kMaxBatch, xerr, 4, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        if (xerr && reinterpret_cast<const unsigned *>(h + kMaxBatch)[0]) {
            set_error("sharded auction: a rank's bids exceeded the exchange bound %lld", (long long)cap);
            return SWARM_ERR_HIP;
        }
        for (int64_t q = r; q <= rend; ++q) {
            const int64_t nb = h[q - r];
            if (nb == 0) {
                found = q;
                break;
            }
            if (bidders_per_round) bidders_per_round[q - 1] = nb;
            total_bids += nb;
        }
        // the global bidder count never grows: the last round read bounds every rank's bids from here
        if (!dense_x && found < 0) cap = std::max<int64_t>(1, std::min<int64_t>(cap0, h[rend - r]));
        r = rend + 1;
        batch = batch < kMaxBatch ? batch * 2 : kMaxBatch;
    }
    *rounds_exec = int32_t(found > 0 ? found - 1 : max_rounds);
    if (stats) {
        stats->rounds_launched = launched;
        stats->bids_total = total_bids;
    }
    return found > 0 ? SWARM_OK : SWARM_NOT_CONVERGED;
}

}  // extern "C"
