// Leader election (contract E2) on gfx950.
//
// Replaces the per-message handlers _handle_election_acclaim (agent.py:263-275) and
// _handle_heartbeat (agent.py:243-261) applied by every agent to every neighbour's
// re-advertised leader, one synchronous round at a time, starting from the state a won
// _check_election_timeout leaves (agent.py:234-241).  Under E2 both reduce to
//     leader'[v] = max(leader[v], max_{u in N(v)} leader[u])
// (verified bit-exact against the handlers; tests/golden/elect_*.npz).
//
// Two exact strategies:
//   DENSE     every round every agent gathers its whole CSR row (Jacobi, double-buffered).
//             HBM bytes per round = 12N + 8E (+ the gather, mostly served on-die).
//   FRONTIER  an agent can only change in round t+1 if a neighbour changed in round t, so
//             round t+1 gathers only those agents.  Same leaders, same per-round change
//             counts, same rounds_exec -- each agent's row is read O(changes) times instead
//             of O(rounds) times.  Per round: a 1-byte-per-agent stamp scan, the gathers of
//             active agents, a block-aggregated append of (agent, new leader), and an apply
//             pass that writes the new leaders and stamps their neighbours for round t+1.
//
// Gather: one wave serves 64 agents at once (lane = agent).  Their rows are concatenated
// virtually (wave prefix sum of degrees) and swept 64*U edges at a time, lane-contiguous, so
// col reads coalesce and each lane keeps U independent col loads and then U independent
// leader gathers in flight; each edge finds its row by a 6-step binary search over the lanes'
// row offsets and max-combines into a per-wave LDS slot.
//
// Counters: every per-round count (changes, active agents, edges) is a 64-way sharded 64-bit
// counter on its own 128-byte line, added once per workgroup: one contended counter per round
// costs ~12 ns per arrival (MI355X_MICROARCH.md, 'fanin'), i.e. ~0.8 ms per round at one
// arrival per wave at 10M agents.  The shards live in a ring of kRing rounds; the host zeroes
// a batch's slots before launching it and reads them back after.
#include <climits>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "swarm_common.h"

namespace swarm {
namespace {

constexpr int kShards = 64;
constexpr int kShardStride = 16;                    // u64 per shard: one 128-B line each
constexpr int kRing = 512;                          // rounds of counter slots
constexpr int kRoundWords = kShards * kShardStride; // u64 per round per counter
constexpr int kCounters = 3;                        // changes, active, edges
constexpr int kScan = 8;                            // stamps per thread (one 8-B load)
constexpr int kChunk = kBlock * kScan;              // agents per frontier work unit
constexpr int kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ unsigned long long *slot(unsigned long long *ring, int t, int counter, int shard) {
    return ring + (size_t(t % kRing) * kCounters + counter) * kRoundWords + size_t(shard) * kShardStride;
}

// Sum of the 64 change shards of round t (every thread of the block gets it).
__device__ __forceinline__ unsigned long long round_total(unsigned long long *ring, int t,
                                                          unsigned long long *s_bcast) {
    if (threadIdx.x < kWave) {
        unsigned long long v = *slot(ring, t, 0, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) *s_bcast = v;
    }
    __syncthreads();
    return *s_bcast;
}

__device__ __forceinline__ int wave_excl_scan(int v, int *total) {
    const int lane = threadIdx.x & 63;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    *total = __shfl(incl, 63, 64);
    return incl - v;
}

// 4-bit mask of the bytes of w equal to the byte replicated in b4 (exact, no carry leakage).
__device__ __forceinline__ unsigned bytes_eq4(unsigned w, unsigned b4) {
    const unsigned x = w ^ b4;
    const unsigned z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// Dense gather.  Wave task = 64 consecutive agents (lane = agent); their rows are one
// contiguous slice of col.  The slice is staged through LDS in windows of kWin edges with
// coalesced, unconditional (clamped) loads; then every lane reads its own row's part of the
// window from LDS and issues kK leader gathers at once (clamped, branch-free: a conditional
// load would make the compiler wait for it at the join).
constexpr int kWin = 1024;  // edges per LDS window per wave (4 KiB)
constexpr int kK = 16;      // gathers in flight per lane

template <typename Off, int K = kK>
__device__ __forceinline__ int row_max_from_lds(const int *s_col, Off w0, Off lo, Off hi,
                                                const int32_t *__restrict__ lin, int m) {
    for (Off k = lo; k < hi; k += K) {
        int c[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const Off kk = (k + j < hi) ? k + j : hi - 1;
            c[j] = s_col[kk - w0];
        }
        int val[K];
#pragma unroll
        for (int j = 0; j < K; ++j) val[j] = lin[c[j]];
#pragma unroll
        for (int j = 0; j < K; ++j) m = max(m, val[j]);  // duplicates of the last edge are harmless
    }
    return m;
}

// ---------------------------------------------------------------- dense Jacobi round
template <typename Off>
__global__ __launch_bounds__(kBlock) void k_elect_dense(
    const Off *__restrict__ rp, const int32_t *__restrict__ col, const int32_t *__restrict__ lin,
    int32_t *__restrict__ lout, int64_t n, unsigned long long *__restrict__ ring, int t, int guard) {
    __shared__ int s_col[kWavesPerBlock][kWin];
    __shared__ unsigned long long s_bc, s_cnt[kWavesPerBlock];
    if (guard && t > 1 && round_total(ring, t - 1, &s_bc) == 0) return;  // converged: no-op
    if (guard && blockIdx.x == 0)  // recycle the counter slots of round t + kRing/2
        for (int i = threadIdx.x; i < kCounters * kShards; i += kBlock)
            *slot(ring, t + kRing / 2, i / kShards, i % kShards) = 0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int *sc = s_col[wid];
    unsigned long long mine = 0;
    const int64_t ntask = (n + 63) / 64;
    const int64_t stride = int64_t(gridDim.x) * kWavesPerBlock;
    int64_t task = int64_t(blockIdx.x) * kWavesPerBlock + wid;
    // software pipeline: a task's row bounds are loaded during the previous task.  Lanes past
    // n get the empty row [rp[n], rp[n]) so lane 0 / lane 63 bound the wave's col slice.
    auto bounds = [&](int64_t tk, Off &b_, Off &e_) {
        const int64_t vv = tk * 64 + lane;
        b_ = rp[vv < n ? vv : n];
        e_ = rp[vv + 1 < n ? vv + 1 : n];
    };
    Off b = 0, e = 0;
    if (task < ntask) bounds(task, b, e);
    for (; task < ntask; task += stride) {
        const int64_t v = task * 64 + lane;
        const bool valid = v < n;
        const Off W0 = __shfl(b, 0, 64), W1 = __shfl(e, 63, 64);
        const int own = lin[valid ? v : n - 1];
        Off nb = 0, ne = 0;
        if (task + stride < ntask) bounds(task + stride, nb, ne);  // wave-uniform branch
        int m = INT_MIN;
        for (Off w0 = W0; w0 < W1; w0 += kWin) {
            const Off wend = (W1 - w0 < kWin) ? W1 : w0 + kWin;
#pragma unroll
            for (int j = 0; j < kWin / 64; ++j) {
                const Off k = w0 + j * 64 + lane;
                sc[j * 64 + lane] = col[k < wend ? k : wend - 1];
            }
            __builtin_amdgcn_wave_barrier();
            const Off lo = b > w0 ? b : w0, hi = e < wend ? e : wend;
            m = row_max_from_lds<Off>(sc, w0, lo, hi, lin, m);
            __builtin_amdgcn_wave_barrier();
        }
        const bool up = valid && m > own;
        if (valid) lout[v] = up ? m : own;
        mine += __popcll(__ballot(up));
        b = nb;
        e = ne;
    }
    if (lane == 0) s_cnt[wid] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += s_cnt[w];
        if (s) atomicAdd(slot(ring, t, 0, blockIdx.x & (kShards - 1)), s);
    }
}

// ------------------------------------------------------------- frontier: fused round
// One kernel per round.  Buffers alternate by round parity:
//   leaders  Lr = L[(t-1)&1] (state after round t-1, read), Lw = L[t&1] (written)
//   stamps   act[t&1] (agents active in round t carry t&255), act[(t+1)&1] (written)
// Invariant: before round t, Lw holds the state after round t-2.  An agent that changes in a
// round stamps its neighbours AND itself for the next round, so every agent that changed in
// round t-1 is active in round t; every active agent writes its round-t value to Lw.  Agents
// that changed in neither round t-1 nor t already hold the right value in Lw.  Hence Lw is the
// state after round t, with no fold, no change list and no global atomic on the critical path.
// A chunk's workgroup finds its active agents (8 stamp bytes per lane), compacts them in LDS and
// gathers them from Lr, kG lanes per agent with kKs loads in flight per lane.  (A dense variant
// that staged whole chunks through LDS windows measured no faster even on the first, nearly
// all-active rounds, and its registers cost occupancy: 62 VGPRs now = 8 waves per SIMD.)
// Counters are fire-and-forget shard adds.
constexpr int kG = 4;                    // sparse chunk: lanes per active agent
constexpr int kKs = 8;                   // sparse chunk: loads in flight per lane

template <typename Off>
__global__ __launch_bounds__(kBlock, sizeof(Off) == 4 ? 8 : 6) void k_frontier_round(
    const Off *__restrict__ rp, const int32_t *__restrict__ col, const int32_t *__restrict__ Lr,
    int32_t *__restrict__ Lw, const uint8_t *__restrict__ act_r, uint8_t *__restrict__ act_w,
    int64_t n, unsigned long long *__restrict__ ring, unsigned long long *__restrict__ tot, int t,
    int with_stats, int guard) {
    __shared__ struct {
        int list[kChunk];
    } u;
    __shared__ int s_wave[kWavesPerBlock];
    __shared__ long long s_red[3][kWavesPerBlock];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (blockIdx.x == 0) {  // bookkeeping: total of round t-1 (guard word), recycle slots
        if (t > 1 && threadIdx.x < kWave) {
            unsigned long long v = *slot(ring, t - 1, 0, threadIdx.x);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (threadIdx.x == 0) tot[(t - 1) % kRing] = v;
        }
        for (int i = threadIdx.x; i < kCounters * kShards; i += kBlock)
            *slot(ring, t + kRing / 2, i / kShards, i % kShards) = 0;
    }
    // single-GPU runs: round t-2 changed nothing => round t-1 had no active agent => neither t
    if (guard && t > 2 && tot[(t - 2) % kRing] == 0) return;
    const unsigned stamp = unsigned(t & 0xFF);
    const unsigned stamp4 = stamp * 0x01010101u;
    const uint8_t next = uint8_t((t + 1) & 0xFF);
    long long my_active = 0, my_edges = 0, my_chg = 0;
    const int64_t nchunks = (n + kChunk - 1) / kChunk;
    for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        const int64_t c0 = chunk * kChunk;
        // 1. my 8 stamps -> the chunk's active agents
        const int64_t v0 = c0 + int64_t(threadIdx.x) * kScan;
        unsigned mask = 0;
        if (v0 + kScan <= n) {
            const uint2 w = *reinterpret_cast<const uint2 *>(act_r + v0);
            mask = bytes_eq4(w.x, stamp4) | (bytes_eq4(w.y, stamp4) << 4);
        } else {
            for (int j = 0; j < kScan && v0 + j < n; ++j)
                if (act_r[v0 + j] == stamp) mask |= 1u << j;
        }
        const int cnt = __popc(mask);
        int wtot;
        const int wexcl = wave_excl_scan(cnt, &wtot);
        if (lane == 0) s_wave[wid] = wtot;
        __syncthreads();
        int off = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) {
            off += (w < wid) ? s_wave[w] : 0;
            total += s_wave[w];
        }
        if (total > 0) {
            // 2. compacted active agents, kG lanes per agent, kKs loads per lane
            int pos = off + wexcl;
            while (mask) {
                const int j = __ffs(mask) - 1;
                mask &= mask - 1;
                u.list[pos++] = threadIdx.x * kScan + j;
            }
            __syncthreads();
            const int sub = lane & (kG - 1);
            for (int base = wid * (64 / kG); base < total; base += kBlock / kG) {
                const int i = base + lane / kG;
                const bool valid = i < total;
                const int64_t v = c0 + u.list[valid ? i : total - 1];
                const Off b = rp[v], e = rp[v + 1];
                const int own = Lr[v];
                int m = own;
                int c[kKs];
                for (Off k = b + sub * kKs; k < e; k += kG * kKs) {
#pragma unroll
                    for (int j = 0; j < kKs; ++j) c[j] = col[(k + j < e) ? k + j : e - 1];
                    int val[kKs];
#pragma unroll
                    for (int j = 0; j < kKs; ++j) val[j] = Lr[c[j]];
#pragma unroll
                    for (int j = 0; j < kKs; ++j) m = max(m, val[j]);
                }
#pragma unroll
                for (int o2 = 1; o2 < kG; o2 <<= 1) m = max(m, __shfl_xor(m, o2, 64));
                const bool up = valid && m > own;
                if (valid && sub == 0) Lw[v] = m;
                if (up) {
                    if (sub == 0) act_w[v] = next;
                    if (e - b <= kG * kKs) {  // one pass per lane: c[] still holds this lane's edges
#pragma unroll
                        for (int j = 0; j < kKs; ++j)
                            if (b + sub * kKs + j < e) act_w[c[j]] = next;
                    } else {
                        for (Off k = b + sub; k < e; k += kG) act_w[col[k]] = next;
                    }
                }
                my_chg += __popcll(__ballot(up && sub == 0));
                if (with_stats && valid && sub == 0) {
                    my_active += 1;
                    my_edges += (long long)(e - b);
                }
            }
        }
        __syncthreads();  // LDS (s_wave, u) reused by the next chunk
    }
    // per-workgroup totals -> one shard add per counter
    if (lane == 0) s_red[0][wid] = my_chg;  // my_chg is wave-uniform (ballot counts)
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
        my_active += __shfl_xor(my_active, o2, 64);
        my_edges += __shfl_xor(my_edges, o2, 64);
    }
    if (lane == 0) { s_red[1][wid] = my_active; s_red[2][wid] = my_edges; }
    __syncthreads();
    if (threadIdx.x < kCounters) {
        long long a = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) a += s_red[threadIdx.x][w];
        if (a) atomicAdd(slot(ring, t, threadIdx.x, blockIdx.x & (kShards - 1)), (unsigned long long)a);
    }
}

// Sharded runs: halo values received for ghost agents [begin, begin + count) after round t.
// A ghost whose leader rose is written to BOTH leader buffers (ghosts are never gathered, so
// either buffer may serve round t+1 and t+2) and its local neighbours are stamped for round
// t+1 (ghost rows of the local CSR list them).  Ghost changes are counted by their owner.
template <int G, typename Off>
__global__ __launch_bounds__(kBlock) void k_frontier_ghosts(
    const Off *__restrict__ rp, const int32_t *__restrict__ col, int32_t *__restrict__ L0,
    int32_t *__restrict__ L1, uint8_t *__restrict__ act_w, int64_t begin, int64_t count,
    const int32_t *__restrict__ incoming, int t) {
    const uint8_t next = uint8_t((t + 1) & 0xFF);
    int32_t *Lcur = (t & 1) ? L1 : L0;
    constexpr int GPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    for (int64_t base = int64_t(blockIdx.x) * GPB; base < count; base += int64_t(gridDim.x) * GPB) {
        const int64_t i = base + threadIdx.x / G;
        if (i < count) {
            const int64_t g = begin + i;
            const int nv = incoming[i];
            if (nv > Lcur[g]) {
                if (sub == 0) {
                    L0[g] = nv;
                    L1[g] = nv;
                }
                const Off e1 = rp[g + 1];
                for (Off k = rp[g] + sub; k < e1; k += G) act_w[col[k]] = next;
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_state(const int32_t *__restrict__ leader,
                                                 const int32_t *__restrict__ ids,
                                                 uint8_t *__restrict__ state, int64_t n) {
    for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < n;
         v += int64_t(gridDim.x) * kBlock)
        state[v] = leader[v] == ids[v] ? SWARM_LEADER : SWARM_FOLLOWER;
}

// *out += sum of the 64 change shards of ring round t (single-round API).
__global__ void k_sum_shards(unsigned long long *ring, int t, unsigned long long *out) {
    unsigned long long v = *slot(ring, t, 0, threadIdx.x);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (threadIdx.x == 0) *out += v;
}

// totals[(r - t0) * 3 + c] = sum over shards of counter c of round r, one wave per round.
__global__ void k_batch_totals(unsigned long long *ring, int t0, unsigned long long *totals) {
    const int r = t0 + blockIdx.x;
#pragma unroll
    for (int c = 0; c < kCounters; ++c) {
        unsigned long long v = *slot(ring, r, c, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) totals[size_t(blockIdx.x) * kCounters + c] = v;
    }
}

int env_int(const char *name, int dflt) {
    const char *s = getenv(name);
    return s ? atoi(s) : dflt;
}

struct Tuning {
    int dense_blocks = 2048;     // grid cap of the dense round kernel
    Tuning() { dense_blocks = env_int("SWARM_DENSE_BLOCKS", 2048); }
};

const Tuning &tuning() {
    static Tuning tu;
    return tu;
}

template <typename Off>
int launch_dense_round(const Off *rp, const int32_t *col, const int32_t *lin, int32_t *lout,
                       int64_t n, unsigned long long *ring, int t, int guard, hipStream_t s) {
    const unsigned grid = grid_for((n + 63) / 64, kWavesPerBlock, unsigned(tuning().dense_blocks));
    hipLaunchKernelGGL((k_elect_dense<Off>), dim3(grid), dim3(kBlock), 0, s, rp, col, lin, lout, n,
                       ring, t, guard);
    SW_LAUNCHED();
    return SWARM_OK;
}

// Frontier state: two leader buffers and two stamp arrays (round parity), counter ring.
struct Frontier {
    int32_t *L[2];
    uint8_t *act[2];
    unsigned long long *ring, *tot;
    int64_t n_rows;
};

int frontier_alloc(swarm_ctx *ctx, int64_t n_rows, int64_t n_all, int32_t *L0, int32_t *L1, Frontier *f,
                   hipStream_t s) {
    const size_t na = size_t(n_all) + 16;
    uint8_t *act;
    SW_ALLOC(act, ctx, S_ACT, 2 * na);
    const size_t ring_words = size_t(kRing) * kCounters * kRoundWords;
    SW_ALLOC(f->ring, ctx, S_CHANGES, (ring_words + kRing) * 8);
    f->tot = f->ring + ring_words;
    f->L[0] = L0;
    f->L[1] = L1;
    f->act[0] = act;
    f->act[1] = act + na;
    f->n_rows = n_rows;
    SW_HIP(hipMemsetAsync(f->ring, 0, (ring_words + kRing) * 8, s));
    SW_HIP(hipMemsetAsync(act, 0, 2 * na, s));
    if (n_all) SW_HIP(hipMemsetAsync(f->act[1], 1, size_t(n_all), s));  // round 1 reads act[1]: all active
    return SWARM_OK;
}

template <typename Off>
int launch_frontier_round(const Off *rp, const int32_t *col, const Frontier &f, int t, int with_stats,
                          int guard, hipStream_t s) {
    const int64_t nchunks = (f.n_rows + kChunk - 1) / kChunk;
    const unsigned grid = grid_for(nchunks > 0 ? nchunks : 1, 1, 1u << 20);
    const int r = t & 1, p = r ^ 1;
    hipLaunchKernelGGL((k_frontier_round<Off>), dim3(grid), dim3(kBlock), 0, s, rp, col, f.L[p], f.L[r],
                       f.act[r], f.act[p], f.n_rows, f.ring, f.tot, t, with_stats, guard);
    SW_LAUNCHED();
    return SWARM_OK;
}

template <typename Off>
int elect_impl(swarm_ctx *ctx, int64_t n, const Off *rp, const int32_t *col, const int32_t *ids,
               int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
               int32_t *rounds_exec, int64_t *changes_host, swarm_elect_stats *st,
               void *stream) {
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0, "n < 0");
    SW_ARG(n < (int64_t(1) << 31), "n must be < 2^31");
    SW_ARG(max_rounds >= 1, "max_rounds < 1");
    const bool timed = (mode & SWARM_ELECT_TIMED) != 0;
    mode &= ~SWARM_ELECT_TIMED;
    SW_ARG(mode == SWARM_ELECT_DENSE || mode == SWARM_ELECT_FRONTIER, "unknown mode");
    SW_ARG(rounds_exec != nullptr, "rounds_exec is NULL");
    SW_ARG(n == 0 || (rp && ids && leader && state), "NULL array (col may be NULL only without edges)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st) *st = swarm_elect_stats{0, 0, 0, 0, 0.0, 0.0, 0};
    if (n == 0) {  // an empty swarm: round 1 changes nothing
        *rounds_exec = 1;
        if (changes_host) changes_host[0] = 0;
        if (st) st->rounds_launched = 1;
        return SWARM_OK;
    }
    int32_t *bufs[2] = {leader, nullptr};
    SW_ALLOC(bufs[1], ctx, S_LEADER_B, size_t(n) * 4);
    SW_HIP(hipMemcpyAsync(leader, ids, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
    Frontier f{};
    unsigned long long *ring;
    const size_t ring_words = size_t(kRing) * kCounters * kRoundWords;
    if (mode == SWARM_ELECT_FRONTIER) {
        SW_HIP(hipMemcpyAsync(bufs[1], ids, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
        int rc0 = frontier_alloc(ctx, n, n, bufs[0], bufs[1], &f, s);
        if (rc0) return rc0;
        ring = f.ring;
    } else {
        SW_ALLOC(ring, ctx, S_CHANGES, (ring_words + kRing) * 8);
    }
    const int with_stats = (st != nullptr && mode == SWARM_ELECT_FRONTIER) ? 1 : 0;
    constexpr int kMaxBatch = 256;
    const size_t per_round = size_t(kCounters) * kRoundWords;
    unsigned long long *hbuf = static_cast<unsigned long long *>(pinned(ctx, size_t(kCounters) * 8 * kMaxBatch));
    if (!hbuf) return SWARM_ERR_OOM;
    unsigned long long *dtot;
    SW_ALLOC(dtot, ctx, S_ESTATS, size_t(kCounters) * 8 * kMaxBatch);

    int found = -1, t = 1, batch = 8, launched = 0;
    int64_t act_sum = 0, edge_sum = 0, chg_sum = 0;
    // optional per-kernel timing: events [3r] before gather, [3r+1] between, [3r+2] after apply
    std::vector<hipEvent_t> ev;
    double g_ms = 0, a_ms = 0;
    int64_t timed_rounds = 0;
    if (timed) {
        ev.resize(3 * kMaxBatch);
        for (auto &x : ev) SW_HIP(hipEventCreate(&x));
    }
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() { for (auto x : v) (void)hipEventDestroy(x); }
    } ev_free{ev};
    // every counter slot starts at zero; afterwards each round's kernel recycles the slots of
    // the round kRing/2 ahead
    if (mode == SWARM_ELECT_DENSE) SW_HIP(hipMemsetAsync(ring, 0, (ring_words + kRing) * 8, s));
    (void)per_round;
    // slot of round 0 (read by round 1's guard only when t > 1: never) stays untouched
    while (t <= max_rounds && found < 0) {
        const int tend = (max_rounds - t + 1 < batch) ? max_rounds : t + batch - 1;
        int rc = 0;
        for (int r = t; r <= tend; ++r) {
            hipEvent_t *e3 = timed ? &ev[3 * (r - t)] : nullptr;
            if (e3) SW_HIP(hipEventRecord(e3[0], s));
            rc = (mode == SWARM_ELECT_DENSE)
                     ? launch_dense_round<Off>(rp, col, bufs[(r - 1) & 1], bufs[r & 1], n, ring, r, 1, s)
                     : launch_frontier_round<Off>(rp, col, f, r, with_stats, /*guard=*/1, s);
            if (rc) return rc;
            if (e3) SW_HIP(hipEventRecord(e3[2], s));
        }
        launched = tend;
        // per-round totals of rounds [t, tend], reduced on device, then one small copy
        hipLaunchKernelGGL(k_batch_totals, dim3(tend - t + 1), dim3(kWave), 0, s, ring, t, dtot);
        SW_LAUNCHED();
        SW_HIP(hipMemcpyAsync(hbuf, dtot, size_t(tend - t + 1) * kCounters * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        for (int r = t; r <= tend; ++r) {
            const unsigned long long *rb = hbuf + size_t(r - t) * kCounters;
            const unsigned long long c = rb[0], a = rb[1], ed = rb[2];
            if (changes_host) changes_host[r - 1] = int64_t(c);
            act_sum += int64_t(a);
            edge_sum += int64_t(ed);
            chg_sum += int64_t(c);
            if (timed) {
                float x = 0, y = 0;
                hipEvent_t *e3 = &ev[3 * (r - t)];
                SW_HIP(hipEventElapsedTime(&x, e3[0], e3[2]));  // one kernel per round
                g_ms += x;
                a_ms += y;
                ++timed_rounds;
            }
            if (c == 0) {
                found = r;
                break;
            }
        }
        t = tend + 1;
        batch = batch < kMaxBatch ? batch * 2 : kMaxBatch;
    }
    const int last = found > 0 ? found : max_rounds;
    // after a zero-change round both buffers hold the final state (dense and frontier alike);
    // otherwise the newest is bufs[last & 1]
    if (found < 0 && (last & 1))
        SW_HIP(hipMemcpyAsync(leader, bufs[1], size_t(n) * 4, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_state, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, leader,
                       ids, state, n);
    SW_LAUNCHED();
    *rounds_exec = last;
    if (st) {
        st->rounds_launched = launched;
        st->changes_total = chg_sum;
        st->gather_ms = g_ms;
        st->apply_ms = a_ms;
        st->gather_launches = timed_rounds;
        if (mode == SWARM_ELECT_DENSE) {
            Off e = 0;
            SW_HIP(hipMemcpyAsync(&e, rp + n, sizeof(Off), hipMemcpyDeviceToHost, s));
            SW_HIP(hipStreamSynchronize(s));
            st->active_total = n * int64_t(last);
            st->edges_total = int64_t(e) * int64_t(last);
        } else {
            st->active_total = act_sum;
            st->edges_total = edge_sum;
        }
    }
    return found > 0 ? SWARM_OK : SWARM_NOT_CONVERGED;
}

}  // namespace

// Internal entry points for comm.hip (the RCCL round loop): one stepper round, and the device
// per-round totals [changes, active, edges] of rounds t0..t1 into dtot.
int frontier_round_stepper(swarm_ctx *ctx, int t, const int32_t *rp, const int32_t *col, int32_t *L0,
                           int32_t *L1, hipStream_t s, uint8_t **act_next) {
    Frontier f{};
    SW_ARG(ctx->slot[S_ACT] != nullptr && ctx->slot[S_CHANGES] != nullptr, "swarm_frontier_begin first");
    const size_t na = size_t(ctx->step_all) + 16;
    f.L[0] = L0;
    f.L[1] = L1;
    f.act[0] = static_cast<uint8_t *>(ctx->slot[S_ACT]);
    f.act[1] = f.act[0] + na;
    f.ring = static_cast<unsigned long long *>(ctx->slot[S_CHANGES]);
    f.tot = f.ring + size_t(kRing) * kCounters * kRoundWords;
    f.n_rows = ctx->step_rows;
    *act_next = f.act[(t + 1) & 1];
    if (f.n_rows == 0) return SWARM_OK;
    return launch_frontier_round<int32_t>(rp, col, f, t, 0, /*guard=*/0, s);
}

int frontier_round_totals(swarm_ctx *ctx, int t0, int t1, unsigned long long *dtot, hipStream_t s) {
    SW_ARG(t1 >= t0 && t1 - t0 < kRing / 2, "round range");
    unsigned long long *ring = static_cast<unsigned long long *>(ctx->slot[S_CHANGES]);
    hipLaunchKernelGGL(k_batch_totals, dim3(t1 - t0 + 1), dim3(kWave), 0, s, ring, t0, dtot);
    SW_LAUNCHED();
    return SWARM_OK;
}

}  // namespace swarm

extern "C" {

int swarm_elect(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds,
                int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                swarm_elect_stats *stats, void *stream) {
    return swarm::elect_impl<int32_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode,
                                      rounds_exec, changes_per_round, stats, stream);
}

int swarm_elect_i64(swarm_ctx *ctx, int64_t n, const int64_t *row_ptr, const int32_t *col,
                    const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds,
                    int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                    swarm_elect_stats *stats, void *stream) {
    return swarm::elect_impl<int64_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode,
                                      rounds_exec, changes_per_round, stats, stream);
}

int swarm_frontier_begin(swarm_ctx *ctx, int64_t n_rows, int64_t n_all, const int32_t *init,
                         int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n_rows >= 0 && n_all >= n_rows && n_all < (int64_t(1) << 31), "sizes out of range");
    SW_ARG(n_all == 0 || (init && leader0 && leader1), "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    Frontier f{};
    int rc = frontier_alloc(ctx, n_rows, n_all, leader0, leader1, &f, s);
    if (rc) return rc;
    if (n_all) {
        SW_HIP(hipMemcpyAsync(leader0, init, size_t(n_all) * 4, hipMemcpyDeviceToDevice, s));
        SW_HIP(hipMemcpyAsync(leader1, init, size_t(n_all) * 4, hipMemcpyDeviceToDevice, s));
    }
    ctx->step_rows = n_rows;
    ctx->step_all = n_all;
    return SWARM_OK;
}

static int stepper_state(swarm_ctx *ctx, int32_t *leader0, int32_t *leader1, swarm::Frontier *f) {
    using namespace swarm;
    SW_ARG(ctx->slot[S_ACT] != nullptr && ctx->slot[S_CHANGES] != nullptr, "swarm_frontier_begin first");
    const size_t na = size_t(ctx->step_all) + 16;
    f->L[0] = leader0;
    f->L[1] = leader1;
    f->act[0] = static_cast<uint8_t *>(ctx->slot[S_ACT]);
    f->act[1] = f->act[0] + na;
    f->ring = static_cast<unsigned long long *>(ctx->slot[S_CHANGES]);
    f->tot = f->ring + size_t(kRing) * kCounters * kRoundWords;
    f->n_rows = ctx->step_rows;
    return SWARM_OK;
}

int swarm_frontier_step(swarm_ctx *ctx, int32_t t, const int32_t *row_ptr, const int32_t *col,
                        int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(t >= 1, "round must be >= 1");
    if (ctx->step_rows == 0) return SWARM_OK;
    SW_ARG(row_ptr && leader0 && leader1, "NULL array");
    Frontier f{};
    int rc = stepper_state(ctx, leader0, leader1, &f);
    if (rc) return rc;
    return launch_frontier_round<int32_t>(row_ptr, col, f, t, 0, /*guard=*/0, static_cast<hipStream_t>(stream));
}

int swarm_frontier_ghosts(swarm_ctx *ctx, int32_t t, int64_t begin, int64_t count,
                          const int32_t *incoming, const int32_t *row_ptr, const int32_t *col,
                          int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(begin >= 0 && count >= 0 && begin + count <= ctx->step_all, "ghost range out of bounds");
    if (count == 0) return SWARM_OK;
    SW_ARG(incoming && row_ptr && leader0 && leader1, "NULL array");
    Frontier f{};
    int rc = stepper_state(ctx, leader0, leader1, &f);
    if (rc) return rc;
    hipLaunchKernelGGL((k_frontier_ghosts<8, int32_t>), dim3(grid_for(count, kBlock / 8, 2048)), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), row_ptr, col, leader0, leader1,
                       f.act[(t + 1) & 1], begin, count, incoming, t);
    SW_LAUNCHED();
    return SWARM_OK;
}

int swarm_frontier_changes(swarm_ctx *ctx, int32_t t0, int32_t t1, int64_t *out, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && out != nullptr, "NULL argument");
    SW_ARG(t0 >= 1 && t1 >= t0 && t1 - t0 < kRing / 2, "round range must be 1 <= t0 <= t1 < t0 + 256");
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *ring = static_cast<unsigned long long *>(ctx->slot[S_CHANGES]);
    SW_ARG(ring != nullptr, "swarm_frontier_begin first");
    const int nr = t1 - t0 + 1;
    unsigned long long *dtot;
    SW_ALLOC(dtot, ctx, S_ESTATS, size_t(kCounters) * 8 * (kRing / 2));
    hipLaunchKernelGGL(k_batch_totals, dim3(nr), dim3(kWave), 0, s, ring, t0, dtot);
    SW_LAUNCHED();
    unsigned long long *h = static_cast<unsigned long long *>(pinned(ctx, size_t(kCounters) * 8 * (kRing / 2)));
    if (!h) return SWARM_ERR_OOM;
    SW_HIP(hipMemcpyAsync(h, dtot, size_t(nr) * kCounters * 8, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < nr; ++i) out[i] = int64_t(h[size_t(i) * kCounters]);
    return SWARM_OK;
}

int swarm_elect_round(swarm_ctx *ctx, int64_t n_rows, const int32_t *row_ptr,
                      const int32_t *col, const int32_t *leader_in, int32_t *leader_out,
                      int64_t *changed, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n_rows >= 0 && n_rows < (int64_t(1) << 31), "n_rows out of range");
    SW_ARG(changed != nullptr, "changed is NULL");
    if (n_rows == 0) return SWARM_OK;
    SW_ARG(row_ptr && leader_in && leader_out, "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *ring;
    SW_ALLOC(ring, ctx, S_TMP0, size_t(kCounters) * kRoundWords * 8);
    SW_HIP(hipMemsetAsync(ring, 0, size_t(kRoundWords) * 8, s));
    int rc = launch_dense_round<int32_t>(row_ptr, col, leader_in, leader_out, n_rows, ring, 0, 0, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_sum_shards, dim3(1), dim3(kWave), 0, s, ring, 0,
                       reinterpret_cast<unsigned long long *>(changed));
    SW_LAUNCHED();
    return SWARM_OK;
}

}  // extern "C"
