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
//   FRONTIER  an agent can only change in round t+1 if a neighbour changed in round t (its own
//             value already dominates every unchanged neighbour), so after a few dense rounds
//             only the agents MARKED by the previous round's risers gather.  Same leaders, same
//             per-round change counts, same rounds_exec; each agent's row is read O(changes)
//             times instead of O(rounds) times.
//
// One kernel per round, picked by the host per round from the last change counts it has read
// (every batch of rounds):
//   k_elect_dense<MARK=false>  the first dense_rounds-1 rounds (nearly every agent changes)
//   k_elect_dense<MARK=true>   the last dense round: also marks the risers' neighbourhoods
//   k_sparse_block             2 048 resident workgroups; each loads the stamp words of all its
//                              2048-stamp chunks at once, lists their marked agents in LDS and
//                              gathers them, 4 lanes per marked agent with interleaved edges.
//                              Stamps are dealt in 32-agent blocks over the chunks while rounds
//                              are busy (balance), in agent order in the tail (stamp_slot)
// Marks are plain byte stores, no atomics: stamp act[v] = stamp_of(t+1) (1..255, never 0, so an
// unmarked byte never matches), double-buffered by round parity and consumed (zeroed) by the
// sparse round that reads them.  Leaders alternate by
// parity: round t reads L[(t-1)&1] and writes L[t&1], which still holds the state after t-2; it
// differs from the state after t-1 only on round t-1's risers, all marked (self-mark), so all
// rewrite their entry.
//
// Counters: every per-round count (changes, marked agents, edges, ghost rises) is a 64-way
// sharded 64-bit counter on its own 128-byte line, added once per workgroup: one contended
// counter per round costs ~12 ns per arrival (MI355X_MICROARCH.md, 'fanin').  The shards live
// in a ring of kRing rounds; one workgroup of round t (block 0 of a dense round, the last block
// of a sparse one) recycles the slots of round t + kRing/2 and publishes the total changes of
// round t-1 (tot[]), which sparse rounds use as their guard.
//
// Measured and rejected: a push variant (risers atomicMax their value into the
// neighbours: scattered device-scope atomics run at ~20 G/s), dense and sparse paths fused in
// one kernel (register pressure: 6 instead of 8 waves per SIMD, +10 %), per-wave chunks with no
// workgroup barrier (+6..30 %), 1 / 2 / 8 / 16 lanes per marked agent (+28..65 %), contiguous
// instead of interleaved edge slices per lane (+14 %), paired / edge-flat / wave-flat / run-unit
// gathers (+16..66 %).
#include <algorithm>
#include <type_traits>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "swarm_common.h"

namespace swarm {
namespace {

constexpr int kShards = 64;
constexpr int kShardStride = 16;                    // u64 per shard: one 128-B line each
constexpr int kRing = 512;                          // rounds of counter slots
constexpr int kRoundWords = kShards * kShardStride; // u64 per round per counter
constexpr int kCounters = kElectCounters;
constexpr int C_CHG = 0, C_ACT = 1, C_EDGE = 2, C_GHOST = 3;
constexpr int kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ unsigned long long *slot(unsigned long long *ring, int t, int counter, int shard) {
    return ring + (size_t(t % kRing) * kCounters + counter) * kRoundWords + size_t(shard) * kShardStride;
}

// Sum of the 64 change shards of round t (every thread of the block gets it).
__device__ __forceinline__ unsigned long long round_total(unsigned long long *ring, int t,
                                                          unsigned long long *s_bcast) {
    if (threadIdx.x < kWave) {
        unsigned long long v = *slot(ring, t, C_CHG, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) *s_bcast = v;
    }
    __syncthreads();
    return *s_bcast;
}

// Block 0 of round t: publish the total changes of round t-1 and recycle round t + kRing/2.
__device__ __forceinline__ void bookkeeping(unsigned long long *ring, unsigned long long *tot, int t) {
    if (blockIdx.x != 0) return;
    if (tot && t > 1 && threadIdx.x < kWave) {
        unsigned long long v = *slot(ring, t - 1, C_CHG, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) tot[(t - 1) % kRing] = v;
    }
    for (int i = threadIdx.x; i < kCounters * kShards; i += kBlock)
        *slot(ring, t + kRing / 2, i / kShards, i % kShards) = 0;
}

// The same, done by the LAST workgroup of a sparse round: grid-stride over M chunks gives the last
// workgroups one chunk fewer than the first ones, so the dependent load is off the round's
// critical path.  (Done synchronously: a shard sum held in registers through the gather was
// spilled to scratch by every thread of every workgroup -- 4 MB written per round.)
__device__ __forceinline__ void bookkeeping_last(unsigned long long *ring, unsigned long long *tot, int t) {
    if (blockIdx.x != gridDim.x - 1) return;
    if (tot && t > 1 && threadIdx.x < kWave) {
        unsigned long long v = *slot(ring, t - 1, C_CHG, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) tot[(t - 1) % kRing] = v;
    }
    for (int i = threadIdx.x; i < kCounters * kShards; i += kBlock)
        *slot(ring, t + kRing / 2, i / kShards, i % kShards) = 0;
}

#ifdef SWARM_PHASES  // debug build only: per-wave phase timestamps of the last launched round
__device__ unsigned long long g_phase[8192 * 8];
#define PHASE(k)                                                                         \
    do {                                                                                 \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                      \
        const int64_t wg_ = int64_t(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);   \
        if ((threadIdx.x & 63) == 0 && wg_ < 8192) g_phase[wg_ * 8 + (k)] = wall_clock64(); \
    } while (0)
#else
#define PHASE(k) do {} while (0)
#endif

// Stamp byte of round t: 1, 2, ..., 255, 1, ...  (0 is "unmarked"; a round whose stamp were 0
// would gather every agent).
__host__ __device__ __forceinline__ uint8_t stamp_of(int t) { return uint8_t(1 + (t - 1) % 255); }

// 4-bit mask of the bytes of w equal to the byte replicated in b4 (exact, no carry leakage).
__device__ __forceinline__ unsigned bytes_eq4(unsigned w, unsigned b4) {
    const unsigned x = w ^ b4;
    const unsigned z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// ------------------------------------------------------------------ stamp layout
// Stamps are not stored in agent order.  Agents are grouped in blocks of B = 2^bshift consecutive
// storage indices; block b lives in chunk b mod M, at block position b div M, so a chunk (the
// sparse round's unit of work: C = 2^cshift = 2 048 or 512 stamps, one workgroup pass) holds
// blocks spread evenly over the whole swarm.  A wave front that lies along a cell row marks a long
// run of consecutive agents; in agent order that run lands in one or two chunks (hundreds of
// marked agents, the slowest workgroup of the round), here it is dealt out B agents per chunk.
// Within a block the agents stay consecutive: their rows are one contiguous slice of col.  B = C
// is the identity (agent order).
struct StampMap {
    uint32_t M;   // chunks
    float invM;   // 1 / M: the block's chunk and position from one float product, corrected by +-1
    int cshift;   // log2(C)
    int bshift;   // log2(B)
};

// 32-bit on the device (register pressure: the sparse kernel runs at the 64-VGPR cap of 8 waves
// per SIMD).  b < 2^28 and the quotient is below C / B <= 256, so the float product is within
// 2^-14 of b / M: one correction step makes it exact.
__device__ __forceinline__ uint32_t stamp_slot(const StampMap &m, int32_t v) {
    const uint32_t b = uint32_t(v) >> m.bshift;
    uint32_t q = __float2uint_rz(__uint2float_rz(b) * m.invM);
    int32_t r = int32_t(b - q * m.M);
    if (r < 0) {
        --q;
        r += int32_t(m.M);
    } else if (r >= int32_t(m.M)) {
        ++q;
        r -= int32_t(m.M);
    }
    return (uint32_t(r) << m.cshift) + (q << m.bshift) + (uint32_t(v) & ((1u << m.bshift) - 1));
}

// storage index of in-chunk stamp position j of chunk k (32-bit: every slot's agent is < 2^31, and
// a 64-bit per-lane product hoisted out of the scan loop is a VGPR pair the sparse kernel spills)
__device__ __forceinline__ int64_t stamp_agent(const StampMap &m, int64_t k, int j) {
    return int64_t(((uint32_t(j >> m.bshift) * m.M + uint32_t(k)) << m.bshift) | uint32_t(j & ((1 << m.bshift) - 1)));
}

// 4-byte element idx of base with a 32-bit byte offset (idx < 2^30): the load takes the uniform
// base in SGPRs and one offset VGPR, where a 64-bit index costs an address pair per load in flight
// (the sparse kernel runs at the 64-VGPR cap).  Int64 offsets (graphs >= 2^30 edges or agents) use
// plain indexing.
template <typename T, typename I>
__device__ __forceinline__ T ld4(const T *__restrict__ base, I idx) {
    if constexpr (sizeof(I) == 4 && sizeof(T) == 4)
        return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t(idx) << 2));
    else
        return base[idx];
}
template <typename T, typename I>
__device__ __forceinline__ void st4(T *__restrict__ base, I idx, T v) {
    if constexpr (sizeof(I) == 4 && sizeof(T) == 4)
        *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (uint32_t(idx) << 2)) = v;
    else
        base[idx] = v;
}

// Neighbour columns.  Col32: the CSR's int32 storage indices.  Col16: the same graph with each column
// stored as a 16-bit delta from its row's 64-agent task base (v & ~63): col16[k] = col[k] - (v & ~63)
// (swarm_graph_compact; only when every delta fits).  In the spatial storage order a neighbour lies
// within about one cell row of its agent (7 000 agents at 10M), so the deltas fit, and every column
// read -- the dense sweep streams all of them -- moves half the bytes.  The base is known wherever a
// column is read: the dense wave's task, the sparse lane's agent.
struct Col32 {
    const int32_t *p;
    template <typename I>
    __device__ __forceinline__ int32_t at(I k, int32_t) const { return p[k]; }
    // 32-bit byte offsets (k < 2^30: the int32-CSR elections)
    template <typename I>
    __device__ __forceinline__ int32_t at32(I k, int32_t) const { return ld4(p, k); }
};
struct Col16 {
    const int16_t *p;
    template <typename I>
    __device__ __forceinline__ int32_t at(I k, int32_t base) const { return base + int32_t(p[k]); }
    // 32-bit byte offsets for the int32-CSR elections; plain indexing for int64 offsets
    template <typename I>
    __device__ __forceinline__ int32_t at32(I k, int32_t base) const {
        if constexpr (sizeof(I) == 4)
            return base + int32_t(*reinterpret_cast<const int16_t *>(reinterpret_cast<const char *>(p) + (uint32_t(k) << 1)));
        else
            return base + int32_t(p[k]);
    }
};

// Col16 whose base is 16-byte aligned: the dense rounds read it 8 columns per 16-byte load
struct Col16A : Col16 {};

// Col16 with escapes (swarm_graph_compact_escaped): a neighbour more than 32767 storage slots from its
// row's base -- in a shard graph, a ghost stored in another peer's block -- is the sentinel kEsc and is
// read from the int32 columns instead.  The sparse gather checks the wave once per batch of columns, so
// a batch with no escaped column costs one compare per column.
constexpr int kEsc = -32768;
struct Col16E {
    const int16_t *p;
    const int32_t *c;  // the int32 columns of the same graph
    template <typename I>
    __device__ __forceinline__ int32_t at(I k, int32_t base) const {
        const int32_t d = p[k];
        return d == kEsc ? c[k] : base + d;
    }
    // the sparse gather's form: base + delta without the escape test; the caller fixes escaped columns
    // for a whole batch at once (gather_listed: one wave vote per batch, a taken branch only when a
    // column of the batch is escaped)
    template <typename I>
    __device__ __forceinline__ int32_t raw32(I k, int32_t base, bool &esc) const {
        const int32_t d = *reinterpret_cast<const int16_t *>(reinterpret_cast<const char *>(p) + (uint32_t(k) << 1));
        esc = d == kEsc;
        return base + d;
    }
};


constexpr int kKm = 8;  // marking re-walks: col loads in flight per lane

// Mark col[k] for k = k0, k0 + step, ... < e with kKm loads in flight per batch.
template <typename Off, typename CT>
__device__ __forceinline__ void mark_row(uint8_t *aw, const StampMap &sm, CT cols, int32_t base, Off k0, Off e,
                                         Off step, uint8_t s) {
    for (Off k = k0; k < e; k += step * kKm) {
        int c[kKm];
#pragma unroll
        for (int j = 0; j < kKm; ++j) {
            const Off kk = k + step * j;
            c[j] = cols.at(kk < e ? kk : e - 1, base);
        }
#pragma unroll
        for (int j = 0; j < kKm; ++j)
            if (k + step * j < e) aw[stamp_slot(sm, c[j])] = s;
    }
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
// MARK: also stamp every riser and its neighbours for round t+1 (act_w = t+1), so that round
// t+1 can run sparse.
// DIR: directed graph -- a riser marks the agents that HEAR it (hrp/hcol, the transpose of
// rp/col), not the agents it hears.
template <typename Off, bool MARK, bool DIR = false, bool FLAT = false, typename CT = Col32>
__global__ __launch_bounds__(kBlock) void k_elect_dense(
    const Off *__restrict__ rp, CT cols, const int32_t *__restrict__ lin,
    int32_t *__restrict__ lout, int64_t n, int64_t c_lo, int64_t n_count, unsigned long long *__restrict__ ring,
    unsigned long long *__restrict__ tot, uint8_t *__restrict__ act_w, StampMap sm, int t, int guard,
    const Off *__restrict__ hrp = nullptr, const int32_t *__restrict__ hcol = nullptr) {
    // VEC: 16-bit columns read 8 per lane with one 16-byte load (FLAT windows start 8-aligned)
    constexpr bool VEC = FLAT && std::is_same_v<CT, Col16A>;
    __shared__ __attribute__((aligned(16))) int s_col[kWavesPerBlock][kWin];
    __shared__ unsigned long long s_bc, s_cnt[kWavesPerBlock];
    if (guard && t > 1 && round_total(ring, t - 1, &s_bc) == 0) return;  // converged: no-op
    if (guard || tot) bookkeeping(ring, tot, t);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint8_t sw = stamp_of(t + 1);
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
    const Off e_all = VEC ? rp[n] : Off(0);  // VEC: a 16-byte load must end inside the column array
    for (; task < ntask; task += stride) {
        const int64_t v = task * 64 + lane;
        const int32_t tbase = int32_t(task * 64);  // Col16 deltas are relative to the task's first agent
        const bool valid = v < n;
        const Off W0 = __shfl(b, 0, 64), W1 = __shfl(e, 63, 64);
        const int own = lin[valid ? v : n - 1];
        Off nb = 0, ne = 0;
        if (task + stride < ntask) bounds(task + stride, nb, ne);  // wave-uniform branch
        int m = INT_MIN;
        for (Off w0 = VEC ? (W0 & ~Off(7)) : W0; w0 < W1; w0 += kWin) {
            const Off wend = (W1 - w0 < kWin) ? W1 : w0 + kWin;
            if constexpr (VEC) {
                // the window's columns 8 per lane (one 16-byte load: an eighth of the column load
                // instructions of the 64-lane form -- the round is bound by the texture unit's cost
                // per instruction), their leaders gathered and stored to LDS 4 per store; slots
                // outside [W0, wend) (the 8-alignment prefix, the next task's edges) read agent tbase
#pragma unroll 1
                for (int h = 0; h < 2; ++h) {
                    const Off kb = w0 + h * (kWin / 2) + lane * 8;
                    int c[8];
                    if (kb + 8 <= e_all) {
                        const int4 q = *reinterpret_cast<const int4 *>(cols.p + kb);
                        const int w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            c[2 * i] = tbase + int32_t(int16_t(w[i] & 0xffff));
                            c[2 * i + 1] = tbase + (w[i] >> 16);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const Off k = kb + i;
                            c[i] = cols.at(k < e_all ? k : e_all - 1, tbase);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const Off k = kb + i;
                        if (!(k >= W0 && k < wend)) c[i] = tbase;
                    }
                    int val[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) val[i] = lin[c[i]];
                    int4 *dst = reinterpret_cast<int4 *>(sc + h * (kWin / 2) + lane * 8);
                    dst[0] = make_int4(val[0], val[1], val[2], val[3]);
                    dst[1] = make_int4(val[4], val[5], val[6], val[7]);
                }
                __builtin_amdgcn_wave_barrier();
                const Off lo = b > w0 ? b : w0, hi = e < wend ? e : wend;
                for (Off k = lo; k < hi; ++k) m = max(m, sc[k - w0]);
            } else if constexpr (FLAT) {
                // flat: the window's columns AND their leaders, 64 consecutive edges per load (the
                // neighbours of ~4 consecutive agents: few cache lines per instruction), leaders
                // into LDS, each lane then maxes its own row from LDS
                constexpr int kH = kWin / 128;  // two halves: 8 columns + 8 leaders in flight per lane
#pragma unroll 1
                for (int h = 0; h < 2; ++h) {
                    int c[kH];
#pragma unroll
                    for (int j = 0; j < kH; ++j) {
                        const Off k = w0 + (h * kH + j) * 64 + lane;
                        c[j] = cols.at(k < wend ? k : wend - 1, tbase);
                    }
#pragma unroll
                    for (int j = 0; j < kH; ++j) sc[(h * kH + j) * 64 + lane] = lin[c[j]];
                }
                __builtin_amdgcn_wave_barrier();
                const Off lo = b > w0 ? b : w0, hi = e < wend ? e : wend;
                for (Off k = lo; k < hi; ++k) m = max(m, sc[k - w0]);
            } else {
#pragma unroll
                for (int j = 0; j < kWin / 64; ++j) {
                    const Off k = w0 + j * 64 + lane;
                    sc[j * 64 + lane] = cols.at(k < wend ? k : wend - 1, tbase);
                }
                __builtin_amdgcn_wave_barrier();
                const Off lo = b > w0 ? b : w0, hi = e < wend ? e : wend;
                m = row_max_from_lds<Off>(sc, w0, lo, hi, lin, m);
            }
            __builtin_amdgcn_wave_barrier();
        }
        const bool up = valid && m > own;
        if (valid) lout[v] = up ? m : own;
        mine += __popcll(__ballot(up && v >= c_lo && v < n_count));  // sharded: ghost rows step, owners count
        if (MARK && up) {
            act_w[stamp_slot(sm, v)] = sw;
            if (DIR)
                mark_row<Off>(act_w, sm, Col32{hcol}, 0, hrp[v], hrp[v + 1], Off(1), sw);
            else if (!FLAT)
                mark_row<Off>(act_w, sm, cols, tbase, b, e, Off(1), sw);
        }
        if constexpr (MARK && FLAT && !DIR) {
            // risers' neighbours marked by a flat re-walk of the wave's col slice: every lane flags
            // its own row's slots in LDS (1 = riser), then 64 consecutive columns per load (L2-hot,
            // two cache lines per instruction, where a lane walking its own row touches 64)
            if (__ballot(up)) {
                for (Off w0 = W0; w0 < W1; w0 += kWin) {
                    const Off wend = (W1 - w0 < kWin) ? W1 : w0 + kWin;
                    const Off lo = b > w0 ? b : w0, hi = e < wend ? e : wend;
                    for (Off k = lo; k < hi; ++k) sc[k - w0] = up ? 1 : 0;
                    __builtin_amdgcn_wave_barrier();
                    constexpr int kH = kWin / 128;
#pragma unroll 1
                    for (int h = 0; h < 2; ++h) {
                        int c[kH];
                        bool fl[kH];
#pragma unroll
                        for (int j = 0; j < kH; ++j) {
                            const Off k = w0 + (h * kH + j) * 64 + lane;
                            c[j] = cols.at(k < wend ? k : wend - 1, tbase);
                            fl[j] = k < wend && sc[(h * kH + j) * 64 + lane] != 0;
                        }
#pragma unroll
                        for (int j = 0; j < kH; ++j)
                            if (fl[j]) act_w[stamp_slot(sm, c[j])] = sw;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        b = nb;
        e = ne;
    }
    if (lane == 0) s_cnt[wid] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) s += s_cnt[w];
        if (s) atomicAdd(slot(ring, t, C_CHG, blockIdx.x & (kShards - 1)), s);
    }
}

// ------------------------------------------------------------------ sparse rounds
constexpr int kScan = 8;                 // stamps per thread (one 8-B load)
constexpr int kChunk = kBlock * kScan;   // k_sparse_block: agents per workgroup work unit
constexpr int kG = 4;                    // lanes per marked agent
constexpr int kKs = 8;                   // loads in flight per lane
constexpr int kListCap = 4096;           // marked agents listed in LDS per workgroup (16 KiB)

struct Frontier {
    int32_t *L[2];
    uint8_t *act[2];         // stamps, sm.M << sm.cshift bytes each (stamp_slot layout)
    // sm: the layout this round's stamps were written in (read and consumed); wsm: the layout of
    // the marks it writes for the next round.  Same chunk size and count, so the host may switch
    // the layout at any round boundary (stamp_map).
    unsigned long long *ring, *tot;
    int64_t n_rows, n_all;   // rows stepped (owned + ghosts in sharded runs), all agents
    int64_t c_lo, n_count;   // rows [c_lo, n_count) are owned: only their changes are counted
    StampMap sm, wsm;
    const int16_t *c16;      // Col16 columns of the same graph (swarm_graph_compact), or nullptr
    bool c16_esc;            // c16 holds escapes (swarm_graph_compact_escaped): read as Col16E
};

// Max over the G lanes of an agent's group (G = 4: a quad) through DPP quad permutes -- register
// moves inside the wave, where __shfl_xor would be two LDS round trips (ds_bpermute).
template <int G>
__device__ __forceinline__ int group_max(int m) {
    if constexpr (G == 4) {
        m = max(m, __builtin_amdgcn_update_dpp(m, m, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
        m = max(m, __builtin_amdgcn_update_dpp(m, m, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    } else {
#pragma unroll
        for (int o2 = 1; o2 < G; o2 <<= 1) m = max(m, __shfl_xor(m, o2, 64));
    }
    return m;
}

// Wave sum (full exec): DPP within rows of 16 (quad xor 1, xor 2, half-row mirror, row mirror),
// then the four row sums read into scalars -- no ds_bpermute round trips.
__device__ __forceinline__ int wave_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);  // row_mirror
    return __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) + __builtin_amdgcn_readlane(x, 32) +
           __builtin_amdgcn_readlane(x, 48);
}

// Exclusive prefix over the wave of c (0 <= c < 2^B) and the wave total, from B ballots and
// mbcnt (no LDS round trip: a __shfl_up scan is six ds_bpermute waits).
template <int B>
__device__ __forceinline__ int wave_excl_scan(int c, int &total) {
    int ex = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const unsigned long long m = __ballot((c >> b) & 1);
        ex += int(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u))) << b;
        tot += __popcll(m) << b;
    }
    total = tot;
    return ex;
}

// Gather of the marked agents listed (chunk-relative) in lst[0, total), G lanes per agent,
// `first`/`step` select this wave's share; risers mark themselves and their neighbours.  Lane
// `sub` of an agent takes edges b + sub + G*j (interleaved: one load instruction covers G
// consecutive edges of every agent it serves, so each touches one cache line per agent).
template <typename Off, int G, int K, bool DIR, typename CT>
__device__ __forceinline__ void gather_listed(const Off *__restrict__ rp, CT cols,
                                              const Off *__restrict__ hrp, const int32_t *__restrict__ hcol,
                                              const int32_t *__restrict__ P, int32_t *__restrict__ Q,
                                              uint8_t *__restrict__ aw, const StampMap &sm, uint8_t sw,
                                              const int *lst, int total, int first, int step, int64_t c_lo,
                                              int64_t n_count,
                                              long long &my_chg, int &my_act, int &my_edges) {
    const int lane = threadIdx.x & 63, sub = lane & (G - 1);
    using Ix = Off;  // 32-bit offsets in the int32-CSR instantiation (host: < 2^30 agents and edges)
    if (first >= total) return;
    // software pipeline: a pass's agent, row bounds and own leader are loaded during the previous
    // pass, so a pass's chain is columns -> leaders only
    int32_t nv = lst[first + lane / G < total ? first + lane / G : total - 1];
    Off nb = ld4(rp, Ix(nv)), ne = ld4(rp, Ix(nv + 1));
    int nown = ld4(P, Ix(nv));
    for (int base = first; base < total; base += step) {
        const int i = base + lane / G;
        const bool valid = i < total;
        const int32_t v = nv;
        const Off b = nb, e = ne;
        const int own = nown;
        {  // unconditional (clamped past the end): a load behind a branch is waited for at the join
            const int i2 = base + step + lane / G;
            nv = lst[i2 < total ? i2 : total - 1];
            nb = ld4(rp, Ix(nv));
            ne = ld4(rp, Ix(nv + 1));
            nown = ld4(P, Ix(nv));
        }
        int m = own;
        int c[K];
        for (Off k = b + sub; k < e; k += G * K) {
            if constexpr (std::is_same_v<CT, Col16E>) {
                bool esc[K];
                bool any = false;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    c[j] = cols.raw32((k + G * j < e) ? k + G * j : e - 1, v & ~63, esc[j]);
                    any |= esc[j];
                }
                if (__builtin_expect(__ballot(any) != 0, 0)) {
#pragma unroll
                    for (int j = 0; j < K; ++j)
                        if (esc[j]) c[j] = ld4(cols.c, (k + G * j < e) ? k + G * j : e - 1);
                }
            } else {
#pragma unroll
                for (int j = 0; j < K; ++j) c[j] = cols.at32((k + G * j < e) ? k + G * j : e - 1, v & ~63);
            }
            int val[K];
#pragma unroll
            for (int j = 0; j < K; ++j) val[j] = ld4(P, Ix(c[j]));
#pragma unroll
            for (int j = 0; j < K; ++j) m = max(m, val[j]);
        }
        m = group_max<G>(m);
        const bool up = valid && m > own;
        if (valid && sub == 0) st4(Q, Ix(v), m);
        if (up) {
            if (sub == 0) aw[stamp_slot(sm, v)] = sw;
            if (DIR) {  // the agents that hear v
                mark_row<Off>(aw, sm, Col32{hcol}, 0, hrp[v] + sub, hrp[v + 1], Off(G), sw);
            } else if (e - b <= G * K) {  // one pass: c[] still holds this lane's edges
#pragma unroll
                for (int j = 0; j < K; ++j)
                    if (b + sub + G * j < e) aw[stamp_slot(sm, c[j])] = sw;
            } else {
                mark_row<Off>(aw, sm, cols, v & ~63, b + sub, e, Off(G), sw);
            }
        }
        my_chg += __popcll(__ballot(up && sub == 0 && v >= c_lo && v < n_count));
        if (valid && sub == 0) {
            my_act += 1;
            my_edges += int(e - b);
        }
    }
}

// S stamps per thread as one word: 8 (uint2, 2 048-agent chunks) or 2 (uint16, 512-agent chunks:
// small swarms, whose 2 048-agent chunks would leave most CUs idle).
template <int S> struct StampWord;
template <> struct StampWord<8> { using T = uint2; };
template <> struct StampWord<2> { using T = uint16_t; };

__device__ __forceinline__ unsigned stamp_bits(uint2 w, unsigned stamp4) {
    return bytes_eq4(w.x, stamp4) | (bytes_eq4(w.y, stamp4) << 4);
}
__device__ __forceinline__ unsigned stamp_bits(uint16_t w, unsigned stamp4) {
    return bytes_eq4(unsigned(w), stamp4) & 3u;  // the two zero high bytes never match (stamps >= 1)
}
__device__ __forceinline__ bool any_stamp(uint2 w) { return (w.x | w.y) != 0; }
__device__ __forceinline__ bool any_stamp(uint16_t w) { return w != 0; }

// Marked lanes of S stamps (v0: the word's first agent; its S slots are agents v0 .. v0+S-1).
// Stamps are not consumed here: a stamp left behind holds an older round's value and matches
// only a round 510 rounds later (same parity, same stamp_of), and launch_frontier_round clears
// each parity's buffer every 256 rounds (a bulk memset instead of a store per marked word).
// (A stale match would only cost work: an agent none of whose neighbours changed recomputes its
// own value and counts no change.)
template <int S, typename W>
__device__ __forceinline__ unsigned take_stamps(int64_t v0, int64_t n, W wv, unsigned stamp4) {
    unsigned mask = stamp_bits(wv, stamp4);
    if (v0 + S > n) mask &= (v0 >= n) ? 0u : ((1u << (n - v0)) - 1u);
    return mask;
}

// my_act / my_edges: this lane's marked agents and edges of the round (32-bit per lane: VGPRs are
// at the 8-waves-per-SIMD cap in the sparse kernel)
__device__ __forceinline__ void flush_counts(unsigned long long *ring, int t, long long my_chg, int my_act,
                                             int my_edges, long long (*s_red)[kWavesPerBlock]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    my_act = wave_sum(my_act);
    my_edges = wave_sum(my_edges);
    if (lane == 0) {
        s_red[0][wid] = my_chg;  // wave-uniform (ballot counts)
        s_red[1][wid] = my_act;
        s_red[2][wid] = my_edges;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        long long a = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) a += s_red[threadIdx.x][w];
        if (a) atomicAdd(slot(ring, t, threadIdx.x, blockIdx.x & (kShards - 1)), (unsigned long long)a);
    }
}

// One workgroup per chunk of kBlock * S agents: S stamps per thread, the chunk's marked agents
// compacted in LDS and gathered by the whole workgroup.
template <typename Off, int S = kScan, bool DIR = false, typename CT = Col32, int G = kG, int K = kKs>
__global__ __launch_bounds__(kBlock, sizeof(Off) == 4 ? 8 : 6) void k_sparse_block(
    const Off *__restrict__ rp, CT cols, Frontier f, int t, int guard,
    const Off *__restrict__ hrp = nullptr, const int32_t *__restrict__ hcol = nullptr) {
    using W = typename StampWord<S>::T;
    constexpr int kChunk = kBlock * S;
    __shared__ int s_list[kListCap];
    __shared__ int s_wave[kWavesPerBlock];
    __shared__ long long s_red[3][kWavesPerBlock];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#ifdef SWARM_PHASES  // debug build: per-workgroup start/end clocks, marked agents (sum, max chunk)
    const unsigned long long ph_t0 = wall_clock64();
    long long ph_sum = 0, ph_max = 0;
    unsigned long long ph_stamps = 0, ph_listed = 0, ph_gathered = 0;
#endif
    bookkeeping_last(f.ring, f.tot, t);
    // single-GPU runs: round t-2 changed nothing => round t-1 had no marked agent => neither t.
    // Loaded here, tested only once the first stamp words are in flight (no dependent load in
    // front of the round's own chain).
    const unsigned long long prev2 = (guard && t > 2) ? f.tot[(t - 2) % kRing] : 1ull;
    const int32_t *__restrict__ P = f.L[(t - 1) & 1];
    int32_t *__restrict__ Q = f.L[t & 1];
    uint8_t *ar = f.act[t & 1], *aw = f.act[(t + 1) & 1];
    const unsigned stamp4 = unsigned(stamp_of(t)) * 0x01010101u;
    const uint8_t sw = stamp_of(t + 1);
    const int64_t n = f.n_rows;
    long long my_chg = 0;
    int my_act = 0, my_edges = 0;
    const int64_t nchunks = f.sm.M;  // chunk k: stamp slots [k*kChunk, (k+1)*kChunk)
    const int64_t NG = gridDim.x;
    const int j0 = threadIdx.x * S;  // this thread's S slots: consecutive agents of one block
    // The stamp words of all this workgroup's chunks (grid-stride, up to kPre at a time) are loaded
    // at once, with clamped addresses so that no load waits on a branch; their marked lanes are
    // kept as S bits per chunk.  The marked agents of all those chunks then go into ONE list in
    // LDS, gathered together: a round costs one stamp load latency and one gather chain per
    // workgroup, not one of each per chunk.  (List order is free: every listed agent is
    // independent of the others within a round.)
    constexpr int kPre = 32 / S < 4 ? 32 / S : 4;
    constexpr int kLogS = S == 8 ? 3 : 1;
    int listed = 0;  // workgroup-uniform
    for (int64_t cg = blockIdx.x; cg < nchunks; cg += NG * kPre) {
        W wv[kPre];
#pragma unroll
        for (int p = 0; p < kPre; ++p) {
            // past the end: this thread's own first word again (a shared fallback address would
            // put every workgroup's redundant loads on one L2 channel)
            const int64_t chunk = cg + p * NG < nchunks ? cg + p * NG : cg;
            // chunk base uniform (SGPRs), 32-bit lane offset: no 64-bit per-lane address kept live
            wv[p] = *reinterpret_cast<const W *>(ar + chunk * kChunk + uint32_t(threadIdx.x * sizeof(W)));
        }
        if (prev2 == 0) break;  // converged: nothing is marked
        unsigned masks = 0;
#pragma unroll
        for (int p = 0; p < kPre; ++p) {
            const int64_t chunk = cg + p * NG;
            if (chunk < nchunks)
                masks |= take_stamps<S>(stamp_agent(f.sm, chunk, j0), n, wv[p], stamp4) << (p * S);
        }
#ifdef SWARM_PHASES
        if (!ph_stamps) ph_stamps = wall_clock64() + (masks & 0);
#endif
        // append the group's marked agents, gathering whenever the list fills up
        for (;;) {
            const int cnt = __popc(masks);  // <= kPre * S <= 32
            int wtot;
            const int excl = wave_excl_scan<6>(cnt, wtot);
            if (lane == 0) s_wave[wid] = wtot;
            __syncthreads();
            int off = 0, total = 0;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) {
                off += (w < wid) ? s_wave[w] : 0;
                total += s_wave[w];
            }
            __syncthreads();  // s_wave read by all
            if (total == 0) break;
#ifdef SWARM_PHASES
            ph_sum += total;
            ph_max = total > ph_max ? total : ph_max;
#endif
            int pos = listed + off + excl;
            while (masks && pos < kListCap) {
                const int bit = __ffs(masks) - 1;
                masks &= masks - 1;
                s_list[pos++] = int(stamp_agent(f.sm, cg + (bit >> kLogS) * NG, j0)) + (bit & (S - 1));
            }
            listed = listed + total < kListCap ? listed + total : kListCap;
            __syncthreads();  // list entries visible
            if (listed < kListCap) break;  // everything fitted
            gather_listed<Off, G, K, DIR>(rp, cols, hrp, hcol, P, Q, aw, f.wsm, sw, s_list, listed, wid * (64 / G),
                                          kBlock / G, f.c_lo, f.n_count, my_chg, my_act, my_edges);
            listed = 0;
            __syncthreads();  // the list is reused
        }
    }
#ifdef SWARM_PHASES
    ph_listed = wall_clock64();
#endif
    if (listed > 0)
        gather_listed<Off, G, K, DIR>(rp, cols, hrp, hcol, P, Q, aw, f.wsm, sw, s_list, listed, wid * (64 / G),
                                      kBlock / G, f.c_lo, f.n_count, my_chg, my_act, my_edges);
#ifdef SWARM_PHASES
    ph_gathered = wall_clock64() + (my_chg & 0);
#endif
    flush_counts(f.ring, t, my_chg, my_act, my_edges, s_red);
#ifdef SWARM_PHASES
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_phase[blockIdx.x * 8 + 0] = ph_t0;
        g_phase[blockIdx.x * 8 + 1] = wall_clock64();
        g_phase[blockIdx.x * 8 + 2] = (unsigned long long)ph_sum;
        g_phase[blockIdx.x * 8 + 3] = (unsigned long long)ph_max;
        g_phase[blockIdx.x * 8 + 4] = ph_stamps;
        g_phase[blockIdx.x * 8 + 5] = ph_listed;
        g_phase[blockIdx.x * 8 + 6] = ph_gathered;
    }
#endif
}

// Sharded runs: halo values for ghosts [b_lo, b_lo + n_lo) and [b_hi, b_hi + n_hi) after round
// t.  A ghost whose leader rose is written to BOTH leader buffers (ghosts are never gathered)
// and its local neighbours are marked for round t+1 (ghost rows of the local CSR list them).
// Rises are counted in C_GHOST; the owner counts them as changes.
template <typename Off>
__global__ __launch_bounds__(kBlock) void k_frontier_ghosts(const Off *__restrict__ rp, const int32_t *__restrict__ col,
                                                            Frontier f, int64_t b_lo, int64_t n_lo,
                                                            const int32_t *__restrict__ in_lo, int64_t b_hi,
                                                            int64_t n_hi, const int32_t *__restrict__ in_hi, int t) {
    constexpr int G = 8;
    const uint8_t sw = stamp_of(t + 1);
    uint8_t *aw = f.act[(t + 1) & 1];
    const int32_t *Lcur = f.L[t & 1];
    const int sub = threadIdx.x & (G - 1);
    const int64_t total = n_lo + n_hi;
    long long rises = 0;
    for (int64_t base = int64_t(blockIdx.x) * (kBlock / G); base < total; base += int64_t(gridDim.x) * (kBlock / G)) {
        const int64_t i = base + threadIdx.x / G;
        if (i < total) {
            const int64_t g = i < n_lo ? b_lo + i : b_hi + (i - n_lo);
            const int nv = i < n_lo ? in_lo[i] : in_hi[i - n_lo];
            if (nv > Lcur[g]) {
                if (sub == 0) {
                    f.L[0][g] = nv;
                    f.L[1][g] = nv;
                    ++rises;
                }
                for (Off k = rp[g] + sub; k < rp[g + 1]; k += G) {
                    const int32_t c = col[k];
                    if (c < f.n_rows) aw[stamp_slot(f.wsm, c)] = sw;
                }
            }
        }
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) rises += __shfl_xor(rises, o2, 64);
    if ((threadIdx.x & 63) == 0 && rises)
        atomicAdd(slot(f.ring, t, C_GHOST, blockIdx.x & (kShards - 1)), (unsigned long long)rises);
}

// ------------------------------------------------------------------ one-workgroup tail (opt-in)
// SWARM_TAIL_WG=cap (a bounded experiment): once the marked set of the next round fits
// `cap`, ONE 1 024-thread workgroup runs the remaining rounds in one launch, the marked list and the
// next round's dedupe in LDS, rounds separated by __syncthreads only (one CU: no grid barrier, no
// cross-XCD hand-off).  Round t as k_sparse_block's: the listed agents gather their rows from
// L[(t-1)&1] and write L[t&1] (4 lanes per agent), risers are listed; the next round's list is the
// risers and their neighbours, deduplicated by an LDS hash set.  It exits at the first zero-change
// round, at t_end, or when the next list outgrows LDS: then the risers' neighbourhoods are written as
// stamps for round t+1 (agent-order layout f.wsm) and the frontier rounds take over.  Per-round
// counters go to the counter ring as the sparse rounds' (C_CHG / C_ACT / C_EDGE, tot[], recycling).
constexpr int kTailThreads = 1024;
constexpr int kTailCap = 2048;   // list capacity (agents per round)
constexpr int kTailHash = 8192;  // LDS hash-set slots
constexpr int kTailProbe = 64;   // linear probes before the set counts as full
enum TailReason : unsigned long long { TAIL_DONE = 1, TAIL_HANDBACK = 2, TAIL_NOT_STARTED = 3 };

// Stamp marks of the round after `t` for risers ris[0, nr) and their neighbours (hand-back).
template <typename CT>
__device__ void tail_handback(const int32_t *__restrict__ rp, CT cols, const Frontier &f, const int *ris, int nr,
                              int t) {
    uint8_t *aw = f.act[(t + 1) & 1];
    const uint8_t sw = stamp_of(t + 1);
    for (int r = threadIdx.x; r < nr; r += kTailThreads) {
        const int32_t v = ris[r];
        aw[stamp_slot(f.wsm, v)] = sw;
        for (int32_t k = rp[v]; k < rp[v + 1]; ++k) aw[stamp_slot(f.wsm, cols.at(k, v & ~63))] = sw;
    }
}

// The marked agents of round t0 (stamps act[t0 & 1] in layout f.sm: S stamps per thread, 256 S-stamp
// chunks -- k_sparse_block's reading) into glist[0, cap) and *gcount (the count keeps counting past cap:
// the tail then does not start).
template <int S>
__global__ __launch_bounds__(kBlock) void k_tail_collect(Frontier f, int t0, int32_t *__restrict__ glist,
                                                         unsigned *__restrict__ gcount, int cap) {
    using W = typename StampWord<S>::T;
    constexpr int kC = kBlock * S;
    const uint8_t *ar = f.act[t0 & 1];
    const unsigned stamp4 = unsigned(stamp_of(t0)) * 0x01010101u;
    const int64_t nchunks = f.sm.M;
    const int j0 = threadIdx.x * S;
    for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        const W w = *reinterpret_cast<const W *>(ar + chunk * kC + uint32_t(threadIdx.x * sizeof(W)));
        unsigned mask = take_stamps<S>(stamp_agent(f.sm, chunk, j0), f.n_rows, w, stamp4);
        const int cnt = __popc(mask);
        int wtot;
        const int ex = wave_excl_scan<4>(cnt, wtot);
        unsigned base = 0;
        if ((threadIdx.x & 63) == 0 && wtot) base = atomicAdd(gcount, unsigned(wtot));
        base = __shfl(base, 0, 64);
        int pos = int(base) + ex;
        while (mask) {
            const int bit = __ffs(mask) - 1;
            mask &= mask - 1;
            if (pos < cap) glist[pos] = int32_t(stamp_agent(f.sm, chunk, j0)) + bit;
            ++pos;
        }
    }
}

// Both stamp buffers zeroed when the tail will start (*gcount <= cap): it writes fresh marks at its exit.
__global__ __launch_bounds__(kBlock) void k_tail_clear(uint4 *__restrict__ a, int64_t n16,
                                                       const unsigned *__restrict__ gcount, int cap) {
    if (*gcount > unsigned(cap)) return;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n16; i += int64_t(gridDim.x) * kBlock)
        a[i] = make_uint4(0, 0, 0, 0);
}

// out[0] last round run, out[1] reason, out[2] rounds run, out[3] done flag (the host's wait word);
// clk (optional, debug): per round the wall clock at its start and its marked count.
template <typename CT>
__global__ __launch_bounds__(kTailThreads) void k_tail_wg(const int32_t *__restrict__ rp, CT cols, Frontier f,
                                                          const int32_t *__restrict__ glist,
                                                          const unsigned *__restrict__ gcount, int t0, int t_end,
                                                          int cap, unsigned long long *out,
                                                          unsigned long long ep, unsigned long long *clk) {
    constexpr int G = 4, K = 4;
    __shared__ int s_list[2][kTailCap];
    __shared__ int s_ris[kTailCap];
    __shared__ int s_hash[kTailHash];
    __shared__ int s_n[2], s_nris, s_over;
    __shared__ unsigned long long s_edges;
    const int tid = threadIdx.x, sub = tid & (G - 1);
    const unsigned m0 = *gcount;
    auto finish = [&](unsigned long long last, unsigned long long why, unsigned long long runs) {
        if (tid == 0) {
            out[0] = last;
            out[1] = why;
            out[2] = runs;
            __threadfence_system();
            __hip_atomic_store(&out[3], ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };
    if (m0 == 0 || m0 > unsigned(cap) || cap > kTailCap) {
        finish(t0 - 1, TAIL_NOT_STARTED, 0);
        return;
    }
    for (int q = tid; q < int(m0); q += kTailThreads) s_list[0][q] = glist[q];
    for (int q = tid; q < kTailHash; q += kTailThreads) s_hash[q] = -1;
    if (tid < kWave && t0 > 1) {  // round t0's bookkeeping: publish round t0-1's total (the sparse guard's)
        unsigned long long v = *slot(f.ring, t0 - 1, C_CHG, tid);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (tid == 0) f.tot[(t0 - 1) % kRing] = v;
    }
    if (tid == 0) {
        s_n[0] = int(m0);
        s_n[1] = 0;
        s_nris = 0;
        s_over = 0;
        s_edges = 0;
    }
    __syncthreads();
    int cur = 0;
    for (int t = t0;; ++t) {
        const int m = s_n[cur];
        if (clk && tid == 0) {
            clk[2 * (t - t0)] = wall_clock64();
            clk[2 * (t - t0) + 1] = unsigned(m);
        }
        const int32_t *__restrict__ P = f.L[(t - 1) & 1];
        int32_t *__restrict__ Q = f.L[t & 1];
        unsigned my_edges = 0;
        // gather: 4 lanes per listed agent, K columns in flight per lane
        for (int base = 0; base < m; base += kTailThreads / G) {
            const int i = base + tid / G;
            const int32_t v0 = s_list[cur][i < m ? i : m - 1];
            const bool valid = i < m && v0 >= 0 && v0 < f.n_rows;  // (a bad entry is never gathered)
            const int32_t v = valid ? v0 : 0;
            const int32_t b = rp[v], e = rp[v + 1];
            const int own = P[v];
            int mx = own;
            for (int32_t k = b + sub; k < e; k += G * K) {
                int c[K];
#pragma unroll
                for (int j = 0; j < K; ++j) c[j] = cols.at((k + G * j < e) ? k + G * j : e - 1, v & ~63);
                int val[K];
#pragma unroll
                for (int j = 0; j < K; ++j) val[j] = P[c[j]];
#pragma unroll
                for (int j = 0; j < K; ++j) mx = max(mx, val[j]);
            }
            mx = group_max<G>(mx);
            if (valid && sub == 0) {
                Q[v] = mx;
                my_edges += unsigned(e - b);
                if (mx > own) s_ris[atomicAdd(&s_nris, 1)] = v;
            }
        }
        const int wsum = wave_sum(int(my_edges));
        if ((tid & 63) == 0 && wsum) atomicAdd(&s_edges, (unsigned long long)wsum);
        __syncthreads();
        const int nr = s_nris;
        if (tid == 0) {  // the round's counters, as a sparse round leaves them (shard 0 of each)
            *slot(f.ring, t, C_CHG, 0) = (unsigned long long)nr;
            *slot(f.ring, t, C_ACT, 0) = (unsigned long long)m;
            *slot(f.ring, t, C_EDGE, 0) = s_edges;
            f.tot[t % kRing] = (unsigned long long)nr;
        }
        for (int q = tid; q < kCounters * kShards; q += kTailThreads)  // recycle round t + kRing/2's slots
            *slot(f.ring, t + kRing / 2, q / kShards, q % kShards) = 0;
        if (nr == 0) {
            finish(t, TAIL_DONE, t - t0 + 1);
            return;
        }
        if (t >= t_end) {
            tail_handback(rp, cols, f, s_ris, nr, t);
            finish(t, TAIL_HANDBACK, t - t0 + 1);
            return;
        }
        // the next list: the risers and their neighbours, each once (LDS hash set)
        const int nxt = cur ^ 1;
        auto insert = [&](int32_t key) {
            uint32_t h = (uint32_t(key) * 2654435761u) & (kTailHash - 1);
            for (int p = 0; p < kTailProbe; ++p) {
                const int old = atomicCAS(&s_hash[h], -1, key);
                if (old == -1) {
                    const int idx = atomicAdd(&s_n[nxt], 1);
                    if (idx < cap)
                        s_list[nxt][idx] = key;
                    else
                        s_over = 1;
                    return;
                }
                if (old == key) return;
                h = (h + 1) & (kTailHash - 1);
            }
            s_over = 1;
        };
        for (int r = tid / G; r < nr; r += kTailThreads / G) {
            const int32_t v = s_ris[r];
            if (sub == 0) insert(v);
            for (int32_t k = rp[v] + sub; k < rp[v + 1]; k += G) insert(cols.at(k, v & ~63));
        }
        __syncthreads();
        if (s_over) {
            tail_handback(rp, cols, f, s_ris, nr, t);
            finish(t, TAIL_HANDBACK, t - t0 + 1);
            return;
        }
        // reset for the next round (8 slots of the set per thread)
        for (int q = tid; q < kTailHash; q += kTailThreads) s_hash[q] = -1;
        if (tid == 0) {
            s_n[cur] = 0;
            s_nris = 0;
            s_edges = 0;
        }
        cur = nxt;
        __syncthreads();
    }
}

// Col16 copy of an int32 CSR: col16[k] = col[k] - (v & ~63) for every edge k of row v; *bad is set
// when a delta does not fit 16 bits (the caller then keeps the int32 columns).
// Deltas fit in [-32767, 32767]: -32768 is kEsc.  ESC: an out-of-range delta is stored as kEsc and
// counted in *bad (unsigned long long); otherwise *bad (int) is set and the caller keeps the int32 columns.
template <bool ESC>
__global__ __launch_bounds__(kBlock) void k_build_col16(const int32_t *__restrict__ rp, const int32_t *__restrict__ col,
                                                        int64_t n, int16_t *__restrict__ col16, void *__restrict__ bad) {
    int out = 0;
    for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < n; v += int64_t(gridDim.x) * kBlock) {
        const int32_t base = int32_t(v) & ~63;
        for (int32_t k = rp[v]; k < rp[v + 1]; ++k) {
            const int32_t d = col[k] - base;
            const bool fits = d >= -32767 && d <= 32767;
            out += fits ? 0 : 1;
            col16[k] = int16_t(fits ? d : kEsc);
        }
    }
    if constexpr (ESC) {
        if (out) atomicAdd(static_cast<unsigned long long *>(bad), (unsigned long long)out);
    } else {
        if (__ballot(out) && (threadIdx.x & 63) == 0) atomicOr(static_cast<int *>(bad), 1);
    }
}

// Check of a 16-bit column copy before any election reads it (swarm_elect_compact*, the frontier
// stepper): every column of row v must name a storage index in [0, n_idx).  A wave takes a task of 64
// rows -- one delta base (v & ~63) and one contiguous edge slice -- and reads it 8 columns per lane per
// pass.  ESC = false: the sentinel kEsc is an error (swarm_graph_compact_escaped's columns, which the
// plain Col16 readers would decode as a delta 32768 below the base); ESC = true: an escaped column's
// int32 entry is checked instead.  *bad |= 1 (an escape where none may be) or 2 (out of range).
template <typename Off, bool ESC>
__global__ __launch_bounds__(kBlock) void k_check_col16(const Off *__restrict__ rp, const int16_t *__restrict__ c16,
                                                        const int32_t *__restrict__ col, int64_t n_rows, int64_t n_idx,
                                                        unsigned *__restrict__ bad) {
    constexpr int kU = 8;
    const int lane = threadIdx.x & 63;
    const int64_t ntask = (n_rows + 63) / 64;
    unsigned out = 0;
    for (int64_t task = int64_t(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6); task < ntask;
         task += int64_t(gridDim.x) * kWavesPerBlock) {
        const int64_t base = task * 64;
        const Off b = rp[base], e = rp[base + 64 < n_rows ? base + 64 : n_rows];
        for (Off k0 = b; k0 < e; k0 += 64 * kU) {
            int32_t d[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const Off k = k0 + j * 64 + lane;
                d[j] = k < e ? int32_t(c16[k]) : 0;
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const Off k = k0 + j * 64 + lane;
                if (k >= e) continue;
                if (d[j] == kEsc) {
                    if constexpr (ESC) {
                        const int32_t c = col[k];
                        out |= (c < 0 || c >= n_idx) ? 2u : 0u;
                    } else {
                        out |= 1u;
                    }
                } else {
                    const int64_t c = base + d[j];
                    out |= (c < 0 || c >= n_idx) ? 2u : 0u;
                }
            }
        }
    }
    // one atomic per wave that found something
    const unsigned long long any = __ballot(out != 0);
    if (any) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) out |= __shfl_xor(out, off, 64);
        if (lane == 0) atomicOr(bad, out);
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
    unsigned long long v = *slot(ring, t, C_CHG, threadIdx.x);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (threadIdx.x == 0) *out += v;
}

// *w = v in mapped host memory, after a system-scope fence: the host's wait word for everything the stream
// wrote there before this kernel (k_batch_totals' per-round totals).
__global__ void k_signal(unsigned long long *w, unsigned long long v) {
    __threadfence_system();
    __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// totals[(r - t0) * kCounters + c] = sum over shards of counter c of round r, one wave per round.
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
    int dense_blocks = 8192;  // grid cap of the dense round kernel (C3 election, same box, 3 runs each:
                              // 8192 23.96-24.07 ms, 2048 24.05-24.16, 4096 24.00-24.13, 16384 23.99-24.12)
    int dense_rounds = 9;     // frontier: rounds 1..dense_rounds run dense (the last one marks)
    int sparse_blocks = 2048; // grid cap of k_sparse_block (8 resident workgroups per CU)
    int small_chunks = 512;   // fewer 2048-agent chunks than this: 512-agent chunks instead
    int stamp_bshift = 5;     // log2 of the stamp layout's block (stamp_slot)
    int dense_flat = 1;       // dense rounds gather leaders 64 consecutive edges per load (FLAT)
    int dense_vec = 1;        // FLAT with 16-bit columns: 8 columns per lane per 16-byte load
    int use_c16 = 1;          // swarm_elect_compact reads the 16-bit columns (0: its int32 ones; A/B aid)
    int il_min_changes = -1;   // interleaved stamp layout while the last read round changed >= this
                               // (-1: 8e-4 x agents, measured best at 100k, 1M and 10M agents)
    int tail_wg = 0;           // > 0: the one-workgroup tail (k_tail_wg) once a round's marks fit this many
    int tail_log = 0;          // SWARM_TAIL_LOG=1: per-round clocks of the tail to stderr (experiment aid)
    int look = 8;              // SWARM_LOOKAHEAD: rounds between a batch's read-back point and its end
    Tuning() {
        look = env_int("SWARM_LOOKAHEAD", 8);
        if (look < 1) look = 1;
        if (look > 64) look = 64;
        tail_wg = env_int("SWARM_TAIL_WG", 0);
        if (tail_wg > kTailCap) tail_wg = kTailCap;
        tail_log = env_int("SWARM_TAIL_LOG", 0);
        il_min_changes = env_int("SWARM_IL_MIN_CHANGES", -1);
        use_c16 = env_int("SWARM_C16", 1);
        dense_flat = env_int("SWARM_DENSE_FLAT", 1);
        dense_vec = env_int("SWARM_DENSE_VEC", 1);
        stamp_bshift = env_int("SWARM_STAMP_BSHIFT", 5);
        dense_blocks = env_int("SWARM_DENSE_BLOCKS", 8192);
        dense_rounds = env_int("SWARM_DENSE_ROUNDS", 9);
        sparse_blocks = env_int("SWARM_SPARSE_BLOCKS", 2048);
        small_chunks = env_int("SWARM_SMALL_CHUNKS", 512);
        if (dense_blocks < 1) dense_blocks = 1;
        if (dense_rounds < 0) dense_rounds = 0;
        if (sparse_blocks < 1) sparse_blocks = 1;
    }
};

const Tuning &tuning() {
    static Tuning tu;
    return tu;
}

size_t ring_bytes() { return size_t(kRing) * kCounters * kRoundWords * 8 + size_t(kRing) * 8; }

// Stamp layout of an n_all-agent stepper (stamp_slot): 2 048-stamp chunks, or 512 when a swarm has
// fewer than small_chunks of the large ones (more workgroups for small swarms).
// interleaved: blocks of 2^bshift agents dealt over the chunks (default); otherwise agent order.
StampMap stamp_map(int64_t n_all, bool interleaved = true) {
    const bool small = (n_all + kChunk - 1) / kChunk < tuning().small_chunks;
    StampMap m{};
    m.cshift = small ? 9 : 11;  // kBlock * 2 or kBlock * kScan stamps
    m.bshift = tuning().stamp_bshift < 3 ? 3 : tuning().stamp_bshift;  // a thread's 8 stamps: one block
    if (m.bshift > m.cshift || !interleaved) m.bshift = m.cshift;
    const int64_t per = int64_t(1) << (m.cshift - m.bshift);  // blocks per chunk
    const int64_t nblocks = (n_all + (int64_t(1) << m.bshift) - 1) >> m.bshift;
    m.M = uint32_t(nblocks > 0 ? (nblocks + per - 1) / per : 1);  // = ceil(n_all / C) for every bshift
    m.invM = 1.0f / float(m.M);
    return m;
}

size_t act_bytes(int64_t n_all) {  // one parity: every chunk of the stamp layout
    const StampMap m = stamp_map(n_all);
    return size_t(m.M) << m.cshift;
}

template <typename Off>
int launch_dense_round(const Off *rp, const int32_t *col, const int32_t *lin, int32_t *lout, int64_t n, int64_t c_lo,
                       int64_t n_count,
                       unsigned long long *ring, unsigned long long *tot, uint8_t *act_w, StampMap sm, int t,
                       int guard, hipStream_t s, const Off *hrp = nullptr, const int32_t *hcol = nullptr,
                       const int16_t *c16 = nullptr) {
    const unsigned grid = grid_for((n + 63) / 64, kWavesPerBlock, unsigned(tuning().dense_blocks));
    const Col32 c32{col};
    if (!hrp && sizeof(Off) == 4 && tuning().dense_flat && c16) {
        const Col16 cc{c16};
        Col16A ca;
        ca.p = c16;
        const bool vec = tuning().dense_vec && (reinterpret_cast<uintptr_t>(c16) & 15) == 0;
        if (act_w && vec)
            hipLaunchKernelGGL((k_elect_dense<Off, true, false, true, Col16A>), dim3(grid), dim3(kBlock), 0, s, rp, ca,
                               lin, lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
        else if (vec)
            hipLaunchKernelGGL((k_elect_dense<Off, false, false, true, Col16A>), dim3(grid), dim3(kBlock), 0, s, rp, ca,
                               lin, lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
        else if (act_w)
            hipLaunchKernelGGL((k_elect_dense<Off, true, false, true, Col16>), dim3(grid), dim3(kBlock), 0, s, rp, cc,
                               lin, lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_elect_dense<Off, false, false, true, Col16>), dim3(grid), dim3(kBlock), 0, s, rp, cc,
                               lin, lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
    } else if (!hrp && sizeof(Off) == 4 && tuning().dense_flat) {
        if (act_w)
            hipLaunchKernelGGL((k_elect_dense<Off, true, false, true>), dim3(grid), dim3(kBlock), 0, s, rp, c32, lin,
                               lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_elect_dense<Off, false, false, true>), dim3(grid), dim3(kBlock), 0, s, rp, c32, lin,
                               lout, n, c_lo, n_count, ring, tot, act_w, sm, t, guard, nullptr, nullptr);
    } else if (act_w && hrp)
        hipLaunchKernelGGL((k_elect_dense<Off, true, true>), dim3(grid), dim3(kBlock), 0, s, rp, c32, lin, lout, n,
                           c_lo, n_count, ring, tot, act_w, sm, t, guard, hrp, hcol);
    else if (act_w)
        hipLaunchKernelGGL((k_elect_dense<Off, true>), dim3(grid), dim3(kBlock), 0, s, rp, c32, lin, lout, n, c_lo, n_count, ring,
                           tot, act_w, sm, t, guard, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_elect_dense<Off, false>), dim3(grid), dim3(kBlock), 0, s, rp, c32, lin, lout, n, c_lo, n_count, ring,
                           tot, act_w, sm, t, guard, nullptr, nullptr);
    SW_LAUNCHED();
    return SWARM_OK;
}

// Frontier view of the ctx slots: every one of the n_all agents is stepped (ghost rows too: with a
// halo deeper than one radius they are computed locally between exchanges), the first
// step_rows (owned) are counted.
int frontier_bind(swarm_ctx *ctx, int32_t *L0, int32_t *L1, Frontier *f) {
    if (!ctx_on_current_device(ctx)) return SWARM_ERR_ARG;
    SW_ARG(ctx->slot[S_ACT] != nullptr && ctx->slot[S_CHANGES] != nullptr, "swarm_frontier_begin first");
    f->n_rows = ctx->step_all;
    f->c_lo = ctx->step_lo;
    f->n_count = ctx->step_lo + ctx->step_rows;
    f->n_all = ctx->step_all;
    f->c16 = ctx->step_c16;
    f->c16_esc = ctx->step_c16_esc;
    f->L[0] = L0;
    f->L[1] = L1;
    uint8_t *a = static_cast<uint8_t *>(ctx->slot[S_ACT]);
    f->act[0] = a;
    f->act[1] = a + act_bytes(f->n_all);
    f->sm = stamp_map(f->n_all, !ctx->step_rd_agent);
    f->wsm = stamp_map(f->n_all, !ctx->step_wr_agent);
    f->ring = static_cast<unsigned long long *>(ctx->slot[S_CHANGES]);
    f->tot = f->ring + size_t(kRing) * kCounters * kRoundWords;
    return SWARM_OK;
}

// Scratch for a frontier run: stamps of both parities, the counter ring (all zeroed).  With no
// dense round, round 1 reads act[1]: every agent marked.
int frontier_alloc(swarm_ctx *ctx, int64_t n_rows, int64_t n_all, int32_t *L0, int32_t *L1, Frontier *f,
                   hipStream_t s) {
    const size_t sb = 2 * act_bytes(n_all);
    void *p;
    SW_ALLOC(p, ctx, S_ACT, sb);
    SW_ALLOC(p, ctx, S_CHANGES, ring_bytes());
    (void)p;
    ctx->step_rows = n_rows;
    ctx->step_all = n_all;
    ctx->step_lo = 0;
    ctx->step_c16 = nullptr;
    ctx->step_c16_esc = false;
    ctx->step_c16_checked = false;
    ctx->step_rd_agent = ctx->step_wr_agent = 0;
    int rc = frontier_bind(ctx, L0, L1, f);
    if (rc) return rc;
    SW_HIP(hipMemsetAsync(f->ring, 0, ring_bytes(), s));
    SW_HIP(hipMemsetAsync(f->act[0], 0, sb, s));
    // every slot, padding included: take_stamps drops slots past n_all
    if (tuning().dense_rounds == 0 && n_all) SW_HIP(hipMemsetAsync(f->act[1], 1, sb / 2, s));
    return SWARM_OK;
}

enum RoundKind { RK_DENSE = 0, RK_DENSE_MARK = 1, RK_SPARSE = 2 };

// Kind of frontier round t: the first dense_rounds rounds dense (nearly every agent changes;
// measured best at 9 for 10M agents with the 16-bit columns: 24.15 vs 24.23 ms at 8), the last of
// them marking, then sparse.
RoundKind plan_round(int t) {
    const int R = tuning().dense_rounds;
    if (t < R) return RK_DENSE;
    if (t == R) return RK_DENSE_MARK;
    return RK_SPARSE;
}

// hrp/hcol: the transpose CSR of a directed graph (who hears each agent), or NULL (symmetric).
template <typename Off>
int launch_frontier_round(const Off *rp, const int32_t *col, const Frontier &f, int t, RoundKind k, int guard,
                          hipStream_t s, const Off *hrp = nullptr, const int32_t *hcol = nullptr) {
    if (k == RK_DENSE || k == RK_DENSE_MARK)
        return launch_dense_round<Off>(rp, col, f.L[(t - 1) & 1], f.L[t & 1], f.n_rows, f.c_lo, f.n_count, f.ring,
                                       f.tot,
                                       k == RK_DENSE_MARK ? f.act[(t + 1) & 1] : nullptr, f.wsm, t, guard, s, hrp,
                                       hcol, f.c16_esc ? nullptr : f.c16);  // escapes: dense rounds read int32
    // the buffer this round marks into (parity t+1) was read by round t-1; every 256 rounds, per
    // parity, it is cleared first, so no stamp outlives the 510 rounds after which its value
    // recurs (take_stamps)
    if (t > 2 && ((t - 1) & 255) < 2) SW_HIP(hipMemsetAsync(f.act[(t + 1) & 1], 0, act_bytes(f.n_all), s));
    const bool small = f.sm.cshift == 9;  // small swarm: 512-agent chunks, 4x the workgroups
    const dim3 grid(grid_for(f.sm.M, 1, unsigned(tuning().sparse_blocks)));
    const Col32 c32{col};
    if (hrp && small)
        hipLaunchKernelGGL((k_sparse_block<Off, 2, true>), grid, dim3(kBlock), 0, s, rp, c32, f, t, guard, hrp, hcol);
    else if (hrp)
        hipLaunchKernelGGL((k_sparse_block<Off, kScan, true>), grid, dim3(kBlock), 0, s, rp, c32, f, t, guard, hrp, hcol);
    else if (f.c16 && f.c16_esc && small)
        hipLaunchKernelGGL((k_sparse_block<Off, 2, false, Col16E>), grid, dim3(kBlock), 0, s, rp, Col16E{f.c16, col},
                           f, t, guard, nullptr, nullptr);
    else if (f.c16 && f.c16_esc)
        hipLaunchKernelGGL((k_sparse_block<Off, kScan, false, Col16E>), grid, dim3(kBlock), 0, s, rp,
                           Col16E{f.c16, col}, f, t, guard, nullptr, nullptr);
    else if (f.c16 && small)
        hipLaunchKernelGGL((k_sparse_block<Off, 2, false, Col16>), grid, dim3(kBlock), 0, s, rp, Col16{f.c16}, f, t,
                           guard, nullptr, nullptr);
    else if (f.c16)
        hipLaunchKernelGGL((k_sparse_block<Off, kScan, false, Col16>), grid, dim3(kBlock), 0, s, rp, Col16{f.c16}, f, t,
                           guard, nullptr, nullptr);
    else if (small)
        hipLaunchKernelGGL((k_sparse_block<Off, 2>), grid, dim3(kBlock), 0, s, rp, c32, f, t, guard, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_sparse_block<Off>), grid, dim3(kBlock), 0, s, rp, c32, f, t, guard, nullptr, nullptr);
    SW_LAUNCHED();
    return SWARM_OK;
}

// Algorithmic HBM bytes of one round:
//   dense   12 n + 8 E + 4: row offsets, own leader, leader write, col, gathered leader
//   sparse  n (stamps) + 16 per marked agent (row offsets, own leader, leader write) + 8 per
//           edge (col, neighbour leader); marks (1 B per riser and neighbour) not counted
double round_bytes(bool dense, int64_t n, int64_t e, int64_t active, int64_t edges) {
    if (dense) return 12.0 * n + 8.0 * e + 4.0;
    return double(n) + 16.0 * active + 8.0 * edges;
}

bool esc_registered(const swarm_ctx *ctx, const int16_t *c16) {
    return std::find(ctx->esc_built.begin(), ctx->esc_built.end(), c16) != ctx->esc_built.end();
}

// swarm_graph_compact's records of the buffers it wrote (SWARM_ELECT_TRUST_C16)
void c16_forget(swarm_ctx *ctx, const int16_t *c16) {
    auto &v = ctx->c16_built;
    v.erase(std::remove_if(v.begin(), v.end(), [&](const swarm_ctx::C16Built &b) { return b.c16 == c16; }), v.end());
}

const swarm_ctx::C16Built *c16_record(swarm_ctx *ctx, const int16_t *c16, const void *rp, const int32_t *col,
                                      int64_t n) {
    for (const auto &b : ctx->c16_built)
        if (b.c16 == c16 && b.rp == rp && b.col == col && b.n == n) return &b;
    return nullptr;
}

// Enqueues the column check of rows [0, n_rows) of (rp, c16) into the ctx's verdict word (zeroed
// first) and its copy into *hflag; the caller reads *hflag after its next stream synchronisation.
template <typename Off>
int enqueue_col16_check(swarm_ctx *ctx, const Off *rp, const int16_t *c16, const int32_t *col, bool esc,
                        int64_t n_rows, int64_t n_idx, unsigned *hflag, hipStream_t s) {
    unsigned *d;
    SW_ALLOC(d, ctx, S_CHECK, sizeof(unsigned));
    SW_HIP(hipMemsetAsync(d, 0, sizeof(unsigned), s));
    if (n_rows > 0) {
        const dim3 grid(grid_for((n_rows + 63) / 64, kWavesPerBlock, 4096));
        if (esc)
            hipLaunchKernelGGL((k_check_col16<Off, true>), grid, dim3(kBlock), 0, s, rp, c16, col, n_rows, n_idx, d);
        else
            hipLaunchKernelGGL((k_check_col16<Off, false>), grid, dim3(kBlock), 0, s, rp, c16, col, n_rows, n_idx, d);
        SW_LAUNCHED();
    }
    SW_HIP(hipMemcpyAsync(hflag, d, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    return SWARM_OK;
}

// SWARM_ERR_ARG with the reason for a non-zero check verdict (SWARM_OK for 0).
int col16_verdict(unsigned hflag, const char *who) {
    if (hflag & 1u) {
        set_error("invalid argument: %s: the 16-bit columns hold escapes (swarm_graph_compact_escaped's): "
                  "pass them through swarm_frontier_set_compact_escaped / swarm_shard.col16_escaped, or build "
                  "them with swarm_graph_compact", who);
        return SWARM_ERR_ARG;
    }
    if (hflag) {
        set_error("invalid argument: %s: a 16-bit column names an agent outside the graph (not swarm_graph_compact "
                  "of this row_ptr / col)", who);
        return SWARM_ERR_ARG;
    }
    return SWARM_OK;
}

template <typename Off>
int elect_impl(swarm_ctx *ctx, int64_t n, const Off *rp, const int32_t *col, const int32_t *ids,
               int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
               int32_t *rounds_exec, int64_t *changes_host, swarm_elect_stats *st,
               void *stream, const Off *hrp = nullptr, const int32_t *hcol = nullptr,
               const int16_t *c16 = nullptr) {
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0, "n < 0");
    SW_ARG(n < (int64_t(1) << 31), "n must be < 2^31");
    SW_ARG(max_rounds >= 1, "max_rounds < 1");
    const bool timed = (mode & SWARM_ELECT_TIMED) != 0;
    const bool trust_c16 = (mode & SWARM_ELECT_TRUST_C16) != 0;
    mode &= ~(SWARM_ELECT_TIMED | SWARM_ELECT_TRUST_C16);
    SW_ARG(mode == SWARM_ELECT_DENSE || mode == SWARM_ELECT_FRONTIER, "unknown mode");
    SW_ARG(rounds_exec != nullptr, "rounds_exec is NULL");
    SW_ARG(n == 0 || (rp && ids && leader && state), "NULL array (col may be NULL only without edges)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st) *st = swarm_elect_stats{};
    if (n == 0) {  // an empty swarm: round 1 changes nothing
        *rounds_exec = 1;
        if (changes_host) changes_host[0] = 0;
        if (st) st->rounds_launched = 1;
        return SWARM_OK;
    }
    // 16-bit columns are checked before any round reads them (one pass over the columns, read back with
    // the edge count): escaped columns or a foreign buffer are refused, never gathered through
    SW_ARG(!c16 || !esc_registered(ctx, c16), "col16 holds swarm_graph_compact_escaped's columns (escapes)");
    // SWARM_ELECT_TRUST_C16 with this ctx's record of the buffer: its columns and the edge count are known
    const swarm_ctx::C16Built *rec = (trust_c16 && c16 && !hrp) ? c16_record(ctx, c16, rp, col, n) : nullptr;
    Off e_total = 0;
    if (rec) {
        e_total = Off(rec->e_total);
    } else {
        unsigned c16_bad = 0;
        if (c16) {
            if (int rc = enqueue_col16_check<Off>(ctx, rp, c16, col, false, n, n, &c16_bad, s)) return rc;
        }
        SW_HIP(hipMemcpyAsync(&e_total, rp + n, sizeof(Off), hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        if (int rc = col16_verdict(c16_bad, "swarm_elect_compact")) return rc;
    }
    SW_ARG(e_total == 0 || col != nullptr, "col is NULL but the graph has edges");
    // the int32-CSR kernels address with 32-bit byte offsets (gather_listed's ld4 / Col16::at32):
    // 4-byte columns need < 2^30 edges, 2-byte ones < 2^31 (less a margin for the clamped offsets a
    // window or a pass computes past its row's end) -- C5's 100M agents (1.6e9 edges) fit with them
    const bool c16_only = c16 && !hrp && tuning().dense_flat;
    const int64_t e_cap = c16_only ? (int64_t(1) << 31) - (int64_t(1) << 20) : (int64_t(1) << 30);
    SW_ARG(sizeof(Off) == 8 || (n < (int64_t(1) << 30) && int64_t(e_total) < e_cap),
           "int32 CSR supports < 2^30 agents and edges (< 2^31 - 2^20 edges with 16-bit columns): use "
           "swarm_elect_i64 / swarm_elect_compact_i64");
    if (hrp) {  // directed: the transpose must hold the same edges
        Off h_total = 0;
        SW_HIP(hipMemcpyAsync(&h_total, hrp + n, sizeof(Off), hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        SW_ARG(h_total == e_total, "hear_row_ptr[n] != row_ptr[n]: not the transpose of the graph");
        SW_ARG(h_total == 0 || hcol != nullptr, "hear_col is NULL but the graph has edges");
    }
    int32_t *bufs[2] = {leader, nullptr};
    SW_ALLOC(bufs[1], ctx, S_LEADER_B, size_t(n) * 4);
    SW_HIP(hipMemcpyAsync(leader, ids, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
    Frontier f{};
    unsigned long long *ring;
    if (mode == SWARM_ELECT_FRONTIER) {
        SW_HIP(hipMemcpyAsync(bufs[1], ids, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
        int rc0 = frontier_alloc(ctx, n, n, bufs[0], bufs[1], &f, s);
        if (rc0) return rc0;
        ring = f.ring;
        f.c16 = c16;
    } else {
        SW_ALLOC(ring, ctx, S_CHANGES, ring_bytes());
        SW_HIP(hipMemsetAsync(ring, 0, ring_bytes(), s));
        ctx->step_rows = ctx->step_all = 0;  // the stepper state is gone
    }
    constexpr int kMaxBatch = 256;
    // the per-round totals land in mapped host memory, written by k_batch_totals itself, then the batch's
    // epoch word after them (k_signal), which the host spins on
    void *dmap = nullptr;
    unsigned long long *hbuf =
        static_cast<unsigned long long *>(mapped(ctx, size_t(kCounters) * 8 * kMaxBatch + 128, &dmap));
    if (!hbuf) return SWARM_ERR_OOM;
    unsigned long long *dtot = static_cast<unsigned long long *>(dmap);
    unsigned long long *h_epoch = hbuf + size_t(kCounters) * kMaxBatch;
    unsigned long long *d_epoch = dtot + size_t(kCounters) * kMaxBatch;
    // a tag no counter value reaches, then the batch number (the word is shared with other calls)
    const unsigned long long ep_tag = 0xE1EC7ull << 40;
    unsigned long long ep = 0;
    __atomic_store_n(h_epoch, 0ull, __ATOMIC_RELEASE);

    int found = -1, t = 1, batch = 8, launched = 0;
    std::vector<int64_t> hist;  // per-round change counts read so far (batch sizing, layout)
    const StampMap il_map = stamp_map(n, true), ag_map = stamp_map(n, false);
    const int64_t il_min = tuning().il_min_changes >= 0 ? tuning().il_min_changes
                                                        : std::max<int64_t>(1, int64_t(8e-4 * double(n)));
    StampMap rd_map = il_map;
    int64_t act_sum = 0, edge_sum = 0, chg_sum = 0, dense_rounds = 0, sp_launches = 0;
    double bytes = 0.0, sp_bytes = 0.0, sp_ms = 0.0;
    std::vector<RoundKind> kinds(kMaxBatch);
    std::vector<float> ktime(kMaxBatch);
    // optional per-round timing: events before and after every round kernel
    std::vector<hipEvent_t> ev;
    double k_ms = 0;
    int64_t timed_rounds = 0;
    if (timed) {
        ev.resize(2 * kMaxBatch + 2);
        for (auto &x : ev) SW_HIP(hipEventCreate(&x));
    }
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() { for (auto x : v) (void)hipEventDestroy(x); }
    } ev_free{ev};
    FILE *rlog = nullptr;  // SWARM_ROUND_LOG=path: one line per round (tuning aid)
    if (const char *pth = getenv("SWARM_ROUND_LOG")) rlog = fopen(pth, "w");
    struct LogClose {
        FILE *&f;
        ~LogClose() { if (f) fclose(f); }
    } log_close{rlog};
    // Look-ahead: each batch's counters are read back from a point kLook rounds before its end, so
    // the GPU is still running the batch's last rounds while the host reads, decides the next batch
    // and enqueues it (no idle gap at a batch boundary).  Rounds launched past convergence are
    // guarded no-ops.  Per-round timing and the round log keep the plain read-at-the-end batches.
    const int kLook = (timed || rlog) ? 0 : tuning().look;
    int read_upto = 0;  // rounds whose counters the host has read
    // the per-round counters of rounds (read_upto, tread], read back into hbuf: hist, stats, found
    auto consume = [&](int tread) {
        for (int r = read_upto + 1; r <= tread; ++r) {
            const unsigned long long *rb = hbuf + size_t(r - read_upto - 1) * kCounters;
            const int64_t c = int64_t(rb[C_CHG]);
            hist.push_back(c);
            const RoundKind kind = mode == SWARM_ELECT_DENSE ? RK_DENSE : plan_round(r);
            const bool dn = kind == RK_DENSE || kind == RK_DENSE_MARK;
            if (changes_host) changes_host[r - 1] = c;
            const int64_t act = dn ? n : int64_t(rb[C_ACT]);
            const int64_t ed = dn ? int64_t(e_total) : int64_t(rb[C_EDGE]);
            act_sum += act;
            edge_sum += ed;
            chg_sum += c;
            dense_rounds += dn ? 1 : 0;
            const double rbytes = round_bytes(dn, n, int64_t(e_total), act, ed);
            bytes += rbytes;
            if (kind == RK_SPARSE) sp_bytes += rbytes;
            if (rlog)
                fprintf(rlog, "%d %lld %lld %lld %d %.2f\n", r, (long long)c, (long long)act, (long long)ed,
                        int(kind), timed && r >= t ? ktime[r - t] * 1e3 : 0.0);
            if (c == 0) {
                found = r;
                break;
            }
        }
        read_upto = tread;
    };
    // the counters of rounds (read_upto, upto] read back and consumed (every launched round drained)
    auto read_rounds = [&](int upto) -> int {
        if (upto <= read_upto) return SWARM_OK;
        hipLaunchKernelGGL(k_batch_totals, dim3(upto - read_upto), dim3(kWave), 0, s, ring, read_upto + 1, dtot);
        SW_LAUNCHED();
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(1), 0, s, d_epoch, ep_tag | ++ep);
        SW_LAUNCHED();
        if (int rc2 = wait_mapped_word(h_epoch, ep_tag | ep, s, "election read-back")) return rc2;
        consume(upto);
        return SWARM_OK;
    };
    int64_t tail_retry_below = INT64_MAX;  // the tail did not start: retry once the changes halve
    // One-workgroup tail from round launched + 1: drain, collect the marked agents, run k_tail_wg, read its
    // rounds' counters.  Leaves launched / rd_map where the frontier rounds go on.
    auto tail_rounds = [&](int cap) -> int {
        if (int rc2 = read_rounds(launched)) return rc2;
        if (found > 0 || launched >= max_rounds) return SWARM_OK;
        const int t0 = launched + 1;
        const int t_end = std::min(max_rounds, t0 + 199);  // <= 200 rounds: one counter read-back
        char *tb;
        const size_t clk_words = tuning().tail_log ? 2 * 201 : 0;
        SW_ALLOC(tb, ctx, S_LIST, 64 + size_t(kTailCap) * 4 + clk_words * 8);
        unsigned *gcount = reinterpret_cast<unsigned *>(tb);
        int32_t *glist = reinterpret_cast<int32_t *>(tb + 64);
        unsigned long long *clk = clk_words ? reinterpret_cast<unsigned long long *>(tb + 64 + size_t(kTailCap) * 4)
                                            : nullptr;
        SW_HIP(hipMemsetAsync(gcount, 0, 4, s));
        f.sm = rd_map;
        const dim3 cgrid(grid_for(f.sm.M, 1, unsigned(tuning().sparse_blocks)));
        if (f.sm.cshift == 9)  // small swarm: 512-stamp chunks (2 per thread)
            hipLaunchKernelGGL((k_tail_collect<2>), cgrid, dim3(kBlock), 0, s, f, t0, glist, gcount, cap);
        else
            hipLaunchKernelGGL((k_tail_collect<kScan>), cgrid, dim3(kBlock), 0, s, f, t0, glist, gcount, cap);
        SW_LAUNCHED();
        const int64_t n16 = int64_t(2 * act_bytes(n)) / 16;
        hipLaunchKernelGGL(k_tail_clear, dim3(grid_for(n16, kBlock, 2048)), dim3(kBlock), 0, s,
                           reinterpret_cast<uint4 *>(f.act[0]), n16, gcount, cap);
        SW_LAUNCHED();
        f.wsm = ag_map;  // hand-back marks in agent order
        // out[0..3] in mapped memory after the batch totals' epoch word
        unsigned long long *h_out = h_epoch + 1, *d_out = d_epoch + 1;
        const unsigned long long tep = (0x7A11ull << 40) | ++ep;
        __atomic_store_n(&h_out[3], 0ull, __ATOMIC_RELEASE);
        if (c16)
            hipLaunchKernelGGL((k_tail_wg<Col16>), dim3(1), dim3(kTailThreads), 0, s,
                               reinterpret_cast<const int32_t *>(rp), Col16{c16}, f, glist, gcount, t0, t_end, cap,
                               d_out, tep, clk);
        else
            hipLaunchKernelGGL((k_tail_wg<Col32>), dim3(1), dim3(kTailThreads), 0, s,
                               reinterpret_cast<const int32_t *>(rp), Col32{col}, f, glist, gcount, t0, t_end, cap,
                               d_out, tep, clk);
        SW_LAUNCHED();
        if (int rc2 = wait_mapped_word(&h_out[3], tep, s, "one-workgroup tail")) return rc2;
        const unsigned long long why = __atomic_load_n(&h_out[1], __ATOMIC_ACQUIRE);
        const int last = int(__atomic_load_n(&h_out[0], __ATOMIC_ACQUIRE));
        if (why == TAIL_NOT_STARTED) {
            tail_retry_below = std::max<int64_t>(1, hist.back() / 2);
            return SWARM_OK;
        }
        if (clk) {  // experiment aid: per-round microseconds (100 MHz wall clock) and marked agents
            SW_HIP(hipStreamSynchronize(s));
            std::vector<unsigned long long> hc(clk_words);
            SW_HIP(hipMemcpy(hc.data(), clk, clk_words * 8, hipMemcpyDeviceToHost));
            for (int r = t0; r < last; ++r)
                fprintf(stderr, "[tail] round %d marked %llu us %.2f\n", r, hc[2 * (r - t0) + 1],
                        double(hc[2 * (r - t0 + 1)] - hc[2 * (r - t0)]) / 100.0);
        }
        launched = last;
        if (int rc2 = read_rounds(last)) return rc2;
        rd_map = ag_map;  // the hand-back marks (if the run goes on)
        batch = 8;
        return SWARM_OK;
    };
    while (read_upto < max_rounds && found < 0) {
        t = launched + 1;  // first round launched in this batch (> tend when only a read is left)
        const int tend = std::min(max_rounds, launched + batch);
        // read rounds (read_upto, tread]: at least one (the first batches are shorter than kLook)
        const int tread = tend == max_rounds ? tend : std::max(read_upto + 1, tend - kLook);
        int rc = 0;
        // per-round totals of rounds (read_upto, tread], reduced on device into mapped host memory, then
        // the batch's epoch word
        auto enqueue_read = [&]() -> int {
            hipLaunchKernelGGL(k_batch_totals, dim3(tread - read_upto), dim3(kWave), 0, s, ring, read_upto + 1, dtot);
            SW_LAUNCHED();
            hipLaunchKernelGGL(k_signal, dim3(1), dim3(1), 0, s, d_epoch, ep_tag | ++ep);
            SW_LAUNCHED();
            return SWARM_OK;
        };
        if (tread <= launched && (rc = enqueue_read())) return rc;
        // timing: dense rounds (and every round when a per-round log is written) get an event pair
        // each; a batch's run of back-to-back sparse rounds gets ONE pair around it -- events
        // between every launch would add their own cost to each round (rocprof's per-dispatch
        // durations are the reference for this figure)
        int seg_n = 0;  // sparse launches inside this batch's segment
        for (int r = t; r <= tend; ++r) {
            const bool sparse = mode == SWARM_ELECT_FRONTIER && plan_round(r) == RK_SPARSE;
            const bool seg = timed && sparse && !rlog;
            if (seg && seg_n++ == 0) SW_HIP(hipEventRecord(ev[2 * kMaxBatch], s));
            hipEvent_t *e2 = (timed && !seg) ? &ev[2 * (r - t)] : nullptr;
            if (e2) SW_HIP(hipEventRecord(e2[0], s));
            if (mode == SWARM_ELECT_DENSE) {
                kinds[r - t] = RK_DENSE;
                rc = launch_dense_round<Off>(rp, col, bufs[(r - 1) & 1], bufs[r & 1], n, 0, n, ring, nullptr, nullptr,
                                             StampMap{}, r, 1, s, nullptr, nullptr, c16);
            } else {
                kinds[r - t] = plan_round(r);
                // marks for round r+1: interleaved layout while rounds are busy (balance), agent
                // order once they are sparse (locality of the few gathers)
                f.sm = rd_map;
                f.wsm = (hist.empty() || hist.back() >= il_min) ? il_map : ag_map;
                rc = launch_frontier_round<Off>(rp, col, f, r, kinds[r - t], 1, s, hrp, hcol);
                rd_map = f.wsm;
            }
            if (rc) return rc;
            if (e2) SW_HIP(hipEventRecord(e2[1], s));
            if (r == tread && (rc = enqueue_read())) return rc;
        }
        if (seg_n) SW_HIP(hipEventRecord(ev[2 * kMaxBatch + 1], s));
        launched = std::max(launched, tend);
        if ((rc = wait_mapped_word(h_epoch, ep_tag | ep, s, "election read-back"))) return rc;
        if (timed) {  // kLook == 0: this batch's rounds are exactly the rounds read
            SW_HIP(hipStreamSynchronize(s));
            for (int r = t; r <= tend; ++r) {  // every launched round's kernel time (rocprof's view)
                if (seg_n && kinds[r - t] == RK_SPARSE) continue;  // in the segment
                float x = 0;
                SW_HIP(hipEventElapsedTime(&x, ev[2 * (r - t)], ev[2 * (r - t) + 1]));
                k_ms += x;
                ++timed_rounds;
                if (kinds[r - t] == RK_SPARSE) {
                    sp_ms += x;
                    ++sp_launches;
                }
                ktime[r - t] = x;
            }
            if (seg_n) {
                float x = 0;
                SW_HIP(hipEventElapsedTime(&x, ev[2 * kMaxBatch], ev[2 * kMaxBatch + 1]));
                k_ms += x;
                sp_ms += x;
                timed_rounds += seg_n;
                sp_launches += seg_n;
            }
        }
        consume(tread);
        // a batch spans at most kRing/2 rounds of counter slots, look-ahead included (bookkeeping
        // recycles the slot of round t - kRing/2 in round t)
        batch = next_round_batch(hist.data(), hist.size(), batch, kMaxBatch - kLook);
        // the one-workgroup tail (opt-in experiment): once the last read round's risers x 4 fit its list (the
        // marked agents of a tail round are ~3x the previous round's risers at 100k-10M agents; a list that
        // does not fit is caught by the collect), with short batches once that is near, so that the switch
        // is not a long batch late
        const int cap = tuning().tail_wg;
        if (cap > 0 && !hist.empty() && hist.back() * 4 <= 8 * int64_t(cap)) batch = std::min(batch, 8);
        if (cap > 0 && found < 0 && mode == SWARM_ELECT_FRONTIER && !hrp && !timed && !rlog && sizeof(Off) == 4 &&
            !hist.empty() && hist.back() > 0 && hist.back() * 4 <= cap && hist.back() < tail_retry_below &&
            launched < max_rounds && plan_round(launched + 1) == RK_SPARSE) {
            if ((rc = tail_rounds(cap))) return rc;
        }
    }
    const int last = found > 0 ? found : max_rounds;
    if (found < 0 && (last & 1)) {
        // after a zero-change round both buffers hold the final state (dense and frontier alike);
        // otherwise the newest is bufs[last & 1]
        SW_HIP(hipMemcpyAsync(leader, bufs[1], size_t(n) * 4, hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL(k_state, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, leader,
                       ids, state, n);
    SW_LAUNCHED();
    *rounds_exec = last;
    if (st) {
        st->rounds_launched = launched;
        st->changes_total = chg_sum;
        st->gather_ms = k_ms;
        st->apply_ms = 0.0;
        st->gather_launches = timed_rounds;
        st->active_total = act_sum;
        st->edges_total = edge_sum;
        st->dense_rounds = dense_rounds;
        st->bytes_total = bytes;
        st->sparse_ms = sp_ms;
        st->sparse_launches = sp_launches;
        st->sparse_bytes = sp_bytes;
    }
    return found > 0 ? SWARM_OK : SWARM_NOT_CONVERGED;
}

}  // namespace

// Internal entry points for comm.hip (the RCCL round loop): one stepper round, the ghost update
// of both borders, and the device per-round totals (kCounters each) of rounds t0..t1.
// The column check of the stepper's 16-bit columns against the stepped graph (rows and indices
// [0, n_all)), once per set_compact: comm.hip runs it before its agreement, the public stepper at its
// first round.
int frontier_check_compact(swarm_ctx *ctx, const int32_t *rp, const int32_t *col, hipStream_t s) {
    if (!ctx->step_c16 || ctx->step_c16_checked || ctx->step_all == 0) return SWARM_OK;
    SW_ARG(rp != nullptr, "row_ptr is NULL");
    SW_ARG(!ctx->step_c16_esc || col != nullptr, "escaped 16-bit columns need the int32 columns (col is NULL)");
    unsigned bad = 0;
    if (int rc = enqueue_col16_check<int32_t>(ctx, rp, ctx->step_c16, col, ctx->step_c16_esc, ctx->step_all,
                                              ctx->step_all, &bad, s))
        return rc;
    SW_HIP(hipStreamSynchronize(s));
    if (int rc = col16_verdict(bad, ctx->step_c16_esc ? "swarm_frontier_set_compact_escaped"
                                                      : "swarm_frontier_set_compact"))
        return rc;
    ctx->step_c16_checked = true;
    return SWARM_OK;
}

int frontier_round_stepper(swarm_ctx *ctx, int t, const int32_t *rp, const int32_t *col, int32_t *L0,
                           int32_t *L1, hipStream_t s) {
    Frontier f{};
    int rc = frontier_bind(ctx, L0, L1, &f);
    if (rc) return rc;
    if (f.n_rows == 0) return SWARM_OK;
    if ((rc = frontier_check_compact(ctx, rp, col, s))) return rc;
    rc = launch_frontier_round<int32_t>(rp, col, f, t, plan_round(t), /*guard=*/0, s);
    ctx->step_rd_agent = ctx->step_wr_agent;  // the marks this round wrote
    return rc;
}

// Whether round t of the frontier stepper is a dense sweep (its active / edge counters are not kept).
bool frontier_round_dense(int t) { return plan_round(t) != RK_SPARSE; }

// The interleaved -> agent-order switch point of the stamp layout for an n-agent swarm (elect_impl's
// il_min; the sharded C loop compares the global changes against it for the global agent count).
int64_t frontier_il_min(int64_t n) {
    return tuning().il_min_changes >= 0 ? tuning().il_min_changes : std::max<int64_t>(1, int64_t(8e-4 * double(n)));
}

int frontier_ghosts_both(swarm_ctx *ctx, int t, const int32_t *rp, const int32_t *col, int64_t b_lo, int64_t n_lo,
                         const int32_t *in_lo, int64_t b_hi, int64_t n_hi, const int32_t *in_hi, int32_t *L0,
                         int32_t *L1, hipStream_t s) {
    Frontier f{};
    int rc = frontier_bind(ctx, L0, L1, &f);
    if (rc) return rc;
    const auto outside = [&](int64_t b, int64_t c) {  // [b, b + c) within [0, n_all) and off the owned rows
        return c == 0 || (b >= 0 && b + c <= f.n_all && (b + c <= f.c_lo || b >= f.n_count));
    };
    SW_ARG(outside(b_lo, n_lo) && outside(b_hi, n_hi), "ghost ranges must lie in [0, n_all) outside the owned rows");
    if (n_lo + n_hi == 0) return SWARM_OK;
    f.wsm = f.sm;  // ghost rises mark for the next round, in the layout that round reads
    hipLaunchKernelGGL((k_frontier_ghosts<int32_t>), dim3(grid_for(n_lo + n_hi, kBlock / 8, 1024)), dim3(kBlock), 0,
                       s, rp, col, f, b_lo, n_lo, in_lo, b_hi, n_hi, in_hi, t);
    SW_LAUNCHED();
    return SWARM_OK;
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

int swarm_graph_compact(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col, int16_t *col16,
                        void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    if (!ctx_on_current_device(ctx)) return SWARM_ERR_ARG;
    SW_ARG(n >= 0 && n < (int64_t(1) << 30), "n out of range (< 2^30)");
    if (n == 0) return SWARM_OK;
    SW_ARG(row_ptr != nullptr, "row_ptr is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int32_t e_total = 0;
    SW_HIP(hipMemcpyAsync(&e_total, row_ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    SW_ARG(e_total >= 0, "row_ptr[n] < 0");  // >= 2^30 edges: for swarm_elect_compact_i64
    if (e_total == 0) return SWARM_OK;
    SW_ARG(col && col16, "NULL array");
    int *bad;
    SW_ALLOC(bad, ctx, S_TMP1, sizeof(int));
    SW_HIP(hipMemsetAsync(bad, 0, sizeof(int), s));
    hipLaunchKernelGGL(k_build_col16<false>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, row_ptr, col, n,
                       col16, static_cast<void *>(bad));
    SW_LAUNCHED();
    int hbad = 0;
    SW_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    // the buffer now holds plain deltas (or a refused build): no longer escaped
    ctx->esc_built.erase(std::remove(ctx->esc_built.begin(), ctx->esc_built.end(), col16), ctx->esc_built.end());
    c16_forget(ctx, col16);
    if (!hbad) ctx->c16_built.push_back({col16, row_ptr, col, n, e_total});
    if (hbad) {
        set_error("a neighbour lies more than 32767 storage slots from its row's 64-agent base: keep the int32 columns");
        return SWARM_ERR_RANGE;
    }
    return SWARM_OK;
}

int swarm_graph_compact_escaped(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                                int16_t *col16, int64_t *n_escaped, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    if (!ctx_on_current_device(ctx)) return SWARM_ERR_ARG;
    SW_ARG(n_escaped != nullptr, "n_escaped is NULL");
    *n_escaped = 0;
    SW_ARG(n >= 0 && n < (int64_t(1) << 30), "n out of range (< 2^30)");
    if (n == 0) return SWARM_OK;
    SW_ARG(row_ptr != nullptr, "row_ptr is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int32_t e_total = 0;
    SW_HIP(hipMemcpyAsync(&e_total, row_ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    SW_ARG(e_total >= 0 && e_total < (int64_t(1) << 30), "escaped 16-bit columns: < 2^30 edges (int32 escapes)");
    if (e_total == 0) return SWARM_OK;
    SW_ARG(col && col16, "NULL array");
    unsigned long long *cnt;
    SW_ALLOC(cnt, ctx, S_TMP1, sizeof(unsigned long long));
    SW_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_build_col16<true>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, row_ptr, col, n,
                       col16, static_cast<void *>(cnt));
    SW_LAUNCHED();
    unsigned long long h = 0;
    SW_HIP(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    *n_escaped = int64_t(h);
    c16_forget(ctx, col16);
    if (h && !esc_registered(ctx, col16))
        ctx->esc_built.push_back(col16);
    else if (!h)  // no escape: plain deltas, valid for every reader
        ctx->esc_built.erase(std::remove(ctx->esc_built.begin(), ctx->esc_built.end(), col16), ctx->esc_built.end());
    return SWARM_OK;
}

int swarm_elect_compact(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col, const int16_t *col16,
                        const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
                        int32_t *rounds_exec, int64_t *changes_per_round, swarm_elect_stats *stats, void *stream) {
    return swarm::elect_impl<int32_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode, rounds_exec,
                                      changes_per_round, stats, stream, nullptr, nullptr,
                                      swarm::tuning().use_c16 ? col16 : nullptr);
}

int swarm_elect_directed(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col,
                         const int32_t *hear_row_ptr, const int32_t *hear_col, const int32_t *ids,
                         int32_t *leader, uint8_t *state, int32_t max_rounds, int32_t mode,
                         int32_t *rounds_exec, int64_t *changes_per_round, swarm_elect_stats *stats,
                         void *stream) {
    SW_ARG(hear_row_ptr != nullptr || n == 0, "hear_row_ptr is NULL (use swarm_elect for a symmetric graph)");
    return swarm::elect_impl<int32_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode,
                                      rounds_exec, changes_per_round, stats, stream, hear_row_ptr, hear_col);
}

int swarm_elect_i64(swarm_ctx *ctx, int64_t n, const int64_t *row_ptr, const int32_t *col,
                    const int32_t *ids, int32_t *leader, uint8_t *state, int32_t max_rounds,
                    int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                    swarm_elect_stats *stats, void *stream) {
    return swarm::elect_impl<int64_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode,
                                      rounds_exec, changes_per_round, stats, stream);
}

int swarm_elect_compact_i64(swarm_ctx *ctx, int64_t n, const int64_t *row_ptr, const int32_t *col,
                            const int16_t *col16, const int32_t *ids, int32_t *leader, uint8_t *state,
                            int32_t max_rounds, int32_t mode, int32_t *rounds_exec, int64_t *changes_per_round,
                            swarm_elect_stats *stats, void *stream) {
    return swarm::elect_impl<int64_t>(ctx, n, row_ptr, col, ids, leader, state, max_rounds, mode, rounds_exec,
                                      changes_per_round, stats, stream, nullptr, nullptr,
                                      swarm::tuning().use_c16 ? col16 : nullptr);
}

int swarm_frontier_begin(swarm_ctx *ctx, int64_t n_rows, int64_t n_all, const int32_t *init,
                         int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n_rows >= 0 && n_all >= n_rows && n_all < (int64_t(1) << 30), "sizes out of range (n_all < 2^30)");
    SW_ARG(n_all == 0 || (init && leader0 && leader1), "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    Frontier f{};
    int rc = frontier_alloc(ctx, n_rows, n_all, leader0, leader1, &f, s);
    if (rc) return rc;
    if (n_all) {
        SW_HIP(hipMemcpyAsync(leader0, init, size_t(n_all) * 4, hipMemcpyDeviceToDevice, s));
        SW_HIP(hipMemcpyAsync(leader1, init, size_t(n_all) * 4, hipMemcpyDeviceToDevice, s));
    }
    return SWARM_OK;
}

int swarm_frontier_begin_range(swarm_ctx *ctx, int64_t own_begin, int64_t n_own, int64_t n_all, const int32_t *init,
                               int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(own_begin >= 0 && n_own >= 0 && own_begin + n_own <= n_all, "owned range out of [0, n_all)");
    int rc = swarm_frontier_begin(ctx, n_own, n_all, init, leader0, leader1, stream);
    if (rc) return rc;
    ctx->step_lo = own_begin;
    return SWARM_OK;
}

// Both setters leave the columns unchecked: the stepper checks them against its graph before the first
// round that reads them (frontier_check_compact), and refuses a buffer with escapes here already when
// this ctx built it with swarm_graph_compact_escaped.
int swarm_frontier_set_compact(swarm_ctx *ctx, const int16_t *col16) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(!col16 || !esc_registered(ctx, col16),
           "col16 holds swarm_graph_compact_escaped's columns: use swarm_frontier_set_compact_escaped");
    ctx->step_c16 = tuning().use_c16 ? col16 : nullptr;
    ctx->step_c16_esc = false;
    ctx->step_c16_checked = false;
    return SWARM_OK;
}

int swarm_frontier_set_compact_escaped(swarm_ctx *ctx, const int16_t *col16) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    ctx->step_c16 = tuning().use_c16 ? col16 : nullptr;
    ctx->step_c16_esc = ctx->step_c16 != nullptr;
    ctx->step_c16_checked = false;
    return SWARM_OK;
}

int swarm_frontier_step(swarm_ctx *ctx, int32_t t, const int32_t *row_ptr, const int32_t *col,
                        int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(t >= 1, "round must be >= 1");
    if (ctx->step_all == 0) return SWARM_OK;
    SW_ARG(row_ptr && leader0 && leader1, "NULL array");
    return frontier_round_stepper(ctx, t, row_ptr, col, leader0, leader1, static_cast<hipStream_t>(stream));
}

int swarm_frontier_ghosts(swarm_ctx *ctx, int32_t t, int64_t begin, int64_t count,
                          const int32_t *incoming, const int32_t *row_ptr, const int32_t *col,
                          int32_t *leader0, int32_t *leader1, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(begin >= 0 && count >= 0 && begin + count <= ctx->step_all, "ghost range out of bounds");
    if (count == 0) return SWARM_OK;
    SW_ARG(incoming && row_ptr && leader0 && leader1, "NULL array");
    return frontier_ghosts_both(ctx, t, row_ptr, col, begin, count, incoming, ctx->step_all, 0, nullptr, leader0,
                                leader1, static_cast<hipStream_t>(stream));
}

#ifdef SWARM_PHASES
int swarm_debug_phases(unsigned long long *out, int count) {
    SW_HIP(hipDeviceSynchronize());
    SW_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(swarm::g_phase), size_t(count) * 8));
    return SWARM_OK;
}
#endif

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
    for (int i = 0; i < nr; ++i) out[i] = int64_t(h[size_t(i) * kCounters + C_CHG]);
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
    int rc = launch_dense_round<int32_t>(row_ptr, col, leader_in, leader_out, n_rows, 0, n_rows, ring, nullptr, nullptr,
                                        StampMap{}, 0, 0, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_sum_shards, dim3(1), dim3(kWave), 0, s, ring, 0,
                       reinterpret_cast<unsigned long long *>(changed));
    SW_LAUNCHED();
    return SWARM_OK;
}

}  // extern "C"
