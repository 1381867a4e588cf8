// Record-list tail of an election (contract E2) on gfx950.
//
// Replaces the same handlers as swarm_elect (_handle_election_acclaim / _handle_heartbeat,
// agent.py:243-275) for the LATE rounds of an election, with the same results: leaders, states,
// rounds_exec and every per-round change count.
//
// Why: late in an election the changes sit on a few thin fronts.  A synchronous round costs its
// fixed chain (kernel boundary, stamp words, list, row bounds, columns, leaders: ~9-13 us at 10M
// agents) for a few thousand changes, and the fronts need ~1 000 more rounds to cross the swarm.
// The rounds are only a way to compute, for every agent v, the step function
//     f_v(t) = max{ id(u) : d(v, u) <= t }
// (E2's leader after round t).  After round T0 every agent holds L_v = f_v(T0), and for t > T0
//     f_v(t) = max{ L_w : d(v, w) <= t - T0 }.
// That step function is its pareto set of RECORDS (d, val) -- v reaches val at round T0 + d --
// and the record lists are the least fixpoint of
//     list_v = pareto( {(0, L_v)}  u  { (d + 1, val) : (d, val) in {(0, L_u)} u list_u, u in N(v) } ).
// Every pair any relaxation produces is a true statement ("a value >= val lies within T0 + d hops"),
// so relaxations may run in ANY order and still end at the fixpoint: tiles of cells run to a local
// fixpoint on chip and only their borders wait for the next launch.  Per-round changes are then
// the histogram of the records' d, the leaders the last record of each list.  The frontier rounds'
// per-round semantics are kept exactly; only the order of work changes.
//
// Layout (swarm_record_index, built once per graph): the cell grid of the storage order is cut into
// tiles of kRT x kRT cells; a tile's REGION is its core plus the ring of cells around it (an edge
// joins cells at most one apart: swarm_tile_index checks).  Region slots: the core agents first
// (core grid rows, each one contiguous storage run), then the ring (bottom row, left/right cells of
// each core row, top row).  Per tile the index holds the core agents' rows as u16 region slots
// (rcol, rows rrow) and every region slot's storage index (ragent), each tile's block padded to
// 16 bytes so a launch loads it with 16-byte loads.
//
// Tail state: per agent kRR list entries in HBM, u64 each = (gen << 20 | d) << 32 | val, written
// whole (a reader may see a mix of two versions of a list, but every entry it sees is a true
// statement; entries of another election have another gen and are ignored); launch-stamped agent
// marks and tile flags, u32 (gen << 20 | launch).
//
// A launch k: one wave per active tile (k_rec_tiles), the tile's region in LDS (lists, base
// values, local CSR); marked core agents pull from their neighbours, Gauss-Seidel inside the wave,
// until no core agent is marked; changed border agents mark their neighbours in other tiles for
// launch k+1 (agent mark + tile flag; the first flagger appends the tile to launch k+1's list).
// WINDOW: launch k only admits records with d <= k * delta; a record beyond it leaves its agent
// marked for the next launch.  Without it a tile races ahead on stale borders and redoes the work
// when the true fronts arrive (tools/record_tail_sim.py: 6x the frontier's recomputes at 10M agents
// unbounded, 1.5x with delta = 8).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "swarm_common.h"

namespace swarm {
namespace {

constexpr int kRT = kRecTile;          // core cells per tile side
constexpr int kRR = kRecEntries;       // list entries per agent
constexpr int kRSlots = 640;           // region agents per tile held in LDS
constexpr int kRCore = 448;            // core agents per tile
constexpr int kREdges = 8192;          // core edges per tile
constexpr int kRRuns = 3 * kRT + 2;    // region runs: kRT core rows, bottom row, left+right cells, top row
constexpr int kRLevelCap = 4095;       // levels per activation (a safety net: never reached)
constexpr int kRHist = 4096;           // LDS histogram bins of the finalize pass

__device__ __forceinline__ uint32_t rtag(uint32_t gen, uint32_t k) { return (gen << kRecDBits) | k; }

__device__ __forceinline__ int64_t tile_of_cell(int32_t c, int64_t ncx, int64_t ntx) {
    return (int64_t(c) / ncx) / kRT * ntx + (int64_t(c) % ncx) / kRT;
}

// Cells of run r of tile `tile`'s region: one grid row's range [a, b) (contiguous storage).
// Runs that do not exist (grid edge) are empty.
__device__ __forceinline__ void region_run_cells(const RecGeom &g, int64_t tile, int r, int64_t &a, int64_t &b) {
    const int64_t tx = tile % g.ntx, ty = tile / g.ntx;
    const int64_t x0 = tx * kRT, x1 = x0 + kRT < g.ncx ? x0 + kRT : g.ncx;
    const int64_t y0 = ty * kRT, y1 = y0 + kRT < g.ncy ? y0 + kRT : g.ncy;
    const int h = int(y1 - y0);
    const int64_t rx0 = x0 > 0 ? x0 - 1 : 0, rx1 = x1 < g.ncx ? x1 + 1 : g.ncx;
    a = b = 0;
    if (r < h) {
        a = (y0 + r) * g.ncx + x0;
        b = (y0 + r) * g.ncx + x1;
    } else if (r == h) {
        if (y0 > 0) {
            a = (y0 - 1) * g.ncx + rx0;
            b = (y0 - 1) * g.ncx + rx1;
        }
    } else if (r <= 3 * h) {
        const int j = (r - h - 1) >> 1;
        if (((r - h - 1) & 1) == 0) {
            if (x0 > 0) {
                a = (y0 + j) * g.ncx + x0 - 1;
                b = a + 1;
            }
        } else if (x1 < g.ncx) {
            a = (y0 + j) * g.ncx + x1;
            b = a + 1;
        }
    } else if (r == 3 * h + 1) {
        if (y1 < g.ncy) {
            a = y1 * g.ncx + rx0;
            b = y1 * g.ncx + rx1;
        }
    }
}

// Run of tile `tile`'s region holding cell (cx, cy), or -1 (the cell is outside the region).
__device__ __forceinline__ int run_of_cell(const RecGeom &g, int64_t tile, int64_t cx, int64_t cy) {
    const int64_t tx = tile % g.ntx, ty = tile / g.ntx;
    const int64_t x0 = tx * kRT, x1 = x0 + kRT < g.ncx ? x0 + kRT : g.ncx;
    const int64_t y0 = ty * kRT, y1 = y0 + kRT < g.ncy ? y0 + kRT : g.ncy;
    const int h = int(y1 - y0);
    if (cy >= y0 && cy < y1) {
        if (cx >= x0 && cx < x1) return int(cy - y0);
        if (cx == x0 - 1) return h + 1 + 2 * int(cy - y0);
        if (cx == x1) return h + 2 + 2 * int(cy - y0);
        return -1;
    }
    if (cx < x0 - 1 || cx > x1) return -1;
    if (cy == y0 - 1) return h;
    if (cy == y1) return 3 * h + 1;
    return -1;
}

__device__ __forceinline__ int nruns_of(const RecGeom &g, int64_t tile) {
    const int64_t ty = tile / g.ntx, y0 = ty * kRT, y1 = y0 + kRT < g.ncy ? y0 + kRT : g.ncy;
    return 3 * int(y1 - y0) + 2;
}

__device__ __forceinline__ int wave_incl_scan(int x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ int wave_sum64(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__host__ __device__ __forceinline__ int64_t pad8(int64_t x) { return (x + 7) & ~int64_t(7); }
__host__ __device__ __forceinline__ int64_t pad4(int64_t x) { return (x + 3) & ~int64_t(3); }

// ------------------------------------------------------------------ index build
// One wave per tile: core agents m, padded core edges, padded region slots, padded rows (m + 1).
__global__ __launch_bounds__(64) void k_ri_count(const uint32_t *__restrict__ off, const int32_t *__restrict__ rp,
                                                 RecGeom g, int32_t *__restrict__ cnt, unsigned *__restrict__ err) {
    const int lane = threadIdx.x;
    const int64_t ntiles = g.ntx * g.nty;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int nr = nruns_of(g, tile), h = (nr - 2) / 3;
        int len = 0, edges = 0;
        if (lane < nr) {
            int64_t a, b;
            region_run_cells(g, tile, lane, a, b);
            if (b > a) {
                const uint32_t s = off[a], e = off[b];
                len = int(e - s);
                if (lane < h) edges = rp[e] - rp[s];
            }
        }
        const int m = wave_sum64(lane < h ? len : 0), slots = wave_sum64(len), ne = wave_sum64(edges);
        if (lane == 0) {
            cnt[tile] = m;
            cnt[ntiles + 1 + tile] = int32_t(pad8(ne));
            cnt[2 * (ntiles + 1) + tile] = int32_t(pad4(slots));
            cnt[3 * (ntiles + 1) + tile] = int32_t(pad8(m + 1));
            if (m > kRCore || slots > kRSlots || ne > kREdges) atomicOr(err, 1u);
        }
    }
}

// One wave per tile: region slot -> storage index, core rows -> local edge offsets, core columns ->
// region slots.  A neighbour outside the region (an edge joining cells more than one apart) sets err.
__global__ __launch_bounds__(64) void k_ri_fill(const uint32_t *__restrict__ off, const int32_t *__restrict__ rp,
                                                const int32_t *__restrict__ col, const int32_t *__restrict__ acell,
                                                RecGeom g, RecIndex ix, unsigned *__restrict__ err) {
    __shared__ int32_t s_st[kRRuns], s_base[kRRuns + 1], s_erow[kRT + 1];
    const int lane = threadIdx.x;
    const int64_t ntiles = g.ntx * g.nty;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int nr = nruns_of(g, tile), h = (nr - 2) / 3;
        int len = 0, edges = 0, st = 0;
        if (lane < nr) {
            int64_t a, b;
            region_run_cells(g, tile, lane, a, b);
            if (b > a) {
                st = int(off[a]);
                len = int(off[b]) - st;
                if (lane < h) edges = rp[st + len] - rp[st];
            }
        }
        const int incl = wave_incl_scan(len), eincl = wave_incl_scan(lane < h ? edges : 0);
        if (lane < nr) {
            s_st[lane] = st;
            s_base[lane + 1] = incl;
        }
        if (lane < h) s_erow[lane + 1] = eincl;
        if (lane == 0) {
            s_base[0] = 0;
            s_erow[0] = 0;
        }
        __syncthreads();
        const int slots = s_base[nr], m = s_base[h];
        const int32_t a0 = ix.ra[tile], e0 = ix.re[tile], s0 = ix.rs[tile], q0 = ix.rq[tile];
        for (int l = lane; l < pad4(slots); l += 64) {  // padding slots name agent 0 (never an edge's slot)
            int r = 0;
            while (r + 1 < nr && s_base[r + 1] <= l) ++r;
            ix.ragent[s0 + l] = l < slots ? s_st[r] + (l - s_base[r]) : 0;
        }
        for (int k = lane; k < m; k += 64) {
            int r = 0;
            while (r + 1 < h && s_base[r + 1] <= k) ++r;
            const int32_t v = s_st[r] + (k - s_base[r]);
            const int32_t lo = s_erow[r] + (rp[v] - rp[s_st[r]]);
            ix.rrow[q0 + k] = uint16_t(lo);
            const int32_t eb = rp[v], ee = rp[v + 1];
            for (int32_t e = eb; e < ee; ++e) {
                const int32_t u = col[e];
                const int32_t c = acell[u];
                const int rr = run_of_cell(g, tile, int64_t(c) % g.ncx, int64_t(c) / g.ncx);
                uint16_t slot = 0;
                if (rr < 0) {
                    atomicOr(err, 2u);
                } else {
                    slot = uint16_t(s_base[rr] + (u - s_st[rr]));
                }
                ix.rcol[e0 + lo + (e - eb)] = slot;
            }
        }
        if (lane == 0) ix.rrow[q0 + m] = uint16_t(s_erow[h]);
        (void)a0;
        __syncthreads();
    }
}

// ------------------------------------------------------------------ tail launches
struct RecState {
    RecIndex ix;
    const int32_t *L;          // state after round T0 (the records' base values)
    unsigned long long *glist; // kRR entries per agent
    uint32_t *gmark;           // agent marks (rtag of the launch that must recompute the agent)
    uint32_t *gchg;            // rtag of the launch an agent's list last changed in
    uint32_t *gpull;           // rtag of the launch an agent last pulled in (0: pull every neighbour)
    uint32_t *tflag;           // tile flags (rtag of the launch that processes the tile)
    int32_t *tlist[2];         // tiles of launch k in tlist[k & 1]
    uint32_t *tcnt;            // tiles of launch k: tcnt[k]
    unsigned *err;             // 1: region over capacity, 2: list overflow, 4: level cap
    unsigned long long *stats; // [0] activations, [1] levels, [2] agent recomputes, [3] region agents loaded,
                               // [4..6] wall clock of the load / levels / end phases
    const int32_t *acell;
    int64_t ncx, ntx;
    uint32_t gen;
};

__device__ __forceinline__ void flag_tile(const RecState &S, int64_t tile, uint32_t tg, int k1) {
    const uint32_t old = atomicMax(&S.tflag[tile], tg);
    if (old < tg) {
        const uint32_t pos = atomicAdd(&S.tcnt[k1], 1u);
        S.tlist[k1 & 1][pos] = int32_t(tile);
    }
}

__device__ __forceinline__ unsigned long long rpack(int d, int32_t val) {
    return (static_cast<unsigned long long>(uint32_t(d)) << 32) | uint32_t(val);
}
__device__ __forceinline__ int rdist(unsigned long long x) { return int(uint32_t(x >> 32)); }
__device__ __forceinline__ int32_t rval(unsigned long long x) { return int32_t(uint32_t(x)); }

// An agent's list while it recomputes, in registers: d = INT_MAX past the end.  Sorted by d
// ascending with values ascending (a pareto list); the base (0, L_v) is implicit.
template <int R>
struct OwnList {
    int d[R];
    int32_t v[R];
    int n;
    __device__ __forceinline__ void load(const unsigned long long *own, int len) {
        n = len;
        const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(own);
#pragma unroll
        for (int q = 0; q < R / 2; ++q) {
            const ulonglong2 w = p[q];
            d[2 * q] = 2 * q < len ? rdist(w.x) : INT_MAX;
            v[2 * q] = 2 * q < len ? rval(w.x) : INT_MIN;
            d[2 * q + 1] = 2 * q + 1 < len ? rdist(w.y) : INT_MAX;
            v[2 * q + 1] = 2 * q + 1 < len ? rval(w.y) : INT_MIN;
        }
    }
    __device__ __forceinline__ void store(unsigned long long *own) const {
        ulonglong2 *p = reinterpret_cast<ulonglong2 *>(own);
#pragma unroll
        for (int q = 0; q < R / 2; ++q) p[q] = ulonglong2{rpack(d[2 * q], v[2 * q]), rpack(d[2 * q + 1], v[2 * q + 1])};
    }
    // the list's value at distance dd: the last entry with d <= dd (values ascend), else the base
    __device__ __forceinline__ int32_t at(int dd, int32_t base) const {
        int32_t m = base;
#pragma unroll
        for (int q = 0; q < R; ++q) m = d[q] <= dd ? v[q] : m;
        return m;
    }
    // insert (dd, val), not dominated (val > at(dd)): the c entries [a, a + c) it dominates
    // (d >= dd, v <= val) go and the rest shift; false on overflow (list unchanged).  Usually
    // c = 0 (shift right by one) or 1 (replace): a few selects per entry, no R x R network.
    __device__ __forceinline__ bool insert(int dd, int32_t val) {
        int a = 0, c = 0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            a += d[q] < dd ? 1 : 0;
            c += (d[q] != INT_MAX && d[q] >= dd && v[q] <= val) ? 1 : 0;
        }
        const int nn = n + 1 - c;
        if (nn > R) return false;
        if (c == 0) {
#pragma unroll
            for (int p = R - 1; p > 0; --p)
                if (p > a) {
                    d[p] = d[p - 1];
                    v[p] = v[p - 1];
                }
        } else {
            for (int t = 1; t < c; ++t) {
#pragma unroll
                for (int p = 1; p < R - 1; ++p)
                    if (p > a) {
                        d[p] = d[p + 1];
                        v[p] = v[p + 1];
                    }
                d[R - 1] = INT_MAX;
                v[R - 1] = INT_MIN;
            }
        }
#pragma unroll
        for (int p = 0; p < R; ++p)
            if (p == a) {
                d[p] = dd;
                v[p] = val;
            }
        n = nn;
        return true;
    }
};

template <int R>
__global__ __launch_bounds__(64) void k_rec_tiles(RecState S, int k, int W, int dcap) {
    __shared__ unsigned long long sE[kRSlots * R];
    __shared__ int32_t sL[kRSlots];
    __shared__ __attribute__((aligned(16))) int32_t sA[kRSlots];       // 16-byte LDS stores below
    __shared__ __attribute__((aligned(16))) uint16_t sCol[kREdges];
    __shared__ __attribute__((aligned(16))) uint16_t sRow[kRCore + 8];
    __shared__ uint8_t sN[kRSlots];
    __shared__ unsigned sMark[kRCore];  // queued for the next level (LDS atomics: first marker appends)
    __shared__ uint8_t sDirty[kRCore];  // 1: list changed, 2: pulled, 4: deferred a record
    __shared__ uint16_t sList[2][kRCore];
    // pull filter: times (launch << 12 | level) of a slot's last change and a core agent's last pull;
    // an agent pulls only from neighbours that changed at or after its last pull
    __shared__ uint32_t sLast[kRCore];
    __shared__ int sCnt[2];
    __shared__ uint32_t sChg[kRSlots];
    __shared__ int32_t sMaxV[kRSlots];  // a slot's largest value (its last record, else its base)
    __shared__ uint8_t sRing[kRSlots];  // ring slots next to a change in this activation
    __shared__ int sDefer;              // an agent of this tile deferred a record past the window
    const int lane = threadIdx.x;
    const uint32_t cnt = S.tcnt[k];
    const uint32_t tgk = rtag(S.gen, uint32_t(k)), tg1 = rtag(S.gen, uint32_t(k + 1));
    const uint32_t genhi = S.gen << kRecDBits;
    const int32_t *list = S.tlist[k & 1];
    unsigned long long my_lev = 0, my_rec = 0, my_load = 0, my_act = 0, c_load = 0, c_lev = 0, c_end = 0;
    for (uint32_t li = blockIdx.x; li < cnt; li += gridDim.x) {
        const int64_t tile = list[li];
        const int32_t a0 = S.ix.ra[tile], m = S.ix.ra[tile + 1] - a0;
        const int32_t e0 = S.ix.re[tile], ne = S.ix.re[tile + 1] - e0;
        const int32_t s0 = S.ix.rs[tile], nr = S.ix.rs[tile + 1] - s0;
        const int32_t q0 = S.ix.rq[tile], nq = S.ix.rq[tile + 1] - q0;
        if (m < 1 || m > kRCore || nr > kRSlots || ne > kREdges || nq > kRCore + 8) {  // the index bounds every tile
            if (lane == 0) atomicOr(S.err, 1u);
            continue;
        }
        ++my_act;
        if (lane == 0) sDefer = 0;
        const unsigned long long w0 = wall_clock64();
        // (a) slot -> agent, the core rows and columns: 16-byte loads, 8 in flight per lane
        {
            const int n16 = nr >> 2, c16 = ne >> 3, r16 = nq >> 3;
            const uint4 *src = reinterpret_cast<const uint4 *>(S.ix.ragent + s0);
            const uint4 *csrc = reinterpret_cast<const uint4 *>(S.ix.rcol + e0);
            const uint4 *rsrc = reinterpret_cast<const uint4 *>(S.ix.rrow + q0);
            uint4 *dst = reinterpret_cast<uint4 *>(sA), *cdst = reinterpret_cast<uint4 *>(sCol),
                  *rdst = reinterpret_cast<uint4 *>(sRow);
            const int tot = n16 + c16 + r16;  // one flat range over the three blocks
            constexpr int kB = 8;
            for (int i0 = 0; i0 < tot; i0 += 64 * kB) {
                uint4 x[kB];
#pragma unroll
                for (int j = 0; j < kB; ++j) {
                    const int i = i0 + lane + 64 * j;
                    const uint4 *p = i < n16 ? src + i : i < n16 + c16 ? csrc + (i - n16) : rsrc + (i - n16 - c16);
                    x[j] = i < tot ? *p : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < kB; ++j) {
                    const int i = i0 + lane + 64 * j;
                    if (i < n16)
                        dst[i] = x[j];
                    else if (i < n16 + c16)
                        cdst[i - n16] = x[j];
                    else if (i < tot)
                        rdst[i - n16 - c16] = x[j];
                }
            }
        }
        __syncthreads();
        // (b) base values, lists of this election (gen), core marks: kU slots per lane per batch,
        // all their loads in flight before the first is used
        constexpr int kU = 4;
        for (int l0 = 0; l0 < nr; l0 += 64 * kU) {
            int32_t v[kU], lv[kU];
            uint32_t mk[kU], gc[kU], gp[kU];
            ulonglong2 w[kU][R / 2];
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int l = l0 + lane + 64 * j;
                v[j] = sA[l < nr ? l : nr - 1];
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                lv[j] = S.L[v[j]];
                mk[j] = S.gmark[v[j]];
                gc[j] = S.gchg[v[j]];
                gp[j] = S.gpull[v[j]];
                const ulonglong2 *g = reinterpret_cast<const ulonglong2 *>(S.glist + size_t(v[j]) * R);
#pragma unroll
                for (int i = 0; i < R / 2; ++i) w[j][i] = g[i];
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int l = l0 + lane + 64 * j;
                if (l >= nr) break;
                sL[l] = lv[j];
                int c = 0;
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const unsigned long long x = (i & 1) ? w[j][i >> 1].y : w[j][i >> 1].x;
                    const uint32_t hi = uint32_t(x >> 32);
                    if ((hi >> kRecDBits) == S.gen && (hi & kRecDMask) != 0) {
                        sE[l * R + c] = (static_cast<unsigned long long>(hi & kRecDMask) << 32) | (x & 0xffffffffull);
                        ++c;
                    }
                }
                sN[l] = uint8_t(c);
                sMaxV[l] = c ? rval(sE[l * R + c - 1]) : lv[j];
                // a change in launch kc (any level: 0xFFF), a pull in launch kp (level 0)
                sChg[l] = (gc[j] >> kRecDBits) == S.gen ? ((gc[j] & kRecDMask) << 12) | 0xFFFu : 0u;
                sRing[l] = 0;
                if (l < m) {
                    const bool marked = mk[j] >= tgk;
                    sMark[l] = marked ? 1u : 0u;
                    // unmarked: consistent with every neighbour as loaded -> only this launch's changes
                    sLast[l] = marked ? ((gp[j] >> kRecDBits) == S.gen ? (gp[j] & kRecDMask) << 12 : 0u)
                                      : (uint32_t(k) << 12) | 1u;
                    sDirty[l] = 0;
                }
            }
        }
        my_load += uint64_t(nr);
        __syncthreads();
        const unsigned long long w1 = wall_clock64();
        // (c) levels: the queued core agents pull from the neighbours that changed since their last
        // pull (every neighbour the first time); a change queues the agent's core neighbours for the
        // next level (in place: a reader sees each entry whole, old or new, and every change
        // re-queues its readers)
        {
            int total = 0;  // level 1's queue: the agents marked from outside
            for (int j0 = 0; j0 < m; j0 += 64) {
                const int l = j0 + lane;
                const bool f = l < m && sMark[l] != 0;
                const unsigned long long b = __ballot(f);
                if (f) sList[0][total + int(__popcll(b & ((1ull << lane) - 1ull)))] = uint16_t(l);
                total += int(__popcll(b));
            }
            if (lane == 0) sCnt[0] = total;
        }
        __syncthreads();
        int lev = 0, cur = 0;
        for (;;) {
            const int total = sCnt[cur];
            if (total == 0) break;
            if (++lev > kRLevelCap) {
                if (lane == 0) atomicOr(S.err, 4u);
                break;
            }
            if (lane == 0) sCnt[cur ^ 1] = 0;
            __syncthreads();
            my_rec += uint64_t(total);
            for (int i = lane; i < total; i += 64) {
                const int l = sList[cur][i];
                sMark[l] = 0u;
                const int32_t base = sL[l];
                OwnList<R> ol;
                ol.load(&sE[l * R], sN[l]);
                const uint32_t since = sLast[l];
                const uint32_t now = (uint32_t(k) << 12) | uint32_t(lev);
                sLast[l] = now;
                bool changed = false, defer = false, ovf = false;
                const int eb = sRow[l], ee = sRow[l + 1];
                // one copy of the candidate code, not unrolled (an unrolled 8 x 8 nest of inlined
                // inserts made the kernel ~200 KB of code); a neighbour's records are loaded at once
                // and walked in registers (no LDS round trip per record); a neighbour whose largest
                // value does not beat this agent's value after one round offers nothing
                const int32_t v1 = ol.at(1, base);
#pragma unroll 1
                for (int e = eb; e < ee; ++e) {
                    const int u = sCol[e];
                    if (sChg[u] < since || sMaxV[u] <= v1) continue;
                    const int nu = sN[u];
                    const ulonglong2 *pu = reinterpret_cast<const ulonglong2 *>(&sE[u * R]);
                    unsigned long long x[R];
#pragma unroll
                    for (int q = 0; q < R / 2; ++q) {
                        const ulonglong2 w = pu[q];
                        x[2 * q] = w.x;
                        x[2 * q + 1] = w.y;
                    }
                    int dd = 1;
                    int32_t val = sL[u];
#pragma unroll 1
                    for (int q = -1; q < nu; ++q) {
                        if (q >= 0) {
                            dd = rdist(x[0]) + 1;
                            val = rval(x[0]);
#pragma unroll
                            for (int t = 0; t + 1 < R; ++t) x[t] = x[t + 1];  // next record to the front
                        }
                        if (dd > dcap || val <= ol.at(dd, base)) continue;
                        if (dd > W) {  // beyond this launch's window: next launch
                            defer = true;
                            continue;
                        }
                        if (ol.insert(dd, val))
                            changed = true;
                        else
                            ovf = true;
                    }
                }
                if (ovf) atomicOr(S.err, 2u);
                if (changed) {
                    ol.store(&sE[l * R]);
                    sN[l] = uint8_t(ol.n);
                    sMaxV[l] = ol.at(INT_MAX - 1, base);
                    sChg[l] = now;
#pragma unroll 1
                    for (int e0 = eb; e0 < ee; e0 += 8) {  // queue the core neighbours, 8 at a time
                        int u[8];
                        unsigned old[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) u[j] = sCol[e0 + j < ee ? e0 + j : ee - 1];
#pragma unroll
                        for (int j = 0; j < 8; ++j) old[j] = (e0 + j < ee && u[j] < m) ? atomicOr(&sMark[u[j]], 1u) : 1u;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (e0 + j < ee && u[j] >= m) sRing[u[j]] = 1;  // a ring agent: flagged below
                            if (old[j] == 0u) sList[cur ^ 1][atomicAdd(&sCnt[cur ^ 1], 1)] = uint16_t(u[j]);
                        }
                    }
                }
                // pulled; changed; deferred (its next pull must see every neighbour again)
                sDirty[l] |= uint8_t(2 | (changed ? 1 : 0) | (defer ? 4 : 0));
                if (defer) {  // a record beyond the window: this agent again next launch
                    S.gmark[sA[l]] = tg1;
                    sDefer = 1;
                }
            }
            __syncthreads();
            cur ^= 1;
        }
        my_lev += uint64_t(lev);
        const unsigned long long w2 = wall_clock64();
        // ring agents next to a change: marked for the next launch, their tiles flagged (once per
        // activation, all lanes' flags at once: a flag is a returning atomic round trip)
        for (int l = m + lane; l < nr; l += 64) {
            if (!sRing[l]) continue;
            const int32_t vu = sA[l];
            S.gmark[vu] = tg1;
            flag_tile(S, tile_of_cell(S.acell[vu], S.ncx, S.ntx), tg1, k + 1);
        }
        if (sDefer && lane == 0) flag_tile(S, tile, tg1, k + 1);
        // (d) changed core lists back to HBM, whole entries, tagged with this election's gen
        for (int l = lane; l < m; l += 64) {
            const int dirty = sDirty[l];
            if (!dirty) continue;
            const int32_t va = sA[l];
            S.gpull[va] = (dirty & 4) ? 0u : tgk;
            if (!(dirty & 1)) continue;
            S.gchg[va] = tgk;
            const int n = sN[l];
            ulonglong2 *g = reinterpret_cast<ulonglong2 *>(S.glist + size_t(va) * R);
#pragma unroll
            for (int i = 0; i < R / 2; ++i) {
                const unsigned long long x0 = 2 * i < n ? sE[l * R + 2 * i] | (static_cast<unsigned long long>(genhi) << 32) : 0ull;
                const unsigned long long x1 =
                    2 * i + 1 < n ? sE[l * R + 2 * i + 1] | (static_cast<unsigned long long>(genhi) << 32) : 0ull;
                g[i] = ulonglong2{x0, x1};
            }
        }
        __syncthreads();  // LDS reused by the next tile
        const unsigned long long w3 = wall_clock64();
        c_load += w1 - w0;
        c_lev += w2 - w1;
        c_end += w3 - w2;
    }
    if (lane == 0 && my_act) {
        atomicAdd(&S.stats[0], my_act);
        atomicAdd(&S.stats[1], my_lev);
        atomicAdd(&S.stats[2], my_rec);
        atomicAdd(&S.stats[3], my_load);
        atomicAdd(&S.stats[4], c_load);  // wall_clock64 ticks (100 MHz) per phase, summed over activations
        atomicAdd(&S.stats[5], c_lev);
        atomicAdd(&S.stats[6], c_end);

    }
}

// Leaders after round T0 + dcap (the last record with d <= dcap), histogram of the records' d
// (changes of round T0 + d), the largest d.
// L and out may be the same buffer (each thread reads its agent's base before writing it).
template <int R>
__global__ __launch_bounds__(kBlock) void k_rec_final(int64_t n, const int32_t *L,
                                                     const unsigned long long *__restrict__ glist, uint32_t gen,
                                                     int dcap, int32_t *out,
                                                     unsigned long long *__restrict__ hist, int hist_len,
                                                     unsigned *__restrict__ dmax) {
    __shared__ unsigned s_h[kRHist];
    for (int i = threadIdx.x; i < kRHist; i += kBlock) s_h[i] = 0;
    __syncthreads();
    unsigned md = 0;
    for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < n; v += int64_t(gridDim.x) * kBlock) {
        int32_t best = L[v];
        const ulonglong2 *g = reinterpret_cast<const ulonglong2 *>(glist + size_t(v) * R);
        unsigned long long e[R];
#pragma unroll
        for (int i = 0; i < R / 2; ++i) {
            const ulonglong2 w = g[i];
            e[2 * i] = w.x;
            e[2 * i + 1] = w.y;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const uint32_t hi = uint32_t(e[i] >> 32);
            const int d = int(hi & kRecDMask);
            if ((hi >> kRecDBits) != gen || d == 0 || d > dcap) continue;
            const int32_t val = int32_t(uint32_t(e[i]));
            best = val > best ? val : best;
            md = unsigned(d) > md ? unsigned(d) : md;
            if (d < kRHist)
                atomicAdd(&s_h[d], 1u);
            else if (d < hist_len)
                atomicAdd(&hist[d], 1ull);
        }
        out[v] = best;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned y = __shfl_xor(md, o, 64);
        md = y > md ? y : md;
    }
    if ((threadIdx.x & 63) == 0 && md) atomicMax(dmax, md);
    __syncthreads();
    for (int i = threadIdx.x; i < kRHist && i < hist_len; i += kBlock)
        if (s_h[i]) atomicAdd(&hist[i], (unsigned long long)s_h[i]);
}

// Index blob layout (swarm_record_index_bytes): ra, re, rs, rq (ntiles + 1 int32 each), rrow (u16),
// rcol (u16), ragent (int32), each section 256-byte aligned.
struct IxSizes {
    size_t ra, rrow, rcol, ragent, total;
};

IxSizes ix_sizes(int64_t n, int64_t e, int64_t ntiles) {
    auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
    IxSizes z{};
    z.ra = up(size_t(ntiles + 1) * 4);
    z.rrow = up(size_t(n + 8 * ntiles + 8) * 2);
    z.rcol = up(size_t(e + 8 * ntiles + 8) * 2);
    // region slots: every agent is in its own tile's core and in the rings of at most 3 more
    z.ragent = up(size_t(4 * n + 4 * ntiles + 4) * 4);
    z.total = 4 * z.ra + z.rrow + z.rcol + z.ragent;
    return z;
}

RecIndex ix_view(void *index, int64_t n, int64_t e, int64_t ntiles) {
    const IxSizes z = ix_sizes(n, e, ntiles);
    char *p = static_cast<char *>(index);
    RecIndex ix{};
    ix.ra = reinterpret_cast<int32_t *>(p);
    ix.re = reinterpret_cast<int32_t *>(p + z.ra);
    ix.rs = reinterpret_cast<int32_t *>(p + 2 * z.ra);
    ix.rq = reinterpret_cast<int32_t *>(p + 3 * z.ra);
    ix.rrow = reinterpret_cast<uint16_t *>(p + 4 * z.ra);
    ix.rcol = reinterpret_cast<uint16_t *>(p + 4 * z.ra + z.rrow);
    ix.ragent = reinterpret_cast<int32_t *>(p + 4 * z.ra + z.rrow + z.rcol);
    return ix;
}

}  // namespace

int64_t rec_ntiles(int64_t ncx, int64_t ncy) { return ((ncx + kRT - 1) / kRT) * ((ncy + kRT - 1) / kRT); }

RecGeom rec_geom(int64_t ncx, int64_t ncy) {
    return RecGeom{ncx, ncy, (ncx + kRT - 1) / kRT, (ncy + kRT - 1) / kRT};
}

int rec_index_view(const void *index, int64_t n, int64_t e, int64_t ncx, int64_t ncy, RecIndex *out) {
    *out = ix_view(const_cast<void *>(index), n, e, rec_ntiles(ncx, ncy));
    return SWARM_OK;
}

// ------------------------------------------------------------------ tail driver
int rec_tail_prepare(swarm_ctx *ctx, RecTail *rt, hipStream_t s) {
    const int64_t n = rt->n, ntiles = rec_ntiles(rt->ncx, rt->ncy);
    rt->ntiles = ntiles;
    const size_t lbytes = size_t(n) * kRR * 8;
    void *old_list = ctx->slot[S_REC_LIST], *old_mark = ctx->slot[S_REC_MARK];
    unsigned long long *glist;
    SW_ALLOC(glist, ctx, S_REC_LIST, lbytes);
    const size_t mbytes = size_t(n) * 12 + size_t(ntiles) * 4 * 3 + size_t(kRecMaxLaunch + 2) * 4 + 64 * 8 + 256;
    char *mb;
    SW_ALLOC(mb, ctx, S_REC_MARK, mbytes);
    const bool fresh = glist != old_list || static_cast<void *>(mb) != old_mark || ctx->rec_gen + 1 >= (1u << kRecGenBits);
    uint32_t *gmark = reinterpret_cast<uint32_t *>(mb);
    uint32_t *gchg = gmark + n, *gpull = gchg + n;
    uint32_t *tflag = gpull + n;
    int32_t *tl0 = reinterpret_cast<int32_t *>(tflag + ntiles);
    int32_t *tl1 = tl0 + ntiles;
    uint32_t *tcnt = reinterpret_cast<uint32_t *>(tl1 + ntiles);
    unsigned long long *misc = reinterpret_cast<unsigned long long *>(
        (reinterpret_cast<uintptr_t>(tcnt + kRecMaxLaunch + 2) + 7) & ~uintptr_t(7));
    if (fresh) {  // a new buffer, or the generations ran out: no stale entry may match the next gen
        SW_HIP(hipMemsetAsync(glist, 0, ctx->cap[S_REC_LIST], s));
        SW_HIP(hipMemsetAsync(mb, 0, ctx->cap[S_REC_MARK], s));
        ctx->rec_gen = 0;
    }
    ctx->rec_gen += 1;
    SW_HIP(hipMemsetAsync(tcnt, 0, size_t(kRecMaxLaunch + 2) * 4 + 64 * 8 + 8, s));
    RecState &S = *reinterpret_cast<RecState *>(rt->state);
    static_assert(sizeof(RecState) <= sizeof(rt->state), "RecTail::state too small");
    S = RecState{};
    S.ix = ix_view(const_cast<void *>(rt->index), n, rt->n_edges, ntiles);
    S.L = rt->L;
    S.glist = glist;
    S.gmark = gmark;
    S.gchg = gchg;
    S.gpull = gpull;
    S.tflag = tflag;
    S.tlist[0] = tl0;
    S.tlist[1] = tl1;
    S.tcnt = tcnt;
    S.err = reinterpret_cast<unsigned *>(misc);         // misc[0]: err (u32), misc[0] hi: dmax
    S.stats = misc + 2;                                  // misc[2..10]
    S.acell = rt->acell;
    S.ncx = rt->ncx;
    S.ntx = (rt->ncx + kRT - 1) / kRT;
    S.gen = ctx->rec_gen;
    rt->gmark = gmark;
    rt->tflag = tflag;
    rt->tlist0 = tl0;
    rt->tlist1 = tl1;
    rt->tcnt = tcnt;
    rt->gen = ctx->rec_gen;
    rt->tag1 = (ctx->rec_gen << kRecDBits) | 1u;
    return SWARM_OK;
}

// Launches until no tile is flagged (or an error: rt->fallback = 1, nothing written), then the
// leaders after round T0 + dcap into `out` and the per-round changes of rounds T0 + 1 ...
int rec_tail_run(swarm_ctx *ctx, RecTail *rt, int32_t *out, hipStream_t s) {
    const RecState &S = *reinterpret_cast<const RecState *>(rt->state);
    const int dcap = rt->max_rounds - rt->T0;  // rounds the tail may still compute
    const int delta = rt->delta > 0 ? rt->delta : 8;
    int dev = 0, ncu = 0;
    SW_HIP(hipGetDevice(&dev));
    SW_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const unsigned grid = unsigned(rt->grid > 0 ? rt->grid : 2 * std::max(ncu, 1));
    uint32_t *h = static_cast<uint32_t *>(pinned(ctx, 64));
    if (!h) return SWARM_ERR_OOM;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (rt->timed) {
        SW_HIP(hipEventCreate(&ev0));
        SW_HIP(hipEventCreate(&ev1));
        SW_HIP(hipEventRecord(ev0, s));
    }
    struct EvFree {
        hipEvent_t a, b;
        ~EvFree() {
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        }
    } evf{ev0, ev1};
    int k = 1, batch = rt->batch > 0 ? rt->batch : 8;
    rt->fallback = 0;
    for (;;) {
        const int kend = std::min(kRecMaxLaunch, k + batch - 1);
        for (int j = k; j <= kend; ++j) {
            const int W = int(std::min<int64_t>(int64_t(j) * delta, dcap));
            hipLaunchKernelGGL(k_rec_tiles<kRR>, dim3(grid), dim3(64), 0, s, S, j, W, dcap);
            SW_LAUNCHED();
        }
        SW_HIP(hipMemcpyAsync(h, S.tcnt + kend + 1, 4, hipMemcpyDeviceToHost, s));
        SW_HIP(hipMemcpyAsync(h + 1, S.err, 4, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        rt->launches = kend;
        if (h[1]) {  // over capacity / overflow: the frontier rounds take over from T0 + 1
            rt->fallback = int(h[1]);
            return SWARM_OK;
        }
        if (h[0] == 0) break;
        if (kend >= kRecMaxLaunch) {
            rt->fallback = 8;
            return SWARM_OK;
        }
        k = kend + 1;
    }
    // the largest d <= dcap is at most launches * delta (a record beyond a launch's window waits)
    const int64_t hlen = std::min<int64_t>(int64_t(dcap), int64_t(rt->launches) * delta) + 1;
    unsigned long long *hist;
    SW_ALLOC(hist, ctx, S_TMP1, size_t(hlen) * 8 + 16);
    unsigned *dmax = reinterpret_cast<unsigned *>(hist + hlen);
    SW_HIP(hipMemsetAsync(hist, 0, size_t(hlen) * 8 + 16, s));
    hipLaunchKernelGGL(k_rec_final<kRR>, dim3(grid_for(rt->n, kBlock, 2048)), dim3(kBlock), 0, s, rt->n, S.L, S.glist,
                       S.gen, dcap, out, hist, int(hlen), dmax);
    SW_LAUNCHED();
    if (rt->timed) SW_HIP(hipEventRecord(ev1, s));
    unsigned long long hs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned hd = 0;
    SW_HIP(hipMemcpyAsync(&hd, dmax, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipMemcpyAsync(hs, S.stats, 80, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    rt->dmax = int(hd);
    rt->hist.assign(size_t(hd) + 1, 0);
    if (hd) {
        std::vector<unsigned long long> tmp(size_t(hd) + 1);
        SW_HIP(hipMemcpy(tmp.data(), hist, (size_t(hd) + 1) * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i <= hd; ++i) rt->hist[i] = int64_t(tmp[i]);
    }
    rt->activations = int64_t(hs[0]);
    rt->levels = int64_t(hs[1]);
    rt->recomputes = int64_t(hs[2]);
    rt->loaded = int64_t(hs[3]);
    if (getenv("SWARM_REC_DEBUG"))
        fprintf(stderr, "record tail: T0 %d launches %lld activations %lld levels %lld recomputes %lld loaded %lld | "
                        "us per activation: load %.2f levels %.2f end %.2f | dmax %d\n", rt->T0, (long long)rt->launches,
                (long long)hs[0], (long long)hs[1], (long long)hs[2], (long long)hs[3],
                hs[0] ? double(hs[4]) / 100.0 / double(hs[0]) : 0.0, hs[0] ? double(hs[5]) / 100.0 / double(hs[0]) : 0.0,
                hs[0] ? double(hs[6]) / 100.0 / double(hs[0]) : 0.0,
                rt->dmax);
    if (rt->timed) {
        float x = 0;
        SW_HIP(hipEventElapsedTime(&x, ev0, ev1));
        rt->ms = x;
    }
    return SWARM_OK;
}

}  // namespace swarm

extern "C" {

int64_t swarm_record_index_bytes(int64_t n, int64_t n_edges, const swarm_grid *grid) {
    using namespace swarm;
    if (!grid || n < 0 || n_edges < 0 || grid->ncx < 1 || grid->ncy < 1) return -1;
    return int64_t(ix_sizes(n, n_edges, rec_ntiles(grid->ncx, grid->ncy)).total);
}

int swarm_record_index(swarm_ctx *ctx, int64_t n, const int32_t *row_ptr, const int32_t *col, const swarm_grid *grid,
                       const uint32_t *cell_off, const int32_t *acell, void *index, int64_t index_bytes, int32_t *ok,
                       void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && grid != nullptr && ok != nullptr, "NULL argument");
    if (!ctx_on_current_device(ctx)) return SWARM_ERR_ARG;
    SW_ARG(n >= 1 && n < (int64_t(1) << 30), "n out of range (1 .. 2^30 - 1)");
    SW_ARG(row_ptr && cell_off && acell && index, "NULL array");
    SW_ARG(grid->ncx >= 1 && grid->ncy >= 1, "bad grid");
    hipStream_t s = static_cast<hipStream_t>(stream);
    *ok = 0;
    int32_t e_total = 0;
    SW_HIP(hipMemcpyAsync(&e_total, row_ptr + n, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    SW_ARG(e_total == 0 || col != nullptr, "col is NULL but the graph has edges");
    const int64_t ntiles = rec_ntiles(grid->ncx, grid->ncy);
    const IxSizes z = ix_sizes(n, e_total, ntiles);
    SW_ARG(index_bytes >= int64_t(z.total), "index smaller than swarm_record_index_bytes()");
    const RecGeom g = rec_geom(grid->ncx, grid->ncy);
    const RecIndex ix = ix_view(index, n, e_total, ntiles);
    // counts (4 x (ntiles + 1), the last of each 0) + error word
    int32_t *cnt;
    SW_ALLOC(cnt, ctx, S_TMP0, size_t(4 * (ntiles + 1)) * 4 + 16);
    unsigned *err = reinterpret_cast<unsigned *>(cnt + 4 * (ntiles + 1));
    SW_HIP(hipMemsetAsync(cnt, 0, size_t(4 * (ntiles + 1)) * 4 + 16, s));
    const unsigned tg = unsigned(std::min<int64_t>(ntiles, 65535));
    hipLaunchKernelGGL(k_ri_count, dim3(tg), dim3(64), 0, s, cell_off, row_ptr, g, cnt, err);
    SW_LAUNCHED();
    int32_t *outs[4] = {ix.ra, ix.re, ix.rs, ix.rq};
    size_t tmp_bytes = 0;
    SW_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, ix.ra, int(ntiles + 1), s));
    void *tmp;
    SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
    for (int i = 0; i < 4; ++i)
        SW_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt + i * (ntiles + 1), outs[i], int(ntiles + 1), s));
    int32_t tot[4] = {0, 0, 0, 0};
    unsigned herr = 0;
    for (int i = 0; i < 4; ++i) SW_HIP(hipMemcpyAsync(&tot[i], outs[i] + ntiles, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    if (herr) return SWARM_OK;  // a tile over the on-chip capacity: *ok = 0
    // the sections hold what the counts need (bounds of ix_sizes)
    SW_ARG(int64_t(tot[0]) == n, "cell_off does not cover the n agents (the index of another swarm?)");
    if (size_t(tot[1]) * 2 > z.rcol || size_t(tot[2]) * 4 > z.ragent || size_t(tot[3]) * 2 > z.rrow) return SWARM_OK;
    hipLaunchKernelGGL(k_ri_fill, dim3(tg), dim3(64), 0, s, cell_off, row_ptr, col, acell, g, ix, err);
    SW_LAUNCHED();
    SW_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    *ok = herr == 0 ? 1 : 0;
    return SWARM_OK;
}

}  // extern "C"
