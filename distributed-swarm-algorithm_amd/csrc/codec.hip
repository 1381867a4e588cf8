// Batched wire codec on gfx950.
//
// The reference's transport seam frames every message as a big-endian '!BBI' header (type u8,
// sender u8, tick u32; agent.py:184-186) followed by a type-specific payload -- HEARTBEAT
// '!ff' leader position (agent.py:283-289), ELECTION_ACCLAIM '!B' own ID (agent.py:240),
// COORDINATOR none (241), TASK_CLAIM '!If' task + utility (302), TASK_CONFLICT '!IB' task +
// winner (322, 325) -- and parses inbound packets in on_message_received (agent.py:197-214).
// These kernels do both for a whole batch of messages (one thread per message / packet; a
// byte-moving, HBM-bound job: no arithmetic worth the name):
//   encode  one pass (k_enc_one below): a workgroup per tile of 2 048 messages reads the fields once,
//           computes status + length, finds the tile's byte offset by a decoupled look-back over the
//           lower tiles' published counts, and stores packets, status and offsets (the three-launch
//           tile / base / place form stays as SWARM_ENC_PASSES=3).  Errors as the reference raises them, payload
//           first (it packs the payload before _send_msg packs the header): an out-of-range
//           integer field -> struct.error (status 1), a finite value beyond the f32 range ->
//           OverflowError (status 2); an unknown type -> status 3.  Errored messages take no
//           bytes.  wide = 1 widens the u8 ID fields to u32 ('!BII' header, '!I' acclaim,
//           '!II' conflict) for swarms with IDs > 255 (an extension: the reference cannot
//           frame them).
//   decode  per packet, the reference's dispatch: shorter than the header -> dropped (1);
//           unknown type -> ignored (2); TASK_CLAIM / TASK_CONFLICT whose payload is not
//           exactly '!If' / '!IB' sized -> the handler's struct.unpack raises (3); a HEARTBEAT
//           payload carries a position only when it is exactly 8 bytes (agent.py:256-258).
//           A packet whose offsets fall outside [0, buf_len] or run backwards is not read
//           (status 4).
#include <cmath>

#include "swarm_common.h"

namespace swarm {
namespace {

enum : int { T_HB = 1, T_ACCLAIM = 2, T_COORD = 3, T_CLAIM = 4, T_CONFLICT = 5 };

__device__ __forceinline__ bool u8_ok(int64_t v) { return v >= 0 && v <= 0xFF; }
__device__ __forceinline__ bool u32_ok(int64_t v) { return v >= 0 && v <= 0xFFFFFFFFll; }
__device__ __forceinline__ bool f32_ok(double v) { return !std::isfinite(v) || std::isfinite(float(v)); }

// Status (0 ok, 1 struct.error, 2 OverflowError, 3 unknown type) and packet length.
__device__ __forceinline__ int enc_status(int64_t ty, int64_t snd, int64_t tick, double a, double b, int64_t task,
                                          int64_t win, int wide, int *len) {
    const int hdr = wide ? 9 : 6;
    const auto id_ok = [wide](int64_t v) { return wide ? u32_ok(v) : u8_ok(v); };  // (a function pointer here
    // compiled to an indirect call: SGPR spills and no inlining in the encode kernels)
    int st = 0, pl = 0;
    switch (int(ty)) {
        case T_HB:  // payload '!ff' first
            if (!f32_ok(a) || !f32_ok(b)) st = 2;
            pl = 8;
            break;
        case T_ACCLAIM:
            if (!id_ok(snd)) st = 1;
            pl = wide ? 4 : 1;
            break;
        case T_COORD:
            break;
        case T_CLAIM:
            if (!u32_ok(task)) st = 1;
            else if (!f32_ok(a)) st = 2;
            pl = 8;
            break;
        case T_CONFLICT:
            if (!u32_ok(task) || !id_ok(win)) st = 1;
            pl = wide ? 8 : 5;
            break;
        default:
            st = 3;
    }
    if (st == 0 && (!u8_ok(ty) || !id_ok(snd) || !u32_ok(tick))) st = 1;  // then the header
    *len = st ? 0 : hdr + pl;
    return st;
}

__device__ __forceinline__ void put_u32(uint8_t *p, uint32_t v) {
    p[0] = uint8_t(v >> 24);
    p[1] = uint8_t(v >> 16);
    p[2] = uint8_t(v >> 8);
    p[3] = uint8_t(v);
}

__device__ __forceinline__ uint32_t get_u32(const uint8_t *p) {
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

struct EncIn {
    const int64_t *type, *sender, *tick, *task, *winner;
    const double *a, *b;
};

// Packet bytes of one message (status 0) at p, from its fields in registers.
__device__ __forceinline__ void write_packet(uint8_t *p, int ty, int64_t snd, int64_t tick, double a, double b,
                                             int64_t task, int64_t win, int wide) {
    p[0] = uint8_t(ty);
    int h;
    if (wide) {
        put_u32(p + 1, uint32_t(snd));
        put_u32(p + 5, uint32_t(tick));
        h = 9;
    } else {
        p[1] = uint8_t(snd);
        put_u32(p + 2, uint32_t(tick));
        h = 6;
    }
    p += h;
    switch (ty) {
        case T_HB:
            put_u32(p, __float_as_uint(float(a)));
            put_u32(p + 4, __float_as_uint(float(b)));
            break;
        case T_ACCLAIM:
            if (wide) put_u32(p, uint32_t(snd));
            else p[0] = uint8_t(snd);
            break;
        case T_CLAIM:
            put_u32(p, uint32_t(task));
            put_u32(p + 4, __float_as_uint(float(a)));
            break;
        case T_CONFLICT:
            put_u32(p, uint32_t(task));
            if (wide) put_u32(p + 4, uint32_t(win));
            else p[4] = uint8_t(win);
            break;
        default:
            break;
    }
}

// The same bytes from the fields already narrowed to their wire types (status 0: every value in range).
__device__ __forceinline__ void write_packet_n(uint8_t *p, int ty, uint32_t snd, uint32_t tick, float a, float b,
                                               uint32_t task, uint32_t win, int wide) {
    p[0] = uint8_t(ty);
    int h;
    if (wide) {
        put_u32(p + 1, snd);
        put_u32(p + 5, tick);
        h = 9;
    } else {
        p[1] = uint8_t(snd);
        put_u32(p + 2, tick);
        h = 6;
    }
    p += h;
    switch (ty) {
        case T_HB:
            put_u32(p, __float_as_uint(a));
            put_u32(p + 4, __float_as_uint(b));
            break;
        case T_ACCLAIM:
            if (wide) put_u32(p, snd);
            else p[0] = uint8_t(snd);
            break;
        case T_CLAIM:
            put_u32(p, task);
            put_u32(p + 4, __float_as_uint(a));
            break;
        case T_CONFLICT:
            put_u32(p, task);
            if (wide) put_u32(p + 4, win);
            else p[4] = uint8_t(win);
            break;
        default:
            break;
    }
}

// Encode in tiles (round 5): every field is read ONCE.
//   k_enc_tile   a workgroup per tile of kTile messages, each wave its own 512 consecutive ones: status
//                and length per message (8 slabs of 64, a wave scan each -- no workgroup barrier), the
//                packets assembled in the wave's LDS region at wave-relative offsets, then each wave's
//                packed bytes stored to its scratch segment (16-byte stores), the wave totals, and each
//                message's tile-relative offset (u16) once the tile's wave offsets are known;
//   k_enc_base   one workgroup: exclusive scan of the tile totals -> each tile's base, the total;
//   k_enc_place  a workgroup per tile: the four wave segments staged in LDS at their tile offsets and the
//                output's 16-byte phase, stored at base (16-byte stores, partial head / tail bytewise),
//                and the int64 offsets base + local.
// Per message: fields 56 B read once, status 1 B, local offset 2 + 2 B, the packet 3 x ~10 B (scratch
// write, scratch read, output), offsets 8 B.  (Rounds 1-4: k_enc_len + hipCUB scan + host sync +
// k_enc_write, the fields read twice: 0.40 ms at 10M messages.  A single kernel with a decoupled
// look-back over 1 024-message chunks: 0.43 ms, the look-back chain the bound.  Round 5's first tiled
// form scanned each 256-message slab across the workgroup, 16 barriers per tile: 0.338 ms.)
#ifndef SWARM_ENC_TILEJ
#define SWARM_ENC_TILEJ 4  // slabs of 64 per wave (A/B builds: -DSWARM_ENC_TILEJ=8, tools/build_variant.sh; profiles/r5/ab_r5g.log)
#endif
#ifndef SWARM_ENC_BLOCK
#define SWARM_ENC_BLOCK 512  // threads per encode workgroup: 8 waves, 2 048-message tiles (A/B: -DSWARM_ENC_BLOCK=256)
#endif
constexpr int kEB = SWARM_ENC_BLOCK;
constexpr int kTileJ = SWARM_ENC_TILEJ, kTile = kEB * kTileJ, kMaxPkt = 17;
constexpr int kWaveMsgs = kWave * kTileJ;                // 256 consecutive messages per wave (kTileJ 4)
constexpr int kWaveBytes = kWaveMsgs * kMaxPkt;          // 4 352: its LDS region and scratch segment
constexpr int kTileBytes = kTile * kMaxPkt;              // scratch bytes per tile (wide worst case)
constexpr int kTileLds = (kTileBytes + 16 + 15) / 16;    // uint4 words (+16: the output phase)
constexpr int kWavesT = kEB / kWave;
static_assert(kTileBytes < 65536, "tile-relative packet offsets are u16 (k_enc_tile)");

__global__ __launch_bounds__(kEB) void k_enc_tile(int64_t m, EncIn in, int wide, int8_t *__restrict__ status,
                                                    uint16_t *__restrict__ loc, uint8_t *__restrict__ tmp,
                                                    int32_t *__restrict__ wave_tot) {
    __shared__ uint4 s_buf[kTileLds];
    __shared__ int s_wt[kWavesT];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint8_t *wl = reinterpret_cast<uint8_t *>(s_buf) + w * kWaveBytes;
    const int64_t ntiles = (m + kTile - 1) / kTile;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t c0 = tile * kTile + int64_t(w) * kWaveMsgs;
        int run = 0;  // wave-uniform: bytes of this wave's slabs so far
        int wpos[kTileJ];
#pragma unroll
        for (int j = 0; j < kTileJ; ++j) {
            const int64_t i = c0 + j * kWave + lane;
            const bool ok = i < m;
            const int64_t ty = ok ? in.type[i] : 0, snd = ok ? in.sender[i] : 0, tk = ok ? in.tick[i] : 0;
            const double fa = ok ? in.a[i] : 0.0, fb = ok ? in.b[i] : 0.0;
            const int64_t task = ok ? in.task[i] : 0, win = ok ? in.winner[i] : 0;
            int len = 0;
            const int st = ok ? enc_status(ty, snd, tk, fa, fb, task, win, wide, &len) : 3;
            int total = 0, ex = 0;
#pragma unroll
            for (int b = 0; b < 5; ++b) {  // wave exclusive scan of len (< 32): ballots + mbcnt
                const unsigned long long mk = __ballot((len >> b) & 1);
                ex += int(__builtin_amdgcn_mbcnt_hi(uint32_t(mk >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mk), 0u))) << b;
                total += __popcll(mk) << b;
            }
            wpos[j] = run + ex;
            if (ok) {
                status[i] = int8_t(st);
                if (st == 0) write_packet(wl + run + ex, int(ty), snd, tk, fa, fb, task, win, wide);
            }
            run += total;
        }
        __builtin_amdgcn_wave_barrier();  // the wave's packets are in its LDS region
        uint4 *dst = reinterpret_cast<uint4 *>(tmp + tile * int64_t(kTileBytes) + w * kWaveBytes);
        const uint4 *src = reinterpret_cast<const uint4 *>(wl);
        for (int q = lane; q < (run + 15) / 16; q += kWave) dst[q] = src[q];
        if (lane == 0) {
            s_wt[w] = run;
            wave_tot[tile * kWavesT + w] = run;
        }
        __syncthreads();
        int wo = 0;
#pragma unroll
        for (int q = 0; q < kWavesT; ++q) wo += q < w ? s_wt[q] : 0;
#pragma unroll
        for (int j = 0; j < kTileJ; ++j) {
            const int64_t i = c0 + j * kWave + lane;
            if (i < m) loc[i] = uint16_t(wo + wpos[j]);
        }
        __syncthreads();  // s_buf / s_wt reused by the next tile
    }
}

// Exclusive scan of the tile totals (one workgroup; a tile's total = its waves'): base[t], base[ntiles] = all.
__global__ __launch_bounds__(1024) void k_enc_base(int64_t ntiles, const int32_t *__restrict__ wave_tot,
                                                  int64_t *__restrict__ base) {
    __shared__ int64_t s_part[1024];
    auto tot = [&](int64_t q) {
        int64_t v = 0;
#pragma unroll
        for (int w = 0; w < kWavesT; ++w) v += wave_tot[q * kWavesT + w];
        return v;
    };
    const int64_t per = (ntiles + 1023) / 1024, b = int64_t(threadIdx.x) * per;
    int64_t sum = 0;
    for (int64_t q = b; q < b + per && q < ntiles; ++q) sum += tot(q);
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan of the 1 024 parts
        const int64_t v = threadIdx.x >= unsigned(off) ? s_part[threadIdx.x - off] : 0;
        __syncthreads();
        s_part[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t run = threadIdx.x ? s_part[threadIdx.x - 1] : 0;
    for (int64_t q = b; q < b + per && q < ntiles; ++q) {
        base[q] = run;
        run += tot(q);
    }
    if (threadIdx.x == 1023) base[ntiles] = s_part[1023];
}

__global__ __launch_bounds__(kEB) void k_enc_place(int64_t m, const uint8_t *__restrict__ tmp,
                                                     const int32_t *__restrict__ wave_tot,
                                                     const int64_t *__restrict__ base_of,
                                                     const uint16_t *__restrict__ loc, int64_t cap,
                                                     int64_t *__restrict__ off, uint8_t *__restrict__ out,
                                                     unsigned *__restrict__ err) {
    __shared__ uint4 s_buf[kTileLds];
    uint8_t *lb = reinterpret_cast<uint8_t *>(s_buf);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int64_t ntiles = (m + kTile - 1) / kTile;
    if (base_of[ntiles] > cap) {  // the caller's buffer is too small: nothing is written
        if (blockIdx.x == 0 && threadIdx.x == 0) *err = 1u;
        return;
    }
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t c0 = tile * kTile, base = base_of[tile];
        int wo = 0, n = 0, mine = 0;
#pragma unroll
        for (int q = 0; q < kWavesT; ++q) {
            const int v = wave_tot[tile * kWavesT + q];
            wo += q < w ? v : 0;
            mine = q == w ? v : mine;
            n += v;
        }
        // LDS byte ph + x holds out[base + x] (ph: the output's 16-byte phase); wave w stages its segment
        const int ph = int(base & 15);
        const uint4 *src = reinterpret_cast<const uint4 *>(tmp + tile * int64_t(kTileBytes) + w * kWaveBytes);
        for (int q = lane; q < (mine + 15) / 16; q += kWave) {
            const uint4 v4 = src[q];
            const uint32_t v[4] = {v4.x, v4.y, v4.z, v4.w};
            const int lim = mine - 16 * q < 16 ? mine - 16 * q : 16;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < lim) lb[ph + wo + 16 * q + k] = uint8_t(v[k >> 2] >> (8 * (k & 3)));
        }
#pragma unroll 4
        for (int j = 0; j < kTileJ; ++j) {
            const int64_t i = c0 + j * kEB + threadIdx.x;
            if (i < m) off[i] = base + loc[i];
        }
        __syncthreads();
        const int64_t end = base + n, abase = base - ph;
        const int64_t A = (base + 15) & ~int64_t(15), B = end & ~int64_t(15);
        if (A >= B) {
            for (int64_t x = base + threadIdx.x; x < end; x += kEB) out[x] = lb[x - abase];
        } else {
            if (threadIdx.x < A - base) out[base + threadIdx.x] = lb[base + threadIdx.x - abase];
            if (threadIdx.x < end - B) out[B + threadIdx.x] = lb[B + threadIdx.x - abase];
            uint4 *dst = reinterpret_cast<uint4 *>(out + A);
            const uint4 *sb = s_buf + (A - abase) / 16;
            for (int64_t q = threadIdx.x; q < (B - A) / 16; q += kEB) dst[q] = sb[q];
        }
        __syncthreads();  // s_buf reused by the next tile
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) off[m] = base_of[ntiles];
}

// One-pass encode (round 5): a workgroup per tile, the tile's base by a decoupled look-back.
// The tile comes from a ticket (an atomic counter, reset by the workgroup that draws the last one), so
// every lower tile belongs to a workgroup that is already running and publishes its byte count without
// waiting for anything: the look-back always ends.
// A tile's word, one 8-byte agent-scope atomic (no other data is handed over, so no fence):
//   bits 63..40 epoch (the call), 39..38 state (1 = this tile's count, 2 = inclusive prefix), 37..0 value.
// Order inside a workgroup: fields -> status + lengths (wave scans) -> the tile count published -> the
// packets assembled in LDS at tile offsets (the fields narrowed to wire types, then dead) -> wave 0 walks
// back while the others wait -> offsets, and the packets stored with 16-byte stores shifted to the output's
// byte phase.  Per message the compulsory bytes only: fields once, status, the int64 offset, the packet
// (PMC 760 MB at 10M messages against 754 MB compulsory, profiles/r5/codec_*).
// Measured and kept at their defaults (profiles/r5/ab_r5k.log, ab_r5l.log, 10M messages): one look-back
// word per lane and poll -- 4 or 8 (wider windows, contiguous or strided) were slower, 0.255-0.34 ms per
// call against 0.218, each poll's extra agent-coherent loads costing more than the round trips they save;
// the sleep between polls (1, 8, 32) makes no difference.  Tiles (ab_r5m.log, ab_r5n.log): 2 048 messages
// on 8 waves 0.201-0.204 ms, 1 024 on 4 (or on 8) 0.217-0.219, 4 096 on 16 0.207, 512 on 4 0.29.
#ifndef SWARM_ENC_LB_PER
#define SWARM_ENC_LB_PER 1  // look-back words per lane and poll (A/B builds: -DSWARM_ENC_LB_PER=4)
#endif
#ifndef SWARM_ENC_LB_SLEEP
#define SWARM_ENC_LB_SLEEP 1  // s_sleep between polls (units of 64 cycles)
#endif
constexpr int kLbShift = 40, kLbStateShift = 38, kLbPer = SWARM_ENC_LB_PER;
constexpr unsigned kLbMaxPolls = 1u << 22;  // seconds of polling: only a broken call gets there
constexpr unsigned long long kLbValue = (1ull << kLbStateShift) - 1;

__device__ __forceinline__ unsigned long long lb_word(uint32_t epoch, unsigned state, unsigned long long v) {
    return (static_cast<unsigned long long>(epoch) << kLbShift) |
           (static_cast<unsigned long long>(state) << kLbStateShift) | v;
}

// P consecutive messages per lane and slab (P = 2: 16-byte field loads and offset stores, for 16-byte
// aligned arrays; the 8-byte accesses of P = 1 move data at ~0.6x the 16-byte rate).
#ifdef SWARM_ENC_WPE  // A/B builds: a minimum of waves per SIMD for the one-pass kernel
#define SWARM_ENC_ATTR __attribute__((amdgpu_waves_per_eu(SWARM_ENC_WPE)))
#else
#define SWARM_ENC_ATTR
#endif
template <int P>
__global__ __launch_bounds__(kEB) SWARM_ENC_ATTR void k_enc_one(int64_t m, EncIn in, int wide, int8_t *__restrict__ status,
                                                   int64_t *__restrict__ off, uint8_t *__restrict__ out, int64_t cap,
                                                   unsigned long long *__restrict__ lb, uint32_t epoch,
                                                   int64_t *__restrict__ total,
                                                   unsigned *__restrict__ err, unsigned *__restrict__ fail) {
    constexpr int J = kTileJ / P;  // slabs per wave, kWave * P messages each
    static_assert(J * P == kTileJ, "slabs");
    __shared__ uint4 s_buf[kTileLds];
    __shared__ int s_wt[kWavesT];
    __shared__ int64_t s_base;
    __shared__ uint32_t s_tile;
    uint8_t *lbuf = reinterpret_cast<uint8_t *>(s_buf);
    unsigned *ticket = reinterpret_cast<unsigned *>(lb);  // word 0: the ticket counter; words 1.. the tiles
    unsigned long long *word = lb + 1;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int64_t ntiles = (m + kTile - 1) / kTile;
    if (threadIdx.x == 0) {
        const unsigned t = atomicAdd(ticket, 1u);
        if (t == unsigned(ntiles - 1))  // the last ticket: every other one is taken, so reset for the next call
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_tile = t;
    }
    __syncthreads();
    const int64_t tile = s_tile;
    if (tile >= ntiles) {  // only if another call shares this ctx's counter at the same time (not supported)
        if (threadIdx.x == 0) *fail = 2u;
        return;
    }
    const int64_t c0 = tile * kTile + int64_t(w) * kWaveMsgs + int64_t(lane) * P;
    int64_t ty[J][P], snd[J][P], tk[J][P], task[J][P], win[J][P];
    double fa[J][P], fb[J][P];
    int wpos[J][P], st[J][P];
    int run = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t i = c0 + j * kWave * P;
        if (P == 2 && i + 1 < m) {
            const auto l2 = [&](const int64_t *p, int64_t *d) {
                const longlong2 v = *reinterpret_cast<const longlong2 *>(p + i);
                d[0] = v.x;
                d[P - 1] = v.y;
            };
            const auto d2 = [&](const double *p, double *d) {
                const double2 v = *reinterpret_cast<const double2 *>(p + i);
                d[0] = v.x;
                d[P - 1] = v.y;
            };
            l2(in.type, ty[j]);
            l2(in.sender, snd[j]);
            l2(in.tick, tk[j]);
            d2(in.a, fa[j]);
            d2(in.b, fb[j]);
            l2(in.task, task[j]);
            l2(in.winner, win[j]);
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const bool ok = i + k < m;
                ty[j][k] = ok ? in.type[i + k] : 0;
                snd[j][k] = ok ? in.sender[i + k] : 0;
                tk[j][k] = ok ? in.tick[i + k] : 0;
                fa[j][k] = ok ? in.a[i + k] : 0.0;
                fb[j][k] = ok ? in.b[i + k] : 0.0;
                task[j][k] = ok ? in.task[i + k] : 0;
                win[j][k] = ok ? in.winner[i + k] : 0;
            }
        }
    }
    // what the packets need, narrowed once the status is known (the int64 / f64 fields die here: 7 registers
    // per message across the look-back instead of 14)
    uint32_t nty[J][P], nsnd[J][P], ntk[J][P], ntask[J][P], nwin[J][P];
    float nfa[J][P], nfb[J][P];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t i = c0 + j * kWave * P;
        int len = 0;  // the lane's P packets
#pragma unroll
        for (int k = 0; k < P; ++k) {
            int l = 0;
            st[j][k] = i + k < m ? enc_status(ty[j][k], snd[j][k], tk[j][k], fa[j][k], fb[j][k], task[j][k],
                                              win[j][k], wide, &l)
                                 : 3;
            wpos[j][k] = len;
            len += l;
            nty[j][k] = uint32_t(ty[j][k]);
            nsnd[j][k] = uint32_t(snd[j][k]);
            ntk[j][k] = uint32_t(tk[j][k]);
            ntask[j][k] = uint32_t(task[j][k]);
            nwin[j][k] = uint32_t(win[j][k]);
            nfa[j][k] = float(fa[j][k]);
            nfb[j][k] = float(fb[j][k]);
        }
        int tot = 0, ex = 0;
#pragma unroll
        for (int b = 0; b < (P == 1 ? 5 : 6); ++b) {  // wave exclusive scan of len (< 32 P): ballots + mbcnt
            const unsigned long long mk = __ballot((len >> b) & 1);
            ex += int(__builtin_amdgcn_mbcnt_hi(uint32_t(mk >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mk), 0u))) << b;
            tot += __popcll(mk) << b;
        }
#pragma unroll
        for (int k = 0; k < P; ++k) wpos[j][k] += run + ex;
        if (P == 2 && i + 1 < m) {
            *reinterpret_cast<uint16_t *>(status + i) = uint16_t(uint8_t(st[j][0]) | (uint8_t(st[j][P - 1]) << 8));
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k)
                if (i + k < m) status[i + k] = int8_t(st[j][k]);
        }
        run += tot;
    }
    if (lane == 0) s_wt[w] = run;
    __syncthreads();
    int wo = 0, n = 0;
#pragma unroll
    for (int q = 0; q < kWavesT; ++q) {
        wo += q < w ? s_wt[q] : 0;
        n += s_wt[q];
    }
    if (w == 0 && lane == 0)  // this tile's count, before anything else: the look-backs of later tiles wait on it
        __hip_atomic_store(&word[tile], lb_word(epoch, tile ? 1u : 2u, unsigned(n)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (out) {  // the packets into LDS at their tile offsets (16-byte phase 0; the stores below shift them)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int k = 0; k < P; ++k)
                if (st[j][k] == 0)  // (3 beyond m)
                    write_packet_n(lbuf + wo + wpos[j][k], int(nty[j][k]), nsnd[j][k], ntk[j][k], nfa[j][k],
                                   nfb[j][k], ntask[j][k], nwin[j][k], wide);
    }
    if (w == 0) {
        int64_t excl = 0;
        unsigned polls = 0;  // bounded: a walk that never ends (a broken call) gives up and reports it
        // a poll reads tiles j - L - 64 q (lane L, q = 0 .. kLbPer-1): each load instruction covers 64
        // consecutive words (4 lines); the nearest inclusive word ends the walk
        for (int64_t j = tile - 1; j >= 0;) {
            unsigned long long v[kLbPer], incb[kLbPer];
            unsigned okm = 0;  // bit q: word q valid
#pragma unroll
            for (int q = 0; q < kLbPer; ++q) {
                const int64_t k = j - lane - int64_t(kWave) * q;
                v[q] = k >= 0 ? __hip_atomic_load(&word[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : lb_word(epoch, 2u, 0);
            }
#pragma unroll
            for (int q = 0; q < kLbPer; ++q) {
                const unsigned sv = unsigned(v[q] >> kLbStateShift) & 3u;
                const bool valid = uint32_t(v[q] >> kLbShift) == epoch && sv != 0;
                okm |= unsigned(valid) << q;
                incb[q] = __ballot(valid && sv == 2u);
            }
            int qq = kLbPer;  // the first q holding an inclusive word, and its nearest lane p
#pragma unroll
            for (int q = kLbPer - 1; q >= 0; --q)
                if (incb[q]) qq = q;
            const int p = qq < kLbPer ? __ffsll(static_cast<long long>(incb[qq])) - 1 : kWave - 1;
            unsigned needm = 0;
#pragma unroll
            for (int q = 0; q < kLbPer; ++q)
                needm |= unsigned(q < qq || (q == qq && lane <= p)) << q;
            if (__ballot((okm & needm) != needm)) {  // a needed tile has not published yet
                if (++polls > kLbMaxPolls) {
                    if (lane == 0) *fail = 1u;  // (mapped host memory: a plain store, no atomics)
                    break;
                }
                __builtin_amdgcn_s_sleep(SWARM_ENC_LB_SLEEP);
                continue;
            }
            long long add = 0;
#pragma unroll
            for (int q = 0; q < kLbPer; ++q) add += (needm >> q) & 1u ? static_cast<long long>(v[q] & kLbValue) : 0;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) add += __shfl_xor(add, d);
            excl += add;
            if (qq < kLbPer) break;
            j -= int64_t(kWave) * kLbPer;
        }
        if (lane == 0) {
            if (tile) __hip_atomic_store(&word[tile], lb_word(epoch, 2u, static_cast<unsigned long long>(excl + n)),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_base = excl;
            if (tile == ntiles - 1) {
                *total = excl + n;
                off[m] = excl + n;
                *err = out && excl + n > cap ? 1u : 0u;
            }
        }
    }
    __syncthreads();
    const int64_t base = s_base;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t i = c0 + j * kWave * P;
        if (P == 2 && i + 1 < m) {
            *reinterpret_cast<longlong2 *>(off + i) = longlong2{base + wo + wpos[j][0], base + wo + wpos[j][P - 1]};
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k)
                if (i + k < m) off[i + k] = base + wo + wpos[j][k];
        }
    }
    if (!out || base + n > cap) return;  // sizing call, or a buffer too small (err set by the last tile)
    // out[base + x] = lbuf[x]: bytewise head and tail, 16-byte stores between, each composed from five
    // LDS dwords shifted by the tile's byte phase
    const int64_t end = base + n;
    const int64_t A = (base + 15) & ~int64_t(15), B = end & ~int64_t(15);
    if (A >= B) {
        for (int64_t x = base + threadIdx.x; x < end; x += kEB) out[x] = lbuf[x - base];
        return;
    }
    if (threadIdx.x < A - base) out[base + threadIdx.x] = lbuf[threadIdx.x];
    if (threadIdx.x < end - B) out[B + threadIdx.x] = lbuf[B - base + threadIdx.x];
    const int s0 = int(A - base), r = s0 & 3;
    const uint32_t *ld = reinterpret_cast<const uint32_t *>(s_buf) + (s0 >> 2);
    uint4 *dst = reinterpret_cast<uint4 *>(out + A);
    for (int q = threadIdx.x; q < int(B - A) / 16; q += kEB) {
        const uint32_t *d = ld + 4 * q;
        const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
        dst[q] = r == 0 ? uint4{d0, d1, d2, d3}
                        : uint4{__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r),
                                __builtin_amdgcn_alignbyte(d3, d2, r), __builtin_amdgcn_alignbyte(d4, d3, r)};
    }
}

// decode: packets [c0, c0 + kEncPer) per workgroup (LDS staging below)
constexpr int kEncJ = 4, kEncPer = kBlock * kEncJ;
constexpr int kEncLds = (kEncPer * kMaxPkt + 32 + 15) / 16;  // uint4 words

struct DecOut {
    int8_t *status;
    int64_t *type, *sender, *tick, *task, *winner;
    float *a, *b;
    uint8_t *has_pos;
};

// Parse one packet p[0, len) (the dispatch of on_message_received + the handlers' unpack).
__device__ __forceinline__ void parse_packet(const uint8_t *p, int64_t len, bool inside, int wide, int64_t i,
                                             const DecOut &o) {
    const int hdr = wide ? 9 : 6;
    int st = inside ? 1 : 4;
    int64_t ty = 0, snd = 0, tick = 0, task = 0, win = 0;
    float a = 0.f, b = 0.f;
    uint8_t hp = 0;
    if (inside && len >= hdr) {
        ty = p[0];
        snd = wide ? int64_t(get_u32(p + 1)) : int64_t(p[1]);
        tick = int64_t(get_u32(p + (wide ? 5 : 2)));
        const uint8_t *q = p + hdr;
        const int64_t pl = len - hdr;
        st = 0;
        switch (int(ty)) {
            case T_HB:
                if (pl == 8) {
                    a = __uint_as_float(get_u32(q));
                    b = __uint_as_float(get_u32(q + 4));
                    hp = 1;
                }
                break;
            case T_ACCLAIM:
            case T_COORD:
                break;
            case T_CLAIM:
                if (pl == 8) {
                    task = int64_t(get_u32(q));
                    a = __uint_as_float(get_u32(q + 4));
                } else {
                    st = 3;
                }
                break;
            case T_CONFLICT:
                if (pl == (wide ? 8 : 5)) {
                    task = int64_t(get_u32(q));
                    win = wide ? int64_t(get_u32(q + 4)) : int64_t(q[4]);
                } else {
                    st = 3;
                }
                break;
            default:
                st = 2;
        }
    }
    o.status[i] = int8_t(st);
    o.type[i] = (inside && len >= hdr) ? ty : 0;
    o.sender[i] = snd;
    o.tick[i] = tick;
    o.task[i] = task;
    o.winner[i] = win;
    o.a[i] = a;
    o.b[i] = b;
    o.has_pos[i] = hp;
}

// Packets [c0, c0 + kEncPer) per workgroup: when their offsets are in range and their bytes fit,
// the workgroup's contiguous input range is loaded into LDS with 16-byte loads and parsed from
// there; otherwise (malformed offsets, oversized packets) straight from global memory.
__global__ __launch_bounds__(kBlock) void k_decode(int64_t m, const uint8_t *__restrict__ buf, int64_t buf_len,
                                                  const int64_t *__restrict__ off, int wide, DecOut o) {
    __shared__ uint4 s_buf[kEncLds];
    uint8_t *lb = reinterpret_cast<uint8_t *>(s_buf);
    for (int64_t c0 = int64_t(blockIdx.x) * kEncPer; c0 < m; c0 += int64_t(gridDim.x) * kEncPer) {
        const int64_t c1 = c0 + kEncPer < m ? c0 + kEncPer : m;
        const int64_t lo = off[c0], hi = off[c1], alo = lo & ~int64_t(15);
        const bool staged = 0 <= lo && lo <= hi && hi <= buf_len && hi - alo <= int64_t(kEncLds) * 16 &&
                            (reinterpret_cast<uintptr_t>(buf) & 15) == 0;
        if (staged) {  // [alo, A) and [B, hi) bytewise, [A, B) as 16-byte words
            const int64_t A = (lo + 15) & ~int64_t(15), B = hi & ~int64_t(15);
            if (A >= B) {
                for (int64_t x = lo + threadIdx.x; x < hi; x += kBlock) lb[x - alo] = buf[x];
            } else {
                if (threadIdx.x < A - lo) lb[lo + threadIdx.x - alo] = buf[lo + threadIdx.x];
                if (threadIdx.x < hi - B) lb[B + threadIdx.x - alo] = buf[B + threadIdx.x];
                const uint4 *src = reinterpret_cast<const uint4 *>(buf + A);
                for (int64_t q = threadIdx.x; q < (B - A) / 16; q += kBlock) s_buf[(A - alo) / 16 + q] = src[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kEncJ; ++j) {
            const int64_t i = c0 + j * kBlock + threadIdx.x;
            if (i >= c1) continue;
            const int64_t pb = off[i], pe = off[i + 1];
            const bool inside = 0 <= pb && pb <= pe && pe <= buf_len;  // else status 4, nothing read
            const bool in_lds = staged && inside && pb >= lo && pe <= hi;
            const uint8_t *p = in_lds ? lb + (pb - alo) : buf + (inside ? pb : 0);
            parse_packet(p, inside ? pe - pb : 0, inside, wide, i, o);
        }
        __syncthreads();  // s_buf reused by the next chunk
    }
}

}  // namespace
}  // namespace swarm

namespace swarm {
// Grid cap of the codec kernels (10M messages: 16 384 -> encode 0.419-0.433 ms, decode 0.153-0.155;
// 4 096 -> 0.440-0.451 / 0.158-0.162; 1 024 -> 0.484-0.493 / 0.173-0.178, same box,
// profiles/r4_d/physics_codec_grid_ab.log; SWARM_CODEC_WGS overrides, A/B aid).
// Encode form: 1 = one pass (k_enc_one, the default), 3 = tile / base / place (SWARM_ENC_PASSES=3, A/B aid).
int enc_passes() {
    static const int p = [] {
        const char *e = getenv("SWARM_ENC_PASSES");
        return e && atoi(e) == 3 ? 3 : 1;
    }();
    return p;
}

// One-pass encode, two messages per lane when the arrays allow 16-byte accesses (SWARM_ENC_PAIR=0: one, A/B aid).
bool enc_pair() {
    static const bool p = [] {
        const char *e = getenv("SWARM_ENC_PAIR");
        return !(e && atoi(e) == 0);
    }();
    return p;
}

unsigned codec_grid_cap() {
    static const unsigned cap = [] {
        const char *e = getenv("SWARM_CODEC_WGS");
        return e && atoi(e) > 0 ? unsigned(atoi(e)) : 16384u;
    }();
    return cap;
}
}  // namespace swarm

extern "C" {

int swarm_codec_encode(swarm_ctx *ctx, int64_t m, const int64_t *type, const int64_t *sender, const int64_t *tick,
                       const double *a, const double *b, const int64_t *task, const int64_t *winner, int32_t wide,
                       uint8_t *out, int64_t cap, int64_t *offsets, int8_t *status, int64_t *total_bytes,
                       void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && total_bytes != nullptr, "NULL argument");
    SW_ARG(m >= 0 && m < (int64_t(1) << 31), "m out of range");
    SW_ARG(m == 0 || (type && sender && tick && a && b && task && winner && offsets && status), "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    *total_bytes = 0;
    if (m == 0) {
        if (offsets) SW_HIP(hipMemsetAsync(offsets, 0, 8, s));
        return SWARM_OK;
    }
    const EncIn in{type, sender, tick, task, winner, a, b};
    const int64_t ntiles = (m + kTile - 1) / kTile;
    if (enc_passes() == 1) {
        unsigned long long *lb;
        SW_ALLOC(lb, ctx, S_ENC_FLAGS, size_t(ntiles + 1) * 8 + 64);
        void *mdev = nullptr;  // the total and the error flag, written by the last tile into mapped host memory
        volatile int64_t *host = static_cast<volatile int64_t *>(mapped(ctx, 24, &mdev));
        if (!host) return SWARM_ERR_OOM;
        int64_t *dev_tot = static_cast<int64_t *>(mdev);
        unsigned *err = reinterpret_cast<unsigned *>(dev_tot + 1);
        unsigned *fail = reinterpret_cast<unsigned *>(dev_tot + 2);
        reinterpret_cast<volatile unsigned *>(host + 2)[0] = 0u;  // (no kernel of this ctx is running: calls sync)
        if (ctx->enc_flags != lb || ctx->enc_cap != ctx->cap[S_ENC_FLAGS] || ctx->enc_epoch >= (1u << 24) - 1) {
            SW_HIP(hipMemsetAsync(lb, 0, ctx->cap[S_ENC_FLAGS], s));  // a new buffer, or the epoch tags used up
            ctx->enc_flags = lb;
            ctx->enc_cap = ctx->cap[S_ENC_FLAGS];
            ctx->enc_epoch = 0;
        }
        const uint32_t epoch = ++ctx->enc_epoch;
        SW_ARG(ntiles < (int64_t(1) << 31), "m out of range");
        if (const char *e = getenv("SWARM_ENC_TEST_POISON"); e && e[0] == '1')  // test aid: a ticket left over
            SW_HIP(hipMemsetAsync(lb, 0x40, 4, s));                             // by a failed call
        const auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
        const bool pair = enc_pair() && al16(type) && al16(sender) && al16(tick) && al16(a) && al16(b) &&
                          al16(task) && al16(winner) && al16(offsets) && (reinterpret_cast<uintptr_t>(status) & 1) == 0;
        hipLaunchKernelGGL(pair ? k_enc_one<2> : k_enc_one<1>, dim3(unsigned(ntiles)), dim3(kEB), 0, s, m, in,
                           int(wide != 0), status, offsets, out, out ? cap : int64_t(0), lb, epoch, dev_tot, err,
                           fail);
        SW_LAUNCHED();
        SW_HIP(hipStreamSynchronize(s));
        *total_bytes = host[0];
        if (const unsigned fl = reinterpret_cast<volatile const unsigned *>(host + 2)[0]) {
            // the ticket and the look-back words are in an unknown state: the next call zeroes them first
            ctx->enc_flags = nullptr;
            set_error("encode: tile offsets lost (%s); concurrent encode calls on one ctx are not supported",
                      fl & 2u ? "a tile ticket out of range" : "a look-back walk gave up");
            return SWARM_ERR_HIP;
        }
        if (reinterpret_cast<volatile const unsigned *>(host + 1)[0]) {
            set_error("output buffer holds %lld bytes, the packets need %lld", (long long)cap, (long long)host[0]);
            return SWARM_ERR_RANGE;
        }
        return SWARM_OK;
    }
    uint8_t *tmp;
    int32_t *wt;
    SW_ALLOC(tmp, ctx, S_TMP0, size_t(ntiles) * kTileBytes);
    SW_ALLOC(wt, ctx, S_TMP1, size_t(m) * 2 + size_t(ntiles) * kWavesT * 4 + size_t(ntiles + 1) * 8 + 128);
    int64_t *base = reinterpret_cast<int64_t *>(wt + ((size_t(ntiles) * kWavesT + 1) & ~size_t(1)));
    unsigned *err = reinterpret_cast<unsigned *>(base + ntiles + 1);
    uint16_t *loc = reinterpret_cast<uint16_t *>(err + 16);
    const unsigned codec_wgs = swarm::codec_grid_cap();
    const unsigned grid = grid_for(ntiles, 1, codec_wgs);
    hipLaunchKernelGGL(k_enc_tile, dim3(grid), dim3(kEB), 0, s, m, in, int(wide != 0), status, loc, tmp, wt);
    SW_LAUNCHED();
    hipLaunchKernelGGL(k_enc_base, dim3(1), dim3(1024), 0, s, ntiles, wt, base);
    SW_LAUNCHED();
    int64_t *host = static_cast<int64_t *>(pinned(ctx, 16));
    if (!host) return SWARM_ERR_OOM;
    if (out == nullptr) {  // sizing call: the lengths only
        SW_HIP(hipMemcpyAsync(host, base + ntiles, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        *total_bytes = host[0];
        return SWARM_OK;
    }
    SW_HIP(hipMemsetAsync(err, 0, 4, s));
    hipLaunchKernelGGL(k_enc_place, dim3(grid), dim3(kEB), 0, s, m, tmp, wt, base, loc, cap, offsets, out, err);
    SW_LAUNCHED();
    SW_HIP(hipMemcpyAsync(host, base + ntiles, 8, hipMemcpyDeviceToHost, s));
    SW_HIP(hipMemcpyAsync(host + 1, err, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    *total_bytes = host[0];
    if (reinterpret_cast<const unsigned *>(host + 1)[0]) {
        set_error("output buffer holds %lld bytes, the packets need %lld", (long long)cap, (long long)host[0]);
        return SWARM_ERR_RANGE;
    }
    return SWARM_OK;
}

int swarm_codec_decode(swarm_ctx *ctx, int64_t m, const uint8_t *buf, int64_t buf_len, const int64_t *offsets,
                       int32_t wide,
                       int8_t *status, int64_t *type, int64_t *sender, int64_t *tick, float *a, float *b,
                       int64_t *task, int64_t *winner, uint8_t *has_pos, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(m >= 0 && m < (int64_t(1) << 31) && buf_len >= 0, "m / buf_len out of range");
    SW_ARG(buf != nullptr || buf_len == 0, "buf is NULL");
    SW_ARG(m == 0 || (offsets && status && type && sender && tick && a && b && task && winner && has_pos),
           "NULL array");
    if (m == 0) return SWARM_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const DecOut o{status, type, sender, tick, task, winner, a, b, has_pos};
    hipLaunchKernelGGL(k_decode, dim3(grid_for(m, kEncPer, codec_grid_cap())), dim3(kBlock), 0, s, m, buf, buf_len, offsets,
                       int(wide != 0), o);
    SW_LAUNCHED();
    return SWARM_OK;
}

}  // extern "C"
