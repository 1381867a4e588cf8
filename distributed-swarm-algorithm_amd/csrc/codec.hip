// Batched wire codec on gfx950.
//
// The reference's transport seam frames every message as a big-endian '!BBI' header (type u8,
// sender u8, tick u32; agent.py:184-186) followed by a type-specific payload -- HEARTBEAT
// '!ff' leader position (agent.py:283-289), ELECTION_ACCLAIM '!B' own ID (agent.py:240),
// COORDINATOR none (241), TASK_CLAIM '!If' task + utility (302), TASK_CONFLICT '!IB' task +
// winner (322, 325) -- and parses inbound packets in on_message_received (agent.py:197-214).
// These kernels do both for a whole batch of messages (one thread per message / packet; a
// byte-moving, HBM-bound job: no arithmetic worth the name):
//   encode  status + length per message, an exclusive scan into packet offsets, then every
//           thread writes its packet's bytes.  Errors as the reference raises them, payload
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
#include <hipcub/hipcub.hpp>

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
    bool (*id_ok)(int64_t) = wide ? u32_ok : u8_ok;
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

__global__ __launch_bounds__(kBlock) void k_enc_len(int64_t m, EncIn in, int wide, int64_t *__restrict__ len,
                                                   int8_t *__restrict__ status) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < m; i += int64_t(gridDim.x) * kBlock) {
        int l;
        status[i] = int8_t(enc_status(in.type[i], in.sender[i], in.tick[i], in.a[i], in.b[i], in.task[i],
                                      in.winner[i], wide, &l));
        len[i] = l;
    }
}

// Packet bytes of message i at p (status 0).
__device__ __forceinline__ void write_packet(uint8_t *p, const EncIn &in, int64_t i, int wide) {
    const int ty = int(in.type[i]);
    p[0] = uint8_t(ty);
    int h;
    if (wide) {
        put_u32(p + 1, uint32_t(in.sender[i]));
        put_u32(p + 5, uint32_t(in.tick[i]));
        h = 9;
    } else {
        p[1] = uint8_t(in.sender[i]);
        put_u32(p + 2, uint32_t(in.tick[i]));
        h = 6;
    }
    p += h;
    switch (ty) {
        case T_HB:
            put_u32(p, __float_as_uint(float(in.a[i])));
            put_u32(p + 4, __float_as_uint(float(in.b[i])));
            break;
        case T_ACCLAIM:
            if (wide) put_u32(p, uint32_t(in.sender[i]));
            else p[0] = uint8_t(in.sender[i]);
            break;
        case T_CLAIM:
            put_u32(p, uint32_t(in.task[i]));
            put_u32(p + 4, __float_as_uint(float(in.a[i])));
            break;
        case T_CONFLICT:
            put_u32(p, uint32_t(in.task[i]));
            if (wide) put_u32(p + 4, uint32_t(in.winner[i]));
            else p[4] = uint8_t(in.winner[i]);
            break;
        default:
            break;
    }
}

// Messages [c0, c0 + kEncPer) per workgroup: packets are assembled in LDS at the same 16-byte
// alignment they have in `out`, then the workgroup's contiguous output range is stored with
// 16-byte vector stores (its partial first / last 16 bytes byte by byte: they share lines with
// the neighbouring workgroups' packets).
constexpr int kEncJ = 4, kEncPer = kBlock * kEncJ, kMaxPkt = 17;
constexpr int kEncLds = (kEncPer * kMaxPkt + 32 + 15) / 16;  // uint4 words

__global__ __launch_bounds__(kBlock) void k_enc_write(int64_t m, EncIn in, int wide, const int64_t *__restrict__ off,
                                                     const int8_t *__restrict__ status, uint8_t *__restrict__ out) {
    __shared__ uint4 s_buf[kEncLds];
    uint8_t *lb = reinterpret_cast<uint8_t *>(s_buf);
    for (int64_t c0 = int64_t(blockIdx.x) * kEncPer; c0 < m; c0 += int64_t(gridDim.x) * kEncPer) {
        const int64_t c1 = c0 + kEncPer < m ? c0 + kEncPer : m;
        const int64_t base = off[c0], end = off[c1], abase = base & ~int64_t(15);
#pragma unroll
        for (int j = 0; j < kEncJ; ++j) {
            const int64_t i = c0 + j * kBlock + threadIdx.x;
            if (i < c1 && status[i] == 0) write_packet(lb + (off[i] - abase), in, i, wide);
        }
        __syncthreads();
        const int64_t A = (base + 15) & ~int64_t(15), B = end & ~int64_t(15);
        if (A >= B) {  // no whole 16-byte block: bytewise
            for (int64_t x = base + threadIdx.x; x < end; x += kBlock) out[x] = lb[x - abase];
        } else {
            if (threadIdx.x < A - base) out[base + threadIdx.x] = lb[base + threadIdx.x - abase];
            if (threadIdx.x < end - B) out[B + threadIdx.x] = lb[B + threadIdx.x - abase];
            uint4 *dst = reinterpret_cast<uint4 *>(out + A);
            const uint4 *src = s_buf + (A - abase) / 16;
            for (int64_t q = threadIdx.x; q < (B - A) / 16; q += kBlock) dst[q] = src[q];
        }
        __syncthreads();  // s_buf reused by the next chunk
    }
}

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
    int64_t *len;
    SW_ALLOC(len, ctx, S_TMP1, size_t(m + 1) * 8);
    const unsigned codec_wgs = swarm::codec_grid_cap();
    const unsigned grid = grid_for(m, kBlock, codec_wgs);
    hipLaunchKernelGGL(k_enc_len, dim3(grid), dim3(kBlock), 0, s, m, in, int(wide != 0), len, status);
    SW_LAUNCHED();
    SW_HIP(hipMemsetAsync(len + m, 0, 8, s));
    size_t tmp_bytes = 0;
    SW_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, len, offsets, int(m + 1), s));
    void *tmp;
    SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
    SW_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, len, offsets, int(m + 1), s));
    SW_HIP(hipMemcpyAsync(total_bytes, offsets + m, 8, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    if (out == nullptr) return SWARM_OK;  // sizing call
    if (cap < *total_bytes) {
        set_error("output buffer holds %lld bytes, the packets need %lld", (long long)cap, (long long)*total_bytes);
        return SWARM_ERR_RANGE;
    }
    hipLaunchKernelGGL(k_enc_write, dim3(grid_for(m, kEncPer, codec_wgs)), dim3(kBlock), 0, s, m, in, int(wide != 0),
                       offsets, status, out);
    SW_LAUNCHED();
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
