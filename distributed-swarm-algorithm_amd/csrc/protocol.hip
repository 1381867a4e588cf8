// Timer FSM / protocol ticks on gfx950.
//
// The reference runs every agent's update_loop at 10 Hz (agent.py:66-80): each tick it handles
// inbound packets and then _process_logic -- the failure detector / election timer
// _check_election_timeout (217-241) and the leader's _send_heartbeat (283-289).  Here the whole
// swarm ticks at once under contract T1 (tools/gen_golden.py ref_fsm, pinned against the real
// handlers): one launch per tick, one thread per agent, which
//   receives  the packets its CSR neighbours sent during the previous tick, in CSR order, as the
//             handlers process them (_handle_election_acclaim 263-275 + _handle_coordinator
//             277-281, _handle_heartbeat 243-261; the bully heartbeat only when the agent's own
//             tick % 10 == 0, 288);
//   ticks     its election timer: FOLLOWER silent for > timeout -> ELECTION_WAIT with a jitter
//             delay (a counter-based hash of (seed, id, tick), so every run draws the same);
//             ELECTION_WAIT past its delay -> LEADER + ELECTION_ACCLAIM + COORDINATOR;
//   sends     into its outbox byte (tick-parity double buffer): bit 0 ACCLAIM+COORDINATOR,
//             bit 1 HEARTBEAT -- exact, see swarm_oracle.c orc_protocol.
// Push mode (the hearers CSR given), one launch per tick:
//   k_tick   receive + timers, its workgroups in two roles: the receive role lists each 4 096-agent
//            chunk's receivers (mail bit set: 1 bit per agent, set by last tick's senders) in LDS
//            and serves them one per thread -- its one sender directly, or its CSR row in order
//            (col / outbox loads in chunks of kRecv, all in flight) when it has several -- then
//            their timers; the sweep role streams every other agent's timers (kSweepV agents per
//            thread); sends are listed in the workgroup's own segment (no global atomics),
//            per-tick counters; then each workgroup mails the hearers of the senders it listed
//            (64-bit atomicOr into the next tick's words, combined per word, all hearer loads in
//            flight).  The words rotate over three buffers: tick t reads buf(t), mails into
//            buf(t+1) and clears buf(t+2).
// (Rounds 2-3 ran k_compact + k_receive + k_sweep + k_mail, round 4 first k_tick + k_mail: the
// boundaries and the list round trips per tick.)
// A quiet agent costs ~9 B (its 8-byte record -- state, alive, leader-position flag, tick phase and its
// timer as a tick of the run -- and its outbox byte) plus its mail bit; only receivers pay for their
// rows.  Storm ticks: when a workgroup's senders exceed pull_frac x the agents of its share (a timeout wave: thousands of ACCLAIMs at once), it skips the mail atomics
// and the next tick pulls instead -- every alive agent walks its own row, as pull mode does.  Same results: an agent
// without a sender in its row hears nothing either way.  Pull mode (no hearers CSR): one fused
// launch in which every agent walks its row -- the cross-check.  Both are latency-bound gathers, no
// arithmetic worth the name.
// Agents killed at a kill tick (every alive LEADER then) stop receiving and sending.
#include <cmath>

#include "swarm_common.h"

namespace swarm {
namespace {

constexpr uint8_t kAcclaim = 1, kHeartbeat = 2;
constexpr int kRecv = 8;  // CSR entries loaded per receive chunk (pull mode, hearer walks)
// k_tick's row walks (75 VGPRs, 6 waves per SIMD; 4 entries per chunk: 63 VGPRs, 8 waves, but
// 0.135 against 0.128 ms per tick -- the walks' chunks one after the other cost more than the
// occupancy gains; SWARM_RECV_TICK: A/B builds)
#ifndef SWARM_RECV_TICK
#define SWARM_RECV_TICK 8
#endif
constexpr int kRecvTick = SWARM_RECV_TICK;
constexpr uint8_t ST_F = SWARM_FOLLOWER, ST_W = SWARM_ELECTION_WAIT, ST_L = SWARM_LEADER;

__device__ __forceinline__ double jitter_u(uint64_t seed, int32_t id, int64_t t) {
    uint64_t x = seed ^ (uint64_t(uint32_t(id)) * 0x9E3779B97F4A7C15ull) ^ (uint64_t(t) * 0xD1B54A32D192ED03ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return double(x >> 11) * (1.0 / 9007199254740992.0);
}

// An agent's per-tick fields for the run, in one 8-byte record (the C-ABI's separate arrays are packed at
// the start of a run and unpacked at its end): a receiver touches one line for them instead of four, and
// the sweep streams 8 B per agent instead of 15.
//   x: the flag word -- byte 0 state, byte 1 alive, byte 2 bits (kHL: has_leader_pos, kH64, kDirty),
//      byte 3 tick phase = tick_off mod 10 in [0, 9] ((t + tick_off) % 10 == 0 iff (t + phase) % 10 == 0
//      for every tick t >= 0);
//   y: the agent's timer as a tick of the run (relative to t0), exact because the reference's clock is
//      t * dt: FOLLOWER -- the tick its last_heartbeat_time was set at (last_hb == double(t0 + y) * dt,
//      the timeout test evaluated on that value, as _check_election_timeout does, agent.py:223);
//      ELECTION_WAIT -- the first tick t at which now - election_wait_start > election_delay holds
//      (agent.py:234; found once, when the wait starts: the test is monotone in t for dt > 0), 0 = never.
//   kH64: the timer is in the caller's f64 arrays instead (a value no tick of the run represents, or
//      dt <= 0): the test reads them, as before.  kDirty: last_hb changed in the run; the unpack writes
//      double(t0 + y) * dt (a FOLLOWER entering ELECTION_WAIT writes it at once).
// Leader and leader position are write-only during a run: one 16-byte record per agent (LRec), one line
// per heartbeat receiver instead of two.
constexpr uint32_t kHL = 1, kH64 = 2, kDirty = 4;
__host__ __device__ __forceinline__ uint8_t fw_state(uint32_t w) { return uint8_t(w); }
__host__ __device__ __forceinline__ uint8_t fw_alive(uint32_t w) { return uint8_t(w >> 8); }
__host__ __device__ __forceinline__ uint32_t fw_bits(uint32_t w) { return (w >> 16) & 0xFFu; }
__host__ __device__ __forceinline__ int32_t fw_phase(uint32_t w) { return int32_t(w >> 24); }
__host__ __device__ __forceinline__ uint32_t fw_make(uint8_t st, uint8_t al, uint32_t bits, int32_t ph) {
    return uint32_t(st) | (uint32_t(al) << 8) | (bits << 16) | (uint32_t(ph) << 24);
}

struct alignas(16) LRec {
    float x, y;      // leader_pos
    int32_t leader;  // leader
    int32_t pad;
};

struct Fsm {
    uint2 *rec;  // (flag word, timer tick)
    LRec *lrec;
    double *last_hb, *wait_start, *delay;  // the caller's (kH64 timers; written when a wait starts)
    int64_t t0, t_end;                     // the run's ticks: t0 + 1 .. t_end
    double dt;
};

__device__ __forceinline__ void set_lpos(const Fsm &f, int64_t i, float x, float y) {
    *reinterpret_cast<float2 *>(&f.lrec[i].x) = make_float2(x, y);
}

// The first tick t in [lo, t_end] with double(t) * dt - ws > d, relative to t0; 0 when there is none
// (dt > 0: the test is monotone in t).  Tried first at the estimate floor((ws + d) / dt) + 1, clamped to
// [lo, t_end] (right but for rounding: then one test each side), bisection only when that is off.
__host__ __device__ __forceinline__ int32_t wait_exit(int64_t lo, int64_t t_end, int64_t t0, double dt, double ws,
                                                      double d) {
    auto go = [&](int64_t t) { return double(t) * dt - ws > d; };
    if (lo > t_end || !go(t_end)) return 0;
    int64_t hi = t_end;  // go(hi)
    const double g = std::floor((ws + d) / dt) + 1.0;
    if (g == g) {
        const int64_t c = g <= double(lo) ? lo : g >= double(t_end) ? t_end : int64_t(g);
        if (go(c)) {
            if (c == lo || !go(c - 1)) return int32_t(c - t0);
            hi = c - 1;
        } else {
            lo = c + 1;  // c < t_end: go(t_end) holds
        }
    }
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (go(mid)) hi = mid;
        else lo = mid + 1;
    }
    return int32_t(lo - t0);
}

__global__ __launch_bounds__(kBlock) void k_kill_leaders(int64_t n, uint2 *__restrict__ rec) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const uint32_t w = rec[i].x;
        if (fw_alive(w) && fw_state(w) == ST_L) rec[i].x = w & ~0xFF00u;
    }
}

// The C-ABI's fields -> records (once per run).
__global__ __launch_bounds__(kBlock) void k_pack_fsm(int64_t n, const uint8_t *__restrict__ state,
                                                    const uint8_t *__restrict__ alive,
                                                    const uint8_t *__restrict__ hl,
                                                    const int32_t *__restrict__ tick_off,
                                                    const int32_t *__restrict__ leader,
                                                    const float2 *__restrict__ lpos, Fsm f) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const int32_t ph = ((tick_off[i] % 10) + 10) % 10;
        const uint8_t st = state[i];
        uint32_t bits = hl[i] ? kHL : 0u;
        int32_t y = 0;
        if (st == ST_F) {  // last_hb as a tick of the run, if one represents it exactly
            const double lhb = f.last_hb[i];
            const double k = f.dt != 0.0 ? std::nearbyint(lhb / f.dt) : 0.0;
            const bool ok = f.dt != 0.0 && std::fabs(k) < 9.0e15 && k * f.dt == lhb &&
                            k - double(f.t0) > -2147483647.0 && k - double(f.t0) < 2147483647.0;
            if (ok) y = int32_t(int64_t(k) - f.t0);
            else bits |= kH64;
        } else if (st == ST_W) {
            if (f.dt > 0.0) y = wait_exit(f.t0 + 1, f.t_end, f.t0, f.dt, f.wait_start[i], f.delay[i]);
            else bits |= kH64;
        }
        f.rec[i] = make_uint2(fw_make(st, alive[i], bits, ph), uint32_t(y));
        const float2 q = lpos[i];
        f.lrec[i] = LRec{q.x, q.y, leader[i], 0};
    }
}

// Records -> the C-ABI's fields (once per run).
__global__ __launch_bounds__(kBlock) void k_unpack_fsm(int64_t n, uint8_t *__restrict__ state,
                                                      uint8_t *__restrict__ alive, uint8_t *__restrict__ hl,
                                                      int32_t *__restrict__ leader, float2 *__restrict__ lpos,
                                                      Fsm f) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const uint2 r = f.rec[i];
        state[i] = fw_state(r.x);
        alive[i] = fw_alive(r.x);
        hl[i] = (fw_bits(r.x) & kHL) ? 1 : 0;
        if (fw_bits(r.x) & kDirty) f.last_hb[i] = double(f.t0 + int32_t(r.y)) * f.dt;
        const LRec q = f.lrec[i];
        leader[i] = q.leader;
        lpos[i] = make_float2(q.x, q.y);
    }
}

// Handlers for everything agent (me) hears in CSR row [b, e) (see the header).  The row in
// chunks of kRecv: all column loads, then all outbox loads in flight, then the handlers in CSR
// order on registers; sender IDs only for neighbours that sent something.
struct Heard {
    uint8_t st, ob;
    bool live, lead_set;
    int32_t lead, hb_from;  // hb_from: the last accepted heartbeat's sender (its position -> leader_pos)
};

// What one sender's packets of a tick do to the receiver (s: sender ID, j: its index), in the
// order it sent them: ACCLAIM then COORDINATOR, then HEARTBEAT.
__device__ __forceinline__ void hear(Heard &h, uint8_t o, int32_t s, int32_t j, int32_t me, bool hb_tick) {
    if (o & kAcclaim) {
        if (s < me && (h.st == ST_L || h.st == ST_W) && hb_tick) h.ob |= kHeartbeat;  // bully back
        h.lead = s;  // (higher sender: follow) then COORDINATOR: unconditional takeover
        h.lead_set = true;
        h.st = ST_F;
        h.live = true;
    }
    if (o & kHeartbeat) {
        if (h.st == ST_L && s < me) {
            if (hb_tick) h.ob |= kHeartbeat;
        } else {
            h.st = ST_F;  // yield (LEADER) / stop waiting (ELECTION_WAIT) / stay FOLLOWER
            h.lead = s;
            h.lead_set = true;
            h.live = true;
            h.hb_from = j;
        }
    }
}

template <int R>
__device__ __forceinline__ void receive_row(int32_t b, int32_t e, const int32_t *__restrict__ col,
                                            const uint8_t *__restrict__ ob_in, const int32_t *__restrict__ ids,
                                            int32_t me, bool hb_tick, Heard &h) {
    for (int32_t k0 = b; k0 < e; k0 += R) {
        int32_t jj[R];
        uint8_t oo[R];
#pragma unroll
        for (int u = 0; u < R; ++u) jj[u] = k0 + u < e ? col[k0 + u] : -1;
        uint8_t any = 0;
#pragma unroll
        for (int u = 0; u < R; ++u) {
            oo[u] = jj[u] >= 0 ? ob_in[jj[u]] : uint8_t(0);
            any |= oo[u];
        }
        if (!any) continue;
        int32_t ss[R];  // the senders' IDs, all loads in flight
#pragma unroll
        for (int u = 0; u < R; ++u) ss[u] = oo[u] ? ids[jj[u]] : 0;
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint8_t o = oo[u] & (kAcclaim | kHeartbeat);
            if (o) hear(h, o, ss[u], jj[u], me, hb_tick);
        }
    }
}

// A liveness proof sets last_hb = now: the timer becomes this tick; the heartbeat's leader position (state
// / leader: caller).
__device__ __forceinline__ void apply_heard(int64_t i, const Heard &h, int64_t t, const double2 *__restrict__ pos,
                                            const Fsm &f, uint32_t &bits, int32_t &y) {
    if (h.live) {
        y = int32_t(t - f.t0);
        bits = (bits & ~kH64) | kDirty;
    }
    if (h.hb_from >= 0) {
        const double2 q = pos[h.hb_from];
        set_lpos(f, i, float(q.x), float(q.y));
        bits |= kHL;
    }
}

// _check_election_timeout (217-241) and the leader's heartbeat (283-289) for agent i in state
// st; `heard`: it got a liveness proof this tick (its timer is now).  Returns the sends.
__device__ __forceinline__ uint8_t timers(int64_t i, uint8_t &st, bool heard, int32_t &lead, bool &lead_set,
                                          int64_t t, double now, double timeout, double jitter, uint64_t seed,
                                          const int32_t *__restrict__ ids, int32_t phase, const Fsm &f,
                                          uint32_t &bits, int32_t &y) {
    uint8_t ob = 0;
    if (st == ST_F && !heard) {
        const double last_hb = (bits & kH64) ? f.last_hb[i] : double(f.t0 + y) * f.dt;
        if (now - last_hb > timeout) {
            if (bits & kDirty) f.last_hb[i] = last_hb;
            st = ST_W;
            const double d = 0.0 + jitter * jitter_u(seed, ids[i], t);
            f.wait_start[i] = now;
            f.delay[i] = d;
            lead = -1;
            lead_set = true;
            bits &= ~(kHL | kDirty);
            set_lpos(f, i, 0.f, 0.f);
            if (f.dt > 0.0) {
                y = wait_exit(t + 1, f.t_end, f.t0, f.dt, now, d);
                bits &= ~kH64;
            } else {
                bits |= kH64;
            }
        }
    }
    if (st == ST_W) {
        const bool done = (bits & kH64) ? now - f.wait_start[i] > f.delay[i] : (y != 0 && t - f.t0 >= int64_t(y));
        if (done) {
            st = ST_L;
            lead = ids[i];
            lead_set = true;
            ob |= kAcclaim;
        }
    }
    if (st == ST_L && ((t + phase) % 10) == 0) ob |= kHeartbeat;
    return ob;
}

// Per-tick counters: wave reduce, one LDS atomic per wave, one global atomic per workgroup into
// one of kShards copies (blockIdx-interleaved; k_sum_counts adds them up).  A single copy made
// every workgroup's 4 atomics queue on the same 4 addresses: ~50 us per tick at 4 096
// workgroups, ~470 us at one agent per thread (measured).
constexpr int kShards = 64;
constexpr int kTraffic = 8;  // traffic counters (swarm_protocol_run_ex), sharded like the tick counts

// Per-workgroup traffic counts into one of kShards copies (one atomic per nonzero value).
__device__ __forceinline__ void add_traffic(unsigned long long *tr, int k, unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (tr && (threadIdx.x & 63) == 0 && v) atomicAdd(&tr[(blockIdx.x & (kShards - 1)) * kTraffic + k], v);
}

__device__ __forceinline__ void add_counts(unsigned c0, unsigned c1, unsigned c2, unsigned c3, unsigned *s_cnt,
                                           unsigned long long *counts) {
    counts += 4 * (blockIdx.x & (kShards - 1));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        c0 += __shfl_xor(c0, off, 64);
        c1 += __shfl_xor(c1, off, 64);
        c2 += __shfl_xor(c2, off, 64);
        c3 += __shfl_xor(c3, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c0) atomicAdd(&s_cnt[0], c0);
        if (c1) atomicAdd(&s_cnt[1], c1);
        if (c2) atomicAdd(&s_cnt[2], c2);
        if (c3) atomicAdd(&s_cnt[3], c3);
    }
    __syncthreads();
    if (threadIdx.x < 4 && s_cnt[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)s_cnt[threadIdx.x]);
}

// counts[t][shard][c] -> out[t][c]
__global__ __launch_bounds__(kBlock) void k_sum_counts(int64_t ticks, const unsigned long long *__restrict__ part,
                                                      unsigned long long *__restrict__ out) {
    for (int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x; q < ticks * 4; q += int64_t(gridDim.x) * kBlock) {
        const int64_t t = q / 4, c = q % 4;
        unsigned long long sum = 0;
        for (int sh = 0; sh < kShards; ++sh) sum += part[(t * kShards + sh) * 4 + c];
        out[q] = sum;
    }
}

// ---------------------------------------------------------------- pull mode: one fused launch
__global__ __launch_bounds__(kBlock) void k_tick_pull(int64_t n, int64_t t, const int32_t *__restrict__ ids,
                                                     const double2 *__restrict__ pos, const int32_t *__restrict__ rp,
                                                     const int32_t *__restrict__ col, Fsm f,
                                                     const uint8_t *__restrict__ ob_in, uint8_t *__restrict__ ob_out,
                                                     double dt, double timeout, double jitter, uint64_t seed,
                                                     unsigned long long *__restrict__ counts) {
    __shared__ unsigned s_cnt[4];
    if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const double now = double(t) * dt;
    unsigned c_lead = 0, c_wait = 0, c_acc = 0, c_hb = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const uint2 r = f.rec[i];
        const uint32_t fw = r.x;
        if (!fw_alive(fw)) {
            ob_out[i] = 0;
            continue;
        }
        const uint8_t st0 = fw_state(fw);
        const int32_t ph = fw_phase(fw);
        uint32_t bits = fw_bits(fw);
        int32_t y = int32_t(r.y);
        Heard h{st0, 0, false, false, 0, -1};
        receive_row<kRecv>(rp[i], rp[i + 1], col, ob_in, ids, ids[i], ((t + ph) % 10) == 0, h);
        apply_heard(i, h, t, pos, f, bits, y);
        const uint8_t ob = h.ob | timers(i, h.st, h.live, h.lead, h.lead_set, t, now, timeout, jitter, seed, ids,
                                         ph, f, bits, y);
        const uint32_t fw1 = fw_make(h.st, 1, bits, ph);
        if (fw1 != fw || uint32_t(y) != r.y) f.rec[i] = make_uint2(fw1, uint32_t(y));
        if (h.lead_set) f.lrec[i].leader = h.lead;
        ob_out[i] = ob;
        c_lead += h.st == ST_L;
        c_wait += h.st == ST_W;
        c_acc += (ob & kAcclaim) != 0;
        c_hb += (ob & kHeartbeat) != 0;
    }
    add_counts(c_lead, c_wait, c_acc, c_hb, s_cnt, counts);
}

// ---------------------------------------------------------------- push mode

// Mail for the hearers of sender i: one bit per agent (one atomicOr per distinct 64-agent word).
// The atomic returns the word's previous bits: a hearer whose bit was clear gets from[r] = i (its
// only sender so far); one whose bit was already set gets its `multi` bit (several senders: it
// walks its row).  (Plain byte marks were tried: the scan of 1-byte marks dirtied by scattered
// byte stores costs 5x the 64-bit bitmap's, more than the atomics save.)
struct Mail {
    unsigned long long *bits, *multi;
    int32_t *from;
};

// Up to kFlush word runs of one sender at once: every returning atomic in flight before the first
// result is used (one after the other, a sender's ~3 words cost ~3 atomic round trips).
constexpr int kFlush = 4;

__device__ __forceinline__ void mail_flush(const Mail &m, const int32_t *pw, const unsigned long long *pb, int np,
                                           int32_t sender) {
    unsigned long long old[kFlush];
#pragma unroll
    for (int j = 0; j < kFlush; ++j) old[j] = j < np ? atomicOr(&m.bits[pw[j]], pb[j]) : 0ull;
#pragma unroll
    for (int j = 0; j < kFlush; ++j) {
        if (j >= np) break;
        const unsigned long long dup = old[j] & pb[j];
        if (dup) atomicOr(&m.multi[pw[j]], dup);
        unsigned long long fresh = pb[j] & ~old[j];
        while (fresh) {
            const int q = __ffsll((long long)fresh) - 1;
            fresh &= fresh - 1;
            m.from[int64_t(pw[j]) * 64 + q] = sender;
        }
    }
}

__device__ __forceinline__ void mail_hearers(int32_t b, int32_t e, const int32_t *__restrict__ tcol, const Mail &m,
                                             int32_t sender) {
    int32_t w = -1, pw[kFlush];
    unsigned long long bits = 0, pb[kFlush];
    int np = 0;
    for (int32_t k0 = b; k0 < e; k0 += kRecv) {
        int32_t rr[kRecv];  // all hearer loads of the chunk in flight
#pragma unroll
        for (int u = 0; u < kRecv; ++u) rr[u] = k0 + u < e ? tcol[k0 + u] : -1;
#pragma unroll
        for (int u = 0; u < kRecv; ++u) {
            const int32_t r = rr[u];
            if (r < 0) continue;
            if ((r >> 6) != w) {
                if (bits) {
                    if (np == kFlush) {
                        mail_flush(m, pw, pb, np, sender);
                        np = 0;
                    }
                    pw[np] = w;
                    pb[np++] = bits;
                }
                w = r >> 6;
                bits = 0;
            }
            bits |= 1ull << (r & 63);
        }
    }
    if (bits) {
        if (np == kFlush) {
            mail_flush(m, pw, pb, np, sender);
            np = 0;
        }
        pw[np] = w;
        pb[np++] = bits;
    }
    if (np) mail_flush(m, pw, pb, np, sender);
}

// Resumed run: mail for the receivers of tick t0's sends.
__global__ __launch_bounds__(kBlock) void k_mail_from_outbox(int64_t n, const uint8_t *__restrict__ ob,
                                                            const int32_t *__restrict__ trp,
                                                            const int32_t *__restrict__ tcol, Mail m) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        if (ob[i]) mail_hearers(trp[i], trp[i + 1], tcol, m, int32_t(i));
}

// One launch per tick for receive + timers (push mode), its workgroups in two roles that run side
// by side: the receivers' short dependent chains overlap the sweep's streaming instead of following
// it.  (A single role -- each sweep wave serving its own receivers -- held every wave for its
// receivers' chains: 0.170 vs 0.152 ms per tick with separate kernels.)
//   sweep    (workgroups g_recv ..): kSweepV consecutive agents per thread, their byte fields
//            (outbox) as one 32-bit word, their flag words as one 16-byte load, their timers (last_hb) and
//            their 64-agent mail word loaded up front; agents with a mail bit are left to the
//            receive role, the others tick their timers.
//   receive  (workgroups 0 .. g_recv - 1; all of them on a pulled tick): chunks of 4 096 agents;
//            the chunk's receivers (mail bit set; on a pulled tick every agent) are listed in LDS
//            and served one per thread -- its one sender directly (from[]), or its CSR row in
//            order when it has several (multi bit) or the tick is pulled -- then its timers run on
//            the result.
// Senders of both roles are listed in the workgroup's own segment, then mailed by it.
#ifndef SWARM_SWEEP_V  // A/B aid: agents per sweep thread (4 or 8)
#define SWARM_SWEEP_V 4
#endif
constexpr int kSweepV = SWARM_SWEEP_V;
static_assert(kSweepV == 4 || kSweepV == 8, "sweep: 4 or 8 agents per thread");
constexpr int kRecvChunk = 4096;  // agents per receive-role pass (64 mail words, 16 agents per thread;
                                  // 2 048: 0.144 vs 0.138 ms per tick)

// Sender segments of k_tick's workgroups (each mails its own): the g_recv receive-role ones first
// (rcap entries each: their chunks' agents), then the sweep-role ones (scap each: their agents, or
// their chunks' on a pulled tick, when every workgroup receives).
struct Segs {
    int32_t *base;
    int64_t rcap, scap;
    int g_recv;
    __device__ __forceinline__ int32_t *of(int b) const {
        return b < g_recv ? base + int64_t(b) * rcap : base + int64_t(g_recv) * rcap + int64_t(b - g_recv) * scap;
    }
};

// Exclusive prefix over the workgroup of c (0 <= c < 2^B) and the total (every thread gets it).
template <int B>
__device__ __forceinline__ int block_excl_scan(int c, int &total, int *s_wave) {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    int ex = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const unsigned long long m = __ballot((c >> b) & 1);
        ex += int(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u))) << b;
        tot += __popcll(m) << b;
    }
    if (lane == 0) s_wave[wid] = tot;
    __syncthreads();
    int off = 0, all = 0;
#pragma unroll
    for (int q = 0; q < kBlock / kWave; ++q) {
        off += q < wid ? s_wave[q] : 0;
        all += s_wave[q];
    }
    __syncthreads();  // s_wave read by all
    total = all;
    return off + ex;
}

struct TickCounts {
    unsigned lead = 0, wait = 0, acc = 0, hb = 0;
    unsigned single = 0, multi = 0, edges = 0;  // one thread's, one tick: < 2^32 (32-bit: VGPRs)
};

// k_tick's own mail: once a workgroup's agents are done it mails the hearers of the senders it
// listed, into tick t+1's words; the words are rotated over three buffers (tick t reads buf(t),
// mails into buf(t+1) and clears buf(t+2), read in tick t-1 and next mailed in tick t+1) and the
// single-sender slots over two, so no workgroup of tick t touches what another one still reads.
// Storms are decided per workgroup: more senders than frac x the agents of its share -> it mails
// nothing and flags tick t+1 as pulled.  (Round 4's separate k_mail launch after k_tick, deciding
// on the tick's total senders: 0.128 against 0.123 ms per tick, same box.)
struct NextMail {
    Mail next;                       // tick t+1's words and single-sender slots
    unsigned long long *clear;       // buf(t+2), n_clear words
    int64_t n_clear;
    unsigned *pull_next, *pull_clear;
    double frac;                     // < 0: never a storm
    const int32_t *trp, *tcol;       // who hears each agent
    int64_t clk_t0;                  // SWARM_TICK_CLOCKS: the run's first tick
};

// Timers and writes of alive agent i after what it heard (h; r0: its record at the start of the tick,
// bits / y: after the receive), its sends listed.
__device__ __forceinline__ void finish_agent(int64_t i, Heard &h, uint2 r0, uint32_t bits, int32_t y, uint8_t prev,
                                             int64_t t, double now, double timeout, double jitter, uint64_t seed,
                                             const int32_t *__restrict__ ids, const Fsm &f,
                                             uint8_t *__restrict__ ob_out, int32_t *seg, int *s_ns, TickCounts &c) {
    uint8_t st = h.st;
    const int32_t ph = fw_phase(r0.x);
    const uint8_t ob = uint8_t(h.ob | timers(i, st, h.live, h.lead, h.lead_set, t, now, timeout, jitter, seed, ids,
                                             ph, f, bits, y));
    const uint32_t fw1 = fw_make(st, 1, bits, ph);
    if (fw1 != r0.x || uint32_t(y) != r0.y) f.rec[i] = make_uint2(fw1, uint32_t(y));
    if (h.lead_set) f.lrec[i].leader = h.lead;
    if (ob != prev) ob_out[i] = ob;
    if (ob) seg[atomicAdd(s_ns, 1)] = int32_t(i);  // this workgroup's sender segment (LDS counter)
    c.lead += st == ST_L;
    c.wait += st == ST_W;
    c.acc += (ob & kAcclaim) != 0;
    c.hb += (ob & kHeartbeat) != 0;
}

// k_tick at >= 7 waves per SIMD (72 VGPRs, a few spilled): 0.1111 ms per tick against 0.1142 at 6 (79 VGPRs)
// and 0.1194 at the compiler's 5 (82), 0.129 at 8 (64 VGPRs, 26 spilled); 6 row entries per chunk at 7
// waves 0.1110-0.1116, 4 entries 0.1181 at 7 / 0.1156 at 8 (same box; SWARM_TICK_WAVES=0: the compiler's
// choice, A/B aid)
#ifndef SWARM_TICK_WAVES
#define SWARM_TICK_WAVES 7
#endif
// Experiment aid (A/B builds with -DSWARM_TICK_CLOCKS=1): per tick and workgroup, the 100 MHz wall clock
// at its start, after its role's work (all threads: add_counts' barrier), after its storm decision and at
// its end, plus its sender count; written to SWARM_TICK_CLOCKS_FILE after the run.
#ifndef SWARM_TICK_CLOCKS
#define SWARM_TICK_CLOCKS 0
#endif
#if SWARM_TICK_CLOCKS
__device__ unsigned long long *g_tick_clk;
#define TICK_CLK(slot, v)                                                                        \
    do {                                                                                          \
        if (threadIdx.x == 0 && g_tick_clk)                                                       \
            g_tick_clk[((t - 1 - clk_t0) * int64_t(gridDim.x) + blockIdx.x) * 5 + (slot)] = (v);  \
    } while (0)
#else
#define TICK_CLK(slot, v) \
    do {                  \
    } while (0)
#endif
#if SWARM_TICK_WAVES
#define SWARM_TICK_BOUNDS __launch_bounds__(kBlock, SWARM_TICK_WAVES)
#else
#define SWARM_TICK_BOUNDS __launch_bounds__(kBlock)
#endif
__global__ SWARM_TICK_BOUNDS void k_tick(int64_t n, int64_t t, const int32_t *__restrict__ ids,
                                                const double2 *__restrict__ pos, const int32_t *__restrict__ rp,
                                                const int32_t *__restrict__ col,
                                                Fsm f, Mail mail, const uint8_t *__restrict__ ob_in,
                                                uint8_t *__restrict__ ob_out, const unsigned *__restrict__ pull,
                                                Segs segs, double dt, double timeout,
                                                double jitter, uint64_t seed, unsigned long long *__restrict__ counts,
                                                int vec, unsigned long long *__restrict__ tr, NextMail im, int xg) {
    __shared__ unsigned s_cnt[4];
    __shared__ int s_ns;
    __shared__ int s_wave[kBlock / kWave];
    __shared__ uint32_t s_list[kRecvChunk];  // receive role: the chunk's receivers (agent | multi bit 31)
    static_assert(kRecvChunk % kBlock == 0 && kRecvChunk / kBlock <= 16, "receive slice: <= 16 bits of a word");
    if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_ns = 0;
#if SWARM_TICK_CLOCKS
    const int64_t clk_t0 = im.clk_t0;
#endif
    TICK_CLK(0, wall_clock64());
    __syncthreads();
#ifndef SWARM_SWEEP_FIRST  // A/B aid: the sweep role's workgroups dispatched before the receive role's
#define SWARM_SWEEP_FIRST 0
#endif
    // the workgroup's place in the role order (receive role first)
    const int lb = SWARM_SWEEP_FIRST ? (int(blockIdx.x) < int(gridDim.x) - segs.g_recv
                                            ? int(blockIdx.x) + segs.g_recv
                                            : int(blockIdx.x) - (int(gridDim.x) - segs.g_recv))
                                     : int(blockIdx.x);
    int32_t *seg = segs.of(lb);
    const int g_recv = segs.g_recv;
    // receive-role workgroups first: dispatched first, all their chains in flight at once (every
    // R-th workgroup instead, the roles side by side: 0.151 vs 0.138 ms per tick)
    const bool recv_role = lb < g_recv;
    const int rank = recv_role ? lb : lb - g_recv;
    const double now = double(t) * dt;
    const bool pulled = *pull != 0;
    TickCounts c;
    int64_t span = 0;  // agents of this workgroup's share (the storm rule)
    if (pulled || recv_role) {
        // ---- receive role
        // a pulled tick: every workgroup, 1 024-agent units (every agent walks its row: 4x the units,
        // a quarter of the row walks one after the other per thread)
        const int64_t nrole = pulled ? int64_t(gridDim.x) : int64_t(g_recv);
        const int kPerT = pulled ? kRecvChunk / 4 / kBlock : kRecvChunk / kBlock;  // agents per thread
        const int64_t unit = int64_t(kPerT) * kBlock;
        const int64_t nchunks = (n + unit - 1) / unit;
        // xg > 0: groups of xg chunks (4 xg units on a pulled tick) dealt round robin to the 8 XCDs
        // (workgroup r runs on XCD r % 8 under round-robin dispatch), so a receiver's neighbours -- in the
        // chunks around its own -- are mostly fetched into the L2 of the XCD that serves it
        const int64_t me = pulled ? int64_t(lb) : int64_t(rank);
        const int64_t gsz = pulled ? 4 * int64_t(xg) : int64_t(xg);
        const int64_t nl = nrole / 8, xcd = me % 8, l = me / 8;
        for (int64_t q = xg ? l : me;; q += xg ? nl : nrole) {
            int64_t ck = q;
            if (xg) {
                const int64_t gi = xcd + 8 * (q / gsz);
                if (gi * gsz >= nchunks) break;
                ck = gi * gsz + q % gsz;
                if (ck >= nchunks) continue;
            } else if (ck >= nchunks) {
                break;
            }
            span += unit;
            // thread: kPerT agents, a slice of mail word (ck * unit + threadIdx.x * kPerT) / 64
            const int64_t a0 = ck * unit + int64_t(threadIdx.x) * kPerT;
            unsigned b16 = 0, m16 = 0;
            if (a0 < n) {
                const unsigned valid = n - a0 >= kPerT ? (1u << kPerT) - 1u : ((1u << (n - a0)) - 1u);
                if (pulled) {
                    b16 = valid;  // every agent (the dead ones clear their outbox)
                    m16 = valid;
                } else {
                    const int64_t w = a0 >> 6;
                    const int sh = int(a0 & 63);
                    b16 = unsigned(mail.bits[w] >> sh) & valid;
                    if (b16) m16 = unsigned(mail.multi[w] >> sh) & b16;
                }
            }
            int total;
            int pos_ = block_excl_scan<5>(__popc(b16), total, s_wave);
            while (b16) {
                const int q = __ffs(b16) - 1;
                b16 &= b16 - 1;
                s_list[pos_++] = uint32_t(a0 + q) | (((m16 >> q) & 1u) ? 0x80000000u : 0u);
            }
            __syncthreads();
            for (int q = threadIdx.x; q < total; q += kBlock) {
                const uint32_t entry = s_list[q];
                const int64_t i = int32_t(entry & 0x7FFFFFFFu);
                const bool multi = (entry & 0x80000000u) != 0;
                // the receiver's fields and its single sender, all loads at once (no load behind the
                // alive test), then the sender's outbox, ID and position at once
                const uint8_t prev = ob_out[i];
                const uint2 r = f.rec[i];
                const int32_t me = ids[i];
                const int32_t j = multi ? 0 : mail.from[i];
                if (!fw_alive(r.x)) {
                    if (prev) ob_out[i] = 0;
                    continue;
                }
                Heard h{fw_state(r.x), 0, false, false, 0, -1};
                uint32_t bits = fw_bits(r.x);
                int32_t y = int32_t(r.y);
                const bool hb_tick = ((t + fw_phase(r.x)) % 10) == 0;
                if (multi) {  // several senders (or a pull): the row, in CSR order
                    const int32_t b = rp[i], e = rp[i + 1];
                    receive_row<kRecvTick>(b, e, col, ob_in, ids, me, hb_tick, h);
                    ++c.multi;
                    c.edges += unsigned(e - b);
                    apply_heard(i, h, t, pos, f, bits, y);
                } else {  // exactly one sender: no row walk
                    const uint8_t o = ob_in[j] & (kAcclaim | kHeartbeat);
                    const int32_t sid = ids[j];
                    const double2 sp = pos[j];  // used when its heartbeat is accepted (hb_from = j)
                    if (o) hear(h, o, sid, j, me, hb_tick);
                    ++c.single;
                    if (h.live) {
                        y = int32_t(t - f.t0);
                        bits = (bits & ~kH64) | kDirty;
                    }
                    if (h.hb_from >= 0) {
                        set_lpos(f, i, float(sp.x), float(sp.y));
                        bits |= kHL;
                    }
                }
                finish_agent(i, h, r, bits, y, prev, t, now, timeout, jitter, seed, ids, f, ob_out, seg, &s_ns, c);
            }
            __syncthreads();  // the list is reused
        }
    } else {
        // ---- sweep role
        const int64_t ngroups = (n + kSweepV - 1) / kSweepV;
        const int64_t stride = int64_t(int(gridDim.x) - g_recv) * kBlock;
        {  // the workgroup's groups (uniform)
            const int64_t g0 = int64_t(rank) * kBlock;
            span = g0 < ngroups ? ((ngroups - g0 + stride - 1) / stride) * kBlock * kSweepV : 0;
        }
        for (int64_t gi = int64_t(rank) * kBlock + threadIdx.x; gi < ngroups; gi += stride) {
            const int64_t i0 = gi * kSweepV;
            const bool full = vec && i0 + kSweepV <= n;
            uint2 rv[kSweepV];
            uint8_t pv[kSweepV];
            const unsigned mine = unsigned(mail.bits[i0 >> 6] >> (i0 & 63)) & ((1u << kSweepV) - 1u);
            if (full) {  // vec: the host checked the outbox's alignment; i0 is a multiple of 4 (records: scratch)
#pragma unroll
                for (int q = 0; q < kSweepV / 2; ++q) {
                    const uint4 r2 = *reinterpret_cast<const uint4 *>(f.rec + i0 + 2 * q);
                    rv[2 * q] = make_uint2(r2.x, r2.y);
                    rv[2 * q + 1] = make_uint2(r2.z, r2.w);
                }
#pragma unroll
                for (int q = 0; q < kSweepV / 4; ++q) {
                    const uint32_t wp = *reinterpret_cast<const uint32_t *>(ob_out + i0 + 4 * q);
#pragma unroll
                    for (int v = 0; v < 4; ++v) pv[4 * q + v] = uint8_t(wp >> (8 * v));
                }
            } else {
#pragma unroll
                for (int v = 0; v < kSweepV; ++v) {
                    const int64_t i = i0 + v < n ? i0 + v : n - 1;
                    rv[v] = i0 + v < n ? f.rec[i] : make_uint2(0u, 0u);  // past n: not alive
                    pv[v] = ob_out[i];
                }
            }
#pragma unroll
            for (int v = 0; v < kSweepV; ++v) {
                const int64_t i = i0 + v;
                if ((mine >> v) & 1u) continue;  // a receiver: the receive role's
                const uint8_t prev = pv[v];      // this slot's byte from tick t-2
                if (!fw_alive(rv[v].x)) {
                    if (i < n && prev) ob_out[i] = 0;
                    continue;
                }
                Heard h{fw_state(rv[v].x), 0, false, false, 0, -1};
                finish_agent(i, h, rv[v], fw_bits(rv[v].x), int32_t(rv[v].y), prev, t, now, timeout, jitter, seed,
                             ids, f, ob_out, seg, &s_ns, c);
            }
        }
    }
    if (tr) {
        add_traffic(tr, pulled ? 5 : 0, pulled ? 0ull : c.single);
        add_traffic(tr, pulled ? 6 : 1, c.multi);
        add_traffic(tr, 2, c.edges);
        if (pulled && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&tr[7], 1ull);  // pulled ticks
    }
    add_counts(c.lead, c.wait, c.acc, c.hb, s_cnt, counts);  // (ends with a barrier: s_ns is final)
    TICK_CLK(1, wall_clock64());
    for (int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x; q < im.n_clear; q += int64_t(gridDim.x) * kBlock)
        if (im.clear[q]) im.clear[q] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *im.pull_clear = 0;
    const int ns = s_ns;
    TICK_CLK(4, (unsigned long long)ns | ((unsigned long long)recv_role << 40) | ((unsigned long long)pulled << 41));
    TICK_CLK(2, wall_clock64());
    if (im.frac >= 0.0 && double(ns) > im.frac * double(span)) {
        if (threadIdx.x == 0) *im.pull_next = 1u;
        TICK_CLK(3, wall_clock64());
        return;
    }
    // the segment was written by this workgroup's threads before add_counts' barrier
    unsigned long long c_edges = 0;
    for (int q = threadIdx.x; q < ns; q += kBlock) {
        const int32_t i = seg[q];
        const int32_t b = im.trp[i], e = im.trp[i + 1];
        mail_hearers(b, e, im.tcol, im.next, i);
        c_edges += uint64_t(e - b);
    }
    if (tr) {
        add_traffic(tr, 3, threadIdx.x < unsigned(ns) ? uint64_t((ns - int(threadIdx.x) + kBlock - 1) / kBlock) : 0ull);
        add_traffic(tr, 4, c_edges);
    }
#if SWARM_TICK_CLOCKS
    __syncthreads();
#endif
    TICK_CLK(3, wall_clock64());
}

// traffic shards -> out[kTraffic]
__global__ void k_sum_traffic(const unsigned long long *__restrict__ tr, unsigned long long *__restrict__ out) {
    if (threadIdx.x < kTraffic) {
        unsigned long long v = 0;
        for (int sh = 0; sh < kShards; ++sh) v += tr[sh * kTraffic + threadIdx.x];
        out[threadIdx.x] = v;
    }
}

}  // namespace
}  // namespace swarm

extern "C" {

int swarm_protocol_run(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *pos, const int32_t *row_ptr,
                       const int32_t *col, const int32_t *hear_row_ptr, const int32_t *hear_col,
                       const int32_t *tick_off, const swarm_fsm *fsm, int64_t t0, int32_t ticks,
                       double dt, double timeout, double jitter, uint64_t seed, const int64_t *kill_ticks,
                       int32_t n_kill, int64_t *counts, void *stream) {
    return swarm_protocol_run_ex(ctx, n, ids, pos, row_ptr, col, hear_row_ptr, hear_col, tick_off, fsm, t0, ticks, dt,
                                 timeout, jitter, seed, kill_ticks, n_kill, -1.0, counts, nullptr, stream);
}

int swarm_protocol_run_ex(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *pos, const int32_t *row_ptr,
                          const int32_t *col, const int32_t *hear_row_ptr, const int32_t *hear_col,
                          const int32_t *tick_off, const swarm_fsm *fsm, int64_t t0, int32_t ticks,
                          double dt, double timeout, double jitter, uint64_t seed, const int64_t *kill_ticks,
                          int32_t n_kill, double pull_frac, int64_t *counts, int64_t *traffic, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && fsm != nullptr, "NULL argument");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) && ticks >= 0 && t0 >= 0 && n_kill >= 0, "sizes out of range");
    SW_ARG(n_kill == 0 || kill_ticks != nullptr, "kill_ticks is NULL");
    SW_ARG(std::isfinite(dt) && timeout >= 0.0 && jitter >= 0.0, "dt / timeout / jitter out of range");
    SW_ARG(hear_row_ptr != nullptr || hear_col == nullptr, "hear_col without hear_row_ptr");
    SW_ARG(n == 0 || (ids && pos && row_ptr && tick_off && fsm->state && fsm->leader && fsm->last_hb &&
                      fsm->wait_start && fsm->delay && fsm->leader_pos && fsm->has_leader_pos && fsm->alive &&
                      fsm->outbox),
           "NULL agent array");
    SW_ARG(!std::isnan(pull_frac), "pull_frac is NaN");
    if (traffic) for (int q = 0; q < kTraffic; ++q) traffic[q] = 0;
    if (n == 0 || ticks == 0) {
        if (counts) for (int64_t q = 0; q < int64_t(ticks) * 4; ++q) counts[q] = 0;
        return SWARM_OK;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *d_cnt;  // per tick: kShards x 4 partial counters, then the 4 sums
    const size_t part_bytes = size_t(ticks) * kShards * 4 * 8;
    const size_t tr_bytes = size_t(kShards) * kTraffic * 8;
    SW_ALLOC(d_cnt, ctx, S_TMP0, part_bytes + size_t(ticks) * 4 * 8 + tr_bytes + kTraffic * 8);
    SW_HIP(hipMemsetAsync(d_cnt, 0, part_bytes, s));
    unsigned long long *d_sum = d_cnt + size_t(ticks) * kShards * 4;
    unsigned long long *d_tr = traffic ? d_sum + size_t(ticks) * 4 : nullptr;
    if (d_tr) SW_HIP(hipMemsetAsync(d_tr, 0, tr_bytes, s));
    // the run's records (flag word + timer tick, leader + leader position; unpacked into the caller's arrays
    // at the end of the run)
    uint8_t *recs;
    SW_ALLOC(recs, ctx, S_FSM_FLAGS, size_t(n) * 24);
    const Fsm f{reinterpret_cast<uint2 *>(recs), reinterpret_cast<LRec *>(recs + size_t(n) * 8), fsm->last_hb,
                fsm->wait_start, fsm->delay, t0, t0 + ticks, dt};
    // the sweep role's grid: 2 560 workgroups at most, with half as many in the receive role (10M
    // agents, one-launch ticks, two boxes: 0.1208-0.1212 ms per tick against 0.1232-0.1234 for
    // 2 048 + 1 280, 0.122 for 1 536 + 1 280, 2 560 + 1 536 and 3 072 + 1 280; the two-launch form
    // had 2 048 + 1 280 at 0.128, 4 096 + 2 048 at 0.131; SWARM_FSM_SWEEP_WGS overrides, A/B aid)
    static const int sweep_env = [] {
        const char *e = getenv("SWARM_FSM_SWEEP_WGS");
        return e ? atoi(e) : 0;
    }();
    const unsigned grid = grid_for(n, kBlock, sweep_env > 0 ? unsigned(sweep_env) : 2560u);
    auto a16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    // the sweep's word loads: the outbox 4-byte aligned (the tick's half too; records: scratch)
    const int vec = a16(fsm->outbox) && a16(recs);
    SW_ARG((reinterpret_cast<uintptr_t>(fsm->leader_pos) & 7) == 0, "leader_pos is not 8-byte aligned");
    hipLaunchKernelGGL(k_pack_fsm, dim3(grid), dim3(kBlock), 0, s, n, fsm->state, fsm->alive, fsm->has_leader_pos,
                       tick_off, fsm->leader, reinterpret_cast<const float2 *>(fsm->leader_pos), f);
    SW_LAUNCHED();
    const bool push = hear_row_ptr != nullptr;
    const int64_t n_words = (n + 63) / 64;
    Mail mail{};
    Segs segs{};
    unsigned *pullf = nullptr;
    constexpr int nbuf = 3;            // mail word buffers, rotated by tick (NextMail)
    unsigned long long *mw = nullptr;  // buffer b: mail bits at mw + 2b n_words, multi bits after them
    int32_t *from_base = nullptr;      // single-sender slots, two buffers by tick parity
    auto mail_of = [&](int64_t tick) {  // the mail a tick receives
        Mail m = mail;
        m.bits = mw + size_t(tick % nbuf) * 2 * size_t(n_words);
        m.multi = m.bits + n_words;
        m.from = from_base + size_t(tick & 1) * size_t(n);
        return m;
    };
    // k_tick's receive role: a workgroup per 4 096-agent chunk, at most half the sweep grid (10M
    // agents: 1 280 of 2 442 chunks' workgroups; two-launch form, sweep grid 2 048: 1 280 -> 0.1279
    // ms per tick, 1 536 -> 0.1281, 2 048 -> 0.1298, 1 024 -> 0.1303; sweep grid 4 096: 2 048 ->
    // 0.138, 512 -> 0.160, 256 -> 0.214; SWARM_FSM_RECV_WGS overrides, A/B aid)
    static const int recv_env = [] {
        const char *e = getenv("SWARM_FSM_RECV_WGS");
        return e ? atoi(e) : 0;
    }();
    const int64_t nchunks_all = (n + kRecvChunk - 1) / kRecvChunk;
    const int g_recv = int(std::max<int64_t>(
        1, std::min<int64_t>(nchunks_all, recv_env > 0 ? recv_env : std::max<int64_t>(1, int64_t(grid) / 2))));
    const unsigned tgrid = grid + unsigned(g_recv);  // k_tick: both roles
    // the receive role's XCD-grouped chunk order (SWARM_TICK_XCD_GROUP chunks per group, 0 = plain
    // grid stride); only when both role grids split evenly over the 8 XCDs
    static const int xg_env = [] {
        const char *e = getenv("SWARM_TICK_XCD_GROUP");
        return e ? atoi(e) : 0;
    }();
    const int xg = (xg_env > 0 && g_recv % 8 == 0 && tgrid % 8 == 0) ? xg_env : 0;
    if (push) {  // mail bitmaps (nbuf buffers) + the pull flags (by tick, nbuf) after them
        SW_ALLOC(mw, ctx, S_FSM_MAIL, size_t(n_words) * 48 + 64);
        SW_ALLOC(from_base, ctx, S_FSM_FROM, size_t(n) * 8);
        // per-workgroup sender segments of k_tick (each workgroup lists at most the agents it sees:
        // a grid-stride share of kSweepV-agent groups, or of 4 096-agent chunks), then their counts
        const int64_t ngroups = (n + kSweepV - 1) / kSweepV;
        const int64_t nchunks = (n + kRecvChunk - 1) / kRecvChunk;
        segs.g_recv = g_recv;
        segs.rcap = (nchunks + g_recv - 1) / g_recv * kRecvChunk;
        segs.scap = std::max((ngroups + int64_t(grid) * kBlock - 1) / (int64_t(grid) * kBlock) * kBlock * kSweepV,
                             (nchunks + tgrid - 1) / tgrid * kRecvChunk);
        if (xg) {  // the grouped order may deal a workgroup more chunks than the grid stride: its segment holds them
            auto most = [&](int64_t nch, int64_t g, int64_t nrole) {  // max chunks of one workgroup
                const int64_t ngr = (nch + g - 1) / g;
                int64_t worst = 0;
                for (int64_t x = 0; x < 8; ++x) {
                    const int64_t full = ngr > x ? (ngr - 1 - x) / 8 + 1 : 0;  // groups of XCD x
                    int64_t cx = full * g;
                    if (full && (x + 8 * (full - 1)) == ngr - 1) cx -= ngr * g - nch;  // its last group is partial
                    worst = std::max(worst, (cx + nrole / 8 - 1) / (nrole / 8));
                }
                return worst;
            };
            segs.rcap = std::max(segs.rcap, most(nchunks, xg, g_recv) * kRecvChunk);
            const int64_t unit = kRecvChunk / 4, nunits = (n + unit - 1) / unit;
            segs.scap = std::max(segs.scap, most(nunits, 4 * int64_t(xg), tgrid) * unit);
            segs.rcap = std::max(segs.rcap, segs.scap);  // a pulled tick: the receive-role workgroups too
        }
        const size_t seg_total = size_t(g_recv) * segs.rcap + size_t(grid) * segs.scap;
        SW_ALLOC(segs.base, ctx, S_FSM_SEND, seg_total * 4);
        pullf = reinterpret_cast<unsigned *>(mw + 6 * n_words);  // [nbuf] by tick: the tick pulls
        SW_HIP(hipMemsetAsync(mw, 0, size_t(n_words) * 48 + 64, s));
        hipLaunchKernelGGL(k_mail_from_outbox, dim3(grid), dim3(kBlock), 0, s, n,
                           fsm->outbox + size_t(t0 & 1) * size_t(n), hear_row_ptr, hear_col, mail_of(t0 + 1));
        SW_LAUNCHED();
    }
#if SWARM_TICK_CLOCKS
    unsigned long long *clk_buf = nullptr;
    const char *clk_file = getenv("SWARM_TICK_CLOCKS_FILE");
    if (push && clk_file) {
        SW_HIP(hipMalloc(&clk_buf, size_t(ticks) * tgrid * 5 * 8));
        SW_HIP(hipMemsetAsync(clk_buf, 0, size_t(ticks) * tgrid * 5 * 8, s));
    }
    SW_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tick_clk), &clk_buf, sizeof(clk_buf), 0, hipMemcpyHostToDevice, s));
#endif
    for (int64_t t = t0 + 1; t <= t0 + ticks; ++t) {
        bool kill = false;
        for (int32_t k = 0; k < n_kill; ++k) kill |= kill_ticks[k] == t;
        if (kill) {
            hipLaunchKernelGGL(k_kill_leaders, dim3(grid), dim3(kBlock), 0, s, n, f.rec);
            SW_LAUNCHED();
        }
        const uint8_t *ob_in = fsm->outbox + size_t((t - 1) & 1) * size_t(n);
        uint8_t *ob_out = fsm->outbox + size_t(t & 1) * size_t(n);
        unsigned long long *cnt = d_cnt + size_t(t - t0 - 1) * kShards * 4;
        if (push) {
            NextMail im{};
            im.next = mail_of(t + 1);
            im.clear = mail_of(t + 2).bits;
            im.n_clear = 2 * n_words;
            im.pull_next = pullf + (t + 1) % nbuf;
            im.pull_clear = pullf + (t + 2) % nbuf;
            im.frac = pull_frac < 0.0 ? -1.0 : pull_frac;
            im.trp = hear_row_ptr;
            im.tcol = hear_col;
            im.clk_t0 = t0;
            hipLaunchKernelGGL(k_tick, dim3(tgrid), dim3(kBlock), 0, s, n, t, ids,
                               reinterpret_cast<const double2 *>(pos), row_ptr, col, f, mail_of(t), ob_in,
                               ob_out, pullf + t % nbuf, segs, dt, timeout, jitter, seed, cnt,
                               int(vec && (reinterpret_cast<uintptr_t>(ob_out) & 3) == 0), d_tr, im, xg);
        } else {
            hipLaunchKernelGGL(k_tick_pull, dim3(grid), dim3(kBlock), 0, s, n, t, ids,
                               reinterpret_cast<const double2 *>(pos), row_ptr, col, f, ob_in, ob_out, dt,
                               timeout, jitter, seed, cnt);
        }
        SW_LAUNCHED();
    }
#if SWARM_TICK_CLOCKS
    if (clk_buf) {  // experiment aid: header (ticks, workgroups, receive-role workgroups) + the records
        std::vector<unsigned long long> hc(size_t(ticks) * tgrid * 5);
        SW_HIP(hipMemcpyAsync(hc.data(), clk_buf, hc.size() * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        SW_HIP(hipFree(clk_buf));
        if (FILE *fp = fopen(clk_file, "wb")) {
            const long long hdr[3] = {ticks, (long long)tgrid, g_recv};
            fwrite(hdr, 8, 3, fp);
            fwrite(hc.data(), 8, hc.size(), fp);
            fclose(fp);
        }
    }
#endif
    hipLaunchKernelGGL(k_unpack_fsm, dim3(grid), dim3(kBlock), 0, s, n, fsm->state, fsm->alive, fsm->has_leader_pos,
                       fsm->leader, reinterpret_cast<float2 *>(fsm->leader_pos), f);
    SW_LAUNCHED();
    if (d_tr) {  // pull-mode runs: every tick walks every row (the receivers are all agents)
        unsigned long long *hs = static_cast<unsigned long long *>(pinned(ctx, kTraffic * 8));
        if (!hs) return SWARM_ERR_OOM;
        hipLaunchKernelGGL(k_sum_traffic, dim3(1), dim3(kWave), 0, s, d_tr, d_tr + size_t(kShards) * kTraffic);
        SW_LAUNCHED();
        SW_HIP(hipMemcpyAsync(hs, d_tr + size_t(kShards) * kTraffic, kTraffic * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < kTraffic; ++q) traffic[q] = int64_t(hs[q]);
    }
    if (counts) {
        hipLaunchKernelGGL(k_sum_counts, dim3(grid_for(int64_t(ticks) * 4, kBlock, 256)), dim3(kBlock), 0, s,
                           int64_t(ticks), d_cnt, d_sum);
        SW_LAUNCHED();
        SW_HIP(hipMemcpyAsync(counts, d_sum, size_t(ticks) * 4 * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
    }
    return SWARM_OK;
}

}  // extern "C"
