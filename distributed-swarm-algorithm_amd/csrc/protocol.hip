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
// A tick reads, per agent, its ~24 B of state plus a CSR row (4 B per edge) and one outbox byte
// per neighbour (spatially ordered agents: mostly L2 hits); sender IDs and positions are read
// only for neighbours that sent something.  HBM-bound, no arithmetic worth the name.
// Agents killed at a kill tick (every alive LEADER then) stop receiving and sending.
#include "swarm_common.h"

namespace swarm {
namespace {

constexpr uint8_t kAcclaim = 1, kHeartbeat = 2;
constexpr uint8_t ST_F = SWARM_FOLLOWER, ST_W = SWARM_ELECTION_WAIT, ST_L = SWARM_LEADER;

__device__ __forceinline__ double jitter_u(uint64_t seed, int32_t id, int64_t t) {
    uint64_t x = seed ^ (uint64_t(uint32_t(id)) * 0x9E3779B97F4A7C15ull) ^ (uint64_t(t) * 0xD1B54A32D192ED03ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return double(x >> 11) * (1.0 / 9007199254740992.0);
}

struct Fsm {
    uint8_t *state;
    int32_t *leader;
    double *last_hb, *wait_start, *delay;
    float2 *lpos;
    uint8_t *has_lpos, *alive;
};

__global__ __launch_bounds__(kBlock) void k_kill_leaders(int64_t n, const uint8_t *__restrict__ state,
                                                        uint8_t *__restrict__ alive) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
        if (alive[i] && state[i] == ST_L) alive[i] = 0;
}

__global__ __launch_bounds__(kBlock) void k_tick(int64_t n, int64_t t, const int32_t *__restrict__ ids,
                                                const double2 *__restrict__ pos, const int32_t *__restrict__ rp,
                                                const int32_t *__restrict__ col,
                                                const int32_t *__restrict__ tick_off, Fsm f,
                                                const uint8_t *__restrict__ ob_in, uint8_t *__restrict__ ob_out,
                                                double dt, double timeout, double jitter, uint64_t seed,
                                                unsigned long long *__restrict__ counts) {
    __shared__ unsigned s_cnt[4];
    if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const double now = double(t) * dt;
    unsigned c_lead = 0, c_wait = 0, c_acc = 0, c_hb = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        if (!f.alive[i]) {
            ob_out[i] = 0;
            continue;
        }
        const int32_t me = ids[i];
        const bool hb_tick = ((t + tick_off[i]) % 10) == 0;
        uint8_t st = f.state[i], ob = 0;
        const uint8_t st0 = st;
        int32_t lead = f.leader[i];
        const int32_t lead0 = lead;
        bool live = false, pos_set = false;
        float2 lp;
        for (int32_t k = rp[i], e = rp[i + 1]; k < e; ++k) {
            const int32_t j = col[k];
            const uint8_t o = ob_in[j];
            if (!o) continue;
            const int32_t s = ids[j];
            if (o & kAcclaim) {
                if (s > me) {
                    live = true;
                } else if (s < me && (st == ST_L || st == ST_W)) {
                    if (hb_tick) ob |= kHeartbeat;  // bully back (state/leader: overwritten below)
                }
                lead = s;  // COORDINATOR: unconditional takeover
                st = ST_F;
                live = true;
            }
            if (o & kHeartbeat) {
                if (st == ST_L && s < me) {
                    if (hb_tick) ob |= kHeartbeat;
                } else {
                    st = ST_F;  // yield (LEADER) / stop waiting (ELECTION_WAIT) / stay FOLLOWER
                    lead = s;
                    live = true;
                    const double2 q = pos[j];
                    lp = make_float2(float(q.x), float(q.y));
                    pos_set = true;
                }
            }
        }
        if (live) f.last_hb[i] = now;
        if (pos_set) {
            f.lpos[i] = lp;
            f.has_lpos[i] = 1;
        }
        if (st != ST_L) {
            if (st == ST_F && now - (live ? now : f.last_hb[i]) > timeout) {
                st = ST_W;
                f.wait_start[i] = now;
                f.delay[i] = 0.0 + jitter * jitter_u(seed, me, t);
                lead = -1;
                f.has_lpos[i] = 0;
                f.lpos[i] = make_float2(0.f, 0.f);
            }
            if (st == ST_W && now - f.wait_start[i] > f.delay[i]) {
                st = ST_L;
                lead = me;
                ob |= kAcclaim;
            }
        }
        if (st == ST_L && hb_tick) ob |= kHeartbeat;
        if (st != st0) f.state[i] = st;
        if (lead != lead0) f.leader[i] = lead;
        ob_out[i] = ob;
        c_lead += st == ST_L;
        c_wait += st == ST_W;
        c_acc += (ob & kAcclaim) != 0;
        c_hb += (ob & kHeartbeat) != 0;
    }
    // wave reduce, then one LDS atomic per wave and one global atomic per workgroup
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        c_lead += __shfl_xor(c_lead, off, 64);
        c_wait += __shfl_xor(c_wait, off, 64);
        c_acc += __shfl_xor(c_acc, off, 64);
        c_hb += __shfl_xor(c_hb, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_cnt[0], c_lead);
        atomicAdd(&s_cnt[1], c_wait);
        atomicAdd(&s_cnt[2], c_acc);
        atomicAdd(&s_cnt[3], c_hb);
    }
    __syncthreads();
    if (threadIdx.x < 4 && s_cnt[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)s_cnt[threadIdx.x]);
}

}  // namespace
}  // namespace swarm

extern "C" {

int swarm_protocol_run(swarm_ctx *ctx, int64_t n, const int32_t *ids, const double *pos, const int32_t *row_ptr,
                       const int32_t *col, const int32_t *tick_off, const swarm_fsm *fsm, int64_t t0, int32_t ticks,
                       double dt, double timeout, double jitter, uint64_t seed, const int64_t *kill_ticks,
                       int32_t n_kill, int64_t *counts, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr && fsm != nullptr, "NULL argument");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) && ticks >= 0 && t0 >= 0 && n_kill >= 0, "sizes out of range");
    SW_ARG(n_kill == 0 || kill_ticks != nullptr, "kill_ticks is NULL");
    SW_ARG(n == 0 || (ids && pos && row_ptr && tick_off && fsm->state && fsm->leader && fsm->last_hb &&
                      fsm->wait_start && fsm->delay && fsm->leader_pos && fsm->has_leader_pos && fsm->alive &&
                      fsm->outbox),
           "NULL agent array");
    if (n == 0 || ticks == 0) {
        if (counts) for (int64_t q = 0; q < int64_t(ticks) * 4; ++q) counts[q] = 0;
        return SWARM_OK;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned long long *d_cnt;
    SW_ALLOC(d_cnt, ctx, S_TMP0, size_t(ticks) * 4 * 8);
    SW_HIP(hipMemsetAsync(d_cnt, 0, size_t(ticks) * 4 * 8, s));
    const Fsm f{fsm->state, fsm->leader, fsm->last_hb, fsm->wait_start, fsm->delay,
                reinterpret_cast<float2 *>(fsm->leader_pos), fsm->has_leader_pos, fsm->alive};
    const unsigned grid = grid_for(n, kBlock, 4096);
    for (int64_t t = t0 + 1; t <= t0 + ticks; ++t) {
        bool kill = false;
        for (int32_t k = 0; k < n_kill; ++k) kill |= kill_ticks[k] == t;
        if (kill) {
            hipLaunchKernelGGL(k_kill_leaders, dim3(grid), dim3(kBlock), 0, s, n, fsm->state, fsm->alive);
            SW_LAUNCHED();
        }
        const uint8_t *ob_in = fsm->outbox + size_t((t - 1) & 1) * size_t(n);
        uint8_t *ob_out = fsm->outbox + size_t(t & 1) * size_t(n);
        hipLaunchKernelGGL(k_tick, dim3(grid), dim3(kBlock), 0, s, n, t, ids,
                           reinterpret_cast<const double2 *>(pos), row_ptr, col, tick_off, f, ob_in, ob_out, dt,
                           timeout, jitter, seed, d_cnt + 4 * (t - t0 - 1));
        SW_LAUNCHED();
    }
    if (counts) {
        SW_HIP(hipMemcpyAsync(counts, d_cnt, size_t(ticks) * 4 * 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
    }
    return SWARM_OK;
}

}  // extern "C"
