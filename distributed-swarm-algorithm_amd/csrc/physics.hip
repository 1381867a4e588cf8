// Physics / formation step on gfx950.
//
// Replaces SwarmAgent._update_physics (agent.py:94-181) run by every agent of the swarm, as one
// synchronous step (contract P1, tools/gen_golden.py): every agent reads the step-start snapshot
// of all positions (pos_in) and writes its new position to pos_out (double-buffered), so the
// result does not depend on the order agents are updated in.
//   formation  a FOLLOWER with a leader targets its V slot behind the leader's position as the
//              heartbeat carries it ('!ff': f32-rounded, agent.py:256-258, 283-289):
//              x - 2 id, y + 2 id (even id) / y - 2 id (odd id)  (agent.py:96-111)
//   forces     attraction to the target beyond 0.5 (118-125); obstacle repulsion, obstacles in
//              list order (128-146); neighbour separation within 2.0, neighbours in CSR order
//              (149-160) -- sums in the reference's order, so the result is bit-exact against
//              the CPU restatement's x*x arithmetic (the reference squares with libm pow: <= 1
//              ulp per square, checked with a tolerance against its fixtures)
//   update     speed clamp to max_speed (169-174), Euler step (177-178).
// One thread per agent (fp64 VALU + the neighbour gathers; the snapshot of the neighbourhood is
// the HBM traffic: 16 B per edge + 80 B per agent); obstacles staged in LDS per workgroup.
// A zero distance to an obstacle centre or a neighbour makes the reference raise
// ZeroDivisionError; here it yields non-finite values and is counted (n_singular).
#include <cmath>

#include "swarm_common.h"

namespace swarm {
namespace {

constexpr int kObsLds = 1024;  // obstacles staged in LDS per pass (3 doubles each)
#ifndef SWARM_PHYS_NB
#define SWARM_PHYS_NB 6
#endif
constexpr int kNb = SWARM_PHYS_NB;  // neighbour positions in flight per thread (6: 0.869-0.879 ms, 4: 0.898, 8: 0.92; r5 physics_nb_ab.log)

// Correctly rounded f64 division and square root, written out as LLVM expands them for gfx950 but
// without their range steps (div_scale / div_fmas scaling / div_fixup; the ldexp pre-scale and class
// test of sqrt), which are the identity when every operand and result is normal and far from the
// exponent limits -- in_range() below, checked by the caller, who falls back to '/' and sqrt()
// otherwise.  Same instructions on the same operands: the same bits.  (Round 5: the separation
// terms' three divisions and square root were ~60 % of k_physics' fp64 instructions; two divisions
// by the same norm share its refined reciprocal.)
#ifndef SWARM_PHYS_LIBM
#define SWARM_PHYS_LIBM 0  // 1: the library '/' and sqrt() everywhere (A/B builds)
#endif
__device__ __forceinline__ bool in_range(double x) {
    const double a = fabs(x);
    return a >= 0x1p-500 && a <= 0x1p500;  // (false for 0, denormals, inf, NaN)
}
__device__ __forceinline__ double rcp_refined(double den) {  // v_rcp_f64 + two Newton steps
    double r = __builtin_amdgcn_rcp(den);
    double e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-den, r, 1.0);
    return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double div_by(double num, double den, double r) {  // num / den, r = rcp_refined(den)
    const double q = num * r;
    const double rem = __builtin_fma(-den, q, num);
    return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double sqrt_core(double x) {  // v_rsq_f64 + Newton steps on (g, h)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}

__global__ __launch_bounds__(kBlock, 8) void k_physics(int64_t n, const int32_t *__restrict__ ids,
                                                   const uint8_t *__restrict__ state,
                                                   const int32_t *__restrict__ leader,
                                                   const double2 *__restrict__ pin, double2 *__restrict__ pout,
                                                   double2 *__restrict__ vel, double2 *__restrict__ tgt,
                                                   uint8_t *__restrict__ has_t, int64_t m,
                                                   const double *__restrict__ obs, const int32_t *__restrict__ rp,
                                                   const int32_t *__restrict__ col, double dt, double max_speed,
                                                   unsigned long long *__restrict__ singular) {
    __shared__ double s_obs[kObsLds * 3];
    unsigned long long sing = 0;
    for (int64_t base = int64_t(blockIdx.x) * kBlock; base < n; base += int64_t(gridDim.x) * kBlock) {
        const int64_t i = base + threadIdx.x;
        const bool valid = i < n;
        double px = 0, py = 0, frx = 0.0, fry = 0.0;
        bool moving = false;
        double2 t = make_double2(0, 0);
        if (valid) {
            const double2 p = pin[i];
            px = p.x;
            py = p.y;
            t = tgt[i];
            bool has = has_t[i] != 0;
            const int32_t L = leader[i];
            if (state[i] == SWARM_FOLLOWER && L >= 0) {
                const double2 lp = pin[L];
                const double lx = double(float(lp.x)), ly = double(float(lp.y));
                const double rank = double(ids[i]);
                const double xo = -2.0 * rank;
                const double yo = (ids[i] % 2 == 0) ? 2.0 * rank : -2.0 * rank;
                t = make_double2(lx + xo, ly + yo);
                tgt[i] = t;
                if (!has) has_t[i] = 1;
                has = true;
            }
            moving = has;
        }
        // obstacles: every workgroup stages them through LDS (all lanes join the barriers)
        for (int64_t o0 = 0; o0 < m; o0 += kObsLds) {
            const int64_t cnt = (m - o0 < kObsLds) ? m - o0 : kObsLds;
            __syncthreads();
            for (int64_t q = threadIdx.x; q < 3 * cnt; q += kBlock) s_obs[q] = obs[3 * o0 + q];
            __syncthreads();
            if (moving)
                for (int64_t o = 0; o < cnt; ++o) {
                    const double ox = s_obs[3 * o], oy = s_obs[3 * o + 1], r = s_obs[3 * o + 2];
                    const double ex = px - ox, ey = py - oy;
                    const double s2 = ex * ex + ey * ey;
                    // far obstacles (most): sqrt(s2) - r >= 5 for certain, so the exact test below could
                    // not apply the force -- skip its square root (the margin 1e-12 is far above the
                    // roundings of s2, the square root and the subtraction; NaN falls through)
                    const double rr = 5.0 + r;
                    if (s2 > rr * rr * (1.0 + 1e-12)) continue;
                    double d = sqrt(s2) - r;
                    if (d <= 0.001) d = 0.001;
                    if (d < 5.0) {
                        const double mag = 50.0 * (1.0 / d - 1.0 / 5.0) / (d * d);
                        const double nrm = sqrt(s2);
                        sing += nrm == 0.0;
                        frx += (ex / nrm) * mag;
                        fry += (ey / nrm) * mag;
                    }
                }
        }
        if (!moving) {  // keeps its position (in the output buffer too: synchronous step)
            if (valid) pout[i] = make_double2(px, py);
            continue;
        }
        double fax = 0.0, fay = 0.0;
        const double gx = t.x - px, gy = t.y - py;
        if (sqrt(gx * gx + gy * gy) > 0.5) {
            fax = 1.0 * gx;
            fay = 1.0 * gy;
        }
        double fsx = 0.0, fsy = 0.0;
        // the row in chunks of kNb: all column loads, then all position gathers in flight, then
        // the separation terms summed in CSR order (the reference's order: bit-exact)
        for (int32_t k0 = rp[i], e = rp[i + 1]; k0 < e; k0 += kNb) {
            int32_t jj[kNb];
#pragma unroll
            for (int u = 0; u < kNb; ++u) jj[u] = k0 + u < e ? col[k0 + u] : -1;
            double2 qq[kNb];
#pragma unroll
            for (int u = 0; u < kNb; ++u) qq[u] = jj[u] >= 0 ? pin[jj[u]] : make_double2(0.0, 0.0);
#pragma unroll
            for (int u = 0; u < kNb; ++u) {
                if (jj[u] < 0) continue;
                const double ex = px - qq[u].x, ey = py - qq[u].y;
                const double s2 = ex * ex + ey * ey;
                if (!SWARM_PHYS_LIBM && in_range(ex) && in_range(ey) && in_range(s2)) {
                    // both offsets nonzero and normal: the norm is in [2^-500, 2^251), d * d in
                    // [1e-6, 4), every quotient normal -- the range steps are the identity
                    const double nrm = sqrt_core(s2);
                    if (nrm < 2.0) {
                        const double d = nrm <= 0.001 ? 0.001 : nrm;
                        const double dd = d * d;
                        const double mag = div_by(20.0, dd, rcp_refined(dd));
                        const double rn = rcp_refined(nrm);
                        fsx += div_by(ex, nrm, rn) * mag;
                        fsy += div_by(ey, nrm, rn) * mag;
                    }
                    continue;
                }
                double d = sqrt(s2);
                if (d < 2.0) {
                    if (d <= 0.001) d = 0.001;
                    const double mag = 20.0 / (d * d);
                    const double nrm = sqrt(s2);
                    sing += nrm == 0.0;
                    fsx += (ex / nrm) * mag;
                    fsy += (ey / nrm) * mag;
                }
            }
        }
        const double f0 = fax + frx + fsx, f1 = fay + fry + fsy;
        const double vmag = sqrt(f0 * f0 + f1 * f1);
        double2 v;
        if (vmag > max_speed) {
            const double scale = max_speed / vmag;
            v = make_double2(f0 * scale, f1 * scale);
        } else {
            v = make_double2(f0, f1);
        }
        vel[i] = v;
        pout[i] = make_double2(px + v.x * dt, py + v.y * dt);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sing += __shfl_xor(sing, off, 64);
    if ((threadIdx.x & 63) == 0 && sing) atomicAdd(singular, sing);
}

}  // namespace
}  // namespace swarm

extern "C" {

int swarm_physics_step(swarm_ctx *ctx, int64_t n, const int32_t *ids, const uint8_t *state,
                       const int32_t *leader_index, const double *pos_in, double *pos_out, double *vel,
                       double *target, uint8_t *has_target, int64_t m, const double *obstacles,
                       const int32_t *row_ptr, const int32_t *col, double dt, double max_speed,
                       int64_t *n_singular, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) && m >= 0, "sizes out of range");
    SW_ARG(std::isfinite(dt) && std::isfinite(max_speed), "dt / max_speed must be finite");
    SW_ARG(n == 0 || (ids && state && leader_index && pos_in && pos_out && vel && target && has_target && row_ptr),
           "NULL agent array");
    SW_ARG(m == 0 || obstacles != nullptr, "obstacles is NULL");
    SW_ARG(pos_in != pos_out || n == 0, "pos_in and pos_out must differ (synchronous step)");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n_singular) *n_singular = 0;
    if (n == 0) return SWARM_OK;
    unsigned long long *d_sing;
    SW_ALLOC(d_sing, ctx, S_TMP0, 64);
    SW_HIP(hipMemsetAsync(d_sing, 0, 8, s));
    hipLaunchKernelGGL(k_physics, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, n, ids, state, leader_index,
                       reinterpret_cast<const double2 *>(pos_in), reinterpret_cast<double2 *>(pos_out),
                       reinterpret_cast<double2 *>(vel), reinterpret_cast<double2 *>(target), has_target, m, obstacles,
                       row_ptr, col, dt, max_speed, d_sing);
    SW_LAUNCHED();
    if (n_singular) {
        unsigned long long *h = static_cast<unsigned long long *>(pinned(ctx, 64));
        if (!h) return SWARM_ERR_OOM;
        SW_HIP(hipMemcpyAsync(h, d_sing, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        *n_singular = int64_t(*h);
    }
    return SWARM_OK;
}

}  // extern "C"
