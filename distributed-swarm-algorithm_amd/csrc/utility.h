// The reference utility on the device, shared by the allocation and auction kernels.
// _calculate_utility (agent.py:338-347): d = sqrt(dx**2 + dy**2), U = (100 / (1 + d)) * has_cap.
// The reference squares with libm pow; this computes dx*dx (separately rounded products: the
// library is built with -ffp-contract=off), IEEE sqrt and division.  guard_flag() marks the
// values a <= 2-ulp difference could push across the claim threshold or an f32 rounding
// boundary.
#pragma once

#include <cmath>
#include <cstdint>

namespace swarm {
namespace {

__device__ __forceinline__ double utility(double ax, double ay, uint32_t caps, double tx, double ty,
                                          int rq, double u_scale) {
    const double dx = ax - tx, dy = ay - ty;
    const double d = sqrt(dx * dx + dy * dy);
    // agent.py:343-345: a required capability the agent lacks -> 0.  rq in [0, 31] is a bit of
    // the mask; rq >= 32 names a capability no agent holds (never a shift by >= 32: the ISA
    // would wrap it mod 32 and alias bit rq - 32).  The entry points reject treq outside
    // [-1, 31] with SWARM_ERR_ARG; this keeps the arithmetic defined either way.
    const double has = (rq < 0) ? 1.0 : (rq < 32 && ((caps >> rq) & 1u)) ? 1.0 : 0.0;
    return (u_scale / (1.0 + d)) * has;
}

// treq outside [-1, 31] (counted by the kernels, reported as SWARM_ERR_ARG by the entry points)
__host__ __device__ __forceinline__ bool bad_req(int rq) { return rq < -1 || rq > 31; }

// Could the reference (libm pow for the squares, <= 2 ulp away) decide or round differently?
// U == 0 is exact under either arithmetic (has_cap = 0, u_scale = 0 or an infinite distance).
__device__ __forceinline__ bool guard_flag(double U, double thr) {
    if (U == 0.0) return false;
    const double band = fmax(fabs(thr), fabs(U)) * 0x1p-49;
    if (fabs(U - thr) <= band) return true;
    if (U > thr) {
        const double e = fabs(U) * 0x1p-50;
        return float(U - e) != float(U + e);
    }
    return false;
}

}  // namespace
}  // namespace swarm
