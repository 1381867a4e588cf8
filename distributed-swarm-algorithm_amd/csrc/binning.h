// Uniform-grid binning of agents (cell-list), shared by the RGG builder, the spatial storage
// order and the binned allocation.  Agents are bucketed by row-major cell key with a hipCUB
// radix sort; cell_off[c] is the first sorted position of cell c (exclusive prefix), so the
// agents of cells [c0, c1] of one grid row are the contiguous range [cell_off[c0],
// cell_off[c1 + 1]).
#pragma once

#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>

#include "swarm_common.h"

namespace swarm {

struct Grid {
    double xmin, ymin, xmax, ymax;
    double cell, inv_cell;
    int64_t ncx, ncy;
};

__device__ __forceinline__ int64_t cell_coord(double v, double vmin, double inv_cell, int64_t nc) {
    double f = floor((v - vmin) * inv_cell);
    if (!(f >= 0.0)) return 0;            // also catches NaN
    if (f >= double(nc - 1)) return nc - 1;
    return int64_t(f);
}

static __global__ __launch_bounds__(kBlock) void k_bbox_partial(const double2 *__restrict__ pos,
                                                               int64_t n, double *__restrict__ part) {
    double mnx = DBL_MAX, mny = DBL_MAX, mxx = -DBL_MAX, mxy = -DBL_MAX;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const double2 p = pos[i];
        mnx = fmin(mnx, p.x); mny = fmin(mny, p.y);
        mxx = fmax(mxx, p.x); mxy = fmax(mxy, p.y);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mnx = fmin(mnx, __shfl_xor(mnx, off, 64));
        mny = fmin(mny, __shfl_xor(mny, off, 64));
        mxx = fmax(mxx, __shfl_xor(mxx, off, 64));
        mxy = fmax(mxy, __shfl_xor(mxy, off, 64));
    }
    __shared__ double s[4][kBlock / kWave];
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s[0][wid] = mnx; s[1][wid] = mny; s[2][wid] = mxx; s[3][wid] = mxy; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w) {
            s[0][0] = fmin(s[0][0], s[0][w]); s[1][0] = fmin(s[1][0], s[1][w]);
            s[2][0] = fmax(s[2][0], s[2][w]); s[3][0] = fmax(s[3][0], s[3][w]);
        }
        part[4 * blockIdx.x + 0] = s[0][0]; part[4 * blockIdx.x + 1] = s[1][0];
        part[4 * blockIdx.x + 2] = s[2][0]; part[4 * blockIdx.x + 3] = s[3][0];
    }
}

// One wave folds the per-block partials.
static __global__ void k_bbox_final(const double *__restrict__ part, int nparts, double *__restrict__ out) {
    double b0 = DBL_MAX, b1 = DBL_MAX, b2 = -DBL_MAX, b3 = -DBL_MAX;
    for (int i = threadIdx.x; i < nparts; i += kWave) {
        b0 = fmin(b0, part[4 * i + 0]); b1 = fmin(b1, part[4 * i + 1]);
        b2 = fmax(b2, part[4 * i + 2]); b3 = fmax(b3, part[4 * i + 3]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        b0 = fmin(b0, __shfl_xor(b0, off, 64)); b1 = fmin(b1, __shfl_xor(b1, off, 64));
        b2 = fmax(b2, __shfl_xor(b2, off, 64)); b3 = fmax(b3, __shfl_xor(b3, off, 64));
    }
    if (threadIdx.x == 0) { out[0] = b0; out[1] = b1; out[2] = b2; out[3] = b3; }
}

static __global__ __launch_bounds__(kBlock) void k_cell_keys(const double2 *__restrict__ pos, int64_t n,
                                                            Grid g, uint32_t *__restrict__ keys,
                                                            int32_t *__restrict__ vals) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const double2 p = pos[i];
        const int64_t cx = cell_coord(p.x, g.xmin, g.inv_cell, g.ncx);
        const int64_t cy = cell_coord(p.y, g.ymin, g.inv_cell, g.ncy);
        keys[i] = uint32_t(cy * g.ncx + cx);
        vals[i] = int32_t(i);
    }
}

// cell_off[c] = #agents with key < c, for c in [0, ncells]
static __global__ __launch_bounds__(kBlock) void k_cell_offsets(const uint32_t *__restrict__ skeys, int64_t n,
                                                               int64_t ncells, uint32_t *__restrict__ off) {
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i <= n; i += int64_t(gridDim.x) * kBlock) {
        const int64_t lo = (i == 0) ? 0 : int64_t(skeys[i - 1]) + 1;
        const int64_t hi = (i == n) ? ncells : int64_t(skeys[i]);
        for (int64_t c = lo; c <= hi; ++c) off[c] = uint32_t(i);
    }
}

// Bounding box of n positions -> host Grid with cells of side >= `cell` (enlarged if the grid
// would exceed max_cells).  One host sync (the grid shape sizes the launch).
static inline int make_grid(swarm_ctx *ctx, int64_t n, const double *pos, double cell, int64_t max_cells,
                            Grid *g, hipStream_t s) {
    const unsigned np = grid_for(n, kBlock, 1024);
    double *part;
    SW_ALLOC(part, ctx, S_BBOX, size_t(np) * 4 * 8 + 64);
    double *fin = part + size_t(np) * 4;
    hipLaunchKernelGGL(k_bbox_partial, dim3(np), dim3(kBlock), 0, s,
                       reinterpret_cast<const double2 *>(pos), n, part);
    SW_LAUNCHED();
    hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(64), 0, s, part, int(np), fin);
    SW_LAUNCHED();
    double *hb = static_cast<double *>(pinned(ctx, 64));
    if (!hb) return SWARM_ERR_OOM;
    SW_HIP(hipMemcpyAsync(hb, fin, 32, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    if (!(std::isfinite(hb[0]) && std::isfinite(hb[1]) && std::isfinite(hb[2]) && std::isfinite(hb[3]))) {
        set_error("positions must be finite");
        return SWARM_ERR_ARG;
    }
    g->xmin = hb[0]; g->ymin = hb[1]; g->xmax = hb[2]; g->ymax = hb[3];
    double c = cell > 0 ? cell : 1.0;
    for (;;) {
        const double fx = std::floor((g->xmax - g->xmin) / c) + 1.0;
        const double fy = std::floor((g->ymax - g->ymin) / c) + 1.0;
        if (fx * fy <= double(max_cells)) {
            g->ncx = int64_t(fx);
            g->ncy = int64_t(fy);
            break;
        }
        c *= 1.4142135623730951;
    }
    g->cell = c;
    g->inv_cell = 1.0 / c;
    return SWARM_OK;
}

// Sort agents by cell.  On return *sorted_idx (device, n) lists agent indices cell by cell
// (ascending index within a cell: the radix sort is stable) and *cell_off (device,
// ncells + 1) is the exclusive prefix.
static inline int bin_agents(swarm_ctx *ctx, int64_t n, const double *pos, const Grid &g,
                             int32_t **sorted_idx, uint32_t **cell_off, hipStream_t s) {
    const int64_t ncells = g.ncx * g.ncy;
    uint32_t *kin, *kout, *off;
    int32_t *vin, *vout;
    SW_ALLOC(kin, ctx, S_KEYS_IN, size_t(n) * 4);
    SW_ALLOC(kout, ctx, S_KEYS_OUT, size_t(n) * 4);
    SW_ALLOC(vin, ctx, S_VALS_IN, size_t(n) * 4);
    SW_ALLOC(vout, ctx, S_VALS_OUT, size_t(n) * 4);
    SW_ALLOC(off, ctx, S_CELL_START, size_t(ncells + 1) * 4);
    hipLaunchKernelGGL(k_cell_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s,
                       reinterpret_cast<const double2 *>(pos), n, g, kin, vin);
    SW_LAUNCHED();
    int end_bit = 1;
    while (end_bit < 32 && (int64_t(1) << end_bit) < ncells) ++end_bit;
    size_t tmp_bytes = 0;
    SW_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, vout, int(n), 0, end_bit, s));
    void *tmp;
    SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
    SW_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, int(n), 0, end_bit, s));
    hipLaunchKernelGGL(k_cell_offsets, dim3(grid_for(n + 1, kBlock, 8192)), dim3(kBlock), 0, s, kout, n,
                       ncells, off);
    SW_LAUNCHED();
    *sorted_idx = vout;
    *cell_off = off;
    return SWARM_OK;
}

}  // namespace swarm
