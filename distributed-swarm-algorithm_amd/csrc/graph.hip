// Input side of the round: the radius-r neighbour graph and the spatial storage order.
// Not reference code (agent.py has no graph: its transport is a stub, agent.py:191-194);
// this builds the synthetic "who hears whom" CSR of SURVEY.md §8d on the device.
#include "binning.h"

#include <cstring>

namespace swarm {
namespace {

__global__ __launch_bounds__(kBlock) void k_rgg_rows(const double2 *__restrict__ pos, int64_t n, Grid g,
                                                    double r2, const int32_t *__restrict__ sorted_idx,
                                                    const uint32_t *__restrict__ off,
                                                    int32_t *__restrict__ deg,
                                                    const int32_t *__restrict__ row_ptr,
                                                    int32_t *__restrict__ col,
                                                    unsigned long long *__restrict__ total, int sort_rows) {
    unsigned long long mine = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
        const double2 p = pos[i];
        const int64_t cx = cell_coord(p.x, g.xmin, g.inv_cell, g.ncx);
        const int64_t cy = cell_coord(p.y, g.ymin, g.inv_cell, g.ncy);
        const int64_t x0 = cx > 0 ? cx - 1 : 0, x1 = cx + 1 < g.ncx ? cx + 1 : g.ncx - 1;
        int cnt = 0;
        const int64_t base = col ? row_ptr[i] : 0;
        for (int64_t yy = (cy > 0 ? cy - 1 : 0); yy <= cy + 1 && yy < g.ncy; ++yy) {
            const uint32_t a = off[yy * g.ncx + x0], b = off[yy * g.ncx + x1 + 1];
            for (uint32_t q = a; q < b; ++q) {
                const int32_t j = sorted_idx[q];
                if (j == int32_t(i)) continue;
                const double2 o = pos[j];
                const double dx = p.x - o.x, dy = p.y - o.y;
                if (dx * dx + dy * dy <= r2) {
                    if (col) col[base + cnt] = j;
                    ++cnt;
                }
            }
        }
        if (col && sort_rows) {  // rows ascending (insertion sort: every window is short)
            for (int a = 1; a < cnt; ++a) {
                const int32_t key = col[base + a];
                int b = a - 1;
                while (b >= 0 && col[base + b] > key) {
                    col[base + b + 1] = col[base + b];
                    --b;
                }
                col[base + b + 1] = key;
            }
        } else if (!col) {
            deg[i] = cnt;
        }
        mine += unsigned(cnt);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(total, mine);
}

// Work the row kernel will do, from the cell occupancies alone: each agent scans the agents of its
// 3 x 3 cell window, so W = sum over agents of their window's occupancy (a double: a bound, not a
// count) and the longest serial scan is the largest window (max_win).
__global__ __launch_bounds__(kBlock) void k_window_work(const uint32_t *__restrict__ off, Grid g,
                                                       double *__restrict__ out,
                                                       unsigned long long *__restrict__ max_win) {
    double w = 0.0;
    unsigned long long mx = 0;
    const int64_t ncells = g.ncx * g.ncy;
    for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < ncells; c += int64_t(gridDim.x) * kBlock) {
        const uint32_t occ = off[c + 1] - off[c];
        if (occ == 0) continue;
        const int64_t cx = c % g.ncx, cy = c / g.ncx;
        const int64_t x0 = cx > 0 ? cx - 1 : 0, x1 = cx + 1 < g.ncx ? cx + 1 : g.ncx - 1;
        unsigned long long win = 0;
        for (int64_t yy = (cy > 0 ? cy - 1 : 0); yy <= cy + 1 && yy < g.ncy; ++yy)
            win += off[yy * g.ncx + x1 + 1] - off[yy * g.ncx + x0];
        w += double(occ) * double(win);
        mx = win > mx ? win : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        w += __shfl_xor(w, o, 64);
        const unsigned long long m = __shfl_xor(mx, o, 64);
        mx = m > mx ? m : mx;
    }
    if ((threadIdx.x & 63) == 0 && w > 0.0) {
        atomicAdd(out, w);
        atomicMax(max_win, mx);
    }
}

// Bounds on the row kernel's work (one thread per agent): a radius graph over co-located agents
// (a million agents in one cell) would make swarm_build_rgg run for hours on the device.  A deg-16
// RGG has windows of ~45 agents: W ~ 45 n (100M agents: 4.5e9), far below these.
constexpr double kMaxScanPairs = 68719476736.0;          // 2^36 candidate checks in all
constexpr unsigned long long kMaxWindow = 1ull << 20;    // candidates one thread scans
constexpr unsigned long long kInKernelSort = 64;         // longer windows: rows sorted by hipCUB

}  // namespace
}  // namespace swarm

namespace swarm {
static int check_window_work(swarm_ctx *ctx, const uint32_t *off, const Grid &g, hipStream_t s,
                             unsigned long long *max_window) {
    double *acc;
    SW_ALLOC(acc, ctx, S_CELL_END, 64);
    SW_HIP(hipMemsetAsync(acc, 0, 16, s));
    unsigned long long *mx = reinterpret_cast<unsigned long long *>(acc + 1);
    hipLaunchKernelGGL(k_window_work, dim3(grid_for(g.ncx * g.ncy, kBlock, 8192)), dim3(kBlock), 0, s, off, g, acc,
                       mx);
    SW_LAUNCHED();
    double *h = static_cast<double *>(pinned(ctx, 64));
    if (!h) return SWARM_ERR_OOM;
    SW_HIP(hipMemcpyAsync(h, acc, 16, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    unsigned long long m;
    memcpy(&m, h + 1, 8);
    *max_window = m;
    if (h[0] > kMaxScanPairs || m > kMaxWindow) {
        set_error("radius graph too dense to build: %.3g candidate pairs to scan (limit %.3g), the largest 3x3-cell "
                  "window holds %llu agents (limit %llu) -- co-located agents?",
                  h[0], kMaxScanPairs, m, kMaxWindow);
        return SWARM_ERR_RANGE;
    }
    return SWARM_OK;
}
}  // namespace swarm

extern "C" {

int swarm_build_rgg(swarm_ctx *ctx, int64_t n, const double *pos, double radius, int32_t *row_ptr,
                    int32_t *col, int64_t col_capacity, int64_t *n_edges, void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31) - 1, "n out of range");
    SW_ARG(radius > 0 && std::isfinite(radius), "radius must be positive and finite");
    SW_ARG(row_ptr != nullptr && n_edges != nullptr, "row_ptr / n_edges is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n == 0) {
        SW_HIP(hipMemsetAsync(row_ptr, 0, 4, s));
        SW_HIP(hipStreamSynchronize(s));
        *n_edges = 0;
        return SWARM_OK;
    }
    SW_ARG(pos != nullptr, "pos is NULL");
    Grid g;
    int rc = make_grid(ctx, n, pos, radius * (1.0 + 1e-9), 4 * n + 1024, &g, s);
    if (rc) return rc;
    int32_t *sorted;
    uint32_t *off;
    if ((rc = bin_agents(ctx, n, pos, g, &sorted, &off, s))) return rc;
    unsigned long long max_win = 0;
    if ((rc = check_window_work(ctx, off, g, s, &max_win))) return rc;
    const int sort_rows = max_win <= kInKernelSort ? 1 : 0;
    int32_t *deg;
    unsigned long long *total;
    SW_ALLOC(deg, ctx, S_DEG, size_t(n + 1) * 4);
    SW_ALLOC(total, ctx, S_TMP0, 64);
    unsigned long long *htot = static_cast<unsigned long long *>(pinned(ctx, 64));
    if (!htot) return SWARM_ERR_OOM;
    const double r2 = radius * radius;
    const dim3 grid(grid_for(n, kBlock, 8192));
    const double2 *p2 = reinterpret_cast<const double2 *>(pos);
    if (col == nullptr) {
        SW_HIP(hipMemsetAsync(total, 0, 8, s));
        SW_HIP(hipMemsetAsync(deg + n, 0, 4, s));
        hipLaunchKernelGGL(k_rgg_rows, grid, dim3(kBlock), 0, s, p2, n, g, r2, sorted, off, deg,
                           nullptr, nullptr, total, 0);
        SW_LAUNCHED();
        SW_HIP(hipMemcpyAsync(htot, total, 8, hipMemcpyDeviceToHost, s));
        SW_HIP(hipStreamSynchronize(s));
        if (htot[0] >= (1ull << 31)) {
            set_error("graph has %llu edges: int32 row offsets overflow", htot[0]);
            return SWARM_ERR_RANGE;
        }
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, deg, row_ptr, int(n + 1), s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, deg, row_ptr, int(n + 1), s));
        SW_HIP(hipStreamSynchronize(s));
        *n_edges = int64_t(htot[0]);
        return SWARM_OK;
    }
    int32_t e = 0;
    SW_HIP(hipMemcpyAsync(&e, row_ptr + n, 4, hipMemcpyDeviceToHost, s));
    SW_HIP(hipStreamSynchronize(s));
    SW_ARG(int64_t(e) <= col_capacity, "col_capacity smaller than the edge count");
    SW_HIP(hipMemsetAsync(total, 0, 8, s));
    hipLaunchKernelGGL(k_rgg_rows, grid, dim3(kBlock), 0, s, p2, n, g, r2, sorted, off, deg,
                       row_ptr, col, total, sort_rows);
    SW_LAUNCHED();
    if (!sort_rows && e > 0) {  // long rows: one segmented radix sort instead of O(deg^2) per thread
        int32_t *tmpcol;
        SW_ALLOC(tmpcol, ctx, S_TMP1, size_t(e) * 4);
        SW_HIP(hipMemcpyAsync(tmpcol, col, size_t(e) * 4, hipMemcpyDeviceToDevice, s));
        size_t tmp_bytes = 0;
        SW_HIP(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tmp_bytes, tmpcol, col, int(e), int(n), row_ptr,
                                                          row_ptr + 1, 0, 32, s));
        void *tmp;
        SW_ALLOC(tmp, ctx, S_CUB_TMP, tmp_bytes);
        SW_HIP(hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tmp_bytes, tmpcol, col, int(e), int(n), row_ptr,
                                                          row_ptr + 1, 0, 32, s));
    }
    SW_HIP(hipStreamSynchronize(s));
    *n_edges = e;
    return SWARM_OK;
}

int swarm_cell_order(swarm_ctx *ctx, int64_t n, const double *pos, double cell, int32_t *perm,
                     void *stream) {
    using namespace swarm;
    SW_ARG(ctx != nullptr, "ctx is NULL");
    SW_ARG(n >= 0 && n < (int64_t(1) << 31), "n out of range");
    SW_ARG(cell > 0 && std::isfinite(cell), "cell must be positive and finite");
    if (n == 0) return SWARM_OK;
    SW_ARG(pos && perm, "NULL array");
    hipStream_t s = static_cast<hipStream_t>(stream);
    Grid g;
    int rc = make_grid(ctx, n, pos, cell, 4 * n + 1024, &g, s);
    if (rc) return rc;
    int32_t *sorted;
    uint32_t *off;
    if ((rc = bin_agents(ctx, n, pos, g, &sorted, &off, s))) return rc;
    SW_HIP(hipMemcpyAsync(perm, sorted, size_t(n) * 4, hipMemcpyDeviceToDevice, s));
    return SWARM_OK;
}

}  // extern "C"
