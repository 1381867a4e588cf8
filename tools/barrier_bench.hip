// Device-wide synchronisation price on gfx950, for the election's per-round floor:
// what a round boundary costs as (a) a kernel boundary between back-to-back launches on one stream,
// (b) a hand-written XCD-hierarchical barrier inside one persistent launch (per-shard arrival
// counters, the last arriver of each shard bumps a top counter, the last top arriver publishes the
// generation; waiters poll it with sc1 loads + s_sleep), without and with the agent-scope release /
// acquire fences a round's data hand-off needs.  Grids of 256 .. 2 048 workgroups of 256 threads
// (1 .. 8 per CU).  Every spin is bounded (1 s), so a non-resident grid ends with an error, not a hang.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/build/barrier_bench tools/barrier_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

constexpr int kShards = 8;
constexpr int kStride = 32;  // u32 between counters: one 128-B line each

__global__ __launch_bounds__(256) void k_empty(unsigned *sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFF) *sink = 1;
}

// One stamp-like word per workgroup read, one written: the smallest "round" a kernel boundary separates.
__global__ __launch_bounds__(256) void k_touch(const unsigned *in, unsigned *out, int it) {
    if (threadIdx.x == 0) out[blockIdx.x * kStride] = in[blockIdx.x * kStride] + unsigned(it);
}

__device__ __forceinline__ unsigned ld_coh(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool FENCE>
__global__ __launch_bounds__(256) void k_barrier(unsigned *ctr, unsigned *gen, unsigned *err, int iters) {
    __shared__ int s_abort;
    const int G = gridDim.x, b = blockIdx.x, sh = b % kShards;
    const int per = G / kShards + (sh < G % kShards ? 1 : 0);  // workgroups of shard sh
    if (threadIdx.x == 0) s_abort = 0;
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const unsigned a = atomicAdd(ctr + sh * kStride, 1u);
            if (a == unsigned((i + 1) * per - 1)) {  // last of the shard
                const unsigned t = atomicAdd(ctr + kShards * kStride, 1u);
                if (t == unsigned((i + 1) * kShards - 1))  // last shard: release the generation
                    __hip_atomic_store(gen, unsigned(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const unsigned long long t0 = wall_clock64();
            while (ld_coh(gen) < unsigned(i + 1)) {
                if (ld_coh(err) || wall_clock64() - t0 > 100000000ull) {
                    atomicMax(err, 1u);
                    s_abort = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
        if (s_abort) return;
    }
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    unsigned *buf;
    CK(hipMalloc(&buf, 1 << 24));
    unsigned *ctr = buf, *gen = buf + 4096, *err = buf + 4128, *in = buf + 8192, *out = buf + (1 << 21);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    printf("{\"cus\": %d, \"iters\": %d, \"rows\": [\n", ncu, iters);
    const int grids[] = {256, 512, 1024, 2048};
    bool first = true;
    for (int G : grids) {
        float ms[4] = {0, 0, 0, 0};
        // (a) kernel boundaries
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, 0, err);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[0], e0, e1));
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_touch, dim3(G), dim3(256), 0, 0, in, out, i);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[1], e0, e1));
        }
        // (b) persistent barrier, plain and fenced
        for (int f = 0; f < 2; ++f) {
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipMemset(buf, 0, 1 << 16));
                void *args[] = {&ctr, &gen, &err, (void *)&iters};
                CK(hipEventRecord(e0, 0));
                if (hipLaunchCooperativeKernel(f ? (const void *)k_barrier<true> : (const void *)k_barrier<false>,
                                               dim3(G), dim3(256), args, 0, 0) != hipSuccess) {
                    (void)hipGetLastError();
                    fprintf(stderr, "cooperative launch of %d workgroups refused\n", G);
                    ms[2 + f] = -2.f * iters / 1e3f;
                    continue;
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[2 + f], e0, e1));
                unsigned herr = 0;
                CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
                if (herr) {
                    fprintf(stderr, "barrier at %d workgroups timed out\n", G);
                    ms[2 + f] = -1.f;
                }
            }
        }
        printf("%s  {\"workgroups\": %d, \"per_cu\": %.1f, \"boundary_empty_us\": %.3f, \"boundary_touch_us\": %.3f, "
               "\"barrier_us\": %.3f, \"barrier_fenced_us\": %.3f}",
               first ? "" : ",\n", G, double(G) / ncu, ms[0] * 1e3 / iters, ms[1] * 1e3 / iters, ms[2] * 1e3 / iters,
               ms[3] * 1e3 / iters);
        first = false;
    }
    printf("\n]}\n");
    return 0;
}
