// Single-XCD persistent rounds on gfx950 ("one XCD for the tail"): launch 8*G workgroups,
// keep those whose hardware XCC_ID is 0 (read from the XCC_ID hwreg, so placement is checked, not assumed),
// count them with a census, then run `iters` barrier-separated rounds among them only.  Every round each
// participant stores a word with a plain store, drains, crosses the barrier and reads its neighbour's word
// with an sc1 load (L1 bypass, served by the shared L2): a stale read is counted, so the run says whether
// the L2-local hand-off needs no fences.  The "chain" variant adds three dependent sc1 loads per thread into
// a table of `table_mb` MB (an L2-resident vs an HBM-resident gather chain), the shape of a tail round.
// Two ways to read what other CUs of the XCD wrote: "sc1" loads (L1 bypass per load) or "inv": one
// L1 invalidate (buffer_inv sc0) after each barrier, then plain loads (L2 hits).
// Every spin is bounded (1 s); a timeout ends the run with an error, not a hang.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/build/xcd_barrier_bench tools/xcd_barrier_bench.hip
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

constexpr int kStride = 32;
struct Ctl {  // one 128-B line per field
    unsigned ctr[kStride], gen[kStride], err[kStride], seen[kStride], joined[kStride], stale[kStride];
    unsigned xcc_hist[16 * kStride];
    unsigned grp[8 * kStride];
};

__device__ __forceinline__ unsigned ld_coh(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned xcc_id() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xF;
}

__device__ bool spin_until(const unsigned *p, unsigned want, unsigned *err) {
    const unsigned long long t0 = wall_clock64();
    while (ld_coh(p) < want) {
        if (ld_coh(err) || wall_clock64() - t0 > 100000000ull) {
            atomicMax(err, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

template <bool CHAIN, bool INV, bool HIER, bool FLAGS = false>
__global__ __launch_bounds__(256) void k_xcd(Ctl *c, unsigned *words, const unsigned *__restrict__ table, unsigned tmask,
                                             unsigned *sink, int iters, int total) {
    __shared__ int s_rank, s_P, s_ok;
    const unsigned x = xcc_id();
    if (threadIdx.x == 0) {
        atomicAdd(&c->xcc_hist[x * kStride], 1u);
        s_rank = x == 0 ? int(atomicAdd(c->joined, 1u)) : -1;
        atomicAdd(c->seen, 1u);
        s_ok = 1;
        if (s_rank >= 0) {
            s_ok = spin_until(c->seen, unsigned(total), c->err);
            s_P = int(ld_coh(c->joined));
        }
    }
    __syncthreads();
    if (s_rank < 0 || !s_ok) return;
    const int r = s_rank, P = s_P;
    unsigned acc = threadIdx.x * 2654435761u + r;
    for (int i = 0; i < iters; ++i) {
        if (CHAIN) {
            unsigned v = (acc ^ (unsigned(i) * 40503u)) & tmask;
            for (int k = 0; k < 3; ++k) v = ((INV ? table[v] : ld_coh(table + v)) + v) & tmask;
            acc += v;
        }
        if (threadIdx.x == 0) words[r * kStride] = unsigned(i + 1);  // plain store
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (FLAGS) {  // flag barrier: plain-store arrival flags, rank 0 polls them all, plain-store gen
            if (threadIdx.x == 0) words[(1 << 16) + r] = unsigned(i + 1);
            if (r == 0) {
                if (threadIdx.x < P) {
                    const unsigned long long t0 = wall_clock64();
                    while (ld_coh(words + (1 << 16) + threadIdx.x) < unsigned(i + 1))
                        if (wall_clock64() - t0 > 100000000ull) {
                            atomicMax(c->err, 1u);
                            break;
                        }
                }
                __syncthreads();
                if (threadIdx.x == 0) words[(1 << 17)] = unsigned(i + 1);
            }
            if (threadIdx.x == 0) s_ok = spin_until(words + (1 << 17), unsigned(i + 1), c->err);
        } else if (threadIdx.x == 0) {
            if (HIER) {  // 8 group counters, the last of a group arrives at the top counter
                const int g = r & 7, per = P / 8 + ((r & 7) < P % 8 ? 1 : 0);
                const unsigned a = atomicAdd(c->grp + g * kStride, 1u);
                if (a == unsigned((i + 1) * per - 1)) {
                    const int ng = P < 8 ? P : 8;
                    if (atomicAdd(c->ctr, 1u) == unsigned((i + 1) * ng - 1))
                        __hip_atomic_store(c->gen, unsigned(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                const unsigned a = atomicAdd(c->ctr, 1u);
                if (a == unsigned((i + 1) * P - 1))
                    __hip_atomic_store(c->gen, unsigned(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_ok = spin_until(c->gen, unsigned(i + 1), c->err);
        }
        __syncthreads();
        if (INV) asm volatile("buffer_inv sc0" ::: "memory");
        if (threadIdx.x == 0 && s_ok) {
            const unsigned nb = INV ? words[((r + 1) % P) * kStride]
                                    : ld_coh(words + ((r + 1) % P) * kStride);
            if (nb < unsigned(i + 1)) atomicAdd(c->stale, 1u);  // older than round i (a newer value is fine)
        }
        if (!s_ok) return;
    }
    if (acc == 0xFFFFFFFFu) *sink = acc;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    Ctl *c;
    unsigned *words, *table, *sink;
    const size_t tbytes = size_t(256) << 20;
    CK(hipMalloc(&c, sizeof(Ctl)));
    CK(hipMalloc(&words, 1 << 20));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&table, tbytes));
    {
        std::vector<unsigned> h(tbytes / 4);
        unsigned s = 12345;
        for (auto &v : h) v = (s = s * 1664525u + 1013904223u);
        CK(hipMemcpy(table, h.data(), tbytes, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"iters\": %d, \"rows\": [\n", iters);
    const int per_xcd[] = {16, 32, 64, 128};
    const int table_mb[] = {0, 1, 64, 256};
    bool first = true;
    for (int mode = 0; mode < 4; ++mode) {  // 0: sc1 loads, flat barrier; 1: L1 invalidate; 2: sc1, 2-level
        const int inv = mode == 1, hier = mode == 2, flags = mode == 3;  // 3: flag barrier (no atomics)
        for (int G : per_xcd) {
            for (int tm : table_mb) {
                const int total = 8 * G;
                const unsigned tmask = tm ? unsigned((size_t(tm) << 20) / 4 - 1) : 0;
                float ms = 0;
                Ctl h{};
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipMemset(c, 0, sizeof(Ctl)));
                    CK(hipEventRecord(e0, 0));
                    CK(hipMemset(words, 0, 1 << 20));
                    auto kern = flags ? (tm ? k_xcd<true, false, false, true> : k_xcd<false, false, false, true>)
                              : hier ? (tm ? k_xcd<true, false, true> : k_xcd<false, false, true>)
                                     : tm ? (inv ? k_xcd<true, true, false> : k_xcd<true, false, false>)
                                          : (inv ? k_xcd<false, true, false> : k_xcd<false, false, false>);
                    hipLaunchKernelGGL(kern, dim3(total), dim3(256), 0, 0, c, words, table, tmask, sink, iters, total);
                    CK(hipGetLastError());
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    CK(hipMemcpy(&h, c, sizeof(Ctl), hipMemcpyDeviceToHost));
                }
                printf("%s  {\"load\": \"%s\", \"per_xcd\": %d, \"table_mb\": %d, \"participants\": %u, "
                       "\"round_us\": %.3f, \"stale\": %u, \"err\": %u, \"xcc_hist\": [",
                       first ? "" : ",\n", flags ? "sc1-flags" : hier ? "sc1-2level" : inv ? "inv" : "sc1", G, tm, h.joined[0], ms * 1e3 / iters, h.stale[0],
                       h.err[0]);
                for (int k = 0; k < 8; ++k) printf("%s%u", k ? ", " : "", h.xcc_hist[k * kStride]);
                printf("]}");
                fflush(stdout);
                first = false;
            }
        }
    }
    printf("\n]}\n");
    return 0;
}
