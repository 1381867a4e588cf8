// Persistent rounds on ONE XCD (gfx950): the plumbing of a kernel whose workgroups run many
// rounds back to back inside one launch, separated by a barrier of their own, all on one XCD.
//
// Why one XCD: the eight XCDs' L2s are not coherent with each other, so a round boundary between
// workgroups on different XCDs needs write-backs and invalidates (a device barrier with the
// release / acquire a round needs: 5-31 us, tools/barrier_bench).  Within one XCD the L2 is
// shared: stores are plain (L1 is write-through), loads of data another workgroup wrote in the
// launch use sc1 (L1 bypass), and no fence is needed -- tools/xcd_barrier_bench counts 0 stale
// hand-offs that way, and a flag barrier costs 1.0 us at any participant count.
//
//   census   8 x kXcdPer workgroups are launched; workgroup 0 names its XCD (hardware XCC_ID --
//            checked, not assumed from the dispatch order), the workgroups on it stay (rank =
//            arrival order) and wait until every workgroup has been counted; the others count
//            themselves on their own XCD's counter (one counter for 1 024 arrivals costs ~12 us of
//            serialised device-scope atomics) and leave.
//   barrier  each participant stores its round counts in its slot (by round parity), drains its
//            stores, then stores its arrival flag 2 (i + 1) + bit; rank 0 polls all flags, ORs the
//            bits and publishes gen = 2 (i + 1) + stop.  No atomics.
// Every wait is bounded (1 s): a timeout sets err, which ends every participant; the host reads it
// from mapped memory (*herr) and fails the call loudly -- the rounds it covered are undone.
#pragma once

#include "swarm_common.h"

namespace swarm {
namespace xcd {

constexpr int kXcdPer = 128;  // participants requested per XCD: 4 per CU
constexpr int kCtlLine = 32;  // u32 per control line

struct Ctl {  // zeroed before every launch (hipMemsetAsync of sizeof(Ctl))
    unsigned chosen[kCtlLine], joined[kCtlLine], nonpart[16][kCtlLine], gen[kCtlLine], err[kCtlLine];
    unsigned flag[kBlock];       // arrival of participant r in round i: 2 (i + 1) + (its bit)
    unsigned cnt[2][kBlock][4];  // participant r's counts of a round (by round parity)
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned *p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned xcc_id() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}
__device__ __forceinline__ bool timed_out(unsigned long long t0) { return wall_clock64() - t0 > 100000000ull; }

// Bounded wait (1 s) for *p >= want; on timeout or another workgroup's error: err set, false.
__device__ inline bool wait_ge(const unsigned *p, unsigned want, unsigned *err) {
    const unsigned long long t0 = wall_clock64();
    while (ld_sc1(p) < want) {
        if (ld_sc1(err) || timed_out(t0)) {
            atomicMax(err, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// The census (every thread of every workgroup calls it).  Returns true in the participants, with
// *rank and *P set; false in the workgroups that leave (and in all of them after an error).
__device__ inline bool census(Ctl *c, int total, int *rank, int *P) {
    __shared__ int s_rank, s_P, s_ok;
    if (threadIdx.x == 0) {
        const unsigned x = xcc_id();
        s_rank = -1;
        s_ok = 1;
        if (blockIdx.x == 0) st_sc1(c->chosen, x + 1);
        if (wait_ge(c->chosen, 1u, c->err) && ld_sc1(c->chosen) == x + 1)
            s_rank = int(atomicAdd(c->joined, 1u));
        else
            atomicAdd(&c->nonpart[x][0], 1u);
    }
    __syncthreads();
    if (s_rank >= 0 && threadIdx.x < kWave) {  // wait until every workgroup is counted: P = joined
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            unsigned v = threadIdx.x < 16 ? ld_sc1(&c->nonpart[threadIdx.x][0])
                                          : threadIdx.x == 16 ? ld_sc1(c->joined) : 0u;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (v >= unsigned(total)) break;
            if (ld_sc1(c->err) || timed_out(t0)) {
                if (threadIdx.x == 0) {
                    atomicMax(c->err, 1u);
                    s_ok = 0;
                }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (threadIdx.x == 0 && s_ok) {
            s_P = int(ld_sc1(c->joined));
            if (s_P > kBlock) {  // rank 0 polls one arrival flag per thread
                atomicMax(c->err, 2u);
                s_ok = 0;
            }
        }
    }
    __syncthreads();
    *rank = s_rank;
    *P = s_P;
    return s_rank >= 0 && s_ok;
}

// Round i's barrier among the P participants (every thread calls it, after this workgroup's
// counts are in c->cnt[i & 1][rank]).  bit: this workgroup's vote (e.g. "I placed a bid").
// Returns, in every thread: 1 when no participant voted (stop after this round), 0 to go on,
// -1 after an error.  Rank 0 gets the OR of the votes before the others are released, and sums the
// counts after (in *sum, rank 0's thread 0 only) -- they stay valid until round i + 2 overwrites
// the slot.
__device__ inline int barrier(Ctl *c, int i, int rank, int P, unsigned bit, unsigned long long *sum) {
    __shared__ int s_res;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's stores of the round are in L2
    __syncthreads();
    if (threadIdx.x == 0) c->flag[rank] = unsigned(2 * (i + 1)) + (bit ? 1u : 0u);
    if (rank == 0) {
        unsigned any = 0;
        if (threadIdx.x < P) {
            const unsigned long long t0 = wall_clock64();
            unsigned fv;
            while ((fv = ld_sc1(&c->flag[threadIdx.x])) < unsigned(2 * (i + 1))) {
                if (ld_sc1(c->err) || timed_out(t0)) {
                    atomicMax(c->err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            any = fv & 1u;
        }
        any = __syncthreads_or(int(any));
        if (threadIdx.x == 0) {
            c->gen[0] = unsigned(2 * (i + 1)) + (any ? 0u : 1u);
            s_res = ld_sc1(c->err) ? -1 : (any ? 0 : 1);
        }
        // the round's counts (after the release: off the others' critical path)
        unsigned long long v = threadIdx.x < P ? ld_sc1(&c->cnt[i & 1][threadIdx.x][0]) : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        __shared__ unsigned long long s_sum[kBlock / kWave];
        if ((threadIdx.x & (kWave - 1)) == 0) s_sum[threadIdx.x / kWave] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long a = 0;
            for (int w = 0; w < kBlock / kWave; ++w) a += s_sum[w];
            *sum = a;
        }
    } else if (threadIdx.x == 0) {
        s_res = wait_ge(c->gen, unsigned(2 * (i + 1)), c->err) ? int(ld_sc1(c->gen) & 1u) : -1;
    }
    __syncthreads();
    return s_res;
}

}  // namespace xcd
}  // namespace swarm
