// Context, scratch ownership and error reporting for libswarm.so.
#include <cstdarg>
#include <new>

#include "swarm_common.h"
#include "build/src_hash.h"  // SWARM_SRC_HASH (Makefile: sha256 of the library's sources)

namespace swarm {

static thread_local char g_err[1024] = "";
static thread_local int g_scratch_code = SWARM_ERR_OOM;

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int scratch_code() { return g_scratch_code; }

// A ctx's scratch lives on the device it was created on: using it from another device would
// hand that device's kernels foreign buffers.
bool ctx_on_current_device(const swarm_ctx *ctx) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != ctx->device) {
        set_error("invalid argument: ctx was created on device %d but device %d is current (one ctx per device)",
                  ctx->device, dev);
        g_scratch_code = SWARM_ERR_ARG;
        return false;
    }
    return true;
}

void *scratch(swarm_ctx *ctx, Slot s, size_t bytes) {
    if (!ctx_on_current_device(ctx)) return nullptr;
    g_scratch_code = SWARM_ERR_OOM;
    if (bytes == 0) bytes = 16;
    if (ctx->cap[s] >= bytes) return ctx->slot[s];
    if (ctx->slot[s]) {
        (void)hipFree(ctx->slot[s]);
        ctx->slot[s] = nullptr;
        ctx->cap[s] = 0;
    }
    size_t want = bytes + bytes / 8;  // headroom against small growth
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
        set_error("scratch slot %d: hipMalloc(%zu) -> %s", int(s), want, hipGetErrorString(e));
        return nullptr;
    }
    ctx->slot[s] = p;
    ctx->cap[s] = want;
    return p;
}

void *pinned(swarm_ctx *ctx, size_t bytes) {
    if (ctx->host_cap >= bytes) return ctx->host_pinned;
    if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
    ctx->host_pinned = nullptr;
    ctx->host_cap = 0;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        set_error("hipHostMalloc(%zu) -> %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    ctx->host_pinned = p;
    ctx->host_cap = bytes;
    return p;
}

int side_stream(swarm_ctx *ctx, hipStream_t *side, hipEvent_t *fork, hipEvent_t *join) {
    if (!ctx_on_current_device(ctx)) return SWARM_ERR_ARG;
    if (!ctx->side) {
        SW_HIP(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        SW_HIP(hipEventCreateWithFlags(&ctx->side_ev[0], hipEventDisableTiming));
        SW_HIP(hipEventCreateWithFlags(&ctx->side_ev[1], hipEventDisableTiming));
    }
    *side = ctx->side;
    *fork = ctx->side_ev[0];
    *join = ctx->side_ev[1];
    return SWARM_OK;
}

// Host memory the device writes directly (coherent, mapped): the election's per-batch counter
// read-back lands here from the totals kernel itself, with no copy in the stream.
void *mapped(swarm_ctx *ctx, size_t bytes, void **dev) {
    if (ctx->mapped_cap < bytes) {
        if (ctx->host_mapped) (void)hipHostFree(ctx->host_mapped);
        ctx->host_mapped = ctx->mapped_dev = nullptr;
        ctx->mapped_cap = 0;
        void *p = nullptr;
        hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped);
        if (e != hipSuccess) {
            set_error("hipHostMalloc(%zu, coherent|mapped) -> %s", bytes, hipGetErrorString(e));
            return nullptr;
        }
        void *d = nullptr;
        e = hipHostGetDevicePointer(&d, p, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(p);
            set_error("hipHostGetDevicePointer -> %s", hipGetErrorString(e));
            return nullptr;
        }
        ctx->host_mapped = p;
        ctx->mapped_dev = d;
        ctx->mapped_cap = bytes;
    }
    *dev = ctx->mapped_dev;
    return ctx->host_mapped;
}

int wait_mapped_word(const unsigned long long *w, unsigned long long v, hipStream_t s, const char *what) {
    for (uint64_t spin = 1; __atomic_load_n(w, __ATOMIC_ACQUIRE) != v; ++spin) {
        if ((spin & 255) != 0) continue;
        const hipError_t q = hipStreamQuery(s);
        if (q == hipErrorNotReady) continue;
        SW_HIP(q);
        if (__atomic_load_n(w, __ATOMIC_ACQUIRE) != v) {
            set_error("%s: the stream finished without writing its read-back word", what);
            return SWARM_ERR_HIP;
        }
    }
    return SWARM_OK;
}

}  // namespace swarm

extern "C" {

const char *swarm_last_error(void) { return swarm::g_err; }

const char *swarm_version(void) { return "swarm-mi355x 0.2.0 (gfx950) src=" SWARM_SRC_HASH; }

int swarm_ctx_create(swarm_ctx **out) {
    SW_ARG(out != nullptr, "out is NULL");
    swarm_ctx *c = new (std::nothrow) swarm_ctx();
    if (!c) {
        swarm::set_error("out of host memory");
        return SWARM_ERR_OOM;
    }
    SW_HIP(hipGetDevice(&c->device));
    *out = c;
    return SWARM_OK;
}

int swarm_ctx_destroy(swarm_ctx *ctx) {
    if (!ctx) return SWARM_OK;
    for (int s = 0; s < swarm::S_NUM; ++s)
        if (ctx->slot[s]) (void)hipFree(ctx->slot[s]);
    if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
    if (ctx->host_mapped) (void)hipHostFree(ctx->host_mapped);
    for (auto e : ctx->side_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    delete ctx;
    return SWARM_OK;
}

}  // extern "C"
