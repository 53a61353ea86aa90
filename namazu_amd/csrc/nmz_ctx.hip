#include <algorithm>
#include <cstdlib>
// Context management, error plumbing, parameter resolution and the seed
// bucketing pass shared by the replayable and random sweeps.
#include <cstdio>
#include <cstring>
#include <new>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int HostPin::ensure(size_t bytes) {
    if (busy && hipEventSynchronize(busy) != hipSuccess) return fail(NMZ_EHIP, "pinned staging wait failed");
    if (bytes <= cap) return NMZ_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
    // a power of two of at least 1 MiB: a stream of plans of slightly different sizes settles on one buffer
    // (hipHostFree of an outgrown one synchronises the device)
    size_t want = size_t(1) << 20;
    while (want < bytes) want <<= 1;
    if (hipHostMalloc(&ptr, want, hipHostMallocDefault) != hipSuccess) {
        ptr = nullptr;
        return fail(NMZ_ENOMEM, "hipHostMalloc of " + std::to_string(want) + " bytes failed");
    }
    cap = want;
    return NMZ_OK;
}

int HostPin::mark(hipStream_t st) {
    if (!busy && hipEventCreateWithFlags(&busy, hipEventDisableTiming) != hipSuccess) {
        busy = nullptr;
        return fail(NMZ_EHIP, "hipEventCreate failed");
    }
    return hipEventRecord(busy, st) == hipSuccess ? NMZ_OK : fail(NMZ_EHIP, "hipEventRecord failed");
}

void HostPin::release() {
    if (busy) {
        (void)hipEventSynchronize(busy);
        (void)hipEventDestroy(busy);
    }
    busy = nullptr;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
}

int DevBuf::ensure(size_t bytes) {
    if (bytes <= cap) return NMZ_OK;
    ++gen;
    // a pooled buffer that grows goes back to the pool, where the next plan of this context may take it and
    // memset / upload into it on another stream: kernels of earlier calls that still read it must be done
    // (unpooled buffers are released with hipFree, which synchronises by itself)
    if (ptr && pool && hipDeviceSynchronize() != hipSuccess) return fail(NMZ_EHIP, "hipDeviceSynchronize failed");
    release();
    size_t want = bytes < 256 ? 256 : bytes;
    if (pool && want >= (size_t(1) << 16)) {  // pooled: 1/8-power-of-two steps, so similar sizes reuse a buffer
        size_t g = size_t(1) << 13;
        while ((g << 4) <= want) g <<= 1;
        want = (want + g - 1) & ~(g - 1);
    }
    if (pool) {  // best fit among the pooled buffers, at most 1.25x the request: a plan's buffers of other roles
                 // (and small plans' large ones) stay for the requests they fit (a fresh hipMalloc of tens of MB
                 // stalls the host for ~40 ms)
        size_t best = pool->size();
        for (size_t i = 0; i < pool->size(); ++i)
            if ((*pool)[i].cap >= want && (*pool)[i].cap <= want + want / 4 &&
                (best == pool->size() || (*pool)[i].cap < (*pool)[best].cap))
                best = i;
        if (best < pool->size()) {
            ptr = (*pool)[best].ptr;
            cap = (*pool)[best].cap;
            (*pool)[best] = pool->back();
            pool->pop_back();
            return NMZ_OK;
        }
    }
    if (hipMalloc(&ptr, want) != hipSuccess) {
        ptr = nullptr;
        return fail(NMZ_ENOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
    }
    cap = want;
    return NMZ_OK;
}

void DevBuf::release() {
    if (ptr) {
        if (pool) {
            DevBuf b;
            b.ptr = ptr;
            b.cap = cap;
            pool->push_back(b);
        } else {
            (void)hipFree(ptr);
        }
    }
    ptr = nullptr;
    cap = 0;
}

static hipEvent_t timing_event(nmz_ctx *c) {
    if (!c->timing.pool.empty()) {
        hipEvent_t e = c->timing.pool.back();
        c->timing.pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

KernelTimer::KernelTimer(nmz_ctx *c, hipStream_t s, const char *n) : ctx(c), st(s), name(n) {
    if (!ctx || !ctx->timing.enabled) return;
    if (ctx->timing.spans_only) {
        spans_only = true;
        return;
    }
    a = timing_event(ctx);
    b = timing_event(ctx);
    if (a) (void)hipEventRecord(a, st);
}

unsigned long long *KernelTimer::span() {
    if (!spans_only && (!a || !b)) return nullptr;
    NmzTiming &t = ctx->timing;
    if (!t.span_dev) {
        if (hipMalloc(&t.span_dev, NMZ_SPAN_SLOTS * 16) != hipSuccess) {
            t.span_dev = nullptr;
            return nullptr;
        }
        if (hipMemset(t.span_dev, 0, NMZ_SPAN_SLOTS * 16) != hipSuccess) return nullptr;
    }
    if (t.span_next >= NMZ_SPAN_SLOTS) return nullptr;  // full until the next read with reset
    const uint32_t slot = t.span_next++;
    t.spans[name].push_back(slot);
    return t.span_dev + 2 * slot;
}

KernelTimer::~KernelTimer() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    ctx->timing.events[name].push_back({a, b});
}

// ---------------------------------------------------------------------------
// Seed bucketing: counting sort of seeds by (FNV prefix state & 0xff; the
// histogram is fused into the sweeps' prefix kernels), so a
// wave's lanes share one row of the per-event tables and every table read in
// the sweep loop is wave-uniform (scalar loads, no LDS, no gathers).
// ---------------------------------------------------------------------------
// one block per bucket b: the column b of the prefix kernels' rows of counts (hist[rows][256]) becomes, in place,
// each row's offset inside the bucket (the counts of the earlier rows), and total[b] the bucket's size. Thread t
// owns the rows [t q, (t + 1) q) (q = 2 for 2^20 seeds): one load round trip, a block scan, the stores.
__global__ __launch_bounds__(256) void k_bucket_colscan(uint32_t *__restrict__ hist, uint32_t rows,
                                                        uint32_t *__restrict__ total) {
    __shared__ uint32_t wsum[4];
    const uint32_t b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t q = (rows + 255) / 256, r0 = min(rows, t * q), r1 = min(rows, r0 + q);
    uint32_t s = 0;
    for (uint32_t r = r0; r < r1; ++r) s += hist[(size_t)r * 256 + b];
    uint32_t a = s;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(a, d, 64);
        if (lane >= d) a += x;
    }
    if (lane == 63) wsum[w] = a;
    __syncthreads();
    uint32_t run = a - s;
    for (uint32_t x = 0; x < w; ++x) run += wsum[x];
    if (t == 255) total[b] = run + s;
    for (uint32_t r = r0; r < r1; ++r) {
        const uint32_t v = hist[(size_t)r * 256 + b];
        hist[(size_t)r * 256 + b] = run;
        run += v;
    }
}

const char *ab_env(const char *name) {
    const char *ab = getenv("NMZ_AB");
    return (ab && ab[0] == '1' && ab[1] == 0) ? getenv(name) : nullptr;
}

// Scatter of one block of BUCKET_BLK seeds (the prefix kernel's block of the same index). Every block scans the
// 256 bucket totals into the bucket starts (block 0 also writes them, the work-unit table (bucket, start, count)
// of `per_unit` seeds and the caller's zeroed work-item counter); the block's write base in bucket b is b's start +
// its row offset from k_bucket_colscan. The block's seeds are first counting-sorted by bucket in LDS (block-local
// ranks from LDS atomics, a scan of the 256 counts), then written out in that order: consecutive threads write
// consecutive slots of one bucket's range, so a wave's stores are runs of ~BUCKET_PT entries instead of 64
// scattered 8-B writes. Order inside a bucket is irrelevant: results go to the original index.
__global__ __launch_bounds__(256) void k_bucket_scatter(const uint64_t *__restrict__ h0, uint64_t n,
                                                        const uint32_t *__restrict__ rowoff,
                                                        const uint32_t *__restrict__ total,
                                                        uint32_t *__restrict__ offset, uint32_t per_unit,
                                                        uint4 *__restrict__ units, uint32_t *__restrict__ n_units,
                                                        uint32_t *__restrict__ zero_word,
                                                        uint64_t *__restrict__ sorted_h0,
                                                        uint32_t *__restrict__ sorted_idx) {
    constexpr uint32_t SCATTER_PER_THREAD = BUCKET_PT, NB = BUCKET_BLK;
    __shared__ uint32_t cnt[256], base[256], loff[256];
    __shared__ uint16_t si[NB];  // the block's seeds in bucket order (offsets in the block; h0 re-read from L2)
    __shared__ uint32_t wsum[4];
    __shared__ uint2 wsum2[4];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    cnt[t] = 0;
    {  // bucket starts (and, block 0, the unit table): inclusive wave scans of (count, units), the 4 wave totals
        const uint32_t c0 = total[t], u0 = (c0 + per_unit - 1) / per_unit;
        uint32_t a = c0, bu = u0;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t pa = __shfl_up(a, d, 64), pb = __shfl_up(bu, d, 64);
            if (lane >= d) a += pa, bu += pb;
        }
        if (lane == 63) wsum2[w] = make_uint2(a, bu);
        __syncthreads();
        uint32_t ba = 0, bb = 0;
        for (uint32_t i = 0; i < w; ++i) ba += wsum2[i].x, bb += wsum2[i].y;
        const uint32_t start = ba + a - c0;
        base[t] = start + rowoff[(size_t)blockIdx.x * 256 + t];
        if (blockIdx.x == 0) {
            offset[t] = start;
            if (t == 255) {
                offset[256] = ba + a;
                *n_units = bb + bu;
            }
            if (zero_word && t == 0) *zero_word = 0;
            uint32_t u = bb + bu - u0;
            for (uint32_t x = 0; x < c0; x += per_unit, ++u) units[u] = make_uint4(t, start + x, min(per_unit, c0 - x), 0);
        }
    }
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * NB;
    uint64_t hv[SCATTER_PER_THREAD];
    uint32_t rk[SCATTER_PER_THREAD];
#pragma unroll
    for (uint32_t r = 0; r < SCATTER_PER_THREAD; ++r) {
        const uint64_t i = b0 + (uint64_t)r * 256 + t;
        hv[r] = i < n ? h0[i] : 0;
        rk[r] = i < n ? atomicAdd(&cnt[hv[r] & 0xff], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t c = cnt[t];
    // exclusive scan of the 256 counts: the buckets' local offsets
    uint32_t a = c;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(a, d, 64);
        if (lane >= d) a += v;
    }
    if (lane == 63) wsum[w] = a;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t i = 0; i < w; ++i) pre += wsum[i];
    loff[t] = pre + a - c;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < SCATTER_PER_THREAD; ++r) {
        const uint64_t i = b0 + (uint64_t)r * 256 + t;
        if (i < n) {
            si[loff[hv[r] & 0xff] + rk[r]] = (uint16_t)(r * 256 + t);
        }
    }
    __syncthreads();
    const uint32_t m = (uint32_t)min<uint64_t>(NB, n - b0);
#pragma unroll
    for (uint32_t r = 0; r < SCATTER_PER_THREAD; ++r) {
        const uint32_t j = r * 256 + t;
        if (j < m) {
            const uint32_t o = si[j];
            const uint64_t h = h0[b0 + o];  // read by this block above: an L2 hit
            const uint32_t bk = (uint32_t)h & 0xff;
            const uint32_t pos = base[bk] + (j - loff[bk]);
            sorted_h0[pos] = h;
            sorted_idx[pos] = (uint32_t)(b0 + o);
        }
    }
}

int bucket_seeds_counted(hipStream_t st, const uint64_t *d_h0, uint64_t n_seeds, uint32_t per_unit, Buckets &b,
                         uint32_t *zero_word) {
    const uint32_t rows = (uint32_t)bucket_rows(n_seeds);
    hipLaunchKernelGGL(k_bucket_colscan, dim3(256), dim3(256), 0, st, b.hist, rows, b.total);
    // (no seeds: one block writes the empty bucket starts and unit table)
    hipLaunchKernelGGL(k_bucket_scatter, dim3(rows ? rows : 1), dim3(256), 0, st, d_h0, n_seeds, b.hist, b.total,
                       b.offset, per_unit, b.units, b.n_units, zero_word, b.sorted_h0, b.sorted_idx);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz

using namespace nmz;

extern "C" {

const char *nmz_last_error(void) { return g_err.c_str(); }

int nmz_abi_version(void) { return NMZ_ABI_VERSION; }

int nmz_device_count(int *count) {
    NMZ_CHECK(count != nullptr, "count is NULL");
    int n = 0;
    NMZ_HIP(hipGetDeviceCount(&n));
    *count = n;
    return NMZ_OK;
}

int nmz_ctx_stream(nmz_ctx *ctx, void **stream) {
    NMZ_CHECK(ctx != nullptr && stream != nullptr, "NULL argument");
    *stream = ctx->stream;
    return NMZ_OK;
}

int nmz_open(int device, nmz_ctx **out) {
    NMZ_CHECK(out != nullptr, "out is NULL");
    *out = nullptr;
    int n = 0;
    NMZ_HIP(hipGetDeviceCount(&n));
    NMZ_CHECK(device >= 0 && device < n, "device ordinal out of range");
    NMZ_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    NMZ_HIP(hipGetDeviceProperties(&prop, device));
    NMZ_CHECK(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0,
              std::string("libnmz_gpu is built for gfx950 only, device is ") + prop.gcnArchName);
    nmz_ctx *c = new (std::nothrow) nmz_ctx();
    if (!c) return fail(NMZ_ENOMEM, "out of host memory");
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    // NMZ_CTX_CUMASK=1 (A/B): the stream with a CU mask of every CU (a mask is a hardware queue's property, so the
    // stream has a queue of its own instead of one of the process's GPU_MAX_HW_QUEUES shared ones). Measured: the
    // configs[1] stream of traces on four such contexts 0.148-0.162 ms per trace vs 0.175 on plain ones, but the
    // headline step 0.070-0.072 vs 0.069 ms and a serial K1 launch 64 vs 62.6 us, so plain streams stay the default
    const char *cm = ab_env("NMZ_CTX_CUMASK");
    if (cm && cm[0] == '1') {
        std::vector<uint32_t> mask((c->n_cu + 31) / 32, 0xffffffffu);
        if (c->n_cu % 32) mask.back() = (1u << (c->n_cu % 32)) - 1u;
        if (hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            delete c;
            return fail(NMZ_EHIP, "hipExtStreamCreateWithCUMask failed");
        }
    } else if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(NMZ_EHIP, "hipStreamCreate failed");
    }
    *out = c;
    return NMZ_OK;
}

int nmz_close(nmz_ctx *ctx) {
    if (!ctx) return NMZ_OK;
    if (ctx->helper) {
        (void)nmz_close(ctx->helper);
        ctx->helper = nullptr;
    }
    {
        CtxGuard g(ctx);
        for (int i = 0; i < 2; ++i)
            if (ctx->sweep_st[i]) (void)hipStreamDestroy(ctx->sweep_st[i]);
        for (int i = 0; i < 3; ++i)
            if (ctx->sweep_ev[i]) (void)hipEventDestroy(ctx->sweep_ev[i]);
        ctx->tkpin.release();
        for (auto &b : ctx->buf) b.release();
        for (auto &b : ctx->pin) b.release();
        for (auto &b : ctx->pool) (void)hipFree(b.ptr);
        ctx->pool.clear();
        for (auto &kv : ctx->timing.events)
            for (auto &ab : kv.second) {
                (void)hipEventDestroy(ab.first);
                (void)hipEventDestroy(ab.second);
            }
        for (auto e : ctx->timing.pool) (void)hipEventDestroy(e);
        if (ctx->timing.span_dev) (void)hipFree(ctx->timing.span_dev);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
    return NMZ_OK;
}

int nmz_timing_enable(nmz_ctx *ctx, int on) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    std::lock_guard<std::mutex> lk(ctx->mu);
    NMZ_CHECK(on >= 0 && on <= NMZ_TIMING_SPANS, "on must be 0, 1 or NMZ_TIMING_SPANS");
    NmzTiming &t = ctx->timing;
    if (on && !t.span_dev) {  // the span slots now, not at a timed launch (hipMalloc synchronises the device)
        DeviceRestore dr;
        NMZ_HIP(hipSetDevice(ctx->device));
        NMZ_HIP(hipMalloc(&t.span_dev, NMZ_SPAN_SLOTS * 16));
        const hipError_t e = hipMemset(t.span_dev, 0, NMZ_SPAN_SLOTS * 16);
        if (e != hipSuccess) {
            (void)hipFree(t.span_dev);
            t.span_dev = nullptr;
            return fail(NMZ_EHIP, std::string("hipMemset of the span slots: ") + hipGetErrorString(e));
        }
    }
    t.enabled = on != 0;
    t.spans_only = on == NMZ_TIMING_SPANS;
    return NMZ_OK;
}

int nmz_timing_read(nmz_ctx *ctx, const char *kernel, double *total_ms, uint64_t *count, int reset) {
    NMZ_CHECK(ctx && kernel && total_ms && count, "NULL argument");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    *total_ms = 0;
    *count = 0;
    auto it = ctx->timing.events.find(kernel);
    if (it == ctx->timing.events.end()) return NMZ_OK;
    for (auto &ab : it->second) {
        NMZ_HIP(hipEventSynchronize(ab.second));
        float ms = 0;
        NMZ_HIP(hipEventElapsedTime(&ms, ab.first, ab.second));
        *total_ms += ms;
        *count += 1;
    }
    if (reset) {
        for (auto &ab : it->second) {
            ctx->timing.pool.push_back(ab.first);
            ctx->timing.pool.push_back(ab.second);
        }
        it->second.clear();
    }
    return NMZ_OK;
}

int nmz_timing_read_span(nmz_ctx *ctx, const char *kernel, double *total_ms, uint64_t *count, int reset) {
    NMZ_CHECK(ctx && kernel && total_ms && count, "NULL argument");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    *total_ms = 0;
    *count = 0;
    NmzTiming &t = ctx->timing;
    if (!t.span_dev) return NMZ_OK;
    NMZ_HIP(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)NMZ_SPAN_SLOTS * 2);
    NMZ_HIP(hipMemcpy(h.data(), t.span_dev, h.size() * 8, hipMemcpyDeviceToHost));
    int khz = 0;
    NMZ_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
    NMZ_CHECK(khz > 0, "no wall clock rate");
    auto it = t.spans.find(kernel);
    if (it != t.spans.end()) {
        std::vector<std::pair<unsigned long long, unsigned long long>> iv;
        for (uint32_t slot : it->second) {
            const unsigned long long st = ~h[2 * slot], en = h[2 * slot + 1];
            if (h[2 * slot] == 0 || en < st) continue;  // the launch had no work
            iv.push_back({st, en});
        }
        // the union of the spans: launches of several streams that overlap share their common time
        std::sort(iv.begin(), iv.end());
        unsigned long long cur_s = 0, cur_e = 0, ticks = 0;
        for (size_t i = 0; i < iv.size(); ++i) {
            if (i == 0 || iv[i].first > cur_e) {
                ticks += cur_e - cur_s;
                cur_s = iv[i].first;
                cur_e = iv[i].second;
            } else if (iv[i].second > cur_e) {
                cur_e = iv[i].second;
            }
        }
        ticks += cur_e - cur_s;
        *total_ms = (double)ticks / khz;
        *count = iv.size();
    }
    if (reset) {  // every kernel's slots: the ring restarts empty
        NMZ_HIP(hipMemset(t.span_dev, 0, NMZ_SPAN_SLOTS * 16));
        t.spans.clear();
        t.span_next = 0;
    }
    return NMZ_OK;
}

}  // extern "C"

namespace nmz {
// one thread per string: FNV-1a 64 over its bytes (event identities)
__global__ __launch_bounds__(256) void k_fnv_batch(const uint64_t *__restrict__ off, const uint8_t *__restrict__ bytes,
                                                   uint64_t n, uint64_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t h = FNV_OFFSET;
    for (uint64_t b = off[i], e = off[i + 1]; b < e; ++b) h = fnv_step(h, bytes[b]);
    out[i] = h;
}
}  // namespace nmz

extern "C" {

int nmz_fnv1a64_batch(nmz_ctx *ctx, const uint64_t *off, const uint8_t *bytes, uint64_t n, uint64_t *out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n == 0) return NMZ_OK;
    NMZ_CHECK(off && out, "NULL argument");
    for (uint64_t i = 0; i < n; ++i) NMZ_CHECK(off[i] <= off[i + 1], "offsets must not decrease");
    const uint64_t nb = off[n];
    NMZ_CHECK(nb == 0 || bytes, "bytes is NULL");
    hipStream_t st = ctx->stream;
    NMZ_TRY(ctx->buf[12].ensure(Carve::bytes_for(n + 1, 8) * 2 + Carve::bytes_for(nb + 1, 1)));
    Carve cv(ctx->buf[12].ptr);
    uint64_t *d_off = cv.take<uint64_t>(n + 1), *d_out = cv.take<uint64_t>(n + 1);
    uint8_t *d_b = cv.take<uint8_t>(nb + 1);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, st));
    if (nb) NMZ_HIP(hipMemcpyAsync(d_b, bytes, nb, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_fnv_batch, dim3(ceil_div(n, 256)), dim3(256), 0, st, d_off, d_b, n, d_out);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipMemcpyAsync(out, d_out, n * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_fnv1a64_batch_host(const uint64_t *off, const uint8_t *bytes, uint64_t n, uint64_t *out) {
    if (n == 0) return NMZ_OK;
    NMZ_CHECK(off && out, "NULL argument");
    for (uint64_t i = 0; i < n; ++i) {
        NMZ_CHECK(off[i] <= off[i + 1], "offsets must not decrease");
        NMZ_CHECK(off[i] == off[i + 1] || bytes, "bytes is NULL");
        uint64_t h = FNV_OFFSET;
        for (uint64_t b = off[i]; b < off[i + 1]; ++b) h = fnv_step(h, bytes[b]);
        out[i] = h;
    }
    return NMZ_OK;
}

int nmz_random_params_resolve(int64_t min_ns, int64_t max_ns, double p, nmz_random_params *out) {
    NMZ_CHECK(out != nullptr, "out is NULL");
    // randompolicy.go:223-225: "bad faultActionProbability"
    if (!(p >= 0.0 && p <= 1.0)) {
        char m[96];
        std::snprintf(m, sizeof m, "bad faultActionProbability %f", p);
        return fail(NMZ_EINVAL, m);
    }
    out->min_ns[0] = min_ns;
    out->max_ns[0] = max_ns;
    // randompolicy.go:337-339: time.Duration(float64(x) * 0.8), IEEE double, trunc toward 0
    out->min_ns[1] = (int64_t)((double)min_ns * 0.8);
    out->max_ns[1] = (int64_t)((double)max_ns * 0.8);
    out->fault_threshold = (int32_t)(p * 1000.0);  // randompolicy.go:310 int(p*1000.0)
    out->reserved = 0;
    for (int i = 0; i < 2; ++i) {
        if (out->min_ns[i] > out->max_ns[i]) {  // util/queue/impl.go:36-38
            char m[128];
            std::snprintf(m, sizeof m, "minDuration %lldns > maxDuration %lldns",
                          (long long)out->min_ns[i], (long long)out->max_ns[i]);
            return fail(NMZ_EINVAL, m);
        }
    }
    return NMZ_OK;
}

}  // extern "C"
