// Cross-translation-unit declarations inside libnmz_gpu.so.
#pragma once
#include "nmz_common.h"

namespace nmz {

uint64_t topk_scratch_entries(uint64_t n, uint32_t k);
int topk_select(hipStream_t st, const nmz_sched_stats *d_stats, uint64_t n, uint64_t seed0, uint32_t k,
                nmz_topk_entry *d_scratch, nmz_topk_entry *d_out);

// scratch carving helper: bump allocator over one device buffer (256-B aligned)
struct Carve {
    char *base;
    size_t off = 0;
    explicit Carve(void *p) : base(static_cast<char *>(p)) {}
    template <typename T>
    T *take(size_t count) {
        T *p = reinterpret_cast<T *>(base + off);
        off += (count * sizeof(T) + 255) & ~size_t(255);
        return p;
    }
    static size_t bytes_for(size_t count, size_t elem) { return (count * elem + 255) & ~size_t(255); }
};

}  // namespace nmz
