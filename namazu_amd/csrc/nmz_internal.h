// Cross-translation-unit declarations inside libnmz_gpu.so.
#pragma once
#include "nmz_common.h"

namespace nmz {

uint64_t topk_scratch_entries(uint64_t n, uint32_t k);
int topk_merge_lists(hipStream_t st, nmz_topk_entry *a, nmz_topk_entry *b, uint64_t lists, uint32_t k,
                     nmz_topk_entry *d_out);
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

// The shard that owns query block qb (64 queries) of the bit-parallel search, in both its forms (two-phase and the
// single kernel, so the pairs a shard owns do not depend on which form a rank's plan took): rotated snake order. A query block's
// work falls with qb inside the upper triangle (fewer candidates j > q) and inside every family of near-duplicates;
// in each period of 2S blocks, block r and its mirror 2S-1-r form pair min(r, 2S-1-r), so linear trends cancel, and
// the pair goes to shard (pair + period) mod S, so over the periods every shard takes every pair position. (A plain
// snake gives shard s the same two positions in every period: when the work's own period matches -- families of 16
// blocks at 8 shards -- shard 0 always held each family's first and last block, whose short candidate lists run the
// DP less efficiently (1.15x); the MurmurHash3 deal of round 2 left max/mean 1.15. DESIGN.md section 6.) A fixed
// rule, not a knob: one process per GPU computes its own shards' tiles, so the rule must be the same everywhere.
// (Dealing runs of 4 or 16 consecutive blocks instead, to keep a family's candidates in one shard's L2, measured
// worse: 8-shard sum / unsharded 1.17 / 1.16 clustered vs 1.14; profiles/r04/ed_deal_chunk_ab.)
__host__ __device__ inline uint32_t ed_block_shard(uint32_t qb, uint32_t n_shards) {
    if (n_shards <= 1) return 0;
    const uint32_t r = qb % (2 * n_shards), pr = r < n_shards ? r : 2 * n_shards - 1 - r;
    return (pr + qb / (2 * n_shards)) % n_shards;
}
bool ed_bv_supported(uint32_t band);   // band <= 64
uint32_t ed_bv_template(uint32_t band);  // the kernels' template band W >= band: 8, 16, 32 or 64
// LDS of one bit-parallel workgroup: the kernels with a pool (k_ed_bv, k_ed_bv_dp) stay within 64 KiB (several
// workgroups per CU); single queries (k_ed_bv_query, ~N / 256 workgroups) may take up to ED_BV_LDS_MAX
constexpr size_t ED_BV_LDS_MAX = 160 * 1024;

// bit-parallel banded edit distance (ed_bv.hip): 2 queries x a pool of ED_BV_POOL candidates per workgroup
constexpr uint32_t ED_BV_POOL = 1024;  // base pool; the plan scales it up to 4x for large N (ed.hip)
struct EdBvArgs {
    const uint16_t *bsym;         // per-trace streams of Peq-row byte offsets (u16), padded to 32-blocks + 1
    const uint64_t *soff;         // [N] element offset of each trace's stream
    const uint32_t *len;          // [N]
    const uint64_t *chunk_start;  // [G+1] this shard's first chunk of each 64-query block row (row b's chunks
                                  // cr = ((shard - b) mod n_shards) + n_shards * t, t = 0, 1, ...)
    uint64_t *knn;                // [N][k]
    uint64_t *counters;           // [ED_BV_NCOUNTERS] work counters (nmz_ed_plan_counters), or nullptr
    const uint4 *prof;            // [N][ED_QG_DW / 4] q-gram profiles (ed_qgram_profiles), or nullptr: no filter
    uint64_t n_chunks;            // chunks of this shard
    uint32_t N, G, k, lds_dw, shard, n_shards, pool;
    uint32_t w;                   // the requested band (<= the kernel's template W)
    // compact tables (CMP kernels): LDS dword offsets of the id -> row map (u16) and of the claim bitmap, and the
    // bytes per Peq row; lds_dw covers Peq rows + map + bitmap
    uint32_t rmap_dw, claim_dw, row_bytes;
    uint32_t rq;                  // queries per block row (64 x ED_BV_ROW_WAVES64); rq / 2 workgroups share a chunk
};
// Block rows of the bit-parallel search: rq = 64 * ED_BV_RW queries; the rq / 2 workgroups of one chunk (one query
// pair each, the same pool of candidates) are consecutive in the XCD-remapped order, so they run together on one
// XCD and read the pool's candidate streams from its L2. 5 x 32 = 160 workgroups = one XCD's 32 CUs x 5.
constexpr uint32_t ED_BV_RW = 5;
// k_ed_bv work counters, summed over the launch:
//   0 pairs that ran the DP, 1 pairs with a result <= w (in band), 2 lane-candidate 32-column blocks executed,
//   3 candidates that ran the DP, 4 live query-blocks (blocks x queries of that lane still running),
//   5 pairs inside the length band settled at w + 1 by the q-gram bound (no DP)
constexpr int ED_BV_NCOUNTERS = 6;
// the counters live in ED_CNT_STRIPES stripes of 16 u64 (one 128-byte line each); a wave adds to stripe
// (blockIdx mod ED_CNT_STRIPES) and nmz_ed_plan_counters sums the stripes (one address for the whole grid
// serialised ~10^6 same-address atomics: 10 ms of a 16 ms filter pass)
constexpr uint32_t ED_CNT_STRIPES = 64, ED_CNT_LINE = 16, ED_CNT_WORDS = ED_CNT_STRIPES * ED_CNT_LINE;
// q-gram (bigram) profiles: per trace, ED_QG_BUCKETS counts of hashed adjacent symbol pairs, saturated at 255 and
// packed 4 per dword. One edit changes at most 4 bigram counts by one, so ED >= L1(profile_a, profile_b) / 4
// (merging bigrams into buckets and saturating only lower the L1); L1 > 4w settles ED_w = w + 1 without a DP.
constexpr uint32_t ED_QG_BUCKETS = 128, ED_QG_DW = ED_QG_BUCKETS / 4;
int ed_qgram_profiles(const uint16_t *bs, const uint64_t *soff, const uint32_t *len, uint32_t N, uint32_t *prof,
                      hipStream_t st);
// Two-phase bit-parallel search (ed_bv.hip), used when the q-gram filter is on:
//   1. k_ed_qg_filter over tiles of 64 queries x 256 candidates (a candidate's profile in registers against 64
//      query profiles in LDS) decides every pair's length band and q-gram bound; a count pass sizes, and a write
//      pass fills, per query pair (2p, 2p + 1) a list of entries j | run1 << 30 | run2 << 31 (pairs needing a DP);
//   2. k_ed_bv_dp runs work items of <= `item` entries of one query pair each (its Peq tables in LDS);
//      ed_bv_item() picks the size (NMZ_ED_ITEM overrides, a power of two in [64, 4096]).
constexpr uint32_t ED_BV_ITEM = 4096;  // the largest item
uint32_t ed_bv_item();
struct EdQgArgs {
    const uint4 *prof;           // [N][ED_QG_DW / 4] q-gram profiles
    const uint32_t *len;         // [N]
    uint64_t *knn;               // [N][k]: in-band results decided here (an empty trace in the length band)
    uint64_t *counters;          // [ED_BV_NCOUNTERS] or nullptr (count pass only)
    const uint64_t *tiles;       // [n_tiles] this shard's tiles, qb << 32 | cb
    uint32_t *cnt;               // [n_pairs] entries per query pair: the count pass adds, the write pass takes
                                 // them back (its slots: poff[p] + the count left), so they end at zero again
    const uint32_t *poff;        // write pass: [n_pairs] the pairs' entry offsets
    uint32_t *ent;               // write pass: the entries
    uint4 *recs;                 // count pass: one record per (wave, query pair) with survivors -- {pair, first
                                 // candidate, run1 ballot} and {run2 ballot} (2 uint4) -- for the scatter pass, or
                                 // nullptr (the write pass recomputes the filter); ED_REC_STRIPES regions of rec_cap
    uint32_t *n_rec;             // [ED_REC_STRIPES * ED_REC_LINE] records appended per stripe (workgroup mod
                                 // ED_REC_STRIPES; one counter per 128-byte line: a single counter for the grid
                                 // serialised ~10^5-10^6 same-address atomics); past rec_cap the write pass recomputes
    const uint32_t *rec_cnt;     // scatter pass: [ED_REC_STRIPES] the count pass's records per stripe
    uint32_t rec_cap;            // records per stripe
    uint64_t n_tiles;
    uint32_t N, k, QB, NCB, shard, n_shards;
    uint32_t w;                  // band
    // write pass: the entry lists' capacity, and a device flag that, when set, makes the write pass (and the DP,
    // ed_bv_dp_launch's `abort`) skip: a search enqueued with a shard's cached sizes whose own totals differ
    // (k_tp_scan sets it) must not write past lists sized for the cached totals
    uint64_t ent_cap;
    const uint32_t *abort;
};
constexpr uint32_t ED_REC_STRIPES = 64, ED_REC_LINE = 32;
// the two-phase search's cached-size mismatch flag (ed.hip): wait = synchronise `st` and read it; otherwise read the
// last search's pinned copy if it has landed. Fails (and resets the flag and the cache) when it is set.
int ed_tp_flag_check(nmz_ed_plan *p, bool wait, hipStream_t st);
int ed_qg_filter_launch(const EdQgArgs &A, bool count, hipStream_t st);
int ed_qg_scatter_launch(const EdQgArgs &A, uint32_t n_rec, hipStream_t st);
int ed_bv_dp_launch(const EdBvArgs &A, const uint32_t *ioff, const uint32_t *poff, const uint32_t *ent,
                    uint32_t n_pairs, uint32_t n_items, uint32_t item, uint32_t bw, bool cmp, hipStream_t st,
                    const uint32_t *abort = nullptr);
// single-query search on a bit-parallel plan (ed_bv.hip k_ed_bv_query): 1-2 external queries vs every stored trace
struct EdBvQueryArgs {
    const uint16_t *bsym;  // the plan's stored streams
    const uint64_t *soff;
    const uint32_t *len;
    const uint16_t *qs;    // query streams (plan's Peq-row byte offsets; 0xffff = symbol unknown to the store)
    uint64_t qoff[2];
    uint32_t nq[2];
    uint64_t *knn;         // [n_queries][k]
    const uint4 *prof;     // the stored traces' q-gram profiles, or nullptr: no filter
    uint32_t N, k, lds_dw, pool, n_queries;
    uint32_t w, rmap_dw, claim_dw, row_bytes;  // band; compact tables as in EdBvArgs
};
int ed_bv_query_launch(const EdBvQueryArgs &A, uint32_t bw, bool cmp, uint32_t blocks, hipStream_t st);
// unique.hip: sorted distinct symbols on the device (hipcub radix sort + unique); *n_uniq on the host
int device_unique_u64(const uint64_t *d_sym, uint64_t total, uint64_t *d_uniq, uint64_t cap, uint64_t *n_uniq,
                      hipStream_t st);
int ed_bv_launch(const EdBvArgs &A, uint32_t bw, bool cmp, uint64_t blocks, hipStream_t st);

// wide-band bit-parallel edit distance (ed_wide.hip): one pair per wave
struct EdWideArgs {
    const uint16_t *sym;   // dense symbol ids, CSR order (padded with 64 zeros)
    const uint64_t *off;   // [N+1]
    const uint32_t *rowb;  // per trace, per position: byte offset of that symbol's Peq row (c * ndw * 4),
                           // each trace starting at a multiple of 32 entries, padded by >= 64 zero entries
    const uint64_t *rowb_off;  // [N]: first entry of trace j in rowb
    const uint32_t *peq;   // [N][n_sym][ndw] match bitmaps
    uint64_t *knn;         // [N][k]
    uint64_t n_pairs;      // N(N-1)/2
    uint64_t n_waves;      // waves of this shard (chunks of 32 pairs dealt round-robin)
    uint32_t N, k, n_sym, ndw, shard, n_shards;
    uint32_t w;            // the requested band (<= the kernel's W)
};
bool ed_wide_supported(uint32_t band);   // 64 < band <= 8192
uint32_t ed_wide_template(uint32_t band);  // W = 1024, 2048, 4096 or 8192 >= band
uint32_t ed_wide_ndw(uint32_t band, uint32_t max_len);
int ed_wide_build_peq(const uint16_t *d_sym, const uint64_t *d_off, uint32_t N, uint32_t n_sym, uint32_t ndw,
                      uint32_t band, uint32_t *d_peq, hipStream_t st);
int ed_wide_launch(const EdWideArgs &A, uint32_t band, hipStream_t st);
// single queries: wave (q, j) over n_q query tables qpeq + q * qstride (rows over the store's alphabet) x the N
// stored traces of A; in-band results into A.knn + q * k
int ed_wide_query_launch(const EdWideArgs &A, uint32_t band, const uint32_t *qpeq, uint64_t qstride,
                         const uint32_t *qlen, uint32_t n_q, hipStream_t st);

// replayable plan: one hint-length class (a segment of every table row)
struct ClassInfo {
    uint64_t pn;     // P^len
    uint32_t start;  // first position in the length-sorted event order
    uint32_t count;
};
// K1 wavelet-tree statistics (replayable_wt.hip): per-row images built once per plan, staged into LDS per sweep
struct WtState {
    bool on = false;
    uint32_t rb16 = 0, n_classes = 0, msh = 0;
    uint32_t bb = 5;                        // rank blocks of 2^bb ranks below the tree's levels (replayable_wt.hip)
    uint4 *d_blob = nullptr;                // [256][rb16] row images
    unsigned long long *d_rowsum = nullptr;  // [256] sum of C mod m over the row
    void *d_classes = nullptr;              // [n_classes] segment descriptors
    DevBuf mem;                             // the row images
    DevBuf aux;                             // separate path: row sums and segment descriptors
};
bool wt_enabled();
struct WtClass {
    uint64_t pn;              // P^len
    uint32_t start, n;        // table segment (C order)
    uint32_t o_lv, o_cm;      // byte offsets in the row image: wavelet levels [K][nw] {bits, ones before};
    uint32_t o_chi, o_e;      //   Cm by rank (+ sentinel); C's high word by position (+ sentinel); e by rank (u16)
    uint32_t o_im, o_ic;      //   bucket indexes (u16): first rank with Cm >= b << msh (257); first position
                              //   with C_hi >= b << 24 (256)
    uint32_t K, nw;           // rank bits (2^K > n); words per level (n / 32 + 1)
    uint32_t rS;              // lifting-search rounds (the largest bucket's bit length; set by the plan kernel)
    uint32_t o_mk;            //   block masks [(n >> bb) + 1][2^bb + 1] of 2^bb bits: the ranks (bit r mod 2^bb)
                              //   among the first o entries of each 2^bb-rank block's node, o = 0..2^bb
    uint32_t order;           // plan kernel: the segment whose rows the order-th group of 256 workgroups builds
    uint32_t pad;
};
static_assert(sizeof(WtClass) == 64, "WtClass layout");

// The wavelet-tree images: wt_layout (host only) decides whether they apply and lays out the segments (fused: every
// class must be one segment), wt_launch runs the plan kernel with the classes and zeroed row sums already on the
// device -- with hints (fused) the kernel computes the correction table itself (FNV of each hint per row L, C-sorted
// per class) into hints->table and zeroes the two given ranges; wt_build = the separate path (table built first).
struct WtPlanHints {
    const uint32_t *hoff;
    const uint8_t *hbytes;
    const uint32_t *perm;
    uint4 *table;
    uint32_t *zero0;
    uint32_t n_zero0;
    uint32_t *zero1;
    uint32_t n_zero1;
};
bool wt_layout(WtState &w, nmz_ctx *ctx, uint32_t E, const ClassInfo *cls, uint32_t n_cls, const ModParams &mod,
               bool fused, std::vector<WtClass> &oc);
int wt_launch(WtState &w, const uint4 *d_table, uint32_t E, const ModParams &mod, hipStream_t st,
              const WtPlanHints *hints, WtClass *d_cls, unsigned long long *d_rowsum, bool sync);
int wt_build(WtState &w, nmz_ctx *ctx, const uint4 *d_table, uint32_t E, const ClassInfo *cls, uint32_t n_cls,
             const ModParams &mod, hipStream_t st);
// topk_scratch (wt_topk_scratch_bytes(S), or nullptr): the sweep also leaves per-seed sums (in bucketed order) and
// per-workgroup largest sums there for wt_topk
int wt_sweep(const WtState &w, nmz_ctx *ctx, hipStream_t st, const Buckets &b, const uint4 *d_table, uint32_t E,
             const ModParams &mod, nmz_sched_stats *d_stats, uint64_t S, void *topk_scratch, uint32_t k);
size_t wt_topk_scratch_bytes(uint64_t S);
// the top-k (k <= 64) of a sweep that ran with topk_scratch (the sweep zeroes its candidate counter)
int wt_topk(hipStream_t st, void *scratch, const uint32_t *sorted_idx, uint64_t S, uint64_t seed0, uint32_t k,
            nmz_topk_entry *d_out);

}  // namespace nmz
