/* Shared host/device declarations of the count pipeline (see hm_kernels.hip). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

/* level 1: projection + partition by the zoom-z1 digit */
#ifndef HM_P1_THREADS
#define HM_P1_THREADS 512
#endif
#ifndef HM_P1_PPT
#define HM_P1_PPT 16
#endif
#define HM_T1 (HM_P1_THREADS * HM_P1_PPT) /* 8192 points per tile */
#ifndef HM_P1_GROUP
#define HM_P1_GROUP 4                       /* LDS count+rank atomics in flight per thread */
#endif
#ifndef HM_P1_ILP
#define HM_P1_ILP 1                         /* projections the scheduler may interleave */
#endif
#ifndef HM_P1_WAVES
#define HM_P1_WAVES 1                       /* waves per SIMD the register budget targets */
#endif
#define HM_L1_SHARDS 8                      /* sub-regions of a hot level-1 digit */
#ifndef HM_L1_SHARD_TILES
#define HM_L1_SHARD_TILES 16                /* a digit of more points than this many tiles is sharded (64 until round 5) */
#endif
#define HM_L1_ZERO_SAMPLES 24               /* level-1 region slack per digit, in sample strides */
#define HM_Z1 5                             /* level-1 digit: zoom-5 tile */
#define HM_MAX_F1 1024
/* hot tiles: zoom-zb tiles (the last level's bucket zoom) that a sample shows
 * to hold >= 1/4096 (HM_HOT_INV_SHARE) of the points each.  Level 1 gives each its own digit
 * HM_MAX_F1 + h and writes its keys (u16, zb-relative) straight into the
 * final level's key array, so they skip every intermediate partition pass. */
#ifndef HM_MAX_HOT
#define HM_MAX_HOT 512
#endif
/* hot-tile table: HM_HOT_BUCKETS buckets of 2 entries (one 8-B LDS read per
 * lookup, no probe loop).  Zoom-zb tile (rs, cs) (zb <= 11: both < 2^11) sits
 * in bucket (rs * K + cs) mod HM_HOT_BUCKETS, a bijection of cs for a given
 * rs, so an entry needs only the row as its tag: entry = rs << 16 | h,
 * HM_HOT_EMPTY.  XOR with the looked-up tile's rs << 16 leaves exactly h for
 * the matching way and >= 2^16 for any other (or an empty one).  A candidate
 * whose bucket is full stays cold (k_hot_hash). */
#define HM_HOT_LIMIT HM_MAX_HOT
#define HM_D1 (HM_MAX_F1 + HM_MAX_HOT)      /* level-1 digit slots: cold z1 digits, then hot tiles */
#define HM_HOT_WAYS 2
#define HM_HOT_SLOTS 4096
#define HM_HOT_BUCKETS (HM_HOT_SLOTS / HM_HOT_WAYS)
#define HM_HOT_BBITS 11
#define HM_HOT_TAG 16                       /* entry = rs << HM_HOT_TAG | h */
#define HM_HOT_MULT 0x9E3779u               /* low 11 bits 1913: rows 1..7 apart never share a column's bucket */
#define HM_HOT_CAND 4096                    /* candidates k_hot_select may list */
#define HM_HOT_EMPTY 0xFFFFFFFFu
static_assert(HM_MAX_HOT <= 1024 && (HM_MAX_HOT & 255) == 0, "hot tiles");
/* bucket of zoom-zb tile (rs, cs), zb <= HM_HOT_BBITS */
__host__ __device__ inline uint32_t hm_hot_bucket(uint32_t rs, uint32_t cs)
{
    /* rs < 2^16 and HM_HOT_MULT < 2^24: a 24-bit multiply-add (the compiler,
     * unable to bound rs, otherwise picks a 64-bit v_mad_u64_u32) */
#if defined(__HIP_DEVICE_COMPILE__)
    return (__umul24(rs, HM_HOT_MULT) + cs) & (HM_HOT_BUCKETS - 1u);
#else
    return (rs * HM_HOT_MULT + cs) & (HM_HOT_BUCKETS - 1u);
#endif
}
static_assert(HM_HOT_MULT < (1u << 24), "24-bit hash multiplier");
static_assert(HM_HOT_BUCKETS == 1 << HM_HOT_BBITS, "hot-tile table");
/* level-1 (digit, shard) arrays (fill, rbase, rcap) are shard-major: the
 * digits one wave reserves for sit in consecutive words, so its returning
 * atomics coalesce into a few 64-B requests instead of one per digit */
__host__ __device__ inline uint32_t hm_l1i(uint32_t d, uint32_t sh) { return sh * HM_D1 + d; }
/* levels >= 2 */
#ifndef HM_PN_THREADS
#define HM_PN_THREADS 1024
#endif
#ifndef HM_TN
#define HM_TN 8192                          /* keys per partition work item */
#endif
/* level 2 from the level-1 regions (k_partition_fr): keys in registers */
#ifndef HM_FR_THREADS
#define HM_FR_THREADS 1024
#endif
#ifndef HM_K2_FR
#define HM_K2_FR 1                          /* 0: k_partition (run streaming), 1: k_partition_fr */
#endif
#ifndef HM_FR_GROUP
#define HM_FR_GROUP 4
#endif
#ifndef HM_LEVEL_ZOOMS
#define HM_LEVEL_ZOOMS 6                   /* <= 6 zooms per level */
#endif
#define HM_MAX_FN 4096
#define HM_MAX_SHARDS 32                    /* run-counter shards per child */
#ifndef HM_RUN_SHARD_BITS
#define HM_RUN_SHARD_BITS 4
#endif
/* final aggregation: zoom-zb bucket = 128 x 128 zoom-Z bins */
#define HM_AG_THREADS 1024
#define HM_AG_CELLS 16384
#define HM_AG_LG 7
#ifndef HM_AG_FAST
#define HM_AG_FAST 1                        /* k_aggregate: hm_lds_count_fast (merge only wave-heavy keys) */
#endif
#ifndef HM_TA
#define HM_TA (1u << 18)                    /* keys per aggregation work item */
#endif
/* buckets of <= HM_SP_MAX keys get no dense work item: one wavefront sorts
 * each (k_small_sort / k_small_emit); larger ones go to k_aggregate (512
 * against 2048: 1-hour stream batches 0.57-0.59 -> 0.52-0.53 ms, 1e9 hotspot
 * aggregation -50 us, uniform 6e8 -0.9 ms, skew unchanged;
 * profiles/r5_reentry/sp_*_ab.*) */
#ifndef HM_SP_MAX
#define HM_SP_MAX 512
#endif
/* small final buckets (k_small_sort / k_small_emit): one wavefront per bucket */
#ifndef HM_SPW_MAX
#define HM_SPW_MAX HM_SP_MAX                /* up to 2048 keys supported: 32 per lane */
#endif
/* buckets of <= HM_SPW_SPLIT keys: the narrow (high-occupancy) instantiation */
#ifndef HM_SPW_SPLIT
#define HM_SPW_SPLIT 512
#endif
static_assert(HM_SPW_MAX >= HM_SP_MAX, "every bucket without a dense work item needs the wavefront path");
/* HM_SP_FUSED: the <= 32-key, <= 4-run small buckets go through ONE fused
 * sort + count + emit kernel (k_small_pairs) instead of k_small_sort, a scan
 * and k_small_emit */
#ifndef HM_SP_FUSED
#define HM_SP_FUSED 1
#endif
#define HM_SPW_THREADS 256
#define HM_SPW_GRID (256 * 8)
#ifndef HM_SPP_WAVES
#define HM_SPP_WAVES 4      /* k_small_pairs: waves per block (one cursor reservation per block and round) */
#endif
#ifndef HM_SPP_STAGE
#define HM_SPP_STAGE 1      /* k_small_pairs: cells staged in LDS, written a whole line per instruction */
#endif
#ifndef HM_SPP_ROWS
#define HM_SPP_ROWS 32      /* k_small_pairs: rows (wave passes) per wave and round, <= 32 */
#endif
static_assert(HM_SPP_ROWS <= 32, "a row's two cell counts sit in lanes 2p, 2p + 1");
#define HM_SPP_STAGE_CELLS 512   /* >= a row's cells: 2 segments x 32 keys x 7 levels */
#ifndef HM_SPW_RESIDENT
#define HM_SPW_RESIDENT 0   /* 1: small-bucket grids of the blocks resident at once (hm_spw_grid; slower) */
#endif
#define HM_POOL_THREADS 256
#define HM_MAX_LEVELS 4
#define HM_COUNT_MAX_ZOOM 21                /* level-1 keys 2*(Z-5) bits fit u32 */
#define HM_SCAN_LIMIT (4096ull * 4096ull)   /* dense children per level */
/* run streaming: runs staged per chunk; runs of >= HM_LONG_RUN keys are read
 * by a whole wave with 16-B loads, shorter ones by one lane each */
#define HM_RCH 1024
#define HM_LONG_RUN 32

/* Sharded run region of child (p, d) as the partition kernels write it:
 * parent p owns level tiles [t0, t0+tp); its children's regions start at
 * F*(t0 + S*p), each S*ceil(tp/S) records, shard s of a child at offset
 * s*ceil(tp/S).  Capacity: F*(tiles + S*parents).  The run scan copies every
 * child's shards into one flat, child-ordered list (HmRuns). */
__host__ __device__ inline uint64_t hm_run_base(uint64_t t0, uint64_t tp, uint64_t p, uint64_t d, int dbits,
                                               int shard_bits)
{
    const uint64_t S = 1ull << shard_bits;
    const uint64_t cap = (tp + S - 1) >> shard_bits;
    return ((t0 + S * p) << dbits) + d * (cap << shard_bits);
}

/* Grids with one block per item can exceed the 2^32 work-items a 1-D
 * dispatch allows (4M buckets x 1024 threads): they are 2-D, <= 65536 blocks
 * in x; kernels read their linear block id with hm_block_id(). */
inline dim3 hm_grid2(uint32_t nblocks)
{
    const uint32_t x = nblocks < 65536u ? (nblocks ? nblocks : 1u) : 65536u;
    return dim3(x, (nblocks + x - 1) / x);
}

/* Flat run list of a level: run j holds cnt = run[j].y keys starting at key
 * index run[j].x of the level's key array; its keys are the global logical
 * positions [excl[j], excl[j] + cnt) (exclusive prefix over all runs).  The
 * runs of one bucket are consecutive, so a bucket is a position range. */
struct HmRuns {
    const uint2* run;
    const uint64_t* excl;
};

struct HmBuckets {
    uint32_t count;             /* compact buckets */
    const uint32_t* nkeys;
    const uint32_t* nruns;
    const uint32_t* rbase;      /* first run (flat index) */
    const uint32_t* keybase;    /* first global logical key position */
    const uint32_t* item_begin; /* [count+1] work-item prefix for the next stage */
    const uint32_t* digit;
    const uint64_t* coord;      /* (row << 32) | col of the bucket tile at its zoom */
    const int32_t* slots;       /* last level: merge slot or -1 */
    const uint4* desc;          /* [2*items] work-item descriptors (k_items) */
};

/* work item g: desc[2g] = (bucket, j, nitems, r0), desc[2g+1] = (r1, -, a, b):
 * logical positions [a, b) of the bucket, runs [r0, r1) overlap them */
struct HmItem {
    uint32_t bucket, j, nitems;
    uint32_t r0, r1;
    uint32_t a, b;
};

struct HmOut {
    uint64_t* keys;
    uint64_t* counts;
    uint64_t capacity;
    unsigned long long* cursor;
    int zmin, zmax;
};

/* kept points whose zoom-Z tile lies outside [0, 2^Z)^2, appended (exact
 * tile, input index) for the general path (hm_general.hip); count may pass
 * cap, then the list is rebuilt by k_collect_exotic at the right size */
struct HmExotic {
    int64_t* row;
    int64_t* col;
    int64_t* idx;
    uint64_t cap;
    unsigned long long* count;
};

struct HmCompactOut {
    uint32_t* nkeys;
    uint32_t* nruns;
    uint32_t* rbase;
    uint32_t* keybase;
    uint32_t* item_begin;
    uint32_t* digit;
    uint64_t* coord;
};

/* level 1 (k_project_partition): every kept in-square point's key goes to
 * the contiguous region of its zoom-z1 digit d -- keys [rbase[d], rbase[d] +
 * rcap[d]) of keys_out, filled through the counter fill[d] (one returning
 * atomic per tile and non-empty digit).  Regions are sized from a sampled
 * histogram (k_sample_digits); a tile whose reservation passes rcap[d] drops
 * it and raises *overflow, and the host re-runs the level with exact sizes. */
struct HmPart1Args {
    const double* lat;
    const double* lon;
    const int64_t* rows_in;   /* hm_count_tiles, and resolved redo points */
    const int64_t* cols_in;
    const uint8_t* keep;
    int64_t n;
    int64_t tile0;            /* first tile of the launch (hm_launch_part1 sets it) */
    const unsigned long long* n_dev;   /* tile input: min(*n_dev, n) points (the resolved redo list) */
    int Z, dbits, restbits;
    uint32_t* redo_idx;       /* fast mode: points the fast path could not settle */
    unsigned long long* redo_count;
    uint64_t redo_cap;
    void* keys_out;
    uint32_t* fill;           /* [HM_D1 * HM_L1_SHARDS] per (digit, shard): hm_l1i */
    const uint32_t* rbase;    /* [HM_D1 * HM_L1_SHARDS] */
    const uint32_t* rcap;     /* [HM_D1 * HM_L1_SHARDS] */
    const uint8_t* smask;     /* [F]: shards of digit d - 1 (0 or HM_L1_SHARDS - 1) */
    unsigned long long* overflow;
    unsigned long long* err_word;
    HmExotic x;
    unsigned long long* slow_count;
    /* hot tiles (hot_z >= 0): keys of hot tile h go to the u16 array keys_hot
     * at the regions of digit HM_MAX_F1 + h (same position space as keys_out) */
    int hot_z;
    int hot_bytes;              /* 2: u16 keys_hot (hot tiles at the last level's bucket zoom); 4: u32
                                 * (mid-level hot tiles of a 3-level plan: the middle level's key form) */
    void* keys_hot;
    const uint32_t* hot_hash;   /* [HM_HOT_SLOTS]: bucketed table, tile id << HM_HOT_HBITS | h, HM_HOT_EMPTY */
    const uint32_t* hot_n;      /* device word: number of hot tiles */
};

/* hot-tile selection from the sampled zoom-zb counts (k_hot_select) */
struct HmHotArgs {
    uint32_t* counts;           /* [4^zb] sampled points per zoom-zb tile (zeroed before sampling) */
    int zb, z1;
    uint32_t thresh;            /* sampled points a hot tile needs */
    uint32_t* tiles;            /* [HM_MAX_HOT] tile id (row << zb | col) */
    uint32_t* hist;             /* [HM_D1] level-1 sampled histogram: hot h at HM_MAX_F1 + h */
    uint8_t* hotparent;         /* [HM_MAX_F1] z1 digits that hold a hot tile */
    uint32_t* n;                /* device word: hot tiles found (<= HM_MAX_HOT) */
    uint32_t* hash;             /* [HM_HOT_SLOTS] */
    uint32_t* cand;             /* [2 * HM_HOT_CAND + 1]: (tile, count) candidates, then their number */
};

/* hot tiles as children of the last level's run scan (k_hot_nr / k_hot_runs):
 * their parent is their z1 bucket (d2b) at level 2, or their zoom-zp
 * ancestor's level-2 bucket (c2b) at level 3 */
struct HmHotRunArgs {
    const uint32_t* tiles;
    const uint32_t* n;
    int zb, z1, dbits;
    int zp;                     /* the parent level's zoom */
    const uint32_t* c2b;        /* level 3: level-2 child -> bucket, else NULL */
    const uint32_t* fill;       /* level-1 [HM_D1 * HM_L1_SHARDS] */
    const uint32_t* rbase;
    const uint32_t* d2b;        /* [HM_MAX_F1] z1 digit -> level-1 bucket */
    uint64_t* nr;               /* runs per level-2 child */
    const uint64_t* runbase;
    uint2* flat;
    uint64_t* cnt;
};

/* level-1 buckets (k_level1_buckets) from the filled regions */
struct HmL1Args {
    int F, dbits;
    const uint32_t* fill;
    const uint32_t* rbase;
    const uint8_t* smask;
    uint32_t item_keys, sparse_max;
    HmCompactOut out;
    uint2* runs;
    uint64_t* excl;
    uint32_t* child_begin;
    uint64_t* total;           /* count << 32 | items */
    int32_t* slots;            /* last level only */
    unsigned long long* nslots;   /* multi-item buckets (their merge slots) */
    uint32_t* slot_bucket;
    const uint8_t* hotparent;  /* digits that are buckets for their hot children alone (or null) */
    uint32_t* d2b;             /* digit -> bucket index (or null) */
};

struct HmPartNArgs {
    HmBuckets parent;
    const uint32_t* keys_in;
    HmRuns in;
    int dbits, restbits, shard_bits;
    uint32_t items;             /* blocks of the (2-D) grid that have an item */
    const uint32_t* seg;        /* level-1 parents: per item its runs (k_items), for k_partition_fr */
    void* keys_out;             /* item g writes its keys at its positions [a, b) */
    uint32_t* nruns_out;
    uint2* runs_out;
    /* k_partition_fr, child-contiguous levels (HM_PN_HIST / HM_PN_CONTIG):
     * child = bucket << dbits | digit.  HIST: every item adds its digit
     * counts into ctot[child] and writes nothing else.  CONTIG: with cbase =
     * the exclusive scan of ctot, an item reserves its keys of a child at
     * cbase[child] + atomicAdd(ccur[child]) and the child gets ONE run
     * (cbase, ctot): the next level reads each child as one contiguous run */
    int mode;
    unsigned long long* ctot;
    const unsigned long long* cbase;
    uint32_t* ccur;
    uint32_t cbase_off;         /* CONTIG: added to every child base (hot keys hold the positions below it) */
};
void hm_launch_partition_hist(hipStream_t s, const HmPartNArgs& a);
#define HM_PN_RUNS 0
#define HM_PN_HIST 1
#define HM_PN_CONTIG 2

/* run scan of one level (sharded counters -> flat child-ordered runs) */
struct HmRsArgs {
    uint64_t nchildren;
    int dbits, shard_bits;
    const uint32_t* nruns;      /* [nchildren << shard_bits] sharded counters */
    const uint2* runs;          /* sharded layout */
    const uint32_t* parent_item_begin;
    uint32_t* shoff;            /* [nchildren << shard_bits] shard offset within child */
    uint64_t* nr;               /* [nchildren] runs per child (scan input) */
    const uint64_t* runbase;    /* [nchildren] exclusive scan of nr */
    uint2* flat;                /* flat runs */
    uint64_t* cnt;              /* flat run key counts (scan input) */
    const uint64_t* excl;       /* exclusive scan of cnt */
    uint64_t nflat;             /* total runs (a bound when nflat_dev is set) */
    const uint64_t* nflat_dev;  /* the total on the device, or null */
    const uint64_t* total_keys;
    uint32_t item_keys;
    uint32_t sparse_max;        /* last level: buckets of <= this many keys get no work items */
    uint32_t* nkeys;            /* [nchildren] */
    uint32_t* keybase;          /* [nchildren] */
    uint64_t* vals;             /* [nchildren] (1 << 32 | items) for non-empty children */
    const uint8_t* force;       /* [nchildren] or NULL: children kept as buckets without keys (hot ancestors) */
    uint32_t* big;              /* [HM_RS_BIG_MAX] children with many runs (k_rs_copy_big) */
    uint32_t* nbig;             /* their count */
    uint64_t big_min;           /* runs above which a child is listed */
};
#define HM_RS_BIG_MAX 4096
#define HM_RS_BIG 2048              /* default big_min (HM_RS_BIG_MIN in the environment overrides) */


struct HmCompactArgs {
    uint64_t nchildren;
    uint32_t nparents;
    int dbits;
    const uint64_t* vals;
    const uint64_t* prefix;
    const uint64_t* total;
    const uint32_t* nkeys;
    const uint64_t* nr;
    const uint64_t* runbase;
    const uint32_t* keybase;
    const uint64_t* parent_coord;
    HmCompactOut out;
    uint32_t* child_begin;
    uint32_t* c2b;          /* [nchildren] or NULL: bucket index of each kept child */
    int32_t* slots;         /* last level only */
    unsigned long long* nslots;   /* multi-item buckets (their merge slots) */
    uint32_t* slot_bucket;
};

struct HmAggArgs {
    HmBuckets B;
    const uint16_t* keys;
    HmRuns in;
    int Z, lg;
    uint32_t items, nslots;     /* blocks with work in the (2-D) grids */
    /* small buckets (k_small_sort / k_small_emit) */
    uint16_t* codes;            /* sorted in-bucket Morton codes at each bucket's key range */
    uint64_t* spcnt;            /* [count] cells per small bucket (0 otherwise) */
    const uint64_t* spoff;      /* exclusive scan of spcnt */
    uint64_t* sptotal;
    unsigned long long* spbase; /* output position of the small buckets' region */
    uint32_t spbatch;           /* consecutive buckets per wave step (power of 2, <= 64) */
    uint32_t* spq;              /* k_small_pairs' block-batch counter (zero at launch) */
    unsigned long long* totals;
    uint32_t* gslots;           /* [nslots][HM_AG_CELLS]: a multi-item bucket's summed histogram */
    const uint32_t* slot_bucket;
    HmOut out;
};

struct HmPoolArgs {
    int dbits, z_child, emit_root;
    uint32_t nparents;
    const uint32_t* child_begin;
    const uint32_t* child_digit;
    const unsigned long long* child_totals;
    const uint64_t* parent_coord;
    unsigned long long* parent_totals;
    HmOut out;
};

/* row JSON text of bins (k_format_bins, hm_general.hip) */
struct HmFormatArgs {
    const int64_t *zoom, *row, *col, *value;
    const uint8_t *head, *last;
    const int64_t* offset;
    int64_t n;
    uint8_t* text;
};
void hm_launch_format_bins(hipStream_t s, const HmFormatArgs& a);
struct HmIdArgs {
    const uint8_t* names;
    const int64_t *name_off, *label;
    const uint8_t* spans;
    const int64_t *span_off, *span, *tz, *tr, *tc, *offset;
    int64_t n;
    uint8_t* text;
};
void hm_launch_format_ids(hipStream_t s, const HmIdArgs& a);

/* several memsets in one dispatch (a small call is launch-bound: each
 * hipMemsetAsync is a dispatch of its own) */
#define HM_FILL_MAX 10
struct HmFill {
    void* p[HM_FILL_MAX];
    uint64_t bytes[HM_FILL_MAX];
    uint32_t word[HM_FILL_MAX];    /* the byte value replicated 4 times */
    uint32_t unit[HM_FILL_MAX];    /* 16, 4 or 1: store width (alignment of p and bytes) */
    int k;
};
void hm_fill_add(HmFill& f, void* p, int value, uint64_t bytes);
void hm_launch_fill(hipStream_t s, const HmFill& f);

void hm_launch_project(hipStream_t s, const double* lat, const double* lon, int64_t n, int zoom, int64_t* row,
                       int64_t* col, uint8_t* status, unsigned long long* err_word, unsigned long long* slow);
/* mode: 0 fast path + redo list, 1 tile input (exact row/col given), 2 fused exact (fallback) */
void hm_launch_part1(hipStream_t s, const HmPart1Args& a, uint32_t grid, bool out16, int mode);
/* hot_counts (or null): sampled points per zoom-a.hot_z tile, dense */
void hm_launch_sample_digits(hipStream_t s, const HmPart1Args& a, uint64_t stride_pts, uint32_t* hist,
                             uint32_t* hot_counts);
void hm_launch_hot_select(hipStream_t s, const HmHotArgs& a);
/* region sizes of the F cold digits and (hot_n) the hot tiles' digits; their
 * total -> *total */
void hm_launch_l1_sizes(hipStream_t s, const uint32_t* hist, int F, const uint32_t* hot_n, uint64_t stride,
                        uint32_t* rcap, uint32_t* rbase, uint8_t* smask, unsigned long long* total);
void hm_launch_hot_nr(hipStream_t s, const HmHotRunArgs& a);
void hm_launch_hot_force(hipStream_t s, const HmHotRunArgs& a, uint8_t* force);
void hm_launch_hot_runs(hipStream_t s, const HmHotRunArgs& a);
void hm_launch_level1_buckets(hipStream_t s, const HmL1Args& a);
struct HmRedoArgs {
    const double* lat;
    const double* lon;
    const uint8_t* keep;
    int Z;
    const uint32_t* redo_idx;
    const unsigned long long* redo_count;
    uint64_t cap;
    int64_t* rows_out;
    int64_t* cols_out;
    unsigned long long* out_count;
    unsigned long long* err_word;
    HmExotic x;
};
void hm_launch_redo(hipStream_t s, const HmRedoArgs& a, uint64_t n);
/* every point again (exact projection), appending the kept out-of-square
 * ones: the exotic list outgrew its first capacity.  rows/cols: tile input */
void hm_launch_collect_exotic(hipStream_t s, const double* lat, const double* lon, const int64_t* rows,
                              const int64_t* cols, const uint8_t* keep, int64_t n, int Z, HmExotic x);
/* grouped counts: project every point exactly (errors), list the kept ones */
void hm_launch_project_list(hipStream_t s, const double* lat, const double* lon, const uint8_t* keep,
                            const uint32_t* group, int64_t n, int Z, int64_t* row, int64_t* col, uint32_t* grp,
                            int64_t* idx, unsigned long long* count, unsigned long long* err_word);
/* few_runs: every parent item spans <= HM_L1_SHARDS runs (parents are the
 * level-1 regions): k_partition_fr, else k_partition */
void hm_launch_partN(hipStream_t s, const HmPartNArgs& a, uint32_t items, bool out16, bool few_runs);
/* run scan steps: per-child shard offsets + run totals; flat copy; per-child keys */
void hm_launch_rs_count(hipStream_t s, const HmRsArgs& a);
void hm_launch_rs_copy(hipStream_t s, const HmRsArgs& a);
void hm_launch_rs_keys(hipStream_t s, const HmRsArgs& a);
/* exclusive scan of v[0..n) into out (any n), total into *total; partial: 4096 u64 */
void hm_launch_scan(hipStream_t s, const uint64_t* v, uint64_t n, uint64_t* partial, uint64_t* out, uint64_t* total,
                    const uint64_t* ndev = nullptr);
void hm_launch_compact(hipStream_t s, const HmCompactArgs& a);
/* seg (or null): per item 16 u32, its <= HM_L1_SHARDS runs (k_partition_fr) */
void hm_launch_items(hipStream_t s, const HmBuckets& B, HmRuns in, uint32_t items, uint32_t T, uint4* desc,
                     uint32_t* seg);
void hm_launch_aggregate(hipStream_t s, const HmAggArgs& a, uint32_t items, uint32_t nslots);
/* small buckets: sort pass, scan, one reservation, emit pass (partial: 4096 u64) */
void hm_launch_small(hipStream_t s, const HmAggArgs& a, uint64_t* partial);
void hm_launch_pool(hipStream_t s, const HmPoolArgs& a, uint32_t nparents);
void hm_launch_read_stream(hipStream_t s, const void* a, const void* b, uint64_t bytes_each, uint64_t* sink);
void hm_launch_synth(hipStream_t s, int kind, uint64_t seed, int64_t start, int64_t n, double* lat, double* lon,
                     const double* tab, int k);

/* resident streaming heatmap (hm_stream.hip) */
#define HMS_EMPTY 0xFFFFFFFFFFFFFFFFull   /* empty hash-table key (hm_table.h) */
enum {
    HMS_ST_OCCUPIED = 0, HMS_ST_OVERFLOW = 1, HMS_ST_CURSOR = 2, HMS_ST_BUCKETS = 3, HMS_ST_BFULL = 4,
    HMS_ST_EXOTIC = 5, HMS_ST_BMM = 6 /* a bucket of the batch (the only one if NLIST == 1) */, HMS_ST_NLIST = 7,
    HMS_ST_ERR = 8 /* first bad hour: index << 8 | HM_E_RANGE */, HMS_ST_COUNT = 16
};
#define HMS_MAX_PARTS 64                 /* batches of more buckets take the grouped general path */
#define HMS_NOGROUP 0xFFFFFFFEu          /* kept points without a user group */
#define HMS_ALLGROUPS 0xFFFFFFFFu        /* rollup over every group */
#define HMS_UNDATED 0x50000000u          /* period word of points added without an hour */
#define HMS_MAX_HOUR_OFFSET (1u << 28)   /* hours base .. base + 2^28 - 1 */
#define HMS_TYPE_DAY 1u
#define HMS_TYPE_MONTH 2u
#define HMS_TYPE_YEAR 3u
#define HMS_TYPE_ALLTIME 4u
#define HMS_SKIP 0xFFFFFFFFu
#define HMS_NO_BUCKET 0xFFFFFFFFu
struct HmsTable {
    uint64_t* slots; /* capacity x {key, count} */
    uint64_t mask;   /* capacity - 1 (power of two) */
    unsigned long long* state;
};
struct HmsBuckets {
    uint64_t* keys;  /* capacity x {group << 32 | period word}; the slot index is the bucket id */
    uint64_t mask;
};
struct HmsBucketArgs {
    const uint32_t* group;   /* NULL: HMS_NOGROUP */
    const uint32_t* hour;    /* NULL: HMS_UNDATED */
    const uint8_t* keep;
    uint64_t n;
    uint32_t base;
    HmsBuckets buckets;
    uint32_t* out;           /* bucket per kept point (NULL: not needed) */
    uint32_t* bflag;         /* per bucket: epoch of the last batch that met it */
    uint32_t epoch;          /* this batch's (nonzero) */
    uint32_t* list;          /* the batch's distinct buckets */
    unsigned long long* state;
    unsigned long long* err_word;
};
struct HmsScatterArgs {
    const double* lat;
    const double* lon;
    const uint8_t* keep;
    const uint32_t* bids;
    const uint32_t* loc;     /* bucket -> run */
    uint64_t n;
    uint32_t nparts;         /* kept runs; run nparts = points not kept */
    const uint64_t* start;   /* nparts + 1 run starts */
    unsigned long long* cursor;   /* k_stream_part_count: the run sizes */
    double* lat_out;
    double* lon_out;
};
/* a rollup's cells: the log's, relabeled (k_stream_relabel) */
struct HmsRelabelArgs {
    const uint64_t* keys;    /* the log */
    const uint64_t* counts;
    uint64_t n;
    HmsBuckets buckets;
    int cb, span, merge;
    uint32_t base;
    int64_t select;          /* -1, or the one period value kept */
    uint64_t* keys_out;      /* label bucket << cb | cell */
    uint64_t* counts_out;
    unsigned long long* cursor;   /* cells written */
    unsigned long long* state;
};
/* merged label cells -> caller's arrays (k_stream_emit) */
struct HmsEmitArgs {
    const uint64_t* keys;
    const uint64_t* counts;
    uint64_t n;
    HmsBuckets buckets;
    int cb, zmin, zmax;
    uint32_t base;
    uint64_t* keys_out;
    uint64_t* counts_out;
    uint32_t* groups_out;
    uint32_t* periods_out;
};
void hm_launch_stream_buckets(hipStream_t s, const HmsBucketArgs& a);
void hm_launch_stream_batch_list(hipStream_t s, const uint32_t* list, uint32_t nlist, uint32_t* loc);
void hm_launch_stream_collect(hipStream_t s, const uint32_t* bflag, uint64_t nb, uint32_t epoch, uint32_t* list,
                              unsigned long long* state);
void hm_launch_stream_part_count(hipStream_t s, const HmsScatterArgs& a);
void hm_launch_stream_scatter(hipStream_t s, const HmsScatterArgs& a);
void hm_launch_stream_rekey(hipStream_t s, uint64_t* keys, uint64_t m, uint64_t prefix);
/* the same with the count m = min(*m_dev, cap) and the bucket (the batch's
 * only one: state[HMS_ST_BMM] when state[HMS_ST_NLIST] != 0, else 0) read on
 * the device */
void hm_launch_stream_rekey_dev(hipStream_t s, uint64_t* keys, const unsigned long long* m_dev, uint64_t cap,
                                const unsigned long long* state, int cb);
void hm_launch_stream_convert(hipStream_t s, const int64_t* rec, uint64_t m, int cb, uint64_t* keys, uint64_t* counts,
                              unsigned long long* state);
void hm_launch_stream_init(hipStream_t s, const HmsTable& t);
void hm_launch_stream_fill(hipStream_t s, uint64_t* p, uint64_t n, uint64_t v);
void hm_launch_stream_relabel(hipStream_t s, const HmsRelabelArgs& a);
void hm_launch_stream_emit(hipStream_t s, const HmsEmitArgs& a);

/* general count path (hm_general.hip): sort of 128-bit cell keys + zoom cascade */
struct HmGenArgs {
    const int64_t* row;
    const int64_t* col;
    const uint32_t* group;      /* or null */
    const int64_t* index;       /* input index per entry (error reports), or null */
    uint64_t n;
    int Z;
    uint64_t* klo;              /* key halves (hm_genkey.h) */
    uint64_t* khi;
    unsigned long long* orand;  /* [or_lo, or_hi, and_lo, and_hi] */
    unsigned long long* err_word;
};
/* records of `width` int64: [group,] zoom, row, col, count; with keys set
 * (hm_count's fallback) cells inside [0, 2^z)^2 go to keys/counts instead,
 * both kinds appended at the cursors */
struct HmGenEmit {
    int64_t* cells;
    uint64_t capacity;
    int width;
    int split;
    uint64_t* keys;
    uint64_t* counts;
    uint64_t kcapacity;
    unsigned long long* kcursor;
    unsigned long long* xcursor;
};
void hm_launch_gen_keys(hipStream_t s, const HmGenArgs& a);
/* points -> general-path keys (k_project_keys_fast + k_project_keys_slow) */
struct HmPkArgs {
    const double* lat;
    const double* lon;
    const uint8_t* keep;
    const uint32_t* group;
    int64_t n;
    int Z;
    uint64_t* klo;
    uint64_t* khi;
    unsigned long long* count;      /* keys written (zeroed) */
    unsigned long long* err_word;
    unsigned long long* orand;
    int dense;                      /* no keep mask: key of point i at i (count untouched) */
    int write_hi;                   /* store the high halves (wide keys) */
    uint32_t* redo_idx;             /* points the fast form leaves to the exact chain */
    unsigned long long* redo_count; /* (zeroed) */
    uint64_t redo_cap;
};
void hm_launch_project_keys(hipStream_t s, const HmPkArgs& a);
void hm_launch_tiles_list(hipStream_t s, const int64_t* rows, const int64_t* cols, const uint8_t* keep,
                          const uint32_t* group, int64_t n, int64_t* row, int64_t* col, uint32_t* grp, int64_t* idx,
                          unsigned long long* count);
uint64_t hm_rx_os_tiles(uint64_t n);
int hm_launch_rx_sort(hipStream_t s, bool wide, uint64_t* const* lo, uint64_t* const* hi, uint64_t n, const int* sh,
                      int np, uint8_t* state);
struct HmCascArgs {
    const uint64_t* kin_lo;     /* sorted level-(z+1) cells (or raw keys), low halves */
    const uint64_t* kin_hi;     /* high halves (wide keys only) */
    uint64_t hic;               /* narrow keys: the high half of every key */
    const uint32_t* ein;        /* their END prefixes; null: raw keys, END = i + 1 */
    const uint32_t* m_in;       /* item count on the device (null: m_host) */
    uint64_t m_host;
    int clr;                    /* low key bits cleared for the output level: 2 (Z - z) */
    int Z;                      /* zoom of the raw keys */
    int zin;                    /* zoom of the input cells (their records) */
    int emit;                   /* write the input level's records */
    uint64_t* kout_lo;
    uint64_t* kout_hi;
    uint32_t* eout;
    uint32_t* m_out;
    uint64_t* tstat;            /* look-back words, one per tile */
    uint64_t* tstat2;           /* k_cascade2: the middle level's look-back words */
    uint64_t epoch;             /* distinct per step of a call (tstat zeroed per call) */
    unsigned* ticket;
    const unsigned long long* rbase_in;   /* record offset of the input level */
    unsigned long long* rbase_out;        /* = rbase_in + m (offset of the next level) */
    HmGenEmit e;
};
/* emit_only: 0 one zoom step (k_cascade), 1 the last level's records (k_cascade_emit), 2 two zoom steps
 * (k_cascade2, packed records) */
void hm_launch_cascade(hipStream_t s, const HmCascArgs& a, uint64_t bound, int emit_only, bool wide);
uint64_t hm_cascade_tiles(uint64_t n);

/* multi-GPU cell exchange (hm_merge.hip) */
struct HmRouteArgs {
    const uint64_t* keys;
    const uint64_t* counts;
    uint64_t n;
    int nranks, delta, dense_zmax;
    uint64_t* grid;            /* dense zooms 0..dense_zmax, Morton order per zoom */
    uint64_t* block_cnt;       /* [nranks * blocks] pass 1 */
    const uint64_t* block_off; /* [nranks * blocks] exclusive scan of block_cnt */
    uint64_t* keys_out;
    uint64_t* counts_out;      /* u64 counts, or */
    uint32_t* counts_out32;    /* u32 counts, or */
    uint16_t* rec_out;         /* 10-B records (48-bit key, u32 count; hm_rec_put) */
    unsigned long long* wide;  /* u32 counts: set when a sent count needs 64 bits */
    int grouped;               /* HM_CELLS_G12: counts = group << 32 | count (hm_count_grouped_packed);
                                  the owner hashes (group, row key); keys_out = hm_gkey packed merge keys */
    /* hm_cells_route_pieces (k_xroute_*): digit = owner << bits | the top `bits` bits of the merge
     * key's hash (the owner's first merge digit); C blocks, block_cnt/block_off [digits * C]
     * digit-major; sizes: device rows of `stride` int64 per owner (sent, wide, pieces) */
    int bits;
    uint32_t C;
    long long* sizes;
    int stride;
    int self;                  /* >= 0: that owner's group goes last (the others in rank order) */
};
#define HM_XR_MAXD 1024               /* route digits (nranks << bits) */
void hm_launch_xroute(hipStream_t s, const HmRouteArgs& a, bool scatter, int layout);
void hm_launch_xroute_sizes(hipStream_t s, const HmRouteArgs& a);
/* owner side of the pieces exchange: run r's piece of first digit s (all of
 * its cells with that digit) starts at device address kp[s R + r] (records,
 * or keys with their counts at cp[s R + r]); the S segments are each cut into
 * C chunks of their R pieces' concatenation (virtual starts vpre[s (R + 1) + r])
 * and partitioned by the next `bits` hash bits into u64 keys and u32 (records
 * and u32 input) or u64 counts */
struct HmMbGather {
    const unsigned long long* vpre;
    const unsigned long long* kp;
    const unsigned long long* cp;
    uint32_t R, S, C;
    int shift, bits, in_layout;
    uint64_t* cnt;
    const uint64_t* off;
    uint64_t* kout;
    void* cout;
    /* fill mode (no count pass): bucket (s, d) holds <= bcap cells at
     * kout/cout + (s << bits | d) * bcap, claimed per tile from fill[]; a
     * bucket that would pass bcap sets *over (the caller partitions again
     * with the count pass) */
    unsigned long long* fill;
    uint64_t bcap;
    unsigned long long* over;
};
void hm_launch_mb_gather(hipStream_t s, const HmMbGather& a, bool scatter);
/* grouped exchange key: group (17 bits) | zoom (5) | row (21) | col (21) */
#define HM_GKEY_GROUP_BITS 17
__host__ __device__ inline uint64_t hm_gkey(uint64_t hmkey, uint32_t g)
{
    return ((uint64_t)g << 47) | ((hmkey >> 58) << 42) | (((hmkey >> 29) & 0x1FFFFFull) << 21) | (hmkey & 0x1FFFFFull);
}
unsigned hm_route_blocks(uint64_t n);
/* bucketed merge of (key, count) cells: hash-partition into 2^lb buckets
 * (count + scatter passes over nblocks input chunks), then one block per
 * bucket sums equal keys in an LDS table and writes the distinct cells */
#define HM_MB_TS 4096                 /* LDS table slots per merge block (buckets of <= ~1800 cells: one pass) */
#define HM_MB_THREADS 1024
struct HmMergeArgs {
    const uint64_t* keys;
    const uint64_t* counts;
    uint64_t n;
    int lb;
    uint32_t nblocks;
    uint64_t* bcnt;            /* [2^lb * nblocks] cells per (bucket, chunk), bucket-major */
    uint64_t* boff;            /* its exclusive scan, total at [2^lb * nblocks] */
    uint64_t* pkeys;           /* partitioned cells */
    uint64_t* pcounts;
    const uint32_t* pcounts32; /* k_mb_merge2: u32 counts instead of pcounts */
    const unsigned long long* bfill;   /* k_mb_merge2: buckets of bfill[b] cells at b * bcap (else boff) */
    uint64_t bcap;
    uint64_t* keys_out;
    uint64_t* counts_out;
    uint64_t cap;
    unsigned long long* cursor;
    unsigned long long* overflow;   /* an LDS table filled up: the caller falls back */
};
/* one hash-partition pass of the bucketed merge (k_mb_pass): segment s of
 * the input (all of it when segoff is null, else [segoff[s * segstride],
 * segoff[(s + 1) * segstride])) is cut into C chunks, one block each; digit
 * = (hms_hash(key) >> shift) & (2^bits - 1); cnt/off index ((s << bits) + d)
 * * C + c, so their scan is in (segment, digit, chunk) order */
struct HmMbPass {
    const uint64_t* kin;
    const uint64_t* cin;
    const uint32_t* cin32;      /* u32 input counts instead of cin (pass 1 of a merge of received cells) */
    const uint16_t* rin;        /* or 10-B records instead of kin/cin (hm_rec_put) */
    uint64_t n;
    const uint64_t* segoff;
    uint32_t segstride, nseg, C;
    int shift, bits;
    uint64_t* cnt;
    const uint64_t* off;
    uint64_t* kout;
    uint64_t* cout;
};
void hm_launch_mb_pass(hipStream_t s, const HmMbPass& a, bool scatter);
void hm_launch_mb_merge(hipStream_t s, const HmMergeArgs& a);
/* the pieces merge (k_mb_merge2): LDS tables of HM_MB2_TS slots, blocks of
 * HM_MB2_T threads; the host sizes buckets to <= HM_MB2_TARGET cells */
#ifndef HM_MB2_TS
#define HM_MB2_TS 4096
#endif
#ifndef HM_MB2_T
#define HM_MB2_T 512
#endif
#define HM_MB2_TARGET (HM_MB2_TS * 7 / 16)
void hm_launch_mb_merge2(hipStream_t s, const HmMergeArgs& a);
void hm_launch_cells_merge32(hipStream_t s, const uint64_t* keys, const uint32_t* counts, uint64_t n,
                             const HmsTable& t);
void hm_launch_cells_route(hipStream_t s, const HmRouteArgs& a, bool scatter);
void hm_launch_cells_merge(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n, const HmsTable& t);
void hm_launch_cells_merge_unique(hipStream_t s, const uint64_t* keys, const uint64_t* counts, uint64_t n,
                                  const HmsTable& t);
void hm_launch_table_extract(hipStream_t s, const HmsTable& t, uint64_t* keys_out, uint64_t* counts_out, uint64_t cap,
                             unsigned long long* cursor);
void hm_launch_dense_extract(hipStream_t s, const uint64_t* grid, uint64_t total, int dense_zmax, uint64_t* keys_out,
                             uint64_t* counts_out, uint64_t cap, unsigned long long* cursor);
