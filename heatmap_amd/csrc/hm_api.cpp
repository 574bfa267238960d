/* C-ABI of heatmap_amd (include/heatmap_amd.h): context, device memory arena
 * and the host-side orchestration of the count pipeline.
 *
 * Per hm_count call (Z = zmax, zb = max(0, Z-7)):
 *   levels z_1 = min(6, zb), z_{l+1} = min(z_l + 5, zb) ... z_L = zb
 *   k_project_partition (level 1) -> [k_runscan, scan, k_compact, k_partition]*
 *   -> k_aggregate (zooms Z..zb+1) -> k_pool for l = L..1 (zooms zb..0).
 * The host reads back two or three scalars per level (bucket and work-item
 * counts) to size the next grid; everything else stays on the device.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <math.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/heatmap_amd.h"
#include "hm_genkey.h"
#include "hm_pipeline.h"

namespace {

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
};

struct Level {
    int zc;              /* child zoom z_l */
    int dbits;           /* 2*(z_l - z_{l-1}) */
    uint32_t nparents;   /* |B_{l-1}| */
    uint64_t nchildren;  /* nparents << dbits */
    uint32_t count = 0;  /* |B_l| */
    uint32_t items = 0;  /* work items of the next stage */
    bool out16 = false;
};

}  // namespace

#define HM_SPREAD_MIN_KEYS (1u << 19)
/* with hot tiles: the cold keys' mean level-1 bucket above which they take
 * 3-zoom levels.  Off by default: measured slower (hotspots 6.6 -> 7.0 ms,
 * skew 15.4 -> 24.7 ms: the middle level's run-streaming partition and a
 * pool over 64K zoom-8 buckets cost more than the short runs they save) */
#define HM_SPREAD_MIN_COLD 1e30
#define HM_SPREAD_ZOOMS 3

/* per-call stage events: [0..4] stage boundaries, [5..] pairs around the
 * level >= 2 partition launches */
#define HM_NEV 12

struct hm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<Buf> bufs;
    unsigned long long* state = nullptr;      /* device: err, exotic count, slow, cursor, nslots, ... */
    unsigned long long* host_state = nullptr; /* pinned mirror */
    int last_levels = 0;                      /* partition levels of the last count (stats [7]) */
    uint32_t* host_aux = nullptr;             /* pinned: level-1 histogram / region sizes */
    int64_t last_err_index = -1;
    int last_err_kind = 0;
    int64_t last_slow = 0;
    double stage_us[8] = {0};
    hipEvent_t ev[HM_NEV];
    /* plan-tuning knobs, read once from the environment at hm_ctx_create
     * (INTEGRATION.md): HM_SPREAD_MIN_KEYS, HM_RS_BIG_MIN */
    double spread_min_keys = 0;
    double spread_min_cold = 0;
    int sample_log2 = 18;              /* level-1 region sizing: ~2^sample_log2 sampled points */
    int debug_l1 = 0;                  /* HM_DEBUG_L1: report level-1 region overflows on stderr */
    int stage_timing = 1;              /* HM_STAGE_TIMING=0: no stage events (hm_last_stats stages read 0) */
    int contig = 1;                    /* HM_CONTIG=0: 3-level plans keep run-streaming at the last level */
    uint32_t ta_min = 16384;           /* HM_TA_MIN: smallest aggregation work item (keys) */
    uint32_t ta_items = 128;           /* HM_TA_ITEMS: items' worth of points a call must have before ta halves */
    /* a stream's tail cells: the count re-keys them under the batch's bucket
     * (read on the device from the stream state) before its last read-back */
    uint64_t* tail_keys = nullptr;
    const unsigned long long* tail_state = nullptr;
    int tail_cb = 0;
    int tail_done = 0;
    uint64_t rs_big_min = 0;
    /* hot tiles (hm_pipeline.h): HM_HOT=0 turns them off; a tile is hot with
     * >= 1/hot_inv_share of the sampled points and >= hot_min_keys estimated */
    int hot = 1;
    int hot_mid = 1;               /* HM_HOT_MID=0: no hot tiles in 3-level plans (zmax 19-21) */
    double hot_inv_share = 4096;   /* 2048 -> 4096: 291 -> 470 hot tiles on the bench cloud, -0.13 ms */
    double hot_min_keys = 65536;
    int run_shard_bits = -1;   /* HM_RUN_SHARD_BITS: level >= 2 run-counter shards (-1: by plan) */
};

enum {
    ST_ERR = 0,
    ST_XCOUNT = 1,
    ST_SLOW = 2,
    ST_CURSOR = 3,
    ST_NSLOTS = 4,
    ST_REDO = 5,
    ST_REDO_OUT = 6,
    ST_XCURSOR = 7,
    ST_OVERFLOW = 8,
    ST_NHOT = 9,          /* hot tiles of this call (k_hot_select; low 32 bits) */
    ST_L1TOTAL = 10,      /* level-1 regions' total capacity (k_l1_sizes) */
    ST_LTOT = 12,         /* 12..14: a partition level's run, key and bucket totals (its run scans),
                           * read back with the state in one copy */
    ST_COUNT = 16
};

static int hip_fail(hipError_t e, const char* what)
{
    if (e == hipSuccess) return HM_OK;
    fprintf(stderr, "heatmap_amd: HIP error in %s: %s\n", what, hipGetErrorString(e));
    return HM_E_HIP;
}

#define HIPCHK(x)                                  \
    do {                                           \
        int _st = hip_fail((x), #x);               \
        if (_st != HM_OK) return _st;              \
    } while (0)

/* Wait for the stream.  HM_SYNC_SPIN_US > 0 (environment, read once per
 * process): poll it for up to that long first, then block.  (Measured with a
 * HIP API trace: after a polled wait the next few launches took ~60 us each
 * instead of ~6, so the default is a plain blocking wait.) */
static int hm_spin_us()
{
    static const int us = [] {
        const char* e = getenv("HM_SYNC_SPIN_US");
        return e ? atoi(e) : 0;
    }();
    return us;
}
static hipError_t hm_sync(hipStream_t s)
{
    const int spin = hm_spin_us();
    if (spin > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady) return e;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin)) break;
        }
    }
    return hipStreamSynchronize(s);
}

/* named arena slots */
enum {
    B_KEYS_A, B_KEYS_B, B_RUNS_SH, B_FLAT_A, B_FLAT_B, B_EXCL_A, B_EXCL_B, B_CNT, B_SHOFF, B_NR, B_NRUNS,
    B_NKEYS, B_KEYBASE, B_VALS, B_PREFIX, B_PARTIAL, B_TOTAL, B_ROOT, B_REDO_IDX, B_REDO_ROWS, B_REDO_COLS,
    B_RUNBASE0,
    B_BK0 = B_RUNBASE0 + HM_MAX_LEVELS, /* 4 levels x 8 arrays */
    B_CHILD0 = B_BK0 + HM_MAX_LEVELS * 8,
    B_TOT0 = B_CHILD0 + HM_MAX_LEVELS,
    B_SLOTS = B_TOT0 + HM_MAX_LEVELS + 1,
    B_SLOTBKT, B_GSLOTS, B_SPCODES, B_DESC0,
    /* exotic list and the general path (hm_general.hip) */
    B_X_ROW = B_DESC0 + HM_MAX_LEVELS, B_X_COL, B_X_IDX, B_GEN_KA, B_GEN_KB, B_GEN_FLAG, B_GEN_IDX, B_GEN_C,
    B_GEN_KHA, B_GEN_KHB, B_GEN_HIST, B_GEN_ORAND, B_GL_GRP,
    B_L1_FILL, B_L1_RBASE, B_L1_RCAP, B_L1_HIST, B_L1_SMASK,
    B_RT_CNT, B_RT_OFF, B_MG_TABLE, B_MG_STATE, B_SEG, B_RS_BIG,
    B_HOT, B_HOT_COUNTS, B_HOT_PARENT, B_D2B, B_MB_CNT, B_MB_OFF, B_MB_KEYS, B_MB_COUNTS, B_MB_CNT2, B_MB_OFF2,
    B_MB_KEYS2, B_MB_COUNTS2, B_KEYS_C, B_HOT_FORCE, B_C2B, B_SEG2, B_CTOT, B_CBASE, B_CCUR, B_MG_PIECES,
    B_COUNT
};

static int ensure(hm_ctx* c, int slot, size_t bytes, void** out)
{
    if (bytes == 0) bytes = 16;
    Buf& b = c->bufs[slot];
    if (b.cap < bytes) {
        if (b.p) HIPCHK(hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        size_t want = bytes + bytes / 8;
        if (hipMalloc(&b.p, want) != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            return HM_E_NOMEM;
        }
        b.cap = want;
    }
    *out = b.p;
    return HM_OK;
}

/* the arena is a cache: after an allocation failure every buffer is
 * released at the API boundary (nothing of the failed call is in flight
 * past the synchronisation) so the next call starts from an empty arena */
static void arena_release(hm_ctx* c)
{
    (void)hipStreamSynchronize(c->stream);
    for (auto& b : c->bufs) {
        if (b.p) (void)hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    (void)hipGetLastError();
}

#define ENSURE(slot, bytes, ptr)                                         \
    do {                                                                 \
        void* _p = nullptr;                                              \
        int _st = ensure(ctx, (slot), (size_t)(bytes), &_p);             \
        if (_st != HM_OK) return _st;                                    \
        ptr = (decltype(ptr))_p;                                         \
    } while (0)

extern "C" {

int hm_abi_version(void) { return HM_ABI_VERSION; }

const char* hm_status_string(int s)
{
    switch (s) {
    case HM_OK: return "ok";
    case HM_E_NAN: return "cannot convert float NaN to integer";
    case HM_E_DOMAIN: return "math domain error";
    case HM_E_INF: return "cannot convert float infinity to integer";
    case HM_E_RANGE: return "value outside the range supported by the device path";
    case HM_E_EXOTIC: return "the streaming heatmap holds tiles inside [0, 2^zmax)^2 only";
    case HM_E_ARG: return "invalid argument";
    case HM_E_CAPACITY: return "output capacity too small";
    case HM_E_WIDE: return "a routed count needs 64 bits (route again with count_bytes = 8)";
    case HM_E_HIP: return "HIP runtime error";
    case HM_E_NOMEM: return "device allocation failed";
    default: return "unknown status";
    }
}

int hm_ctx_create(hm_ctx** out, int device, void* stream)
{
    if (!out) return HM_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
        (void)hipGetLastError();
        fprintf(stderr, "heatmap_amd: no HIP device %d (found %d); there is no CPU fallback\n", device, n);
        return HM_E_HIP;
    }
    HIPCHK(hipSetDevice(device));
    hm_ctx* c = new hm_ctx();
    c->device = device;
    c->stream = (hipStream_t)stream;
    c->bufs.resize(B_COUNT);
    for (int i = 0; i < HM_NEV; i++) c->ev[i] = nullptr;
    c->spread_min_keys = HM_SPREAD_MIN_KEYS;
    if (const char* e = getenv("HM_SPREAD_MIN_KEYS")) c->spread_min_keys = atof(e);
    c->spread_min_cold = HM_SPREAD_MIN_COLD;
    if (const char* e = getenv("HM_SPREAD_MIN_COLD")) c->spread_min_cold = atof(e);
    c->rs_big_min = HM_RS_BIG;
    if (const char* e = getenv("HM_RS_BIG_MIN")) c->rs_big_min = (uint64_t)atoll(e);
    if (const char* e = getenv("HM_HOT")) c->hot = atoi(e);
    if (const char* e = getenv("HM_HOT_MID")) c->hot_mid = atoi(e);
    if (const char* e = getenv("HM_HOT_INV_SHARE")) c->hot_inv_share = atof(e);
    if (const char* e = getenv("HM_HOT_MIN_KEYS")) c->hot_min_keys = atof(e);
    if (const char* e = getenv("HM_RUN_SHARD_BITS")) c->run_shard_bits = atoi(e);
    if (const char* e = getenv("HM_SAMPLE_LOG2")) c->sample_log2 = std::min(30, std::max(8, atoi(e)));
    if (const char* e = getenv("HM_DEBUG_L1")) c->debug_l1 = atoi(e);
    if (const char* e = getenv("HM_STAGE_TIMING")) c->stage_timing = atoi(e);
    if (const char* e = getenv("HM_CONTIG")) c->contig = atoi(e);
    if (const char* e = getenv("HM_TA_MIN")) c->ta_min = (uint32_t)std::max(1024, std::min((int)HM_TA, atoi(e)));
    if (const char* e = getenv("HM_TA_ITEMS")) c->ta_items = (uint32_t)std::max(1, atoi(e));
    int st = HM_OK;
    if (hipMalloc(&c->state, ST_COUNT * sizeof(unsigned long long)) != hipSuccess) {
        c->state = nullptr;
        st = HM_E_NOMEM;
    } else if (hipHostMalloc(&c->host_state, 4 * ST_COUNT * sizeof(unsigned long long)) != hipSuccess) {
        c->host_state = nullptr;
        st = HM_E_NOMEM;
    } else if (hipHostMalloc(&c->host_aux, (2 + 2 * HM_L1_SHARDS) * HM_D1 * sizeof(uint32_t)) != hipSuccess) {
        c->host_aux = nullptr;
        st = HM_E_NOMEM;
    }
    for (int i = 0; i < HM_NEV && st == HM_OK; i++)
        if (hipEventCreate(&c->ev[i]) != hipSuccess) {
            c->ev[i] = nullptr;
            st = HM_E_HIP;
        }
    if (st != HM_OK) {
        (void)hipGetLastError();
        hm_ctx_destroy(c);
        return st;
    }
    *out = c;
    return HM_OK;
}

int hm_ctx_set_stream(hm_ctx* c, void* stream)
{
    if (!c) return HM_E_ARG;
    c->stream = (hipStream_t)stream;
    return HM_OK;
}

int hm_ctx_tune(hm_ctx* c, const char* name, double value, double* old)
{
    if (!c || !name) return HM_E_ARG;
    double prev;
    if (!strcmp(name, "HM_SPREAD_MIN_KEYS")) {
        prev = c->spread_min_keys;
        c->spread_min_keys = value;
    } else if (!strcmp(name, "HM_SPREAD_MIN_COLD")) {
        prev = c->spread_min_cold;
        c->spread_min_cold = value;
    } else if (!strcmp(name, "HM_CONTIG")) {
        prev = c->contig;
        c->contig = value != 0;
    } else if (!strcmp(name, "HM_STAGE_TIMING")) {
        prev = c->stage_timing;
        c->stage_timing = value != 0;
    } else if (!strcmp(name, "HM_SAMPLE_LOG2")) {
        if (!(value >= 8 && value <= 30)) return HM_E_ARG;
        prev = c->sample_log2;
        c->sample_log2 = (int)value;
    } else if (!strcmp(name, "HM_RS_BIG_MIN")) {
        prev = (double)c->rs_big_min;
        c->rs_big_min = (uint64_t)(value < 0 ? 0 : value);
    } else if (!strcmp(name, "HM_HOT")) {
        prev = c->hot;
        c->hot = value != 0;
    } else if (!strcmp(name, "HM_HOT_MID")) {
        prev = c->hot_mid;
        c->hot_mid = value != 0;
    } else if (!strcmp(name, "HM_HOT_INV_SHARE")) {
        if (!(value >= 1)) return HM_E_ARG;
        prev = c->hot_inv_share;
        c->hot_inv_share = value;
    } else if (!strcmp(name, "HM_HOT_MIN_KEYS")) {
        prev = c->hot_min_keys;
        c->hot_min_keys = value;
    } else if (!strcmp(name, "HM_RUN_SHARD_BITS")) {
        if (value > 5) return HM_E_ARG;
        prev = c->run_shard_bits;
        c->run_shard_bits = value < 0 ? -1 : (int)value;
    } else {
        return HM_E_ARG;
    }
    if (old) *old = prev;
    return HM_OK;
}

/* the plan-tuning fields of one context copied to another (a stream's helper
 * contexts count with the settings of the stream's own) */
static void ctx_copy_tuning(hm_ctx* d, const hm_ctx* c)
{
    d->spread_min_keys = c->spread_min_keys;
    d->spread_min_cold = c->spread_min_cold;
    d->sample_log2 = c->sample_log2;
    d->debug_l1 = c->debug_l1;
    d->stage_timing = c->stage_timing;
    d->contig = c->contig;
    d->ta_min = c->ta_min;
    d->ta_items = c->ta_items;
    d->rs_big_min = c->rs_big_min;
    d->hot = c->hot;
    d->hot_mid = c->hot_mid;
    d->hot_inv_share = c->hot_inv_share;
    d->hot_min_keys = c->hot_min_keys;
    d->run_shard_bits = c->run_shard_bits;
}

int hm_ctx_destroy(hm_ctx* c)
{
    if (!c) return HM_OK;
    (void)hipSetDevice(c->device);
    for (auto& b : c->bufs)
        if (b.p) (void)hipFree(b.p);
    if (c->state) (void)hipFree(c->state);
    if (c->host_state) (void)hipHostFree(c->host_state);
    if (c->host_aux) (void)hipHostFree(c->host_aux);
    for (int i = 0; i < HM_NEV; i++)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    delete c;
    return HM_OK;
}

int hm_last_error(hm_ctx* c, int64_t* index, int* kind)
{
    if (!c) return HM_E_ARG;
    if (index) *index = c->last_err_index;
    if (kind) *kind = c->last_err_kind;
    return HM_OK;
}

int hm_last_stats(hm_ctx* c, int64_t* slow_points, double* stage_us, int n_stages)
{
    if (!c) return HM_E_ARG;
    if (slow_points) *slow_points = c->last_slow;
    for (int i = 0; i < n_stages && i < 8; i++) stage_us[i] = c->stage_us[i];
    if (n_stages > 7) stage_us[7] = (double)c->last_levels;
    return HM_OK;
}

}  // extern "C"

static int reset_state(hm_ctx* ctx)
{
    HIPCHK(hipMemsetAsync(ctx->state, 0, ST_COUNT * sizeof(unsigned long long), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->state + ST_ERR, 0xFF, sizeof(unsigned long long), ctx->stream));
    return HM_OK;
}

static int read_state(hm_ctx* ctx)
{
    HIPCHK(hipMemcpyAsync(ctx->host_state, ctx->state, ST_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hm_sync(ctx->stream));
    return HM_OK;
}

static int take_error(hm_ctx* ctx)
{
    const unsigned long long e = ctx->host_state[ST_ERR];
    ctx->last_slow = (int64_t)ctx->host_state[ST_SLOW];
    /* the first failing point in input order (atomicMin of index << 8 | kind) */
    if (e == ~0ull) {
        ctx->last_err_index = -1;
        ctx->last_err_kind = HM_OK;
        return HM_OK;
    }
    ctx->last_err_index = (int64_t)(e >> 8);
    ctx->last_err_kind = (int)(e & 0xFF);
    return ctx->last_err_kind;
}

extern "C" int hm_project(hm_ctx* ctx, const double* lat, const double* lon, int64_t n, int zoom, int64_t* row,
                          int64_t* col, uint8_t* status)
{
    /* zoom may be negative: Tile.parent_id of a zoom-0 tile projects at zoom
     * -1, i.e. times 2**-1 = 0.5 (tile.py:60-61) */
    if (!ctx || n < 0 || zoom < -30 || zoom > 30 || (n > 0 && (!lat || !lon || !row || !col || !status)))
        return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    int st = reset_state(ctx);
    if (st) return st;
    if (n > 0)
        hm_launch_project(ctx->stream, lat, lon, n, zoom, row, col, status, ctx->state + ST_ERR, ctx->state + ST_SLOW);
    HIPCHK(hipGetLastError());
    if ((st = read_state(ctx))) return st;
    return take_error(ctx);
}

/* ------------------------------------------------------------------------ */

/* ------------------------------------------------------------------------ */
/* general path: n exact zoom-Z tiles (device lists) -> records of zooms       */
/* [zmin, Z] (hm_general.hip).  *total = records (all of them, even past the   */
/* capacity).  Errors (tiles beyond the key's range) go to the error word.      */
/* ------------------------------------------------------------------------ */
#ifndef HM_CS_FUSE
#define HM_CS_FUSE 1   /* packed grouped records: two zoom steps per cascade launch (k_cascade2) */
#endif
static int gen_count(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint32_t* group, const int64_t* index,
                     uint64_t n, int Z, int zmin, const HmGenEmit& e, uint64_t* total, const double* lat = nullptr,
                     const double* lon = nullptr, const uint8_t* keep = nullptr)
{
    *total = 0;
    if (n == 0) return HM_OK;
    if (n >= (1ull << 32)) return HM_E_ARG;   /* radix ranks are u32 */
    hipStream_t s = ctx->stream;
    uint64_t *klo[2], *khi[2];
    unsigned long long* orand;
    ENSURE(B_GEN_KA, n * 8, klo[0]);
    ENSURE(B_GEN_KB, n * 8, klo[1]);
    ENSURE(B_GEN_KHA, n * 8, khi[0]);
    ENSURE(B_GEN_KHB, n * 8, khi[1]);
    ENSURE(B_GEN_ORAND, 4 * 8, orand);
    unsigned long long* up = ctx->host_state + ST_COUNT;
    HIPCHK(hm_sync(s));
    up[0] = 0;
    up[1] = 0;
    up[2] = ~0ull;
    up[3] = ~0ull;
    HIPCHK(hipMemcpyAsync(orand, up, 4 * 8, hipMemcpyHostToDevice, s));
    if (lat) {
        /* points: projected straight into keys (the kept ones, compacted) */
        HmPkArgs pk;
        pk.lat = lat;
        pk.lon = lon;
        pk.keep = keep;
        pk.group = group;
        pk.n = (int64_t)n;
        pk.Z = Z;
        pk.klo = klo[0];
        pk.khi = khi[0];
        pk.count = ctx->state + ST_XCOUNT;
        pk.err_word = ctx->state + ST_ERR;
        pk.orand = orand;
        pk.redo_cap = std::min<uint64_t>(n, std::max<uint64_t>(1u << 16, n / 256));
        ENSURE(B_REDO_IDX, pk.redo_cap * sizeof(uint32_t) + 4, pk.redo_idx);
        pk.redo_count = ctx->state + ST_REDO;
        pk.dense = keep == nullptr;
        pk.write_hi = 0;
        HIPCHK(hipMemsetAsync(ctx->state + ST_XCOUNT, 0, sizeof(unsigned long long), s));
        HIPCHK(hipMemsetAsync(ctx->state + ST_REDO, 0, sizeof(unsigned long long), s));
        hm_launch_project_keys(s, pk);
        HIPCHK(hipGetLastError());
        unsigned long long* dn = ctx->host_state + 2 * ST_COUNT;
        HIPCHK(hipMemcpyAsync(dn, orand, 4 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hm_sync(s));
        if (dn[1] != dn[3]) {
            /* wide keys (groups past 2^22 at zoom 21, tiles outside the
             * square): again, with the high halves */
            HIPCHK(hipMemcpyAsync(orand, up, 4 * 8, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemsetAsync(ctx->state + ST_XCOUNT, 0, sizeof(unsigned long long), s));
            HIPCHK(hipMemsetAsync(ctx->state + ST_REDO, 0, sizeof(unsigned long long), s));
            pk.write_hi = 1;
            hm_launch_project_keys(s, pk);
        }
    } else {
        HmGenArgs ga;
        ga.row = row;
        ga.col = col;
        ga.group = group;
        ga.index = index;
        ga.n = n;
        ga.Z = Z;
        ga.klo = klo[0];
        ga.khi = khi[0];
        ga.orand = orand;
        ga.err_word = ctx->state + ST_ERR;
        hm_launch_gen_keys(s, ga);
    }
    HIPCHK(hipGetLastError());
    unsigned long long* down = ctx->host_state + 2 * ST_COUNT;
    HIPCHK(hipMemcpyAsync(down, orand, 4 * 8, hipMemcpyDeviceToHost, s));
    int st;
    if ((st = read_state(ctx))) return st;
    if ((st = take_error(ctx))) return st;
    if (lat && keep) {
        n = ctx->host_state[ST_XCOUNT];
        if (n == 0) return HM_OK;
    }
    /* LSD passes over the digits that differ between keys; the high halves
     * move only when they differ */
    const bool wide = down[1] != down[3];
    const unsigned __int128 var = ((((unsigned __int128)down[1]) << 64) | down[0]) ^
                                  ((((unsigned __int128)down[3]) << 64) | down[2]);
    if (e.width == 2) {
        /* packed records hold HM_KEYs: every key's super tile (its zoom-0
         * tile) must be (0, 0), i.e. the same super-tile field in all keys
         * (OR == AND there) and that field the encoding of (0, 0) */
        const int f0 = 2 * Z + 32;
        const unsigned __int128 fm = (((unsigned __int128)1 << (5 + HM_GEN_SC_BITS)) - 1) << f0;
        const unsigned __int128 orv = (((unsigned __int128)down[1]) << 64) | down[0];
        const unsigned __int128 zero = ((unsigned __int128)((uint64_t)HM_GEN_SR_BIAS << HM_GEN_SC_BITS |
                                                           (uint64_t)HM_GEN_SC_BIAS)) << f0;
        if ((var & fm) != 0 || (orv & fm) != zero) return HM_E_EXOTIC;
    }
    int shs[16], np = 0;
    for (int sh = 0; sh < 128; sh += 8)
        if ((uint64_t)((var >> sh) & 0xFF)) shs[np++] = sh;
    uint8_t* rxs;
    ENSURE(B_GEN_HIST, 256 + 16 * 2048 + hm_rx_os_tiles(n) * 2048, rxs);
    const int cur = hm_launch_rx_sort(s, wide, klo, khi, n, shs, np, rxs);
    HIPCHK(hipGetLastError());
    /* zoom cascade (k_cascade): step k makes the zoom-(Z-k) cells and writes
     * the records of zoom Z-k+1; a last launch writes the zmin records.  Item
     * counts and record offsets stay on the device (one read-back at the end) */
    const int K = Z - zmin + 1;
    const uint64_t ntc = hm_cascade_tiles(n);
    uint8_t* cs;
    uint32_t *e0, *e1;
    ENSURE(B_GEN_FLAG, 512 + 2 * ntc * 8, cs);
    ENSURE(B_GEN_IDX, n * 4, e0);
    ENSURE(B_GEN_C, n * 4, e1);
    unsigned* tick = (unsigned*)cs;
    uint32_t* mdev = (uint32_t*)(cs + 128);
    unsigned long long* rbase = (unsigned long long*)(cs + 256);
    static_assert(HM_MAX_ZOOM + 3 <= 32, "cascade state slots");
    HIPCHK(hipMemsetAsync(cs, 0, 512 + 2 * ntc * 8, s));
    HmCascArgs ca;
    memset(&ca, 0, sizeof(ca));
    ca.tstat = (uint64_t*)(cs + 512);
    ca.tstat2 = ca.tstat + ntc;
    ca.e = e;
    ca.hic = down[1];
    /* packed records: two zoom steps per launch where two levels of records
     * are left before the last (k_cascade2) */
    const bool fuse = HM_CS_FUSE && e.width == 2 && !e.split;
    int in = cur;                       /* key buffer of the launch's input */
    uint32_t* ecur = nullptr;           /* ENDs of the input cells (none: raw keys) */
    uint32_t* eb[2] = {e0, e1};
    int eo = 0;
    int slot = 0;                       /* launch index: its count, record base, ticket and epoch */
    for (int kz = 0;;) {                /* the input level is zoom Z - kz + 1 (kz >= 1), raw keys at kz = 0 */
        const bool last = kz == K;
        const bool two = fuse && kz >= 1 && kz + 2 <= K;
        ca.kin_lo = klo[in];
        ca.kin_hi = khi[in];
        ca.ein = ecur;
        ca.m_in = slot ? mdev + (slot - 1) : nullptr;
        ca.m_host = n;
        ca.clr = 2 * (two ? kz + 1 : kz);
        ca.Z = Z;
        ca.zin = Z - kz + 1;
        ca.emit = kz > 0;
        ca.kout_lo = klo[1 - in];
        ca.kout_hi = khi[1 - in];
        ca.eout = eb[eo];
        ca.m_out = mdev + slot;
        ca.epoch = (uint64_t)slot + 1;
        ca.ticket = tick + slot;
        ca.rbase_in = slot ? rbase + slot : nullptr;
        ca.rbase_out = slot ? rbase + slot + 1 : nullptr;
        hm_launch_cascade(s, ca, n, last ? 1 : (two ? 2 : 0), wide);
        HIPCHK(hipGetLastError());
        slot++;
        if (last) break;
        in = 1 - in;
        ecur = eb[eo];
        eo ^= 1;
        kz += two ? 2 : 1;
    }
    HIPCHK(hipMemcpyAsync(down, rbase + slot, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hm_sync(s));
    *total = down[0];
    return HM_OK;
}

#define HM_FALLBACK (-1)   /* count_impl: the pipeline's dense child space is too large */

/* hm_count for data too sparse for the pipeline's dense per-level child
 * arrays (e.g. uniform clouds at zoom 21): every kept point through the
 * general path, cells inside the square emitted as HM_KEYs */
static int count_fallback(hm_ctx* ctx, const double* lat, const double* lon, const int64_t* rows,
                          const int64_t* cols, const uint8_t* keep, int64_t n, int zmin, int zmax, uint64_t* keys_out,
                          uint64_t* counts_out, int64_t capacity, int64_t* n_out, int64_t* xcells_out,
                          int64_t xcapacity, int64_t* nx_out)
{
    int st = reset_state(ctx);
    if (st) return st;
    int64_t *row = nullptr, *col = nullptr, *idx = nullptr;
    if (rows) {
        uint32_t* grp;
        ENSURE(B_X_ROW, (uint64_t)n * 8 + 8, row);
        ENSURE(B_X_COL, (uint64_t)n * 8 + 8, col);
        ENSURE(B_X_IDX, (uint64_t)n * 8 + 8, idx);
        ENSURE(B_GL_GRP, (uint64_t)n * 4 + 4, grp);
        hm_launch_tiles_list(ctx->stream, rows, cols, keep, nullptr, n, row, col, grp, idx, ctx->state + ST_XCOUNT);
        HIPCHK(hipGetLastError());
        if ((st = read_state(ctx))) return st;
        if ((st = take_error(ctx))) return st;
    }
    HmGenEmit e;
    memset(&e, 0, sizeof(e));
    e.cells = xcells_out;
    e.capacity = (uint64_t)xcapacity;
    e.width = 4;
    e.split = 1;
    e.keys = keys_out;
    e.counts = counts_out;
    e.kcapacity = (uint64_t)capacity;
    e.kcursor = ctx->state + ST_CURSOR;
    e.xcursor = ctx->state + ST_XCURSOR;
    uint64_t total = 0;
    if (rows)
        st = gen_count(ctx, row, col, nullptr, idx, ctx->host_state[ST_XCOUNT], zmax, zmin, e, &total);
    else   /* points projected straight into keys */
        st = gen_count(ctx, nullptr, nullptr, nullptr, nullptr, (uint64_t)n, zmax, zmin, e, &total, lat, lon, keep);
    if (st) return st;
    if ((st = read_state(ctx))) return st;
    *n_out = (int64_t)ctx->host_state[ST_CURSOR];
    *nx_out = (int64_t)ctx->host_state[ST_XCURSOR];
    ctx->last_slow = 0;
    ctx->last_levels = 0;
    for (int i = 0; i < 8; i++) ctx->stage_us[i] = 0;
    return (*n_out > capacity || *nx_out > xcapacity) ? HM_E_CAPACITY : HM_OK;
}

/* Level plan for dense, evenly spread clouds (uniform-like). With 6 zooms
 * per level, each level-2 work item (HM_TN keys) of such a cloud scatters
 * over ~3400 of its 4^6 digits: runs of one or two keys, each a run-slot
 * atomic, a run record and a scan entry (1e9 uniform points: 24 ms of
 * level-2 partitioning). Levels of 3 zooms (64 digits) keep the runs long
 * at the price of one more pass over the keys (1e9 uniform points: 68 -> 48
 * ms per count; the same plan costs hotspot clouds 60%, so it is chosen only
 * when level 1's sampled histogram is flat -- no digit above 4x the mean --
 * and the mean level-1 bucket holds >= HM_SPREAD_MIN_KEYS keys; the
 * environment variable of that name overrides the threshold). */
static void spread_replan(const uint32_t* h, int F, double npts, int zb, int* zs, int* L, double min_keys,
                          bool flat)
{
    uint64_t tot = 0, mx = 0;
    int ne = 0;
    for (int i = 0; i < F; i++) {
        tot += h[i];
        mx = std::max<uint64_t>(mx, h[i]);
        ne += h[i] != 0;
    }
    if (ne == 0 || npts < min_keys * ne || (flat && (double)mx * ne > 4.0 * (double)tot)) return;
    int step = HM_SPREAD_ZOOMS;
    while (zs[0] + step * (HM_MAX_LEVELS - 1) < zb) step++;
    if (step >= HM_LEVEL_ZOOMS) return;
    int l = 1, z = zs[0];
    while (z < zb) {
        z = std::min(z + step, zb);
        zs[l++] = z;
    }
    *L = l;
}

static int count_impl(hm_ctx* ctx, const double* lat, const double* lon, const int64_t* rows, const int64_t* cols,
                      const uint8_t* keep, int64_t n, int zmin, int zmax, uint64_t* keys_out, uint64_t* counts_out,
                      int64_t capacity, int64_t* n_out, int64_t* xcells_out, int64_t xcapacity, int64_t* nx_out)
{
    if (!ctx || !n_out || !nx_out || n < 0 || n >= (int64_t)0xFFFFFFF0ll || zmin < 0 || zmax < zmin ||
        zmax > HM_COUNT_MAX_ZOOM || capacity < 0 || (capacity > 0 && (!keys_out || !counts_out)) || xcapacity < 0 ||
        (xcapacity > 0 && !xcells_out))
        return HM_E_ARG;
    *n_out = 0;
    *nx_out = 0;
    /* set again only when THIS attempt re-keys a stream's tail (an attempt
     * that fails after it, then count_fallback, leaves the keys un-keyed) */
    ctx->tail_done = 0;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int Z = zmax;
    const int zb = Z > HM_AG_LG ? Z - HM_AG_LG : 0;
    int zs[HM_MAX_LEVELS];
    int L = 0;
    {
        int z = zb < HM_Z1 ? zb : HM_Z1;
        zs[L++] = z;
        while (z < zb) {
            z = std::min(z + HM_LEVEL_ZOOMS, zb);
            if (L >= HM_MAX_LEVELS) return HM_E_ARG;
            zs[L++] = z;
        }
    }
    /* key bits after level l: 2*(Z - zs[l]); must fit u32 (level 1 output) */
    if (2 * (Z - zs[0]) > 32) return HM_E_ARG;
    int st = HM_OK;
    /* the call's state words and level 1's zeroed buffers: one fill dispatch,
     * launched before level 1's sampling */
    HmFill f1;
    memset(&f1, 0, sizeof(f1));
    hm_fill_add(f1, ctx->state + 1, 0, (ST_COUNT - 1) * sizeof(unsigned long long));
    hm_fill_add(f1, ctx->state + ST_ERR, 0xFF, sizeof(unsigned long long));
    static_assert(ST_ERR == 0, "error word first");

    hipEvent_t* ev = ctx->ev;
    int nev = 0;
    /* stage timings (hm_last_stats) for calls of >= 2^24 points: each event
     * record is an API call, and small calls (stream batches) are bound by
     * the host's issue rate */
    const bool timing = n >= (1ll << 24) && ctx->stage_timing;
    /* keys per aggregation work item: HM_TA, halved (down to 16K) until the
     * call has >= 512 items' worth of points -- a 1e7-point call otherwise
     * runs ~40 items on 256 CUs */
    uint32_t ta = HM_TA;
    while (ta > ctx->ta_min && (uint64_t)n < (uint64_t)ta * ctx->ta_items) ta >>= 1;
    for (int i = 0; i < 8; i++) ctx->stage_us[i] = 0;
    ctx->last_levels = L;

    /* level 1 reads the input in HM_T1-point tiles; points the fast path
     * defers (lat/lon input only) go to k_redo, at most redo_cap of them */
    const uint32_t tiles_in = (uint32_t)((n + HM_T1 - 1) / HM_T1);
    const bool from_tiles = rows != nullptr;
    uint64_t redo_cap = from_tiles ? 0 : std::max<uint64_t>(1u << 20, (uint64_t)n / 256);
    if (redo_cap > (uint64_t)n) redo_cap = (uint64_t)n;
    /* exotic list: first capacity like the redo list's; rebuilt if it overflows */
    HmExotic xl;
    xl.cap = std::min<uint64_t>((uint64_t)n, std::max<uint64_t>(1u << 20, (uint64_t)n / 256));
    ENSURE(B_X_ROW, xl.cap * 8 + 8, xl.row);
    ENSURE(B_X_COL, xl.cap * 8 + 8, xl.col);
    ENSURE(B_X_IDX, xl.cap * 8 + 8, xl.idx);
    xl.count = ctx->state + ST_XCOUNT;
    const uint32_t* parent_item_begin = nullptr;
    const uint64_t* parent_coord = nullptr;
    uint32_t nparents = 1;

    Level lv[HM_MAX_LEVELS];
    HmBuckets B[HM_MAX_LEVELS];
    memset(B, 0, sizeof(B));
    void* keys_cur = nullptr;
    HmRuns runs_cur = {nullptr, nullptr};
    int slot_k = 0; /* ping-pong A/B */
    uint32_t nslots = 0;
    int32_t* slots = nullptr;
    uint32_t* slot_bucket = nullptr;
    uint64_t level_keys = 0;    /* keys entering level l >= 2 (global positions) */
    uint64_t nx = 0;            /* kept points outside [0, 2^Z)^2 */
    int npart = 0;              /* level >= 2 partition launches timed (ev[5..]) */

    uint32_t* seg1 = nullptr;   /* level-1 items' run tables (k_partition_fr) */
    uint32_t* seg2 = nullptr;   /* level-2 items' run tables after a child-contiguous level */
    bool hot_on = false;        /* hot tiles sampled and looked up by level 1 */
    bool hot_mid = false;       /* ... at zs[1] of a 3-level plan (they skip level 2 only) */
    int hz = zb;                /* zoom of the hot tiles: the bucket zoom of level 2 */
    bool spread = false;        /* levels 2.. take fewer zooms (spread_replan) */
    uint32_t nhot = 0;          /* hot tiles found */
    uint64_t l2_elems = 0;      /* mid-level hot tiles: level 2's key array (elements) */
    int l1_reruns = 0;          /* level-1 re-runs after a region overflow */
    HmHotRunArgs hr;            /* hot tiles as level-2 children */
    memset(&hr, 0, sizeof(hr));
    for (int l = 0; l < L; l++) {
        Level& V = lv[l];
        V.zc = zs[l];
        V.dbits = 2 * (zs[l] - (l ? zs[l - 1] : 0));
        V.nparents = nparents;
        V.nchildren = (uint64_t)nparents << V.dbits;
        V.out16 = (l == L - 1);
        const int restbits = 2 * (Z - zs[l]);
        if (V.nchildren > (uint64_t)HM_SCAN_LIMIT) return HM_FALLBACK;
        if (l == 0) {
            /* ---- level 1: projection + partition into per-digit regions ---- */
            const int F = 1 << V.dbits;
            /* digit slots: F cold digits, hot tile h at HM_MAX_F1 + h */
            const int FS = HM_D1 * HM_L1_SHARDS;
            uint32_t *fill, *rbase, *rcap, *hist;
            uint8_t* smask;
            ENSURE(B_L1_FILL, FS * 4, fill);
            ENSURE(B_L1_RBASE, FS * 4, rbase);
            ENSURE(B_L1_RCAP, FS * 4, rcap);
            ENSURE(B_L1_HIST, HM_D1 * 4, hist);
            ENSURE(B_L1_SMASK, HM_D1, smask);
            /* hot tiles are level-2 buckets: zoom zs[1], a dense sample
             * histogram of <= 4^11 tiles.  In the two-level plan (level 1 at
             * z1, the last at zb) they skip every partition after level 1; in
             * a three-level plan (zmax 19-21: z5 -> z11 -> zb) they skip level 2
             * and join level 3 with the level-2 buckets (HM_HOT_MID) */
            hot_mid = ctx->hot && ctx->hot_mid && L == 3 && zs[1] <= 11 && zs[0] == HM_Z1 && n > 0 &&
                      V.dbits == 2 * HM_Z1;
            hot_on = hot_mid || (ctx->hot && L == 2 && zb <= 11 && zs[0] == HM_Z1 && n > 0 && V.dbits == 2 * HM_Z1);
            hz = hot_mid ? zs[1] : zb;
            uint32_t* redo_idx = nullptr;
            int64_t *redo_rows = nullptr, *redo_cols = nullptr;
            if (!from_tiles) {
                ENSURE(B_REDO_IDX, redo_cap * sizeof(uint32_t), redo_idx);
                ENSURE(B_REDO_ROWS, redo_cap * sizeof(int64_t), redo_rows);
                ENSURE(B_REDO_COLS, redo_cap * sizeof(int64_t), redo_cols);
            }
            HmPart1Args a;
            memset(&a, 0, sizeof(a));
            a.lat = lat;
            a.lon = lon;
            a.rows_in = rows;
            a.cols_in = cols;
            a.keep = keep;
            a.n = n;
            a.Z = Z;
            a.dbits = V.dbits;
            a.restbits = restbits;
            a.fill = fill;
            a.rbase = rbase;
            a.rcap = rcap;
            a.smask = smask;
            a.overflow = ctx->state + ST_OVERFLOW;
            a.err_word = ctx->state + ST_ERR;
            a.x = xl;
            a.slow_count = ctx->state + ST_SLOW;
            a.redo_idx = redo_idx;
            a.redo_count = ctx->state + ST_REDO;
            a.redo_cap = redo_cap;
            /* region sizes: a sampled digit histogram with a generous margin */
            /* ~256K samples (1M samples above 2^28 points took 90 us per 1e9-point
             * count; the regions' 8-sigma margins scale with sqrt(stride)) */
            /* (2^16 samples below 2^24 points, where the sample pass's ~30 us
             * is a batch's cost; the regions' slack scales with the stride) */
            const int slog = n < (1ll << 24) ? std::min(ctx->sample_log2, 16) : ctx->sample_log2;
            const uint64_t stride = std::max<uint64_t>(1, (uint64_t)n >> slog);
            hm_fill_add(f1, hist, 0, HM_D1 * 4);
            hm_fill_add(f1, fill, 0, FS * 4);
            uint32_t* hot_counts = nullptr;
            uint32_t* hot_tiles = nullptr;
            uint32_t* hot_hash = nullptr;
            uint8_t* hot_parent = nullptr;
            uint32_t* hot_n = (uint32_t*)(ctx->state + ST_NHOT);
            if (hot_on) {
                ENSURE(B_HOT_COUNTS, (4ull << (2 * hz)), hot_counts);
                ENSURE(B_HOT, (HM_MAX_HOT + HM_HOT_SLOTS + 2 * HM_HOT_CAND + 1) * 4, hot_tiles);
                ENSURE(B_HOT_PARENT, HM_MAX_F1, hot_parent);
                hot_hash = hot_tiles + HM_MAX_HOT;
                hm_fill_add(f1, hot_counts, 0, 4ull << (2 * hz));
                hm_fill_add(f1, hot_hash + HM_HOT_SLOTS + 2 * HM_HOT_CAND, 0, 4);   /* candidates */
                hm_fill_add(f1, hot_parent, 0, HM_MAX_F1);
                a.hot_z = hz;
                a.hot_bytes = hot_mid ? 4 : 2;
                a.hot_hash = hot_hash;
                a.hot_n = hot_n;
            } else {
                a.hot_z = -1;
            }
            hm_launch_fill(s, f1);
            f1.k = 0;
            if (n > 0) hm_launch_sample_digits(s, a, stride, hist, hot_counts);
            HIPCHK(hipGetLastError());
            if (hot_on) {
                hr.tiles = hot_tiles;
                hr.n = hot_n;
                hr.zb = hz;
                hr.z1 = zs[0];
                hr.fill = fill;
                hr.rbase = rbase;
                HmHotArgs ha;
                ha.counts = hot_counts;
                ha.zb = hz;
                ha.z1 = zs[0];
                const uint64_t m = ((uint64_t)n + stride - 1) / stride;
                ha.thresh = (uint32_t)std::max<double>(
                    {1.0, ceil((double)m / ctx->hot_inv_share), ceil(ctx->hot_min_keys / (double)stride)});
                ha.tiles = hot_tiles;
                ha.hist = hist;
                ha.hotparent = hot_parent;
                ha.n = hot_n;
                ha.hash = hot_hash;
                ha.cand = hot_hash + HM_HOT_SLOTS;
                hm_launch_hot_select(s, ha);
                HIPCHK(hipGetLastError());
            }
            /* pinned host scratch (the overflow retry): caps [FS] | bases [FS] */
            uint32_t* hc = ctx->host_aux + HM_D1;
            uint32_t* hb = hc + HM_D1 * HM_L1_SHARDS;
            /* the region sizes are computed on the device (k_l1_sizes); the key
             * buffer takes the host's bound of their total: est sums to at
             * most nn (a hot tile's samples leave its cold digit), at most M
             * (digit, shard) entries are non-empty, and sum sqrt(e stride) <=
             * sqrt(M nn stride) (Cauchy-Schwarz) */
            const double nn = (double)n + (double)(F + (hot_on ? HM_MAX_HOT : 0)) * (double)stride;
            const double M = F + std::min((double)F, nn / ((double)HM_L1_SHARD_TILES * HM_T1)) * (HM_L1_SHARDS - 1) +
                             (hot_on ? (double)HM_MAX_HOT * HM_L1_SHARDS : 0.0);
            double bound = nn * 17.0 / 16.0 + 8.0 * sqrt(M * nn * (double)stride) + M * 2.0 * HM_T1 +
                           (double)(F + (hot_on ? HM_MAX_HOT : 0)) * HM_L1_ZERO_SAMPLES * (double)stride + 1024.0;
            hm_launch_l1_sizes(s, hist, F, hot_on ? hot_n : nullptr, stride, rcap, rbase, smask,
                               ctx->state + ST_L1TOTAL);
            HIPCHK(hipGetLastError());
            if (bound >= (double)0xFFF00000ull) {
                /* the bound passes the u32 key positions (n above ~1.5e9):
                 * read the exact total of the sized regions instead */
                if ((st = read_state(ctx))) return st;
                bound = (double)ctx->host_state[ST_L1TOTAL] + 1024.0;
                if (bound >= (double)0xFFF00000ull) return HM_FALLBACK;   /* key positions are u32 */
            }
            /* the non-empty digits are the level's buckets, one run each */
            HmL1Args ba;
            memset(&ba, 0, sizeof(ba));
            const uint64_t cap = (uint64_t)F + 1;
            ENSURE(B_BK0 + 0, cap * 4, ba.out.nkeys);
            ENSURE(B_BK0 + 1, cap * 4, ba.out.nruns);
            ENSURE(B_BK0 + 2, cap * 4, ba.out.rbase);
            ENSURE(B_BK0 + 3, cap * 4, ba.out.item_begin);
            ENSURE(B_BK0 + 4, cap * 4, ba.out.digit);
            ENSURE(B_BK0 + 5, cap * 8, ba.out.coord);
            ENSURE(B_BK0 + 6, cap * 4, ba.out.keybase);
            ENSURE(B_FLAT_A, (uint64_t)FS * sizeof(uint2) + 8, ba.runs);
            ENSURE(B_EXCL_A, (uint64_t)FS * sizeof(uint64_t) + 8, ba.excl);
            ENSURE(B_CHILD0, 2 * 4, ba.child_begin);
            uint64_t* tot = (uint64_t*)(ctx->state + ST_LTOT);   /* comes back with the state */
            ba.F = F;
            ba.dbits = V.dbits;
            ba.fill = fill;
            ba.rbase = rbase;
            ba.smask = smask;
            ba.item_keys = (L == 1) ? ta : HM_TN;
            ba.sparse_max = (L == 1) ? HM_SP_MAX : 0u;
            ba.total = tot;
            if (hot_on) {   /* hot parents all zero when no tile turned out hot */
                uint32_t* d2b;
                ENSURE(B_D2B, HM_MAX_F1 * 4, d2b);
                ba.hotparent = hr.tiles ? (const uint8_t*)ctx->bufs[B_HOT_PARENT].p : nullptr;
                ba.d2b = d2b;
                hr.d2b = d2b;
            }
            if (L == 1) {
                ENSURE(B_SLOTS, cap * 4, slots);
                ENSURE(B_SLOTBKT, cap * 4, slot_bucket);
                ba.slots = slots;
                ba.nslots = ctx->state + ST_NSLOTS;
                ba.slot_bucket = slot_bucket;
            }
            unsigned long long* down = ctx->host_state + 2 * ST_COUNT;
            void* kout = nullptr;
            uint64_t total_cap = (uint64_t)bound;
            for (int attempt = 0;; attempt++) {
                if (attempt > 0) {
                    /* a digit's shards stay consecutive: its keys' logical
                     * positions are one range (k_level1_buckets) */
                    total_cap = 0;
                    for (int d = 0; d < HM_D1; d++)
                        for (int sh = 0; sh < HM_L1_SHARDS; sh++) {
                            hb[hm_l1i(d, sh)] = (uint32_t)total_cap;
                            total_cap += hc[hm_l1i(d, sh)];
                        }
                    if (total_cap >= 0xFFF00000ull) return HM_FALLBACK;
                    HIPCHK(hipMemcpyAsync(rcap, hc, FS * 4, hipMemcpyHostToDevice, s));
                    HIPCHK(hipMemcpyAsync(rbase, hb, FS * 4, hipMemcpyHostToDevice, s));
                }
                ENSURE(slot_k ? B_KEYS_B : B_KEYS_A, (total_cap + 8) * (V.out16 ? 2 : 4), kout);
                a.keys_out = kout;
                if (hot_on) {
                    /* hot keys: straight into level 2's output key array (level 2
                     * writes the cold keys' positions of it): u16 when that is the
                     * last level's, u32 for mid-level hot tiles -- whose array
                     * also holds the child-contiguous cold keys above every
                     * level-1 position (l2_elems) */
                    void* kh = nullptr;
                    if (hot_mid) l2_elems = total_cap + (uint64_t)n + 16;
                    ENSURE(slot_k ? B_KEYS_A : B_KEYS_B, hot_mid ? l2_elems * 4 : (total_cap + 8) * 2, kh);
                    a.keys_hot = kh;
                }
                if (attempt > 0) {
                    /* (the first attempt's are zero from the call's fill) */
                    HIPCHK(hipMemsetAsync(fill, 0, FS * 4, s));
                    /* ST_XCOUNT .. ST_OVERFLOW (XCOUNT, SLOW, REDO, REDO_OUT, OVERFLOW;
                     * CURSOR, NSLOTS, XCURSOR are still 0 here) in one memset */
                    static_assert(ST_XCOUNT == 1 && ST_OVERFLOW == 8 && ST_NHOT > ST_OVERFLOW, "level-1 words");
                    HIPCHK(hipMemsetAsync(ctx->state + ST_XCOUNT, 0, 8 * 8, s));
                }
                if (timing) HIPCHK(hipEventRecord(ev[0], s));
                hm_launch_part1(s, a, tiles_in, V.out16, from_tiles ? 1 : 0);
                HIPCHK(hipGetLastError());
                if (timing) HIPCHK(hipEventRecord(ev[1], s));
                nev = 2;
                if (!from_tiles) {
                    HmRedoArgs ra;
                    ra.lat = lat;
                    ra.lon = lon;
                    ra.keep = keep;
                    ra.Z = Z;
                    ra.redo_idx = redo_idx;
                    ra.redo_count = ctx->state + ST_REDO;
                    ra.rows_out = redo_rows;
                    ra.cols_out = redo_cols;
                    ra.out_count = ctx->state + ST_REDO_OUT;
                    ra.err_word = ctx->state + ST_ERR;
                    ra.x = xl;
                    ra.cap = redo_cap;
                    hm_launch_redo(s, ra, redo_cap);
                    HIPCHK(hipGetLastError());
                }
                if (!from_tiles) {
                    /* the deferred points, resolved exactly, as tile input; the
                     * launch covers the list's capacity and reads its length
                     * on the device (no host round trip) */
                    HmPart1Args b = a;
                    b.lat = nullptr;
                    b.lon = nullptr;
                    b.rows_in = redo_rows;
                    b.cols_in = redo_cols;
                    b.keep = nullptr;
                    b.n = (int64_t)redo_cap;
                    b.n_dev = ctx->state + ST_REDO_OUT;
                    hm_launch_part1(s, b, (uint32_t)((redo_cap + HM_T1 - 1) / HM_T1), V.out16, 1);
                    HIPCHK(hipGetLastError());
                }
                /* the level's buckets from the filled regions, launched before
                 * the one host sync of level 1 (its results are used only if
                 * the level turns out clean: no error, no redo or region
                 * overflow) */
                auto buckets1 = [&]() -> int {
                    hm_launch_level1_buckets(s, ba);
                    HIPCHK(hipGetLastError());
                    if (L > 1) HIPCHK(hipMemcpyAsync(ctx->host_aux, hist, F * 4, hipMemcpyDeviceToHost, s));
                    return read_state(ctx);
                };
                if ((st = buckets1())) return st;
                if ((st = take_error(ctx))) return st;
                const uint64_t nredo = ctx->host_state[ST_REDO];
                ctx->last_slow = (int64_t)nredo;
                if (!from_tiles && nredo > redo_cap) {
                    /* adversarial input (mostly polar / guard band): redo the
                     * level with the exact chain fused into the kernel */
                    HIPCHK(hipMemsetAsync(fill, 0, FS * 4, s));
                    HIPCHK(hipMemsetAsync(ctx->state + ST_OVERFLOW, 0, 8, s));
                    HIPCHK(hipMemsetAsync(xl.count, 0, 8, s));
                    HIPCHK(hipMemsetAsync(ctx->state + ST_NSLOTS, 0, 8, s));   /* buckets1 again */
                    hm_launch_part1(s, a, tiles_in, V.out16, 2);
                    HIPCHK(hipGetLastError());
                    if ((st = buckets1())) return st;
                    if ((st = take_error(ctx))) return st;
                }
                if (!ctx->host_state[ST_OVERFLOW]) break;
                /* a region overflowed: fill[] now holds the exact sizes (the
                 * shard of every tile is fixed by its block id) */
                if (attempt > 0) return HM_E_HIP;   /* cannot happen: the same points */
                l1_reruns++;
                HIPCHK(hipMemcpyAsync(hc, fill, FS * 4, hipMemcpyDeviceToHost, s));
                if (ctx->debug_l1) HIPCHK(hipMemcpyAsync(hb, rcap, FS * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hm_sync(s));
                if (ctx->debug_l1) {
                    /* HM_DEBUG_L1=1: the overflowing regions, and the sample behind them */
                    for (int i = 0; i < FS; i++)
                        if (hc[i] > hb[i])
                            fprintf(stderr, "hm l1 overflow: digit %d shard %d fill %u cap %u hist %u stride %llu\n",
                                    i % HM_D1, i / HM_D1, hc[i], hb[i], ctx->host_aux[i % HM_D1],
                                    (unsigned long long)stride);
                }
                for (int i = 0; i < FS; i++) hc[i] += 64;
            }
            nx = ctx->host_state[ST_XCOUNT];
            if (nx > xl.cap) {
                /* more kept out-of-square points than the list held: rebuild it */
                xl.cap = nx;
                ENSURE(B_X_ROW, xl.cap * 8, xl.row);
                ENSURE(B_X_COL, xl.cap * 8, xl.col);
                ENSURE(B_X_IDX, xl.cap * 8, xl.idx);
                HIPCHK(hipMemsetAsync(xl.count, 0, sizeof(unsigned long long), s));
                hm_launch_collect_exotic(s, lat, lon, rows, cols, keep, n, Z, xl);
                HIPCHK(hipGetLastError());
                if ((st = read_state(ctx))) return st;
                nx = ctx->host_state[ST_XCOUNT];
                if (nx > xl.cap) return HM_E_HIP;   /* cannot happen: the same points */
            }
            nhot = hot_on ? (uint32_t)(ctx->host_state[ST_NHOT] & 0xFFFFFFFFull) : 0u;
            if (!nhot) hot_mid = false;
            /* levels 2.. may take the spread plan (the level-1 pass is the
             * same under both: its output is u32 keys whenever L > 1) */
            if (hot_mid) {
                /* the plan stays z5 -> z11 -> zb: the hot tiles are zoom-11 buckets */
            } else if (L > 1 && !nhot) {
                spread_replan(ctx->host_aux, F, (double)n, zb, zs, &L, ctx->spread_min_keys, true);
            } else if (L > 1) {
                /* with hot tiles the rest is the cloud's sparse background: 3
                 * zooms per level unless it is tiny (a 6-zoom level scatters
                 * each 8192-key item over 4096 children, runs of ~1 key); the
                 * hot tiles then join at the last level.  (host_aux holds the
                 * cold digits' sampled counts: the hot samples were taken off) */
                double cold = 0;
                for (int i = 0; i < F; i++) cold += ctx->host_aux[i];
                spread_replan(ctx->host_aux, F, cold * (double)stride, zb, zs, &L, ctx->spread_min_cold, false);
            }
            spread = L > 2 && zs[1] - zs[0] < HM_LEVEL_ZOOMS;
            ctx->last_levels = L;
            V.count = (uint32_t)(ctx->host_state[ST_LTOT] >> 32);
            V.items = (uint32_t)(ctx->host_state[ST_LTOT] & 0xFFFFFFFFull);
            if (L == 1) nslots = (uint32_t)(ctx->host_state[ST_NSLOTS] & 0xFFFFFFFFull);
            level_keys = total_cap;
            HmBuckets& b = B[0];
            b.count = V.count;
            b.nkeys = ba.out.nkeys;
            b.nruns = ba.out.nruns;
            b.rbase = ba.out.rbase;
            b.keybase = ba.out.keybase;
            b.item_begin = ba.out.item_begin;
            b.digit = ba.out.digit;
            b.coord = ba.out.coord;
            b.slots = (L == 1) ? slots : nullptr;
            runs_cur.run = ba.runs;
            runs_cur.excl = ba.excl;
            {
                uint4* desc;
                ENSURE(B_DESC0 + 0, ((uint64_t)V.items + 1) * 2 * sizeof(uint4), desc);
                b.desc = desc;
                if (L > 1) ENSURE(B_SEG, ((uint64_t)V.items + 1) * 16 * sizeof(uint32_t), seg1);
                hm_launch_items(s, b, runs_cur, V.items, (L == 1) ? ta : HM_TN, desc, L > 1 ? seg1 : nullptr);
                HIPCHK(hipGetLastError());
            }
            keys_cur = kout;
            parent_item_begin = ba.out.item_begin;
            parent_coord = ba.out.coord;
            nparents = V.count;
            slot_k ^= 1;
            continue;
        }
        /* ---- levels >= 2 ---- */
        const uint64_t ntiles = lv[l - 1].items;
        /* run-counter shards: up to 32 (a hot child takes one returning atomic
         * per parent work item; one counter per child made k_partition 16%
         * slower), fewer when the dense child space is large; <= 2^25 */
        /* with hot tiles (their children skip this level) or the spread plan,
         * no child is hot: one counter per child, and the partition kernels'
         * run-slot atomics coalesce (lanes own consecutive digits) */
        /* a child-contiguous level (HM_PN_CONTIG): the middle level of a
         * 3-level plan without hot tiles (Z >= 19) writes each child's keys
         * as ONE run, so the last level reads every item from <= 8 runs
         * (k_partition_fr) instead of streaming runs of a few keys each */
        /* (with mid-level hot tiles the cold keys go above every level-1
         * position, where the hot tiles' keys are: cbase_off) */
        /* level 1's positions end at its regions' total capacity (k_l1_sizes),
         * or, after an overflow re-run, at the exact sizes' total (level_keys) */
        const uint64_t l1_total = l1_reruns ? level_keys : ctx->host_state[ST_L1TOTAL];
        const bool contig = ctx->contig && l == 1 && L == 3 && (!nhot || hot_mid) && !V.out16 && seg1 != nullptr &&
                            (!hot_mid || l1_total + (uint64_t)n < 0xFFF00000ull);
        int sb = ctx->run_shard_bits >= 0 ? ctx->run_shard_bits : ((nhot || spread) ? 0 : HM_RUN_SHARD_BITS);
        if (contig) sb = 0;
        while (sb > 0 && (V.nchildren << sb) > (1ull << 25)) sb--;
        const uint64_t run_cap = (ntiles + ((uint64_t)nparents << sb)) << V.dbits;
        if (run_cap >= (1ull << 32)) return HM_E_NOMEM;

        /* outputs of the level's partition kernel: keys at the item's global
         * positions, and sharded runs */
        void* kout;
        uint2* runs_sh;
        uint32_t* nruns;
        const uint64_t nkeys_out = level_keys;
        /* with hot tiles the last level's keys go where level 1 put the hot
         * tiles' (B); a 3-level plan's middle level then takes a third array */
        const bool hot3 = nhot && L == 3 && !hot_mid;
        const int kslot = hot3 ? (l == 1 ? B_KEYS_C : B_KEYS_B) : (slot_k ? B_KEYS_B : B_KEYS_A);
        ENSURE(kslot, std::max<uint64_t>(nkeys_out + 8, (hot_mid && l == 1) ? l2_elems : 0) * (V.out16 ? 2 : 4), kout);
        ENSURE(B_RUNS_SH, run_cap * sizeof(uint2), runs_sh);
        ENSURE(B_NRUNS, (V.nchildren << sb) * sizeof(uint32_t), nruns);
        uint32_t* rs_big;
        ENSURE(B_RS_BIG, (HM_RS_BIG_MAX + 1) * sizeof(uint32_t), rs_big);
        {
            /* the level's zeroed counters in one launch */
            HmFill zf;
            zf.k = 0;
            hm_fill_add(zf, nruns, 0, (V.nchildren << sb) * sizeof(uint32_t));
            hm_fill_add(zf, rs_big + HM_RS_BIG_MAX, 0, sizeof(uint32_t));   /* the run scan's big-child count */
            hm_launch_fill(s, zf);
        }

        {
            HmPartNArgs a;
            memset(&a, 0, sizeof(a));
            a.parent = B[l - 1];
            a.keys_in = (const uint32_t*)keys_cur;
            a.in = runs_cur;
            a.dbits = V.dbits;
            a.restbits = restbits;
            a.shard_bits = sb;
            a.keys_out = kout;
            a.nruns_out = nruns;
            a.runs_out = runs_sh;
            a.items = lv[l - 1].items;
            a.seg = l == 1 ? seg1 : seg2;
            if (timing) HIPCHK(hipEventRecord(ev[5 + 2 * (l - 1)], s));
            if (contig) {
                /* child totals, their scan, then the partition proper */
                uint64_t *ptl, *ttl;
                ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), ptl);
                ENSURE(B_TOTAL, 4 * sizeof(uint64_t), ttl);
                ENSURE(B_CTOT, V.nchildren * 8, a.ctot);
                ENSURE(B_CBASE, V.nchildren * 8, a.cbase);
                ENSURE(B_CCUR, V.nchildren * 4, a.ccur);
                HIPCHK(hipMemsetAsync(a.ctot, 0, V.nchildren * 8, s));
                HIPCHK(hipMemsetAsync(a.ccur, 0, V.nchildren * 4, s));
                a.mode = HM_PN_HIST;
                a.cbase_off = hot_mid ? (uint32_t)l1_total : 0u;
                hm_launch_partition_hist(s, a);
                hm_launch_scan(s, (const uint64_t*)a.ctot, V.nchildren, ptl, (uint64_t*)a.cbase, ttl + 3);
                a.mode = HM_PN_CONTIG;
            }
            hm_launch_partN(s, a, lv[l - 1].items, V.out16, (l == 1 && seg1 != nullptr) || (l == 2 && seg2 != nullptr));
            HIPCHK(hipGetLastError());
            if (timing) HIPCHK(hipEventRecord(ev[6 + 2 * (l - 1)], s));
            npart = l;
        }

        /* run scan: sharded counters -> flat child-ordered runs + key prefix */
        HmRsArgs ra;
        memset(&ra, 0, sizeof(ra));
        ra.nchildren = V.nchildren;
        ra.dbits = V.dbits;
        ra.shard_bits = sb;
        ra.nruns = nruns;
        ra.runs = runs_sh;
        ra.parent_item_begin = parent_item_begin;
        ra.item_keys = (l == L - 1) ? ta : HM_TN;
        ra.sparse_max = (l == L - 1) ? HM_SP_MAX : 0u;
        uint64_t *partial, *tot;
        ENSURE(B_SHOFF, (V.nchildren << sb) * sizeof(uint32_t), ra.shoff);
        ENSURE(B_NR, V.nchildren * sizeof(uint64_t), ra.nr);
        uint64_t* runbase;
        ENSURE(B_RUNBASE0 + l, V.nchildren * sizeof(uint64_t), runbase);
        ra.runbase = runbase;
        ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
        tot = (uint64_t*)(ctx->state + ST_LTOT);
        hm_launch_rs_count(s, ra);
        /* hot tiles are children of the last level: of their z5 bucket at
         * level 2, of their zs[1] ancestor (kept as a bucket, below) at level 3 */
        const bool hot_level = nhot && l == (hot_mid ? 1 : L - 1);
        if (hot_level) {
            hr.dbits = V.dbits;
            hr.nr = ra.nr;
            hr.zp = zs[l - 1];
            hr.c2b = (l == 2 && hot3) ? (const uint32_t*)ctx->bufs[B_C2B].p : nullptr;
            hm_launch_hot_nr(s, hr);
        }
        /* a 3-level plan with hot tiles: each hot tile's zs[1] ancestor must be
         * a level-2 bucket (its parent at level 3) even without cold keys */
        uint8_t* force = nullptr;
        if (hot3 && l == 1) {
            ENSURE(B_HOT_FORCE, V.nchildren, force);
            HIPCHK(hipMemsetAsync(force, 0, V.nchildren, s));
            hr.dbits = V.dbits;
            hr.zp = zs[1];
            hm_launch_hot_force(s, hr, force);
        }
        ra.force = force;
        hm_launch_scan(s, ra.nr, V.nchildren, partial, runbase, tot + 0);
        HIPCHK(hipGetLastError());
        unsigned long long* down = ctx->host_state + 2 * ST_COUNT;
        /* the flat run list is sized by a bound, its length stays on the
         * device (tot[0]): at most one run per (parent item, child) and per
         * key, plus the hot tiles' region shards */
        uint64_t nflat = std::min<uint64_t>(level_keys, (uint64_t)lv[l - 1].items << V.dbits) +
                         (uint64_t)HM_MAX_HOT * HM_L1_SHARDS + 1;
        ra.nflat_dev = tot + 0;
        if (nflat * 24 > (8ull << 30)) {
            /* a bound of more than 8 GiB of run buffers: read the count back */
            HIPCHK(hipMemcpyAsync(down, tot, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hm_sync(s));
            nflat = down[0];
            ra.nflat_dev = nullptr;
        }
        ra.nflat = nflat;
        uint2* flat;
        uint64_t* excl;
        ENSURE(slot_k ? B_FLAT_B : B_FLAT_A, (nflat + 1) * sizeof(uint2), flat);
        ENSURE(slot_k ? B_EXCL_B : B_EXCL_A, (nflat + 1) * sizeof(uint64_t), excl);
        ENSURE(B_CNT, (nflat + 1) * sizeof(uint64_t), ra.cnt);
        ra.flat = flat;
        ra.excl = excl;
        ra.big = rs_big;
        ra.nbig = ra.big + HM_RS_BIG_MAX;   /* zeroed with nruns */
        ra.big_min = ctx->rs_big_min;
        hm_launch_rs_copy(s, ra);
        if (hot_level) {
            hr.runbase = runbase;
            hr.flat = flat;
            hr.cnt = ra.cnt;
            hm_launch_hot_runs(s, hr);
        }
        hm_launch_scan(s, ra.cnt, nflat, partial, excl, tot + 1, ra.nflat_dev);
        ra.total_keys = tot + 1;
        uint32_t* cnkeys;
        uint32_t* ckeybase;
        uint64_t *vals, *prefix;
        ENSURE(B_NKEYS, V.nchildren * sizeof(uint32_t), cnkeys);
        ENSURE(B_KEYBASE, V.nchildren * sizeof(uint32_t), ckeybase);
        ENSURE(B_VALS, V.nchildren * sizeof(uint64_t), vals);
        ENSURE(B_PREFIX, V.nchildren * sizeof(uint64_t), prefix);
        ra.nkeys = cnkeys;
        ra.keybase = ckeybase;
        ra.vals = vals;
        hm_launch_rs_keys(s, ra);
        hm_launch_scan(s, vals, V.nchildren, partial, prefix, tot + 2);
        HIPCHK(hipGetLastError());

        /* B_l arrays: sized by nchildren (upper bound of |B_l|) */
        const uint64_t cap = V.nchildren + 1;
        HmCompactArgs ca;
        memset(&ca, 0, sizeof(ca));
        ENSURE(B_BK0 + l * 8 + 0, cap * 4, ca.out.nkeys);
        ENSURE(B_BK0 + l * 8 + 1, cap * 4, ca.out.nruns);
        ENSURE(B_BK0 + l * 8 + 2, cap * 4, ca.out.rbase);
        ENSURE(B_BK0 + l * 8 + 3, cap * 4, ca.out.item_begin);
        ENSURE(B_BK0 + l * 8 + 4, cap * 4, ca.out.digit);
        ENSURE(B_BK0 + l * 8 + 5, cap * 8, ca.out.coord);
        ENSURE(B_BK0 + l * 8 + 6, cap * 4, ca.out.keybase);
        uint32_t* child_begin;
        ENSURE(B_CHILD0 + l, ((uint64_t)nparents + 1) * 4, child_begin);
        ca.nchildren = V.nchildren;
        ca.nparents = nparents;
        ca.dbits = V.dbits;
        ca.vals = vals;
        ca.prefix = prefix;
        ca.total = tot + 2;
        ca.nkeys = cnkeys;
        ca.nr = ra.nr;
        ca.runbase = runbase;
        ca.keybase = ckeybase;
        ca.parent_coord = parent_coord;
        ca.child_begin = child_begin;
        if (hot3 && l == 1) ENSURE(B_C2B, V.nchildren * 4, ca.c2b);   /* child -> bucket, for level 3 */
        if (l == L - 1) {
            ENSURE(B_SLOTS, cap * 4, slots);
            ENSURE(B_SLOTBKT, cap * 4, slot_bucket);
            ca.slots = slots;
            ca.nslots = ctx->state + ST_NSLOTS;
            ca.slot_bucket = slot_bucket;
        }
        hm_launch_compact(s, ca);
        HIPCHK(hipGetLastError());
        if ((st = read_state(ctx))) return st;   /* the level's totals come with it (ST_LTOT) */
        level_keys = ctx->host_state[ST_LTOT + 1];
        const uint64_t tot_h = ctx->host_state[ST_LTOT + 2];
        V.count = (uint32_t)(tot_h >> 32);
        V.items = (uint32_t)(tot_h & 0xFFFFFFFFull);
        if (l == L - 1) nslots = (uint32_t)(ctx->host_state[ST_NSLOTS] & 0xFFFFFFFFull);

        HmBuckets& b = B[l];
        b.count = V.count;
        b.nkeys = ca.out.nkeys;
        b.nruns = ca.out.nruns;
        b.rbase = ca.out.rbase;
        b.keybase = ca.out.keybase;
        b.item_begin = ca.out.item_begin;
        b.digit = ca.out.digit;
        b.coord = ca.out.coord;
        b.slots = (l == L - 1) ? slots : nullptr;
        runs_cur.run = flat;
        runs_cur.excl = excl;
        {
            uint4* desc;
            ENSURE(B_DESC0 + l, ((uint64_t)V.items + 1) * 2 * sizeof(uint4), desc);
            b.desc = desc;
            /* after a child-contiguous level every item of the next spans one run */
            seg2 = nullptr;
            if (contig) ENSURE(B_SEG2, ((uint64_t)V.items + 1) * 16 * sizeof(uint32_t), seg2);
            hm_launch_items(s, b, runs_cur, V.items, (l == L - 1) ? ta : HM_TN, desc, seg2);
            HIPCHK(hipGetLastError());
        }

        keys_cur = kout;
        parent_item_begin = ca.out.item_begin;
        parent_coord = ca.out.coord;
        nparents = V.count;
        slot_k ^= 1;
    }
    if (timing) HIPCHK(hipEventRecord(ev[nev], s));
    nev++;

    /* final aggregation over B_L */
    HmOut o;
    o.keys = keys_out;
    o.counts = counts_out;
    o.capacity = (uint64_t)capacity;
    o.cursor = ctx->state + ST_CURSOR;
    o.zmin = zmin;
    o.zmax = zmax;
    unsigned long long* totals[HM_MAX_LEVELS + 1];
    for (int l = 0; l < L; l++) ENSURE(B_TOT0 + l, ((uint64_t)lv[l].count + 1) * 8, totals[l]);
    {
        const int l = L - 1;
        uint32_t* gslots = nullptr;
        ENSURE(B_GSLOTS, (uint64_t)(nslots ? nslots : 1) * HM_AG_CELLS * 4, gslots);
        uint64_t* sptot;
        ENSURE(B_TOTAL, 4 * sizeof(uint64_t), sptot);   /* total, base, k_small_pairs' batch counter */
        {
            HmFill zf;
            zf.k = 0;
            if (nslots) hm_fill_add(zf, gslots, 0, (size_t)nslots * HM_AG_CELLS * 4);
            hm_fill_add(zf, totals[l], 0, ((size_t)lv[l].count + 1) * 8);
            hm_fill_add(zf, sptot + 2, 0, 8);
            hm_launch_fill(s, zf);
        }
        HmAggArgs a;
        memset(&a, 0, sizeof(a));
        a.B = B[l];
        a.keys = (const uint16_t*)keys_cur;
        a.in = runs_cur;
        a.Z = Z;
        a.lg = Z - zb;
        a.totals = totals[l];
        a.gslots = gslots;
        a.slot_bucket = slot_bucket;
        a.out = o;
        a.items = lv[l].items;
        a.nslots = nslots;
        const uint64_t cnt = (uint64_t)lv[l].count + 1;
        uint64_t *spcnt, *spoff, *partial;
        ENSURE(B_VALS, cnt * 8, spcnt);
        ENSURE(B_PREFIX, cnt * 8, spoff);
        ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
        ENSURE(B_SPCODES, (level_keys + 8) * 2, a.codes);
        a.spcnt = spcnt;
        a.spoff = spoff;
        a.sptotal = sptot;
        a.spbase = (unsigned long long*)(sptot + 1);
        a.spq = (uint32_t*)(sptot + 2);
        hm_launch_aggregate(s, a, lv[l].items, nslots);
        hm_launch_small(s, a, partial);
        HIPCHK(hipGetLastError());
    }
    if (timing) HIPCHK(hipEventRecord(ev[nev], s));
    nev++;
    /* pooling: level l children -> parents in B_{l-1} (root for l = 0) */
    for (int l = L - 1; l >= 0; l--) {
        HmPoolArgs pa;
        memset(&pa, 0, sizeof(pa));
        pa.dbits = lv[l].dbits;
        pa.z_child = lv[l].zc;
        pa.emit_root = (l == 0);
        void* cb = ctx->bufs[B_CHILD0 + l].p;
        pa.child_begin = (const uint32_t*)cb;
        pa.child_digit = B[l].digit;
        pa.child_totals = totals[l];
        pa.parent_coord = l ? B[l - 1].coord : nullptr;
        pa.parent_totals = l ? totals[l - 1] : nullptr;
        pa.out = o;
        pa.nparents = lv[l].nparents;
        hm_launch_pool(s, pa, lv[l].nparents);
        HIPCHK(hipGetLastError());
    }
    if (timing) HIPCHK(hipEventRecord(ev[nev], s));
    nev++;
    if (ctx->tail_keys) {
        hm_launch_stream_rekey_dev(s, ctx->tail_keys, ctx->state + ST_CURSOR, (uint64_t)capacity, ctx->tail_state,
                                   ctx->tail_cb);
        HIPCHK(hipGetLastError());
        ctx->tail_done = 1;
    }
    if ((st = read_state(ctx))) return st;
    for (int i = 0; timing && i + 1 < nev; i++) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
        ctx->stage_us[i] = ms * 1000.0;
    }
    for (int l = 1; timing && l <= npart; l++) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[5 + 2 * (l - 1)], ev[6 + 2 * (l - 1)]);
        ctx->stage_us[4] += ms * 1000.0;
    }
    ctx->stage_us[5] = (double)l1_reruns;   /* hm_last_stats: level-1 re-runs (a region overflowed) */
    ctx->stage_us[6] = (double)nhot;        /* hm_last_stats: hot tiles of the call */
    const unsigned long long nc = ctx->host_state[ST_CURSOR];
    *n_out = (int64_t)nc;
    /* cells outside the square: the general path over the exotic list */
    uint64_t xt = 0;
    if (nx) {
        HmGenEmit e;
        memset(&e, 0, sizeof(e));
        e.cells = xcells_out;
        e.capacity = (uint64_t)xcapacity;
        e.width = 4;
        if ((st = gen_count(ctx, xl.row, xl.col, nullptr, xl.idx, nx, Z, zmin, e, &xt))) return st;
        if ((st = read_state(ctx))) return st;
    }
    *nx_out = (int64_t)xt;
    if (nc > (unsigned long long)capacity || xt > (uint64_t)xcapacity) return HM_E_CAPACITY;
    return HM_OK;
}

extern "C" int hm_count(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep, int64_t n, int zmin,
                        int zmax, uint64_t* keys_out, uint64_t* counts_out, int64_t capacity, int64_t* n_out,
                        int64_t* xcells_out, int64_t xcapacity, int64_t* nx_out)
{
    if (n > 0 && (!lat || !lon)) return HM_E_ARG;
    int st = HM_OK;
    for (int attempt = 0; attempt < 2; attempt++) {
        st = count_impl(ctx, lat, lon, nullptr, nullptr, keep, n, zmin, zmax, keys_out, counts_out, capacity, n_out,
                        xcells_out, xcapacity, nx_out);
        if (st == HM_FALLBACK)
            st = count_fallback(ctx, lat, lon, nullptr, nullptr, keep, n, zmin, zmax, keys_out, counts_out, capacity,
                                n_out, xcells_out, xcapacity, nx_out);
        if (st != HM_E_NOMEM) break;
        arena_release(ctx);   /* cached buffers of earlier calls may be what is missing */
    }
    return st;
}

extern "C" int hm_count_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint8_t* keep, int64_t n,
                              int zmin, int zmax, uint64_t* keys_out, uint64_t* counts_out, int64_t capacity,
                              int64_t* n_out, int64_t* xcells_out, int64_t xcapacity, int64_t* nx_out)
{
    if (n > 0 && (!row || !col)) return HM_E_ARG;
    int st = HM_OK;
    for (int attempt = 0; attempt < 2; attempt++) {
        st = count_impl(ctx, nullptr, nullptr, row, col, keep, n, zmin, zmax, keys_out, counts_out, capacity, n_out,
                        xcells_out, xcapacity, nx_out);
        if (st == HM_FALLBACK)
            st = count_fallback(ctx, nullptr, nullptr, row, col, keep, n, zmin, zmax, keys_out, counts_out, capacity,
                                n_out, xcells_out, xcapacity, nx_out);
        if (st != HM_E_NOMEM) break;
        arena_release(ctx);
    }
    return st;
}

static int grouped_impl(hm_ctx* ctx, const double* lat, const double* lon, const int64_t* rows, const int64_t* cols,
                        const uint8_t* keep, const uint32_t* group, int64_t n, int zmin, int zmax, int64_t* cells_out,
                        int64_t capacity, int64_t* n_out, uint64_t* pkeys = nullptr, uint64_t* pcounts = nullptr)
{
    const bool packed = pkeys || pcounts;
    if (!ctx || !n_out || n < 0 || n >= (int64_t)0xFFFFFFF0ll || zmin < 0 || zmax < zmin ||
        zmax > HM_COUNT_MAX_ZOOM || capacity < 0 ||
        (capacity > 0 && (packed ? (!pkeys || !pcounts) : !cells_out)))
        return HM_E_ARG;
    *n_out = 0;
    HIPCHK(hipSetDevice(ctx->device));
    int st = reset_state(ctx);
    if (st) return st;
    if (n == 0) return HM_OK;
    uint64_t total = 0;
    HmGenEmit e;
    memset(&e, 0, sizeof(e));
    e.cells = cells_out;
    e.capacity = (uint64_t)capacity;
    e.width = 5;
    if (packed) {
        e.cells = nullptr;
        e.keys = pkeys;
        e.counts = pcounts;
        e.width = 2;
    }
    if (rows) {
        int64_t *row, *col, *idx;
        uint32_t* grp;
        ENSURE(B_X_ROW, (uint64_t)n * 8, row);
        ENSURE(B_X_COL, (uint64_t)n * 8, col);
        ENSURE(B_X_IDX, (uint64_t)n * 8, idx);
        ENSURE(B_GL_GRP, (uint64_t)n * 4, grp);
        hm_launch_tiles_list(ctx->stream, rows, cols, keep, group, n, row, col, grp, idx, ctx->state + ST_XCOUNT);
        HIPCHK(hipGetLastError());
        if ((st = read_state(ctx))) return st;
        if ((st = take_error(ctx))) return st;
        st = gen_count(ctx, row, col, grp, idx, ctx->host_state[ST_XCOUNT], zmax, zmin, e, &total);
    } else {   /* points projected straight into keys */
        st = gen_count(ctx, nullptr, nullptr, group, nullptr, (uint64_t)n, zmax, zmin, e, &total, lat, lon, keep);
    }
    if (st) return st;
    *n_out = (int64_t)total;
    return total > (uint64_t)capacity ? HM_E_CAPACITY : HM_OK;
}

extern "C" int hm_count_grouped(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep,
                                const uint32_t* group, int64_t n, int zmin, int zmax, int64_t* cells_out,
                                int64_t capacity, int64_t* n_out)
{
    if (n > 0 && (!lat || !lon)) return HM_E_ARG;
    int st = grouped_impl(ctx, lat, lon, nullptr, nullptr, keep, group, n, zmin, zmax, cells_out, capacity, n_out);
    if (st == HM_E_NOMEM) {
        arena_release(ctx);
        st = grouped_impl(ctx, lat, lon, nullptr, nullptr, keep, group, n, zmin, zmax, cells_out, capacity, n_out);
    }
    return st;
}

extern "C" int hm_count_grouped_packed(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep,
                                       const uint32_t* group, int64_t n, int zmin, int zmax, uint64_t* keys_out,
                                       uint64_t* gcounts_out, int64_t capacity, int64_t* n_out)
{
    if (n > 0 && (!lat || !lon)) return HM_E_ARG;
    int st = grouped_impl(ctx, lat, lon, nullptr, nullptr, keep, group, n, zmin, zmax, nullptr, capacity, n_out,
                          keys_out, gcounts_out);
    if (st == HM_E_NOMEM) {
        arena_release(ctx);
        st = grouped_impl(ctx, lat, lon, nullptr, nullptr, keep, group, n, zmin, zmax, nullptr, capacity, n_out,
                          keys_out, gcounts_out);
    }
    return st;
}

extern "C" int hm_count_grouped_packed_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col,
                                             const uint8_t* keep, const uint32_t* group, int64_t n, int zmin, int zmax,
                                             uint64_t* keys_out, uint64_t* gcounts_out, int64_t capacity,
                                             int64_t* n_out)
{
    if (n > 0 && (!row || !col)) return HM_E_ARG;
    int st = grouped_impl(ctx, nullptr, nullptr, row, col, keep, group, n, zmin, zmax, nullptr, capacity, n_out,
                          keys_out, gcounts_out);
    if (st == HM_E_NOMEM) {
        arena_release(ctx);
        st = grouped_impl(ctx, nullptr, nullptr, row, col, keep, group, n, zmin, zmax, nullptr, capacity, n_out,
                          keys_out, gcounts_out);
    }
    return st;
}

extern "C" int hm_count_grouped_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint8_t* keep,
                                      const uint32_t* group, int64_t n, int zmin, int zmax, int64_t* cells_out,
                                      int64_t capacity, int64_t* n_out)
{
    if (n > 0 && (!row || !col)) return HM_E_ARG;
    int st = grouped_impl(ctx, nullptr, nullptr, row, col, keep, group, n, zmin, zmax, cells_out, capacity, n_out);
    if (st == HM_E_NOMEM) {
        arena_release(ctx);
        st = grouped_impl(ctx, nullptr, nullptr, row, col, keep, group, n, zmin, zmax, cells_out, capacity, n_out);
    }
    return st;
}

/* ------------------------------------------------------------------------ */
/* multi-GPU cell exchange (kernels in hm_merge.hip)                          */
/* ------------------------------------------------------------------------ */

extern "C" int64_t hm_dense_grid_size(int dense_zmax)
{
    if (dense_zmax < 0) return 0;
    if (dense_zmax > 14) return -1;
    return (int64_t)(((1ull << (2 * (dense_zmax + 1))) - 1) / 3);
}

extern "C" int hm_cells_route(hm_ctx* ctx, const uint64_t* keys, const uint64_t* counts, int64_t n, int nranks,
                              int delta, int dense_zmax, uint64_t* grid, void* keys_out, void* counts_out,
                              int layout, int64_t* send_counts)
{
    const bool rec = layout == HM_CELLS_REC10, grp = layout == HM_CELLS_G12;
    if (!ctx || n < 0 || nranks < 1 || nranks > 64 || delta < 0 || delta > 28 || dense_zmax > 14 ||
        (layout != HM_CELLS_U32 && layout != HM_CELLS_U64 && !rec && !grp) || (dense_zmax >= 0 && !grid) ||
        (grp && dense_zmax >= 0) || !send_counts ||
        (n > 0 && (!keys || !counts || !keys_out || (!rec && !counts_out))))
        return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t gsz = hm_dense_grid_size(dense_zmax);
    if (gsz > 0) HIPCHK(hipMemsetAsync(grid, 0, (size_t)gsz * 8, s));
    for (int r = 0; r < nranks; r++) send_counts[r] = 0;
    if (n == 0) return HM_OK;
    const unsigned blocks = hm_route_blocks((uint64_t)n);
    const uint64_t m = (uint64_t)blocks * nranks;
    HmRouteArgs a;
    memset(&a, 0, sizeof(a));
    ENSURE(B_RT_CNT, m * 8, a.block_cnt);
    uint64_t* off;
    ENSURE(B_RT_OFF, (m + 2) * 8, off);    /* + the total, + the wide flag */
    uint64_t *partial, *tot;
    ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
    ENSURE(B_TOTAL, 4 * sizeof(uint64_t), tot);
    a.keys = keys;
    a.counts = counts;
    a.n = (uint64_t)n;
    a.nranks = nranks;
    a.delta = delta;
    a.dense_zmax = dense_zmax;
    a.grid = grid;
    a.block_off = off;
    if (layout == HM_CELLS_U64) {
        a.keys_out = (uint64_t*)keys_out;
        a.counts_out = (uint64_t*)counts_out;
    } else {
        if (rec) {
            a.rec_out = (uint16_t*)keys_out;
        } else {
            a.keys_out = (uint64_t*)keys_out;
            a.counts_out32 = (uint32_t*)counts_out;
            a.grouped = grp;
        }
        a.wide = (unsigned long long*)(off + m + 1);
        HIPCHK(hipMemsetAsync(a.wide, 0, 8, s));
    }
    hm_launch_cells_route(s, a, false);
    hm_launch_scan(s, a.block_cnt, m, partial, off, off + m);
    hm_launch_cells_route(s, a, true);
    HIPCHK(hipGetLastError());
    std::vector<uint64_t> h(m + 2);
    HIPCHK(hipMemcpyAsync(h.data(), off, (m + 2) * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hm_sync(s));
    for (int r = 0; r < nranks; r++)
        send_counts[r] = (int64_t)(h[(uint64_t)(r + 1) * blocks] - h[(uint64_t)r * blocks]);
    return (layout != HM_CELLS_U64 && h[m + 1]) ? HM_E_WIDE : HM_OK;
}

static int cells_merge(hm_ctx* ctx, const void* keys_in, const void* counts_in, int layout, int64_t n,
                       const int64_t* runs, int nruns, uint64_t* keys_out, uint64_t* counts_out, int64_t capacity,
                       int64_t* n_out)
{
    const uint16_t* recs = layout == HM_CELLS_REC10 ? (const uint16_t*)keys_in : nullptr;
    const uint64_t* keys = recs ? nullptr : (const uint64_t*)keys_in;
    const uint64_t* counts = layout == HM_CELLS_U64 ? (const uint64_t*)counts_in : nullptr;
    const uint32_t* counts32 = layout == HM_CELLS_U32 ? (const uint32_t*)counts_in : nullptr;
    if (((uintptr_t)recs & 1) != 0) return HM_E_ARG;   /* records: u16 words */
    if (!ctx || !n_out || n < 0 || capacity < 0 || (n > 0 && !keys_in) || (n > 0 && !recs && !counts && !counts32) ||
        (capacity > 0 && (!keys_out || !counts_out)) || nruns < 0 || (nruns > 0 && !runs))
        return HM_E_ARG;
    int64_t sum = 0;
    for (int i = 0; i < nruns; i++) {
        if (runs[i] < 0) return HM_E_ARG;
        sum += runs[i];
    }
    if (runs && sum != n) return HM_E_ARG;
    *n_out = 0;
    if (n == 0) return HM_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    unsigned long long* down = ctx->host_state + 2 * ST_COUNT;
    const uint64_t *pk_all = nullptr, *pc_all = nullptr;   /* the first partition pass's copy (u64 counts) */
    {
        /* bucketed LDS merge (hm_merge.hip): 2^lb hash buckets of <= ~1800
         * cells (one LDS table pass each), one block per bucket; the cells are
         * hash-partitioned by the top lb bits in one or two coalesced passes
         * of <= 7 bits */
        HmMergeArgs a;
        memset(&a, 0, sizeof(a));
        int lb = 0;
        while (lb < 14 && ((uint64_t)n >> lb) > 1800) lb++;
        const int b1 = lb <= 7 ? lb : (lb + 1) / 2, b2 = lb - b1;
        auto chunks = [](uint64_t cells, uint64_t per, uint32_t cap) {
            return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cap, (cells + per - 1) / per));
        };
        HmMbPass p1;
        memset(&p1, 0, sizeof(p1));
        p1.kin = keys;
        p1.cin = counts;
        p1.cin32 = counts32;
        p1.rin = recs;
        p1.n = (uint64_t)n;
        p1.nseg = 1;
        p1.C = chunks((uint64_t)n, 65536, 512);
        p1.shift = b1 ? 64 - b1 : 63;   /* b1 = 0: one bucket (digit mask 0; no shift by 64) */
        p1.bits = b1;
        const uint64_t m1 = ((uint64_t)1 << b1) * p1.C;
        uint64_t *cnt1, *off1, *pk, *pc;
        ENSURE(B_MB_CNT, m1 * 8, cnt1);
        ENSURE(B_MB_OFF, (m1 + 1) * 8, off1);
        ENSURE(B_MB_KEYS, (uint64_t)n * 8, pk);
        ENSURE(B_MB_COUNTS, (uint64_t)n * 8, pc);
        uint64_t* partial;
        ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
        p1.cnt = cnt1;
        p1.off = off1;
        p1.kout = pk;
        p1.cout = pc;
        hm_launch_mb_pass(s, p1, false);
        hm_launch_scan(s, cnt1, m1, partial, off1, off1 + m1);
        hm_launch_mb_pass(s, p1, true);
        a.pkeys = pk;
        a.pcounts = pc;
        a.boff = off1;
        a.nblocks = p1.C;
        if (b2 > 0) {
            /* second pass: each first-pass bucket (a segment) by the next b2 bits */
            HmMbPass p2 = p1;
            p2.kin = pk;
            p2.cin = pc;
            p2.cin32 = nullptr;
            p2.rin = nullptr;
            p2.segoff = off1;
            p2.segstride = p1.C;
            p2.nseg = 1u << b1;
            p2.C = chunks((uint64_t)n >> b1, 32768, 64);
            p2.shift = 64 - lb;
            p2.bits = b2;
            const uint64_t m2 = ((uint64_t)1 << lb) * p2.C;
            uint64_t *cnt2, *off2, *qk, *qc;
            ENSURE(B_MB_CNT2, m2 * 8, cnt2);
            ENSURE(B_MB_OFF2, (m2 + 1) * 8, off2);
            ENSURE(B_MB_KEYS2, (uint64_t)n * 8, qk);
            ENSURE(B_MB_COUNTS2, (uint64_t)n * 8, qc);
            p2.cnt = cnt2;
            p2.off = off2;
            p2.kout = qk;
            p2.cout = qc;
            hm_launch_mb_pass(s, p2, false);
            hm_launch_scan(s, cnt2, m2, partial, off2, off2 + m2);
            hm_launch_mb_pass(s, p2, true);
            a.pkeys = qk;
            a.pcounts = qc;
            a.boff = off2;
            a.nblocks = p2.C;
        }
        a.keys = keys;
        a.counts = counts;
        a.n = (uint64_t)n;
        a.lb = lb;
        pk_all = pk;
        pc_all = pc;
        unsigned long long* st;
        ENSURE(B_MG_STATE, 8 * sizeof(unsigned long long), st);
        HIPCHK(hipMemsetAsync(st, 0, 8 * sizeof(unsigned long long), s));
        a.keys_out = keys_out;
        a.counts_out = counts_out;
        a.cap = (uint64_t)capacity;
        a.cursor = st;
        a.overflow = st + 1;
        hm_launch_mb_merge(s, a);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(down, st, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIPCHK(hm_sync(s));
        if (!down[1]) {
            *n_out = (int64_t)down[0];
            return *n_out > capacity ? HM_E_CAPACITY : HM_OK;
        }
        /* a bucket's table filled up (adversarial hash collisions): the
         * global hash table below takes the whole merge again */
    }
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)n) cap <<= 1;
    HmsTable t;
    ENSURE(B_MG_TABLE, cap * 16, t.slots);
    ENSURE(B_MG_STATE, 8 * sizeof(unsigned long long), t.state);
    t.mask = cap - 1;
    HIPCHK(hipMemsetAsync(t.state, 0, 8 * sizeof(unsigned long long), s));
    hm_launch_stream_init(s, t);
    if (!counts) {
        /* u32 counts or records: the partition pass's u64 copy, in partition order */
        hm_launch_cells_merge(s, pk_all, pc_all, (uint64_t)n, t);
    } else if (runs) {
        /* runs of distinct keys: no two threads of a launch insert one key */
        int64_t off = 0;
        for (int i = 0; i < nruns; i++) {
            hm_launch_cells_merge_unique(s, keys + off, counts + off, (uint64_t)runs[i], t);
            off += runs[i];
        }
    } else {
        hm_launch_cells_merge(s, keys, counts, (uint64_t)n, t);
    }
    hm_launch_table_extract(s, t, keys_out, counts_out, (uint64_t)capacity, t.state + HMS_ST_CURSOR);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(down, t.state, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hm_sync(s));
    if (down[HMS_ST_OVERFLOW]) return HM_E_HIP;   /* cannot happen: load factor <= 1/2 */
    *n_out = (int64_t)down[HMS_ST_CURSOR];
    return *n_out > capacity ? HM_E_CAPACITY : HM_OK;
}

static bool cells_layout_ok(int layout)
{
    return layout == HM_CELLS_U64 || layout == HM_CELLS_U32 || layout == HM_CELLS_REC10;
}

extern "C" int hm_cells_merge(hm_ctx* ctx, const void* keys, const void* counts, int layout, int64_t n,
                              uint64_t* keys_out, uint64_t* counts_out, int64_t capacity, int64_t* n_out)
{
    if (!cells_layout_ok(layout)) return HM_E_ARG;
    return cells_merge(ctx, keys, counts, layout, n, nullptr, 0, keys_out, counts_out, capacity, n_out);
}

extern "C" int hm_cells_merge_runs(hm_ctx* ctx, const void* keys, const void* counts, int layout, int64_t n,
                                   const int64_t* runs, int nruns, uint64_t* keys_out, uint64_t* counts_out,
                                   int64_t capacity, int64_t* n_out)
{
    if (!cells_layout_ok(layout)) return HM_E_ARG;
    return cells_merge(ctx, keys, counts, layout, n, runs, nruns, keys_out, counts_out, capacity, n_out);
}

/* the pieces exchange (hm_merge.hip, "the pieces exchange"): the route orders
 * each owner's group by the first merge digit, so the owner gathers digit
 * s's pieces, partitions them by the next bits and merges */
extern "C" int hm_cells_route_pieces(hm_ctx* ctx, const uint64_t* keys, const uint64_t* counts, int64_t n,
                                     int nranks, int delta, int dense_zmax, int bits, int self_rank, uint64_t* grid,
                                     void* keys_out, void* counts_out, int layout, int64_t* sizes, int stride)
{
    const bool rec = layout == HM_CELLS_REC10, grp = layout == HM_CELLS_G12;
    if (!ctx || n < 0 || nranks < 1 || nranks > 64 || delta < 0 || delta > 28 || dense_zmax > 14 || bits < 0 ||
        self_rank < -1 || self_rank >= nranks ||
        bits > 7 || ((int64_t)nranks << bits) > HM_XR_MAXD || stride < 2 + (1 << bits) || !sizes ||
        (layout != HM_CELLS_U32 && layout != HM_CELLS_U64 && !rec && !grp) || (dense_zmax >= 0 && !grid) ||
        (grp && dense_zmax >= 0) || (n > 0 && (!keys || !counts || !keys_out || (!rec && !counts_out))) ||
        (rec && ((uintptr_t)keys_out & 1)))
        return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t gsz = hm_dense_grid_size(dense_zmax);
    if (gsz > 0) HIPCHK(hipMemsetAsync(grid, 0, (size_t)gsz * 8, s));
    HmRouteArgs a;
    memset(&a, 0, sizeof(a));
    a.C = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, ((uint64_t)n + 16383) / 16384));
    const uint64_t m = ((uint64_t)nranks << bits) * a.C;
    ENSURE(B_RT_CNT, m * 8, a.block_cnt);
    uint64_t* off;
    ENSURE(B_RT_OFF, (m + 2) * 8, off);    /* + the total, + the wide flag */
    uint64_t* partial;
    ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
    a.keys = keys;
    a.counts = counts;
    a.n = (uint64_t)n;
    a.nranks = nranks;
    a.delta = delta;
    a.dense_zmax = dense_zmax;
    a.grid = grid;
    a.block_off = off;
    a.bits = bits;
    a.sizes = (long long*)sizes;
    a.stride = stride;
    a.self = self_rank;
    if (layout == HM_CELLS_U64) {
        a.keys_out = (uint64_t*)keys_out;
        a.counts_out = (uint64_t*)counts_out;
    } else if (rec) {
        a.rec_out = (uint16_t*)keys_out;
    } else {
        a.keys_out = (uint64_t*)keys_out;
        a.counts_out32 = (uint32_t*)counts_out;
        a.grouped = grp;
    }
    if (layout != HM_CELLS_U64) {
        a.wide = (unsigned long long*)(off + m + 1);
        HIPCHK(hipMemsetAsync(a.wide, 0, 8, s));
    }
    hm_launch_xroute(s, a, false, layout);
    hm_launch_scan(s, a.block_cnt, m, partial, off, off + m);
    if (n > 0) hm_launch_xroute(s, a, true, layout);
    hm_launch_xroute_sizes(s, a);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

extern "C" int hm_cells_merge_pieces(hm_ctx* ctx, int layout, int nruns, const void* const* key_src,
                                     const void* const* count_src, const int64_t* pieces, int bits,
                                     uint64_t* keys_out, uint64_t* counts_out, int64_t capacity, int64_t* n_out)
{
    const bool rec = layout == HM_CELLS_REC10, c64 = layout == HM_CELLS_U64;
    if (!ctx || !n_out || nruns < 1 || nruns > 64 || bits < 0 || bits > 7 || !pieces || !key_src ||
        (layout != HM_CELLS_U32 && !c64 && layout != HM_CELLS_G12 && !rec) || (!rec && !count_src) ||
        capacity < 0 || (capacity > 0 && (!keys_out || !counts_out)))
        return HM_E_ARG;
    const uint32_t S = 1u << bits, R = (uint32_t)nruns;
    uint64_t n = 0;
    for (uint32_t r = 0; r < R; r++) {
        uint64_t len = 0;
        for (uint32_t d = 0; d < S; d++) {
            if (pieces[r * S + d] < 0) return HM_E_ARG;
            len += (uint64_t)pieces[r * S + d];
        }
        if (len && (!key_src[r] || (!rec && !count_src[r]) || (rec && ((uintptr_t)key_src[r] & 1))))
            return HM_E_ARG;
        n += len;
    }
    *n_out = 0;
    if (n == 0) return HM_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    unsigned long long* down = ctx->host_state + 2 * ST_COUNT;
    /* buckets of <= HM_MB2_TARGET cells (one LDS table pass each) */
    int lb = bits;
    while (lb < bits + 8 && (n >> lb) > HM_MB2_TARGET) lb++;
    const int b2 = lb - bits;
    /* piece table: vpre [S][R + 1], key address [S][R], count address [S][R] */
    const size_t ksz = rec ? 10 : 8, csz = c64 ? 8 : 4;
    std::vector<unsigned long long> tab((size_t)S * (R + 1) + 2 * (size_t)S * R, 0ull);
    unsigned long long *vpre = tab.data(), *kp = vpre + (size_t)S * (R + 1), *cp = kp + (size_t)S * R;
    for (uint32_t r = 0; r < R; r++) {
        uint64_t e = 0;   /* cells of run r before piece d */
        for (uint32_t d = 0; d < S; d++) {
            kp[d * R + r] = (unsigned long long)((uintptr_t)key_src[r] + e * ksz);
            cp[d * R + r] = rec ? 0ull : (unsigned long long)((uintptr_t)count_src[r] + e * csz);
            e += (uint64_t)pieces[r * S + d];
        }
    }
    for (uint32_t d = 0; d < S; d++) {
        uint64_t v = 0;
        for (uint32_t r = 0; r < R; r++) {
            vpre[d * (R + 1) + r] = v;
            v += (uint64_t)pieces[r * S + d];
        }
        vpre[d * (R + 1) + R] = v;
    }
    unsigned long long* dtab;
    ENSURE(B_MG_PIECES, tab.size() * 8, dtab);
    HIPCHK(hipMemcpyAsync(dtab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, s));
    HmMbGather g;
    memset(&g, 0, sizeof(g));
    g.vpre = dtab;
    g.kp = dtab + (size_t)S * (R + 1);
    g.cp = rec ? nullptr : g.kp + (size_t)S * R;
    g.R = R;
    g.S = S;
#ifndef HM_MG_CHUNK
#define HM_MG_CHUNK 16384
#endif
    g.C = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, ((n >> bits) + HM_MG_CHUNK - 1) / HM_MG_CHUNK));
    g.shift = lb ? 64 - lb : 63;
    g.bits = b2;
    g.in_layout = rec ? HM_CELLS_REC10 : (c64 ? HM_CELLS_U64 : HM_CELLS_U32);
    uint64_t *partial, *qk;
    void* qc;
    unsigned long long* st;
    ENSURE(B_PARTIAL, 4096 * sizeof(uint64_t), partial);
    ENSURE(B_MG_STATE, 8 * sizeof(unsigned long long), st);
    HmMergeArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    a.lb = lb;
    a.keys_out = keys_out;
    a.counts_out = counts_out;
    a.cap = (uint64_t)capacity;
    a.cursor = st;
    a.overflow = st + 1;
    /* fill mode: no count pass -- buckets of a fixed capacity (the mean
     * + 1/4 + 64; hash buckets are near the mean), claimed per tile; a bucket
     * past it (st[2]) or a full LDS table sends the call to the counted form */
    const char* fe = getenv("HM_GATHER_FILL");   /* 0: always the counted form (A/B) */
    const char* be = getenv("HM_GATHER_BCAP");   /* test hook: a bucket capacity (forces the fallback) */
    const uint64_t nbk = 1ull << lb;
    const bool fill = (!fe || atoi(fe) != 0) && n >= 4096;
    auto counted = [&]() -> int {
        const uint64_t m2 = ((uint64_t)S << b2) * g.C;
        uint64_t *cnt2, *off2;
        ENSURE(B_MB_CNT2, m2 * 8, cnt2);
        ENSURE(B_MB_OFF2, (m2 + 1) * 8, off2);
        ENSURE(B_MB_KEYS2, n * 8, qk);
        ENSURE(B_MB_COUNTS2, n * csz, qc);
        g.cnt = cnt2;
        g.off = off2;
        g.kout = qk;
        g.cout = qc;
        g.fill = nullptr;
        hm_launch_mb_gather(s, g, false);
        hm_launch_scan(s, cnt2, m2, partial, off2, off2 + m2);
        hm_launch_mb_gather(s, g, true);
        a.boff = off2;
        a.nblocks = g.C;
        a.bfill = nullptr;
        return HM_OK;
    };
    HIPCHK(hipMemsetAsync(st, 0, 8 * sizeof(unsigned long long), s));
    if (fill) {
        const uint64_t mean = (n + nbk - 1) / nbk;
        const uint64_t bcap = be && atoll(be) > 0 ? (uint64_t)atoll(be) : mean + mean / 4 + 64;
        unsigned long long* fc;
        ENSURE(B_MB_CNT2, nbk * 8, fc);
        ENSURE(B_MB_KEYS2, nbk * bcap * 8, qk);
        ENSURE(B_MB_COUNTS2, nbk * bcap * csz, qc);
        HIPCHK(hipMemsetAsync(fc, 0, nbk * 8, s));
        g.kout = qk;
        g.cout = qc;
        g.fill = fc;
        g.bcap = bcap;
        g.over = st + 2;
        hm_launch_mb_gather(s, g, true);
        a.bfill = fc;
        a.bcap = bcap;
    } else {
        int st2 = counted();
        if (st2 != HM_OK) return st2;
    }
    if (c64) a.pcounts = (uint64_t*)qc;
    else a.pcounts32 = (const uint32_t*)qc;
    a.pkeys = qk;
    hm_launch_mb_merge2(s, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(down, st, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hm_sync(s));
    if (fill && (down[1] || down[2])) {
        /* a bucket past its capacity, or a full table: partition again with the
         * count pass (contiguous buckets, which the global table below can take) */
        HIPCHK(hipMemsetAsync(st, 0, 8 * sizeof(unsigned long long), s));
        int st2 = counted();
        if (st2 != HM_OK) return st2;
        a.pkeys = qk;
        if (c64) a.pcounts = (uint64_t*)qc;
        else a.pcounts32 = (const uint32_t*)qc;
        hm_launch_mb_merge2(s, a);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(down, st, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIPCHK(hm_sync(s));
    }
    if (!down[1]) {
        *n_out = (int64_t)down[0];
        return *n_out > capacity ? HM_E_CAPACITY : HM_OK;
    }
    /* a bucket's table filled up (adversarial hash collisions): a global hash
     * table takes the partitioned cells */
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    HmsTable t;
    ENSURE(B_MG_TABLE, cap * 16, t.slots);
    ENSURE(B_MG_STATE, 8 * sizeof(unsigned long long), t.state);
    t.mask = cap - 1;
    HIPCHK(hipMemsetAsync(t.state, 0, 8 * sizeof(unsigned long long), s));
    hm_launch_stream_init(s, t);
    if (c64) hm_launch_cells_merge(s, qk, (const uint64_t*)qc, n, t);
    else hm_launch_cells_merge32(s, qk, (const uint32_t*)qc, n, t);
    hm_launch_table_extract(s, t, keys_out, counts_out, (uint64_t)capacity, t.state + HMS_ST_CURSOR);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(down, t.state, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hm_sync(s));
    if (down[HMS_ST_OVERFLOW]) return HM_E_HIP;
    *n_out = (int64_t)down[HMS_ST_CURSOR];
    return *n_out > capacity ? HM_E_CAPACITY : HM_OK;
}

extern "C" int hm_dense_cells(hm_ctx* ctx, const uint64_t* grid, int dense_zmax, uint64_t* keys_out,
                              uint64_t* counts_out, int64_t capacity, int64_t* n_out)
{
    if (!ctx || !n_out || !grid || dense_zmax < 0 || dense_zmax > 14 || capacity < 0 ||
        (capacity > 0 && (!keys_out || !counts_out)))
        return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    unsigned long long* cur = ctx->state + ST_CURSOR;
    HIPCHK(hipMemsetAsync(cur, 0, 8, s));
    hm_launch_dense_extract(s, grid, (uint64_t)hm_dense_grid_size(dense_zmax), dense_zmax, keys_out, counts_out,
                            (uint64_t)capacity, cur);
    HIPCHK(hipGetLastError());
    int st = read_state(ctx);
    if (st) return st;
    *n_out = (int64_t)ctx->host_state[ST_CURSOR];
    return *n_out > capacity ? HM_E_CAPACITY : HM_OK;
}

extern "C" int hm_format_bins(hm_ctx* ctx, const int64_t* zoom, const int64_t* row, const int64_t* col,
                              const int64_t* value, const uint8_t* head, const uint8_t* last, const int64_t* offset,
                              int64_t n, uint8_t* text)
{
    if (!ctx || n < 0 || (n > 0 && (!zoom || !row || !col || !value || !head || !last || !offset || !text)))
        return HM_E_ARG;
    if (n == 0) return HM_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HmFormatArgs a{zoom, row, col, value, head, last, offset, n, text};
    hm_launch_format_bins(ctx->stream, a);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

extern "C" int hm_format_ids(hm_ctx* ctx, const uint8_t* names, const int64_t* name_off, const int64_t* label,
                             const uint8_t* spans, const int64_t* span_off, const int64_t* span, const int64_t* tz,
                             const int64_t* tr, const int64_t* tc, const int64_t* offset, int64_t n, uint8_t* text)
{
    if (!ctx || n < 0 ||
        (n > 0 && (!names || !name_off || !label || !spans || !span_off || !span || !tz || !tr || !tc || !offset ||
                   !text)))
        return HM_E_ARG;
    if (n == 0) return HM_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HmIdArgs a{names, name_off, label, spans, span_off, span, tz, tr, tc, offset, n, text};
    hm_launch_format_ids(ctx->stream, a);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

extern "C" int hm_synth(hm_ctx* ctx, int kind, uint64_t seed, int64_t start, int64_t n, double* lat, double* lon,
                        const double* table, int k)
{
    if (!ctx || n < 0 || kind < 0 || kind > 2 || (n > 0 && (!lat || !lon)) || (kind == 1 && (!table || k <= 0)))
        return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (n > 0) hm_launch_synth(ctx->stream, kind, seed, start, n, lat, lon, table, k);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

extern "C" int hm_bench_read(hm_ctx* ctx, const void* a, const void* b, int64_t bytes_each, uint64_t* sink)
{
    if (!ctx || bytes_each < 0 || (bytes_each & 15) || (bytes_each > 0 && (!a || !b || !sink))) return HM_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (bytes_each > 0) hm_launch_read_stream(ctx->stream, a, b, (uint64_t)bytes_each, sink);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

/* ------------------------------------------------------------------------ */
/* streaming: resident multi-zoom heatmap (kernels in hm_stream.hip)          */
/* ------------------------------------------------------------------------ */

#define HMS_PAR 4
struct hm_stream {
    hm_ctx* ctx = nullptr;
    int zmin = 0, zmax = 0;
    int cb = 0;                           /* cell bits of a log key */
    uint32_t base = 0;
    unsigned long long* state = nullptr;  /* device HMS_ST_* words */
    HmsBuckets bk{};                      /* (group, period) buckets */
    uint32_t *bflag = nullptr, *blist = nullptr, *bloc = nullptr; /* per bucket: last batch, list, run */
    uint32_t epoch = 0;
    uint32_t last_nparts = 1;             /* buckets of the previous batch (1: count the next one speculatively) */
    /* the cell log: llen cells of lcap; alt: the compaction target */
    uint64_t *lkeys = nullptr, *lcounts = nullptr, *akeys = nullptr, *acounts = nullptr;
    uint64_t lcap = 0, llen = 0;
    bool compact = true;                  /* the log holds distinct keys */
    bool par = true;                      /* several-bucket batches counted concurrently (HM_STREAM_PAR=0: not) */
    /* while compact: the buckets with cells in the log.  A one-bucket batch
     * of a bucket not in it keeps the log compact (one count's cells are
     * distinct), so a stream of new hours never needs a compaction pass */
    std::unordered_set<uint32_t> log_buckets;
    uint64_t nbuckets = 0;
    unsigned long long* hstate = nullptr; /* pinned mirror of state */
    Buf bids, rec;                        /* per-batch scratch */
    Buf plat, plon, pkeep, pstart, pcnt;  /* partition path: bucket-contiguous batch */
    int64_t rcap = 0;                     /* records rec holds */
    Buf rk, rc, mk, mc;                   /* rollup scratch: relabeled and merged cells */
    /* several-bucket batches: up to HMS_PAR buckets counted at once, each by
     * its own context, stream and host thread, into its own scratch */
    hm_ctx* pctx[HMS_PAR] = {};
    Buf pk[HMS_PAR], pc[HMS_PAR];
    hipEvent_t pev = nullptr;
    /* the log arrays as growable reservations (log_alloc): base -> its
     * reservation, so a full log maps more pages behind its cells instead of
     * being copied into a buffer twice the size */
    struct VArr {
        size_t reserved = 0, mapped = 0;
        std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
    };
    std::unordered_map<void*, VArr> varr;
    bool vmm = true;                      /* HM_STREAM_VMM=0: plain allocations, grown by copying */
    /* maps the log's next extent ahead of need, on a host thread, while the
     * batches run (every varr access joins it first) */
    std::thread premap;
};

static void premap_join(hm_stream* s)
{
    if (s->premap.joinable()) s->premap.join();
}

/* ---- the log's growable arrays ---- */
static hipMemAllocationProp log_prop(int device)
{
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    return prop;
}

/* map [mapped, bytes) of reservation v at base p (bytes: a granularity multiple) */
static bool log_map(hm_stream* s, void* p, hm_stream::VArr& v, size_t bytes)
{
    if (bytes <= v.mapped) return true;
    if (bytes > v.reserved) return false;
    const hipMemAllocationProp prop = log_prop(s->ctx->device);
    const size_t add = bytes - v.mapped;
    hipMemGenericAllocationHandle_t h;
    if (hipMemCreate(&h, add, &prop, 0) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    char* at = (char*)p + v.mapped;
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemMap(at, add, 0, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipMemRelease(h);
        return false;
    }
    if (hipMemSetAccess(at, add, &d, 1) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipMemUnmap(at, add);
        (void)hipMemRelease(h);
        return false;
    }
    v.chunks.push_back({h, add});
    v.mapped = bytes;
    return true;
}

static size_t log_round(hm_stream* s, size_t bytes)
{
    const hipMemAllocationProp prop = log_prop(s->ctx->device);
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || !g) {
        (void)hipGetLastError();
        g = 2u << 20;
    }
    return (bytes + g - 1) / g * g;
}

static void log_free(hm_stream* s, void* p)
{
    premap_join(s);
    if (!p) return;
    auto it = s->varr.find(p);
    if (it == s->varr.end()) {
        (void)hipFree(p);
        return;
    }
    size_t off = 0;
    for (auto& c : it->second.chunks) {
        (void)hipMemUnmap((char*)p + off, c.second);
        (void)hipMemRelease(c.first);
        off += c.second;
    }
    (void)hipMemAddressFree(p, it->second.reserved);
    s->varr.erase(it);
}

/* n cells: a reservation of 64x that (at most the device's memory) with the
 * first n mapped, or a plain allocation when reservations are off or fail */
static int log_alloc(hm_stream* s, uint64_t n, uint64_t** out)
{
    premap_join(s);
    *out = nullptr;
    if (s->vmm) {
        size_t total = 0, freeb = 0;
        if (hipMemGetInfo(&freeb, &total) != hipSuccess) {
            (void)hipGetLastError();
            total = 0;
        }
        const size_t want = log_round(s, (size_t)n * 8);
        size_t res = log_round(s, std::max<size_t>(want, std::min<size_t>((size_t)n * 8 * 64, total ? total : want)));
        void* p = nullptr;
        if (hipMemAddressReserve(&p, res, 0, nullptr, 0) == hipSuccess) {
            hm_stream::VArr v;
            v.reserved = res;
            if (log_map(s, p, v, want)) {
                s->varr[p] = std::move(v);
                *out = (uint64_t*)p;
                return HM_OK;
            }
            (void)hipMemAddressFree(p, res);
        }
        (void)hipGetLastError();
    }
    if (hipMalloc((void**)out, n * 8) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return HM_E_NOMEM;
    }
    return HM_OK;
}

/* grow the array at p to n cells in place; false: not a reservation, or it is too small */
static bool log_grow(hm_stream* s, uint64_t* p, uint64_t n)
{
    premap_join(s);
    auto it = s->varr.find((void*)p);
    return it != s->varr.end() && log_map(s, p, it->second, log_round(s, (size_t)n * 8));
}

static int stream_sync_state(hm_stream* s)
{
    HIPCHK(hipMemcpyAsync(s->hstate, s->state, HMS_ST_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          s->ctx->stream));
    HIPCHK(hm_sync(s->ctx->stream));
    s->nbuckets = s->hstate[HMS_ST_BUCKETS];
    return HM_OK;
}

static int stream_buf(hm_stream* s, Buf& b, size_t bytes)
{
    (void)s;
    if (b.cap >= bytes) return HM_OK;
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return HM_E_NOMEM;
    }
    b.cap = bytes;
    return HM_OK;
}

static int stream_alloc2(hm_stream* s, uint64_t n, uint64_t** k, uint64_t** c)
{
    *k = nullptr;
    *c = nullptr;
    if (log_alloc(s, n, k) != HM_OK || log_alloc(s, n, c) != HM_OK) {
        log_free(s, *k);
        *k = nullptr;
        *c = nullptr;
        return HM_E_NOMEM;
    }
    return HM_OK;
}

/* sum the log's equal keys (the bucketed LDS merge) into the alternate
 * arrays, then swap them in */
static int stream_compact(hm_stream* s)
{
    if (s->compact || s->llen == 0) {
        s->compact = true;
        return HM_OK;
    }
    int st;
    if (!s->akeys && (st = stream_alloc2(s, s->lcap, &s->akeys, &s->acounts))) return st;
    int64_t m = 0;
    if ((st = cells_merge(s->ctx, s->lkeys, s->lcounts, HM_CELLS_U64, (int64_t)s->llen, nullptr, 0, s->akeys, s->acounts,
                          (int64_t)s->lcap, &m)))
        return st;
    std::swap(s->lkeys, s->akeys);
    std::swap(s->lcounts, s->acounts);
    s->llen = (uint64_t)m;
    s->compact = true;   /* (compaction adds no bucket: log_buckets stays exact) */
    return HM_OK;
}

/* room for `need` more cells at the log's tail: compact first, then grow */
/* the log will be over 3/4 full: map the next doubling's pages now, on a
 * host thread (hipMemCreate of a few hundred MB costs about a batch) */
static void premap_ahead(hm_stream* s, uint64_t need)
{
    if (!s->vmm || s->premap.joinable() || s->lcap - s->llen - need >= s->lcap / 4) return;
    auto ik = s->varr.find((void*)s->lkeys), ic = s->varr.find((void*)s->lcounts);
    if (ik == s->varr.end() || ic == s->varr.end()) return;
    const size_t bytes = log_round(s, (size_t)s->lcap * 16);
    if (bytes > ik->second.reserved || bytes > ic->second.reserved) return;
    if (ik->second.mapped >= bytes && ic->second.mapped >= bytes) return;
    hm_stream::VArr *vk = &ik->second, *vc = &ic->second;   /* (stable: every insert or erase joins first) */
    void *pk = s->lkeys, *pc = s->lcounts;
    const int dev = s->ctx->device;
    s->premap = std::thread([s, vk, vc, pk, pc, bytes, dev]() {
        (void)hipSetDevice(dev);
        if (log_map(s, pk, *vk, bytes)) (void)log_map(s, pc, *vc, bytes);
    });
}

static int stream_room(hm_stream* s, uint64_t need)
{
    if (s->lcap - s->llen >= need) {
        premap_ahead(s, need);
        return HM_OK;
    }
    premap_join(s);
    int st;
    if ((st = stream_compact(s))) return st;
    if (s->lcap - s->llen >= need) return HM_OK;
    uint64_t cap = s->lcap ? s->lcap : 1024;
    while (cap - s->llen < need) cap <<= 1;
    /* reservations: more pages behind the cells, no copy and no sync (the
     * compaction target, when there is one, grows with them or is dropped) */
    if (log_grow(s, s->lkeys, cap) && log_grow(s, s->lcounts, cap)) {
        if (s->akeys && !(log_grow(s, s->akeys, cap) && log_grow(s, s->acounts, cap))) {
            HIPCHK(hm_sync(s->ctx->stream));
            log_free(s, s->akeys);
            log_free(s, s->acounts);
            s->akeys = s->acounts = nullptr;
        }
        s->lcap = cap;
        return HM_OK;
    }
    uint64_t *k, *c;
    if ((st = stream_alloc2(s, cap, &k, &c))) return st;
    hipStream_t q = s->ctx->stream;
    if (s->llen) {
        HIPCHK(hipMemcpyAsync(k, s->lkeys, s->llen * 8, hipMemcpyDeviceToDevice, q));
        HIPCHK(hipMemcpyAsync(c, s->lcounts, s->llen * 8, hipMemcpyDeviceToDevice, q));
    }
    HIPCHK(hm_sync(q));
    for (uint64_t* p : {s->lkeys, s->lcounts, s->akeys, s->acounts}) log_free(s, p);
    s->lkeys = k;
    s->lcounts = c;
    s->akeys = s->acounts = nullptr;   /* the compaction target, at the new size when needed */
    s->lcap = cap;
    return HM_OK;
}

/* m cells appended at the tail; bucket: the batch's one bucket, or
 * 0xFFFFFFFF for cells of several buckets (from then on the log's buckets
 * are not all known, and every append clears the compact flag) */
static void stream_appended(hm_stream* s, uint64_t m, const uint32_t* buckets, uint32_t nb)
{
    if (m) {
        /* each bucket's cells come from one count, so they are distinct: the
         * log stays compact when it was empty, or when none of the buckets
         * has cells in it yet (the log's buckets all known) */
        if (s->llen == 0) s->log_buckets.clear();
        bool fresh = !s->log_buckets.count(0xFFFFFFFFu);
        for (uint32_t j = 0; j < nb && fresh; j++) fresh = !s->log_buckets.count(buckets[j]);
        s->compact = s->compact && (s->llen == 0 || fresh);
        for (uint32_t j = 0; j < nb; j++) s->log_buckets.insert(buckets[j]);
    }
    s->llen += m;
}

static void stream_appended(hm_stream* s, uint64_t m, uint32_t bucket = 0xFFFFFFFFu)
{
    stream_appended(s, m, &bucket, 1);
}

/* a batch of one bucket, part 1: hm_count's cells written at the log's tail
 * (not yet part of the log) */
static int stream_count_tail(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep, int64_t n,
                             int64_t* m)
{
    int st;
    *m = 0;
    if ((st = stream_room(s, 2 * (uint64_t)n + 1024))) return st; /* typical batches: fewer cells than 2 per point */
    for (;;) {
        int64_t nx = 0;
        s->ctx->tail_keys = s->lkeys + s->llen;
        s->ctx->tail_state = s->state;
        s->ctx->tail_cb = s->cb;
        s->ctx->tail_done = 0;
        st = hm_count(s->ctx, lat, lon, keep, n, s->zmin, s->zmax, s->lkeys + s->llen, s->lcounts + s->llen,
                      (int64_t)(s->lcap - s->llen), m, nullptr, 0, &nx);
        s->ctx->tail_keys = nullptr;
        /* the log's keys hold tiles inside [0, 2^z)^2 only */
        if (nx > 0) return HM_E_EXOTIC;
        if (st != HM_E_CAPACITY) return st;
        if ((st = stream_room(s, (uint64_t)(*m + *m / 4 + 1024)))) return st;
    }
}

/* part 2: the tail's m cells keyed under the bucket and appended */
static int stream_take_tail(hm_stream* s, int64_t m, uint32_t bucket)
{
    /* re-keyed inside the count already unless it took the fallback path */
    if (!s->ctx->tail_done)
        hm_launch_stream_rekey(s->ctx->stream, s->lkeys + s->llen, (uint64_t)m, (uint64_t)bucket << s->cb);
    HIPCHK(hipGetLastError());
    stream_appended(s, (uint64_t)m, bucket);
    return HM_OK;
}

/* a batch of several buckets: one grouped pass with the bucket as group */
static int stream_fold_grouped(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep, int64_t n)
{
    int64_t m = 0;
    int st;
    if (s->rcap < 2 * n + 1024) {
        const int64_t want = 2 * n + 1024;
        if ((st = stream_buf(s, s->rec, (size_t)want * 40))) return st;
        s->rcap = want;
    }
    for (;;) {
        st = grouped_impl(s->ctx, lat, lon, nullptr, nullptr, keep, (const uint32_t*)s->bids.p, n, s->zmin, s->zmax,
                          (int64_t*)s->rec.p, s->rcap, &m);
        if (st != HM_E_CAPACITY) break;
        const int64_t want = m + m / 4 + 1024;
        if ((st = stream_buf(s, s->rec, (size_t)want * 40))) return st;
        s->rcap = want;
    }
    if (st) return st;
    if ((st = stream_room(s, (uint64_t)m + 1))) return st;
    hipStream_t q = s->ctx->stream;
    HIPCHK(hipMemsetAsync(s->state + HMS_ST_EXOTIC, 0, 8, q));
    hm_launch_stream_convert(q, (const int64_t*)s->rec.p, (uint64_t)m, s->cb, s->lkeys + s->llen,
                             s->lcounts + s->llen, s->state);
    HIPCHK(hipGetLastError());
    if ((st = stream_sync_state(s))) return st;
    if (s->hstate[HMS_ST_EXOTIC]) return HM_E_EXOTIC;   /* checked before the cells join the log */
    stream_appended(s, (uint64_t)m);
    return HM_OK;
}

/* The several-bucket batch's runs (gathered by stream_fold_parts, the
 * points not kept last; at most HMS_PAR runs in all) counted at once, each by
 * its own context, HIP stream and host thread into its own scratch, then
 * copied to the log's tail in bucket order and keyed -- nothing joins the
 * log unless every run counted.  HM_FALLBACK: a run failed (the caller's
 * sequential path re-counts and reports the batch's first failing point). */
static int stream_fold_parts_par(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep, int64_t n,
                                 uint32_t nparts, const std::vector<uint64_t>& start, const std::vector<uint32_t>& hb)
{
    hm_ctx* ctx = s->ctx;
    hipStream_t q = ctx->stream;
    int st;
    for (int t = 0; t < HMS_PAR; t++) {
        if (s->pctx[t]) continue;
        hipStream_t pq = nullptr;
        HIPCHK(hipStreamCreateWithFlags(&pq, hipStreamNonBlocking));
        if ((st = hm_ctx_create(&s->pctx[t], ctx->device, pq))) {
            (void)hipStreamDestroy(pq);
            return st;
        }
    }
    for (int t = 0; t < HMS_PAR; t++) ctx_copy_tuning(s->pctx[t], ctx);   /* hm_ctx_tune of the stream's context */
    if (!s->pev) HIPCHK(hipEventCreateWithFlags(&s->pev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(s->pev, q));   /* the gathered runs are written */
    const uint32_t nall = nparts + 1;    /* + the points not kept (errors only) */
    std::vector<int64_t> m(nall, 0);
    std::vector<int> rc(nall, HM_OK);
    for (uint32_t j0 = 0; j0 < nall; j0 += HMS_PAR) {
        const uint32_t j1 = std::min<uint32_t>(nall, j0 + HMS_PAR);
        std::vector<std::thread> th;
        for (uint32_t j = j0; j < j1; j++) {
            const int t = (int)(j - j0);
            th.emplace_back([&, j, t]() {
                hm_ctx* c = s->pctx[t];
                (void)hipSetDevice(c->device);
                const uint64_t nj = (j < nparts ? start[j + 1] : (uint64_t)n) - start[j];
                if (!nj) return;
                if (hipStreamWaitEvent(c->stream, s->pev, 0) != hipSuccess) {
                    rc[j] = HM_E_HIP;
                    return;
                }
                const double* la = (const double*)s->plat.p + start[j];
                const double* lo = (const double*)s->plon.p + start[j];
                const uint8_t* kp = j < nparts ? nullptr : (const uint8_t*)s->pkeep.p;
                uint64_t cap = j < nparts ? 2 * nj + 1024 : 0;
                for (;;) {
                    if (cap && stream_buf(s, s->pk[t], cap * 8) != HM_OK) {
                        rc[j] = HM_E_NOMEM;
                        return;
                    }
                    if (cap && stream_buf(s, s->pc[t], cap * 8) != HM_OK) {
                        rc[j] = HM_E_NOMEM;
                        return;
                    }
                    int64_t mj = 0, nx = 0;
                    const int r = hm_count(c, la, lo, kp, (int64_t)nj, s->zmin, s->zmax,
                                           cap ? (uint64_t*)s->pk[t].p : nullptr, cap ? (uint64_t*)s->pc[t].p : nullptr,
                                           (int64_t)cap, &mj, nullptr, 0, &nx);
                    if (nx > 0) {
                        rc[j] = HM_E_EXOTIC;
                        return;
                    }
                    if (r == HM_E_CAPACITY && j < nparts) {
                        cap = (uint64_t)mj + (uint64_t)mj / 4 + 1024;
                        continue;
                    }
                    rc[j] = (r == HM_E_CAPACITY) ? HM_OK : r;   /* the unkept part has no cells */
                    m[j] = mj;
                    return;
                }
            });
        }
        for (auto& x : th) x.join();
        for (uint32_t j = j0; j < j1; j++)
            if (rc[j] == HM_E_EXOTIC) return HM_E_EXOTIC;
        for (uint32_t j = j0; j < j1; j++)
            if (rc[j] != HM_OK) return HM_FALLBACK;
        /* this group's cells to the tail, in bucket order */
        uint64_t need = 0;
        for (uint32_t j = j0; j < j1 && j < nparts; j++) need += (uint64_t)m[j];
        if ((st = stream_room(s, need + 1024))) return st;
        for (uint32_t j = j0; j < j1 && j < nparts; j++) {
            const int t = (int)(j - j0);
            if (!m[j]) continue;
            uint64_t* tk = s->lkeys + s->llen;
            HIPCHK(hipMemcpyAsync(tk, s->pk[t].p, (size_t)m[j] * 8, hipMemcpyDeviceToDevice, q));
            HIPCHK(hipMemcpyAsync(s->lcounts + s->llen, s->pc[t].p, (size_t)m[j] * 8, hipMemcpyDeviceToDevice, q));
            hm_launch_stream_rekey(q, tk, (uint64_t)m[j], (uint64_t)hb[j] << s->cb);
            HIPCHK(hipGetLastError());
            stream_appended(s, (uint64_t)m[j], &hb[j], 1);
        }
    }
    return HM_OK;
}

/* a batch of a few buckets: gathered into one run per bucket (+ one run of
 * the points not kept), one hm_count per run written at the log's tail, all
 * counted before the tail joins the log.  Errors: the batch is re-counted as
 * a whole so the reported point is the first failing one in input order, as
 * hm_count's. */
static int stream_fold_parts(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep, int64_t n,
                             uint32_t nparts)
{
    hm_ctx* ctx = s->ctx;
    hipStream_t q = ctx->stream;
    int st;
    std::vector<uint32_t> hb(nparts);
    std::vector<uint64_t> start(2 * (nparts + 2), 0);   /* starts | run sizes, then cursors */
    if ((st = stream_buf(s, s->pstart, (size_t)(nparts + 2) * 16))) return st;
    uint64_t* dstart = (uint64_t*)s->pstart.p;
    HmsScatterArgs a;
    a.lat = lat;
    a.lon = lon;
    a.keep = keep;
    a.bids = (const uint32_t*)s->bids.p;
    a.loc = s->bloc;
    a.n = (uint64_t)n;
    a.nparts = nparts;
    a.start = dstart;
    a.cursor = (unsigned long long*)(dstart + nparts + 2);
    hm_launch_stream_batch_list(q, s->blist, nparts, s->bloc);
    HIPCHK(hipMemsetAsync(a.cursor, 0, (size_t)(nparts + 2) * 8, q));
    hm_launch_stream_part_count(q, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(hb.data(), s->blist, nparts * 4, hipMemcpyDeviceToHost, q));
    HIPCHK(hipMemcpyAsync(start.data() + nparts + 2, a.cursor, (size_t)(nparts + 1) * 8, hipMemcpyDeviceToHost, q));
    HIPCHK(hm_sync(q));
    uint64_t kept = 0;
    for (uint32_t j = 0; j < nparts; j++) {
        start[j] = kept;
        kept += start[nparts + 2 + j];
    }
    start[nparts] = kept;
    start[nparts + 1] = (uint64_t)n;
    if (kept + start[2 * nparts + 2] != (uint64_t)n) return HM_E_HIP;   /* cannot happen */
    if ((st = stream_buf(s, s->plat, (size_t)n * 8)) || (st = stream_buf(s, s->plon, (size_t)n * 8))) return st;
    HIPCHK(hipMemcpyAsync(dstart, start.data(), (size_t)(nparts + 2) * 8, hipMemcpyHostToDevice, q));
    HIPCHK(hipMemsetAsync(a.cursor, 0, (size_t)(nparts + 2) * 8, q));
    a.lat_out = (double*)s->plat.p;
    a.lon_out = (double*)s->plon.p;
    hm_launch_stream_scatter(q, a);
    HIPCHK(hipGetLastError());
    const uint64_t nun = (uint64_t)n - kept;
    if (nun) {
        if ((st = stream_buf(s, s->pkeep, (size_t)nun))) return st;
        HIPCHK(hipMemsetAsync(s->pkeep.p, 0, nun, q));
    }
    if (nparts >= 2 && nparts + 1 <= HMS_PAR && s->par) {   /* one group: the batch stays atomic */
        st = stream_fold_parts_par(s, lat, lon, keep, n, nparts, start, hb);
        if (st != HM_FALLBACK) return st;
    }
    if ((st = stream_room(s, 2 * kept + 1024))) return st;
    for (;;) {
        uint64_t off = 0;
        bool grow = false;
        for (uint32_t j = 0; j <= nparts && !grow; j++) {
            const uint64_t nj = (j < nparts ? start[j + 1] : (uint64_t)n) - start[j];
            if (!nj) continue;
            int64_t m = 0, nx = 0;
            uint64_t* tk = s->lkeys + s->llen + off;
            uint64_t* tc = s->lcounts + s->llen + off;
            st = hm_count(ctx, (const double*)s->plat.p + start[j], (const double*)s->plon.p + start[j],
                          j < nparts ? nullptr : (const uint8_t*)s->pkeep.p, (int64_t)nj, s->zmin, s->zmax, tk, tc,
                          (int64_t)(s->lcap - s->llen - off), &m, nullptr, 0, &nx);
            /* the log's keys hold tiles inside [0, 2^z)^2 only (and with no
             * record buffer given, hm_count reports them as capacity) */
            if (nx > 0) return HM_E_EXOTIC;
            if (st == HM_E_CAPACITY) {
                if ((st = stream_room(s, (off + (uint64_t)m) * 5 / 4 + 1024))) return st;
                grow = true;
                break;
            }
            if (st != HM_OK) {
                /* the first failing point in input order */
                int64_t m2 = 0, nx2 = 0;
                const int st2 = hm_count(ctx, lat, lon, keep, n, s->zmin, s->zmax, nullptr, nullptr, 0, &m2, nullptr,
                                         0, &nx2);
                return st2 != HM_OK && st2 != HM_E_CAPACITY ? st2 : st;
            }
            if (j < nparts) {
                hm_launch_stream_rekey(q, tk, (uint64_t)m, (uint64_t)hb[j] << s->cb);
                HIPCHK(hipGetLastError());
                off += (uint64_t)m;
            }
        }
        if (grow) continue;
        /* several buckets' cells, each bucket's from one count */
        stream_appended(s, off, hb.data(), nparts);
        return HM_OK;
    }
}

extern "C" int hm_stream_create(hm_ctx* ctx, int zmin, int zmax, uint32_t base_hour, int64_t initial_cells,
                                int64_t max_buckets, hm_stream** out)
{
    if (!ctx || !out || zmin < 0 || zmax < zmin || zmax > HM_MAX_ZOOM || initial_cells < 0 || max_buckets < 0)
        return HM_E_ARG;
    *out = nullptr;
    HIPCHK(hipSetDevice(ctx->device));
    hm_stream* s = new hm_stream();
    s->ctx = ctx;
    s->zmin = zmin;
    s->zmax = zmax;
    s->base = base_hour;
    /* cell bits: the pyramid index of zooms 0..zmax, (4^(zmax+1) - 1)/3 values */
    const uint64_t ncell = ((1ull << (2 * (zmax + 1))) - 1) / 3;
    while ((1ull << s->cb) < ncell) s->cb++;
    const int bb = 64 - s->cb;   /* bucket bits: 21 at zmax 21 */
    uint64_t nb = 1024;
    const uint64_t want = max_buckets ? (uint64_t)max_buckets : (1ull << 20);
    while (nb < want + want / 4 && nb < (1ull << bb)) nb <<= 1;
    s->bk.mask = nb - 1;
    s->lcap = std::max<uint64_t>(1024, (uint64_t)initial_cells);
    if (const char* e = getenv("HM_STREAM_PAR")) s->par = atoi(e) != 0;
    if (const char* e = getenv("HM_STREAM_VMM")) s->vmm = atoi(e) != 0;
    int st = HM_OK;
    if (hipMalloc((void**)&s->state, HMS_ST_COUNT * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc((void**)&s->hstate, 2 * HMS_ST_COUNT * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void**)&s->bk.keys, nb * 8) != hipSuccess || hipMalloc((void**)&s->bflag, nb * 4) != hipSuccess ||
        hipMalloc((void**)&s->blist, nb * 4) != hipSuccess || hipMalloc((void**)&s->bloc, nb * 4) != hipSuccess ||
        stream_alloc2(s, s->lcap, &s->lkeys, &s->lcounts) != HM_OK) {
        (void)hipGetLastError();
        hm_stream_destroy(s);
        return HM_E_NOMEM;
    }
    st = hip_fail(hipMemsetAsync(s->state, 0, HMS_ST_COUNT * sizeof(unsigned long long), ctx->stream), "memset");
    if (st == HM_OK) {
        hm_launch_stream_fill(ctx->stream, s->bk.keys, nb, HMS_EMPTY);
        st = hip_fail(hipGetLastError(), "fill");
        if (st == HM_OK) st = hip_fail(hipMemsetAsync(s->bflag, 0, nb * 4, ctx->stream), "memset");
    }
    if (st == HM_OK) st = stream_sync_state(s);
    if (st) {
        hm_stream_destroy(s);
        return st;
    }
    *out = s;
    return HM_OK;
}

extern "C" int hm_stream_add(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep,
                             const uint32_t* hour, const uint32_t* group, int64_t n)
{
    if (!s || n < 0 || (n > 0 && (!lat || !lon)) || n >= (int64_t)0xFFFFFFF0ll) return HM_E_ARG;
    if (n == 0) return HM_OK;
    hm_ctx* ctx = s->ctx;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t q = ctx->stream;
    int st;
    /* buckets of the kept points (interned; a failing batch may leave unused
     * buckets behind, never cells) */
    /* reset BFULL, EXOTIC, BMM, NLIST, ERR in one copy */
    unsigned long long* init = s->hstate + HMS_ST_COUNT;
    init[0] = 0;                                    /* BFULL */
    init[1] = 0;                                    /* EXOTIC */
    init[2] = 0;                                    /* BMM */
    init[3] = 0;                                    /* NLIST */
    init[4] = ~0ull;                                /* ERR */
    HIPCHK(hipMemcpyAsync(s->state + HMS_ST_BFULL, init, 5 * 8, hipMemcpyHostToDevice, q));
    const bool per_point = group || hour;
    if (per_point && (st = stream_buf(s, s->bids, (size_t)n * 4))) return st;
    HmsBucketArgs a;
    a.group = group;
    a.hour = hour;
    a.keep = per_point ? keep : nullptr;
    a.n = per_point ? (uint64_t)n : 1;   /* neither: the one (no group, undated) bucket */
    a.base = s->base;
    a.buckets = s->bk;
    /* per-point bucket ids feed only the several-bucket paths: a batch
     * counted speculatively as one bucket skips writing them (and a batch
     * that turns out to hold several runs the pass again, below) */
    const bool spec = s->last_nparts <= 1;   /* the previous batch was one bucket */
    a.out = per_point && !spec ? (uint32_t*)s->bids.p : nullptr;
    if (++s->epoch == 0) s->epoch = 1;   /* wrapped: stale flags only cost an exchange */
    a.bflag = s->bflag;
    a.epoch = s->epoch;
    a.list = s->blist;
    a.state = s->state;
    a.err_word = s->state + HMS_ST_ERR;
    hm_launch_stream_buckets(q, a);
    hm_launch_stream_collect(q, s->bflag, s->bk.mask + 1, s->epoch, s->blist, s->state);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s->hstate, s->state, HMS_ST_COUNT * sizeof(unsigned long long), hipMemcpyDeviceToHost, q));
    /* the usual batch is one bucket: count it right away (into the log's
     * tail); the bucket pass's state arrives with the count's first
     * read-back.  Any other outcome drops the tail and takes the paths below
     * (which count again, so errors and their order are the same). */
    int64_t m1 = 0;
    const int st1 = spec ? stream_count_tail(s, lat, lon, keep, n, &m1) : HM_OK;
    HIPCHK(hm_sync(q));
    s->nbuckets = s->hstate[HMS_ST_BUCKETS];
    const uint32_t nparts = (uint32_t)s->hstate[HMS_ST_NLIST];
    s->last_nparts = nparts;
    const uint32_t lo = (uint32_t)s->hstate[HMS_ST_BMM];
    const unsigned long long e = s->hstate[HMS_ST_ERR];
    if (e != ~0ull) {
        ctx->last_err_index = (int64_t)(e >> 8);
        ctx->last_err_kind = (int)(e & 0xFF);
        return ctx->last_err_kind;
    }
    if (s->hstate[HMS_ST_BFULL]) return HM_E_CAPACITY;   /* max_buckets (group, hour) pairs */
    if (nparts <= 1) { /* one bucket (the usual time-ordered batch), or nothing kept */
        if (!spec && (st = stream_count_tail(s, lat, lon, keep, n, &m1))) return st;
        if (spec && st1) return st1;
        return stream_take_tail(s, m1, nparts ? lo : 0u);
    }
    if (spec && per_point) {
        /* the ids the speculative pass skipped (the buckets are interned and
         * listed already: the same epoch, nothing new to flag) */
        a.out = (uint32_t*)s->bids.p;
        hm_launch_stream_buckets(q, a);
        HIPCHK(hipGetLastError());
    }
    if (nparts <= HMS_MAX_PARTS) return stream_fold_parts(s, lat, lon, keep, n, nparts);
    return stream_fold_grouped(s, lat, lon, keep, n);
}

extern "C" int hm_stream_cells(hm_stream* s, int64_t* cells, int64_t* capacity, int64_t* buckets)
{
    if (!s) return HM_E_ARG;
    HIPCHK(hipSetDevice(s->ctx->device));
    int st;
    if (cells) {
        /* distinct (bucket, cell) pairs: the log compacted */
        if ((st = stream_compact(s))) return st;
        *cells = (int64_t)s->llen;
    }
    if (capacity) *capacity = (int64_t)s->lcap;
    if (buckets) {
        if ((st = stream_sync_state(s))) return st;
        *buckets = (int64_t)s->nbuckets;
    }
    return HM_OK;
}

extern "C" int hm_stream_rollup(hm_stream* s, int span, int merge_groups, int64_t select, uint64_t* keys_out,
                                uint64_t* counts_out, uint32_t* groups_out, uint32_t* periods_out, int64_t capacity,
                                int64_t* n_out)
{
    if (!s || !n_out || span < HM_SPAN_HOUR || span > HM_SPAN_ALLTIME || select < -1 || capacity < 0 ||
        (capacity > 0 && (!keys_out || !counts_out)))
        return HM_E_ARG;
    *n_out = 0;
    hm_ctx* ctx = s->ctx;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t q = ctx->stream;
    int st;
    if (s->llen == 0) return HM_OK;
    /* the log's cells of the rollup, re-keyed to label buckets */
    if ((st = stream_buf(s, s->rk, s->llen * 8)) || (st = stream_buf(s, s->rc, s->llen * 8))) return st;
    unsigned long long* cur = s->state + HMS_ST_CURSOR;
    HIPCHK(hipMemsetAsync(cur, 0, 8, q));
    HIPCHK(hipMemsetAsync(s->state + HMS_ST_BFULL, 0, 8, q));
    HmsRelabelArgs a;
    a.keys = s->lkeys;
    a.counts = s->lcounts;
    a.n = s->llen;
    a.buckets = s->bk;
    a.cb = s->cb;
    a.span = span;
    a.merge = merge_groups ? 1 : 0;
    a.base = s->base;
    a.select = select;
    a.keys_out = (uint64_t*)s->rk.p;
    a.counts_out = (uint64_t*)s->rc.p;
    a.cursor = cur;
    a.state = s->state;
    hm_launch_stream_relabel(q, a);
    HIPCHK(hipGetLastError());
    if ((st = stream_sync_state(s))) return st;
    if (s->hstate[HMS_ST_BFULL]) return HM_E_CAPACITY;   /* no bucket left for a rollup label */
    const uint64_t m = s->hstate[HMS_ST_CURSOR];
    if (m == 0) return HM_OK;
    /* equal label cells summed */
    if ((st = stream_buf(s, s->mk, m * 8)) || (st = stream_buf(s, s->mc, m * 8))) return st;
    int64_t nd = 0;
    if ((st = cells_merge(ctx, (const uint64_t*)s->rk.p, (const uint64_t*)s->rc.p, HM_CELLS_U64, (int64_t)m, nullptr, 0,
                          (uint64_t*)s->mk.p, (uint64_t*)s->mc.p, (int64_t)m, &nd)))
        return st;
    *n_out = nd;
    if (nd > capacity) return HM_E_CAPACITY;
    HmsEmitArgs e;
    e.keys = (const uint64_t*)s->mk.p;
    e.counts = (const uint64_t*)s->mc.p;
    e.n = (uint64_t)nd;
    e.buckets = s->bk;
    e.cb = s->cb;
    e.zmin = s->zmin;
    e.zmax = s->zmax;
    e.base = s->base;
    e.keys_out = keys_out;
    e.counts_out = counts_out;
    e.groups_out = groups_out;
    e.periods_out = periods_out;
    hm_launch_stream_emit(q, e);
    HIPCHK(hipGetLastError());
    return HM_OK;
}

extern "C" int hm_stream_extract(hm_stream* s, int64_t hour, uint64_t* keys_out, uint64_t* counts_out,
                                 uint32_t* hours_out, int64_t capacity, int64_t* n_out)
{
    if (!s) return HM_E_ARG;
    if (hour == HM_STREAM_ALLTIME)
        return hm_stream_rollup(s, HM_SPAN_ALLTIME, 1, -1, keys_out, counts_out, nullptr, nullptr, capacity, n_out);
    if (hour == HM_STREAM_EACH_HOUR)
        return hm_stream_rollup(s, HM_SPAN_HOUR, 1, -1, keys_out, counts_out, nullptr, hours_out, capacity, n_out);
    if (hour < (int64_t)s->base || hour - (int64_t)s->base >= HM_STREAM_MAX_HOURS) return HM_E_ARG;
    return hm_stream_rollup(s, HM_SPAN_HOUR, 1, hour, keys_out, counts_out, nullptr, hours_out, capacity, n_out);
}

extern "C" int hm_stream_destroy(hm_stream* s)
{
    if (!s) return HM_OK;
    premap_join(s);
    if (s->ctx) (void)hipSetDevice(s->ctx->device);
    if (s->ctx && s->ctx->stream) (void)hipStreamSynchronize(s->ctx->stream);
    for (void* p : {(void*)s->state, (void*)s->bk.keys, (void*)s->bflag, (void*)s->blist, (void*)s->bloc, s->bids.p,
                    s->rec.p, s->plat.p, s->plon.p, s->pkeep.p, s->pstart.p, s->pcnt.p, s->rk.p, s->rc.p, s->mk.p,
                    s->mc.p})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)s->lkeys, (void*)s->lcounts, (void*)s->akeys, (void*)s->acounts}) log_free(s, p);
    if (s->hstate) (void)hipHostFree(s->hstate);
    for (int t = 0; t < HMS_PAR; t++) {
        for (void* p : {s->pk[t].p, s->pc[t].p})
            if (p) (void)hipFree(p);
        if (s->pctx[t]) {
            hipStream_t q = s->pctx[t]->stream;
            hm_ctx_destroy(s->pctx[t]);
            if (q) (void)hipStreamDestroy(q);
        }
    }
    if (s->pev) (void)hipEventDestroy(s->pev);
    delete s;
    return HM_OK;
}
