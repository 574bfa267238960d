/* heatmap_amd — C-ABI of the MI355X heatmap aggregation hot path.
 *
 * Drop-in boundary for timfpark/heatmap's hot path.
 * The reference has no FFI: its boundary is the set of Python callables Spark
 * invokes per record.  Each entry point below replaces one of them; the
 * ctypes binding a maintainer would add on the reference side is shown in
 * INTEGRATION.md, and heatmap_amd/tile.py + heatmap_amd/heatmap.py are that
 * binding, re-exposing the reference's own names.
 *
 *   hm_project      <- Tile.row_from_latitude + Tile.column_from_longitude
 *                      (reference tile.py:15-21), vectorised; the per-point
 *                      status reproduces tile_id_from_lat_long's exceptions
 *                      (tile.py:9-13: row is evaluated before column).
 *   hm_count        <- dataframe_loader projection at zoom MAX_ZOOM_LEVEL +
 *                      DETAIL_ZOOM_DELTA (heatmap.py:25-29) fused with the
 *                      per-zoom reduceByKey count pyramid of build_heatmaps
 *                      (heatmap.py:107-118, shuffle 1 at :111) for one user
 *                      group; the row layout (heatmap.py:79-90,120-129) is
 *                      assembled from these counts by heatmap_amd/heatmap.py.
 *   hm_count_tiles  <- the same pyramid starting from already projected tile
 *                      ids (build_heatmaps on locations whose "tileId" is a
 *                      zoom-zmax id, heatmap.py:60-61).
 *   hm_count_grouped <- the same counts per user group in one pass: the
 *                      user|alltime|tile keys of tile_id_timespans_mapper
 *                      (heatmap.py:64-75) with the group as a u32 column
 *                      (build_heatmaps_columnar's group:i32[N]).
 *   hm_last_error   <- the exception a Spark task would raise: first failing
 *                      point in input order and its kind.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (hipMalloc'd or torch CUDA
 *     tensors) owned by the caller; nothing is allocated across the boundary
 *     except the opaque context.
 *   - Work is enqueued on the context's HIP stream (hm_ctx_set_stream).  Calls
 *     that return results through host scalars (n_out, status) synchronise
 *     that stream before returning.
 *   - Return value: HM_OK or an HM_E_* status.  Per-point errors set the
 *     status of the first failing point (input order) and hm_last_error()
 *     reports its index.
 *   - Thread-compatible: one context per host thread / stream.
 *   - Every call fails loudly (HM_E_HIP) when no gfx950 device is present;
 *     there is no CPU fallback in this library.  (hm_project_scalar is the
 *     per-record host form of hm_project, not a fallback: it is what a
 *     one-point call always uses.)
 */
#ifndef HEATMAP_AMD_H
#define HEATMAP_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HM_ABI_VERSION 7

/* status / per-point error kinds */
#define HM_OK 0
#define HM_E_NAN 1       /* ValueError("cannot convert float NaN to integer")   tile.py:17,21 */
#define HM_E_DOMAIN 2    /* ValueError("math domain error")  tan(+-inf) / log(<=0), tile.py:17 */
#define HM_E_INF 3       /* OverflowError("cannot convert float infinity to integer") tile.py:21 */
#define HM_E_RANGE 8     /* representable by the reference but not by this path:
                            hm_count*: |col| >= 2^63 (hm_project returns those
                            columns, HM_BIGCOL), or (cells outside the square) a
                            zoom-0 tile row outside [-16, 16) / column outside
                            [-2^47, 2^47).  (Latitudes of any magnitude are
                            projected: glibc's Payne-Hanek reduction is
                            restated, csrc/hm_branred.h.) */
#define HM_E_EXOTIC 9    /* hm_stream_add only: a kept point whose zoom-zmax tile
                            lies outside [0, 2^zmax)^2 (|lat| > 85.0511..., or
                            lon outside [-180, 180)); the resident table's keys
                            hold in-square tiles, nothing was inserted.  The
                            host side (heatmap_amd/stream.py) then splits the
                            batch and counts those points with hm_count_grouped;
                            hm_count* bin such points directly. */
#define HM_BIGCOL 10     /* hm_project only, not an error: the point projected
                            and its column is beyond int64 (|lon| > ~1.6e15 deg
                            at zoom 21); col holds the column as the bits of
                            an IEEE double -- floor((lon + 180.0) / 360.0 *
                            2^z), integer-valued and exact, which the reference
                            prints as a Python int (tile.py:21) */
#define HM_E_ARG 16      /* bad argument (zoom range, null pointer, n < 0) */
#define HM_E_CAPACITY 17 /* output arrays too small; *n_out holds the size needed */
#define HM_E_HIP 18      /* HIP runtime error (no device, launch failure) */
#define HM_E_NOMEM 19    /* device allocation failed */
#define HM_E_WIDE 20     /* hm_cells_route with u32 counts: a count >= 2^32 (outputs complete otherwise) */

/* Output cell key of hm_count: zoom in bits 58..63, row in 29..57, col in 0..28.
 * Sorting keys sorts by (zoom, row, col). */
#define HM_KEY(z, r, c) (((uint64_t)(z) << 58) | ((uint64_t)(r) << 29) | (uint64_t)(c))
#define HM_KEY_ZOOM(k) ((int)((k) >> 58))
#define HM_KEY_ROW(k) ((int64_t)(((k) >> 29) & 0x1FFFFFFFull))
#define HM_KEY_COL(k) ((int64_t)((k) & 0x1FFFFFFFull))
#define HM_MAX_ZOOM 21   /* largest zmax accepted by hm_count* (level-1 keys fit u32) */

typedef struct hm_ctx hm_ctx;

int hm_abi_version(void);
const char* hm_status_string(int status);

/* device: HIP device ordinal; stream: hipStream_t (NULL = default stream). */
int hm_ctx_create(hm_ctx** out, int device, void* stream);
int hm_ctx_set_stream(hm_ctx* ctx, void* stream);
int hm_ctx_destroy(hm_ctx* ctx);

/* Plan tuning of one context (no effect on results, only on which kernels
 * count them).  hm_ctx_create reads each from the environment variable of the
 * same name once; this sets it afterwards.  HM_E_ARG for an unknown name.
 *   HM_SPREAD_MIN_KEYS  mean level-1 bucket (keys) of a flat histogram above
 *                       which levels 2.. take 3 zooms (default 2^19)
 *   HM_SPREAD_MIN_COLD  with hot tiles: mean level-1 bucket of the other
 *                       (cold) keys above which levels 2.. take 3 zooms and
 *                       the hot tiles join the last level (default off:
 *                       1e30; measured slower on the bench clouds)
 *   HM_SAMPLE_LOG2      level-1 regions are sized from ~2^this sampled
 *                       points (8..30; default 18)
 *   HM_RS_BIG_MIN       runs above which a level child is copied by every
 *                       wave of the run scan (default 2048)
 *   HM_HOT              1 (default): hot tiles skip the intermediate
 *                       partition passes; 0: off
 *   HM_HOT_INV_SHARE    a tile is hot with >= 1/this of the sampled points
 *                       (default 4096)
 *   HM_HOT_MIN_KEYS     ... and >= this many estimated points (default 65536)
 *   HM_RUN_SHARD_BITS   log2 run counters per level-2+ child (0..5; default
 *                       -1: 0 with hot tiles or the spread plan, else 4)
 * Returns the previous value in *old (if not NULL). */
int hm_ctx_tune(hm_ctx* ctx, const char* name, double value, double* old);

/* Project n points at one zoom (-30..30; negative zooms scale by 2^zoom, as
 * Python's 2 ** zoom does for Tile.parent_id at zoom 0, tile.py:60-61).  row/col: int64[n]; status: uint8[n]
 * (HM_OK or the point's error kind; row/col are 0 for failed points).
 * Returns HM_OK if every point projected, else the first failing point's kind.
 * Replaces Tile.row_from_latitude / column_from_longitude (tile.py:15-21). */
int hm_project(hm_ctx* ctx, const double* lat, const double* lon, int64_t n, int zoom,
               int64_t* row, int64_t* col, uint8_t* status);

/* One point, on the host: hm_project's arithmetic (csrc/hm_project.h, the
 * statements the kernels run) compiled for the CPU, for per-record callers
 * -- the reference's scalar Tile.row_from_latitude / column_from_longitude /
 * tile_id_from_lat_long (tile.py:9-21, one call per record at
 * heatmap.py:27) -- for which a launch and a synchronisation would cost
 * ~100x the reference's ~0.3 us.  row_col: int64[2] (host), row then column
 * (HM_BIGCOL: the column as an integer-valued double's bits).  Returns the
 * point's status exactly as hm_project's status[0]; HM_E_ARG for zoom outside
 * -30..30.  The only host computation in the library; needs no context. */
int hm_project_scalar(double lat, double lon, int zoom, int64_t* row_col);

/* Count points per (zoom, row, col) for every zoom in [zmin, zmax].
 * keep: uint8[n] or NULL (NULL = keep all); every point is projected (and
 * can fail) whether kept or not, as dataframe_loader does (heatmap.py:27-29).
 * Cells inside [0, 2^z)^2 go to keys_out/counts_out (HM_KEY layout, capacity
 * entries each, device); *n_out (host) receives how many there are.  The
 * reference also bins kept points outside that square (tile.py:17,21 do not
 * clamp: |lat| > 85.0511... gives negative rows, lon >= 180 columns >= 2^z);
 * their cells go to xcells_out as 4 int64 per cell (zoom, row, col, count),
 * xcapacity cells (device, may be NULL with xcapacity 0); *nx_out receives
 * how many.  Either count above its capacity -> HM_E_CAPACITY with both
 * sizes set.  Cell order is unspecified.
 * Replaces dataframe_loader + build_heatmaps' reduceByKey (heatmap.py:25-111). */
int hm_count(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep, int64_t n,
             int zmin, int zmax, uint64_t* keys_out, uint64_t* counts_out, int64_t capacity,
             int64_t* n_out, int64_t* xcells_out, int64_t xcapacity, int64_t* nx_out);

/* Same pyramid from zoom-zmax tile coordinates (int64 row/col). */
int hm_count_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint8_t* keep,
                   int64_t n, int zmin, int zmax, uint64_t* keys_out, uint64_t* counts_out,
                   int64_t capacity, int64_t* n_out, int64_t* xcells_out, int64_t xcapacity,
                   int64_t* nx_out);

/* Counts per (group, zoom, row, col), zooms [zmin, zmax], of the kept points
 * (keep as hm_count; group: uint32[n], device, or NULL = one group 0), in one
 * pass over the points.  cells_out: 5 int64 per cell (group, zoom, row, col,
 * count), capacity cells (device); *n_out = cells.  Rows/columns outside
 * [0, 2^z) are counted like the others.  Replaces the per-user keys of
 * tile_id_timespans_mapper (heatmap.py:64-75) + reduceByKey (:111). */
int hm_count_grouped(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep,
                     const uint32_t* group, int64_t n, int zmin, int zmax, int64_t* cells_out,
                     int64_t capacity, int64_t* n_out);

/* Same from zoom-zmax tile coordinates (int64 row/col). */
int hm_count_grouped_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint8_t* keep,
                           const uint32_t* group, int64_t n, int zmin, int zmax, int64_t* cells_out,
                           int64_t capacity, int64_t* n_out);

/* hm_count_grouped with a packed output of 16 B per record (SURVEY.md 8(d):
 * the output cell's 16 B): keys_out[i] = HM_KEY(zoom, row, col) and
 * gcounts_out[i] = group << 32 | count (u64 device arrays of capacity
 * entries).  Cells must lie inside [0, 2^z)^2 (every kept point's zoom-zmax
 * tile in the square): HM_E_EXOTIC otherwise, before any record is written
 * (use hm_count_grouped).  Records of one zoom are contiguous, zoom zmax
 * first, in no particular order inside a zoom. */
int hm_count_grouped_packed(hm_ctx* ctx, const double* lat, const double* lon, const uint8_t* keep,
                            const uint32_t* group, int64_t n, int zmin, int zmax, uint64_t* keys_out,
                            uint64_t* gcounts_out, int64_t capacity, int64_t* n_out);
int hm_count_grouped_packed_tiles(hm_ctx* ctx, const int64_t* row, const int64_t* col, const uint8_t* keep,
                                  const uint32_t* group, int64_t n, int zmin, int zmax, uint64_t* keys_out,
                                  uint64_t* gcounts_out, int64_t capacity, int64_t* n_out);

/* First failing point of the last call: index in input order (-1 if none)
 * and its HM_E_* kind. */
int hm_last_error(hm_ctx* ctx, int64_t* index, int* kind);

/* Diagnostics of the last hm_project/hm_count call: points resolved by the
 * bit-exact glibc-restating slow path (guard band / out-of-window), and the
 * per-stage device time in microseconds of the last hm_count (slots 0-4 are
 * timed for calls of >= 2^24 points only, 0 otherwise: the event records are
 * API calls, and a small call's time is the host's issue rate):
 *   [0] k_project_partition (projection + level-1 partition)
 *   [1] level-1 buckets, remaining partition levels, run scans and
 *       compactions (incl. host reads; contains [4])
 *   [2] final aggregation (k_aggregate, sparse/small/merged buckets)
 *   [3] k_pool levels   [4] the level >= 2 k_partition launches alone
 *   [5] level-1 re-runs (a sampled region size was too small; slot 0 then
 *       times the last run only)
 *   [6] hot tiles of the call (their points skipped levels 2..)
 *   [7] partition levels of the pipeline plan (0 if the call took the
 *       general path); 3 zooms per level for dense, evenly spread clouds */
int hm_last_stats(hm_ctx* ctx, int64_t* slow_points, double* stage_us, int n_stages);

/* Streaming: micro-batches folded into a heatmap resident in HBM (BASELINE
 * config 5).  The reference recomputes the pyramid per
 * Spark job (heatmap.py:152-158) and keys each bin by user group and timespan
 * label (heatmap.py:38-75, only 'alltime' live); a stream keeps per (group,
 * epoch hour) buckets (hour = unix_seconds / 3600, uint32) and answers every
 * label -- hour, day, month, year (UTC calendar), alltime -- as a rollup.
 *   hm_stream_create  zooms [zmin, zmax] (zmax <= HM_MAX_ZOOM); hours
 *                     base_hour .. base_hour + 2^28 - 1; initial_cells sizes
 *                     the cell log (batches append to it; it is compacted,
 *                     then grown, when full); max_buckets (0: 2^20) bounds
 *                     the distinct (group, hour) and rollup-label buckets.
 *   hm_stream_add     hm_count semantics per point (projection errors, keep);
 *                     hour: uint32[n] (device) or NULL (undated: alltime
 *                     only); group: uint32[n] (device, < 0xFFFFFFFE) or NULL
 *                     (no group).  One count pass per batch however many hours
 *                     and groups it holds; a failing batch changes no counts.
 *   hm_stream_rollup  cells of span HM_SPAN_* summed per (group, period), or
 *                     over every group (merge_groups: group = 0xFFFFFFFF);
 *                     select = -1 or the one period wanted.  Periods: epoch
 *                     hour, days since 1970-01-01, year*12 + month - 1, year,
 *                     0 (alltime).  groups_out/periods_out may be NULL.  Keys
 *                     in hm_count's layout, unspecified order; HM_E_CAPACITY
 *                     with *n_out = cells needed when capacity is too small.
 *   hm_stream_extract hour = HM_STREAM_ALLTIME, HM_STREAM_EACH_HOUR (hours_out
 *                     receives each cell's hour) or one epoch hour, summed
 *                     over groups (a rollup). */
#define HM_STREAM_ALLTIME (-1)
#define HM_STREAM_EACH_HOUR (-2)
#define HM_STREAM_MAX_HOURS (1 << 28)
#define HM_SPAN_HOUR 0
#define HM_SPAN_DAY 1
#define HM_SPAN_MONTH 2
#define HM_SPAN_YEAR 3
#define HM_SPAN_ALLTIME 4
typedef struct hm_stream hm_stream;
int hm_stream_create(hm_ctx* ctx, int zmin, int zmax, uint32_t base_hour, int64_t initial_cells, int64_t max_buckets,
                     hm_stream** out);
int hm_stream_add(hm_stream* s, const double* lat, const double* lon, const uint8_t* keep, const uint32_t* hour,
                  const uint32_t* group, int64_t n);
/* distinct (bucket, cell) pairs held (cells != NULL compacts the log: one
 * merge), the log's capacity in cells, and the buckets in use */
int hm_stream_cells(hm_stream* s, int64_t* cells, int64_t* capacity, int64_t* buckets);
int hm_stream_rollup(hm_stream* s, int span, int merge_groups, int64_t select, uint64_t* keys_out,
                     uint64_t* counts_out, uint32_t* groups_out, uint32_t* periods_out, int64_t capacity,
                     int64_t* n_out);
int hm_stream_extract(hm_stream* s, int64_t hour, uint64_t* keys_out, uint64_t* counts_out, uint32_t* hours_out,
                      int64_t capacity, int64_t* n_out);
int hm_stream_destroy(hm_stream* s);

/* Multi-GPU exchange of hm_count cells (one process per GPU; the collectives
 * are RCCL calls made by the caller, heatmap_amd/multigpu.py).  They replace
 * the reference's two shuffles, reduceByKey (heatmap.py:111) and groupByKey
 * (heatmap.py:112):
 *   hm_cells_route   cells of zoom <= dense_zmax are summed into grid (device
 *                    u64[hm_dense_grid_size(dense_zmax)], Morton order per zoom,
 *                    zeroed here; -1 = none) for an RCCL reduce; the others go
 *                    to keys_out/counts_out (n entries) grouped by owner rank
 *                    (a hash of the heatmap row key (zoom, row >> delta,
 *                    col >> delta), so each output row has one owner);
 *                    send_counts (host int64[nranks]) receives the group sizes
 *                    for an RCCL all-to-all.  nranks <= 64.  layout (below):
 *                    HM_CELLS_REC10 packs each cell into keys_out as one
 *                    10-byte record (counts_out unused), so ONE all-to-all of
 *                    10 B per cell moves keys and counts (16 B in round 2);
 *                    with u32 counts (REC10, U32) a count >= 2^32 -- or,
 *                    for REC10, a sparse key beyond 48 bits (zoom > 21, row
 *                    or column >= 2^21) -- returns
 *                    HM_E_WIDE after filling everything else (the caller's
 *                    ranks then agree to route again as HM_CELLS_U64: a rank's
 *                    cells count fewer points than it holds, so only shards
 *                    of >= 2^32 points can).
 *   hm_cells_merge   sum the counts of equal keys over n received cells in
 *                    `layout` (outputs: u64 keys, u64 counts);
 *   hm_cells_merge_runs  the same when the n cells are nruns consecutive runs
 *                    (host int64 sizes) each of distinct keys -- one rank's
 *                    cells each -- so only the key claim is atomic.
 *   hm_dense_cells   the non-empty cells of a (reduced) dense grid. */
int64_t hm_dense_grid_size(int dense_zmax);
/* exchanged cell layouts: keys u64[n] + counts u64[n]; keys u64[n] + counts
 * u32[n]; or n records of 10 bytes in `keys` (five u16: the key as zoom << 42
 * | row << 21 | col in 48 bits -- sparse zooms <= 21 -- and the u32 count;
 * the array 2-byte aligned) */
#define HM_CELLS_U64 8
#define HM_CELLS_U32 4
#define HM_CELLS_REC10 10
#define HM_CELLS_G12 12  /* hm_cells_route of grouped cells (hm_count_grouped_packed's keys and
                            group << 32 | count): owner by (group, heatmap row); keys_out = u64
                            merge keys group << 47 | zoom << 42 | row << 21 | col, counts_out =
                            u32 counts (12 B a cell); no dense grid (dense_zmax -1); HM_E_WIDE
                            when a group passes 2^17 or a cell passes zoom 21 (exchange those as
                            int64 records) */
int hm_cells_route(hm_ctx* ctx, const uint64_t* keys, const uint64_t* counts, int64_t n, int nranks, int delta,
                   int dense_zmax, uint64_t* grid, void* keys_out, void* counts_out, int layout,
                   int64_t* send_counts);
int hm_cells_merge(hm_ctx* ctx, const void* keys, const void* counts, int layout, int64_t n, uint64_t* keys_out,
                   uint64_t* counts_out, int64_t capacity, int64_t* n_out);
int hm_cells_merge_runs(hm_ctx* ctx, const void* keys, const void* counts, int layout, int64_t n,
                        const int64_t* runs, int nruns, uint64_t* keys_out, uint64_t* counts_out, int64_t capacity,
                        int64_t* n_out);
int hm_dense_cells(hm_ctx* ctx, const uint64_t* grid, int dense_zmax, uint64_t* keys_out, uint64_t* counts_out,
                   int64_t capacity, int64_t* n_out);
/* The exchange with the owner's first merge pass done by the sender (round 5):
 *   hm_cells_route_pieces  hm_cells_route whose owner groups are each ordered
 *                    by `bits` (0..7, nranks << bits <= 1024) top bits of the
 *                    merge key's hash (the key; for HM_CELLS_G12 the packed
 *                    merge key) -- 2^bits "pieces" per owner.  No host sync:
 *                    the sizes go to the DEVICE int64 array `sizes`, row o
 *                    (row stride `stride` >= 2 + 2^bits) = cells for owner o,
 *                    the wide flag (1: as HM_E_WIDE; every row), the owner's
 *                    2^bits piece sizes -- the row an RCCL all-to-all sends
 *                    to owner o; other columns are left alone.  Asynchronous;
 *                    HM_E_WIDE is never returned (it is in the rows).
 *                    self_rank >= 0: the groups leave in rank order with
 *                    owner self_rank's group moved to the end, so the others
 *                    are one contiguous all-to-all input with a zero own split
 *                    and the own group stays in place (-1: rank order).
 *   hm_cells_merge_pieces  the owner's merge of nruns senders' cells: run r
 *                    is a contiguous device array of records (REC10) or keys
 *                    key_src[r] with counts count_src[r] (u32 for U32/G12 or
 *                    u64 for U64 layouts; count_src NULL for REC10) holding its
 *                    2^bits pieces in digit order, pieces[r * 2^bits + d]
 *                    cells each (host int64); the runs need not be adjacent
 *                    (the sender's own cells can stay in its send buffer).
 *                    Outputs as hm_cells_merge.  Reference: heatmap.py:111-112. */
int hm_cells_route_pieces(hm_ctx* ctx, const uint64_t* keys, const uint64_t* counts, int64_t n, int nranks,
                          int delta, int dense_zmax, int bits, int self_rank, uint64_t* grid, void* keys_out,
                          void* counts_out, int layout, int64_t* sizes, int stride);
int hm_cells_merge_pieces(hm_ctx* ctx, int layout, int nruns, const void* const* key_src,
                          const void* const* count_src, const int64_t* pieces, int bits, uint64_t* keys_out,
                          uint64_t* counts_out, int64_t capacity, int64_t* n_out);

/* Row JSON text (heatmap_to_json, heatmap.py:92-95 via list_to_dict :120-126):
 * the bins of the rows, in row order (device arrays, n of them), are written
 * as  {"z_r_c": V.0, ...}  per row -- json.dumps of the bin dict with Python's
 * float repr of integer-valued counts below 1e16 (callers format others on
 * the host).  head/last: 1 on a row's first/last bin; offset: each bin's
 * first byte (an exclusive scan of the bin lengths the caller computed:
 * 1 + digits(z) + 1 + digits(r) + 1 + digits(c) + 3 + digits(v) + 2, plus
 * 1 for a first bin's "{" and 1 for a last bin's "}" or 2 for ", ").  z, r,
 * c >= 0; v >= 0 integers.  Asynchronous. */
int hm_format_bins(hm_ctx* ctx, const int64_t* zoom, const int64_t* row, const int64_t* col, const int64_t* value,
                   const uint8_t* head, const uint8_t* last, const int64_t* offset, int64_t n, uint8_t* text);

/* Row ids (heatmap.py:55,85-90):  <name>|<span>|<tz>_<tr>_<tc>  per row, the
 * name and span texts taken from byte blobs by index (names + name_off[label],
 * name_off[label + 1] - name_off[label] bytes; likewise spans).  offset: each
 * id's first byte (an exclusive scan of the id lengths the caller computed:
 * name + 1 + span + 1 + digits(tz) + 1 + digits(tr) + 1 + digits(tc)).
 * tz, tr, tc >= 0.  Asynchronous. */
int hm_format_ids(hm_ctx* ctx, const uint8_t* names, const int64_t* name_off, const int64_t* label,
                  const uint8_t* spans, const int64_t* span_off, const int64_t* span, const int64_t* tz,
                  const int64_t* tr, const int64_t* tc, const int64_t* offset, int64_t n, uint8_t* text);

/* Benchmark/test utility, not part of the reference boundary: fill lat/lon
 * (device) with points start..start+n-1 of a synthetic cloud, bit-identical
 * to heatmap_amd/synth.py.  kind: 0 uniform, 1 hotspots (table = device
 * double[4k]: centre lat, centre lon, sigma, Zipf cdf), 2 skew.  Asynchronous. */
#define HM_SYNTH_UNIFORM 0
#define HM_SYNTH_HOTSPOTS 1
#define HM_SYNTH_SKEW 2
int hm_synth(hm_ctx* ctx, int kind, uint64_t seed, int64_t start, int64_t n, double* lat, double* lon,
             const double* table, int k);

/* Benchmark utility, not part of the reference boundary: read two device
 * arrays of bytes_each bytes (a multiple of 16) once with 16-B loads -- the
 * access shape of hm_count's level-1 kernel over lat/lon, with none of its
 * arithmetic -- as bench.py's measured HBM read peak.  sink: device uint64_t
 * array of 4096 words (written only on an improbable checksum).  Asynchronous. */
int hm_bench_read(hm_ctx* ctx, const void* a, const void* b, int64_t bytes_each, uint64_t* sink);

#ifdef __cplusplus
}
#endif

#endif
