/* The one host entry point of libheatmap_amd: hm_project_scalar, the
 * per-record form of hm_project for the reference's scalar callers
 * (Tile.row_from_latitude / column_from_longitude / tile_id_from_lat_long,
 * reference tile.py:9-21, called once per record by dataframe_loader's
 * flatMap, heatmap.py:27).  A device launch plus a synchronisation costs tens
 * of microseconds; CPython's math costs ~0.3 us a call.  This is the SAME
 * arithmetic the gfx950 kernels run -- csrc/hm_project.h (fast polynomial,
 * guard band, glibc 2.35 restated for the exact path, Payne-Hanek for huge
 * latitudes) -- compiled for the host by gcc with contraction off, so a
 * scalar call and the batched device call agree bit for bit
 * (tests/test_abi.py checks it against the reference's 30,093 KATs).  It is
 * not a fallback: every batched projection and every count runs on the
 * device only. */
#include "hm_project.h"

#include "../../include/heatmap_amd.h"

static const double HM_HOST_TAB[HM_YTAB_ROWS * HM_YTAB_STRIDE] = HM_YTAB_INIT;

int hm_project_scalar(double lat, double lon, int zoom, int64_t* row_col)
{
    if (!row_col || zoom < -30 || zoom > 30) return HM_E_ARG;
    int64_t r = 0, c = 0;
    int slow = 0;
    int st = hm_project_point(lat, lon, zoom, &r, &c, &slow, HM_HOST_TAB);
    if (st == HM_E_RANGE && hm_row(lat, zoom, &r, &slow, HM_HOST_TAB) == HM_OK) {
        /* the row projected (its errors come first); the column is beyond
         * int64: returned exactly as an integer-valued double's bits */
        const double f = floor((lon + 180.0) / 360.0 * hm_exp2i(zoom));
        c = (int64_t)hm_d2u(f);
        st = HM_BIGCOL;
    }
    const int good = st == HM_OK || st == HM_BIGCOL;
    row_col[0] = good ? r : 0;
    row_col[1] = good ? c : 0;
    return st;
}
