/*
 * svtme_oracle.c — TEST INFRASTRUCTURE ONLY: CPU oracle of the open-loop ME path.
 *
 * A from-scratch C restatement of the reference's per-SB open-loop motion
 * estimation (ScuffleCloud/SVT-AV1-mirror, Source/Lib/Codec/motion_estimation.c,
 * snapshot 2025-05-23). Every function cites the reference lines it follows.
 * It is pinned bit-exactly against the reference itself (oracle/_ref, built from
 * /root/reference by oracle/Makefile) by tests/test_oracle_vs_ref.py and by the
 * committed golden fixtures in tests/golden/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product (libsvtme.so) never links or calls it.
 *
 * Integer semantics follow the reference exactly: int16 search-area arithmetic,
 * uint32 wrap-around in the 8x8-variance and pruning expressions, strict `<`
 * raster-order argmins.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "svtme_oracle.h"

#define MAX_U32 0xFFFFFFFFu
#define ABS(a) ((a) < 0 ? -(a) : (a))
#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))

/* ---------------------------------------------------------------------------
 * Tables (motion_estimation.h:100-117, motion_estimation.c:2520-2531)
 * ------------------------------------------------------------------------- */
static const uint8_t ora_tab8x8[64] = {0,  1,  4,  5,  16, 17, 20, 21, 2,  3,  6,  7,  18, 19, 22, 23,
                                       8,  9,  12, 13, 24, 25, 28, 29, 10, 11, 14, 15, 26, 27, 30, 31,
                                       32, 33, 36, 37, 48, 49, 52, 53, 34, 35, 38, 39, 50, 51, 54, 55,
                                       40, 41, 44, 45, 56, 57, 60, 61, 42, 43, 46, 47, 58, 59, 62, 63};
static const uint8_t ora_z_to_raster[85] = {
    0,  1,  2,  3,  4,  5,  6,  9,  10, 7,  8,  11, 12, 13, 14, 17, 18, 15, 16, 19, 20, 21,
    22, 29, 30, 23, 24, 31, 32, 37, 38, 45, 46, 39, 40, 47, 48, 25, 26, 33, 34, 27, 28, 35,
    36, 41, 42, 49, 50, 43, 44, 51, 52, 53, 54, 61, 62, 55, 56, 63, 64, 69, 70, 77, 78, 71,
    72, 79, 80, 57, 58, 65, 66, 59, 60, 67, 68, 73, 74, 81, 82, 75, 76, 83, 84};

/* ---------------------------------------------------------------------------
 * Kernels (C_DEFAULT/compute_sad_c.c)
 * ------------------------------------------------------------------------- */
/* absolute differences the reference's searches evaluate (every SAD of the
 * path goes through ora_nxm_sad): bench.py's VALU-SAD roof counts the real
 * work of the benched job with it */
static __thread uint64_t t_absdiff;
static uint64_t g_absdiff;

/* compute_sad_c.c:20-37 */
static uint32_t ora_nxm_sad(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                            uint32_t height, uint32_t width) {
    uint32_t sad = 0;
    t_absdiff += (uint64_t)height * width;
    for (uint32_t r = 0; r < height; r++, src += src_stride, ref += ref_stride)
        for (uint32_t c = 0; c < width; c++) sad += src[c] > ref[c] ? src[c] - ref[c] : ref[c] - src[c];
    return sad;
}

/* compute_sad_c.c:58-101: exhaustive block SAD, strict-< raster argmin,
 * best initialised to 0xffffff, centres untouched if nothing beats it. */
static void ora_sad_loop(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                         uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_center,
                         int16_t *y_center, uint32_t src_stride_raw, uint8_t skip_search_line, int16_t sa_w,
                         int16_t sa_h) {
    *best_sad = 0xffffff;
    const int skip = block_width == 16 && block_height <= 16 && skip_search_line;
    for (int16_t ys = 0; ys < sa_h; ys++) {
        const uint8_t *row = ref + (size_t)ys * src_stride_raw;
        if (skip && (ys & 1) == 0)
            continue;
        for (int16_t xs = 0; xs < sa_w; xs++) {
            const uint32_t sad = ora_nxm_sad(src, src_stride, row + xs, ref_stride, block_height, block_width);
            if (sad < *best_sad) {
                *best_sad = sad;
                *x_center = xs;
                *y_center = ys;
            }
        }
    }
}

/* ---------------------------------------------------------------------------
 * Per-SB state: the MeContext fields the open-loop path reads or writes
 * ------------------------------------------------------------------------- */
typedef struct OraPlane {
    const uint8_t *buf; /* allocation start (padding included) */
    int32_t stride, width, height, org;
} OraPlane;

typedef struct OraSearchInfo {
    uint16_t sa_w, sa_h;
    int16_t col, row;
    uint64_t sad;
    uint8_t valid;
} OraSearchInfo;

typedef struct OraSearchResults {
    int16_t hme_sc_x, hme_sc_y;
    uint64_t hme_sad;
    uint8_t do_ref;
} OraSearchResults;

typedef struct OraCtx {
    const svtme_job *job;
    const svtme_controls *c;
    OraPlane ref[2][4][3]; /* [list][ref][level: 0 full, 1 quarter, 2 sixteenth] */
    const uint8_t *src, *qsrc, *ssrc;
    uint32_t src_stride, qsrc_stride, ssrc_stride;
    uint32_t b64_w, b64_h;
    uint8_t num_lists, num_refs[2];
    svtme_area_minmax hme_l0_sa; /* mutable copy (mutated/restored per ref) */
    OraSearchResults sr[2][4];
    uint32_t reduce_me_sr_divisor[2][4];
    uint32_t zz_sad[2][4];
    OraSearchInfo prehme[2][4][2];
    uint8_t performed_phme[2][4][2];
    int16_t l0x[2][4][2][2], l0y[2][4][2][2], l1x[2][4][2][2], l1y[2][4][2][2], l2x[2][4][2][2], l2y[2][4][2][2];
    uint64_t l0sad[2][4][2][2], l1sad[2][4][2][2], l2sad[2][4][2][2];
    uint32_t best_sad[2][4][85];
    uint32_t best_mv[2][4][85];
    uint32_t me_distortion[85];
} OraCtx;

/* motion_estimation.c:1239-1243 */
static uint16_t ora_scaled_dist(uint16_t dist) {
    uint8_t round_up = ((dist % 8) == 0) ? 0 : 1;
    return (uint16_t)(((dist * 5) / 8) + round_up);
}

/* motion_estimation.c:1232-1234 */
static uint16_t ora_dist(const OraCtx *x, int l, int r) {
    int64_t d = (int64_t)x->job->picture_number - (int64_t)x->job->ref_picture_number[l][r];
    return (uint16_t)(int16_t)(d < 0 ? -d : d);
}

/* ---------------------------------------------------------------------------
 * Zero-zero SAD (motion_estimation.c:1667-1689, 2382-2437)
 * ------------------------------------------------------------------------- */
static uint32_t ora_get_zz_sad(const OraCtx *x, const OraPlane *p, int16_t org_x, int16_t org_y) {
    const uint8_t *r = p->buf + (size_t)(p->org + org_y) * p->stride + p->org + org_x;
    uint32_t zz = ora_nxm_sad(x->src, x->src_stride << 1, r, (uint32_t)p->stride << 1, x->b64_h >> 1, x->b64_w);
    return zz << 1;
}

static void ora_init_zz_sad(OraCtx *x, int16_t org_x, int16_t org_y) {
    const svtme_controls *c = x->c;
    const svtme_job *job    = x->job;
    uint32_t best_zz        = MAX_U32;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            if (job->temporal_layer_index > 0 || l == 0) {
                uint32_t zz = ora_get_zz_sad(x, &x->ref[l][r][0], org_x, org_y);
                zz          = (zz * 64 * 64) / (x->b64_w * x->b64_h);
                x->zz_sad[l][r] = zz;
                best_zz         = MIN(best_zz, zz);
            }
        }
    const uint32_t zz_th = c->zz_sad_th;
    if (job->temporal_layer_index > 0 && best_zz < zz_th) {
        for (int l = 0; l < x->num_lists; l++)
            for (int r = 0; r < x->num_refs[l]; r++) {
                if (r == 0)
                    continue;
                const uint32_t pct = c->zz_sad_pct;
                if ((uint32_t)((x->zz_sad[l][r] - best_zz) * 100u) > (uint32_t)(pct * best_zz))
                    x->sr[l][r].do_ref = 0;
            }
    }
    if (c->me_safe_limit_zz_th) {
        int safe = job->hierarchical_levels > 0 && x->num_lists == 2 &&
            job->temporal_layer_index >= job->hierarchical_levels && job->similar_brightness_refs &&
            x->zz_sad[0][0] < c->me_safe_limit_zz_th && x->zz_sad[1][0] < c->me_safe_limit_zz_th;
        for (int l = 0; l < x->num_lists; l++)
            for (int r = 0; r < x->num_refs[l]; r++)
                if (safe && r > 0)
                    x->sr[l][r].do_ref = 0;
    }
}

/* ---------------------------------------------------------------------------
 * Pre-HME (motion_estimation.c:1568-1666, 1693-1796)
 * ------------------------------------------------------------------------- */
static void ora_prehme_core(OraCtx *x, int16_t org_x, int16_t org_y, uint32_t sb_w, uint32_t sb_h, const OraPlane *p,
                            OraSearchInfo *d) {
    const int16_t pad_w = (int16_t)(p->org - 1), pad_h = (int16_t)(p->org - 1);
    const int16_t pw = (int16_t)p->width, ph = (int16_t)p->height;
    int16_t sa_w = (int16_t)d->sa_w, sa_h = (int16_t)d->sa_h;
    int16_t ox   = -(int16_t)(sa_w >> 1);
    int16_t oy   = -(int16_t)(sa_h >> 1);
    ox   = ((org_x + ox) < -pad_w) ? -pad_w - org_x : ox;
    sa_w = ((org_x + ox) < -pad_w) ? sa_w - (-pad_w - (org_x + ox)) : sa_w;
    ox   = ((org_x + ox) > pw - 1) ? ox - ((org_x + ox) - (pw - 1)) : ox;
    sa_w = ((org_x + ox + sa_w) > pw) ? MAX(1, sa_w - ((org_x + ox + sa_w) - pw)) : sa_w;
    oy   = ((org_y + oy) < -pad_h) ? -pad_h - org_y : oy;
    sa_h = ((org_y + oy) < -pad_h) ? sa_h - (-pad_h - (org_y + oy)) : sa_h;
    oy   = ((org_y + oy) > ph - 1) ? oy - ((org_y + oy) - (ph - 1)) : oy;
    sa_h = (org_y + oy + sa_h > ph) ? MAX(1, sa_h - ((org_y + oy + sa_h) - ph)) : sa_h;

    const int16_t xtl = (int16_t)(p->org + org_x) + ox;
    const int16_t ytl = (int16_t)(p->org + org_y) + oy;
    const uint32_t idx = (uint32_t)(xtl + ytl * p->stride);
    const int full     = x->c->hme_search_method == SVTME_FULL_SAD_SEARCH;
    ora_sad_loop(x->ssrc, full ? x->ssrc_stride : x->ssrc_stride * 2, p->buf + idx,
                 full ? (uint32_t)p->stride : (uint32_t)p->stride * 2, full ? sb_h : sb_h >> 1, sb_w, &d->sad, &d->col,
                 &d->row, (uint32_t)p->stride, x->c->prehme_skip_search_line, sa_w, sa_h);
    d->sad = full ? d->sad : d->sad * 2;
    d->col = (int16_t)(d->col + ox);
    d->col = (int16_t)(d->col * 4);
    d->row = (int16_t)(d->row + oy);
    d->row = (int16_t)(d->row * 4);
    d->valid = 1;
}

static int ora_prehme_early_exit(OraCtx *x, int l, int r, int s) {
    OraSearchInfo *d = &x->prehme[l][r][s];
    if (x->c->me_early_exit_th) {
        if (x->zz_sad[l][r] < x->c->me_early_exit_th) {
            d->col = d->row = 0;
            d->sad          = 0;
            d->valid        = 1;
            return 1;
        }
    }
    if (x->c->prehme_l1_early_exit) {
        const OraSearchInfo *z = &x->prehme[0][r][s];
        if (l == 1 && z->valid && ((z->sad < (32 * 32)) || ((ABS(z->col) < 16) && (ABS(z->row) < 16)))) {
            d->col   = (int16_t)-z->col;
            d->row   = (int16_t)-z->row;
            d->sad   = z->sad;
            d->valid = 1;
            return 1;
        }
    }
    return 0;
}

static void ora_prehme_b64(OraCtx *x, uint32_t org_x, uint32_t org_y) {
    const svtme_controls *c = x->c;
    const svtme_job *job    = x->job;
    uint32_t best_sad       = MAX_U32;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            const uint16_t dist = ora_dist(x, l, r);
            if (job->temporal_layer_index > 0 || l == 0) {
                const uint32_t f = ora_scaled_dist(dist);
                for (int s = 0; s < 2; s++) {
                    if (ora_prehme_early_exit(x, l, r, s))
                        continue;
                    OraSearchInfo *d = &x->prehme[l][r][s];
                    if (!x->sr[l][r].do_ref) {
                        d->col = d->row = 0;
                        d->sad          = MAX_U32;
                        continue;
                    }
                    d->sa_w = (uint16_t)MIN(c->prehme_sa_cfg[s].sa_min.width * f, c->prehme_sa_cfg[s].sa_max.width);
                    d->sa_h = (uint16_t)MIN(c->prehme_sa_cfg[s].sa_min.height * f, c->prehme_sa_cfg[s].sa_max.height);
                    ora_prehme_core(x, (int16_t)(((int16_t)org_x) >> 2), (int16_t)(((int16_t)org_y) >> 2),
                                    x->b64_w >> 2, x->b64_h >> 2, &x->ref[l][r][2], d);
                    x->performed_phme[l][r][s] = 1;
                }
                uint32_t min_sad = (uint32_t)MIN(x->prehme[l][r][0].sad, x->prehme[l][r][1].sad);
                best_sad         = MIN(best_sad, min_sad);
            } else {
                for (int s = 0; s < 2; s++) {
                    x->prehme[1][r][s].col = (int16_t)-x->prehme[0][r][s].col;
                    x->prehme[1][r][s].row = (int16_t)-x->prehme[0][r][s].row;
                    x->prehme[1][r][s].sad = x->prehme[0][r][s].sad;
                }
            }
        }
    if (job->temporal_layer_index > 0 && best_sad < c->phme_sad_th) {
        for (int l = 0; l < x->num_lists; l++)
            for (int r = 0; r < x->num_refs[l]; r++) {
                if (!x->sr[l][r].do_ref)
                    continue;
                if (r == 0)
                    continue;
                const uint32_t th  = c->phme_sad_pct;
                uint32_t       psad = (uint32_t)MIN(x->prehme[l][r][0].sad, x->prehme[l][r][1].sad);
                if ((uint32_t)((psad - best_sad) * 100u) > (uint32_t)(th * best_sad))
                    x->sr[l][r].do_ref = 0;
            }
    }
}

/* ---------------------------------------------------------------------------
 * HME level 0/1/2 (motion_estimation.c:820-1113, 1800-2177)
 * ------------------------------------------------------------------------- */
static void ora_hme_level_0(OraCtx *x, int16_t org_x, int16_t org_y, uint32_t bw, uint32_t bh, int16_t sa_w,
                            int16_t sa_h, const OraPlane *p, uint32_t sr_w, uint32_t sr_h, uint64_t *best_sad,
                            int16_t *scx, int16_t *scy) {
    sa_w = (int16_t)((sa_w + 7) & ~0x07);
    const int16_t pad_w = (int16_t)(p->org - 1), pad_h = (int16_t)(p->org - 1);
    const int16_t pw = (int16_t)p->width, ph = (int16_t)p->height;
    int16_t xd = (int16_t)(sa_w * sr_w);
    int16_t yd = (int16_t)(sa_h * sr_h);
    int16_t ox = (int16_t)(-(int16_t)((sa_w * x->c->num_hme_sa_w) >> 1) + xd);
    int16_t oy = (int16_t)(-(int16_t)((sa_h * x->c->num_hme_sa_h) >> 1) + yd);
    if ((org_x + ox) < -pad_w) {
        ox   = -pad_w - org_x;
        sa_w = (int16_t)(sa_w - (-pad_w - (org_x + ox)));
    }
    if ((org_x + ox) > pw - 1)
        ox = (int16_t)(ox - ((org_x + ox) - (pw - 1)));
    if ((org_x + ox + sa_w) > pw)
        sa_w = (int16_t)MAX(1, sa_w - ((org_x + ox + sa_w) - pw));
    sa_w = (sa_w < 8) ? sa_w : (int16_t)(sa_w & ~0x07);
    if ((org_y + oy) < -pad_h) {
        oy   = -pad_h - org_y;
        sa_h = (int16_t)(sa_h - (-pad_h - (org_y + oy)));
    }
    if ((org_y + oy) > ph - 1)
        oy = (int16_t)(oy - ((org_y + oy) - (ph - 1)));
    if ((org_y + oy + sa_h) > ph)
        sa_h = (int16_t)MAX(1, sa_h - ((org_y + oy + sa_h) - ph));

    const int16_t xtl  = (int16_t)((int16_t)p->org + org_x) + ox;
    const int16_t ytl  = (int16_t)((int16_t)p->org + org_y) + oy;
    const uint32_t idx = (uint32_t)(xtl + ytl * p->stride);
    const int full     = x->c->hme_search_method == SVTME_FULL_SAD_SEARCH;
    ora_sad_loop(x->ssrc, full ? x->ssrc_stride : x->ssrc_stride * 2, p->buf + idx,
                 full ? (uint32_t)p->stride : (uint32_t)p->stride * 2, full ? bh : bh >> 1, bw, best_sad, scx, scy,
                 (uint32_t)p->stride, 0, sa_w, sa_h);
    *best_sad = full ? *best_sad : *best_sad * 2;
    *scx      = (int16_t)(*scx + ox);
    *scx      = (int16_t)(*scx * 4);
    *scy      = (int16_t)(*scy + oy);
    *scy      = (int16_t)(*scy * 4);
}

/* levels 1 (quarter, pad = org-1, x2) and 2 (full, pad 63, x1) share one shape */
static void ora_hme_refine(OraCtx *x, int level, int16_t org_x, int16_t org_y, uint32_t bw, uint32_t bh,
                           const OraPlane *p, int16_t sa_w, int16_t sa_h, int16_t scx_in, int16_t scy_in,
                           uint64_t *best_sad, int16_t *scx, int16_t *scy) {
    sa_w = (int16_t)((sa_w + 7) & ~0x07);
    const int16_t pad_w = level == 1 ? (int16_t)(p->org - 1) : (int16_t)(64 - 1);
    const int16_t pad_h = pad_w;
    const int16_t pw = (int16_t)p->width, ph = (int16_t)p->height;
    int16_t ox = (int16_t)(-(sa_w >> 1) + scx_in);
    int16_t oy = (int16_t)(-(sa_h >> 1) + scy_in);
    if ((org_x + ox) < -pad_w) {
        ox   = -pad_w - org_x;
        sa_w = (int16_t)(sa_w - (-pad_w - (org_x + ox)));
    }
    if ((org_x + ox) > pw - 1)
        ox = (int16_t)(ox - ((org_x + ox) - (pw - 1)));
    if ((org_x + ox + sa_w) > pw)
        sa_w = (int16_t)MAX(1, sa_w - ((org_x + ox + sa_w) - pw));
    sa_w = (sa_w < 8) ? sa_w : (int16_t)(sa_w & ~0x07);
    if ((org_y + oy) < -pad_h) {
        oy   = -pad_h - org_y;
        sa_h = (int16_t)(sa_h - (-pad_h - (org_y + oy)));
    }
    if ((org_y + oy) > ph - 1)
        oy = (int16_t)(oy - ((org_y + oy) - (ph - 1)));
    if ((org_y + oy + sa_h) > ph)
        sa_h = (int16_t)MAX(1, sa_h - ((org_y + oy + sa_h) - ph));

    const int16_t xtl  = (int16_t)((int16_t)p->org + org_x) + ox;
    const int16_t ytl  = (int16_t)((int16_t)p->org + org_y) + oy;
    const uint32_t idx = (uint32_t)(xtl + ytl * p->stride);
    const int full     = x->c->hme_search_method == SVTME_FULL_SAD_SEARCH;
    const uint8_t *src = level == 1 ? x->qsrc : x->src;
    const uint32_t ss  = level == 1 ? x->qsrc_stride : x->src_stride;
    ora_sad_loop(src, full ? ss : ss * 2, p->buf + idx, full ? (uint32_t)p->stride : (uint32_t)p->stride * 2,
                 full ? bh : bh >> 1, bw, best_sad, scx, scy, (uint32_t)p->stride, 0, sa_w, sa_h);
    *best_sad = full ? *best_sad : *best_sad * 2;
    *scx      = (int16_t)(*scx + ox);
    *scy      = (int16_t)(*scy + oy);
    if (level == 1) {
        *scx = (int16_t)(*scx * 2);
        *scy = (int16_t)(*scy * 2);
    }
}

static void ora_hme_l0_search_area(OraCtx *x, int l, int r, uint16_t dist, int16_t *sa_w, int16_t *sa_h) {
    const svtme_controls *c = x->c;
    if (c->enable_me_sr_adjustment && c->distance_based_hme_resizing) {
        uint8_t is_hor = 1, is_ver = 1, is_still = 0;
        if (c->reduce_hme_l0_sr_th_min && c->reduce_hme_l0_sr_th_max) {
            if (l || r) {
                int16_t mvx = x->l0x[0][0][0][0], mvy = x->l0y[0][0][0][0];
                is_ver   = (ABS(mvx) < c->reduce_hme_l0_sr_th_min) && (ABS(mvy) > c->reduce_hme_l0_sr_th_max);
                is_hor   = (ABS(mvx) > c->reduce_hme_l0_sr_th_max) && (ABS(mvy) < c->reduce_hme_l0_sr_th_min);
                is_still = (ABS(mvx) < (c->reduce_hme_l0_sr_th_min * 3)) && (ABS(mvy) < (c->reduce_hme_l0_sr_th_min * 3));
            }
        }
        uint8_t xo = 1, yo = 1;
        if (!is_ver)
            yo = 2;
        if (!is_hor)
            xo = 2;
        if (c->enable_me_sr_adjustment == 2 && is_still)
            xo = yo = 4;
        x->hme_l0_sa.sa_min.width  = (uint16_t)(x->hme_l0_sa.sa_min.width / (xo + r));
        x->hme_l0_sa.sa_min.height = (uint16_t)(x->hme_l0_sa.sa_min.height / (yo + r));
        x->hme_l0_sa.sa_max.width  = (uint16_t)(x->hme_l0_sa.sa_max.width / (xo + r));
        x->hme_l0_sa.sa_max.height = (uint16_t)(x->hme_l0_sa.sa_max.height / (yo + r));
    }
    const int32_t f = ora_scaled_dist(dist);
    int16_t w       = (int16_t)(x->hme_l0_sa.sa_min.width / c->num_hme_sa_w);
    w = (int16_t)MIN((((w * f) + 15) & ~0x0F), (((x->hme_l0_sa.sa_max.width / c->num_hme_sa_w) + 15) & ~0x0F));
    int16_t h = (int16_t)(x->hme_l0_sa.sa_min.height / c->num_hme_sa_h);
    h         = (int16_t)MIN((h * f), x->hme_l0_sa.sa_max.height / c->num_hme_sa_h);
    *sa_w     = w;
    *sa_h     = h;
}

static void ora_hme_level0_b64(OraCtx *x, uint32_t org_x, uint32_t org_y) {
    const svtme_controls *c = x->c;
    const svtme_job *job    = x->job;
    const svtme_area_minmax base = x->hme_l0_sa;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            if (c->me_early_exit_th && x->zz_sad[l][r] < (c->me_early_exit_th >> 2)) {
                for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                    for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                        x->l0x[l][r][sx][sy] = x->l0y[l][r][sx][sy] = 0;
                        x->l0sad[l][r][sx][sy]                      = 0;
                    }
                continue;
            }
            if (c->prev_me_stage_based_exit_th) {
                int s = x->prehme[l][r][0].sad <= x->prehme[l][r][1].sad ? 0 : 1;
                if (x->performed_phme[l][r][s] && x->prehme[l][r][s].sad < (c->prev_me_stage_based_exit_th >> 4)) {
                    for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                        for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                            x->l0x[l][r][sx][sy]   = x->prehme[l][r][s].col;
                            x->l0y[l][r][sx][sy]   = x->prehme[l][r][s].row;
                            x->l0sad[l][r][sx][sy] = x->prehme[l][r][s].sad;
                        }
                    continue;
                }
            }
            if (!x->sr[l][r].do_ref) {
                for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                    for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                        x->l0x[l][r][sx][sy] = x->l0y[l][r][sx][sy] = 0;
                        x->l0sad[l][r][sx][sy]                      = MAX_U32;
                    }
                continue;
            }
            const uint16_t dist = ora_dist(x, l, r);
            if (job->temporal_layer_index > 0 || l == 0) {
                int16_t sa_w = 0, sa_h = 0;
                ora_hme_l0_search_area(x, l, r, dist, &sa_w, &sa_h);
                for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                    for (int sx = 0; sx < c->num_hme_sa_w; sx++)
                        ora_hme_level_0(x, (int16_t)(((int16_t)org_x) >> 2), (int16_t)(((int16_t)org_y) >> 2),
                                        x->b64_w >> 2, x->b64_h >> 2, sa_w, sa_h, &x->ref[l][r][2], (uint32_t)sx,
                                        (uint32_t)sy, &x->l0sad[l][r][sx][sy], &x->l0x[l][r][sx][sy],
                                        &x->l0y[l][r][sx][sy]);
                if (c->enable_me_sr_adjustment && c->distance_based_hme_resizing)
                    x->hme_l0_sa = base;
                if (c->prehme_enable) {
                    /* get_worst_quadrant: strict > from 0, default (0,0) (motion_estimation.c:1872-1901) */
                    uint8_t wx = 0, wy = 0;
                    uint64_t mx = 0;
                    if (x->l0sad[l][r][0][0] > mx) {
                        mx = x->l0sad[l][r][0][0];
                        wx = 0;
                        wy = 0;
                    }
                    if (x->l0sad[l][r][1][0] > mx) {
                        mx = x->l0sad[l][r][1][0];
                        wx = 1;
                        wy = 0;
                    }
                    if (x->l0sad[l][r][0][1] > mx) {
                        mx = x->l0sad[l][r][0][1];
                        wx = 0;
                        wy = 1;
                    }
                    if (x->l0sad[l][r][1][1] > mx) {
                        wx = 1;
                        wy = 1;
                    }
                    int s = x->prehme[l][r][0].sad <= x->prehme[l][r][1].sad ? 0 : 1;
                    if (x->prehme[l][r][s].sad < x->l0sad[l][r][wx][wy]) {
                        x->l0sad[l][r][wx][wy] = x->prehme[l][r][s].sad;
                        x->l0x[l][r][wx][wy]   = x->prehme[l][r][s].col;
                        x->l0y[l][r][wx][wy]   = x->prehme[l][r][s].row;
                    }
                }
            }
        }
}

static void ora_hme_level1_b64(OraCtx *x, uint32_t org_x, uint32_t org_y) {
    const svtme_controls *c = x->c;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            if (!(x->job->temporal_layer_index > 0 || l == 0))
                continue;
            if (c->me_early_exit_th && x->zz_sad[l][r] < (c->me_early_exit_th >> 2)) {
                for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                    for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                        x->l1x[l][r][sx][sy] = x->l1y[l][r][sx][sy] = 0;
                        x->l1sad[l][r][sx][sy]                      = 0;
                    }
                continue;
            }
            if (!x->sr[l][r].do_ref) {
                for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                    for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                        x->l1x[l][r][sx][sy] = x->l1y[l][r][sx][sy] = 0;
                        x->l1sad[l][r][sx][sy]                      = MAX_U32;
                    }
                continue;
            }
            for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                    if (c->prev_me_stage_based_exit_th &&
                        x->l0sad[l][r][sx][sy] < (c->prev_me_stage_based_exit_th >> 5)) {
                        x->l1x[l][r][sx][sy]   = x->l0x[l][r][sx][sy];
                        x->l1y[l][r][sx][sy]   = x->l0y[l][r][sx][sy];
                        x->l1sad[l][r][sx][sy] = x->l0sad[l][r][sx][sy];
                        continue;
                    }
                    ora_hme_refine(x, 1, (int16_t)(((int16_t)org_x) >> 1), (int16_t)(((int16_t)org_y) >> 1),
                                   x->b64_w >> 1, x->b64_h >> 1, &x->ref[l][r][1], (int16_t)c->hme_l1_sa.width,
                                   (int16_t)c->hme_l1_sa.height, (int16_t)(x->l0x[l][r][sx][sy] >> 1),
                                   (int16_t)(x->l0y[l][r][sx][sy] >> 1), &x->l1sad[l][r][sx][sy],
                                   &x->l1x[l][r][sx][sy], &x->l1y[l][r][sx][sy]);
                }
        }
}

static void ora_hme_level2_b64(OraCtx *x, uint32_t org_x, uint32_t org_y) {
    const svtme_controls *c = x->c;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            if (!(x->job->temporal_layer_index > 0 || l == 0))
                continue;
            for (int sy = 0; sy < c->num_hme_sa_h; sy++)
                for (int sx = 0; sx < c->num_hme_sa_w; sx++) {
                    if (c->prev_me_stage_based_exit_th &&
                        x->l1sad[l][r][sx][sy] < (c->prev_me_stage_based_exit_th >> 2)) {
                        x->l2x[l][r][sx][sy]   = x->l1x[l][r][sx][sy];
                        x->l2y[l][r][sx][sy]   = x->l1y[l][r][sx][sy];
                        x->l2sad[l][r][sx][sy] = x->l1sad[l][r][sx][sy];
                        continue;
                    }
                    ora_hme_refine(x, 2, (int16_t)org_x, (int16_t)org_y, x->b64_w, x->b64_h, &x->ref[l][r][0],
                                   (int16_t)c->hme_l2_sa.width, (int16_t)c->hme_l2_sa.height, x->l1x[l][r][sx][sy],
                                   x->l1y[l][r][sx][sy], &x->l2sad[l][r][sx][sy], &x->l2x[l][r][sx][sy],
                                   &x->l2y[l][r][sx][sy]);
                }
        }
}

/* motion_estimation.c:2182-2380: best region centre at the highest enabled level;
 * the centre/SAD variables live across the ref loop (stale for base-layer list 1). */
static void ora_pick(int16_t xs[2][2], int16_t ys[2][2], uint64_t sads[2][2], int nw, int nh, int16_t *bx, int16_t *by,
                     uint64_t *bs) {
    *bx = xs[0][0];
    *by = ys[0][0];
    *bs = sads[0][0];
    uint32_t w = 1, h = 0;
    while (h < (uint32_t)nh) {
        while (w < (uint32_t)nw) {
            if (sads[w][h] < *bs) {
                *bx = xs[w][h];
                *by = ys[w][h];
                *bs = sads[w][h];
            }
            w++;
        }
        w = 0;
        h++;
    }
}

static void ora_set_final_centre(OraCtx *x) {
    const svtme_controls *c = x->c;
    int16_t hx = 0, hy = 0, scx = 0, scy = 0;
    uint64_t hsad = 0;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            if (x->job->temporal_layer_index > 0 || l == 0) {
                if (c->enable_hme_flag) {
                    if (c->enable_hme_level0_flag && !c->enable_hme_level1_flag && !c->enable_hme_level2_flag)
                        ora_pick(x->l0x[l][r], x->l0y[l][r], x->l0sad[l][r], c->num_hme_sa_w, c->num_hme_sa_h, &hx,
                                 &hy, &hsad);
                    if (c->enable_hme_level1_flag && !c->enable_hme_level2_flag)
                        ora_pick(x->l1x[l][r], x->l1y[l][r], x->l1sad[l][r], c->num_hme_sa_w, c->num_hme_sa_h, &hx,
                                 &hy, &hsad);
                    if (c->enable_hme_level2_flag)
                        ora_pick(x->l2x[l][r], x->l2y[l][r], x->l2sad[l][r], c->num_hme_sa_w, c->num_hme_sa_h, &hx,
                                 &hy, &hsad);
                    scx = hx;
                    scy = hy;
                }
            } else {
                scx = 0;
                scy = 0;
            }
            x->sr[l][r].hme_sc_x = scx;
            x->sr[l][r].hme_sc_y = scy;
            x->sr[l][r].hme_sad  = hsad;
        }
}

/* motion_estimation.c:2477-2518 */
static void ora_hme_prune_and_adjust_sr(OraCtx *x) {
    const svtme_controls *c = x->c;
    const uint16_t th       = c->prune_ref_if_hme_sad_dev_bigger_than_th;
    if (c->enable_me_hme_ref_pruning && th != (uint16_t)~0) {
        uint64_t best = (uint64_t)~0;
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 4; j++)
                if (x->sr[i][j].hme_sad < best)
                    best = x->sr[i][j].hme_sad;
        for (int li = 0; li < 2; li++)
            for (int ri = 1; ri < 4; ri++)
                if ((x->sr[li][ri].hme_sad - best) * 100 > (th * best))
                    x->sr[li][ri].do_ref = 0;
    }
    if (c->enable_me_sr_adjustment) {
        for (int li = 0; li < 2; li++)
            for (int ri = 0; ri < 4; ri++) {
                if (ABS(x->sr[li][ri].hme_sc_x) <= c->reduce_me_sr_based_on_mv_length_th &&
                    ABS(x->sr[li][ri].hme_sc_y) <= c->reduce_me_sr_based_on_mv_length_th &&
                    x->sr[li][ri].hme_sad < c->stationary_hme_sad_abs_th)
                    x->reduce_me_sr_divisor[li][ri] = c->stationary_me_sr_divisor;
                else if (x->sr[li][ri].hme_sad < c->reduce_me_sr_based_on_hme_sad_abs_th)
                    x->reduce_me_sr_divisor[li][ri] = c->me_sr_divisor_for_low_hme_sad;
            }
    }
}

/* ---------------------------------------------------------------------------
 * Full-pel search (motion_estimation.c:98-205, 210-425, 429-817)
 * ------------------------------------------------------------------------- */
/* SAD of the 64 8x8 blocks of the 64x64 source at one position, raster 8x8 order */
static void ora_sad8x8_all(const OraCtx *x, const uint8_t *ref, uint32_t ref_stride, uint32_t out[64]) {
    const int sub = x->c->me_search_method == SVTME_SUB_SAD_SEARCH;
    for (int by = 0; by < 8; by++)
        for (int bx = 0; bx < 8; bx++) {
            const uint8_t *s = x->src + (size_t)(by * 8) * x->src_stride + bx * 8;
            const uint8_t *r = ref + (size_t)(by * 8) * ref_stride + bx * 8;
            if (sub)
                out[by * 8 + bx] = ora_nxm_sad(s, x->src_stride * 2, r, ref_stride * 2, 4, 8) << 1;
            else
                out[by * 8 + bx] = ora_nxm_sad(s, x->src_stride, r, ref_stride, 8, 8);
        }
}

/* one search point: update the 85 Z-order PU bests (strict <) */
static void ora_fullpel_point(OraCtx *x, int l, int r, const uint8_t *ref, uint32_t ref_stride, uint32_t mv) {
    uint32_t s8[64];
    ora_sad8x8_all(x, ref, ref_stride, s8);
    uint32_t *bs = x->best_sad[l][r], *bm = x->best_mv[l][r];
    uint32_t s16[16], s32[4];
    for (int i = 0; i < 16; i++) {
        const int qy = i >> 2, qx = i & 3; /* raster 16x16 */
        const uint32_t a = s8[(qy * 2) * 8 + qx * 2], b = s8[(qy * 2) * 8 + qx * 2 + 1],
                       cc = s8[(qy * 2 + 1) * 8 + qx * 2], d = s8[(qy * 2 + 1) * 8 + qx * 2 + 1];
        /* Z-order index of this 16x16 and its 8x8 children */
        const int z16 = ((qy >> 1) * 2 + (qx >> 1)) * 4 + (qy & 1) * 2 + (qx & 1);
        const uint32_t kids[4] = {a, b, cc, d};
        for (int k = 0; k < 4; k++) {
            const int pu = 21 + z16 * 4 + k;
            if (kids[k] < bs[pu]) {
                bs[pu] = kids[k];
                bm[pu] = mv;
            }
        }
        s16[z16] = a + b + cc + d;
    }
    for (int z = 0; z < 16; z++)
        if (s16[z] < bs[5 + z]) {
            bs[5 + z] = s16[z];
            bm[5 + z] = mv;
        }
    for (int q = 0; q < 4; q++) {
        s32[q] = s16[q * 4] + s16[q * 4 + 1] + s16[q * 4 + 2] + s16[q * 4 + 3];
        if (s32[q] < bs[1 + q]) {
            bs[1 + q] = s32[q];
            bm[1 + q] = mv;
        }
    }
    const uint32_t s64 = s32[0] + s32[1] + s32[2] + s32[3];
    if (s64 < bs[0]) {
        bs[0] = s64;
        bm[0] = mv;
    }
}

static void ora_fullpel_search(OraCtx *x, int l, int r, const uint8_t *win, uint32_t stride, int16_t xo, int16_t yo,
                               uint32_t w, uint32_t h) {
    for (uint32_t ys = 0; ys < h; ys++)
        for (uint32_t xs = 0; xs < w; xs++) {
            const uint32_t mv = ((uint32_t)(int16_t)((int32_t)ys + yo) << 16) | (uint16_t)(int16_t)((int32_t)xs + xo);
            ora_fullpel_point(x, l, r, win + (size_t)ys * stride + xs, stride, mv);
        }
}

/* motion_estimation.c:1139-1206 (only reached when me_early_exit_th == 0) */
static uint32_t ora_check_00_center(OraCtx *x, const OraPlane *p, uint32_t ox_u, uint32_t oy_u, int16_t *xc,
                                    int16_t *yc, uint32_t zz_sad) {
    const int16_t org_x = (int16_t)ox_u, org_y = (int16_t)oy_u;
    const int16_t pad   = 63;
    const int16_t pw = (int16_t)p->width, ph = (int16_t)p->height;
    uint32_t zero_sad;
    if (x->c->me_early_exit_th)
        zero_sad = zz_sad;
    else
        zero_sad = ora_nxm_sad(x->src, x->src_stride << 1,
                               p->buf + (uint32_t)((int16_t)p->org + org_x + ((int16_t)p->org + org_y) * p->stride),
                               (uint32_t)p->stride << 1, x->b64_h >> 1, x->b64_w);
    zero_sad = zero_sad << 1;
    *xc = ((org_x + *xc) < -pad) ? -pad - org_x : *xc;
    *xc = ((org_x + *xc) > pw - 1) ? (int16_t)(*xc - ((org_x + *xc) - (pw - 1))) : *xc;
    *yc = ((org_y + *yc) < -pad) ? -pad - org_y : *yc;
    *yc = ((org_y + *yc) > ph - 1) ? (int16_t)(*yc - ((org_y + *yc) - (ph - 1))) : *yc;
    const uint64_t zero_cost = (uint64_t)zero_sad << 8;
    const uint32_t idx =
        (uint32_t)((int16_t)(p->org + org_x) + *xc + ((int16_t)(p->org + org_y) + *yc) * p->stride);
    uint32_t hme_sad = ora_nxm_sad(x->src, x->src_stride << 1, p->buf + idx, (uint32_t)p->stride << 1, x->b64_h >> 1,
                                   x->b64_w);
    hme_sad                    = hme_sad << 1;
    const uint64_t hme_cost    = (uint64_t)hme_sad << 8;
    const uint64_t centre_cost = MIN(zero_cost, hme_cost);
    *xc = (centre_cost == zero_cost) ? 0 : *xc;
    *yc = (centre_cost == zero_cost) ? 0 : *yc;
    return hme_sad;
}

/* motion_estimation.c:1249-1516 */
static void ora_integer_search(OraCtx *x, uint32_t b64_ox, uint32_t b64_oy) {
    const svtme_controls *c = x->c;
    const int16_t pic_w = (int16_t)x->job->width, pic_h = (int16_t)x->job->height;
    const int16_t pad   = 63;
    const int16_t org_x = (int16_t)b64_ox, org_y = (int16_t)b64_oy;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            const OraPlane *p = &x->ref[l][r][0];
            uint16_t dist     = ora_dist(x, l, r);
            if (x->sr[l][r].do_ref == 0)
                continue;
            int16_t xc = x->sr[l][r].hme_sc_x, yc = x->sr[l][r].hme_sc_y;
            int16_t w = (int16_t)c->me_sa.sa_min.width, h = (int16_t)c->me_sa.sa_min.height;
            if (x->job->me_type != SVTME_ME_MCTF) /* motion_estimation.c:1300-1302 */
                dist = ora_scaled_dist(dist);
            w         = (int16_t)MIN((w * dist), c->me_sa.sa_max.width);
            h         = (int16_t)MIN((h * dist), c->me_sa.sa_max.height);
            if (c->mv_sa_adj_enabled && (!c->mv_sa_adj_nearest_ref_only || r == 0)) {
                if (ABS(xc) > c->mv_sa_adj_mv_size_th)
                    w = (int16_t)(w * c->mv_sa_adj_sa_multiplier);
                if (ABS(yc) > c->mv_sa_adj_mv_size_th)
                    h = (int16_t)(h * c->mv_sa_adj_sa_multiplier);
            }
            w = (int16_t)((MAX(1u, ((uint32_t)(int32_t)w / x->reduce_me_sr_divisor[l][r])) + 7) & ~0x07u);
            h = (int16_t)MAX(3u, ((uint32_t)(int32_t)h / x->reduce_me_sr_divisor[l][r]));
            const int16_t h_before = h, w_before = w;
            uint64_t best_hme_sad  = (uint64_t)~0;
            if (c->me_early_exit_th) {
                if (x->zz_sad[l][r] < (c->me_early_exit_th / 6)) {
                    w = 1;
                    h = 1;
                }
            } else {
                uint8_t hme_accurate = 1;
                if ((xc != 0 || yc != 0) && x->job->is_ref) {
                    best_hme_sad = ora_check_00_center(x, p, b64_ox, b64_oy, &xc, &yc, x->zz_sad[l][r]);
                    if (xc == 0 && yc == 0)
                        hme_accurate = 0;
                }
                if (c->enable_me_sr_adjustment == 2) {
                    if ((hme_accurate && (best_hme_sad < (24 * 24))) ||
                        (x->job->is_ref && x->sr[l][r].hme_sad < (24 * 24)))
                        h = (int16_t)(h / 2);
                }
                if (c->enable_me_sr_adjustment == 2) {
                    if (l || r) {
                        if (x->best_sad[0][0][0] < 5000)
                            if (h == h_before && w == w_before) {
                                h = (int16_t)(h >> 1);
                                w = (int16_t)(w >> 1);
                            }
                    }
                }
            }
            for (int i = 0; i < 85; i++) x->best_sad[l][r][i] = SVTME_MAX_SAD_VALUE;

            if (c->me_8x8_var_enabled && (w * h > 24)) {
                const uint8_t *win = p->buf + (size_t)(p->org + b64_oy + yc) * p->stride + p->org + b64_ox + xc;
                ora_fullpel_search(x, l, r, win, (uint32_t)p->stride, xc, yc, 1, 1);
                const uint32_t mean = x->best_sad[l][r][0] / 64;
                uint32_t sum_sq     = 0;
                for (int i = 0; i < 64; i++) {
                    const int32_t diff = (int32_t)x->best_sad[l][r][21 + i] - (int32_t)mean;
                    sum_sq += (uint32_t)(diff * diff);
                }
                const uint32_t var = sum_sq / 64;
                if (var > c->me_sr_mult2_th) {
                    w = (int16_t)((MAX(1, w * 3 / 2) + 7) & ~0x7);
                    h = (int16_t)MAX(1, h * 3 / 2);
                }
                if (var < c->me_sr_div4_th) {
                    w = (int16_t)((MAX(1, w >> 2) + 7) & ~0x7);
                    h = (int16_t)MAX(1, h >> 2);
                    h = (int16_t)MAX(3, h);
                } else if (var < c->me_sr_div2_th) {
                    w = (int16_t)((MIN(w, w >> 1) + 7) & ~0x7);
                    h = (int16_t)MIN(h, h >> 1);
                    h = (int16_t)MAX(3, h);
                }
            }
            int16_t xo = (int16_t)(xc - (w >> 1));
            int16_t yo = (int16_t)(yc - (h >> 1));
            xo = ((org_x + xo) < -pad) ? -pad - org_x : xo;
            w  = ((org_x + xo) < -pad) ? (int16_t)(w - (-pad - (org_x + xo))) : w;
            xo = ((org_x + xo) > pic_w - 1) ? (int16_t)(xo - ((org_x + xo) - (pic_w - 1))) : xo;
            w  = ((org_x + xo + w) > pic_w) ? (int16_t)MAX(1, w - ((org_x + xo + w) - pic_w)) : w;
            w  = (w < 8) ? w : (int16_t)(w & ~0x07);
            yo = ((org_y + yo) < -pad) ? -pad - org_y : yo;
            h  = ((org_y + yo) < -pad) ? (int16_t)(h - (-pad - (org_y + yo))) : h;
            yo = ((org_y + yo) > pic_h - 1) ? (int16_t)(yo - ((org_y + yo) - (pic_h - 1))) : yo;
            h  = (org_y + yo + h > pic_h) ? (int16_t)MAX(1, h - ((org_y + yo + h) - pic_h)) : h;
            const uint8_t *win = p->buf + (size_t)(p->org + (int32_t)b64_oy + yo) * p->stride + p->org +
                (int32_t)b64_ox + xo;
            ora_fullpel_search(x, l, r, win, (uint32_t)p->stride, xo, yo, (uint32_t)(uint16_t)w, (uint32_t)(uint16_t)h);
        }
}

/* motion_estimation.c:1522-1565 */
static void ora_me_prune_ref(OraCtx *x) {
    const svtme_controls *c = x->c;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            x->sr[l][r].hme_sad = 0;
            if (x->sr[l][r].do_ref == 0) {
                x->sr[l][r].hme_sad = (uint64_t)SVTME_MAX_SAD_VALUE * 64;
                continue;
            }
            for (int i = 0; i < 64; i++) x->sr[l][r].hme_sad += x->best_sad[l][r][21 + ora_tab8x8[i]];
        }
    const uint16_t th = c->prune_ref_if_me_sad_dev_bigger_than_th;
    if (c->enable_me_hme_ref_pruning && th != (uint16_t)~0) {
        uint64_t best = (uint64_t)~0;
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 4; j++)
                if (x->sr[i][j].hme_sad < best)
                    best = x->sr[i][j].hme_sad;
        for (int li = 0; li < 2; li++)
            for (int ri = 1; ri < 4; ri++)
                if ((x->sr[li][ri].hme_sad - best) * 100 > (th * best))
                    x->sr[li][ri].do_ref = 0;
    }
}

/* ---------------------------------------------------------------------------
 * Candidate arrays + distortions (motion_estimation.c:2532-3007)
 * ------------------------------------------------------------------------- */
static uint8_t ora_cand(int dir, int r0, int r1, int l0, int l1) {
    return (uint8_t)((dir & 3) | ((r0 & 3) << 2) | ((r1 & 3) << 4) | ((l0 & 1) << 6) | ((l1 & 1) << 7));
}

static void ora_candidates_mrp_off(OraCtx *x, svtme_sb_result *o) {
    const svtme_job *job = x->job;
    uint32_t nl          = x->num_lists;
    uint8_t org0 = x->sr[0][0].do_ref, org1 = (nl == 1) ? 0 : x->sr[1][0].do_ref;
    if (nl < 2 || !x->sr[1][0].do_ref)
        nl = 1;
    const uint32_t prune_th = (org0 && org1) ? (uint32_t)x->c->prune_me_candidates_th : 0;
    const uint8_t npus = job->enable_me_16x16 ? (job->enable_me_8x8 ? 85 : 21) : 5;
    memset(o->total_me_candidate_index, 1, npus);
    for (int n = 0; n < 85; n++) {
        const int pu = ora_z_to_raster[n];
        uint8_t off  = 0;
        const int use = job->enable_me_16x16 ? (job->enable_me_8x8 || n < 21) : n < 5;
        uint8_t blk[2] = {org0, org1};
        const uint32_t best = (org0 && org1) ? MIN(x->best_sad[0][0][n], x->best_sad[1][0][n])
            : org0                           ? x->best_sad[0][0][n]
                                             : x->best_sad[1][0][n];
        x->me_distortion[pu] = best;
        int min_list         = -1;
        if (x->c->use_best_unipred_cand_only && blk[0] && blk[1])
            min_list = x->best_sad[0][0][n] < x->best_sad[1][0][n] ? 0 : 1;
        for (int li = 0; (uint32_t)li < nl && (use || off == 0); ++li) {
            if (blk[li] == 0)
                continue;
            if (prune_th > 0) {
                uint32_t dd = (x->best_sad[li][0][n] - best) * 100;
                if (dd > best * prune_th) {
                    blk[li] = 0;
                    continue;
                }
            }
            if (min_list != -1 && min_list != li) {
                if (use)
                    o->me_mv_array[pu][(li ? job->max_l0 : 0) + 0] = x->best_mv[li][0][n];
                continue;
            }
            if (use) {
                o->me_candidate_array[pu][off] = ora_cand(li, 0, 0, li == 0 ? li : 24, li == 1 ? li : 24);
                o->me_mv_array[pu][(li ? job->max_l0 : 0) + 0] = x->best_mv[li][0][n];
            }
            off++;
        }
        if (blk[0] && blk[1] && use) {
            o->me_candidate_array[pu][off] = ora_cand(2, 0, 0, 0, 1);
            o->total_me_candidate_index[pu] = (uint8_t)(off + 1);
        }
    }
}

static void ora_candidates_single_ref(OraCtx *x, svtme_sb_result *o) {
    const svtme_job *job = x->job;
    const uint8_t blk    = x->sr[0][0].do_ref;
    const uint8_t npus   = job->enable_me_16x16 ? (job->enable_me_8x8 ? 85 : 21) : 5;
    memset(o->total_me_candidate_index, 1, npus);
    for (int n = 0; n < 85; n++) {
        const int pu  = ora_z_to_raster[n];
        const int use = job->enable_me_16x16 ? (job->enable_me_8x8 || n < 21) : n < 5;
        x->me_distortion[pu] = x->best_sad[0][0][n];
        if (blk == 0)
            continue;
        if (use) {
            o->me_candidate_array[pu][0] = ora_cand(0, 0, 0, 0, 0);
            o->me_mv_array[pu][0]        = x->best_mv[0][0][n];
        }
    }
}

static void ora_candidates_general(OraCtx *x, svtme_sb_result *o) {
    const svtme_job *job = x->job;
    const uint32_t nl    = x->num_lists;
    for (uint32_t n = 0; n < 85; n++) {
        const int pu  = (n > 4) ? ora_z_to_raster[n] : (int)n;
        uint8_t off   = 0;
        const int use = job->enable_me_16x16 ? (job->enable_me_8x8 || n < 21) : n < 5;
        uint8_t blk[2][4];
        memset(blk, 0, sizeof(blk));
        const uint32_t prune_th = (uint32_t)x->c->prune_me_candidates_th;
        uint32_t best           = (uint32_t)~0;
        for (uint32_t li = 0; li < nl; li++)
            for (uint32_t r = 0; r < x->num_refs[li]; r++) {
                blk[li][r] = x->sr[li][r].do_ref;
                if (blk[li][r] == 0)
                    continue;
                best = x->best_sad[li][r][n] < best ? x->best_sad[li][r][n] : best;
            }
        x->me_distortion[pu] = best;
        for (uint32_t li = 0; li < nl && (use || off == 0); ++li)
            for (uint32_t r = 0; r < x->num_refs[li] && (use || off == 0); ++r) {
                if (blk[li][r] == 0)
                    continue;
                if (prune_th > 0) {
                    uint32_t dd = (x->best_sad[li][r][n] - best) * 100;
                    if (dd > best * prune_th) {
                        blk[li][r] = 0;
                        continue;
                    }
                }
                if (use) {
                    o->me_candidate_array[pu][off] = ora_cand((int)li, (int)r, (int)r, li == 0 ? (int)li : 24,
                                                              li == 1 ? (int)li : 24);
                    o->me_mv_array[pu][(li ? job->max_l0 : 0) + r] = x->best_mv[li][r][n];
                }
                off++;
            }
        if (nl == 2 && use) {
            for (uint32_t a = 0; a < x->num_refs[0]; a++)
                for (uint32_t b = 0; b < x->num_refs[1]; b++) {
                    if (job->only_l_bwd && (a > 0 || b > 0))
                        continue;
                    if (blk[0][a] && blk[1][b])
                        o->me_candidate_array[pu][off++] = ora_cand(2, (int)a, (int)b, 0, 1);
                }
            if (!job->only_l_bwd) {
                for (uint32_t a = 1; a < x->num_refs[0]; a++)
                    if (blk[0][0] && blk[0][a])
                        o->me_candidate_array[pu][off++] = ora_cand(2, 0, (int)a, 0, 0);
            }
            if (!job->only_l_bwd) {
                if (x->num_refs[1] == 3 && blk[1][0] && blk[1][2])
                    o->me_candidate_array[pu][off++] = ora_cand(2, 0, 2, 1, 1);
            }
        }
        if (use)
            o->total_me_candidate_index[pu] = off;
    }
}

static void ora_compute_distortion(OraCtx *x, svtme_sb_result *o, uint32_t sb_w, uint32_t sb_h) {
    uint32_t d64 = x->me_distortion[0], d32 = 0, d16 = 0, d8 = 0;
    for (int i = 0; i < 4; i++) d32 += x->me_distortion[1 + i];
    for (int i = 0; i < 16; i++) d16 += x->me_distortion[5 + i];
    for (int i = 0; i < 64; i++) d8 += x->me_distortion[21 + i];
    const uint64_t mean = d8 / 64;
    uint64_t sum_sq     = 0;
    for (int i = 0; i < 64; i++) {
        const int64_t diff = (int64_t)x->me_distortion[21 + i] - (int64_t)mean;
        sum_sq += (uint64_t)(diff * diff);
    }
    o->me_8x8_cost_variance = (uint32_t)(sum_sq / 64);
    o->rc_me_distortion     = (x->job->input_resolution <= 2) ? d8 : d16;
    const uint32_t pix      = sb_w * sb_h;
    o->me_64x64_distortion  = (d64 * 4096u) / pix;
    o->me_32x32_distortion  = (d32 * 4096u) / pix;
    o->me_16x16_distortion  = (d16 * 4096u) / pix;
    o->me_8x8_distortion    = (d8 * 4096u) / pix;
}

/* definitions.h:2613-2632 (indexed as the reference indexes them) */
static const uint8_t ora_8x8_to_16x16[64] = {5,  5,  6,  6,  7,  7,  8,  8,  5,  5,  6,  6,  7,  7,  8,  8,
                                             9,  9,  10, 10, 11, 11, 12, 12, 9,  9,  10, 10, 11, 11, 12, 12,
                                             13, 13, 14, 14, 15, 15, 16, 16, 13, 13, 14, 14, 15, 15, 16, 16,
                                             17, 17, 18, 18, 19, 19, 20, 20, 17, 17, 18, 18, 19, 19, 20, 20};
static const uint8_t ora_16x16_to_32x32[16] = {1, 1, 2, 2, 1, 1, 2, 2, 3, 3, 4, 4, 3, 3, 4, 4};

/* motion_estimation.c:2838-2961 */
static void ora_gm_detection(OraCtx *x, svtme_sb_result *o) {
    const svtme_job *job = x->job;
    uint64_t stationary = 0, tot = 0;
    uint64_t cnt[2][4][2][2];
    memset(cnt, 0, sizeof(cnt));
    const int low_res = job->input_resolution <= 2;
    const int n_blk   = low_res ? 64 : 16;
    for (int i = 0; i < n_blk; i++) {
        uint8_t n = (uint8_t)(low_res ? 21 + i : 5 + i);
        if (low_res && !job->enable_me_8x8) {
            if (n >= 21)
                n = ora_8x8_to_16x16[n - 21];
            if (!job->enable_me_16x16 && n >= 5)
                n = ora_16x16_to_32x32[n - 5];
        }
        if (!low_res && !job->enable_me_16x16 && n >= 5)
            n = ora_16x16_to_32x32[n - 5];
        const uint8_t cb = o->me_candidate_array[n][0];
        const int dir = cb & 3, r0 = (cb >> 2) & 3, r1 = (cb >> 4) & 3, l0 = (cb >> 6) & 1, l1 = (cb >> 7) & 1;
        const int li = (dir == 0 || dir == 2) ? l0 : l1;
        const int ri = (dir == 0 || dir == 2) ? r0 : r1;
        int active_th;
        if (low_res) {
            uint64_t a = job->picture_number, b = job->ref_picture_number[li][ri];
            uint16_t dist = (uint16_t)ABS((int16_t)(MAX(a, b) - MIN(a, b)));
            active_th     = job->gm_use_distance_based_active_th ? MAX(dist >> 1, 4) : 4;
        } else {
            uint16_t dist = (uint16_t)ABS((int16_t)(job->picture_number - job->ref_picture_number[li][ri]));
            active_th     = job->gm_use_distance_based_active_th ? MAX(dist * 16, 32) : 32;
        }
        const uint32_t mv = x->best_mv[li][ri][n];
        const int mx = (int)(int16_t)(mv & 0xFFFF) * 4, my = (int)(int16_t)(mv >> 16) * 4; /* full-pel -> 1/4 pel */
        if (mx < -active_th)
            cnt[li][ri][0][0]++;
        else if (mx > active_th)
            cnt[li][ri][0][1]++;
        if (my < -active_th)
            cnt[li][ri][1][0]++;
        else if (my > active_th)
            cnt[li][ri][1][1]++;
        const int st = low_res ? 0 : 4;
        if (ABS(mx) <= st && ABS(my) <= st)
            stationary++;
        tot++;
    }
    if (stationary > ((tot * 5) / 100))
        o->stationary_block_present = 1;
    for (int l = 0; l < 2; l++)
        for (int r = 0; r < 4; r++)
            for (int cc = 0; cc < 2; cc++)
                for (int s = 0; s < 2; s++)
                    if (cnt[l][r][cc][s] > (tot / 2))
                        o->rc_me_allow_gm = 1;
}

/* ---------------------------------------------------------------------------
 * SB driver (motion_estimation.c:3010-3153) and picture loop (me_process.c:174-271)
 * ------------------------------------------------------------------------- */
static void ora_init_me_hme_data(OraCtx *x) {
    memset(x->l0x, 0, sizeof(x->l0x));
    memset(x->l0y, 0, sizeof(x->l0y));
    memset(x->l1x, 0, sizeof(x->l1x));
    memset(x->l1y, 0, sizeof(x->l1y));
    memset(x->l2x, 0, sizeof(x->l2x));
    memset(x->l2y, 0, sizeof(x->l2y));
    memset(x->best_mv, 0, sizeof(x->best_mv));
    for (int l = 0; l < 2; l++)
        for (int r = 0; r < 4; r++) {
            x->sr[l][r].do_ref             = 1;
            x->sr[l][r].hme_sad            = MAX_U32;
            x->reduce_me_sr_divisor[l][r]  = 1;
            x->zz_sad[l][r]                = MAX_U32;
            x->prehme[l][r][0].valid       = 0;
            x->prehme[l][r][1].valid       = 0;
        }
    memset(x->performed_phme, 0, sizeof(x->performed_phme));
}

static void ora_me_b64(OraCtx *x, uint32_t b64_index, uint32_t ox, uint32_t oy, svtme_ref_record *rec,
                       svtme_sb_result *sbres) {
    const svtme_job *job    = x->job;
    const svtme_controls *c = x->c;
    x->b64_w = (job->width - ox) < 64 ? job->width - ox : 64;
    x->b64_h = (job->height - oy) < 64 ? job->height - oy : 64;
    const int mctf      = job->me_type == SVTME_ME_MCTF;
    const int prune_ref = c->enable_hme_flag && !mctf; /* motion_estimation.c:3103 */
    ora_init_me_hme_data(x);
    /* hme_b64 (motion_estimation.c:2441-2475) */
    if (c->me_early_exit_th || c->me_safe_limit_zz_th)
        ora_init_zz_sad(x, (int16_t)ox, (int16_t)oy);
    if (c->prehme_enable)
        ora_prehme_b64(x, ox, oy);
    if (c->enable_hme_flag) {
        if (c->enable_hme_level0_flag)
            ora_hme_level0_b64(x, ox, oy);
        if (c->enable_hme_level1_flag)
            ora_hme_level1_b64(x, ox, oy);
        if (c->enable_hme_level2_flag)
            ora_hme_level2_b64(x, ox, oy);
    }
    ora_set_final_centre(x);
    /* MCTF: HME-only exit (motion_estimation.c:3109-3113) */
    const int tf_exit = mctf && x->sr[0][0].hme_sad < job->tf_me_exit_th;
    uint8_t searched[2][4];
    memset(searched, 0, sizeof(searched));
    if (!tf_exit) {
        if (prune_ref)
            ora_hme_prune_and_adjust_sr(x);
        for (int l = 0; l < 2; l++)
            for (int r = 0; r < 4; r++) searched[l][r] = x->sr[l][r].do_ref;
        ora_integer_search(x, ox, oy);
        if (prune_ref && c->enable_me_hme_ref_pruning)
            ora_me_prune_ref(x);
    }

    int slot = 0;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++, slot++) {
            svtme_ref_record *o = &rec[slot];
            memset(o, 0, sizeof(*o));
            if (searched[l][r])
                memcpy(o->best_sad, x->best_sad[l][r], sizeof(o->best_sad));
            else
                memset(o->best_sad, 0xFF, sizeof(o->best_sad));
            memcpy(o->best_mv, x->best_mv[l][r], sizeof(o->best_mv));
            o->hme_sad  = x->sr[l][r].hme_sad;
            o->hme_sc_x = x->sr[l][r].hme_sc_x;
            o->hme_sc_y = x->sr[l][r].hme_sc_y;
            o->zz_sad   = x->zz_sad[l][r];
            o->searched = searched[l][r];
            o->do_ref   = x->sr[l][r].do_ref;
            o->tf_early_exit = (uint8_t)tf_exit;
        }
    if (sbres)
        memset(sbres, 0, sizeof(*sbres));
    if (sbres && !mctf) { /* motion_estimation.c:3126-3151 */
        if (x->num_refs[0] == 1 && x->num_refs[1] == 0)
            ora_candidates_single_ref(x, sbres);
        else if (x->num_refs[0] == 1 && x->num_refs[1] == 1)
            ora_candidates_mrp_off(x, sbres);
        else
            ora_candidates_general(x, sbres);
        memcpy(sbres->me_distortion, x->me_distortion, sizeof(sbres->me_distortion));
        ora_compute_distortion(x, sbres, x->b64_w, x->b64_h);
        if (job->gm_enabled)
            ora_gm_detection(x, sbres);
    }
    (void)b64_index;
}

typedef struct OraRange {
    const svtme_job *job;
    const svtme_pyr *cur;
    const svtme_pyr *refs;
    svtme_ref_record *out;
    svtme_sb_result *sbres;
    uint32_t first, count;
} OraRange;

static void ora_plane(OraPlane *p, const uint8_t *buf, uint32_t w, uint32_t h, uint32_t pad) {
    p->buf    = buf;
    p->stride = (int32_t)(w + 2 * pad);
    p->width  = (int32_t)w;
    p->height = (int32_t)h;
    p->org    = (int32_t)pad;
}

static void ora_run_range(OraRange *rg) {
    const svtme_job *job = rg->job;
    const uint32_t W = job->width, H = job->height;
    OraCtx *x = (OraCtx *)calloc(1, sizeof(OraCtx));
    x->job       = job;
    x->c         = &job->ctrl;
    x->hme_l0_sa = job->ctrl.hme_l0_sa;
    x->num_lists = job->num_lists;
    x->num_refs[0] = job->num_refs[0];
    x->num_refs[1] = job->num_lists == 2 ? job->num_refs[1] : 0;
    for (int l = 0; l < x->num_lists; l++)
        for (int r = 0; r < x->num_refs[l]; r++) {
            const svtme_pyr *p = &rg->refs[l * 4 + r];
            ora_plane(&x->ref[l][r][0], p->full, W, H, SVTME_PAD_FULL);
            ora_plane(&x->ref[l][r][1], p->quarter, W / 2, H / 2, SVTME_PAD_QUARTER);
            ora_plane(&x->ref[l][r][2], p->sixteenth, W / 4, H / 4, SVTME_PAD_SIXTEENTH);
        }
    const uint32_t fs = W + 2 * SVTME_PAD_FULL, qs = W / 2 + 2 * SVTME_PAD_QUARTER, ss = W / 4 + 2 * SVTME_PAD_SIXTEENTH;
    const uint32_t R = svtme_job_ref_slots(job);
    const uint32_t pic_w_b64 = (W + 63) / 64;
    for (uint32_t k = 0; k < rg->count; k++) {
        const uint32_t b  = rg->first + k;
        const uint32_t ox = (b % pic_w_b64) * 64, oy = (b / pic_w_b64) * 64;
        x->src         = rg->cur->full + (size_t)(SVTME_PAD_FULL + oy) * fs + SVTME_PAD_FULL + ox;
        x->src_stride  = fs;
        x->qsrc        = rg->cur->quarter + (size_t)(SVTME_PAD_QUARTER + (oy >> 1)) * qs + SVTME_PAD_QUARTER + (ox >> 1);
        x->qsrc_stride = qs;
        x->ssrc = rg->cur->sixteenth + (size_t)(SVTME_PAD_SIXTEENTH + (oy >> 2)) * ss + SVTME_PAD_SIXTEENTH + (ox >> 2);
        x->ssrc_stride = ss;
        ora_me_b64(x, b, ox, oy, rg->out + (size_t)(b - job->sb_begin) * R,
                   rg->sbres ? rg->sbres + (b - job->sb_begin) : NULL);
    }
    free(x);
}

static void *ora_thread(void *p) {
    t_absdiff = 0;
    ora_run_range((OraRange *)p);
    __atomic_fetch_add(&g_absdiff, t_absdiff, __ATOMIC_RELAXED);
    return NULL;
}

uint64_t svtora_absdiff(int reset) {
    return reset ? __atomic_exchange_n(&g_absdiff, 0, __ATOMIC_RELAXED) : __atomic_load_n(&g_absdiff, __ATOMIC_RELAXED);
}

uint32_t svtme_sb_total(uint32_t width, uint32_t height) { return ((width + 63) / 64) * ((height + 63) / 64); }

uint32_t svtme_job_ref_slots(const svtme_job *job) {
    return job->num_refs[0] + (job->num_lists == 2 ? job->num_refs[1] : 0);
}

svtme_status svtora_me(const svtme_job *job, const svtme_pyr *cur, const svtme_pyr *refs, svtme_ref_record *out,
                       svtme_sb_result *sbres, int nthreads) {
    if ((job->width & 7) || (job->height & 7) || job->num_lists < 1 || job->num_lists > 2 ||
        job->ctrl.num_hme_sa_w != 2 || job->ctrl.num_hme_sa_h != 2)
        return SVTME_ERR_BAD_PARAMETER;
    const uint32_t total = svtme_sb_total(job->width, job->height);
    const uint32_t count = job->sb_count ? job->sb_count : total - job->sb_begin;
    if (job->sb_begin + count > total)
        return SVTME_ERR_BAD_PARAMETER;
    if (nthreads < 1)
        nthreads = 1;
    if ((uint32_t)nthreads > count)
        nthreads = (int)(count ? count : 1);
    OraRange *rg  = (OraRange *)calloc(nthreads, sizeof(OraRange));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        const uint32_t b = job->sb_begin + (uint32_t)((uint64_t)count * t / nthreads);
        const uint32_t e = job->sb_begin + (uint32_t)((uint64_t)count * (t + 1) / nthreads);
        rg[t] = (OraRange){job, cur, refs, out, sbres, b, e - b};
    }
    if (nthreads == 1)
        ora_thread(&rg[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, ora_thread, &rg[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    free(rg);
    free(th);
    return SVTME_OK;
}

/* ---------------------------------------------------------------------------
 * Pyramid (pic_analysis_process.c:130-158, :1945-2002; pic_operators.c:338-383, :491)
 * ------------------------------------------------------------------------- */
static void ora_pad(uint8_t *buf, uint32_t stride, uint32_t w, uint32_t h, uint32_t pad) {
    /* edge replicate: horizontal first, then whole rows up/down */
    for (uint32_t r = 0; r < h; r++) {
        uint8_t *row = buf + (size_t)(pad + r) * stride + pad;
        memset(row - pad, row[0], pad);
        memset(row + w, row[w - 1], pad);
    }
    for (uint32_t r = 0; r < pad; r++) {
        memcpy(buf + (size_t)r * stride, buf + (size_t)pad * stride, stride);
        memcpy(buf + (size_t)(pad + h + r) * stride, buf + (size_t)(pad + h - 1) * stride, stride);
    }
}

static void ora_downsample2(const uint8_t *in, uint32_t in_stride, uint32_t w, uint32_t h, uint8_t *out,
                            uint32_t out_stride) {
    for (uint32_t y = 1, oy = 0; y < h; y += 2, oy++) {
        const uint8_t *a = in + (size_t)(y - 1) * in_stride, *b = in + (size_t)y * in_stride;
        for (uint32_t xx = 1, ox = 0; xx < w; xx += 2, ox++)
            out[(size_t)oy * out_stride + ox] = (uint8_t)((a[xx - 1] + a[xx] + b[xx - 1] + b[xx] + 2) >> 2);
    }
}

void svtora_build_pyramid(const uint8_t *y, uint32_t stride, uint32_t w, uint32_t h, svtme_pyr *out) {
    const uint32_t W = svtme_align8(w), H = svtme_align8(h);
    const uint32_t fs = W + 2 * SVTME_PAD_FULL, qs = W / 2 + 2 * SVTME_PAD_QUARTER, ss = W / 4 + 2 * SVTME_PAD_SIXTEENTH;
    uint8_t *full = out->full + (size_t)SVTME_PAD_FULL * fs + SVTME_PAD_FULL;
    for (uint32_t r = 0; r < h; r++) {
        memcpy(full + (size_t)r * fs, y + (size_t)r * stride, w);
        memset(full + (size_t)r * fs + w, full[(size_t)r * fs + w - 1], W - w);
    }
    for (uint32_t r = h; r < H; r++) memcpy(full + (size_t)r * fs, full + (size_t)(h - 1) * fs, W);
    ora_pad(out->full, fs, W, H, SVTME_PAD_FULL);
    uint8_t *q = out->quarter + (size_t)SVTME_PAD_QUARTER * qs + SVTME_PAD_QUARTER;
    ora_downsample2(full, fs, W, H, q, qs);
    ora_pad(out->quarter, qs, W / 2, H / 2, SVTME_PAD_QUARTER);
    uint8_t *s = out->sixteenth + (size_t)SVTME_PAD_SIXTEENTH * ss + SVTME_PAD_SIXTEENTH;
    ora_downsample2(q, qs, W / 2, H / 2, s, ss);
    ora_pad(out->sixteenth, ss, W / 4, H / 4, SVTME_PAD_SIXTEENTH);
}
