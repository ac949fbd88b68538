/*
 * svtme_svt_glue.c — the encoder-side binding of libsvtme.so into SVT-AV1.
 *
 * This file is meant to be compiled INSIDE the reference encoder (it includes
 * the reference's own headers: pcs.h, me_context.h, me_sb_results.h,
 * reference_object.h, aom_dsp_rtcd.h) and linked with libsvtme.so. It is what
 * INTEGRATION.md describes; tests/test_integration.py compiles it against
 * /root/reference/Source with gcc in the build container.
 *
 *   svt_aom_setup_rtcd_hip()          register the *_hip rtcd variants over the
 *                                     pointers svt_aom_setup_rtcd_internal set
 *                                     (aom_dsp_rtcd.c:188; called after it from
 *                                     svt_av1_enc_init, enc_handle.c:1445). Each
 *                                     wrapper re-runs a call on the variant it
 *                                     replaced when the HIP call failed
 *                                     (svtme_rtcd_failed), so a kernel never
 *                                     fails visibly (SURVEY.md 8(b) Errors).
 *   svtme_controls_from_me_context()  the per-picture ME controls that
 *                                     svt_aom_sig_deriv_me (enc_mode_config.c:671)
 *                                     wrote into a MeContext, as svtme_controls.
 *   svtme_job_from_pcs()              one PA-ME picture job (me_process.c:217-261).
 *   svtme_scatter_sb()                one SB's outputs into MeSbResults and the
 *                                     pcs per-SB arrays (me_sb_results.h:28-44,
 *                                     pcs.h:871-878), exactly where
 *                                     svt_aom_motion_estimation_b64 leaves them.
 *   svtme_me_picture()                the picture-level replacement of the SB loop
 *                                     of me_process.c:172-290 (segments 1x1).
 *   svtme_picture_redecimated()       re-upload after temporal filtering replaced
 *                                     a picture's planes (temporal_filtering.c:
 *                                     3895-3931 pad_and_decimate_filtered_pic).
 */
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include "aom_dsp_rtcd.h"
#include "mcomp.h"
#include "me_context.h"
#include "me_sb_results.h"
#include "pcs.h"
#include "reference_object.h"
#include "sequence_control_set.h"

#include "svtme.h"

/* --------------------------------------------------------------------------
 * rtcd registration (aom_dsp_rtcd.h:779, 841, 842, 848, 853-856, 863, 868)
 * ------------------------------------------------------------------------ */
static struct {
    void (*sad_loop)(uint8_t *, uint32_t, uint8_t *, uint32_t, uint32_t, uint32_t, uint64_t *, int16_t *,
                     int16_t *, uint32_t, uint8_t, int16_t, int16_t);
    uint32_t (*nxm)(const uint8_t *, uint32_t, const uint8_t *, uint32_t, uint32_t, uint32_t);
    void (*ext_8x8_16x16)(uint8_t *, uint32_t, uint8_t *, uint32_t, uint32_t *, uint32_t *, uint32_t *, uint32_t *,
                          uint32_t, uint32_t *, uint32_t *, bool);
    void (*ext_32x32_64x64)(uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t, uint32_t *);
    void (*ext_all_8x8_16x16)(uint8_t *, uint32_t, uint8_t *, uint32_t, uint32_t, uint32_t *, uint32_t *,
                              uint32_t *, uint32_t *, uint32_t[16][8], uint32_t[64][8], bool);
    void (*ext_eight_32x32_64x64)(uint32_t[16][8], uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t,
                                  uint32_t[4][8]);
    void (*init32)(uint32_t *, uint32_t, uint32_t, uint32_t);
    void (*downsample)(uint8_t *, uint32_t, uint32_t, uint32_t, uint8_t *, uint32_t, uint32_t);
    uint32_t (*sad16b)(uint16_t *, uint32_t, uint16_t *, uint32_t, uint32_t, uint32_t);
    void (*pme)(const struct svt_mv_cost_param *, uint8_t *, uint32_t, uint8_t *, uint32_t, uint32_t, uint32_t,
                uint32_t *, int16_t *, int16_t *, int16_t, int16_t, int16_t, int16_t, int16_t, int16_t, int16_t);
} g_prev;

/* the MV_COST_PARAMS layout (mcomp.h:37-48) svt_pme_sad_loop_kernel_hip reads */
_Static_assert(offsetof(MV_COST_PARAMS, ref_mv) == SVTME_MVCOST_OFF_REF_MV, "MV_COST_PARAMS.ref_mv");
_Static_assert(offsetof(MV_COST_PARAMS, mv_cost_type) == SVTME_MVCOST_OFF_TYPE, "MV_COST_PARAMS.mv_cost_type");
_Static_assert(sizeof(((MV_COST_PARAMS *)0)->mv_cost_type) == 1, "MV_COST_TYPE is one byte");
_Static_assert(offsetof(MV_COST_PARAMS, mvjcost) == SVTME_MVCOST_OFF_MVJCOST, "MV_COST_PARAMS.mvjcost");
_Static_assert(offsetof(MV_COST_PARAMS, mvcost) == SVTME_MVCOST_OFF_MVCOST, "MV_COST_PARAMS.mvcost");
_Static_assert(offsetof(MV_COST_PARAMS, error_per_bit) == SVTME_MVCOST_OFF_ERROR_PER_BIT,
               "MV_COST_PARAMS.error_per_bit");
_Static_assert(offsetof(MV, row) == 0 && offsetof(MV, col) == 2, "MV is (row, col) int16");

static void glue_sad_loop(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride, uint32_t bh,
                          uint32_t bw, uint64_t *best_sad, int16_t *x, int16_t *y, uint32_t src_stride_raw,
                          uint8_t skip, int16_t sa_w, int16_t sa_h) {
    svt_sad_loop_kernel_hip(src, src_stride, ref, ref_stride, bh, bw, best_sad, x, y, src_stride_raw, skip, sa_w, sa_h);
    if (svtme_rtcd_failed())
        g_prev.sad_loop(src, src_stride, ref, ref_stride, bh, bw, best_sad, x, y, src_stride_raw, skip, sa_w, sa_h);
}

static uint32_t glue_nxm(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                         uint32_t h, uint32_t w) {
    const uint32_t v = svt_nxm_sad_kernel_hip(src, src_stride, ref, ref_stride, h, w);
    return svtme_rtcd_failed() ? g_prev.nxm(src, src_stride, ref, ref_stride, h, w) : v;
}

static void glue_ext_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                               uint32_t *b8, uint32_t *b16, uint32_t *m8, uint32_t *m16, uint32_t mv, uint32_t *s16,
                               uint32_t *s8, bool sub) {
    svt_ext_sad_calculation_8x8_16x16_hip(src, src_stride, ref, ref_stride, b8, b16, m8, m16, mv, s16, s8, sub);
    if (svtme_rtcd_failed())
        g_prev.ext_8x8_16x16(src, src_stride, ref, ref_stride, b8, b16, m8, m16, mv, s16, s8, sub);
}

static void glue_ext_32x32_64x64(uint32_t *s16, uint32_t *b32, uint32_t *b64, uint32_t *m32, uint32_t *m64,
                                 uint32_t mv, uint32_t *s32) {
    svt_ext_sad_calculation_32x32_64x64_hip(s16, b32, b64, m32, m64, mv, s32);
    if (svtme_rtcd_failed())
        g_prev.ext_32x32_64x64(s16, b32, b64, m32, m64, mv, s32);
}

static void glue_ext_all_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                   uint32_t mv, uint32_t *b8, uint32_t *b16, uint32_t *m8, uint32_t *m16,
                                   uint32_t e16[16][8], uint32_t e8[64][8], bool sub) {
    svt_ext_all_sad_calculation_8x8_16x16_hip(src, src_stride, ref, ref_stride, mv, b8, b16, m8, m16, e16, e8, sub);
    if (svtme_rtcd_failed())
        g_prev.ext_all_8x8_16x16(src, src_stride, ref, ref_stride, mv, b8, b16, m8, m16, e16, e8, sub);
}

static void glue_ext_eight_32x32_64x64(uint32_t s16[16][8], uint32_t *b32, uint32_t *b64, uint32_t *m32,
                                       uint32_t *m64, uint32_t mv, uint32_t s32[4][8]) {
    svt_ext_eight_sad_calculation_32x32_64x64_hip(s16, b32, b64, m32, m64, mv, s32);
    if (svtme_rtcd_failed())
        g_prev.ext_eight_32x32_64x64(s16, b32, b64, m32, m64, mv, s32);
}

static void glue_init32(uint32_t *p, uint32_t c128, uint32_t c32, uint32_t v) {
    svt_initialize_buffer_32bits_hip(p, c128, c32, v);
    if (svtme_rtcd_failed())
        g_prev.init32(p, c128, c32, v);
}

static void glue_downsample(uint8_t *in, uint32_t in_stride, uint32_t w, uint32_t h, uint8_t *out,
                            uint32_t out_stride, uint32_t step) {
    svt_aom_downsample_2d_hip(in, in_stride, w, h, out, out_stride, step);
    if (svtme_rtcd_failed())
        g_prev.downsample(in, in_stride, w, h, out, out_stride, step);
}

static uint32_t glue_sad16b(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride, uint32_t h,
                            uint32_t w) {
    const uint32_t v = svt_aom_sad_16b_kernel_hip(src, src_stride, ref, ref_stride, h, w);
    return svtme_rtcd_failed() ? g_prev.sad16b(src, src_stride, ref, ref_stride, h, w) : v;
}

static void glue_pme(const struct svt_mv_cost_param *p, uint8_t *src, uint32_t src_stride, uint8_t *ref,
                     uint32_t ref_stride, uint32_t bh, uint32_t bw, uint32_t *best_cost, int16_t *best_mvx,
                     int16_t *best_mvy, int16_t sx, int16_t sy, int16_t sa_w, int16_t sa_h, int16_t step, int16_t mvx,
                     int16_t mvy) {
    svt_pme_sad_loop_kernel_hip(p, src, src_stride, ref, ref_stride, bh, bw, best_cost, best_mvx, best_mvy, sx, sy,
                                sa_w, sa_h, step, mvx, mvy);
    if (svtme_rtcd_failed())
        g_prev.pme(p, src, src_stride, ref, ref_stride, bh, bw, best_cost, best_mvx, best_mvy, sx, sy, sa_w, sa_h,
                   step, mvx, mvy);
}

/* Call right after svt_aom_setup_rtcd_internal(): the pointers it set become the
 * fallbacks, the HIP variants the active ones. */
void svt_aom_setup_rtcd_hip(void) {
    g_prev.sad_loop              = svt_sad_loop_kernel;
    g_prev.nxm                   = svt_nxm_sad_kernel;
    g_prev.ext_8x8_16x16         = svt_ext_sad_calculation_8x8_16x16;
    g_prev.ext_32x32_64x64       = svt_ext_sad_calculation_32x32_64x64;
    g_prev.ext_all_8x8_16x16     = svt_ext_all_sad_calculation_8x8_16x16;
    g_prev.ext_eight_32x32_64x64 = svt_ext_eight_sad_calculation_32x32_64x64;
    g_prev.init32                = svt_initialize_buffer_32bits;
    g_prev.downsample            = downsample_2d;
    g_prev.sad16b                = sad_16b_kernel;
    g_prev.pme                   = svt_pme_sad_loop_kernel;

    svt_sad_loop_kernel                       = glue_sad_loop;                /* :779 */
    svt_nxm_sad_kernel                        = glue_nxm;                     /* :856 */
    svt_ext_sad_calculation_8x8_16x16         = glue_ext_8x8_16x16;           /* :842 */
    svt_ext_sad_calculation_32x32_64x64       = glue_ext_32x32_64x64;         /* :848 */
    svt_ext_all_sad_calculation_8x8_16x16     = glue_ext_all_8x8_16x16;       /* :853 */
    svt_ext_eight_sad_calculation_32x32_64x64 = glue_ext_eight_32x32_64x64;   /* :854 */
    svt_initialize_buffer_32bits              = glue_init32;                  /* :855 */
    downsample_2d                             = glue_downsample;              /* :841 */
    sad_16b_kernel                            = glue_sad16b;                  /* :863 */
    svt_pme_sad_loop_kernel                   = glue_pme;                     /* :868 */
}

/* --------------------------------------------------------------------------
 * Controls: the MeContext fields svt_aom_sig_deriv_me sets (me_context.h:280-509)
 * ------------------------------------------------------------------------ */
static svtme_area area_of(SearchArea a) {
    svtme_area r = {a.width, a.height};
    return r;
}

static svtme_area_minmax minmax_of(SearchAreaMinMax a) {
    svtme_area_minmax r = {area_of(a.sa_min), area_of(a.sa_max)};
    return r;
}

void svtme_controls_from_me_context(svtme_controls *c, const MeContext *m) {
    memset(c, 0, sizeof(*c));
    c->hme_search_method      = m->hme_search_method;
    c->me_search_method       = m->me_search_method;
    c->enable_hme_flag        = m->enable_hme_flag;
    c->enable_hme_level0_flag = m->enable_hme_level0_flag;
    c->enable_hme_level1_flag = m->enable_hme_level1_flag;
    c->enable_hme_level2_flag = m->enable_hme_level2_flag;
    c->num_hme_sa_w           = (uint8_t)m->num_hme_sa_w;
    c->num_hme_sa_h           = (uint8_t)m->num_hme_sa_h;
    c->hme_l0_sa              = minmax_of(m->hme_l0_sa);
    c->hme_l1_sa              = area_of(m->hme_l1_sa);
    c->hme_l2_sa              = area_of(m->hme_l2_sa);
    c->me_sa                  = minmax_of(m->me_sa);

    const MeHmeRefPruneCtrls *pr = &m->me_hme_prune_ctrls;
    c->enable_me_hme_ref_pruning               = pr->enable_me_hme_ref_pruning;
    c->prune_ref_if_hme_sad_dev_bigger_than_th = pr->prune_ref_if_hme_sad_dev_bigger_than_th;
    c->prune_ref_if_me_sad_dev_bigger_than_th  = pr->prune_ref_if_me_sad_dev_bigger_than_th;
    c->zz_sad_th                               = pr->zz_sad_th;
    c->zz_sad_pct                              = pr->zz_sad_pct;
    c->phme_sad_th                             = pr->phme_sad_th;
    c->phme_sad_pct                            = pr->phme_sad_pct;

    /* the disabled control blocks keep stale values in the reference; the job
     * carries zeros for them (the ME code never reads them then) */
    const MeSrCtrls *sr = &m->me_sr_adjustment_ctrls;
    if ((c->enable_me_sr_adjustment = sr->enable_me_sr_adjustment)) {
        c->distance_based_hme_resizing          = sr->distance_based_hme_resizing;
        c->reduce_me_sr_based_on_mv_length_th   = sr->reduce_me_sr_based_on_mv_length_th;
        c->stationary_hme_sad_abs_th            = sr->stationary_hme_sad_abs_th;
        c->stationary_me_sr_divisor             = sr->stationary_me_sr_divisor;
        c->reduce_me_sr_based_on_hme_sad_abs_th = sr->reduce_me_sr_based_on_hme_sad_abs_th;
        c->me_sr_divisor_for_low_hme_sad        = sr->me_sr_divisor_for_low_hme_sad;
    }
    const MvBasedSearchAdj *mv = &m->mv_based_sa_adj;
    if ((c->mv_sa_adj_enabled = mv->enabled)) {
        c->mv_sa_adj_nearest_ref_only = mv->nearest_ref_only;
        c->mv_sa_adj_mv_size_th       = mv->mv_size_th;
        c->mv_sa_adj_sa_multiplier    = mv->sa_multiplier;
    }
    const Me8x8VarCtrls *v = &m->me_8x8_var_ctrls;
    if ((c->me_8x8_var_enabled = v->enabled)) {
        c->me_sr_div4_th  = v->me_sr_div4_th;
        c->me_sr_div2_th  = v->me_sr_div2_th;
        c->me_sr_mult2_th = v->me_sr_mult2_th;
    }
    const PreHmeCtrls *ph = &m->prehme_ctrl;
    if ((c->prehme_enable = ph->enable)) {
        c->prehme_skip_search_line = ph->skip_search_line;
        c->prehme_l1_early_exit    = ph->l1_early_exit;
        for (int i = 0; i < SEARCH_REGION_COUNT; i++) c->prehme_sa_cfg[i] = minmax_of(ph->prehme_sa_cfg[i]);
    }
    c->prune_me_candidates_th      = m->prune_me_candidates_th;
    c->use_best_unipred_cand_only  = m->use_best_unipred_cand_only;
    c->reduce_hme_l0_sr_th_min     = m->reduce_hme_l0_sr_th_min;
    c->reduce_hme_l0_sr_th_max     = m->reduce_hme_l0_sr_th_max;
    c->me_early_exit_th            = m->me_early_exit_th;
    c->me_safe_limit_zz_th         = m->me_safe_limit_zz_th;
    c->prev_me_stage_based_exit_th = m->prev_me_stage_based_exit_th;
}

/* --------------------------------------------------------------------------
 * One PA-ME picture job (me_process.c:217-261; pictures are uploaded under
 * their picture_number by the PA stage, svtme_picture_upload)
 * ------------------------------------------------------------------------ */
void svtme_job_from_pcs(svtme_job *job, const PictureParentControlSet *pcs, const MeContext *me) {
    memset(job, 0, sizeof(*job));
    job->picture_number = pcs->picture_number;
    job->width          = pcs->aligned_width;
    job->height         = pcs->aligned_height;
    job->num_lists      = pcs->slice_type == P_SLICE ? 1 : 2;
    job->num_refs[0]    = pcs->ref_list0_count_try;
    job->num_refs[1]    = pcs->slice_type == B_SLICE ? pcs->ref_list1_count_try : 0;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++) {
            const EbPaReferenceObject *ro = (const EbPaReferenceObject *)pcs->ref_pa_pic_ptr_array[l][r]->object_ptr;
            job->ref_picture_number[l][r] = ro->picture_number;
        }
    job->temporal_layer_index            = pcs->temporal_layer_index;
    job->is_ref                          = pcs->is_ref;
    job->hierarchical_levels             = pcs->hierarchical_levels;
    job->similar_brightness_refs         = pcs->similar_brightness_refs;
    job->enable_me_8x8                   = pcs->enable_me_8x8;
    job->enable_me_16x16                 = pcs->enable_me_16x16;
    job->max_cand                        = pcs->pa_me_data->max_cand;
    job->max_refs                        = pcs->pa_me_data->max_refs;
    job->max_l0                          = pcs->pa_me_data->max_l0;
    job->only_l_bwd                      = pcs->scs->mrp_ctrls.only_l_bwd;
    job->input_resolution                = (uint8_t)pcs->input_resolution;
    job->gm_enabled                      = pcs->gm_ctrls.enabled;
    job->gm_use_distance_based_active_th = pcs->gm_ctrls.use_distance_based_active_th;
    job->me_type                         = SVTME_ME_OPEN_LOOP;
    svtme_controls_from_me_context(&job->ctrl, me);
}

/* --------------------------------------------------------------------------
 * Outputs of one SB back into the reference's storage
 * ------------------------------------------------------------------------ */
void svtme_scatter_sb(PictureParentControlSet *pcs, MeContext *me, uint32_t b64_index,
                      const svtme_ref_record *recs, uint32_t R, const svtme_sb_result *s) {
    MeSbResults *res   = pcs->pa_me_data->me_results[b64_index];
    const uint32_t mc  = pcs->pa_me_data->max_cand, mr = pcs->pa_me_data->max_refs;
    memcpy(res->total_me_candidate_index, s->total_me_candidate_index, SVTME_PU_COUNT);
    for (int pu = 0; pu < SVTME_PU_COUNT; pu++) {
        memcpy(&res->me_candidate_array[pu * mc], s->me_candidate_array[pu], mc); /* 1-byte MeCandidate */
        for (uint32_t k = 0; k < mr; k++) res->me_mv_array[pu * mr + k].as_int = s->me_mv_array[pu][k];
    }
    memcpy(me->me_distortion, s->me_distortion, sizeof(me->me_distortion));
    pcs->me_8x8_cost_variance[b64_index]        = s->me_8x8_cost_variance;
    pcs->rc_me_distortion[b64_index]            = s->rc_me_distortion;
    pcs->me_64x64_distortion[b64_index]         = s->me_64x64_distortion;
    pcs->me_32x32_distortion[b64_index]         = s->me_32x32_distortion;
    pcs->me_16x16_distortion[b64_index]         = s->me_16x16_distortion;
    pcs->me_8x8_distortion[b64_index]           = s->me_8x8_distortion;
    pcs->stationary_block_present_sb[b64_index] = s->stationary_block_present;
    pcs->rc_me_allow_gm[b64_index]              = s->rc_me_allow_gm;
    /* per-reference state the ME context keeps after the SB (search_results,
     * me_context.h:459, read by GM detection and TF) */
    for (uint32_t k = 0; k < R; k++) {
        const int l = k < me->num_of_ref_pic_to_search[0] ? 0 : 1;
        const int r = l ? (int)k - me->num_of_ref_pic_to_search[0] : (int)k;
        me->search_results[l][r].hme_sc_x = recs[k].hme_sc_x;
        me->search_results[l][r].hme_sc_y = recs[k].hme_sc_y;
        me->search_results[l][r].hme_sad  = recs[k].hme_sad;
        me->search_results[l][r].do_ref   = recs[k].do_ref;
        memcpy(me->p_sb_best_sad[l][r], recs[k].best_sad, sizeof(recs[k].best_sad));
        memcpy(me->p_sb_best_mv[l][r], recs[k].best_mv, sizeof(recs[k].best_mv));
    }
}

/* --------------------------------------------------------------------------
 * me_process.c:172-290 for task_type TASK_PAME with ME segments 1x1: one job
 * for every SB of the picture, then the host's picture-level consumers (GM,
 * svt_aom_open_loop_intra_search_mb) run as before.
 * ------------------------------------------------------------------------ */
EbErrorType svtme_me_picture(svtme_ctx *ctx, PictureParentControlSet *pcs, MeContext *me) {
    svtme_job job;
    svtme_job_from_pcs(&job, pcs, me);
    me->num_of_list_to_search       = job.num_lists;
    me->num_of_ref_pic_to_search[0] = job.num_refs[0];
    me->num_of_ref_pic_to_search[1] = job.num_refs[1];
    const uint32_t n_sb = svtme_sb_total(job.width, job.height);
    const uint32_t R    = svtme_job_ref_slots(&job);
    svtme_ref_record *recs = (svtme_ref_record *)malloc((size_t)n_sb * R * sizeof(*recs));
    svtme_sb_result *sbr   = (svtme_sb_result *)malloc((size_t)n_sb * sizeof(*sbr));
    if (!recs || !sbr) {
        free(recs);
        free(sbr);
        return EB_ErrorInsufficientResources;
    }
    const svtme_status st = svtme_submit_picture(ctx, &job, recs, sbr);
    if (st == SVTME_OK)
        for (uint32_t sb = 0; sb < n_sb; sb++) svtme_scatter_sb(pcs, me, sb, &recs[(size_t)sb * R], R, &sbr[sb]);
    free(recs);
    free(sbr);
    return (EbErrorType)st;
}

/* Temporal filtering replaced the picture's padded planes
 * (temporal_filtering.c:3895-3931): re-upload so later PA-ME / TF-ME jobs read
 * the filtered pyramid, never the stale one. */
EbErrorType svtme_picture_redecimated(svtme_ctx *ctx, const PictureParentControlSet *pcs,
                                      const EbPictureBufferDesc *filtered) {
    const uint8_t *y = filtered->buffer_y + (size_t)filtered->org_y * filtered->stride_y + filtered->org_x;
    return (EbErrorType)svtme_picture_invalidate(ctx, pcs->picture_number, y, filtered->stride_y,
                                                 pcs->aligned_width, pcs->aligned_height);
}
