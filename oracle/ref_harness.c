/*
 * ref_harness.c — TEST INFRASTRUCTURE ONLY (oracle/_ref, container build).
 *
 * Drives the REFERENCE's own open-loop ME, compiled unmodified from
 * /root/reference by oracle/Makefile, so that the CPU restatement
 * (svtme_oracle.c) and the HIP path can be pinned against it:
 *   - svt_aom_motion_estimation_b64  (Source/Lib/Codec/motion_estimation.c:3076)
 *     called once per SB exactly as the ME thread does (me_process.c:174-271);
 *   - the rtcd kernel pointers set as svt_aom_setup_rtcd_internal does
 *     (aom_dsp_rtcd.c:501-515): C kernels, or the AVX2/SSE4.1/SSE2 picks;
 *   - the PA pyramid built with the reference's own pad_input_picture,
 *     svt_aom_generate_padding (pic_operators.c:338) and downsample_2d
 *     (pic_analysis_process.c:130, :1945-2002).
 * Nothing here is shipped; libsvtme.so never links it.
 */
#define RTCD_C
#define AOM_RTCD_C
#include "aom_dsp_rtcd.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "me_context.h"
#include "motion_estimation.h"
#include "pcs.h"
#include "pic_operators.h"
#include "sequence_control_set.h"

#include "svtme_oracle.h"

/* reference kernels (declared in the reference's own headers / TUs) */
void svt_memcpy_c(void *dst_ptr, void const *src_ptr, size_t size);
void svt_aom_downsample_2d_c(uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                             uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                             uint32_t decim_step);
void svt_initialize_buffer_32bits_c(uint32_t *pointer, uint32_t count128, uint32_t count32, uint32_t value);
uint32_t svt_nxm_sad_kernel_helper_c(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                                     uint32_t height, uint32_t width);
void svt_sad_loop_kernel_c(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                           uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_search_center,
                           int16_t *y_search_center, uint32_t src_stride_raw, uint8_t skip_search_line,
                           int16_t search_area_width, int16_t search_area_height);
void svt_ext_all_sad_calculation_8x8_16x16_c(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                             uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                             uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                             uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                             bool sub_sad);
void svt_ext_eight_sad_calculation_32x32_64x64_c(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                 uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                 uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]);
void svt_pme_sad_loop_kernel_c(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                               uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                               uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                               int16_t search_position_start_x, int16_t search_position_start_y,
                               int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                               int16_t mvx, int16_t mvy); /* product_coding_loop.c:1811 */
#ifdef SVTREF_WITH_SIMD
void svt_pme_sad_loop_kernel_avx2(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                                  uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                                  uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                                  int16_t search_position_start_x, int16_t search_position_start_y,
                                  int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                                  int16_t mvx, int16_t mvy);
void svt_sad_loop_kernel_avx2_intrin(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                     uint32_t block_height, uint32_t block_width, uint64_t *best_sad,
                                     int16_t *x_search_center, int16_t *y_search_center, uint32_t src_stride_raw,
                                     uint8_t skip_search_line, int16_t search_area_width,
                                     int16_t search_area_height);
void svt_aom_downsample_2d_avx2(uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                                uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                                uint32_t decim_step);
void svt_ext_sad_calculation_8x8_16x16_avx2_intrin(uint8_t *src, uint32_t src_stride, uint8_t *ref,
                                                   uint32_t ref_stride, uint32_t *p_best_sad_8x8,
                                                   uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                                   uint32_t *p_best_mv16x16, uint32_t mv, uint32_t *p_sad16x16,
                                                   uint32_t *p_sad8x8, bool sub_sad);
void svt_ext_sad_calculation_32x32_64x64_sse4_intrin(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                                     uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                     uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32);
void svt_ext_all_sad_calculation_8x8_16x16_avx2(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                                uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                                uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                                uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                                bool sub_sad);
void svt_ext_eight_sad_calculation_32x32_64x64_avx2(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                    uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                    uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]);
void svt_initialize_buffer_32bits_sse2_intrin(uint32_t *pointer, uint32_t count128, uint32_t count32, uint32_t value);
uint32_t svt_nxm_sad_kernel_helper_avx2(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                        uint32_t ref_stride, uint32_t height, uint32_t width);
#endif

static int g_simd = -1;

void svtref_set_simd(int simd) {
    /* aom_dsp_rtcd.c:501-515 (C defaults, or the x86 picks capped at AVX2) */
    svt_memcpy                                = svt_memcpy_c;
    svt_sad_loop_kernel                       = svt_sad_loop_kernel_c;
    downsample_2d                             = svt_aom_downsample_2d_c;
    svt_ext_sad_calculation_8x8_16x16         = svt_ext_sad_calculation_8x8_16x16_c;
    svt_ext_sad_calculation_32x32_64x64       = svt_ext_sad_calculation_32x32_64x64_c;
    svt_ext_all_sad_calculation_8x8_16x16     = svt_ext_all_sad_calculation_8x8_16x16_c;
    svt_ext_eight_sad_calculation_32x32_64x64 = svt_ext_eight_sad_calculation_32x32_64x64_c;
    svt_initialize_buffer_32bits              = svt_initialize_buffer_32bits_c;
    svt_nxm_sad_kernel                        = svt_nxm_sad_kernel_helper_c;
    svt_pme_sad_loop_kernel                   = svt_pme_sad_loop_kernel_c;
#ifdef SVTREF_WITH_SIMD
    if (simd) {
        svt_pme_sad_loop_kernel                   = svt_pme_sad_loop_kernel_avx2;
        svt_sad_loop_kernel                       = svt_sad_loop_kernel_avx2_intrin;
        downsample_2d                             = svt_aom_downsample_2d_avx2;
        svt_ext_sad_calculation_8x8_16x16         = svt_ext_sad_calculation_8x8_16x16_avx2_intrin;
        svt_ext_sad_calculation_32x32_64x64       = svt_ext_sad_calculation_32x32_64x64_sse4_intrin;
        svt_ext_all_sad_calculation_8x8_16x16     = svt_ext_all_sad_calculation_8x8_16x16_avx2;
        svt_ext_eight_sad_calculation_32x32_64x64 = svt_ext_eight_sad_calculation_32x32_64x64_avx2;
        svt_initialize_buffer_32bits              = svt_initialize_buffer_32bits_sse2_intrin;
        svt_nxm_sad_kernel                        = svt_nxm_sad_kernel_helper_avx2;
    }
#else
    (void)simd;
#endif
    g_simd = simd;
}

static void ensure_kernels(void) {
    if (g_simd < 0)
        svtref_set_simd(0);
}

/* ---------------------------------------------------------------------------
 * Pyramid (pic_analysis_process.c:1945-2002, :2004; pic_operators.c:338, :491)
 * ------------------------------------------------------------------------- */
void svtref_build_pyramid(const uint8_t *y, uint32_t stride, uint32_t w, uint32_t h, svtme_pyr *out) {
    ensure_kernels();
    const uint32_t W = svtme_align8(w), H = svtme_align8(h);
    const uint32_t fs = W + 2 * SVTME_PAD_FULL, qs = W / 2 + 2 * SVTME_PAD_QUARTER,
                   ss = W / 4 + 2 * SVTME_PAD_SIXTEENTH;
    uint8_t *full = out->full + SVTME_PAD_FULL * fs + SVTME_PAD_FULL;
    for (uint32_t r = 0; r < h; r++) memcpy(full + r * fs, y + (size_t)r * stride, w);
    /* pad to a multiple of 8 (svt_aom_pad_picture_to_multiple_of_min_blk_size_dimensions) */
    pad_input_picture(full, fs, w, h, W - w, H - h);
    svt_aom_generate_padding(out->full, fs, W, H, SVTME_PAD_FULL, SVTME_PAD_FULL);
    /* quarter = downsample_2d(full, 2) then pad 32; sixteenth = downsample_2d(quarter, 2) then pad 16 */
    downsample_2d(full, fs, W, H, out->quarter + SVTME_PAD_QUARTER + SVTME_PAD_QUARTER * qs, qs, 2);
    svt_aom_generate_padding(out->quarter, qs, W / 2, H / 2, SVTME_PAD_QUARTER, SVTME_PAD_QUARTER);
    downsample_2d(out->quarter + SVTME_PAD_QUARTER + SVTME_PAD_QUARTER * qs, qs, W / 2, H / 2,
                  out->sixteenth + SVTME_PAD_SIXTEENTH + SVTME_PAD_SIXTEENTH * ss, ss, 2);
    svt_aom_generate_padding(out->sixteenth, ss, W / 4, H / 4, SVTME_PAD_SIXTEENTH, SVTME_PAD_SIXTEENTH);
}

/* ---------------------------------------------------------------------------
 * ME driver
 * ------------------------------------------------------------------------- */
static void set_desc(EbPictureBufferDesc *d, uint8_t *buf, uint32_t w, uint32_t h, uint32_t pad) {
    memset(d, 0, sizeof(*d));
    d->buffer_y   = buf;
    d->stride_y   = (uint16_t)(w + 2 * pad);
    d->org_x      = (uint16_t)pad;
    d->org_y      = (uint16_t)pad;
    d->width      = (uint16_t)w;
    d->height     = (uint16_t)h;
    d->max_width  = (uint16_t)w;
    d->max_height = (uint16_t)h;
}

/* MeContext control fields from the POD snapshot (me_context.h:366-509) */
static void apply_controls(MeContext *m, const svtme_controls *c) {
    m->hme_search_method      = c->hme_search_method;
    m->me_search_method       = c->me_search_method;
    m->enable_hme_flag        = c->enable_hme_flag;
    m->enable_hme_level0_flag = c->enable_hme_level0_flag;
    m->enable_hme_level1_flag = c->enable_hme_level1_flag;
    m->enable_hme_level2_flag = c->enable_hme_level2_flag;
    m->num_hme_sa_w           = c->num_hme_sa_w;
    m->num_hme_sa_h           = c->num_hme_sa_h;
    m->hme_l0_sa.sa_min       = (SearchArea){c->hme_l0_sa.sa_min.width, c->hme_l0_sa.sa_min.height};
    m->hme_l0_sa.sa_max       = (SearchArea){c->hme_l0_sa.sa_max.width, c->hme_l0_sa.sa_max.height};
    m->hme_l1_sa              = (SearchArea){c->hme_l1_sa.width, c->hme_l1_sa.height};
    m->hme_l2_sa              = (SearchArea){c->hme_l2_sa.width, c->hme_l2_sa.height};
    m->me_sa.sa_min           = (SearchArea){c->me_sa.sa_min.width, c->me_sa.sa_min.height};
    m->me_sa.sa_max           = (SearchArea){c->me_sa.sa_max.width, c->me_sa.sa_max.height};

    m->me_hme_prune_ctrls.enable_me_hme_ref_pruning               = c->enable_me_hme_ref_pruning;
    m->me_hme_prune_ctrls.prune_ref_if_hme_sad_dev_bigger_than_th = c->prune_ref_if_hme_sad_dev_bigger_than_th;
    m->me_hme_prune_ctrls.prune_ref_if_me_sad_dev_bigger_than_th  = c->prune_ref_if_me_sad_dev_bigger_than_th;
    m->me_hme_prune_ctrls.zz_sad_th                               = c->zz_sad_th;
    m->me_hme_prune_ctrls.zz_sad_pct                              = c->zz_sad_pct;
    m->me_hme_prune_ctrls.phme_sad_th                             = c->phme_sad_th;
    m->me_hme_prune_ctrls.phme_sad_pct                            = c->phme_sad_pct;

    m->me_sr_adjustment_ctrls.enable_me_sr_adjustment              = c->enable_me_sr_adjustment;
    m->me_sr_adjustment_ctrls.reduce_me_sr_based_on_mv_length_th   = c->reduce_me_sr_based_on_mv_length_th;
    m->me_sr_adjustment_ctrls.stationary_hme_sad_abs_th            = c->stationary_hme_sad_abs_th;
    m->me_sr_adjustment_ctrls.stationary_me_sr_divisor             = c->stationary_me_sr_divisor;
    m->me_sr_adjustment_ctrls.reduce_me_sr_based_on_hme_sad_abs_th = c->reduce_me_sr_based_on_hme_sad_abs_th;
    m->me_sr_adjustment_ctrls.me_sr_divisor_for_low_hme_sad        = c->me_sr_divisor_for_low_hme_sad;
    m->me_sr_adjustment_ctrls.distance_based_hme_resizing          = c->distance_based_hme_resizing;

    m->mv_based_sa_adj.enabled          = c->mv_sa_adj_enabled;
    m->mv_based_sa_adj.nearest_ref_only = c->mv_sa_adj_nearest_ref_only;
    m->mv_based_sa_adj.mv_size_th       = c->mv_sa_adj_mv_size_th;
    m->mv_based_sa_adj.sa_multiplier    = c->mv_sa_adj_sa_multiplier;

    m->me_8x8_var_ctrls.enabled        = c->me_8x8_var_enabled;
    m->me_8x8_var_ctrls.me_sr_div4_th  = c->me_sr_div4_th;
    m->me_8x8_var_ctrls.me_sr_div2_th  = c->me_sr_div2_th;
    m->me_8x8_var_ctrls.me_sr_mult2_th = c->me_sr_mult2_th;

    m->prehme_ctrl.enable           = c->prehme_enable;
    m->prehme_ctrl.skip_search_line = c->prehme_skip_search_line;
    m->prehme_ctrl.l1_early_exit    = c->prehme_l1_early_exit;
    for (int i = 0; i < 2; i++) {
        m->prehme_ctrl.prehme_sa_cfg[i].sa_min = (SearchArea){c->prehme_sa_cfg[i].sa_min.width,
                                                              c->prehme_sa_cfg[i].sa_min.height};
        m->prehme_ctrl.prehme_sa_cfg[i].sa_max = (SearchArea){c->prehme_sa_cfg[i].sa_max.width,
                                                              c->prehme_sa_cfg[i].sa_max.height};
    }
    m->prune_me_candidates_th      = c->prune_me_candidates_th;
    m->use_best_unipred_cand_only  = c->use_best_unipred_cand_only;
    m->reduce_hme_l0_sr_th_min     = c->reduce_hme_l0_sr_th_min;
    m->reduce_hme_l0_sr_th_max     = c->reduce_hme_l0_sr_th_max;
    m->me_early_exit_th            = c->me_early_exit_th;
    m->me_safe_limit_zz_th         = c->me_safe_limit_zz_th;
    m->prev_me_stage_based_exit_th = c->prev_me_stage_based_exit_th;
}

typedef struct RefJob {
    const svtme_job *job;
    const svtme_pyr *cur;
    const svtme_pyr *refs;
    svtme_ref_record *out;
    svtme_sb_result *sbres;
    uint32_t first, count; /* absolute SB index range */
    PictureParentControlSet *pcs;
    EbPictureBufferDesc *input_pic, *cur_full, *cur_q, *cur_s;
    EbPictureBufferDesc *ref_desc; /* [2][4][3] */
} RefJob;

static void run_range(RefJob *rj) {
    const svtme_job *job = rj->job;
    const uint32_t W = job->width, H = job->height;
    const uint32_t pic_w_b64 = (W + 63) / 64;
    const uint32_t R = svtme_job_ref_slots(job);
    MeContext *me = (MeContext *)calloc(1, sizeof(MeContext));
    apply_controls(me, &job->ctrl);
    me->me_type                     = job->me_type == SVTME_ME_MCTF ? ME_MCTF : ME_OPEN_LOOP;
    me->tf_me_exit_th               = job->tf_me_exit_th;
    me->num_of_list_to_search       = job->num_lists;
    me->num_of_ref_pic_to_search[0] = job->num_refs[0];
    me->num_of_ref_pic_to_search[1] = job->num_lists == 2 ? job->num_refs[1] : 0;
    me->temporal_layer_index        = job->temporal_layer_index;
    me->is_ref                      = job->is_ref;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < me->num_of_ref_pic_to_search[l]; r++) {
            EbPictureBufferDesc *d                  = &rj->ref_desc[(l * 4 + r) * 3];
            me->me_ds_ref_array[l][r].picture_ptr           = &d[0];
            me->me_ds_ref_array[l][r].quarter_picture_ptr   = &d[1];
            me->me_ds_ref_array[l][r].sixteenth_picture_ptr = &d[2];
            me->me_ds_ref_array[l][r].picture_number        = job->ref_picture_number[l][r];
        }
    EbPictureBufferDesc *full = rj->cur_full, *quarter = rj->cur_q, *sixteenth = rj->cur_s;
    MeSbResults *res = rj->pcs->pa_me_data->me_results[0];

    for (uint32_t k = 0; k < rj->count; k++) {
        const uint32_t b64_index = rj->first + k;
        const uint32_t x_b64 = b64_index % pic_w_b64, y_b64 = b64_index / pic_w_b64;
        const uint32_t ox = x_b64 * 64, oy = y_b64 * 64;
        /* me_process.c:183-214 */
        me->b64_src_ptr    = &full->buffer_y[(full->org_y + oy) * full->stride_y + full->org_x + ox];
        me->b64_src_stride = full->stride_y;
        me->quarter_b64_buffer =
            &quarter->buffer_y[(quarter->org_y + (oy >> 1)) * quarter->stride_y + quarter->org_x + (ox >> 1)];
        me->quarter_b64_buffer_stride = quarter->stride_y;
        me->sixteenth_b64_buffer =
            &sixteenth->buffer_y[(sixteenth->org_y + (oy >> 2)) * sixteenth->stride_y + sixteenth->org_x + (ox >> 2)];
        me->sixteenth_b64_buffer_stride = sixteenth->stride_y;
        /* sentinel so un-searched refs are recognisable (their p_sb_best_sad is stale in the reference) */
        memset(me->p_sb_best_sad, 0xFF, sizeof(me->p_sb_best_sad));
        /* zero the SB's candidate outputs so unwritten entries compare equal */
        MeSbResults *r = rj->pcs->pa_me_data->me_results[b64_index];
        memset(r->total_me_candidate_index, 0, SVTME_PU_COUNT);
        memset(r->me_candidate_array, 0, sizeof(MeCandidate) * SVTME_PU_COUNT * SVTME_MAX_PA_ME_CAND);
        memset(r->me_mv_array, 0, sizeof(MvCandidate) * SVTME_PU_COUNT * SVTME_MAX_PA_ME_MV);
        memset(me->me_distortion, 0, sizeof(me->me_distortion));
        me->tf_use_pred_64x64_only_th = 0;

        svt_aom_motion_estimation_b64(rj->pcs, b64_index, ox, oy, me, rj->input_pic);

        svtme_ref_record *o = rj->out + (size_t)(b64_index - job->sb_begin) * R;
        for (int l = 0, slot = 0; l < job->num_lists; l++)
            for (int ri = 0; ri < me->num_of_ref_pic_to_search[l]; ri++, slot++) {
                svtme_ref_record *rec = &o[slot];
                memset(rec, 0, sizeof(*rec));
                memcpy(rec->best_sad, me->p_sb_best_sad[l][ri], sizeof(rec->best_sad));
                memcpy(rec->best_mv, me->p_sb_best_mv[l][ri], sizeof(rec->best_mv));
                rec->hme_sad  = me->search_results[l][ri].hme_sad;
                rec->hme_sc_x = me->search_results[l][ri].hme_sc_x;
                rec->hme_sc_y = me->search_results[l][ri].hme_sc_y;
                rec->zz_sad   = me->zz_sad[l][ri];
                rec->searched = rec->best_sad[0] != 0xFFFFFFFFu;
                rec->do_ref   = me->search_results[l][ri].do_ref;
                rec->tf_early_exit = me->tf_use_pred_64x64_only_th == (uint8_t)~0;
            }
        if (rj->sbres && me->me_type == ME_MCTF) /* no candidates / distortions (motion_estimation.c:3126) */
            memset(rj->sbres + (b64_index - job->sb_begin), 0, sizeof(svtme_sb_result));
        else if (rj->sbres) {
            svtme_sb_result *s = rj->sbres + (b64_index - job->sb_begin);
            memset(s, 0, sizeof(*s));
            memcpy(s->total_me_candidate_index, r->total_me_candidate_index, SVTME_PU_COUNT);
            /* the reference strides these by pa_me_data->max_cand / max_refs */
            const uint32_t mc = rj->pcs->pa_me_data->max_cand, mr = rj->pcs->pa_me_data->max_refs;
            for (int pu = 0; pu < SVTME_PU_COUNT; pu++) {
                memcpy(s->me_candidate_array[pu], &r->me_candidate_array[pu * mc], mc);
                for (uint32_t k = 0; k < mr; k++) s->me_mv_array[pu][k] = r->me_mv_array[pu * mr + k].as_int;
            }
            memcpy(s->me_distortion, me->me_distortion, sizeof(s->me_distortion));
            s->me_8x8_cost_variance     = rj->pcs->me_8x8_cost_variance[b64_index];
            s->rc_me_distortion         = rj->pcs->rc_me_distortion[b64_index];
            s->me_64x64_distortion      = rj->pcs->me_64x64_distortion[b64_index];
            s->me_32x32_distortion      = rj->pcs->me_32x32_distortion[b64_index];
            s->me_16x16_distortion      = rj->pcs->me_16x16_distortion[b64_index];
            s->me_8x8_distortion        = rj->pcs->me_8x8_distortion[b64_index];
            s->stationary_block_present = rj->pcs->stationary_block_present_sb[b64_index];
            s->rc_me_allow_gm           = rj->pcs->rc_me_allow_gm[b64_index];
        }
    }
    (void)res;
    (void)H;
    free(me);
}

static void *thread_main(void *p) {
    run_range((RefJob *)p);
    return NULL;
}

svtme_status svtref_me(const svtme_job *job, const svtme_pyr *cur, const svtme_pyr *refs, svtme_ref_record *out,
                       svtme_sb_result *sbres, int nthreads) {
    ensure_kernels();
    const uint32_t W = job->width, H = job->height;
    if ((W & 7) || (H & 7) || job->num_lists < 1 || job->num_lists > 2)
        return SVTME_ERR_BAD_PARAMETER;
    const uint32_t sb_total = svtme_sb_total(W, H);
    const uint32_t count    = job->sb_count ? job->sb_count : sb_total - job->sb_begin;
    if (job->sb_begin + count > sb_total)
        return SVTME_ERR_BAD_PARAMETER;

    SequenceControlSet *scs       = (SequenceControlSet *)calloc(1, sizeof(SequenceControlSet));
    PictureParentControlSet *pcs  = (PictureParentControlSet *)calloc(1, sizeof(PictureParentControlSet));
    MotionEstimationData *me_data = (MotionEstimationData *)calloc(1, sizeof(MotionEstimationData));
    scs->input_resolution         = (EbInputResolution)job->input_resolution;
    scs->mrp_ctrls.only_l_bwd     = job->only_l_bwd;
    pcs->scs                      = scs;
    pcs->picture_number           = job->picture_number;
    pcs->aligned_width            = (uint16_t)W;
    pcs->aligned_height           = (uint16_t)H;
    pcs->temporal_layer_index     = job->temporal_layer_index;
    pcs->hierarchical_levels      = job->hierarchical_levels;
    pcs->similar_brightness_refs  = job->similar_brightness_refs;
    pcs->is_ref                   = job->is_ref;
    pcs->enable_me_8x8            = job->enable_me_8x8;
    pcs->enable_me_16x16          = job->enable_me_16x16;
    pcs->max_number_of_pus_per_sb = SVTME_PU_COUNT; /* resource_coordination_process.c:425 */
    pcs->gm_ctrls.enabled         = job->gm_enabled;
    pcs->gm_ctrls.use_distance_based_active_th = job->gm_use_distance_based_active_th;
    me_data->max_cand             = job->max_cand;
    me_data->max_refs             = job->max_refs;
    me_data->max_l0               = job->max_l0;
    me_data->b64_total_count      = (uint16_t)sb_total;
    me_data->me_results           = (MeSbResults **)calloc(sb_total, sizeof(MeSbResults *));
    MeSbResults *res_pool         = (MeSbResults *)calloc(sb_total, sizeof(MeSbResults));
    uint8_t *tci = (uint8_t *)calloc((size_t)sb_total * SVTME_PU_COUNT, 1);
    MeCandidate *mca = (MeCandidate *)calloc((size_t)sb_total * SVTME_PU_COUNT * SVTME_MAX_PA_ME_CAND, sizeof(MeCandidate));
    MvCandidate *mva = (MvCandidate *)calloc((size_t)sb_total * SVTME_PU_COUNT * SVTME_MAX_PA_ME_MV, sizeof(MvCandidate));
    for (uint32_t i = 0; i < sb_total; i++) {
        res_pool[i].total_me_candidate_index = tci + (size_t)i * SVTME_PU_COUNT;
        res_pool[i].me_candidate_array       = mca + (size_t)i * SVTME_PU_COUNT * SVTME_MAX_PA_ME_CAND;
        res_pool[i].me_mv_array              = mva + (size_t)i * SVTME_PU_COUNT * SVTME_MAX_PA_ME_MV;
        me_data->me_results[i]               = &res_pool[i];
    }
    pcs->pa_me_data                  = me_data;
    pcs->me_8x8_cost_variance        = (uint32_t *)calloc(sb_total, 4);
    pcs->rc_me_distortion            = (uint32_t *)calloc(sb_total, 4);
    pcs->me_64x64_distortion         = (uint32_t *)calloc(sb_total, 4);
    pcs->me_32x32_distortion         = (uint32_t *)calloc(sb_total, 4);
    pcs->me_16x16_distortion         = (uint32_t *)calloc(sb_total, 4);
    pcs->me_8x8_distortion           = (uint32_t *)calloc(sb_total, 4);
    pcs->stationary_block_present_sb = (uint8_t *)calloc(sb_total, 1);
    pcs->rc_me_allow_gm              = (uint8_t *)calloc(sb_total, 1);
    pcs->b64_geom                    = (B64Geom *)calloc(sb_total, sizeof(B64Geom));
    const uint32_t pic_w_b64 = (W + 63) / 64;
    for (uint32_t i = 0; i < sb_total; i++) { /* pcs.c:1505-1520 */
        B64Geom *g = &pcs->b64_geom[i];
        g->org_x   = (uint16_t)((i % pic_w_b64) * 64);
        g->org_y   = (uint16_t)((i / pic_w_b64) * 64);
        g->width   = (uint8_t)((W - g->org_x) < 64 ? W - g->org_x : 64);
        g->height  = (uint8_t)((H - g->org_y) < 64 ? H - g->org_y : 64);
    }

    EbPictureBufferDesc input_pic, cur_full, cur_q, cur_s;
    set_desc(&cur_full, cur->full, W, H, SVTME_PAD_FULL);
    set_desc(&cur_q, cur->quarter, W / 2, H / 2, SVTME_PAD_QUARTER);
    set_desc(&cur_s, cur->sixteenth, W / 4, H / 4, SVTME_PAD_SIXTEENTH);
    input_pic = cur_full;
    EbPictureBufferDesc ref_desc[2 * 4 * 3];
    memset(ref_desc, 0, sizeof(ref_desc));
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++) {
            const svtme_pyr *p = &refs[l * 4 + r];
            set_desc(&ref_desc[(l * 4 + r) * 3 + 0], p->full, W, H, SVTME_PAD_FULL);
            set_desc(&ref_desc[(l * 4 + r) * 3 + 1], p->quarter, W / 2, H / 2, SVTME_PAD_QUARTER);
            set_desc(&ref_desc[(l * 4 + r) * 3 + 2], p->sixteenth, W / 4, H / 4, SVTME_PAD_SIXTEENTH);
        }

    if (nthreads < 1)
        nthreads = 1;
    if ((uint32_t)nthreads > count)
        nthreads = (int)(count ? count : 1);
    RefJob *jobs = (RefJob *)calloc(nthreads, sizeof(RefJob));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        const uint32_t b = job->sb_begin + (uint32_t)((uint64_t)count * t / nthreads);
        const uint32_t e = job->sb_begin + (uint32_t)((uint64_t)count * (t + 1) / nthreads);
        jobs[t] = (RefJob){job, cur, refs, out, sbres, b, e - b, pcs, &input_pic, &cur_full, &cur_q, &cur_s, ref_desc};
    }
    if (nthreads == 1)
        run_range(&jobs[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, thread_main, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    free(jobs);
    free(th);
    free(pcs->me_8x8_cost_variance);
    free(pcs->rc_me_distortion);
    free(pcs->me_64x64_distortion);
    free(pcs->me_32x32_distortion);
    free(pcs->me_16x16_distortion);
    free(pcs->me_8x8_distortion);
    free(pcs->stationary_block_present_sb);
    free(pcs->rc_me_allow_gm);
    free(pcs->b64_geom);
    free(tci);
    free(mca);
    free(mva);
    free(res_pool);
    free(me_data->me_results);
    free(me_data);
    free(pcs);
    free(scs);
    return SVTME_OK;
}

uint32_t svtme_sb_total(uint32_t width, uint32_t height) { return ((width + 63) / 64) * ((height + 63) / 64); }

uint32_t svtme_job_ref_slots(const svtme_job *job) {
    return job->num_refs[0] + (job->num_lists == 2 ? job->num_refs[1] : 0);
}

/* ---------------------------------------------------------------------------
 * Controls as the reference derives them: svt_aom_sig_deriv_me
 * (enc_mode_config.c:671-808) on a picture whose HME level flags and
 * use_best_me_unipred_cand_only are set as svt_aom_sig_deriv_multi_processes
 * sets them (enc_mode_config.c:1608-1619, 1802-1805). Random access, no
 * screen content, safe_limit_nref as mrp level 10 (enc_handle.c:3542-3543).
 * ------------------------------------------------------------------------- */
void svt_aom_sig_deriv_me(SequenceControlSet *scs, PictureParentControlSet *pcs, MeContext *me_ctx);

static void export_controls(const MeContext *m, svtme_controls *c) {
    memset(c, 0, sizeof(*c));
    c->hme_search_method      = m->hme_search_method;
    c->me_search_method       = m->me_search_method;
    c->enable_hme_flag        = m->enable_hme_flag;
    c->enable_hme_level0_flag = m->enable_hme_level0_flag;
    c->enable_hme_level1_flag = m->enable_hme_level1_flag;
    c->enable_hme_level2_flag = m->enable_hme_level2_flag;
    c->num_hme_sa_w           = (uint8_t)m->num_hme_sa_w;
    c->num_hme_sa_h           = (uint8_t)m->num_hme_sa_h;
    c->hme_l0_sa              = (svtme_area_minmax){{m->hme_l0_sa.sa_min.width, m->hme_l0_sa.sa_min.height},
                                                    {m->hme_l0_sa.sa_max.width, m->hme_l0_sa.sa_max.height}};
    c->hme_l1_sa              = (svtme_area){m->hme_l1_sa.width, m->hme_l1_sa.height};
    c->hme_l2_sa              = (svtme_area){m->hme_l2_sa.width, m->hme_l2_sa.height};
    c->me_sa                  = (svtme_area_minmax){{m->me_sa.sa_min.width, m->me_sa.sa_min.height},
                                                    {m->me_sa.sa_max.width, m->me_sa.sa_max.height}};
    c->enable_me_hme_ref_pruning               = m->me_hme_prune_ctrls.enable_me_hme_ref_pruning;
    c->prune_ref_if_hme_sad_dev_bigger_than_th = m->me_hme_prune_ctrls.prune_ref_if_hme_sad_dev_bigger_than_th;
    c->prune_ref_if_me_sad_dev_bigger_than_th  = m->me_hme_prune_ctrls.prune_ref_if_me_sad_dev_bigger_than_th;
    c->zz_sad_th                               = m->me_hme_prune_ctrls.zz_sad_th;
    c->zz_sad_pct                              = m->me_hme_prune_ctrls.zz_sad_pct;
    c->phme_sad_th                             = m->me_hme_prune_ctrls.phme_sad_th;
    c->phme_sad_pct                            = m->me_hme_prune_ctrls.phme_sad_pct;
    c->enable_me_sr_adjustment                 = m->me_sr_adjustment_ctrls.enable_me_sr_adjustment;
    if (c->enable_me_sr_adjustment) {
        c->reduce_me_sr_based_on_mv_length_th   = m->me_sr_adjustment_ctrls.reduce_me_sr_based_on_mv_length_th;
        c->stationary_hme_sad_abs_th            = m->me_sr_adjustment_ctrls.stationary_hme_sad_abs_th;
        c->stationary_me_sr_divisor             = m->me_sr_adjustment_ctrls.stationary_me_sr_divisor;
        c->reduce_me_sr_based_on_hme_sad_abs_th = m->me_sr_adjustment_ctrls.reduce_me_sr_based_on_hme_sad_abs_th;
        c->me_sr_divisor_for_low_hme_sad        = m->me_sr_adjustment_ctrls.me_sr_divisor_for_low_hme_sad;
        c->distance_based_hme_resizing          = m->me_sr_adjustment_ctrls.distance_based_hme_resizing;
    }
    c->mv_sa_adj_enabled = m->mv_based_sa_adj.enabled;
    if (c->mv_sa_adj_enabled) {
        c->mv_sa_adj_nearest_ref_only = m->mv_based_sa_adj.nearest_ref_only;
        c->mv_sa_adj_mv_size_th       = m->mv_based_sa_adj.mv_size_th;
        c->mv_sa_adj_sa_multiplier    = m->mv_based_sa_adj.sa_multiplier;
    }
    c->me_8x8_var_enabled = m->me_8x8_var_ctrls.enabled;
    if (c->me_8x8_var_enabled) {
        c->me_sr_div4_th  = m->me_8x8_var_ctrls.me_sr_div4_th;
        c->me_sr_div2_th  = m->me_8x8_var_ctrls.me_sr_div2_th;
        c->me_sr_mult2_th = m->me_8x8_var_ctrls.me_sr_mult2_th;
    }
    c->prehme_enable = m->prehme_ctrl.enable;
    if (c->prehme_enable) {
        c->prehme_skip_search_line = m->prehme_ctrl.skip_search_line;
        c->prehme_l1_early_exit    = m->prehme_ctrl.l1_early_exit;
        for (int i = 0; i < 2; i++)
            c->prehme_sa_cfg[i] = (svtme_area_minmax){
                {m->prehme_ctrl.prehme_sa_cfg[i].sa_min.width, m->prehme_ctrl.prehme_sa_cfg[i].sa_min.height},
                {m->prehme_ctrl.prehme_sa_cfg[i].sa_max.width, m->prehme_ctrl.prehme_sa_cfg[i].sa_max.height}};
    }
    c->prune_me_candidates_th      = m->prune_me_candidates_th;
    c->use_best_unipred_cand_only  = m->use_best_unipred_cand_only;
    c->reduce_hme_l0_sr_th_min     = m->reduce_hme_l0_sr_th_min;
    c->reduce_hme_l0_sr_th_max     = m->reduce_hme_l0_sr_th_max;
    c->me_early_exit_th            = m->me_early_exit_th;
    c->me_safe_limit_zz_th         = m->me_safe_limit_zz_th;
    c->prev_me_stage_based_exit_th = m->prev_me_stage_based_exit_th;
}

void svt_aom_sig_deriv_me_tf(PictureParentControlSet *pcs, MeContext *me_ctx);

/* TF-ME controls as the reference sets them for one temporal-filtering ME call:
 * the tf HME enables by tf_ctrls.hme_me_level (enc_mode_config.c:1620-1645),
 * svt_aom_sig_deriv_me_tf (:814-854), then set_hme_search_params_mctf(ctx, 0)
 * (temporal_filtering.c:2759-2767, static there: its level-0 copy restated). */
void svtref_derive_controls_tf(int hme_me_level, int qp_opt, int qp, int input_resolution, svtme_controls *ctrl) {
    SequenceControlSet *scs      = (SequenceControlSet *)calloc(1, sizeof(SequenceControlSet));
    PictureParentControlSet *pcs = (PictureParentControlSet *)calloc(1, sizeof(PictureParentControlSet));
    MeContext *me                = (MeContext *)calloc(1, sizeof(MeContext));
    scs->input_resolution          = (EbInputResolution)input_resolution;
    scs->static_config.qp          = (uint32_t)qp;
    pcs->scs                       = scs;
    pcs->tf_ctrls.hme_me_level     = (uint8_t)hme_me_level;
    pcs->tf_ctrls.qp_opt           = (uint8_t)qp_opt;
    pcs->tf_enable_hme_flag        = 1;
    pcs->tf_enable_hme_level0_flag = 1;
    pcs->tf_enable_hme_level1_flag = hme_me_level <= 2;
    pcs->tf_enable_hme_level2_flag = hme_me_level == 0;
    svt_aom_sig_deriv_me_tf(pcs, me);
    me->hme_l0_sa.sa_min = me->hme_l0_sa_default_tf.sa_min;
    me->hme_l0_sa.sa_max = me->hme_l0_sa_default_tf.sa_max;
    export_controls(me, ctrl);
    free(me);
    free(pcs);
    free(scs);
}

void svtref_derive_controls(int enc_mode, int qp, int input_resolution, int temporal_layer_index,
                            int hierarchical_levels, int frame_rate_q16, svtme_controls *ctrl) {
    SequenceControlSet *scs      = (SequenceControlSet *)calloc(1, sizeof(SequenceControlSet));
    PictureParentControlSet *pcs = (PictureParentControlSet *)calloc(1, sizeof(PictureParentControlSet));
    MeContext *me                = (MeContext *)calloc(1, sizeof(MeContext));
    scs->input_resolution            = (EbInputResolution)input_resolution;
    scs->static_config.pred_structure = 2; /* SVT_AV1_PRED_RANDOM_ACCESS */
    scs->static_config.qp            = (uint32_t)qp;
    scs->static_config.enc_mode      = (EncMode)enc_mode;
    scs->frame_rate                  = (uint32_t)frame_rate_q16;
    scs->mrp_ctrls.safe_limit_nref   = 2;
    scs->mrp_ctrls.safe_limit_zz_th  = 0;
    pcs->scs                         = scs;
    pcs->enc_mode                    = (EncMode)enc_mode;
    pcs->sc_class1                   = 0;
    pcs->temporal_layer_index        = (uint8_t)temporal_layer_index;
    pcs->hierarchical_levels         = (uint8_t)hierarchical_levels;
    pcs->input_resolution            = (EbInputResolution)input_resolution;
    pcs->enable_hme_flag             = 1;
    pcs->enable_hme_level0_flag      = 1;
    pcs->enable_hme_level1_flag      = 1;
    pcs->enable_hme_level2_flag      = enc_mode <= ENC_M6 ? 1 : 0;
    pcs->use_best_me_unipred_cand_only = enc_mode <= ENC_M3 ? 0 : 1;
    svt_aom_sig_deriv_me(scs, pcs, me);
    export_controls(me, ctrl);
    free(me);
    free(pcs);
    free(scs);
}

/* ---------------------------------------------------------------------------
 * Per-kernel entry points: the reference's rtcd pointers as selected by
 * svtref_set_simd (C or AVX2), exported for the kernel-level parity tests.
 * ------------------------------------------------------------------------- */
void svtref_sad_loop_kernel(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                            uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_search_center,
                            int16_t *y_search_center, uint32_t src_stride_raw, uint8_t skip_search_line,
                            int16_t search_area_width, int16_t search_area_height) {
    ensure_kernels();
    svt_sad_loop_kernel(src, src_stride, ref, ref_stride, block_height, block_width, best_sad, x_search_center,
                        y_search_center, src_stride_raw, skip_search_line, search_area_width, search_area_height);
}

uint32_t svtref_nxm_sad_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                               uint32_t height, uint32_t width) {
    ensure_kernels();
    return svt_nxm_sad_kernel(src, src_stride, ref, ref_stride, height, width);
}

uint32_t svt_aom_sad_16b_kernel_c(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                                  uint32_t height, uint32_t width); /* compute_sad_c.c:39 */

uint32_t svtref_sad_16b_kernel(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                               uint32_t height, uint32_t width) {
    return svt_aom_sad_16b_kernel_c(src, src_stride, ref, ref_stride, height, width);
}

void svtref_ext_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                          uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                          uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16, uint32_t mv,
                                          uint32_t *p_sad16x16, uint32_t *p_sad8x8, bool sub_sad) {
    ensure_kernels();
    svt_ext_sad_calculation_8x8_16x16(src, src_stride, ref, ref_stride, p_best_sad_8x8, p_best_sad_16x16,
                                      p_best_mv8x8, p_best_mv16x16, mv, p_sad16x16, p_sad8x8, sub_sad);
}

void svtref_ext_sad_calculation_32x32_64x64(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                            uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                            uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32) {
    ensure_kernels();
    svt_ext_sad_calculation_32x32_64x64(p_sad16x16, p_best_sad_32x32, p_best_sad_64x64, p_best_mv32x32,
                                        p_best_mv64x64, mv, p_sad32x32);
}

void svtref_ext_all_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                              uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                              uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                              uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                              bool sub_sad) {
    ensure_kernels();
    svt_ext_all_sad_calculation_8x8_16x16(src, src_stride, ref, ref_stride, mv, p_best_sad_8x8, p_best_sad_16x16,
                                          p_best_mv8x8, p_best_mv16x16, p_eight_sad16x16, p_eight_sad8x8, sub_sad);
}

void svtref_ext_eight_sad_calculation_32x32_64x64(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                  uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                  uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]) {
    ensure_kernels();
    svt_ext_eight_sad_calculation_32x32_64x64(p_sad16x16, p_best_sad_32x32, p_best_sad_64x64, p_best_mv32x32,
                                              p_best_mv64x64, mv, p_sad32x32);
}

void svtref_initialize_buffer_32bits(uint32_t *pointer, uint32_t count128, uint32_t count32, uint32_t value) {
    ensure_kernels();
    svt_initialize_buffer_32bits(pointer, count128, count32, value);
}

void svtref_downsample_2d(uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                          uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                          uint32_t decim_step) {
    ensure_kernels();
    downsample_2d(input_samples, input_stride, input_area_width, input_area_height, decim_samples, decim_stride,
                  decim_step);
}

void svtref_pme_sad_loop_kernel(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                                uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                                uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                                int16_t search_position_start_x, int16_t search_position_start_y,
                                int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                                int16_t mvx, int16_t mvy) {
    ensure_kernels();
    svt_pme_sad_loop_kernel(mv_cost_params, src, src_stride, ref, ref_stride, block_height, block_width, best_cost,
                            best_mvx, best_mvy, search_position_start_x, search_position_start_y, search_area_width,
                            search_area_height, search_step, mvx, mvy);
}
