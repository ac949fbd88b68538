/*
 * svtme_svt_glue.c — the encoder-side binding of libsvtme.so into SVT-AV1.
 *
 * Compiled INSIDE the reference encoder (it includes the reference's own
 * headers: pcs.h, me_context.h, me_sb_results.h, reference_object.h,
 * aom_dsp_rtcd.h) and linked with libsvtme.so. oracle/encoder.mk links it into
 * the reference encoder built from its unmodified sources, and
 * tests/test_encoder.py checks that the encoder's bitstream is byte-identical
 * with and without it.
 *
 * Picture-job mode (the performance boundary)
 *   svtme_motion_estimation_b64()  drop-in for svt_aom_motion_estimation_b64
 *                                  (motion_estimation.c:3076), same signature.
 *                                  The first call for a picture (PA-ME,
 *                                  me_process.c:266) or for a (picture,
 *                                  reference) pair (TF-ME, temporal_filtering.c:
 *                                  3169) runs ONE job over every SB of the
 *                                  picture; every call then scatters its SB's
 *                                  results exactly where the reference function
 *                                  leaves them. Jobs are asynchronous: the
 *                                  thread that starts one submits it on the next
 *                                  submission lane and waits for its packed
 *                                  output outside every glue lock, so the ME
 *                                  threads of several pictures keep several
 *                                  jobs in flight (uploads, searches and copies
 *                                  overlap). A picture is uploaded as soon as
 *                                  the encoder has decimated it (picture
 *                                  analysis, pic_analysis_process.c:2151), so
 *                                  its DMA and pyramid run while the picture
 *                                  is still in the encoder's earlier stages,
 *                                  and again whenever the encoder rebuilds its
 *                                  1/4 and 1/16 planes (svtme_picture_changed);
 *                                  a job uploads what is not resident yet (on
 *                                  first use). Pictures the job API
 *                                  does not cover (super-resolution / resize
 *                                  scaled references, me_process.c:229-246;
 *                                  the DG detector's HME, me_process.c:115) and
 *                                  jobs that fail run on the encoder's own SB
 *                                  function (the fallback).
 *   Linking with -Wl,--wrap=svt_aom_motion_estimation_b64
 *   -Wl,--wrap=svt_aom_downsample_filtering_input_picture
 *   -Wl,--wrap=svt_post_full_object -Wl,--wrap=svt_av1_enc_init
 *   -Wl,--wrap=svt_av1_enc_deinit and -DSVTME_GLUE_WRAP routes both call sites
 *   of the SB function, every re-decimation outside pic_analysis_process.c,
 *   the end of each picture's analysis and each encoder's set-up and teardown
 *   through this file without editing the encoder's sources.
 *
 * Parity / debug mode
 *   svt_aom_setup_rtcd_hip_parity() registers the per-kernel *_hip rtcd variants
 *                                  over the pointers svt_aom_setup_rtcd_internal
 *                                  set (aom_dsp_rtcd.c:188). Each call becomes a
 *                                  synchronous GPU round trip, so this is for
 *                                  per-kernel parity runs only; picture-job mode
 *                                  registers nothing and mode decision keeps its
 *                                  CPU kernels (svt_pme_sad_loop_kernel,
 *                                  sad_16b_kernel, ...).
 *
 * Environment (read once): SVTME_DEVICE (HIP device, default 0);
 * SVTME_GLUE_STRICT=1 aborts instead of falling back; SVTME_GLUE_VERIFY=1
 * compares every uploaded pyramid with the encoder's own planes, and every
 * picture a job names with the encoder's planes when the job is submitted;
 * SVTME_GLUE_EAGER=0 leaves every upload to the first job that names the picture;
 * SVTME_GLUE_STATS=<file> appends the counters at exit (jobs, SBs, uploads,
 * timing: upload / submit / wait milliseconds, mean job latency, the busy time
 * with a job in flight and served_sb_per_s = SBs of the jobs / busy time; the
 * analysis threads' upload calls (eager_upload_ms), page-locking of encoder
 * buffers (registrations, register_ms) and the one-off pool fill (prefill_ms); and
 * the rtcd check: how many of the pointers parity mode replaces changed since
 * the first SB call, and how many point at this file's HIP wrappers);
 * SVTME_GLUE_RESIDENT caps the resident pictures (default 128); SVTME_GLUE_PIN=0
 * uploads through the library's own page-locked staging
 * (svtme_picture_upload_copy_async) instead of page-locking the encoder's
 * picture buffers and copying straight from them (measured: the staging copies
 * run on the analysis threads under the submission lock and delay jobs by
 * milliseconds in bursts of uploads).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "aom_dsp_rtcd.h"
#include "mcomp.h"
#include "me_context.h"
#include "me_sb_results.h"
#include "pcs.h"
#include "pic_analysis_results.h"
#include "reference_object.h"
#include "enc_mode_config.h"
#include "pd_results.h"
#include "sequence_control_set.h"
#ifdef SVTME_GLUE_WRAP
#include "enc_handle.h"
#endif

#include "svtme.h"

EbErrorType svtme_motion_estimation_b64(PictureParentControlSet *pcs, uint32_t b64_index, uint32_t b64_origin_x,
                                        uint32_t b64_origin_y, MeContext *me_ctx, EbPictureBufferDesc *input_ptr);
void svtme_glue_prefetch_pa(PictureParentControlSet *pcs);
void svtme_glue_prefetch_tf(PictureParentControlSet *centre);
void svtme_picture_changed(PictureParentControlSet *pcs, const EbPictureBufferDesc *full);
void svtme_glue_release(void);
void svt_aom_setup_rtcd_hip_parity(void);
void svtme_controls_from_me_context(svtme_controls *c, const MeContext *m);
void svtme_job_from_pcs(svtme_job *job, const PictureParentControlSet *pcs, const MeContext *me);
void svtme_job_from_tf(svtme_job *job, const PictureParentControlSet *centre, const MeContext *me,
                       const EbPictureBufferDesc *input_ptr);
void svtme_scatter_sb(PictureParentControlSet *pcs, MeContext *me, uint32_t b64_index, uint32_t b64_origin_x,
                      uint32_t b64_origin_y, const svtme_job *job, const svtme_pack_layout *layout,
                      const uint8_t *packed_sb);

void svtme_glue_release_encoder(const void *enc_ctx);

#ifdef SVTME_GLUE_WRAP
EbErrorType __real_svt_aom_motion_estimation_b64(PictureParentControlSet *, uint32_t, uint32_t, uint32_t,
                                                 MeContext *, EbPictureBufferDesc *);
void __real_svt_aom_downsample_filtering_input_picture(PictureParentControlSet *, EbPictureBufferDesc *,
                                                       EbPictureBufferDesc *, EbPictureBufferDesc *);
#define SVTME_ENCODER_ME_B64 __real_svt_aom_motion_estimation_b64
#else
EbErrorType svt_aom_motion_estimation_b64(PictureParentControlSet *, uint32_t, uint32_t, uint32_t, MeContext *,
                                          EbPictureBufferDesc *);
#define SVTME_ENCODER_ME_B64 svt_aom_motion_estimation_b64
#endif

/* ==========================================================================
 * Encoder instances. Each encoder in the process (the channels of --nch, the
 * passes of a multi-pass encode, an application's own instances) gets a range
 * of its own in the library's picture numbers: its numbers + (slot << 48). Two
 * encoders then never share a resident picture, and one encoder's teardown
 * drops exactly its pictures, jobs and page-locked buffers. An encoder is
 * known by the EncodeContext every copy of its SequenceControlSet points to
 * (pcs->scs->enc_ctx: the copies of resource_coordination_process.c:907-938 are
 * struct copies, sequence_control_set.c:297); svt_av1_enc_init's wrap adds its
 * picture-analysis results resource (enc_handle.h:105), which marks the end of
 * each picture's analysis in svt_post_full_object.
 * ======================================================================== */
#define GLUE_MAX_ENC 64
#define GLUE_NS_SHIFT 48
#define GLUE_PN_MASK ((1ull << GLUE_NS_SHIFT) - 1)
typedef struct GlueEnc {
    const void *enc_ctx; /* NULL: a free slot */
    const void *pa_res;  /* its picture-analysis results resource, or NULL */
    const void *pd_res;  /* its picture-decision results resource (the ME tasks), or NULL */
} GlueEnc;
static GlueEnc g_enc[GLUE_MAX_ENC];
static pthread_mutex_t g_enc_mu = PTHREAD_MUTEX_INITIALIZER;
static unsigned long long g_n_encoders, g_n_released; /* slots taken; pictures released at teardowns (g_enc_mu) */

/* slots in use: GLUE_MAX_ENC, or fewer with SVTME_GLUE_MAX_ENC (tests: an encoder
 * beyond the cap runs the encoder's own ME, and must not disturb the others) */
static int enc_cap(void) {
    static int cap;
    int c = __atomic_load_n(&cap, __ATOMIC_ACQUIRE);
    if (!c) {
        const char *e = getenv("SVTME_GLUE_MAX_ENC");
        c             = e && atoi(e) > 0 && atoi(e) < GLUE_MAX_ENC ? atoi(e) : GLUE_MAX_ENC;
        __atomic_store_n(&cap, c, __ATOMIC_RELEASE);
    }
    return c;
}

/* the slot of an encoder, taken on first sight; -1 when every slot is taken */
static int enc_slot(const void *enc_ctx, const void *pa_res, const void *pd_res) {
    if (!enc_ctx)
        return -1;
    for (int i = 0; i < GLUE_MAX_ENC; i++)
        if (__atomic_load_n(&g_enc[i].enc_ctx, __ATOMIC_ACQUIRE) == enc_ctx && !pa_res && !pd_res)
            return i;
    pthread_mutex_lock(&g_enc_mu);
    int k = -1;
    for (int i = 0; i < GLUE_MAX_ENC && k < 0; i++)
        if (g_enc[i].enc_ctx == enc_ctx)
            k = i;
    for (int i = 0; i < enc_cap() && k < 0; i++)
        if (!g_enc[i].enc_ctx) {
            k = i;
            __atomic_store_n(&g_enc[i].enc_ctx, enc_ctx, __ATOMIC_RELEASE);
            g_n_encoders++;
        }
    if (k >= 0 && pa_res)
        __atomic_store_n(&g_enc[k].pa_res, pa_res, __ATOMIC_RELEASE);
    if (k >= 0 && pd_res)
        __atomic_store_n(&g_enc[k].pd_res, pd_res, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&g_enc_mu);
    return k;
}

static int pcs_slot(const PictureParentControlSet *pcs) {
    return enc_slot(pcs->scs ? (const void *)pcs->scs->enc_ctx : NULL, NULL, NULL);
}

/* the library's number of picture pn of the encoder in `slot` */
static uint64_t ns_pn(int slot, uint64_t pn) { return ((uint64_t)(slot < 0 ? 0 : slot) << GLUE_NS_SHIFT) | pn; }

/* ==========================================================================
 * rtcd registration, parity / debug mode only
 * (aom_dsp_rtcd.h:779, 841, 842, 848, 853-856, 863, 868)
 * ======================================================================== */
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
/* the MeCandidate bit-field byte the records carry (me_sb_results.h:28-34) */
_Static_assert(sizeof(MeCandidate) == 1, "MeCandidate is one byte");
_Static_assert(sizeof(MvCandidate) == 4, "MvCandidate is (x, y) int16");

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

/* the rtcd pointers parity mode replaces (aom_dsp_rtcd.h:779, 841-856, 863, 868) */
#define GLUE_RTCD_N 10
static void rtcd_snapshot(void *out[GLUE_RTCD_N]) {
    out[0] = (void *)svt_sad_loop_kernel;
    out[1] = (void *)svt_nxm_sad_kernel;
    out[2] = (void *)svt_ext_sad_calculation_8x8_16x16;
    out[3] = (void *)svt_ext_sad_calculation_32x32_64x64;
    out[4] = (void *)svt_ext_all_sad_calculation_8x8_16x16;
    out[5] = (void *)svt_ext_eight_sad_calculation_32x32_64x64;
    out[6] = (void *)svt_initialize_buffer_32bits;
    out[7] = (void *)downsample_2d;
    out[8] = (void *)sad_16b_kernel;
    out[9] = (void *)svt_pme_sad_loop_kernel;
}
/* the HIP wrappers parity mode registered (NULL until it runs): the exit stats
 * count the pointers that hold them */
static void *g_hip_wrappers[GLUE_RTCD_N];

/* Parity / debug only: call right after svt_aom_setup_rtcd_internal(); the
 * pointers it set become the fallbacks, the HIP variants the active ones. Never
 * call it in picture-job mode: every rtcd call would become a GPU round trip. */
void svt_aom_setup_rtcd_hip_parity(void) {
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
    rtcd_snapshot(g_hip_wrappers);
}

/* ==========================================================================
 * Controls: the MeContext fields svt_aom_sig_deriv_me[_tf] set (me_context.h:280-509)
 * ======================================================================== */
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

/* ==========================================================================
 * Jobs
 * ======================================================================== */
static uint32_t align8(uint32_t v) { return (v + 7u) & ~7u; }

/* One PA-ME picture job: the fields me_process.c:217-261 and
 * svt_aom_motion_estimation_b64 read from the PCS, the ME context and the
 * reference pictures' PA objects (me_ds_ref_array, set per SB by
 * me_process.c:248-262 before the call). */
void svtme_job_from_pcs(svtme_job *job, const PictureParentControlSet *pcs, const MeContext *me) {
    memset(job, 0, sizeof(*job));
    const int slot      = pcs_slot(pcs); /* the encoder's picture-number range */
    job->picture_number = ns_pn(slot, pcs->picture_number);
    job->width          = pcs->aligned_width;
    job->height         = pcs->aligned_height;
    job->num_lists      = me->num_of_list_to_search;
    job->num_refs[0]    = me->num_of_ref_pic_to_search[0];
    job->num_refs[1]    = job->num_lists == 2 ? me->num_of_ref_pic_to_search[1] : 0;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++)
            job->ref_picture_number[l][r] = ns_pn(slot, me->me_ds_ref_array[l][r].picture_number);
    job->temporal_layer_index            = me->temporal_layer_index;
    job->is_ref                          = me->is_ref;
    job->hierarchical_levels             = pcs->hierarchical_levels;
    job->similar_brightness_refs         = pcs->similar_brightness_refs;
    job->enable_me_8x8                   = pcs->enable_me_8x8;
    job->enable_me_16x16                 = pcs->enable_me_16x16;
    job->max_cand                        = pcs->pa_me_data->max_cand;
    job->max_refs                        = pcs->pa_me_data->max_refs;
    job->max_l0                          = pcs->pa_me_data->max_l0;
    job->only_l_bwd                      = pcs->scs->mrp_ctrls.only_l_bwd;
    job->input_resolution                = (uint8_t)pcs->scs->input_resolution;
    job->gm_enabled                      = pcs->gm_ctrls.enabled;
    job->gm_use_distance_based_active_th = pcs->gm_ctrls.use_distance_based_active_th;
    job->me_type                         = SVTME_ME_OPEN_LOOP;
    svtme_controls_from_me_context(&job->ctrl, me);
}

/* One TF-ME job: the central picture against the one reference
 * temporal_filtering.c:3127-3168 set up (list 0, ref 0) with the TF controls of
 * svt_aom_sig_deriv_me_tf + set_hme_search_params_mctf. */
void svtme_job_from_tf(svtme_job *job, const PictureParentControlSet *centre, const MeContext *me,
                       const EbPictureBufferDesc *input_ptr) {
    memset(job, 0, sizeof(*job));
    const int slot             = pcs_slot(centre);
    job->picture_number        = ns_pn(slot, centre->picture_number);
    job->width                 = align8(input_ptr->width); /* motion_estimation.c:3093-3094 */
    job->height                = align8(input_ptr->height);
    job->num_lists             = 1;
    job->num_refs[0]           = 1;
    job->ref_picture_number[0][0] = ns_pn(slot, me->me_ds_ref_array[0][0].picture_number);
    job->temporal_layer_index  = me->temporal_layer_index;
    job->is_ref                = me->is_ref;
    job->hierarchical_levels   = centre->hierarchical_levels;
    job->input_resolution      = (uint8_t)centre->scs->input_resolution;
    job->me_type               = SVTME_ME_MCTF;
    job->tf_me_exit_th         = me->tf_me_exit_th;
    svtme_controls_from_me_context(&job->ctrl, me);
    /* svt_aom_sig_deriv_me_tf leaves these two PA-ME candidate controls as the ME
     * thread's last PA picture set them; a TF job has no candidate arrays
     * (motion_estimation.c:3126), so they do not change it: zero, so that the
     * same pair is the same job whichever thread asks for it */
    job->ctrl.prune_me_candidates_th     = 0;
    job->ctrl.use_best_unipred_cand_only = 0;
}

/* ==========================================================================
 * Outputs of one SB back into the reference's storage, exactly where
 * svt_aom_motion_estimation_b64 leaves them, from the SB's packed bytes
 * (svtme_pack_layout, include/svtme.h)
 * ======================================================================== */
/* The pack layout a job's consumer reads: TF-ME takes whole records (the 85-PU
 * winners of its reference, temporal_filtering.c:1867-1869, 2232-2233); PA-ME
 * takes the record tails and the SB results sized by its MeSbResults
 * allocation (pcs.c:91-117; 85, 21 without 8x8, 5 without 16x16 PUs, the
 * use_me_pu rule of motion_estimation.c:2561-2563). */
static svtme_pack_layout layout_of(const PictureParentControlSet *pcs, const svtme_job *job) {
    svtme_pack_layout L;
    memset(&L, 0, sizeof(L));
    if (job->me_type == SVTME_ME_MCTF) {
        L.full_records = 1;
        return L;
    }
    L.n_pus      = (uint16_t)(pcs->enable_me_16x16
                                  ? (pcs->enable_me_8x8 ? pcs->max_number_of_pus_per_sb : MAX_SB64_PU_COUNT_NO_8X8)
                                  : MAX_SB64_PU_COUNT_WO_16X16);
    L.max_cand   = pcs->pa_me_data->max_cand;
    L.max_refs   = pcs->pa_me_data->max_refs;
    L.sb_results = 1;
    return L;
}

void svtme_scatter_sb(PictureParentControlSet *pcs, MeContext *me, uint32_t b64_index, uint32_t b64_origin_x,
                      uint32_t b64_origin_y, const svtme_job *job, const svtme_pack_layout *L, const uint8_t *p) {
    /* :3093-3100 */
    me->b64_width  = (job->width - b64_origin_x) < 64 ? job->width - b64_origin_x : 64;
    me->b64_height = (job->height - b64_origin_y) < 64 ? job->height - b64_origin_y : 64;
    /* init_me_hme_data (:3047-3069): every (list, ref) slot */
    memset(me->p_sb_best_mv, 0, sizeof(me->p_sb_best_mv));
    for (int l = 0; l < MAX_NUM_OF_REF_PIC_LIST; l++)
        for (int r = 0; r < REF_LIST_MAX_DEPTH; r++) {
            if (job->me_type != SVTME_ME_MCTF)
                me->search_results[l][r].list_i = (uint8_t)l;
            me->search_results[l][r].ref_i  = (uint8_t)r;
            me->search_results[l][r].do_ref = 1;
            me->search_results[l][r].hme_sad = MAX_U32;
            me->reduce_me_sr_divisor[l][r]  = 1;
            me->zz_sad[l][r]                = (uint32_t)~0;
        }
    /* per-reference state after the SB (search_results, me_context.h:459); with
     * whole records also the integer-search winners p_sb_best_* and the p_best_*
     * views of the last searched reference (:1368-1384), which TF reads. PA-ME's
     * consumer reads only MeSbResults and the PCS arrays below (me_process.c:
     * 266-290), so its jobs carry the record tails alone. */
    const uint32_t rsz = L->full_records ? (uint32_t)sizeof(svtme_ref_record) : (uint32_t)sizeof(svtme_record_tail);
    const uint8_t *rp  = p;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++, rp += rsz) {
            svtme_record_tail t;
            memcpy(&t, L->full_records ? rp + offsetof(svtme_ref_record, hme_sad) : rp, sizeof(t));
            SearchResults *sr = &me->search_results[l][r];
            sr->hme_sc_x      = t.hme_sc_x;
            sr->hme_sc_y      = t.hme_sc_y;
            sr->hme_sad       = t.hme_sad;
            sr->do_ref        = t.do_ref;
            me->zz_sad[l][r]  = t.zz_sad;
            if (!t.searched || !L->full_records)
                continue; /* the reference leaves p_sb_best_sad untouched and p_sb_best_mv zero */
            const svtme_ref_record *rec = (const svtme_ref_record *)rp;
            memcpy(me->p_sb_best_sad[l][r], rec->best_sad, sizeof(rec->best_sad));
            memcpy(me->p_sb_best_mv[l][r], rec->best_mv, sizeof(rec->best_mv));
            me->p_best_sad_64x64 = &me->p_sb_best_sad[l][r][ME_TIER_ZERO_PU_64x64];
            me->p_best_sad_32x32 = &me->p_sb_best_sad[l][r][ME_TIER_ZERO_PU_32x32_0];
            me->p_best_sad_16x16 = &me->p_sb_best_sad[l][r][ME_TIER_ZERO_PU_16x16_0];
            me->p_best_sad_8x8   = &me->p_sb_best_sad[l][r][ME_TIER_ZERO_PU_8x8_0];
            me->p_best_mv64x64   = &me->p_sb_best_mv[l][r][ME_TIER_ZERO_PU_64x64];
            me->p_best_mv32x32   = &me->p_sb_best_mv[l][r][ME_TIER_ZERO_PU_32x32_0];
            me->p_best_mv16x16   = &me->p_sb_best_mv[l][r][ME_TIER_ZERO_PU_16x16_0];
            me->p_best_mv8x8     = &me->p_sb_best_mv[l][r][ME_TIER_ZERO_PU_8x8_0];
        }
    if (job->me_type == SVTME_ME_MCTF) {
        svtme_record_tail t0;
        memcpy(&t0, p + offsetof(svtme_ref_record, hme_sad), sizeof(t0));
        if (t0.tf_early_exit) /* :3109-3112 */
            me->tf_use_pred_64x64_only_th = (uint8_t)~0;
        return;
    }
    /* the SB results, packed (svtme_pack_layout) */
    uint32_t v[6];
    memcpy(v, rp, sizeof(v));
    rp += sizeof(v);
    /* compute_distortion (:2964-3007) and perform_gm_detection (:2838-2961) */
    memcpy(me->me_distortion, rp, sizeof(me->me_distortion));
    rp += sizeof(me->me_distortion);
    const uint8_t *mvs = rp;
    rp += 4u * L->n_pus * L->max_refs;
    const uint8_t stationary = rp[0], allow_gm = rp[1];
    rp += 4;
    const uint8_t *total = rp, *cand = rp + L->n_pus;
    /* candidates (:2532-2835) into MeSbResults (me_sb_results.h:44); the
     * candidates past total_me_candidate_index are not written */
    MeSbResults *res  = pcs->pa_me_data->me_results[b64_index];
    const uint32_t mc = L->max_cand, mr = L->max_refs;
    for (uint32_t pu = 0; pu < L->n_pus; pu++) {
        const uint32_t n = total[pu] < mc ? total[pu] : mc;
        res->total_me_candidate_index[pu] = total[pu];
        memcpy(&res->me_candidate_array[pu * mc], cand + pu * mc, n);
        memcpy(&res->me_mv_array[pu * mr], mvs + 4u * pu * mr, 4u * mr);
    }
    pcs->me_8x8_cost_variance[b64_index]        = v[0];
    pcs->rc_me_distortion[b64_index]            = v[1];
    pcs->me_64x64_distortion[b64_index]         = v[2];
    pcs->me_32x32_distortion[b64_index]         = v[3];
    pcs->me_16x16_distortion[b64_index]         = v[4];
    pcs->me_8x8_distortion[b64_index]           = v[5];
    pcs->stationary_block_present_sb[b64_index] = stationary;
    pcs->rc_me_allow_gm[b64_index]              = allow_gm;
}

/* ==========================================================================
 * Picture-job service of the SB function
 *
 * The encoder's ME threads take the SB segments of whichever pictures are ready
 * (me_process.c:97-174, several pictures at once). The first SB call of a
 * picture (or of a TF reference) makes its pictures resident (asynchronous
 * uploads), submits ONE job over all of its SBs on the next submission lane and
 * waits for the job's packed output outside every glue lock, so the threads of
 * other pictures upload and submit meanwhile: several jobs are in flight, their
 * uploads, searches and copies overlapping on the GPU's copy engines and CUs.
 * Every other SB call of the picture waits for that job and scatters its SB.
 * ======================================================================== */
typedef struct GlueJob {
    svtme_job job;
    svtme_pack_layout layout;
    uint32_t n_sb, R, stride;
    uint8_t *packed;   /* page-locked host buffer (pool) */
    size_t packed_cap;
    uint32_t served;
    uint32_t users;    /* threads between finding the job and the end of their scatter */
    int state;         /* 0 running, 1 done, -1 failed (its SBs run on the encoder's function) */
    uint64_t ticket;   /* a prefetched job's ticket until a thread takes it to wait (0: none) */
    int prefetched;    /* submitted when picture decision posted the picture's ME tasks */
    int stale;         /* a picture it reads was re-decimated after it ran: later calls start a new job */
    struct GlueJob *next;
} GlueJob;

typedef struct GluePic {
    uint64_t pn;
    uint32_t w, h;
    uint64_t last_use;
    int dirty; /* the encoder rebuilt its planes: the next job re-uploads it in place */
} GluePic;

typedef struct GlueBuf {
    uint8_t *p;
    size_t cap;
} GlueBuf;

typedef struct GlueReg { /* an encoder picture span page-locked for uploads */
    const void *p;
    uint64_t bytes;
    int slot; /* the encoder whose buffer it is */
} GlueReg;

typedef struct GlueTrace { /* one job (SVTME_GLUE_TRACE) */
    uint64_t pn;
    int tf;
    uint32_t n_sb, inflight, uploads;
    double t_create, t_submitted, t_done, upload_s;
    float gpu_ms, copy_ms; /* GPU-side: lane turn -> packed output; -> host memory (svtme_ticket_wait_timed) */
    double t_prep, t_locked; /* job(s) built and buffers taken; the GPU lock held (submission starts) */
} GlueTrace;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static struct {
    pthread_once_t once;
    pthread_mutex_t mu;  /* job list, buffer pool, counters */
    pthread_cond_t cv;   /* a job finished */
    pthread_mutex_t gpu; /* one thread uploads / submits at a time (not held while waiting) */
    pthread_mutex_t reg; /* the page-locked encoder buffers (regs) */
    svtme_ctx *ctx;
    int strict, verify, eager, pin, tf_batch, prefetch, max_resident;
    const char *stats_path, *trace_path;
    GlueTrace *trace;
    uint32_t n_trace, cap_trace;
    double t0;
    GlueJob *jobs;
    GluePic *pics;
    uint32_t n_pics, cap_pics;
    uint64_t tick;
    uint32_t next_lane;
    GlueBuf pool[2 * SVTME_MAX_TICKETS];
    uint32_t n_pool;
    GlueReg *regs; /* (G.reg) */
    uint32_t n_regs, cap_regs;
    void *rtcd0[GLUE_RTCD_N]; /* the rtcd pointers at the first SB call (after svt_aom_setup_rtcd_internal) */
    uint32_t inflight;        /* jobs between their submission and their output in host memory */
    double busy_t0;
    /* the last GLUE_CHG_LOG pictures svtme_picture_changed saw (G.mu): a prefetched job is
     * unlisted while it is submitted, so its relink checks the changes made meanwhile */
#define GLUE_CHG_LOG 64
    uint64_t chg_pn[GLUE_CHG_LOG], chg_seq;
    struct {
        unsigned long long pa_jobs, tf_jobs, sbs, fallback_sbs, uploads, invalidations, evictions, verified, stale;
        unsigned long long job_sbs, max_inflight, unpinned, eager_uploads, verified_job, registrations;
        unsigned long long tf_batched, unused_jobs, launches, prefetched, prefetch_hits, prefetch_ready;
        unsigned long long init_registrations; /* PA pool buffers page-locked at svt_av1_enc_init */
        double upload_s, submit_s, wait_s, job_s, busy_s, eager_s, prefill_s, register_s;
    } n;
} G = {PTHREAD_ONCE_INIT, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_MUTEX_INITIALIZER,
     PTHREAD_MUTEX_INITIALIZER};

static void glue_trace_at_exit(void) {
    FILE *f = fopen(G.trace_path, "w");
    if (!f)
        return;
    for (uint32_t i = 0; i < G.n_trace; i++) {
        const GlueTrace *t = &G.trace[i];
        fprintf(f, "{\"pn\": %llu, \"tf\": %d, \"sbs\": %u, \"inflight\": %u, \"uploads\": %u, "
                   "\"upload_ms\": %.4f, \"create_ms\": %.4f, \"submitted_ms\": %.4f, \"done_ms\": %.4f, "
                   "\"gpu_ms\": %.4f, \"copy_ms\": %.4f, \"prep_ms\": %.4f, \"lock_ms\": %.4f}\n",
                (unsigned long long)(t->pn & GLUE_PN_MASK), t->tf, t->n_sb, t->inflight, t->uploads, 1e3 * t->upload_s,
                1e3 * (t->t_create - G.t0), 1e3 * (t->t_submitted - G.t0), 1e3 * (t->t_done - G.t0), t->gpu_ms,
                t->copy_ms, t->t_prep ? 1e3 * (t->t_prep - t->t_create) : 0.0,
                t->t_prep ? 1e3 * (t->t_locked - t->t_prep) : 0.0);
    }
    fclose(f);
}

/* one trace line (G.mu held) */
static void trace_add(const GlueTrace *t) {
    if (G.n_trace == G.cap_trace) {
        G.cap_trace = G.cap_trace ? 2 * G.cap_trace : 256;
        G.trace     = (GlueTrace *)realloc(G.trace, G.cap_trace * sizeof(GlueTrace));
        if (!G.trace)
            abort();
    }
    G.trace[G.n_trace++] = *t;
}

static void glue_stats_at_exit(void) {
    FILE *f = fopen(G.stats_path, "a");
    if (!f)
        return;
    /* rtcd check: every pointer parity mode replaces, against its value at the first SB call,
     * and how many point at this file's HIP wrappers */
    void *rt[GLUE_RTCD_N];
    rtcd_snapshot(rt);
    int changed = 0;
    for (int i = 0; i < GLUE_RTCD_N; i++) changed += G.rtcd0[i] != NULL && rt[i] != G.rtcd0[i];
    int hip = 0;
    for (int i = 0; i < GLUE_RTCD_N; i++) hip += g_hip_wrappers[i] != NULL && rt[i] == g_hip_wrappers[i];
    const double rate = G.n.busy_s > 0 ? (double)G.n.job_sbs / G.n.busy_s : 0.0;
    /* the same with the picture-analysis threads' upload calls counted as busy time */
    const double rate_up = G.n.busy_s + G.n.eager_s > 0 ? (double)G.n.job_sbs / (G.n.busy_s + G.n.eager_s) : 0.0;
    const unsigned long long jobs = G.n.pa_jobs + G.n.tf_jobs;
    fprintf(f,
            "{\"backend\": %d, \"pa_jobs\": %llu, \"tf_jobs\": %llu, \"sbs\": %llu, \"fallback_sbs\": %llu, "
            "\"uploads\": %llu, \"invalidations\": %llu, \"evictions\": %llu, \"verified_planes\": %llu, \"verified_job_planes\": %llu, "
            "\"stale_jobs\": %llu, \"unpinned_uploads\": %llu, \"rtcd_checked\": %d, \"rtcd_changed\": %d, \"rtcd_hip\": %d, "
            "\"job_sbs\": %llu, \"max_inflight\": %llu, \"upload_ms\": %.3f, \"submit_ms\": %.3f, \"wait_ms\": %.3f, "
            "\"job_latency_ms\": %.4f, \"busy_ms\": %.3f, \"served_sb_per_s\": %.1f, \"eager_uploads\": %llu, "
            "\"eager_upload_ms\": %.3f, \"served_sb_per_s_with_uploads\": %.1f, \"prefill_ms\": %.3f, "
            "\"registrations\": %llu, \"register_ms\": %.3f, \"encoders\": %llu, \"released_at_teardown\": %llu, "
            "\"tf_batched\": %llu, \"unused_jobs\": %llu, \"launches\": %llu, \"prefetched\": %llu, "
            "\"prefetch_hits\": %llu, \"prefetch_ready\": %llu, \"init_registrations\": %llu}\n",
            G.ctx != NULL, G.n.pa_jobs, G.n.tf_jobs, G.n.sbs, G.n.fallback_sbs, G.n.uploads, G.n.invalidations,
            G.n.evictions, G.n.verified, G.n.verified_job, G.n.stale, G.n.unpinned, G.rtcd0[0] != NULL ? GLUE_RTCD_N : 0, changed, hip, G.n.job_sbs,
            G.n.max_inflight, 1e3 * G.n.upload_s, 1e3 * G.n.submit_s, 1e3 * G.n.wait_s,
            jobs ? 1e3 * G.n.job_s / (double)jobs : 0.0, 1e3 * G.n.busy_s, rate, G.n.eager_uploads, 1e3 * G.n.eager_s,
            rate_up, 1e3 * G.n.prefill_s, G.n.registrations, 1e3 * G.n.register_s, g_n_encoders, g_n_released,
            G.n.tf_batched, G.n.unused_jobs, G.n.launches, G.n.prefetched, G.n.prefetch_hits, G.n.prefetch_ready,
            G.n.init_registrations);
    fclose(f);
}

static void glue_init(void) {
    const char *e;
    rtcd_snapshot(G.rtcd0);
    G.strict       = (e = getenv("SVTME_GLUE_STRICT")) && atoi(e);
    G.verify       = (e = getenv("SVTME_GLUE_VERIFY")) && atoi(e);
    G.eager        = !(e = getenv("SVTME_GLUE_EAGER")) || atoi(e);
    G.pin          = !(e = getenv("SVTME_GLUE_PIN")) || atoi(e);
    G.tf_batch     = !(e = getenv("SVTME_GLUE_TF_BATCH")) || atoi(e);
    G.prefetch     = !(e = getenv("SVTME_GLUE_PREFETCH")) || atoi(e);
    G.max_resident = (e = getenv("SVTME_GLUE_RESIDENT")) ? atoi(e) : 128;
    if (G.max_resident < 9)
        G.max_resident = 9; /* a job names at most 1 + 8 pictures */
    G.stats_path = getenv("SVTME_GLUE_STATS");
    if (G.stats_path)
        atexit(glue_stats_at_exit);
    G.trace_path = getenv("SVTME_GLUE_TRACE");
    if (G.trace_path)
        atexit(glue_trace_at_exit);
    G.t0 = now_s();
    const int dev = (e = getenv("SVTME_DEVICE")) ? atoi(e) : 0;
    if (svtme_ctx_create(dev, &G.ctx) != SVTME_OK) {
        fprintf(stderr, "svtme glue: no ME device (%s); motion estimation runs on the CPU\n", svtme_last_error());
        G.ctx = NULL;
        if (G.strict)
            abort();
    }
}

static void glue_fallback(const char *what) {
    fprintf(stderr, "svtme glue: %s (%s); the SB runs on the encoder's ME\n", what, svtme_last_error());
    if (G.strict)
        abort();
}

/* ---- page-locked output buffers (G.mu held) */
/* The largest packed output any job of an n_sb-SB picture can have: a PA-ME
 * layout with every PU, candidate and reference slot, or whole TF-ME records */
static size_t buf_worst(uint32_t n_sb) {
    const svtme_pack_layout pa = {SVTME_PU_COUNT, SVTME_MAX_PA_ME_CAND, SVTME_MAX_PA_ME_MV, 0, 1, {0, 0}};
    const svtme_pack_layout tf = {0, 0, 0, 1, 0, {0, 0}};
    const uint32_t a = svtme_packed_sb_bytes(&pa, 8), b = svtme_packed_sb_bytes(&tf, 8);
    return (size_t)n_sb * (a > b ? a : b);
}

#define GLUE_POOL_BATCH 6 /* buffers page-locked together when the pool runs dry */
#define GLUE_RESERVED_PICS 64 /* picture buffers reserved on the device ahead of the first job */

/* Ahead of the first job (called once, from the first picture-analysis upload,
 * no glue lock held): page-lock a batch of worst-case output buffers for the
 * pool, and size the library's device scratch and first tickets (svtme_reserve),
 * so that the first jobs of an encode allocate nothing */
static void buf_prefill(uint32_t w, uint32_t h) {
    static int done;
    if (__atomic_exchange_n(&done, 1, __ATOMIC_ACQ_REL))
        return;
    const double t0 = now_s();
    const size_t sz = (buf_worst(svtme_sb_total(w, h)) + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    uint8_t *b[GLUE_POOL_BATCH];
    int n = 0;
    for (; n < GLUE_POOL_BATCH; n++)
        if (!(b[n] = (uint8_t *)svtme_host_alloc(sz)))
            break;
    (void)svtme_reserve(G.ctx, w, h, 8, GLUE_POOL_BATCH);
    /* device memory for the first pictures: their uploads allocate nothing */
    (void)svtme_reserve_pictures(G.ctx, w, h, G.max_resident < GLUE_RESERVED_PICS ? G.max_resident : GLUE_RESERVED_PICS);
    pthread_mutex_lock(&G.mu);
    for (int k = 0; k < n; k++) {
        if (G.n_pool < sizeof(G.pool) / sizeof(G.pool[0])) {
            G.pool[G.n_pool].p = b[k], G.pool[G.n_pool].cap = sz;
            G.n_pool++;
        } else
            svtme_host_free(b[k]);
    }
    G.n.prefill_s = now_s() - t0;
    pthread_mutex_unlock(&G.mu);
}

/* once per process: the upload stream created and one blocking upload of a small
 * picture under a number no encoder uses (its first kernel launches load the
 * library's code object), then released */
static void glue_warm(void) {
    static int done;
    static uint8_t plane[64 * 64];
    if (__atomic_exchange_n(&done, 1, __ATOMIC_ACQ_REL))
        return;
    const uint64_t pn = ~(uint64_t)0;
    (void)svtme_upload_stream(G.ctx);
    if (svtme_picture_upload(G.ctx, pn, plane, 64, 64, 64) == SVTME_OK)
        (void)svtme_picture_release(G.ctx, pn);
}

static int buf_take(GlueJob *j, size_t need, size_t worst) {
    int best = -1;
    for (uint32_t i = 0; i < G.n_pool; i++)
        if (G.pool[i].cap >= need && (best < 0 || G.pool[i].cap < G.pool[best].cap))
            best = (int)i;
    if (best >= 0) {
        j->packed = G.pool[best].p, j->packed_cap = G.pool[best].cap;
        G.pool[best] = G.pool[--G.n_pool];
        return 0;
    }
    /* new buffers hold the largest output a job of the largest picture seen so far
     * can have (rounded to 1 MB), so the pool serves every later job whatever its
     * layout; page-locking costs milliseconds, so a batch is made at once (the
     * first jobs of an encode would otherwise pay it one job at a time) */
    static size_t largest;
    largest    = need > largest ? need : largest;
    largest    = worst > largest ? worst : largest;
    const size_t sz = (largest + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    j->packed     = (uint8_t *)svtme_host_alloc(sz);
    j->packed_cap = sz;
    if (!j->packed)
        return -1;
    for (int k = 1; k < GLUE_POOL_BATCH && G.n_pool < sizeof(G.pool) / sizeof(G.pool[0]); k++) {
        uint8_t *p = (uint8_t *)svtme_host_alloc(sz);
        if (!p)
            break;
        G.pool[G.n_pool].p = p, G.pool[G.n_pool].cap = sz;
        G.n_pool++;
    }
    return 0;
}

static void buf_give(GlueJob *j) {
    if (!j->packed)
        return;
    if (G.n_pool < sizeof(G.pool) / sizeof(G.pool[0])) {
        G.pool[G.n_pool].p = j->packed, G.pool[G.n_pool].cap = j->packed_cap;
        G.n_pool++;
    } else
        svtme_host_free(j->packed);
    j->packed = NULL;
}

/* ---- residency (G.gpu held) */
static GluePic *pic_find(uint64_t pn) {
    for (uint32_t i = 0; i < G.n_pics; i++)
        if (G.pics[i].pn == pn)
            return &G.pics[i];
    return NULL;
}

static int verify_level(uint64_t pn, int level, const EbPictureBufferDesc *d) {
    uint32_t S, w, h, pad;
    if (svtme_picture_download(G.ctx, pn, level, NULL, &S, &w, &h, &pad) != SVTME_OK)
        return -1;
    uint8_t *buf = (uint8_t *)malloc((size_t)S * (h + 2 * pad));
    if (!buf || svtme_picture_download(G.ctx, pn, level, buf, &S, &w, &h, &pad) != SVTME_OK) {
        free(buf);
        return -1;
    }
    /* compare the searchable extent: the picture and the padding both sides keep */
    const int px = (int)pad < d->org_x ? (int)pad : d->org_x, py = (int)pad < d->org_y ? (int)pad : d->org_y;
    int bad = 0;
    for (int y = -py; y < (int)h + py && !bad; y++) {
        const uint8_t *a = buf + (size_t)(y + (int)pad) * S + pad - px;
        const uint8_t *b = d->buffer_y + (ptrdiff_t)(y + d->org_y) * d->stride_y + d->org_x - px;
        bad = memcmp(a, b, w + 2 * px) != 0;
    }
    free(buf);
    return bad;
}

/* Make picture pn resident with the encoder's current planes of it: an
 * asynchronous upload (the library stages the rows, the pyramid is built on its
 * upload stream, and the first job reading the picture waits for it on the GPU). */
/* Page-lock the span an upload reads, once per encoder buffer: the encoder
 * keeps its input picture buffers from svt_av1_enc_init to svt_av1_enc_deinit
 * and recycles them, so a buffer is locked on its first upload and every later
 * upload from it is one DMA with no staging pass through the CPU (busy with the
 * encoder's threads). Locking takes a fraction of a millisecond, so it runs
 * under its own lock, before the upload takes G.gpu (the picture-analysis
 * thread of a new buffer does not hold up job submissions). svtme_glue_release
 * (called by the svt_av1_enc_deinit wrap) unlocks them all before the encoder
 * frees them. */
static void pin_span(const void *p, uint64_t bytes, int slot) {
    pthread_mutex_lock(&G.reg);
    for (uint32_t i = 0; i < G.n_regs; i++) // inside a range locked already (e.g. a whole buffer at encoder init)
        if ((const uint8_t *)p >= (const uint8_t *)G.regs[i].p &&
            (const uint8_t *)p + bytes <= (const uint8_t *)G.regs[i].p + G.regs[i].bytes) {
            pthread_mutex_unlock(&G.reg);
            return;
        }
    for (uint32_t i = 0; i < G.n_regs; i++)
        if (G.regs[i].p == p) {
            if (G.regs[i].bytes >= bytes) {
                pthread_mutex_unlock(&G.reg);
                return;
            }
            svtme_sync(G.ctx); /* the uploads queued from the old span have run */
            svtme_host_unregister((void *)p);
            G.regs[i] = G.regs[--G.n_regs];
            break;
        }
    if (G.n_regs == G.cap_regs) {
        G.cap_regs = G.cap_regs ? 2 * G.cap_regs : 64;
        G.regs     = (GlueReg *)realloc(G.regs, G.cap_regs * sizeof(GlueReg));
        if (!G.regs)
            abort();
    }
    const double t0 = now_s();
    if (svtme_host_register((void *)p, bytes) == SVTME_OK) {
        G.regs[G.n_regs].p = p, G.regs[G.n_regs].bytes = bytes, G.regs[G.n_regs].slot = slot;
        G.n_regs++;
    } else
        G.n.unpinned++;
    const double t1 = now_s();
    G.n.registrations++;
    G.n.register_s += t1 - t0;
    pthread_mutex_unlock(&G.reg);
    if (G.trace_path) { /* (tf 3: a registration, beside the jobs and uploads it may hold up) */
        const GlueTrace t = {0, 3, 0, 0, 0, t0, t0, t1, t1 - t0, 0, 0, 0, 0};
        pthread_mutex_lock(&G.mu);
        trace_add(&t);
        pthread_mutex_unlock(&G.mu);
    }
}

/* the span of the rows an upload of the w x h visible samples of `full` reads */
static const uint8_t *span_of(const EbPictureBufferDesc *full, uint32_t w, uint32_t h, uint64_t *bytes) {
    *bytes = (uint64_t)(h - 1) * full->stride_y + w;
    return full->buffer_y + (size_t)full->org_y * full->stride_y + full->org_x;
}

/* An encoder's teardown (the svt_av1_enc_deinit wrap, before the encoder frees
 * its buffers): once the work queued for it has run, unlock its page-locked
 * buffers, release its resident pictures, drop its finished jobs and free its
 * slot, so that a later encoder (the next pass, another channel) starts from
 * nothing of it. slot < 0: every encoder. */
static void job_free(GlueJob *j);
static void job_unlink(GlueJob *j);
static void settle_prefetched(int (*pick)(const GlueJob *, int), int arg);
static int pick_slot(const GlueJob *j, int slot) {
    return j->users == 0 && (slot < 0 || (int)(j->job.picture_number >> GLUE_NS_SHIFT) == slot);
}
static void release_slot(int slot) {
    if (!G.ctx)
        return;
    pthread_mutex_lock(&G.gpu);
    pthread_mutex_lock(&G.reg);
    svtme_sync(G.ctx);
    for (uint32_t i = 0; i < G.n_regs;) {
        if (slot < 0 || G.regs[i].slot == slot) {
            svtme_host_unregister((void *)G.regs[i].p);
            G.regs[i] = G.regs[--G.n_regs];
        } else
            i++;
    }
    pthread_mutex_unlock(&G.reg);
    unsigned long long released = 0;
    for (uint32_t i = 0; i < G.n_pics;) {
        if (slot < 0 || (int)(G.pics[i].pn >> GLUE_NS_SHIFT) == slot) {
            svtme_picture_release(G.ctx, G.pics[i].pn);
            G.pics[i] = G.pics[--G.n_pics];
            released++;
        } else
            i++;
    }
    pthread_mutex_lock(&g_enc_mu);
    g_n_released += released;
    pthread_mutex_unlock(&g_enc_mu);
    pthread_mutex_unlock(&G.gpu);
    pthread_mutex_lock(&G.mu);
    settle_prefetched(pick_slot, slot); /* (their work has run: svtme_sync above) */
    for (GlueJob *j = G.jobs, *nx; j; j = nx) {
        nx = j->next;
        if ((slot < 0 || (int)(j->job.picture_number >> GLUE_NS_SHIFT) == slot) && j->users == 0 && j->state != 0) {
            job_unlink(j);
            job_free(j);
        }
    }
    pthread_mutex_unlock(&G.mu);
}

void svtme_glue_release(void) {
    release_slot(-1);
    pthread_mutex_lock(&g_enc_mu);
    for (int i = 0; i < GLUE_MAX_ENC; i++) {
        __atomic_store_n(&g_enc[i].pa_res, NULL, __ATOMIC_RELEASE);
        __atomic_store_n(&g_enc[i].pd_res, NULL, __ATOMIC_RELEASE);
        __atomic_store_n(&g_enc[i].enc_ctx, NULL, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_enc_mu);
}

void svtme_glue_release_encoder(const void *enc_ctx) {
    int slot = -1;
    for (int i = 0; i < GLUE_MAX_ENC && enc_ctx; i++)
        if (__atomic_load_n(&g_enc[i].enc_ctx, __ATOMIC_ACQUIRE) == enc_ctx)
            slot = i;
    if (slot < 0)
        return;
    release_slot(slot);
    pthread_mutex_lock(&g_enc_mu);
    __atomic_store_n(&g_enc[slot].pa_res, NULL, __ATOMIC_RELEASE);
    __atomic_store_n(&g_enc[slot].pd_res, NULL, __ATOMIC_RELEASE);
    __atomic_store_n(&g_enc[slot].enc_ctx, NULL, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&g_enc_mu);
}

/* SVTME_GLUE_VERIFY: the resident pyramid of pn equals the encoder's three planes (aborts if not) */
static void verify_pic(uint64_t pn, const EbPictureBufferDesc *full, const EbPictureBufferDesc *quarter,
                       const EbPictureBufferDesc *sixteenth, unsigned long long *count) {
    if (verify_level(pn, 0, full) || (quarter && verify_level(pn, 1, quarter)) ||
        (sixteenth && verify_level(pn, 2, sixteenth))) {
        fprintf(stderr, "svtme glue: picture %llu: the ME pyramid differs from the encoder's planes\n",
                (unsigned long long)pn);
        abort();
    }
    *count += 1 + (quarter != NULL) + (sixteenth != NULL);
}

static int pic_ensure(uint64_t pn, const EbPictureBufferDesc *full, const EbPictureBufferDesc *quarter,
                      const EbPictureBufferDesc *sixteenth, uint32_t w, uint32_t h, uint64_t pin[9], int npin) {
    GluePic *p = pic_find(pn);
    if (p && p->w == w && p->h == h && !p->dirty) {
        p->last_use = ++G.tick;
        return 0;
    }
    if (!p && G.n_pics >= (uint32_t)G.max_resident) { /* evict the least recently used picture this job does not name */
        GluePic *lru = NULL;
        for (uint32_t i = 0; i < G.n_pics; i++) {
            int pinned = 0;
            for (int k = 0; k < npin; k++) pinned |= G.pics[i].pn == pin[k];
            if (!pinned && (!lru || G.pics[i].last_use < lru->last_use))
                lru = &G.pics[i];
        }
        if (lru) {
            svtme_picture_release(G.ctx, lru->pn);
            *lru = G.pics[--G.n_pics];
            G.n.evictions++;
        }
    }
    uint64_t span;
    const uint8_t *y = span_of(full, w, h, &span);
    const double t0  = now_s();
    double t_pin     = t0;
    if (G.pin) { /* SVTME_GLUE_PIN=1: page-lock the encoder's buffer, one DMA straight from it */
        pin_span(y, span, (int)(pn >> GLUE_NS_SHIFT)); /* (locked already when the caller pinned it first) */
        t_pin = now_s();
        if (svtme_picture_upload_async(G.ctx, pn, y, full->stride_y, w, h) != SVTME_OK)
            return -1;
    } else if (svtme_picture_upload_copy_async(G.ctx, pn, y, full->stride_y, w, h) != SVTME_OK)
        return -1; /* (the rows go through the library's own page-locked staging) */
    const double t1 = now_s();
    G.n.upload_s += t1 - t0;
    if (G.trace_path) { /* uploads in the trace too (tf = 2), to place them beside the jobs */
        const GlueTrace t = {pn & GLUE_PN_MASK, 2, 0, 0, 1, t0, t1, t1, t1 - t0, 0, 0, t_pin, t1}; /* prep: pinned */
        pthread_mutex_lock(&G.mu);
        trace_add(&t);
        pthread_mutex_unlock(&G.mu);
    }
    if (G.verify)
        verify_pic(pn, full, quarter, sixteenth, &G.n.verified);
    if (!p) {
        if (G.n_pics == G.cap_pics) {
            G.cap_pics = G.cap_pics ? 2 * G.cap_pics : 16;
            G.pics     = (GluePic *)realloc(G.pics, G.cap_pics * sizeof(GluePic));
            if (!G.pics)
                abort();
        }
        p = &G.pics[G.n_pics++];
    }
    p->pn = pn, p->w = w, p->h = h, p->last_use = ++G.tick, p->dirty = 0;
    G.n.uploads++;
    return 0;
}

static int job_names(const svtme_job *job, uint64_t pn) {
    if (job->picture_number == pn)
        return 1;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++)
            if (job->ref_picture_number[l][r] == pn)
                return 1;
    return 0;
}
/* a picture the job reads changed after change number gen (G.mu held; every change if
 * the log wrapped) */
static int changed_since(const svtme_job *job, uint64_t gen) {
    if (G.chg_seq - gen > GLUE_CHG_LOG)
        return 1;
    for (uint64_t q = gen; q < G.chg_seq; q++)
        if (job_names(job, G.chg_pn[q % GLUE_CHG_LOG]))
            return 1;
    return 0;
}

static void job_free(GlueJob *j) { /* G.mu held, j already unlinked */
    if (j->served == 0 && j->state == 1)
        G.n.unused_jobs++; /* a batched TF pair the encoder never asked for */
    buf_give(j);
    free(j);
}

static void job_unlink(GlueJob *j) { /* G.mu held */
    GlueJob **pp = &G.jobs;
    while (*pp != j) pp = &(*pp)->next;
    *pp = j->next;
}

/* Prefetched jobs whose ticket no thread has taken, chosen by `pick` (stale
 * ones, an encoder's at its teardown, or the oldest when too many are out):
 * take their tickets, wait for them outside G.mu, and mark them done; the stale
 * ones nobody uses are freed. G.mu held on entry and on return. */
static void settle_prefetched(int (*pick)(const GlueJob *, int), int arg) {
    GlueJob *list[SVTME_MAX_TICKETS];
    uint64_t tk[SVTME_MAX_TICKETS];
    int n = 0;
    for (GlueJob *j = G.jobs; j && n < SVTME_MAX_TICKETS; j = j->next)
        if (j->ticket && pick(j, arg)) {
            tk[n]     = j->ticket;
            j->ticket = 0;
            j->users++; /* held while this thread waits */
            list[n++] = j;
        }
    if (!n)
        return;
    pthread_mutex_unlock(&G.mu);
    int ok[SVTME_MAX_TICKETS];
    for (int k = 0; k < n; k++) ok[k] = svtme_ticket_wait(G.ctx, tk[k]) == SVTME_OK;
    pthread_mutex_lock(&G.mu);
    for (int k = 0; k < n; k++) {
        GlueJob *j = list[k];
        j->state   = ok[k] ? 1 : -1;
        if (--j->users == 0 && (j->stale || j->served >= j->n_sb)) {
            job_unlink(j);
            job_free(j);
        }
    }
    pthread_cond_broadcast(&G.cv);
}
static int pick_stale(const GlueJob *j, int arg) {
    (void)arg;
    return j->stale && j->users == 0;
}

static EbPaReferenceObject *pa_object(const PictureParentControlSet *pcs) {
    return (EbPaReferenceObject *)pcs->pa_ref_pic_wrapper->object_ptr;
}

/* The encoder decimated a picture into its 1/4 and 1/16 planes: picture
 * analysis (pic_analysis_process.c:2151, the first time), temporal filtering's
 * pad_and_decimate_filtered_pic (temporal_filtering.c:3895-3931, the filtered
 * picture), or picture decision (pd_process.c:2720-2739, a re-copy). Jobs still
 * to come read the new planes; jobs already computed read the old ones, as the
 * encoder's SB calls made before the rebuild did, and are no longer matched by
 * later calls.
 *
 * When `full` is the plane the jobs read (the picture's PA reference object's
 * input_padded_pic, which is what submit_job uploads), it is uploaded here,
 * ahead of the picture's jobs: every later change to it is again a decimation
 * through this function, and the encoder's stages that write it (temporal
 * filtering, picture decision) run after the jobs that read the earlier content
 * have completed, which implies their upload has. Other planes (resize.c's
 * scaled pictures) only mark the resident copy out of date. */
void svtme_picture_changed(PictureParentControlSet *pcs, const EbPictureBufferDesc *full) {
    pthread_once(&G.once, glue_init);
    /* one slot lookup; an encoder without a slot (more than GLUE_MAX_ENC live) runs
     * the encoder's own ME for every picture (svtme_motion_estimation_b64), so its
     * pictures are never resident: nothing to pin, upload or mark stale, and its
     * numbers must not alias slot 0's namespace */
    const int slot = G.ctx ? pcs_slot(pcs) : -1;
    if (slot < 0)
        return;
    const EbPictureBufferDesc *pa = pcs->pa_ref_pic_wrapper ? pa_object(pcs)->input_padded_pic : NULL;
    const int eager = G.eager && full && pa && full->buffer_y == pa->buffer_y && full->stride_y == pa->stride_y &&
        full->org_x == pa->org_x && full->org_y == pa->org_y && pcs->aligned_width && pcs->aligned_height &&
        !pcs->frame_superres_enabled && !pcs->frame_resize_enabled;
    if (eager) { /* (SVTME_GLUE_PIN=1: page-lock a new buffer, timed as register_ms) fill the pools before taking G.gpu */
        if (G.pin) {
            uint64_t span;
            const uint8_t *y = span_of(pa, pcs->aligned_width, pcs->aligned_height, &span);
            pin_span(y, span, slot);
        }
        buf_prefill(pcs->aligned_width, pcs->aligned_height); /* (once; timed as prefill_ms) */
    }
    const uint64_t pn = ns_pn(slot, pcs->picture_number);
    pthread_mutex_lock(&G.gpu);
    GluePic *p = pic_find(pn);
    if (p && !p->dirty) {
        p->dirty = 1;
        G.n.invalidations++;
    }
    if (eager) {
        const double t0 = now_s();
        const EbPaReferenceObject *o = pa_object(pcs);
        uint64_t pin[9] = {pn};
        if (pic_ensure(pn, pa, o->quarter_downsampled_picture_ptr, o->sixteenth_downsampled_picture_ptr,
                       pcs->aligned_width, pcs->aligned_height, pin, 1) == 0)
            G.n.eager_uploads++;
        G.n.eager_s += now_s() - t0;
    }
    pthread_mutex_unlock(&G.gpu);
    pthread_mutex_lock(&G.mu);
    G.chg_pn[G.chg_seq++ % GLUE_CHG_LOG] = pn;
    for (GlueJob *j = G.jobs, *nx; j; j = nx) {
        nx = j->next;
        if (j->stale || !job_names(&j->job, pn))
            continue;
        j->stale = 1;
        G.n.stale++;
        if (j->users == 0 && j->state != 0) {
            job_unlink(j);
            job_free(j);
        }
    }
    settle_prefetched(pick_stale, 0); /* (prefetched jobs of the old content nobody took) */
    pthread_mutex_unlock(&G.mu);
}

/* The temporal filter's (central, reference) pairs of one window, in the
 * order its frame loop visits them, with the same outlier skips
 * (temporal_filtering.c:3096-3122; low delay: every frame, :3645-3648): all are
 * known at the window's first ME call (blocks are the outer loop, frames the
 * inner, :3029-3030), so that call submits every pair's job in ONE launch.
 * out[] receives the jobs other than `first` (its clones with another
 * reference), objs[] their reference objects. */
static int tf_window(const PictureParentControlSet *centre, const MeContext *me, const svtme_job *first,
                     svtme_job *out, const EbPaReferenceObject **objs, int max) {
    PictureParentControlSet *const *list = centre->temp_filt_pcs_list;
    const int past = centre->past_altref_nframes, fut = centre->future_altref_nframes, ic = past;
    const int slot   = (int)(first->picture_number >> GLUE_NS_SHIFT);
    const int ld     = centre->scs->static_config.pred_structure == SVT_AV1_PRED_LOW_DELAY_B;
    const int step   = ld || !me->tf_ctrls.ref_frame_factor ? 1 : me->tf_ctrls.ref_frame_factor;
    const int s0[3]  = {0, past, past + 1}, s1[3] = {past - 1, past, past + fut};
    const int nseg   = ld ? 1 : 3;
    const SequenceControlSet *scs = centre->scs;
    int n = 0;
    for (int seg = 0; seg < nseg; seg++)
        for (int fi = ld ? 0 : s0[seg]; fi <= (ld ? past + fut : s1[seg]); fi += step) {
            if (fi == ic || !list[fi] || !list[fi]->pa_ref_pic_wrapper)
                continue;
            const PictureParentControlSet *p = list[fi];
            if (!ld) { /* the outlier skips of :3101-3122 */
                const uint32_t low_ahd_err = centre->aligned_width * centre->aligned_height;
                const uint8_t th           = centre->slice_type == I_SLICE ? 20 : 40;
                if (p->tf_ahd_error_to_central > low_ahd_err &&
                    (int)(((int)p->tf_ahd_error_to_central - (int)centre->tf_avg_ahd_error) * 100) >
                        th * (int)centre->tf_avg_ahd_error)
                    continue;
                uint32_t cnt = 0;
                for (uint32_t rw = 0; rw < scs->picture_analysis_number_of_regions_per_width; rw++)
                    for (uint32_t rh = 0; rh < scs->picture_analysis_number_of_regions_per_height; rh++)
                        if (abs((int)p->average_intensity_per_region[rw][rh] -
                                (int)centre->average_intensity_per_region[rw][rh]) > 2 &&
                            p->avg_luma != centre->tf_avg_luma)
                            cnt++;
                if (cnt >= (14 * scs->picture_analysis_number_of_regions_per_width *
                            scs->picture_analysis_number_of_regions_per_height) / 16)
                    continue;
            }
            const EbPaReferenceObject *o = (const EbPaReferenceObject *)p->pa_ref_pic_wrapper->object_ptr;
            const uint64_t rpn           = ns_pn(slot, o->picture_number);
            if (rpn == first->ref_picture_number[0][0] || n == max)
                continue;
            out[n] = *first;
            out[n].ref_picture_number[0][0] = rpn;
            objs[n++] = o;
        }
    return n;
}

/* make the jobs' pictures resident and submit them in one launch (G.gpu held);
 * tickets[] on success. objs[k] (k > 0) is job k's reference object; job 0's
 * references are the ME context's (me_ds_ref_array, set by the encoder for this call). */
static int submit_jobs(GlueJob **js, const EbPaReferenceObject **objs, int n, const PictureParentControlSet *pcs,
                       const MeContext *me, uint64_t *tickets) {
    uint64_t pin[1 + 8 + SVTME_MAX_BATCH_JOBS];
    int npin = 0;
    const svtme_job *job0 = &js[0]->job;
    pin[npin++] = job0->picture_number;
    for (int l = 0; l < job0->num_lists; l++)
        for (int r = 0; r < job0->num_refs[l]; r++) pin[npin++] = job0->ref_picture_number[l][r];
    for (int k = 1; k < n; k++) pin[npin++] = js[k]->job.ref_picture_number[0][0];
    const EbPaReferenceObject *cur = pa_object(pcs);
    if (pic_ensure(job0->picture_number, cur->input_padded_pic, cur->quarter_downsampled_picture_ptr,
                   cur->sixteenth_downsampled_picture_ptr, job0->width, job0->height, pin, npin))
        return -1;
    for (int l = 0; l < job0->num_lists; l++)
        for (int r = 0; r < job0->num_refs[l]; r++) {
            const EbDownScaledBufDescPtrArray *d = &me->me_ds_ref_array[l][r];
            if (pic_ensure(job0->ref_picture_number[l][r], d->picture_ptr, d->quarter_picture_ptr,
                           d->sixteenth_picture_ptr, job0->width, job0->height, pin, npin))
                return -1;
        }
    for (int k = 1; k < n; k++)
        if (pic_ensure(js[k]->job.ref_picture_number[0][0], objs[k]->input_padded_pic,
                       objs[k]->quarter_downsampled_picture_ptr, objs[k]->sixteenth_downsampled_picture_ptr,
                       job0->width, job0->height, pin, npin))
            return -1;
    if (G.verify) { /* what the jobs read is the encoder's current content, however it became resident */
        verify_pic(job0->picture_number, cur->input_padded_pic, cur->quarter_downsampled_picture_ptr,
                   cur->sixteenth_downsampled_picture_ptr, &G.n.verified_job);
        for (int l = 0; l < job0->num_lists; l++)
            for (int r = 0; r < job0->num_refs[l]; r++) {
                const EbDownScaledBufDescPtrArray *d = &me->me_ds_ref_array[l][r];
                verify_pic(job0->ref_picture_number[l][r], d->picture_ptr, d->quarter_picture_ptr,
                           d->sixteenth_picture_ptr, &G.n.verified_job);
            }
        for (int k = 1; k < n; k++)
            verify_pic(js[k]->job.ref_picture_number[0][0], objs[k]->input_padded_pic,
                       objs[k]->quarter_downsampled_picture_ptr, objs[k]->sixteenth_downsampled_picture_ptr,
                       &G.n.verified_job);
    }
    svtme_job jobs[SVTME_MAX_BATCH_JOBS];
    svtme_pack_layout layouts[SVTME_MAX_BATCH_JOBS];
    void *outs[SVTME_MAX_BATCH_JOBS];
    for (int k = 0; k < n; k++) jobs[k] = js[k]->job, layouts[k] = js[k]->layout, outs[k] = js[k]->packed;
    const double t0 = now_s();
    const svtme_status st = svtme_submit_pictures_packed_async(G.ctx, G.next_lane++ % SVTME_LANES, (uint32_t)n, jobs,
                                                               layouts, outs, tickets);
    G.n.submit_s += now_s() - t0;
    return st == SVTME_OK ? 0 : -1;
}

/* a new job in G.jobs (G.mu held) */
static GlueJob *job_new(const PictureParentControlSet *pcs, const svtme_job *job, uint32_t users) {
    GlueJob *j = (GlueJob *)calloc(1, sizeof(GlueJob));
    if (!j)
        abort();
    j->job    = *job;
    j->layout = layout_of(pcs, job);
    j->n_sb   = svtme_sb_total(job->width, job->height);
    j->R      = svtme_job_ref_slots(job);
    j->stride = svtme_packed_sb_bytes(&j->layout, j->R);
    j->users  = users;
    j->next   = G.jobs;
    G.jobs    = j;
    if (job->me_type == SVTME_ME_MCTF)
        G.n.tf_jobs++;
    else
        G.n.pa_jobs++;
    return j;
}

static GlueJob *job_find(const svtme_job *job) { /* G.mu held */
    GlueJob *j = G.jobs;
    while (j && (j->stale || memcmp(&j->job, job, sizeof(*job)) != 0)) j = j->next;
    return j;
}

/* Picture decision has posted the PA-ME tasks of pcs: build the picture's job
 * as the ME thread will (me_process.c:118-121 svt_aom_sig_deriv_me, :218-257 the
 * lists and references, into a scratch MeContext) and submit it now, so that
 * its results are on their way to host memory before the first segment's first
 * SB call. That call finds it (the same job, field for field) and waits for its
 * ticket; a job the encoder ends up not asking for (a field differs, or a
 * picture it reads is rebuilt first) is settled and dropped (`unused_jobs`),
 * and the SB calls run their own job as without prefetch. SVTME_GLUE_PREFETCH=0
 * turns it off. */
static int pick_oldest(const GlueJob *j, int arg) {
    (void)arg;
    return j->users == 0 && j->prefetched;
}
void svtme_glue_prefetch_pa(PictureParentControlSet *pcs) {
    pthread_once(&G.once, glue_init);
    if (!G.ctx || !G.prefetch || !pcs || pcs_slot(pcs) < 0)
        return;
    if (pcs->slice_type == I_SLICE || svt_aom_is_pic_skipped(pcs) || pcs->frame_superres_enabled ||
        pcs->frame_resize_enabled || !pcs->pa_ref_pic_wrapper)
        return; /* (no PA-ME job; scaled references run the encoder's own search) */
    static __thread MeContext *me;
    if (!me && !(me = (MeContext *)calloc(1, sizeof(MeContext))))
        return;
    svt_aom_sig_deriv_me(pcs->scs, pcs, me);
    me->me_type                     = ME_OPEN_LOOP;
    me->num_of_list_to_search       = pcs->slice_type == P_SLICE ? 1 : 2;
    me->num_of_ref_pic_to_search[0] = pcs->ref_list0_count_try;
    me->num_of_ref_pic_to_search[1] = pcs->slice_type == B_SLICE ? pcs->ref_list1_count_try : 0;
    me->temporal_layer_index        = pcs->temporal_layer_index;
    me->is_ref                      = pcs->is_ref;
    for (int l = 0; l < me->num_of_list_to_search; l++)
        for (int r = 0; r < me->num_of_ref_pic_to_search[l]; r++) {
            if (!pcs->ref_pa_pic_ptr_array[l][r])
                return;
            const EbPaReferenceObject *o = (const EbPaReferenceObject *)pcs->ref_pa_pic_ptr_array[l][r]->object_ptr;
            me->me_ds_ref_array[l][r].picture_ptr           = o->input_padded_pic;
            me->me_ds_ref_array[l][r].quarter_picture_ptr   = o->quarter_downsampled_picture_ptr;
            me->me_ds_ref_array[l][r].sixteenth_picture_ptr = o->sixteenth_downsampled_picture_ptr;
            me->me_ds_ref_array[l][r].picture_number        = o->picture_number;
        }
    svtme_job job;
    svtme_job_from_pcs(&job, pcs, me);
    pthread_mutex_lock(&G.mu);
    int out = 0;
    for (GlueJob *x = G.jobs; x; x = x->next) out += x->ticket != 0;
    if (out >= 8) /* (ME threads that never came: settle the oldest instead of holding tickets) */
        settle_prefetched(pick_oldest, 0);
    if (job_find(&job)) {
        pthread_mutex_unlock(&G.mu);
        return;
    }
    GlueJob *j = job_new(pcs, &job, 0);
    job_unlink(j); /* listed once it is submitted */
    const uint64_t gen = G.chg_seq;
    const int rc0 = buf_take(j, (size_t)j->n_sb * j->stride, buf_worst(j->n_sb));
    pthread_mutex_unlock(&G.mu);
    uint64_t ticket = 0;
    int rc = rc0;
    if (!rc) {
        const EbPaReferenceObject *objs[1] = {NULL};
        pthread_mutex_lock(&G.gpu);
        rc = submit_jobs(&j, objs, 1, pcs, me, &ticket);
        pthread_mutex_unlock(&G.gpu);
    }
    pthread_mutex_lock(&G.mu);
    if (rc) { /* the SB calls start their own job */
        j->state = -1;
        job_free(j);
    } else {
        j->ticket     = ticket;
        j->prefetched = 1;
        G.n.prefetched++;
        G.n.launches++;
        j->next = G.jobs;
        G.jobs  = j;
        /* (an SB call started the same job meanwhile, or a picture it reads changed
         * while it was unlisted: this one goes) */
        if (job_find(&job) != j || changed_since(&job, gen))
            j->stale = 1, settle_prefetched(pick_stale, 0);
    }
    pthread_mutex_unlock(&G.mu);
}

/* Picture decision has posted the temporal-filtering tasks of `centre`
 * (pd_process.c:3404-3426): every (central, reference) pair of its window is
 * known (tf_window: the filter's frame order and outlier skips, all computed
 * by picture decision), so their jobs go to the GPU in one launch now, built
 * as the TF code will build them (svt_aom_sig_deriv_me_tf, me_process.c:123;
 * the filter's controls, temporal_filtering.c:4112; create_me_context_and_
 * picture_control's FULL_SAD HME and set_hme_search_params_mctf(ctx, 0),
 * :2759-2767, 3127-3168). The ME threads' calls then find them as for PA. */
#define GLUE_TF_LAUNCH 4
void svtme_glue_prefetch_tf(PictureParentControlSet *centre) {
    pthread_once(&G.once, glue_init);
    if (!G.ctx || !G.prefetch || !G.tf_batch || !centre || pcs_slot(centre) < 0 || !centre->tf_ctrls.enabled ||
        !centre->temp_filt_pcs_list || !centre->enhanced_unscaled_pic || !centre->pa_ref_pic_wrapper)
        return;
    static __thread MeContext *me;
    if (!me && !(me = (MeContext *)calloc(1, sizeof(MeContext))))
        return;
    svt_aom_sig_deriv_me_tf(centre, me);
    me->tf_ctrls                    = centre->tf_ctrls;
    me->hme_search_method           = FULL_SAD_SEARCH;
    me->hme_l0_sa.sa_min            = me->hme_l0_sa_default_tf.sa_min;
    me->hme_l0_sa.sa_max            = me->hme_l0_sa_default_tf.sa_max;
    me->me_type                     = ME_MCTF;
    me->num_of_list_to_search       = 1;
    me->num_of_ref_pic_to_search[0] = 1;
    me->num_of_ref_pic_to_search[1] = 0;
    me->temporal_layer_index        = centre->temporal_layer_index;
    me->is_ref                      = centre->is_ref;
    me->tf_me_exit_th               = centre->tf_ctrls.me_exit_th;
    me->me_ds_ref_array[0][0].picture_number = 0;
    svtme_job tmpl;
    svtme_job_from_tf(&tmpl, centre, me, centre->enhanced_unscaled_pic);
    tmpl.ref_picture_number[0][0] = ~0ull; /* (tf_window skips the template's own reference) */
    svtme_job pairs[SVTME_MAX_BATCH_JOBS];
    const EbPaReferenceObject *po[SVTME_MAX_BATCH_JOBS];
    const int np = tf_window(centre, me, &tmpl, pairs, po, SVTME_MAX_BATCH_JOBS);
    if (np <= 0)
        return;
    GlueJob *js[SVTME_MAX_BATCH_JOBS];
    const EbPaReferenceObject *objs[SVTME_MAX_BATCH_JOBS];
    int n = 0;
    pthread_mutex_lock(&G.mu);
    const uint64_t gen = G.chg_seq;
    for (int k = 0; k < np; k++) {
        if (job_find(&pairs[k])) /* (already running) */
            continue;
        GlueJob *x = job_new(centre, &pairs[k], 0);
        job_unlink(x); /* listed once submitted */
        if (buf_take(x, (size_t)x->n_sb * x->stride, buf_worst(x->n_sb))) {
            job_free(x);
            break;
        }
        objs[n] = po[k];
        js[n++] = x;
    }
    pthread_mutex_unlock(&G.mu);
    if (!n)
        return;
    /* launches of at most GLUE_TF_LAUNCH pairs on alternating lanes: the window's
     * first pairs (the filter's first calls) are ready before the whole window is */
    uint64_t tickets[SVTME_MAX_BATCH_JOBS] = {0};
    int rc = 0, launches = 0;
    pthread_mutex_lock(&G.gpu);
    for (int k0 = 0; k0 < n && !rc; k0 += GLUE_TF_LAUNCH) {
        const int m = n - k0 < GLUE_TF_LAUNCH ? n - k0 : GLUE_TF_LAUNCH;
        /* the launch's job 0 takes its reference planes through the context, as the TF code sets them */
        me->me_ds_ref_array[0][0].picture_ptr           = objs[k0]->input_padded_pic;
        me->me_ds_ref_array[0][0].quarter_picture_ptr   = objs[k0]->quarter_downsampled_picture_ptr;
        me->me_ds_ref_array[0][0].sixteenth_picture_ptr = objs[k0]->sixteenth_downsampled_picture_ptr;
        me->me_ds_ref_array[0][0].picture_number        = objs[k0]->picture_number;
        rc = submit_jobs(js + k0, objs + k0, m, centre, me, tickets + k0);
        launches += !rc;
    }
    pthread_mutex_unlock(&G.gpu);
    pthread_mutex_lock(&G.mu);
    G.n.launches += launches;
    for (int k = 0; k < n; k++) {
        GlueJob *j = js[k];
        if (!tickets[k]) { /* (its launch failed: the SB calls start their own job) */
            j->state = -1;
            job_free(j);
            continue;
        }
        j->ticket     = tickets[k];
        j->prefetched = 1;
        G.n.prefetched++;
        G.n.tf_batched += k > 0;
        j->next = G.jobs;
        G.jobs  = j;
        if (job_find(&j->job) != j || changed_since(&j->job, gen))
            j->stale = 1;
    }
    settle_prefetched(pick_stale, 0);
    pthread_mutex_unlock(&G.mu);
}

EbErrorType svtme_motion_estimation_b64(PictureParentControlSet *pcs, uint32_t b64_index, uint32_t b64_origin_x,
                                        uint32_t b64_origin_y, MeContext *me_ctx, EbPictureBufferDesc *input_ptr) {
    pthread_once(&G.once, glue_init);
    svtme_job job;
    if (me_ctx->me_type == ME_OPEN_LOOP && !pcs->frame_superres_enabled && !pcs->frame_resize_enabled)
        svtme_job_from_pcs(&job, pcs, me_ctx);
    else if (me_ctx->me_type == ME_MCTF)
        svtme_job_from_tf(&job, pcs, me_ctx, input_ptr);
    else /* scaled references (me_process.c:229-246), DG detector: the encoder's own search */
        return SVTME_ENCODER_ME_B64(pcs, b64_index, b64_origin_x, b64_origin_y, me_ctx, input_ptr);
    if (!G.ctx || pcs_slot(pcs) < 0) { /* (no device, or more than GLUE_MAX_ENC live encoders) */
        pthread_mutex_lock(&G.mu);
        G.n.fallback_sbs++;
        pthread_mutex_unlock(&G.mu);
        return SVTME_ENCODER_ME_B64(pcs, b64_index, b64_origin_x, b64_origin_y, me_ctx, input_ptr);
    }

    /* find or start the picture's job (one per picture, or per TF reference: the
     * first call of a TF window starts every pair's job, in one launch) */
    pthread_mutex_lock(&G.mu);
    GlueJob *j = job_find(&job);
    if (j && j->ticket) { /* prefetched at picture decision, not yet waited for: this thread waits */
        const uint64_t tk = j->ticket;
        j->ticket         = 0;
        j->users++;
        const double t_start = now_s();
        if (G.inflight++ == 0)
            G.busy_t0 = t_start;
        if (G.inflight > G.n.max_inflight)
            G.n.max_inflight = G.inflight;
        const uint32_t inflight = G.inflight;
        pthread_mutex_unlock(&G.mu);
        float gms = 0, cms = 0;
        const int rk       = svtme_ticket_wait_timed(G.ctx, tk, &gms, &cms) == SVTME_OK ? 0 : -1;
        const double t_done = now_s();
        pthread_mutex_lock(&G.mu);
        G.n.wait_s += t_done - t_start;
        G.n.job_s += t_done - t_start;
        G.n.prefetch_hits++;
        G.n.prefetch_ready += t_done - t_start < 10e-6; /* (its results were in host memory already) */
        if (!rk)
            G.n.job_sbs += j->n_sb;
        if (G.trace_path) {
            const GlueTrace t = {j->job.picture_number, j->job.me_type == SVTME_ME_MCTF, j->n_sb, inflight, 0,
                                 t_start, t_start, t_done, 0, gms, cms};
            trace_add(&t);
        }
        j->state = rk ? -1 : 1;
        if (--G.inflight == 0)
            G.n.busy_s += t_done - G.busy_t0;
        pthread_cond_broadcast(&G.cv);
    } else if (j) {
        j->users++;
        while (j->state == 0) pthread_cond_wait(&G.cv, &G.mu);
    } else {
        GlueJob *js[SVTME_MAX_BATCH_JOBS];
        const EbPaReferenceObject *objs[SVTME_MAX_BATCH_JOBS] = {NULL};
        int n = 0;
        j       = job_new(pcs, &job, 1);
        js[n++] = j;
        const double t_start = now_s();
        int rc = buf_take(j, (size_t)j->n_sb * j->stride, buf_worst(j->n_sb));
        if (!rc && job.me_type == SVTME_ME_MCTF && G.tf_batch) {
            svtme_job sib[SVTME_MAX_BATCH_JOBS - 1];
            const EbPaReferenceObject *so[SVTME_MAX_BATCH_JOBS - 1];
            const int ns = tf_window(pcs, me_ctx, &job, sib, so, SVTME_MAX_BATCH_JOBS - 1);
            for (int k = 0; k < ns; k++) {
                if (job_find(&sib[k])) /* (already started) */
                    continue;
                GlueJob *x = job_new(pcs, &sib[k], 0);
                if (buf_take(x, (size_t)x->n_sb * x->stride, buf_worst(x->n_sb))) {
                    job_unlink(x);
                    free(x);
                    continue;
                }
                objs[n] = so[k];
                js[n++] = x;
                G.n.tf_batched++;
            }
        }
        if (G.inflight++ == 0)
            G.busy_t0 = t_start;
        if (G.inflight > G.n.max_inflight)
            G.n.max_inflight = G.inflight;
        const uint32_t inflight = G.inflight;
        pthread_mutex_unlock(&G.mu);
        uint64_t tickets[SVTME_MAX_BATCH_JOBS] = {0};
        unsigned long long up_n = 0;
        double up_s = 0;
        double t_prep = now_s(), t_locked = t_prep;
        if (!rc) {
            pthread_mutex_lock(&G.gpu);
            t_locked = now_s();
            up_n = G.n.uploads, up_s = G.n.upload_s;
            rc   = submit_jobs(js, objs, n, pcs, me_ctx, tickets);
            up_n = G.n.uploads - up_n, up_s = G.n.upload_s - up_s;
            pthread_mutex_unlock(&G.gpu);
        }
        double t_wait = now_s();
        for (int k = 0; k < n; k++) {
            /* no glue lock held: other pictures' threads upload and submit meanwhile */
            float gms = 0, cms = 0;
            const int rk =
                rc ? rc : (svtme_ticket_wait_timed(G.ctx, tickets[k], &gms, &cms) == SVTME_OK ? 0 : -1);
            const double t_done = now_s();
            pthread_mutex_lock(&G.mu);
            if (k == 0) {
                G.n.wait_s += t_done - t_wait;
                G.n.job_s += t_done - t_start;
                G.n.launches += !rc;
            }
            if (!rk)
                G.n.job_sbs += js[k]->n_sb;
            if (G.trace_path) {
                const GlueTrace t = {js[k]->job.picture_number, js[k]->job.me_type == SVTME_ME_MCTF, js[k]->n_sb,
                                     inflight, k ? 0 : (uint32_t)up_n, t_start, t_wait, t_done, k ? 0 : up_s, gms, cms,
                                     t_prep, t_locked};
                trace_add(&t);
            }
            js[k]->state = rk ? -1 : 1;
            if (rk && k == 0)
                glue_fallback("picture job failed");
            if (k == n - 1 && --G.inflight == 0)
                G.n.busy_s += t_done - G.busy_t0;
            pthread_cond_broadcast(&G.cv);
            if (k < n - 1)
                pthread_mutex_unlock(&G.mu);
        }
    }
    const int ok = j->state == 1 && b64_index < j->n_sb;
    if (ok)
        G.n.sbs++;
    else
        G.n.fallback_sbs++;
    pthread_mutex_unlock(&G.mu);

    EbErrorType ret = EB_ErrorNone;
    if (ok)
        svtme_scatter_sb(pcs, me_ctx, b64_index, b64_origin_x, b64_origin_y, &j->job, &j->layout,
                         j->packed + (size_t)b64_index * j->stride);
    else
        ret = SVTME_ENCODER_ME_B64(pcs, b64_index, b64_origin_x, b64_origin_y, me_ctx, input_ptr);

    /* the job is dropped once every SB of the picture has been served (or it went stale) */
    pthread_mutex_lock(&G.mu);
    j->served++;
    if (--j->users == 0 && (j->served >= j->n_sb || j->stale)) {
        job_unlink(j);
        job_free(j);
    }
    pthread_mutex_unlock(&G.mu);
    return ret;
}

#ifdef SVTME_GLUE_WRAP
EbErrorType __wrap_svt_aom_motion_estimation_b64(PictureParentControlSet *pcs, uint32_t b64_index,
                                                 uint32_t b64_origin_x, uint32_t b64_origin_y, MeContext *me_ctx,
                                                 EbPictureBufferDesc *input_ptr) {
    return svtme_motion_estimation_b64(pcs, b64_index, b64_origin_x, b64_origin_y, me_ctx, input_ptr);
}

EbErrorType __real_svt_av1_enc_init(EbComponentType *svt_enc_component);
EbErrorType __real_svt_av1_enc_deinit(EbComponentType *svt_enc_component);

static const void *handle_enc_ctx(const EbComponentType *c) {
    const EbEncHandle *h = c ? (const EbEncHandle *)c->p_component_private : NULL;
    return h && h->scs_instance_array && h->scs_instance_array[0] ? (const void *)h->scs_instance_array[0]->enc_ctx
                                                                  : NULL;
}

/* a new encoder: its slot, and the resource its picture analysis posts its results to.
 * With page-locked uploads (SVTME_GLUE_PIN=1) every 8-bit luma buffer of the
 * encoder's input pool (created by svt_av1_enc_init, enc_handle.c:1773-1787; the
 * PA reference pictures point at them) is page-locked here, before the first picture: hipHostRegister takes 2-3 ms per 4K
 * buffer and holds up the HIP calls of other threads while it runs, so locking
 * them on first upload (the analysis threads, racing the first uploads and jobs)
 * made the encode's first uploads wait milliseconds each. */
EbErrorType __wrap_svt_av1_enc_init(EbComponentType *svt_enc_component) {
    const EbErrorType e = __real_svt_av1_enc_init(svt_enc_component);
    if (e == EB_ErrorNone) {
        const EbEncHandle *h = (const EbEncHandle *)svt_enc_component->p_component_private;
        const int slot       = enc_slot(handle_enc_ctx(svt_enc_component), h->picture_analysis_results_resource_ptr,
                                        h->picture_decision_results_resource_ptr);
        pthread_once(&G.once, glue_init);
        // the luma buffers the PA reference pictures read (resource_coordination_process.c:1118-1130
        // points input_padded_pic->buffer_y at the input's y8b buffer), whole
        const EbSystemResource *pool = h->input_y8b_buffer_resource_ptr;
        if (slot >= 0 && G.ctx && G.pin && G.eager && pool)
            for (uint32_t i = 0; i < pool->object_total_count; i++) {
                const EbBufferHeaderType *hd = (const EbBufferHeaderType *)pool->wrapper_ptr_pool[i]->object_ptr;
                const EbPictureBufferDesc *d = hd ? (const EbPictureBufferDesc *)hd->p_buffer : NULL;
                if (!d || !d->buffer_y || !d->luma_size)
                    continue;
                pin_span(d->buffer_y, d->luma_size, slot);
                G.n.init_registrations++;
            }
        if (slot >= 0 && G.ctx && G.eager) {
            /* the output pool, device scratch and first pictures' memory, sized for the
             * encoder's pictures (pcs.c:1217 aligned_width = max_input_luma_width), and the
             * upload stream and the library's kernels loaded: the first uploads pay none of it */
            const SequenceControlSet *scs = h->scs_instance_array[0]->scs;
            buf_prefill(scs->max_input_luma_width, scs->max_input_luma_height);
            glue_warm();
        }
    }
    return e;
}

EbErrorType __wrap_svt_av1_enc_deinit(EbComponentType *svt_enc_component) {
    /* before the encoder frees the buffers the glue page-locked */
    svtme_glue_release_encoder(handle_enc_ctx(svt_enc_component));
    return __real_svt_av1_enc_deinit(svt_enc_component);
}

void __wrap_svt_aom_downsample_filtering_input_picture(PictureParentControlSet *pcs, EbPictureBufferDesc *full,
                                                       EbPictureBufferDesc *quarter, EbPictureBufferDesc *sixteenth) {
    __real_svt_aom_downsample_filtering_input_picture(pcs, full, quarter, sixteenth);
    svtme_picture_changed(pcs, full);
}

/* Picture analysis decimates inside its own translation unit
 * (pic_analysis_process.c:2151), out of reach of --wrap, and ends each picture
 * by posting a PictureAnalysisResults object (pic_analysis_process.c:2180-2191)
 * to its encoder's picture-analysis results resource: when such an object is
 * posted, the picture is uploaded, as its PA reference planes are final then
 * (until a later decimation). */
EbErrorType __real_svt_post_full_object(EbObjectWrapper *object_ptr);
EbErrorType __wrap_svt_post_full_object(EbObjectWrapper *object_ptr) {
    const void *res = object_ptr ? (const void *)object_ptr->system_resource_ptr : NULL;
    for (int i = 0; res && i < GLUE_MAX_ENC; i++)
        if (__atomic_load_n(&g_enc[i].pd_res, __ATOMIC_ACQUIRE) == res) {
            /* picture decision posts a picture's PA-ME tasks (pd_process.c:3544-3556):
             * its job goes to the GPU before the first segment reaches an ME thread */
            const PictureDecisionResults *r = (const PictureDecisionResults *)object_ptr->object_ptr;
            if (r->task_type == TASK_PAME && r->segment_index == 0)
                svtme_glue_prefetch_pa((PictureParentControlSet *)r->pcs_wrapper->object_ptr);
            else if (r->task_type == TASK_TFME && r->segment_index == 0)
                svtme_glue_prefetch_tf((PictureParentControlSet *)r->pcs_wrapper->object_ptr);
            break;
        } else if (__atomic_load_n(&g_enc[i].pa_res, __ATOMIC_ACQUIRE) == res) {
            const PictureAnalysisResults *r = (const PictureAnalysisResults *)object_ptr->object_ptr;
            PictureParentControlSet *pcs    = (PictureParentControlSet *)r->pcs_wrapper->object_ptr;
            if (!pcs->is_overlay && pcs->pa_ref_pic_wrapper) /* overlays skip the analysis (:2122) */
                svtme_picture_changed(pcs, pa_object(pcs)->input_padded_pic);
            break;
        }
    return __real_svt_post_full_object(object_ptr);
}
#endif
