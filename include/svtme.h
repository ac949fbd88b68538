/*
 * svtme.h — C ABI of the MI355X-native open-loop motion-estimation (ME) stage.
 *
 * Two surfaces, both plain C (pointers + sizes, no torch types):
 *
 *  1. Per-kernel rtcd variants (`*_hip`). Byte-identical signatures to the
 *     reference's run-time-dispatch pointers so an encoder can register them
 *     as a new variant after `svt_aom_setup_rtcd_internal`.
 *     They take caller-owned HOST memory, run synchronously on the GPU and
 *     return through the same out-params. They exist for drop-in registration
 *     and per-kernel parity; one call is far below a GPU launch in size.
 *
 *  2. The picture-level job API (`svtme_*`). This is the performance boundary:
 *     it replaces the per-SB loop of the ME thread
 *     (reference Source/Lib/Codec/me_process.c:174-290) with one GPU job that
 *     covers every 64x64 superblock (SB) x every reference of one picture.
 *     Pictures are uploaded once; their padded full / quarter / sixteenth
 *     pyramids stay resident in HBM, keyed by picture_number, until released.
 *
 * No entry point falls back to a CPU path. A HIP failure is reported through
 * the returned status (job API) or svtme_last_error() (rtcd variants), and a
 * message on stderr.
 */
#ifndef SVTME_H
#define SVTME_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------
 * Constants (reference values cited)
 * ------------------------------------------------------------------------- */
#define SVTME_PU_COUNT 85           /* SQUARE_PU_COUNT, me_sb_results.h:24 */
#define SVTME_MAX_LISTS 2           /* MAX_NUM_OF_REF_PIC_LIST, definitions.h:2337 */
#define SVTME_MAX_REFS 4            /* REF_LIST_MAX_DEPTH, EbSvtAv1Enc.h:36 */
#define SVTME_MAX_PA_ME_CAND 23     /* MAX_PA_ME_CAND, me_sb_results.h:22 */
#define SVTME_MAX_PA_ME_MV 7        /* MAX_PA_ME_MV, me_sb_results.h:21 */
#define SVTME_MAX_SAD_VALUE (128u * 128u * 255u) /* motion_estimation.h:85 */
#define SVTME_SUB_SAD_SEARCH 0      /* definitions.h:2071 */
#define SVTME_FULL_SAD_SEARCH 1     /* definitions.h:2072 */
/* svtme_job.me_type: the EbMeType values of me_context.h:44-51 */
#define SVTME_ME_MCTF 1             /* temporal-filtering ME (temporal_filtering.c:3169) */
#define SVTME_ME_OPEN_LOOP 3        /* pre-analysis open-loop ME (me_process.c:266) */
#define SVTME_PAD_FULL 72           /* PA full-res padding (enc_handle.c:4057-4069) */
#define SVTME_PAD_QUARTER 32        /* b64_size >> 1, reference_object.c:272 */
#define SVTME_PAD_SIXTEENTH 16      /* b64_size >> 2, reference_object.c:287 */

/* Status codes: the values of EbErrorType (API/EbSvtAv1.h:121-130). */
typedef int32_t svtme_status;
#define SVTME_OK 0
#define SVTME_ERR_INSUFFICIENT_RESOURCES ((int32_t)0x80001000)
#define SVTME_ERR_UNDEFINED ((int32_t)0x80001001)
#define SVTME_ERR_BAD_PARAMETER ((int32_t)0x80001005)

/* ---------------------------------------------------------------------------
 * Picture-level ME controls: a POD snapshot of the MeContext control fields
 * (me_context.h:280-364, 366-509) as set per picture by svt_aom_sig_deriv_me
 * (enc_mode_config.c:671-808). The GPU takes them as parameters; it never
 * re-derives them from the preset.
 * ------------------------------------------------------------------------- */
typedef struct svtme_area {
    uint16_t width;
    uint16_t height;
} svtme_area;

typedef struct svtme_area_minmax {
    svtme_area sa_min;
    svtme_area sa_max;
} svtme_area_minmax;

typedef struct svtme_controls {
    /* search methods: SVTME_SUB_SAD_SEARCH / SVTME_FULL_SAD_SEARCH */
    uint8_t hme_search_method;
    uint8_t me_search_method;
    /* HME enables (me_context.h:409-412) */
    uint8_t enable_hme_flag;
    uint8_t enable_hme_level0_flag;
    uint8_t enable_hme_level1_flag;
    uint8_t enable_hme_level2_flag;
    /* number of HME-L0 search regions; only 2x2 is supported (motion_estimation.c:1875) */
    uint8_t num_hme_sa_w;
    uint8_t num_hme_sa_h;
    /* search areas (MeHmeSearchAreaCtrls, me_context.h:342-347 / 421-429) */
    svtme_area_minmax hme_l0_sa;
    svtme_area hme_l1_sa;
    svtme_area hme_l2_sa;
    svtme_area_minmax me_sa;
    /* MeHmeRefPruneCtrls (me_context.h:280-290) */
    uint8_t enable_me_hme_ref_pruning;
    uint8_t pad0;
    uint16_t prune_ref_if_hme_sad_dev_bigger_than_th;
    uint16_t prune_ref_if_me_sad_dev_bigger_than_th;
    uint16_t zz_sad_pct;
    uint32_t zz_sad_th;
    uint32_t phme_sad_th;
    uint16_t phme_sad_pct;
    /* MeSrCtrls (me_context.h:292-305) */
    uint8_t enable_me_sr_adjustment;
    uint8_t distance_based_hme_resizing;
    uint16_t reduce_me_sr_based_on_mv_length_th;
    uint16_t stationary_hme_sad_abs_th;
    uint16_t stationary_me_sr_divisor;
    uint16_t reduce_me_sr_based_on_hme_sad_abs_th;
    uint16_t me_sr_divisor_for_low_hme_sad;
    /* MvBasedSearchAdj (me_context.h:356-364) */
    uint8_t mv_sa_adj_enabled;
    uint8_t mv_sa_adj_nearest_ref_only;
    uint16_t mv_sa_adj_mv_size_th;
    uint16_t mv_sa_adj_sa_multiplier;
    /* Me8x8VarCtrls (me_context.h:310-319) */
    uint8_t me_8x8_var_enabled;
    uint8_t pad1;
    uint32_t me_sr_div4_th;
    uint32_t me_sr_div2_th;
    uint32_t me_sr_mult2_th;
    /* PreHmeCtrls (me_context.h:336-341) */
    uint8_t prehme_enable;
    uint8_t prehme_skip_search_line;
    uint8_t prehme_l1_early_exit;
    uint8_t pad2;
    svtme_area_minmax prehme_sa_cfg[2];
    /* misc (me_context.h:490-508) */
    int32_t prune_me_candidates_th;
    uint8_t use_best_unipred_cand_only;
    uint8_t reduce_hme_l0_sr_th_min;
    uint8_t reduce_hme_l0_sr_th_max;
    uint8_t pad3;
    uint32_t me_early_exit_th;
    uint32_t me_safe_limit_zz_th;
    uint32_t prev_me_stage_based_exit_th;
} svtme_controls;

/* ---------------------------------------------------------------------------
 * One picture's ME job (the fields the reference reads from
 * PictureParentControlSet / SequenceControlSet / MeContext per picture).
 * ------------------------------------------------------------------------- */
typedef struct svtme_job {
    uint64_t picture_number;
    uint32_t width;   /* luma width of the PA picture, multiple of 8 (aligned_width) */
    uint32_t height;  /* luma height, multiple of 8 (aligned_height) */
    uint64_t ref_picture_number[SVTME_MAX_LISTS][SVTME_MAX_REFS];
    uint8_t num_lists;                 /* 1 = P slice, 2 = B slice (me_process.c:219-221) */
    uint8_t num_refs[SVTME_MAX_LISTS]; /* ref_list{0,1}_count_try (me_process.c:223-225) */
    uint8_t temporal_layer_index;
    uint8_t is_ref;
    uint8_t hierarchical_levels;
    uint8_t similar_brightness_refs;
    /* candidate construction (motion_estimation.c:2532-2835) */
    uint8_t enable_me_8x8;
    uint8_t enable_me_16x16;
    uint8_t max_cand;   /* pa_me_data->max_cand (pcs.c:91-96) */
    uint8_t max_refs;   /* pa_me_data->max_refs */
    uint8_t max_l0;     /* pa_me_data->max_l0 */
    uint8_t only_l_bwd; /* scs->mrp_ctrls.only_l_bwd */
    uint8_t input_resolution; /* EbInputResolution: 0=240p .. 6=8K (definitions.h:2079-2085) */
    uint8_t gm_enabled;       /* pcs->gm_ctrls.enabled */
    uint8_t gm_use_distance_based_active_th;
    /* SVTME_ME_OPEN_LOOP (0 is accepted as the same) or SVTME_ME_MCTF. MCTF jobs
     * (one list, one reference) skip the HME/ME reference pruning, search the
     * full-pel area unscaled by distance (motion_estimation.c:1300-1302), stop
     * after HME when the list-0 ref-0 HME SAD is below tf_me_exit_th (:3109-3113)
     * and build no candidate arrays (:3126) */
    uint8_t me_type;
    uint8_t pad;
    uint16_t tf_me_exit_th; /* MeContext.tf_me_exit_th (me_context.h:495) */
    /* SB range [sb_begin, sb_begin + sb_count) in raster b64 order; sb_count 0 = all */
    uint32_t sb_begin;
    uint32_t sb_count;
    svtme_controls ctrl;
} svtme_job;

/* ---------------------------------------------------------------------------
 * Outputs.
 * ------------------------------------------------------------------------- */
/* Per SB x per searched (list, ref) slot; slots ordered list 0 refs then list 1
 * refs, R = num_refs[0] + (num_lists == 2 ? num_refs[1] : 0) slots per SB. */
typedef struct svtme_ref_record {
    uint32_t best_sad[SVTME_PU_COUNT]; /* p_sb_best_sad[l][r][] Z-order PUs; 0xFFFFFFFF if !searched */
    uint32_t best_mv[SVTME_PU_COUNT];  /* p_sb_best_mv[l][r][]: (uint32)(y<<16)|(uint16)x, full-pel */
    uint64_t hme_sad;    /* final search_results[l][r].hme_sad (HME SAD, or me_prune_ref's 8x8 sum) */
    int16_t hme_sc_x;    /* HME search centre (full-pel), search_results[l][r].hme_sc_{x,y} */
    int16_t hme_sc_y;
    uint32_t zz_sad;     /* zz_sad[l][r] (0xFFFFFFFF if not computed) */
    uint8_t searched;    /* do_ref when the integer search ran */
    uint8_t do_ref;      /* final do_ref */
    uint8_t tf_early_exit; /* MCTF only: HME-only exit taken (tf_use_pred_64x64_only_th = ~0, :3111) */
    uint8_t pad[5];
} svtme_ref_record; /* 704 bytes */

/* Per SB candidate list + distortions (MeSbResults, me_sb_results.h:44, and the
 * per-SB pcs arrays written by compute_distortion, motion_estimation.c:2964). */
typedef struct svtme_sb_result {
    uint8_t total_me_candidate_index[SVTME_PU_COUNT];
    uint8_t pad0[3];
    /* MeCandidate bit-field byte: direction | ref_idx_l0<<2 | ref_idx_l1<<4 |
     * ref0_list<<6 | ref1_list<<7 ; indexed [pu_index][cand] */
    uint8_t me_candidate_array[SVTME_PU_COUNT][SVTME_MAX_PA_ME_CAND];
    uint8_t pad1[1];
    uint32_t me_mv_array[SVTME_PU_COUNT][SVTME_MAX_PA_ME_MV]; /* [pu_index][max_refs slot] */
    uint32_t me_distortion[SVTME_PU_COUNT];
    uint32_t me_8x8_cost_variance;
    uint32_t rc_me_distortion;
    uint32_t me_64x64_distortion;
    uint32_t me_32x32_distortion;
    uint32_t me_16x16_distortion;
    uint32_t me_8x8_distortion;
    uint8_t stationary_block_present;
    uint8_t rc_me_allow_gm;
    uint8_t pad2[6];
} svtme_sb_result;

/* The last 24 bytes of svtme_ref_record: the per-reference state an encoder
 * keeps after the SB (search_results[l][r], zz_sad[l][r], me_context.h:459). */
typedef struct svtme_record_tail {
    uint64_t hme_sad;
    int16_t hme_sc_x;
    int16_t hme_sc_y;
    uint32_t zz_sad;
    uint8_t searched;
    uint8_t do_ref;
    uint8_t tf_early_exit;
    uint8_t pad[5];
} svtme_record_tail;

/* Packed host output of svtme_submit_picture_packed_async: per SB, only what the
 * encoder's consumer reads, sized by its MeSbResults allocation (pcs.c:91-117),
 * so the device-to-host copy carries no unused candidate slots. SB k of the job
 * starts at byte k * svtme_packed_sb_bytes(layout, R):
 *   R records: svtme_ref_record (full_records = 1) or svtme_record_tail (0)
 *   when sb_results = 1:
 *     uint32 me_8x8_cost_variance, rc_me_distortion, me_64x64_distortion,
 *            me_32x32_distortion, me_16x16_distortion, me_8x8_distortion
 *     uint32 me_distortion[85]
 *     uint32 me_mv_array[n_pus][max_refs]
 *     uint8  stationary_block_present, rc_me_allow_gm, 0, 0
 *     uint8  total_me_candidate_index[n_pus]
 *     uint8  me_candidate_array[n_pus][max_cand]
 *   zero bytes up to the next multiple of 16. */
typedef struct svtme_pack_layout {
    uint16_t n_pus;       /* PUs with candidates: 85, 21 (no 8x8) or 5 (no 16x16) */
    uint8_t max_cand;     /* pa_me_data->max_cand, 1 .. SVTME_MAX_PA_ME_CAND */
    uint8_t max_refs;     /* pa_me_data->max_refs, 1 .. SVTME_MAX_PA_ME_MV */
    uint8_t full_records; /* 1: whole records (TF-ME reads the 85-PU winners), 0: tails */
    uint8_t sb_results;   /* 1: the SB-result fields (PA-ME) */
    uint8_t pad[2];
} svtme_pack_layout;

static inline uint32_t svtme_packed_sb_bytes(const svtme_pack_layout *L, uint32_t R) {
    uint32_t b = R * (L->full_records ? (uint32_t)sizeof(svtme_ref_record) : (uint32_t)sizeof(svtme_record_tail));
    if (L->sb_results)
        b += 4u * (6u + SVTME_PU_COUNT) + 4u * L->n_pus * L->max_refs + 4u + L->n_pus * (1u + L->max_cand);
    return (b + 15u) & ~15u;
}

/* ---------------------------------------------------------------------------
 * Picture-level job API (the performance boundary)
 * ------------------------------------------------------------------------- */
typedef struct svtme_ctx svtme_ctx;

/* Create a context on HIP device `device`. Sizes the plane cache lazily. */
svtme_status svtme_ctx_create(int device, svtme_ctx **out);
void svtme_ctx_destroy(svtme_ctx *ctx);

/* Upload one 8-bit luma picture (host memory, `stride` bytes per row,
 * width x height visible samples; width/height need not be multiples of 8:
 * the right/bottom are replicated to the next multiple of 8 as
 * svt_aom_pad_picture_to_multiple_of_min_blk_size_dimensions does). Builds the
 * padded full (pad 72), quarter (pad 32) and sixteenth (pad 16) planes on the
 * GPU (svt_aom_downsample_filtering_input_picture, pic_analysis_process.c:1945). */
svtme_status svtme_picture_upload(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *y,
                                  uint32_t stride, uint32_t width, uint32_t height);
/* Same, for a 10-bit picture in uint16 samples (stride in samples): the
 * searched plane is the 8-bit MSB plane p >> 2 (enc_handle.c:4964-4972). */
svtme_status svtme_picture_upload_10bit(svtme_ctx *ctx, uint64_t picture_number, const uint16_t *y,
                                        uint32_t stride, uint32_t width, uint32_t height);
/* Asynchronous form of svtme_picture_upload: the pyramid is built on the
 * context's upload stream, overlapping with jobs already running. From
 * page-locked host memory (svtme_host_alloc, svtme_host_register, hipHostMalloc)
 * the build reads the plane itself over PCIe; from pageable memory the rows are
 * first copied by DMA into a device staging plane (SVTME_UPLOAD_ZERO_COPY=0:
 * always the DMA). The call returns once the work is queued (pageable memory:
 * once the driver has staged it). The first job that reads the picture waits
 * for the upload on the GPU. With pinned host memory the caller keeps `y`
 * unchanged until svtme_sync() or a job reading the picture has completed.
 * Jobs queued earlier that read an older version of the picture finish before
 * it is overwritten. */
svtme_status svtme_picture_upload_async(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *y, uint32_t stride,
                                        uint32_t width, uint32_t height);
/* Asynchronous upload from PAGEABLE memory the library never page-locks (an
 * encoder's own picture buffers): the calling thread copies the w x h samples
 * into a page-locked staging buffer the library owns (a ring of
 * SVTME_UPLOAD_SLOTS, each reused once its DMA has run), outside the context
 * lock, then the DMA and the pyramid build are queued as in
 * svtme_picture_upload_async; `y` may change as soon as the call returns.
 * With more than SVTME_UPLOAD_SLOTS callers at once, a caller waits for a slot
 * (released as soon as its rows are staged and its DMA queued).
 * Page-locking the caller's memory instead (svtme_host_register) makes it a
 * driver user-pointer mapping, which the kernel may invalidate at any time
 * (NUMA balancing, page migration, compaction); every invalidation evicts the
 * process's GPU queues until the mapping is rebuilt -- a stall of the work in
 * flight. */
#define SVTME_UPLOAD_SLOTS 4
svtme_status svtme_picture_upload_copy_async(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *y,
                                             uint32_t stride, uint32_t width, uint32_t height);
/* Same, from a DEVICE pointer already in HBM (no PCIe). */
svtme_status svtme_picture_upload_device(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *d_y,
                                         uint32_t stride, uint32_t width, uint32_t height);
/* Asynchronous form of svtme_picture_upload_device (the input distribution of a
 * picture split over GPUs, SURVEY.md 8(e): the plane arrives in HBM by an RCCL
 * broadcast): the pyramid is built from d_y on the context's upload stream
 * (svtme_upload_stream) and the first job reading the picture waits for it on
 * the GPU. The caller makes the upload stream wait for d_y's producer before the
 * call and keeps d_y unchanged until the work queued on that stream has run. */
svtme_status svtme_picture_upload_device_async(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *d_y,
                                               uint32_t stride, uint32_t width, uint32_t height);
/* The hipStream_t of the asynchronous uploads (created on first use). */
void *svtme_upload_stream(svtme_ctx *ctx);
svtme_status svtme_picture_release(svtme_ctx *ctx, uint64_t picture_number);
/* The resident picture's source planes were replaced (temporal filtering
 * re-decimates the filtered picture, temporal_filtering.c:3895-3931
 * pad_and_decimate_filtered_pic): rebuild its pyramid from the new 8-bit
 * plane. Ordered after every job already submitted on the context (those read
 * the old planes), before every later one. Fails if the picture is not
 * resident (a stale pyramid is never silently kept). */
svtme_status svtme_picture_invalidate(svtme_ctx *ctx, uint64_t picture_number, const uint8_t *y, uint32_t stride,
                                      uint32_t width, uint32_t height);
/* Copy a resident pyramid level back to host (level 0 = full, 1 = quarter,
 * 2 = sixteenth), padding included: dst gets (h + 2 pad) rows of `stride` bytes. */
svtme_status svtme_picture_download(svtme_ctx *ctx, uint64_t picture_number, int level, uint8_t *dst,
                                    uint32_t *stride, uint32_t *width, uint32_t *height, uint32_t *pad);

/* Run ME for one picture. `ref_records` receives sb_count x R records and
 * `sb_results` (may be NULL) sb_count results, in host memory. Synchronous. */
svtme_status svtme_submit_picture(svtme_ctx *ctx, const svtme_job *job, svtme_ref_record *ref_records,
                                  svtme_sb_result *sb_results);

/* Asynchronous variant for pipelining / benchmarking: records stay in device
 * memory owned by ctx; svtme_sync waits, svtme_fetch copies them out. */
svtme_status svtme_submit_picture_async(svtme_ctx *ctx, const svtme_job *job);
svtme_status svtme_sync(svtme_ctx *ctx);
svtme_status svtme_fetch(svtme_ctx *ctx, svtme_ref_record *ref_records, svtme_sb_result *sb_results);
/* Asynchronous variant writing into caller-provided DEVICE buffers (e.g. the
 * slice of an all-gather tensor): sb_count x R records, and sb_count results
 * when d_sb_results is not NULL. */
svtme_status svtme_submit_picture_device(svtme_ctx *ctx, const svtme_job *job, svtme_ref_record *d_ref_records,
                                         svtme_sb_result *d_sb_results);
/* Run ME for a batch of n <= SVTME_MAX_BATCH_JOBS pictures (the ready
 * pictures of a mini-GOP, or this rank's SB band of n pictures) with ONE launch
 * of each stage kernel (jobs needing different kernel variants are launched
 * as separate groups). Job k writes its sb_count x R records to
 * d_ref_records[k] and, when d_sb_results is not NULL and d_sb_results[k] is
 * not NULL, its sb_count results to d_sb_results[k] (DEVICE buffers).
 * Asynchronous on the context's stream; the reference runs these pictures on
 * its ME threads concurrently (me_process.c:97-104). */
#define SVTME_MAX_BATCH_JOBS 16
svtme_status svtme_submit_batch_device(svtme_ctx *ctx, const svtme_job *jobs, uint32_t n,
                                       svtme_ref_record *const *d_ref_records, svtme_sb_result *const *d_sb_results);
/* The same on submission lane `lane` (0 .. SVTME_LANES-1): each lane has its own
 * stream (svtme_lane_stream; lane 0's is svtme_stream) and inter-stage
 * scratch, so batches on different lanes overlap on the GPU (the next batch's
 * workgroups fill the CUs while the previous one drains) the way the
 * reference's ME threads process pictures concurrently. Pictures are shared:
 * a lane waits for asynchronous uploads, and a re-upload or rebuild waits for
 * every lane's queued readers. Completion is signalled on the lane's stream. */
#define SVTME_LANES 2
svtme_status svtme_submit_batch_device_lane(svtme_ctx *ctx, uint32_t lane, const svtme_job *jobs, uint32_t n,
                                            svtme_ref_record *const *d_ref_records,
                                            svtme_sb_result *const *d_sb_results);
/* The hipStream_t of a lane (created on first use), NULL on a bad lane. */
void *svtme_lane_stream(svtme_ctx *ctx, uint32_t lane);

/* Asynchronous job with packed HOST output, for an encoder's ME threads (the
 * reference runs several pictures' ME at once, me_process.c:97-104). The job
 * runs on lane `lane` into device buffers the context keeps per ticket, is
 * packed on the device (svtme_pack_layout) and copied into host_out
 * (sb_count x svtme_packed_sb_bytes(layout, R) bytes) on the context's download
 * stream, overlapping later jobs. Returns at once with *ticket. host_out should
 * be page-locked (svtme_host_alloc): a pageable destination makes the copy
 * synchronous. At most SVTME_MAX_TICKETS tickets are outstanding (the
 * reference runs up to 25 ME threads and the TF threads beside them, one job in
 * flight each, enc_handle.c:744-773). A submission that finds every slot taken
 * waits for svtme_ticket_wait (another thread's) to retire one; it is refused
 * (SVTME_ERR_INSUFFICIENT_RESOURCES) only when no ticket is retired within
 * 100 ms while none is being waited on -- the caller holds them itself. */
#define SVTME_MAX_TICKETS 64
svtme_status svtme_submit_picture_packed_async(svtme_ctx *ctx, uint32_t lane, const svtme_job *job,
                                               const svtme_pack_layout *layout, void *host_out, uint64_t *ticket);
/* The same for n jobs (1 .. SVTME_MAX_BATCH_JOBS) in ONE batched launch: the
 * temporal filter's (central picture, reference) pairs of one window, all
 * known at its first ME call (temporal_filtering.c:3029-3030, 3096). Job k's
 * output goes to host_outs[k] under tickets[k]; each ticket is waited for and
 * retired on its own. */
svtme_status svtme_submit_pictures_packed_async(svtme_ctx *ctx, uint32_t lane, uint32_t n, const svtme_job *jobs,
                                                const svtme_pack_layout *layouts, void *const *host_outs,
                                                uint64_t *tickets);
/* Block until ticket's packed output is in host memory, then retire the ticket.
 * Safe to call from any thread, without holding anything the submitter holds. */
svtme_status svtme_ticket_wait(svtme_ctx *ctx, uint64_t ticket);
/* The same, and the job's GPU-side times (HIP events): from its turn on its
 * lane to its packed output on the device (waits for its pictures' uploads,
 * the search, the pack), and from there to the output in host memory (the
 * download stream's copy). Either pointer may be NULL. */
svtme_status svtme_ticket_wait_timed(svtme_ctx *ctx, uint64_t ticket, float *gpu_ms, float *copy_ms);
/* Page-locked host memory for packed outputs (NULL on failure), and its release. */
void *svtme_host_alloc(uint64_t bytes);
void svtme_host_free(void *p);
/* Page-lock an existing host range (e.g. an encoder's picture buffer) so that
 * svtme_picture_upload_async reads it from the GPU without staging it through
 * the CPU; svtme_host_unregister undoes it once the uploads reading it have run. */
svtme_status svtme_host_register(void *p, uint64_t bytes);
svtme_status svtme_host_unregister(void *p);
/* Size the device memory of later jobs ahead of them: every submission lane's
 * inter-stage scratch and the device buffers of the first `tickets` packed-job
 * slots, for jobs over pictures up to width x height with up to max_refs
 * reference slots and any pack layout, and for batches of up to
 * SVTME_MAX_BATCH_JOBS such pictures of one reference slot each (a TF window).
 * Submissions within those bounds then allocate nothing (a job beyond them
 * still grows the buffers it needs, after its lane's queued work has run). */
svtme_status svtme_reserve(svtme_ctx *ctx, uint32_t width, uint32_t height, uint32_t max_refs, uint32_t tickets);
/* Keep `count` picture buffers of a width x height picture (its three padded
 * planes) in the context's free pool, so that the uploads of up to that many
 * pictures beyond the resident ones allocate no device memory. Released
 * pictures' buffers return to the pool once the work reading them has run
 * (never hipFree on the steady path: it serialises the device). */
svtme_status svtme_reserve_pictures(svtme_ctx *ctx, uint32_t width, uint32_t height, uint32_t count);
/* Kernel timing with HIP events on the context's stream, recorded around every
 * stage launch of every submission while enabled (enable = 1). svtme_timing_read
 * waits for the recorded launch groups and returns the milliseconds of stage 0
 * (k_stage_a: zz / pre-HME / HME-L0, or the fused k_hme), 1 (k_stage_d: their
 * decisions), 2 (k_stage_b: HME-L1/L2), 3 (k_stage_c1, or the per-SB
 * k_stage_c) and 4 (k_stage_e) in stage_ms[0..4], each averaged over the
 * launch groups that ran that stage; returns the number of launch groups read
 * and clears them. At most 256 groups are kept between reads; later ones are
 * not recorded and the read sets svtme_last_error(). */
svtme_status svtme_set_timing(svtme_ctx *ctx, int enable);
uint32_t svtme_timing_read(svtme_ctx *ctx, float stage_ms[5]);
/* Kernel-path selection of a context, for diagnostics and A/B runs: each bit
 * forces a general path where a specialised kernel would apply (results are
 * identical). 0, the default, takes every specialised kernel that applies. A
 * context starts with the bits of the environment variables named below (read
 * once, at svtme_ctx_create); svtme_set_paths replaces them for the jobs
 * submitted after it. */
#define SVTME_PATH_NO_FUSED_HME 1u /* SVTME_NO_FUSED_HME: k_stage_a -> k_stage_d -> k_stage_b, not k_hme */
#define SVTME_PATH_NO_L1_FULL 2u   /* SVTME_NO_L1_FULL: full-SAD HME-L1 on k_stage_b, not k_l1_full */
#define SVTME_PATH_NO_L0_FULL 4u   /* SVTME_NO_L0_FULL: full-SAD stage A on k_stage_a, not k_l0_full */
#define SVTME_PATH_NO_FP_WIDE 8u   /* SVTME_NO_FP_WIDE: wide full-pel areas on k_stage_c1, not k_fp_wide */
#define SVTME_PATH_SPLIT_PASS 16u  /* SVTME_SPLIT_PASS: k_hme -> k_stage_c1 -> k_stage_e, not one k_hme */
#define SVTME_PATH_NO_A1_GATE 32u  /* SVTME_NO_A1_GATE: list-1 pre-HME searched with list 0 (no second A1 round) */
svtme_status svtme_set_paths(svtme_ctx *ctx, uint32_t paths);
/* Device pointer of the last job's record buffer (for RCCL all-gather). */
void *svtme_device_records(svtme_ctx *ctx, uint64_t *bytes);
/* The HIP stream (hipStream_t) the context launches on, for event timing. */
void *svtme_stream(svtme_ctx *ctx);

/* Number of 64x64 SBs of a width x height picture, and R for a job. */
uint32_t svtme_sb_total(uint32_t width, uint32_t height);
uint32_t svtme_job_ref_slots(const svtme_job *job);

/* Last error message of this thread (empty string if none). */
const char *svtme_last_error(void);

/* Fill `ctrl` as svt_aom_sig_deriv_me does for the non-RTC, non-screen-content
 * path (enc_mode_config.c:671-808) for preset `enc_mode`, qp and resolution. */
void svtme_derive_controls(int enc_mode, int qp, int input_resolution, int temporal_layer_index,
                           int hierarchical_levels, int frame_rate_q16, svtme_controls *ctrl);

/* Fill `ctrl` as the reference does for one temporal-filtering ME job
 * (me_type SVTME_ME_MCTF): svt_aom_sig_deriv_me_tf (enc_mode_config.c:814-854)
 * for tf_ctrls.hme_me_level 0..4 and tf_ctrls.qp_opt, the tf HME enables
 * (:1620-1645) and set_hme_search_params_mctf(ctx, 0) (temporal_filtering.c:2759). */
void svtme_derive_controls_tf(int hme_me_level, int qp_opt, int qp, int input_resolution, svtme_controls *ctrl);

/* ---------------------------------------------------------------------------
 * Per-kernel rtcd variants. Signatures identical to the pointers declared in
 * the reference's Source/Lib/Codec/aom_dsp_rtcd.h (line cited per entry).
 * ------------------------------------------------------------------------- */
/* The variants are reentrant (per-thread HIP stream and scratch). They never
 * return an error: on a HIP failure they leave their outputs untouched, set
 * svtme_last_error() and raise the calling thread's failure flag, which
 * svtme_rtcd_failed() returns (1) and clears, so the caller can re-run the call
 * on the variant it replaced (integration/svtme_svt_glue.c). */
int svtme_rtcd_failed(void);

/* aom_dsp_rtcd.h:779 svt_sad_loop_kernel */
void svt_sad_loop_kernel_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                             uint32_t block_height, uint32_t block_width, uint64_t *best_sad,
                             int16_t *x_search_center, int16_t *y_search_center, uint32_t src_stride_raw,
                             uint8_t skip_search_line, int16_t search_area_width, int16_t search_area_height);
/* aom_dsp_rtcd.h:856 svt_nxm_sad_kernel */
uint32_t svt_nxm_sad_kernel_hip(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                                uint32_t height, uint32_t width);
/* aom_dsp_rtcd.h:842 svt_ext_sad_calculation_8x8_16x16 */
void svt_ext_sad_calculation_8x8_16x16_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                           uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                           uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16, uint32_t mv,
                                           uint32_t *p_sad16x16, uint32_t *p_sad8x8, bool sub_sad);
/* aom_dsp_rtcd.h:848 svt_ext_sad_calculation_32x32_64x64 */
void svt_ext_sad_calculation_32x32_64x64_hip(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                             uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                             uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32);
/* aom_dsp_rtcd.h:853 svt_ext_all_sad_calculation_8x8_16x16 */
void svt_ext_all_sad_calculation_8x8_16x16_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                               uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                               uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                               uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                               bool sub_sad);
/* aom_dsp_rtcd.h:854 svt_ext_eight_sad_calculation_32x32_64x64 */
void svt_ext_eight_sad_calculation_32x32_64x64_hip(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                   uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                   uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]);
/* aom_dsp_rtcd.h:855 svt_initialize_buffer_32bits */
void svt_initialize_buffer_32bits_hip(uint32_t *pointer, uint32_t count128, uint32_t count32, uint32_t value);
/* aom_dsp_rtcd.h:841 downsample_2d */
void svt_aom_downsample_2d_hip(uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                               uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                               uint32_t decim_step);
/* aom_dsp_rtcd.h:863 sad_16b_kernel (mode-decision consumer; not on the ME path) */
uint32_t svt_aom_sad_16b_kernel_hip(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                                    uint32_t height, uint32_t width);

/* aom_dsp_rtcd.h:868 svt_pme_sad_loop_kernel (mode decision's full-pel MV
 * refinement, C at product_coding_loop.c:1811): SAD + MV rate of every visited
 * position of a (search_step-strided) area, strict-< update of *best_cost /
 * *best_mvx / *best_mvy (1/8-pel units). mv_cost_params is the reference's
 * MV_COST_PARAMS (mcomp.h:37); this library reads it through the layout below,
 * which integration/svtme_svt_glue.c checks against the reference header. */
struct svt_mv_cost_param;
#define SVTME_MVCOST_OFF_REF_MV 0         /* const MV *ref_mv (int16 row, col) */
#define SVTME_MVCOST_OFF_TYPE 12          /* MV_COST_TYPE (uint8): 0 entropy .. 5 none */
#define SVTME_MVCOST_OFF_MVJCOST 16       /* const int *mvjcost (4 joints) */
#define SVTME_MVCOST_OFF_MVCOST 24        /* const int *mvcost[2] (row, col; centred) */
#define SVTME_MVCOST_OFF_ERROR_PER_BIT 40 /* int error_per_bit */
void svt_pme_sad_loop_kernel_hip(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                                 uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                                 uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                                 int16_t search_position_start_x, int16_t search_position_start_y,
                                 int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                                 int16_t mvx, int16_t mvy);

#ifdef __cplusplus
}
#endif
#endif /* SVTME_H */
