// svtme_device.h — device-side layouts shared by the HIP kernels and the host
// launcher (svtme_host.cpp). gfx950 (MI355X) only.
#pragma once
#include <stdint.h>

#include "../../include/svtme.h"

// Device plane margins. The LOGICAL padding the search clamps use is the
// reference's (72 / 32 / 16, reference_object.c:243-305); the device margins
// are at least as wide and keep each interior row start 16-byte aligned and
// 8 bytes of slack on the right for aligned dword loads. Margins hold the same
// edge-replicated samples as the reference's padding.
#define SVTME_DEV_FULL_LEFT 80
#define SVTME_DEV_FULL_TOP 72
#define SVTME_DEV_Q_LEFT 32
#define SVTME_DEV_Q_TOP 32
#define SVTME_DEV_S_LEFT 16
#define SVTME_DEV_S_TOP 16

struct DevPlane {
    uint8_t *base;   // interior sample (0, 0); negative offsets reach the padding
    int32_t stride;  // bytes per row (multiple of 64)
    int32_t width;   // interior width
    int32_t height;  // interior height
    int32_t pad;     // logical padding (org_x == org_y of the reference plane)
};

struct DevPyramid {
    DevPlane lv[3];  // 0 = full, 1 = quarter, 2 = sixteenth
};

// Stage-A result of one search (svtme_stages.hip). Index layout per SB:
// [0, 8) zz SAD by slot (sad = raw sub-sampled n x m sum), [8, 24) pre-HME
// slot * 2 + region, [24, 56) HME level 0 slot * 4 + quadrant (sx * 2 + sy).
struct ARes {
    uint32_t sad;
    int16_t x, y; // final (scaled, absolute) search-centre MV
};
#define SVTME_A_ZZ 0
#define SVTME_A_PH 8
#define SVTME_A_L0 24
#define SVTME_A_N 56

// Per-SB state between the stages (svtme_stages.hip). Stage D writes each
// slot's zz SAD and do_ref after the zz / pre-HME pruning and the level-0
// centres after the worst-quadrant replacement; stage B writes the level-1/2
// refinement of every (slot, quadrant); stage C selects the search centre
// from the highest enabled level (set_final_seach_centre_sb).
struct BState {
    uint64_t lsad[8][4]; // level 0, [slot][q = sx * 2 + sy]
    uint64_t hsad[8][4]; // highest enabled level above 0
    int16_t lx[8][4], ly[8][4];
    int16_t hx[8][4], hy[8][4];
    uint32_t zz[8];
    uint8_t do_ref[8];
    // real-time tune on the split path (k_stage_d<true>): the HME-L0 area of
    // every slot from slot 0's centre, and the slots whose HME-L0 runs (bit s)
    int16_t rt_sa[8][2];
    uint8_t rt_need;
};

// Per (SB, reference record) state the wide full-pel stage (k_stage_c1)
// leaves for the per-SB decode (k_stage_e), svtme_stages.hip.
struct CSlot {
    uint64_t hme_sad;
    uint32_t zz;
    int16_t sc_x, sc_y;        // HME search centre (record fields)
    int16_t xo, yo, w, xc, yc; // full-pel window origin and width, probe centre
    uint8_t searched, do_ref, probe, tf_exit;
};

// Parameters of one picture job as the kernel sees them.
struct DevJob {
    svtme_job job;                 // controls + picture description (host copy)
    DevPyramid cur;
    DevPyramid ref[2][4];
    svtme_ref_record *out_records; // [sb_count][R]
    svtme_sb_result *out_sb;       // [sb_count] or nullptr
    uint32_t R;
    uint32_t pic_w_b64;
    ARes *ares;                    // [sb_count][SVTME_A_N] stage-A results
    BState *bst;                   // [sb_count] stage-B state
    uint32_t ta_count;             // stage-A searches per SB
    uint8_t ta_list[SVTME_A_N];    // their ARes indices
    uint32_t ta1_count;            // real-time tune, split path: the second stage-A round
    uint8_t ta1_list[8];           // (TA_L0RT << 3 | slot)
    uint32_t tb_count;             // stage-B refinements per SB
    uint8_t tb_list[32];           // their (slot << 2 | quadrant)
    unsigned long long *keys;      // [sb_count][R][85] full-pel argmin keys (sad << 32 | order)
    CSlot *cslot;                  // [sb_count][R]
    uint32_t parts;                // search-row bands per (SB, reference) in k_stage_c1; 0 = per-SB k_stage_c
    // per-slot search parameters independent of the SB (svtme_hme_prepare, host)
    uint16_t sdist[8];             // |picture distance| of slot s (ref_dist_const)
    int16_t l0_sa[8][2];           // HME-L0 area (get_hme_l0_search_area)
    int16_t ph_sa[8][2][2];        // pre-HME region areas (prehme_core)
    uint32_t paths;                // SVTME_PATH_* of the submitting context (host dispatch only)
};

// A launch over a batch of picture jobs (svtme_submit_batch_device). The jobs
// live in device memory; start[k] is the first work unit (wave or workgroup,
// per stage) of job k in this launch, start[n..] = UINT32_MAX. Unit u belongs
// to the job with the largest start[k] <= u (constant-index compares: the
// kernel argument is never indexed dynamically).
#define SVTME_MAX_BATCH 16
struct DevBatch {
    const DevJob *jobs;
    uint32_t n;
    uint32_t total; // units of this launch
    uint32_t start[SVTME_MAX_BATCH];
};

static inline uint32_t svtme_round_up(uint32_t v, uint32_t a) { return (v + a - 1) / a * a; }
static inline uint32_t svtme_align8_u(uint32_t v) { return (v + 7u) & ~7u; }

// plane geometry for an aligned W x H picture
static inline void svtme_plane_geometry(int level, uint32_t W, uint32_t H, uint32_t *w, uint32_t *h, uint32_t *left,
                                        uint32_t *top, uint32_t *stride, uint32_t *rows, uint32_t *pad) {
    if (level == 0) {
        *w = W, *h = H, *left = SVTME_DEV_FULL_LEFT, *top = SVTME_DEV_FULL_TOP, *pad = SVTME_PAD_FULL;
        *stride = svtme_round_up(W + SVTME_DEV_FULL_LEFT + 88, 64);
    } else if (level == 1) {
        *w = W / 2, *h = H / 2, *left = SVTME_DEV_Q_LEFT, *top = SVTME_DEV_Q_TOP, *pad = SVTME_PAD_QUARTER;
        *stride = svtme_round_up(W / 2 + SVTME_DEV_Q_LEFT + 40, 64);
    } else {
        *w = W / 4, *h = H / 4, *left = SVTME_DEV_S_LEFT, *top = SVTME_DEV_S_TOP, *pad = SVTME_PAD_SIXTEENTH;
        *stride = svtme_round_up(W / 4 + SVTME_DEV_S_LEFT + 24, 64);
    }
    *rows = *h + 2 * *top;
}
