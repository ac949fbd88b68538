/*
 * svtme_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Shared ABI of the two CPU checkers of the ME path:
 *   svtora_*  — oracle/svtme_oracle.c, a from-scratch C restatement of the
 *               reference's open-loop ME (Source/Lib/Codec/motion_estimation.c).
 *   svtref_*  — oracle/ref_harness.c, a driver that links the REFERENCE's own
 *               motion_estimation.c + SAD kernels compiled from
 *               /root/reference (oracle/_ref/, container build only).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * these; the product (libsvtme.so) never links them.
 */
#ifndef SVTME_ORACLE_H
#define SVTME_ORACLE_H

#include "../include/svtme.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A picture pyramid in host memory. Each pointer is the START of the padded
 * allocation (top-left padding sample). Geometry for an aligned W x H picture:
 *   full      : stride W + 144,   rows H + 144,   origin (72, 72)
 *   quarter   : stride W/2 + 64,  rows H/2 + 64,  origin (32, 32)
 *   sixteenth : stride W/4 + 32,  rows H/4 + 32,  origin (16, 16)   */
typedef struct svtme_pyr {
    uint8_t *full;
    uint8_t *quarter;
    uint8_t *sixteenth;
} svtme_pyr;

static inline uint32_t svtme_align8(uint32_t v) { return (v + 7u) & ~7u; }

/* Build the padded pyramid of an 8-bit picture (w x h visible samples). */
void svtora_build_pyramid(const uint8_t *y, uint32_t stride, uint32_t w, uint32_t h, svtme_pyr *out);
void svtref_build_pyramid(const uint8_t *y, uint32_t stride, uint32_t w, uint32_t h, svtme_pyr *out);

/* Run open-loop ME over the job's SB range. refs[l * 4 + r] is the pyramid of
 * reference (l, r). out: sb_count x R records; sbres: sb_count results or NULL.
 * nthreads > 1 splits the SB range into contiguous bands (ME segments). */
svtme_status svtora_me(const svtme_job *job, const svtme_pyr *cur, const svtme_pyr *refs, svtme_ref_record *out,
                       svtme_sb_result *sbres, int nthreads);
svtme_status svtref_me(const svtme_job *job, const svtme_pyr *cur, const svtme_pyr *refs, svtme_ref_record *out,
                       svtme_sb_result *sbres, int nthreads);

/* svtora only: absolute differences evaluated by svtora_me calls since the last
 * reset (every SAD of the searches: positions x block pixels); reset != 0 clears it. */
uint64_t svtora_absdiff(int reset);

/* svtref only: select the reference kernels behind the rtcd pointers:
 * 0 = C (asm=0), 1 = the x86 AVX2 picks of aom_dsp_rtcd.c:501-515 capped at AVX2. */
void svtref_set_simd(int simd);

/* svtref only: controls exactly as the reference's svt_aom_sig_deriv_me derives
 * them (enc_mode_config.c:671), for validating svtme_derive_controls. */
void svtref_derive_controls(int enc_mode, int qp, int input_resolution, int temporal_layer_index,
                            int hierarchical_levels, int frame_rate_q16, svtme_controls *ctrl);
/* svtref only: TF-ME controls (svt_aom_sig_deriv_me_tf, enc_mode_config.c:814) for
 * tf_ctrls.hme_me_level / qp_opt, for validating svtme_derive_controls_tf. */
void svtref_derive_controls_tf(int hme_me_level, int qp_opt, int qp, int input_resolution, svtme_controls *ctrl);

#ifdef __cplusplus
}
#endif
#endif
