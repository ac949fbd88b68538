/*
 * svtme_oracle_kernels.c — TEST INFRASTRUCTURE. CPU restatement of the
 * per-kernel rtcd functions the ME path dispatches to (reference
 * Source/Lib/Codec/aom_dsp_rtcd.h:779, 841, 842, 848, 853-856, 863), with
 * the reference signatures, used only as the checker of the `*_hip` variants
 * (tests/test_rtcd_*.py). It is itself pinned against the reference's C and
 * AVX2 kernels compiled from source (oracle/_ref, tests/golden/rtcd_cases.npz).
 * Never linked into or called by the product.
 */
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

static inline uint32_t absd(uint32_t a, uint32_t b) { return a > b ? a - b : b - a; }

/* compute_sad_c.c:20-37 (svt_fast_loop_nxm_sad_kernel via svt_nxm_sad_kernel_helper_c, :209) */
uint32_t svtora_nxm_sad_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                               uint32_t height, uint32_t width) {
    uint32_t sad = 0;
    for (uint32_t r = 0; r < height; r++, src += src_stride, ref += ref_stride)
        for (uint32_t c = 0; c < width; c++) sad += absd(src[c], ref[c]);
    return sad;
}

/* compute_sad_c.c:39-56 */
uint32_t svtora_sad_16b_kernel(const uint16_t *src, uint32_t src_stride, const uint16_t *ref, uint32_t ref_stride,
                               uint32_t height, uint32_t width) {
    uint32_t sad = 0;
    for (uint32_t r = 0; r < height; r++, src += src_stride, ref += ref_stride)
        for (uint32_t c = 0; c < width; c++) sad += absd(src[c], ref[c]);
    return sad;
}

/* compute_sad_c.c:58-101: position row stride is src_stride_raw, block-row
 * stride ref_stride; with 16-wide blocks of <= 16 rows and skip_search_line
 * only odd search rows are searched; strict-< raster argmin from 0xffffff. */
void svtora_sad_loop_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                            uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_search_center,
                            int16_t *y_search_center, uint32_t src_stride_raw, uint8_t skip_search_line,
                            int16_t search_area_width, int16_t search_area_height) {
    *best_sad      = 0xffffff;
    const int skip = block_width == 16 && block_height <= 16 && skip_search_line;
    for (int16_t ys = 0; ys < search_area_height; ys++) {
        const uint8_t *row = ref + (size_t)ys * src_stride_raw;
        if (skip && (ys & 1) == 0)
            continue;
        for (int16_t xs = 0; xs < search_area_width; xs++) {
            const uint32_t sad = svtora_nxm_sad_kernel(src, src_stride, row + xs, ref_stride, block_height, block_width);
            if (sad < *best_sad) {
                *best_sad        = sad;
                *x_search_center = xs;
                *y_search_center = ys;
            }
        }
    }
}

/* 8x8 SAD of one block, sub-sampled (even rows, x2) or full (motion_estimation.c:42-92) */
static uint32_t sad8(const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs, bool sub) {
    return sub ? svtora_nxm_sad_kernel(src, 2 * ss, ref, 2 * rs, 4, 8) << 1 : svtora_nxm_sad_kernel(src, ss, ref, rs, 8, 8);
}

static inline void upd(uint32_t sad, uint32_t *best, uint32_t *best_mv, uint32_t mv) {
    if (sad < *best) {
        *best    = sad;
        *best_mv = mv;
    }
}

/* motion_estimation.c:98-164: the 4 8x8 and the 16x16 SADs at one position */
void svtora_ext_sad_calculation_8x8_16x16(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                          uint32_t ref_stride, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                          uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16, uint32_t mv,
                                          uint32_t *p_sad16x16, uint32_t *p_sad8x8, bool sub_sad) {
    for (int b = 0; b < 4; b++) {
        const uint32_t oy = (uint32_t)(b >> 1) * 8, ox = (uint32_t)(b & 1) * 8;
        p_sad8x8[b] = sad8(src + oy * src_stride + ox, src_stride, ref + oy * ref_stride + ox, ref_stride, sub_sad);
    }
    for (int b = 0; b < 4; b++) upd(p_sad8x8[b], &p_best_sad_8x8[b], &p_best_mv8x8[b], mv);
    const uint32_t s16 = p_sad8x8[0] + p_sad8x8[1] + p_sad8x8[2] + p_sad8x8[3];
    upd(s16, p_best_sad_16x16, p_best_mv16x16, mv);
    *p_sad16x16 = s16;
}

/* motion_estimation.c:171-205 */
void svtora_ext_sad_calculation_32x32_64x64(const uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                            uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                            uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32) {
    uint32_t s64 = 0;
    for (int q = 0; q < 4; q++) {
        const uint32_t s = p_sad16x16[4 * q] + p_sad16x16[4 * q + 1] + p_sad16x16[4 * q + 2] + p_sad16x16[4 * q + 3];
        p_sad32x32[q]    = s;
        upd(s, &p_best_sad_32x32[q], &p_best_mv32x32[q], mv);
        s64 += s;
    }
    upd(s64, p_best_sad_64x64, p_best_mv64x64, mv);
}

static inline uint32_t mv_plus_x(uint32_t mv, int dx) {
    const int16_t x = (int16_t)(mv & 0xFFFF), y = (int16_t)(mv >> 16);
    return ((uint32_t)(uint16_t)y << 16) | (uint16_t)(int16_t)(x + dx);
}

/* motion_estimation.c:210-362: 8 consecutive x positions; the 16 16x16 blocks
 * are visited in raster order and stored at their Z-order index
 * (offsets[] :340); p_eight_sad8x8 is not written. */
void svtora_ext_all_sad_calculation_8x8_16x16(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                              uint32_t ref_stride, uint32_t mv, uint32_t *p_best_sad_8x8,
                                              uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                              uint32_t *p_best_mv16x16, uint32_t p_eight_sad16x16[16][8],
                                              uint32_t p_eight_sad8x8[64][8], bool sub_sad) {
    static const int zoff[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
    (void)p_eight_sad8x8;
    for (int by = 0; by < 4; by++)
        for (int bx = 0; bx < 4; bx++) {
            const int p16 = zoff[4 * by + bx], p8 = 4 * p16;
            const uint8_t *s = src + 16 * by * src_stride + 16 * bx;
            const uint8_t *r = ref + 16 * by * ref_stride + 16 * bx;
            for (int k = 0; k < 8; k++) {
                const uint32_t m = mv_plus_x(mv, k);
                uint32_t t       = 0;
                for (int b = 0; b < 4; b++) {
                    const uint32_t oy = (uint32_t)(b >> 1) * 8, ox = (uint32_t)(b & 1) * 8;
                    const uint32_t v =
                        sad8(s + oy * src_stride + ox, src_stride, r + oy * ref_stride + ox + k, ref_stride, sub_sad);
                    upd(v, &p_best_sad_8x8[p8 + b], &p_best_mv8x8[p8 + b], m);
                    t += v;
                }
                p_eight_sad16x16[p16][k] = t;
                upd(t, &p_best_sad_16x16[p16], &p_best_mv16x16[p16], m);
            }
        }
}

/* motion_estimation.c:369-425 */
void svtora_ext_eight_sad_calculation_32x32_64x64(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                  uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                  uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]) {
    for (int k = 0; k < 8; k++) {
        const uint32_t m = mv_plus_x(mv, k);
        uint32_t s64     = 0;
        for (int q = 0; q < 4; q++) {
            const uint32_t s = p_sad16x16[4 * q][k] + p_sad16x16[4 * q + 1][k] + p_sad16x16[4 * q + 2][k] +
                p_sad16x16[4 * q + 3][k];
            p_sad32x32[q][k] = s;
            upd(s, &p_best_sad_32x32[q], &p_best_mv32x32[q], m);
            s64 += s;
        }
        upd(s64, p_best_sad_64x64, p_best_mv64x64, m);
    }
}

/* me_sad_calculation.c:14-17 */
void svtora_initialize_buffer_32bits(uint32_t *pointer, uint32_t count128, uint32_t count32, uint32_t value) {
    for (uint32_t i = 0; i < count128 * 4 + count32; i++) pointer[i] = value;
}

/* pic_analysis_process.c:130-158: 2x2 average at the (half, half) phase */
void svtora_downsample_2d(const uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                          uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                          uint32_t decim_step) {
    const uint32_t half = decim_step >> 1;
    for (uint32_t v = half, oy = 0; v < input_area_height; v += decim_step, oy++) {
        const uint8_t *cur = input_samples + (size_t)v * input_stride, *prev = cur - input_stride;
        for (uint32_t h = half, ox = 0; h < input_area_width; h += decim_step, ox++) {
            const uint32_t sum = (uint32_t)prev[h - 1] + prev[h] + cur[h - 1] + cur[h];
            decim_samples[(size_t)oy * decim_stride + ox] = (uint8_t)((sum + 2) >> 2);
        }
    }
}

/* MV_COST_PARAMS (mcomp.h:37-48), restated layout: this file does not include
 * the reference headers */
typedef struct {
    const int16_t *ref_mv; /* MV: row, col */
    int16_t full_ref_mv[2];
    uint8_t mv_cost_type; /* MV_COST_TYPE: UENUM1BYTE (mcomp.h:29-36) */
    const int *mvjcost;
    const int *mvcost[2];
    int error_per_bit, early_exit_th, sad_per_bit;
} ora_mv_cost_params;

/* svt_mv_err_cost (mcomp.c:44-68) with svt_mv_cost (mcomp.h:134-137) and
 * svt_av1_get_mv_joint (rd_cost.c:55-60); shift = RDDIV_BITS 7 +
 * AV1_PROB_COST_SHIFT 9 - RD_EPB_SHIFT 6 + PIXEL_TRANSFORM_ERROR_SCALE 4 */
static int ora_mv_err_cost(int16_t row, int16_t col, const ora_mv_cost_params *p) {
    const int dr = (int16_t)(row - p->ref_mv[0]), dc = (int16_t)(col - p->ref_mv[1]);
    /* diff and abs_diff are int16 MVs (mcomp.c:46-47): |-32768| wraps back to -32768 */
    const int ar = (int16_t)(dr < 0 ? -dr : dr), ac = (int16_t)(dc < 0 ? -dc : dc);
    const int sh = 14;
    switch (p->mv_cost_type) {
    case 0: { /* the reference's `if (mvcost)` tests the array parameter: always taken */
        const int j  = dr == 0 ? (dc == 0 ? 0 : 1) : (dc == 0 ? 2 : 3);
        const int cr = dr < -16384 ? -16384 : (dr > 16384 ? 16384 : dr);
        const int cc = dc < -16384 ? -16384 : (dc > 16384 ? 16384 : dc);
        const int64_t v = (int64_t)(p->mvjcost[j] + p->mvcost[0][cr] + p->mvcost[1][cc]) * p->error_per_bit;
        return (int)((v + (((int64_t)1 << sh) >> 1)) >> sh);
    }
    case 1: return (2 * (ar + ac)) >> 3;
    case 2: return 0;
    case 3: return (1 * (ar + ac)) >> 3;
    case 4: {
        const int64_t v = (int64_t)((ar + ac) << 8) * p->error_per_bit;
        return (int)((v + (((int64_t)1 << sh) >> 1)) >> sh);
    }
    default: return 0;
    }
}

/* svt_pme_sad_loop_kernel_c (product_coding_loop.c:1811-1860): the column
 * counter and x step carry across rows; columns with fewer than 8 left are
 * skipped while the counter is 0 */
void svtora_pme_sad_loop_kernel(const void *mv_cost_params, const uint8_t *src, uint32_t src_stride,
                                const uint8_t *ref, uint32_t ref_stride, uint32_t block_height,
                                uint32_t block_width, uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                                int16_t search_position_start_x, int16_t search_position_start_y,
                                int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                                int16_t mvx, int16_t mvy) {
    const ora_mv_cost_params *p = (const ora_mv_cost_params *)mv_cost_params;
    int16_t col_num = 0, step_x = 1;
    for (int16_t y = 0; y < search_area_height; y += search_step) {
        for (int16_t x = 0; x < search_area_width; x += step_x) {
            if ((search_area_width - x) < 8 && col_num == 0)
                continue;
            if (col_num == 7) {
                col_num = 0;
                step_x  = search_step;
            } else {
                col_num++;
                step_x = 1;
            }
            uint32_t cost = 0;
            for (uint32_t r = 0; r < block_height; r++)
                for (uint32_t c = 0; c < block_width; c++)
                    cost += absd(src[r * src_stride + c], ref[(size_t)y * ref_stride + x + r * ref_stride + c]);
            const uint32_t rx = (uint32_t)(search_position_start_x + x), ry = (uint32_t)(search_position_start_y + y);
            const int16_t col = (int16_t)(mvx + rx * 8), row = (int16_t)(mvy + ry * 8);
            cost += (uint32_t)ora_mv_err_cost(row, col, p);
            if (cost < *best_cost) {
                *best_mvx  = col;
                *best_mvy  = row;
                *best_cost = cost;
            }
        }
    }
}
