// svtme_kernels.hip — MI355X (gfx950) kernels of the open-loop ME stage.
//
//   k_build_level   : padded full / quarter / sixteenth planes of one picture
//                     (svt_aom_downsample_filtering_input_picture + generate_padding,
//                      reference pic_analysis_process.c:130-158, :1945-2002;
//                      pic_operators.c:338-383, :491)
//   k_me_sb         : one workgroup per 64x64 superblock, all references:
//                     zz SAD -> pre-HME -> HME L0/L1/L2 -> search centre ->
//                     full-pel search with the 85-PU argmin -> pruning ->
//                     candidate arrays and distortions
//                     (svt_aom_motion_estimation_b64, motion_estimation.c:3076-3153)
//
// Arithmetic is integer only: |a-b| accumulation with v_sad_u8 on dword-packed
// pixels, unaligned pixel runs rebuilt from aligned dwords with v_alignbyte_b32,
// argmins as 64-bit (sad, raster order) keys reduced across the wavefront with
// shuffles and across waves with LDS ds_min_u64. No MFMA: this is not a
// contraction. Scalar control (search-area derivation, pruning, tie rules) runs
// on lane 0 of wave 0 against per-SB state in LDS, between barriers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svtme_device.h"

#define ME_MAX_TASKS 32
#define ME_THREADS 256
#define U32MAX 0xFFFFFFFFu

// Diagnostic build only (-DSVTME_STAMPS): lane 0 stamps s_memtime at phase
// boundaries into dj.stamps[sb][16]; the shipped kernel contains no stamp.
#ifdef SVTME_STAMPS
#define SVTME_STAMP(k)                                                                                              \
    do {                                                                                                            \
        if (threadIdx.x == 0 && dj.stamps)                                                                          \
            dj.stamps[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime();                               \
    } while (0)
#else
#define SVTME_STAMP(k) do { } while (0)
#endif

// ----------------------------------------------------------------------------
// Pyramid
// ----------------------------------------------------------------------------
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// level 0: from the caller's picture (8-bit or 10-bit MSB), pad-to-8 + edge replicate.
// One thread writes 4 bytes of the padded plane (margins included).
template <bool TEN_BIT>
__global__ void __launch_bounds__(256) k_build_full(const void *__restrict__ src, uint32_t src_stride, int w, int h,
                                                    DevPlane dst, int left, int top, int rows) {
    const int dw_per_row = dst.stride >> 2;
    const int idx        = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= dw_per_row * rows)
        return;
    const int ry = idx / dw_per_row, rx4 = (idx - ry * dw_per_row) * 4;
    const int y  = clampi(ry - top, 0, h - 1);
    uint32_t v   = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = clampi(rx4 + k - left, 0, w - 1);
        uint32_t p;
        if (TEN_BIT)
            p = (uint32_t)(((const uint16_t *)src)[(size_t)y * src_stride + x] >> 2);
        else
            p = ((const uint8_t *)src)[(size_t)y * src_stride + x];
        v |= p << (8 * k);
    }
    uint32_t *row = (uint32_t *)(dst.base - (size_t)top * dst.stride - left);
    row[idx]      = v;
}

// levels 1, 2: 2x2 mean (sum + 2) >> 2 of the previous level's interior, edge replicate
__global__ void __launch_bounds__(256) k_build_down(DevPlane prev, DevPlane dst, int left, int top, int rows) {
    const int dw_per_row = dst.stride >> 2;
    const int idx        = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= dw_per_row * rows)
        return;
    const int ry = idx / dw_per_row, rx4 = (idx - ry * dw_per_row) * 4;
    const int y  = clampi(ry - top, 0, dst.height - 1);
    const uint8_t *a = prev.base + (size_t)(2 * y) * prev.stride;
    const uint8_t *b = a + prev.stride;
    uint32_t v       = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x    = clampi(rx4 + k - left, 0, dst.width - 1);
        const uint32_t s = (uint32_t)a[2 * x] + a[2 * x + 1] + b[2 * x] + b[2 * x + 1];
        v |= ((s + 2) >> 2) << (8 * k);
    }
    uint32_t *row = (uint32_t *)(dst.base - (size_t)top * dst.stride - left);
    row[idx]      = v;
}

// ----------------------------------------------------------------------------
// Per-SB state (MeContext fields of the open-loop path, me_context.h:366-509)
// ----------------------------------------------------------------------------
struct SadTask {
    const uint8_t *ref;  // global: window sample of search position (0, 0), block row 0
    int32_t ref_stride;  // bytes between block rows (x2 for SUB_SAD)
    int32_t pos_stride;  // bytes between search rows
    int32_t item_begin;
    int16_t sa_w, sa_h;
    uint16_t src_off;    // LDS offset of the source block
    uint16_t src_stride; // LDS bytes between block rows
    uint8_t bw;          // block width (bytes)
    uint8_t bh;          // block rows
    uint8_t skip;        // search odd rows only (compute_sad_c.c:74-79)
    uint8_t nq;          // quads (4 positions) per search row
    uint8_t rows;        // searched rows
    uint8_t pad[3];
};

struct PreHme {
    uint64_t sad;
    int16_t col, row;
    uint16_t sa_w, sa_h;
    uint8_t valid;
};

struct FpRef {           // full-pel search of one reference
    int16_t xo, yo;      // window origin (MV of position (0,0))
    int16_t w, h;
    int32_t order_base;  // 0 for the var-check centre, 1 for the main search
    int32_t item_begin;
    uint8_t slot;        // 0..7 = list * 4 + ref
    uint8_t nq;
    uint8_t pad[2];
};

struct SbState {
    // source blocks (64x64 full, 32x32 quarter, 16x16 sixteenth)
    uint8_t src[64 * 64 + 32 * 32 + 16 * 16];
    // task machinery
    SadTask tasks[ME_MAX_TASKS];
    unsigned long long task_best[ME_MAX_TASKS];
    int32_t ntasks, nitems;
    // HME state
    int16_t l0x[2][4][2][2], l0y[2][4][2][2], l1x[2][4][2][2], l1y[2][4][2][2], l2x[2][4][2][2], l2y[2][4][2][2];
    uint64_t l0sad[2][4][2][2], l1sad[2][4][2][2], l2sad[2][4][2][2];
    int16_t ox[2][4][2][2], oy[2][4][2][2]; // per-task search-area origins (scratch)
    PreHme prehme[2][4][2];
    uint8_t performed_phme[2][4][2];
    // search results (SearchResults, me_context.h:348-355)
    uint64_t hme_sad[2][4];
    int16_t hme_sc_x[2][4], hme_sc_y[2][4];
    uint8_t do_ref[2][4], searched[2][4];
    uint32_t reduce_div[2][4];
    uint32_t zz_sad[2][4];
    uint32_t nxm_sad[8]; // scratch for zz / check_00_center SADs
    // integer search
    FpRef fp[8];
    int32_t nfp, fp_items;
    int16_t is_w[2][4], is_h[2][4], is_wb[2][4], is_hb[2][4], is_xc[2][4], is_yc[2][4];
    uint64_t is_best_hme[2][4];
    unsigned long long pu_key[8][SVTME_PU_COUNT];
    uint32_t best_sad[2][4][SVTME_PU_COUNT];
    uint32_t best_mv[2][4][SVTME_PU_COUNT];
    uint32_t me_distortion[SVTME_PU_COUNT];
    uint8_t cand0[SVTME_PU_COUNT + 3]; // first candidate byte per PU (GM detection)
    int32_t flag; // uniform decisions broadcast from lane 0
    uint32_t b64_w, b64_h, ox_sb, oy_sb;
};

__device__ __forceinline__ int16_t i16(int v) { return (int16_t)v; }
__device__ __forceinline__ int absi(int v) { return v < 0 ? -v : v; }
__device__ __forceinline__ uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// motion_estimation.c:1239-1243
__device__ __forceinline__ uint16_t scaled_dist(uint16_t dist) {
    uint8_t round_up = ((dist % 8) == 0) ? 0 : 1;
    return (uint16_t)(((dist * 5) / 8) + round_up);
}

__device__ __forceinline__ uint16_t ref_dist(const svtme_job &j, int l, int r) {
    int64_t d = (int64_t)j.picture_number - (int64_t)j.ref_picture_number[l][r];
    return (uint16_t)(int16_t)(d < 0 ? -d : d);
}

__device__ __forceinline__ bool tl_or_l0(const svtme_job &j, int l) { return j.temporal_layer_index > 0 || l == 0; }

// ----------------------------------------------------------------------------
// Wavefront reductions
// ----------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long t = __shfl_xor(v, o, 64);
        v                    = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ----------------------------------------------------------------------------
// SAD of 4 consecutive positions (x0..x0+3) of one block row.
// Pixel runs at arbitrary byte offsets are rebuilt from aligned dwords:
// run(k) = alignbyte(d[k+1], d[k], shift).
// ----------------------------------------------------------------------------
template <int SH>
__device__ __forceinline__ void quad_row(const uint32_t *__restrict__ rd, const uint32_t *__restrict__ sd, int nd,
                                         uint32_t last_mask, uint32_t acc[4]) {
    uint32_t d0 = rd[0], d1 = rd[1];
    for (int j = 0; j < nd; j++) {
        const uint32_t d2 = rd[j + 2];
        const uint32_t m  = (j == nd - 1) ? last_mask : 0xFFFFFFFFu; // partial last dword (block width % 4)
        const uint32_t s  = sd[j] & m;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int t = SH + k;
            uint32_t run;
            if (t == 0)
                run = d0;
            else if (t < 4)
                run = __builtin_amdgcn_alignbyte(d1, d0, t);
            else if (t == 4)
                run = d1;
            else
                run = __builtin_amdgcn_alignbyte(d2, d1, t - 4);
            acc[k] = __builtin_amdgcn_sad_u8(run & m, s, acc[k]);
        }
        d0 = d1;
        d1 = d2;
    }
}

// SADs of positions x0..x0+3 for a bw-byte x bh-row block
__device__ __forceinline__ void quad_sad(const uint8_t *ref, int ref_stride, const uint8_t *src_lds, int src_stride,
                                         int bw, int bh, uint32_t acc[4]) {
    acc[0] = acc[1] = acc[2] = acc[3] = 0;
    const int sh = (int)((uintptr_t)ref & 3);
    const uint8_t *ra = ref - sh;
    const int nd = (bw + 3) >> 2;
    const uint32_t last_mask = (bw & 3) ? ((1u << (8 * (bw & 3))) - 1u) : 0xFFFFFFFFu;
    for (int r = 0; r < bh; r++) {
        const uint32_t *rd = (const uint32_t *)(ra + (size_t)r * ref_stride);
        const uint32_t *sd = (const uint32_t *)(src_lds + r * src_stride);
        switch (sh) {
        case 0: quad_row<0>(rd, sd, nd, last_mask, acc); break;
        case 1: quad_row<1>(rd, sd, nd, last_mask, acc); break;
        case 2: quad_row<2>(rd, sd, nd, last_mask, acc); break;
        default: quad_row<3>(rd, sd, nd, last_mask, acc); break;
        }
    }
}

// Execute all sad_loop tasks of a stage (compute_sad_c.c:58-101 semantics):
// every task's best key (sad << 32 | y << 16 | x) ends in st.task_best[t].
__device__ void run_sad_tasks(SbState &st) {
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < ME_MAX_TASKS)
        st.task_best[tid] = ~0ull;
    __syncthreads();
    const int ntasks = st.ntasks, nitems = st.nitems;
    for (int base = 0; base < nitems; base += ME_THREADS) {
        const int i          = base + tid;
        unsigned long long k = ~0ull;
        int t                = -1;
        if (i < nitems) {
            t = 0;
            while (t + 1 < ntasks && st.tasks[t + 1].item_begin <= i) t++;
            const SadTask &T = st.tasks[t];
            const int li     = i - T.item_begin;
            const int yy = li / T.nq, q = li - yy * T.nq;
            const int y      = T.skip ? 2 * yy + 1 : yy;
            const int x0     = 4 * q;
            uint32_t acc[4];
            quad_sad(T.ref + (size_t)y * T.pos_stride + x0, T.ref_stride, st.src + T.src_off, T.src_stride, T.bw,
                     T.bh, acc);
#pragma unroll
            for (int s = 0; s < 4; s++)
                if (x0 + s < T.sa_w) {
                    unsigned long long kk = ((unsigned long long)acc[s] << 32) | ((uint32_t)y << 16) | (uint32_t)(x0 + s);
                    k                     = kk < k ? kk : k;
                }
        }
        // wave-level pre-reduction when the whole wave works on one task
        const int t0 = __shfl(t, 0, 64);
        if (__all(t == t0)) {
            k = wave_min_u64(k);
            if (lane == 0 && t0 >= 0)
                atomicMin(&st.task_best[t0], k);
        } else if (t >= 0) {
            atomicMin(&st.task_best[t], k);
        }
    }
    __syncthreads();
}

// Append a sad_loop task (lane 0 only).
__device__ void add_task(SbState &st, const uint8_t *ref, int ref_stride, int pos_stride, int src_off, int src_stride,
                         int bw, int bh, int sa_w, int sa_h, int skip) {
    SadTask &T   = st.tasks[st.ntasks];
    T.ref        = ref;
    T.ref_stride = ref_stride;
    T.pos_stride = pos_stride;
    T.src_off    = (uint16_t)src_off;
    T.src_stride = (uint16_t)src_stride;
    T.bw         = (uint8_t)bw;
    T.bh         = (uint8_t)bh;
    T.sa_w       = (int16_t)sa_w;
    T.sa_h       = (int16_t)sa_h;
    // compute_sad_c.c:74: line skipping only for 16-wide blocks of <= 16 rows
    T.skip       = (uint8_t)(skip && bw == 16 && bh <= 16);
    T.nq         = (uint8_t)(sa_w > 0 ? (sa_w + 3) / 4 : 0);
    int rows     = sa_h > 0 ? sa_h : 0;
    if (T.skip)
        rows = rows / 2;
    if (sa_w <= 0)
        rows = 0;
    T.rows       = (uint8_t)0; // unused (rows can exceed 255)
    T.item_begin = st.nitems;
    st.nitems += rows * T.nq;
    st.ntasks++;
}

// sad_loop result of task t: best_sad initialised to 0xffffff, centre untouched
// if nothing beats it (compute_sad_c.c:71, :90)
__device__ __forceinline__ void task_result(const SbState &st, int t, uint64_t *best, int16_t *x, int16_t *y) {
    const unsigned long long k = st.task_best[t];
    const uint32_t sad         = (uint32_t)(k >> 32);
    if (k != ~0ull && sad < 0xffffffu) {
        *best = sad;
        *x    = (int16_t)(k & 0xFFFF);
        *y    = (int16_t)((k >> 16) & 0xFFFF);
    } else {
        *best = 0xffffff;
    }
}

// ----------------------------------------------------------------------------
// zz SAD / check_00_center: n x m SADs of the 64-wide source (sub rows) against
// full-res positions; one wavefront per request (compute_sad_c.c:20-37).
// ----------------------------------------------------------------------------
struct NxmReq {
    const uint8_t *ref; // window top-left (block row 0)
    int32_t stride;     // bytes between block rows (x2 for sub)
};

__device__ void run_nxm(SbState &st, const NxmReq *reqs, int nreq, int rows, int width, int src_stride) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wd4 = (width + 3) >> 2;
    for (int q = wid; q < nreq; q += ME_THREADS / 64) {
        uint32_t acc = 0;
        const int sh = (int)((uintptr_t)reqs[q].ref & 3);
        for (int e = lane; e < rows * wd4; e += 64) {
            const int r = e / wd4, j = e - r * wd4;
            const uint8_t *rp  = reqs[q].ref + (size_t)r * reqs[q].stride + 4 * j;
            const uint32_t *da = (const uint32_t *)(rp - sh);
            uint32_t run       = sh ? __builtin_amdgcn_alignbyte(da[1], da[0], sh) : da[0];
            uint32_t s         = *(const uint32_t *)(st.src + r * src_stride + 4 * j);
            const int valid    = width - 4 * j; // bytes of this dword inside the block
            if (valid < 4) {
                const uint32_t m = (1u << (8 * valid)) - 1u;
                run &= m;
                s &= m;
            }
            acc = __builtin_amdgcn_sad_u8(run, s, acc);
        }
        acc = wave_sum_u32(acc);
        if (lane == 0)
            st.nxm_sad[q] = acc;
    }
    __syncthreads();
}

// ----------------------------------------------------------------------------
// Full-pel search with the 85-PU argmin (motion_estimation.c:98-425, 429-817).
// Lane b of a wavefront owns 8x8 block b in Z-order; one item = 4 consecutive
// x positions of one search row; 16x16 / 32x32 / 64x64 SADs are lane sums
// (xor 1,2 / 4,8 / 16,32). Per-PU best keys (sad << 32 | raster order) merge
// across waves with ds_min_u64.
// ----------------------------------------------------------------------------
__device__ __forceinline__ void flush_pu_keys(SbState &st, int slot, int lane, unsigned long long b8,
                                              unsigned long long b16, unsigned long long b32, unsigned long long b64) {
    unsigned long long *pk = st.pu_key[slot];
    atomicMin(&pk[21 + lane], b8);
    if ((lane & 3) == 0)
        atomicMin(&pk[5 + (lane >> 2)], b16);
    if ((lane & 15) == 0)
        atomicMin(&pk[1 + (lane >> 4)], b32);
    if (lane == 0)
        atomicMin(&pk[0], b64);
}

template <bool SUB>
__device__ void run_fullpel(SbState &st, const svtme_job &job, const DevJob &dj) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // Z-order lane -> raster 8x8 block
    const int z16 = lane >> 2, k4 = lane & 3;
    const int by = ((z16 >> 3) << 2) | (((z16 >> 1) & 1) << 1) | (k4 >> 1);
    const int bx = (((z16 >> 2) & 1) << 2) | ((z16 & 1) << 1) | (k4 & 1);
    constexpr int ROWS = SUB ? 4 : 8;
    constexpr int RSTEP = SUB ? 2 : 1;
    uint32_t src[ROWS][2];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const uint32_t *s = (const uint32_t *)(st.src + (by * 8 + r * RSTEP) * 64 + bx * 8);
        src[r][0]         = s[0];
        src[r][1]         = s[1];
    }
    const int nfp = st.nfp, nitems = st.fp_items;
    int cur_ref = -1;
    unsigned long long b8 = ~0ull, b16 = ~0ull, b32 = ~0ull, b64 = ~0ull;
    for (int i = wid; i < nitems; i += ME_THREADS / 64) {
        int f = 0;
        while (f + 1 < nfp && st.fp[f + 1].item_begin <= i) f++;
        if (f != cur_ref) { // flush running bests of the previous reference (wave-uniform)
            if (cur_ref >= 0)
                flush_pu_keys(st, st.fp[cur_ref].slot, lane, b8, b16, b32, b64);
            b8 = b16 = b32 = b64 = ~0ull;
            cur_ref = f;
        }
        const FpRef &F = st.fp[f];
        const int li = i - F.item_begin;
        const int y = li / F.nq, x0 = 4 * (li - (li / F.nq) * F.nq);
        const int l = F.slot >> 2, r = F.slot & 3;
        const DevPlane &P = dj.ref[l][r].lv[0];
        const uint8_t *rp = P.base + (ptrdiff_t)((int)st.oy_sb + F.yo + y + by * 8) * P.stride +
            ((int)st.ox_sb + F.xo + x0 + bx * 8);
        const int sh = (int)((uintptr_t)rp & 3);
        const uint32_t *ra = (const uint32_t *)(rp - sh);
        uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int rr = 0; rr < ROWS; rr++) {
            const uint32_t *rd = (const uint32_t *)((const uint8_t *)ra + (ptrdiff_t)(rr * RSTEP) * P.stride);
            const uint32_t d0 = rd[0], d1 = rd[1], d2 = rd[2], d3 = rd[3];
            // runs for the 4 shifts: shift k of position x0+k is byte offset sh+k
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int t = sh + k; // 0..6
                uint32_t a0, a1;
                if (t < 4) {
                    a0 = t ? __builtin_amdgcn_alignbyte(d1, d0, t) : d0;
                    a1 = t ? __builtin_amdgcn_alignbyte(d2, d1, t) : d1;
                } else {
                    a0 = (t - 4) ? __builtin_amdgcn_alignbyte(d2, d1, t - 4) : d1;
                    a1 = (t - 4) ? __builtin_amdgcn_alignbyte(d3, d2, t - 4) : d2;
                }
                acc[k] = __builtin_amdgcn_sad_u8(a0, src[rr][0], acc[k]);
                acc[k] = __builtin_amdgcn_sad_u8(a1, src[rr][1], acc[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (x0 + k >= F.w)
                break; // wave-uniform
            uint32_t s8 = SUB ? acc[k] << 1 : acc[k];
            uint32_t s16 = s8 + __shfl_xor(s8, 1, 64);
            s16 += __shfl_xor(s16, 2, 64);
            uint32_t s32 = s16 + __shfl_xor(s16, 4, 64);
            s32 += __shfl_xor(s32, 8, 64);
            uint32_t s64 = s32 + __shfl_xor(s32, 16, 64);
            s64 += __shfl_xor(s64, 32, 64);
            const uint32_t order = (uint32_t)(F.order_base + y * F.w + x0 + k);
            const unsigned long long o = order;
            unsigned long long k8 = ((unsigned long long)s8 << 32) | o, k16 = ((unsigned long long)s16 << 32) | o,
                               k32 = ((unsigned long long)s32 << 32) | o, k64 = ((unsigned long long)s64 << 32) | o;
            b8  = k8 < b8 ? k8 : b8;
            b16 = k16 < b16 ? k16 : b16;
            b32 = k32 < b32 ? k32 : b32;
            b64 = k64 < b64 ? k64 : b64;
        }
    }
    if (cur_ref >= 0)
        flush_pu_keys(st, st.fp[cur_ref].slot, lane, b8, b16, b32, b64);
    __syncthreads();
}

// decode per-PU keys of reference slot s into best_sad / best_mv (strict-<
// update from MAX_SAD_VALUE, motion_estimation.c:1366)
__device__ void decode_keys(SbState &st, int l, int r, int16_t cxo, int16_t cyo, int16_t xo, int16_t yo, int w) {
    const int tid = threadIdx.x;
    if (tid < SVTME_PU_COUNT) {
        const unsigned long long k = st.pu_key[l * 4 + r][tid];
        const uint32_t sad         = (uint32_t)(k >> 32);
        if (k != ~0ull && sad < st.best_sad[l][r][tid]) {
            const uint32_t order = (uint32_t)(k & 0xFFFFFFFFu);
            int16_t mx, my;
            if (order == 0) {
                mx = cxo;
                my = cyo;
            } else {
                const int p = (int)order - 1;
                my          = (int16_t)(yo + p / w);
                mx          = (int16_t)(xo + p % w);
            }
            st.best_sad[l][r][tid] = sad;
            st.best_mv[l][r][tid]  = ((uint32_t)(uint16_t)my << 16) | (uint16_t)mx;
        }
    }
}

// ----------------------------------------------------------------------------
// Scalar control (lane 0): restatements of the reference's per-SB logic
// ----------------------------------------------------------------------------
// prehme_core search-area derivation (motion_estimation.c:1568-1636)
__device__ void prehme_prepare(SbState &st, const DevPlane &p, int16_t org_x, int16_t org_y, PreHme &d, int16_t *oxo,
                               int16_t *oyo, int16_t *saw, int16_t *sah) {
    const int16_t pad_w = i16(p.pad - 1), pad_h = i16(p.pad - 1);
    const int16_t pw = i16(p.width), ph = i16(p.height);
    int16_t sa_w = (int16_t)d.sa_w, sa_h = (int16_t)d.sa_h;
    int16_t ox = -(int16_t)(sa_w >> 1);
    int16_t oy = -(int16_t)(sa_h >> 1);
    ox   = ((org_x + ox) < -pad_w) ? i16(-pad_w - org_x) : ox;
    sa_w = ((org_x + ox) < -pad_w) ? i16(sa_w - (-pad_w - (org_x + ox))) : sa_w;
    ox   = ((org_x + ox) > pw - 1) ? i16(ox - ((org_x + ox) - (pw - 1))) : ox;
    sa_w = ((org_x + ox + sa_w) > pw) ? i16(max(1, sa_w - ((org_x + ox + sa_w) - pw))) : sa_w;
    oy   = ((org_y + oy) < -pad_h) ? i16(-pad_h - org_y) : oy;
    sa_h = ((org_y + oy) < -pad_h) ? i16(sa_h - (-pad_h - (org_y + oy))) : sa_h;
    oy   = ((org_y + oy) > ph - 1) ? i16(oy - ((org_y + oy) - (ph - 1))) : oy;
    sa_h = (org_y + oy + sa_h > ph) ? i16(max(1, sa_h - ((org_y + oy + sa_h) - ph))) : sa_h;
    *oxo = ox;
    *oyo = oy;
    *saw = sa_w;
    *sah = sa_h;
}

// hme_level_0 search-area derivation (motion_estimation.c:835-889)
__device__ void hme_l0_prepare(const svtme_controls &c, const DevPlane &p, int16_t org_x, int16_t org_y, int16_t sa_w,
                               int16_t sa_h, int sr_w, int sr_h, int16_t *oxo, int16_t *oyo, int16_t *saw,
                               int16_t *sah) {
    sa_w = i16((sa_w + 7) & ~0x07);
    const int16_t pad_w = i16(p.pad - 1), pad_h = i16(p.pad - 1);
    const int16_t pw = i16(p.width), ph = i16(p.height);
    int16_t xd = i16(sa_w * sr_w);
    int16_t yd = i16(sa_h * sr_h);
    int16_t ox = i16(-(int16_t)((sa_w * c.num_hme_sa_w) >> 1) + xd);
    int16_t oy = i16(-(int16_t)((sa_h * c.num_hme_sa_h) >> 1) + yd);
    if ((org_x + ox) < -pad_w) {
        ox   = i16(-pad_w - org_x);
        sa_w = i16(sa_w - (-pad_w - (org_x + ox)));
    }
    if ((org_x + ox) > pw - 1)
        ox = i16(ox - ((org_x + ox) - (pw - 1)));
    if ((org_x + ox + sa_w) > pw)
        sa_w = i16(max(1, sa_w - ((org_x + ox + sa_w) - pw)));
    sa_w = (sa_w < 8) ? sa_w : i16(sa_w & ~0x07);
    if ((org_y + oy) < -pad_h) {
        oy   = i16(-pad_h - org_y);
        sa_h = i16(sa_h - (-pad_h - (org_y + oy)));
    }
    if ((org_y + oy) > ph - 1)
        oy = i16(oy - ((org_y + oy) - (ph - 1)));
    if ((org_y + oy + sa_h) > ph)
        sa_h = i16(max(1, sa_h - ((org_y + oy + sa_h) - ph)));
    *oxo = ox;
    *oyo = oy;
    *saw = sa_w;
    *sah = sa_h;
}

// hme_level_1 / hme_level_2 search-area derivation (motion_estimation.c:938-990, 1039-1084)
__device__ void hme_refine_prepare(int level, const DevPlane &p, int16_t org_x, int16_t org_y, int16_t sa_w,
                                   int16_t sa_h, int16_t scx, int16_t scy, int16_t *oxo, int16_t *oyo, int16_t *saw,
                                   int16_t *sah) {
    sa_w = i16((sa_w + 7) & ~0x07);
    const int16_t pad_w = level == 1 ? i16(p.pad - 1) : i16(64 - 1);
    const int16_t pad_h = pad_w;
    const int16_t pw = i16(p.width), ph = i16(p.height);
    int16_t ox = i16(-(sa_w >> 1) + scx);
    int16_t oy = i16(-(sa_h >> 1) + scy);
    if ((org_x + ox) < -pad_w) {
        ox   = i16(-pad_w - org_x);
        sa_w = i16(sa_w - (-pad_w - (org_x + ox)));
    }
    if ((org_x + ox) > pw - 1)
        ox = i16(ox - ((org_x + ox) - (pw - 1)));
    if ((org_x + ox + sa_w) > pw)
        sa_w = i16(max(1, sa_w - ((org_x + ox + sa_w) - pw)));
    sa_w = (sa_w < 8) ? sa_w : i16(sa_w & ~0x07);
    if ((org_y + oy) < -pad_h) {
        oy   = i16(-pad_h - org_y);
        sa_h = i16(sa_h - (-pad_h - (org_y + oy)));
    }
    if ((org_y + oy) > ph - 1)
        oy = i16(oy - ((org_y + oy) - (ph - 1)));
    if ((org_y + oy + sa_h) > ph)
        sa_h = i16(max(1, sa_h - ((org_y + oy + sa_h) - ph)));
    *oxo = ox;
    *oyo = oy;
    *saw = sa_w;
    *sah = sa_h;
}

// get_hme_l0_search_area (motion_estimation.c:1800-1867); the mutate/restore of
// hme_l0_sa per reference makes it a pure function of (list, ref, dist)
__device__ void hme_l0_area(const SbState &st, const svtme_controls &c, int l, int r, uint16_t dist, int16_t *sa_w,
                            int16_t *sa_h) {
    uint32_t mnw = c.hme_l0_sa.sa_min.width, mnh = c.hme_l0_sa.sa_min.height;
    uint32_t mxw = c.hme_l0_sa.sa_max.width, mxh = c.hme_l0_sa.sa_max.height;
    if (c.enable_me_sr_adjustment && c.distance_based_hme_resizing) {
        uint8_t is_hor = 1, is_ver = 1, is_still = 0;
        if (c.reduce_hme_l0_sr_th_min && c.reduce_hme_l0_sr_th_max) {
            if (l || r) {
                const int mvx = st.l0x[0][0][0][0], mvy = st.l0y[0][0][0][0];
                is_ver   = (absi(mvx) < c.reduce_hme_l0_sr_th_min) && (absi(mvy) > c.reduce_hme_l0_sr_th_max);
                is_hor   = (absi(mvx) > c.reduce_hme_l0_sr_th_max) && (absi(mvy) < c.reduce_hme_l0_sr_th_min);
                is_still = (absi(mvx) < (c.reduce_hme_l0_sr_th_min * 3)) && (absi(mvy) < (c.reduce_hme_l0_sr_th_min * 3));
            }
        }
        uint8_t xo = 1, yo = 1;
        if (!is_ver)
            yo = 2;
        if (!is_hor)
            xo = 2;
        if (c.enable_me_sr_adjustment == 2 && is_still)
            xo = yo = 4;
        mnw = (uint16_t)(mnw / (xo + r));
        mnh = (uint16_t)(mnh / (yo + r));
        mxw = (uint16_t)(mxw / (xo + r));
        mxh = (uint16_t)(mxh / (yo + r));
    }
    const int32_t f = scaled_dist(dist);
    int16_t w       = i16(mnw / c.num_hme_sa_w);
    w               = i16(min((((w * f) + 15) & ~0x0F), (int)(((mxw / c.num_hme_sa_w) + 15) & ~0x0F)));
    int16_t h       = i16(mnh / c.num_hme_sa_h);
    h               = i16(min((h * f), (int)(mxh / c.num_hme_sa_h)));
    *sa_w           = w;
    *sa_h           = h;
}

// ----------------------------------------------------------------------------
// Tables for the candidate arrays (motion_estimation.c:2520-2531, definitions.h:2613-2632)
// ----------------------------------------------------------------------------
__constant__ uint8_t c_z_to_raster[85] = {
    0,  1,  2,  3,  4,  5,  6,  9,  10, 7,  8,  11, 12, 13, 14, 17, 18, 15, 16, 19, 20, 21,
    22, 29, 30, 23, 24, 31, 32, 37, 38, 45, 46, 39, 40, 47, 48, 25, 26, 33, 34, 27, 28, 35,
    36, 41, 42, 49, 50, 43, 44, 51, 52, 53, 54, 61, 62, 55, 56, 63, 64, 69, 70, 77, 78, 71,
    72, 79, 80, 57, 58, 65, 66, 59, 60, 67, 68, 73, 74, 81, 82, 75, 76, 83, 84};
__constant__ uint8_t c_8x8_to_16x16[64] = {5,  5,  6,  6,  7,  7,  8,  8,  5,  5,  6,  6,  7,  7,  8,  8,
                                           9,  9,  10, 10, 11, 11, 12, 12, 9,  9,  10, 10, 11, 11, 12, 12,
                                           13, 13, 14, 14, 15, 15, 16, 16, 13, 13, 14, 14, 15, 15, 16, 16,
                                           17, 17, 18, 18, 19, 19, 20, 20, 17, 17, 18, 18, 19, 19, 20, 20};
__constant__ uint8_t c_16x16_to_32x32[16] = {1, 1, 2, 2, 1, 1, 2, 2, 3, 3, 4, 4, 3, 3, 4, 4};

__device__ __forceinline__ uint8_t mk_cand(int dir, int r0, int r1, int l0, int l1) {
    return (uint8_t)((dir & 3) | ((r0 & 3) << 2) | ((r1 & 3) << 4) | ((l0 & 1) << 6) | ((l1 & 1) << 7));
}

// Candidate arrays + distortions + GM detection for one SB, all threads
// (motion_estimation.c:2532-3007). Thread n builds Z-order PU n.
__device__ void finish_sb(SbState &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh) {
    const svtme_job &job = dj.job;
    const int tid = threadIdx.x;
    const int nl = job.num_lists, nr0 = job.num_refs[0], nr1 = nl == 2 ? job.num_refs[1] : 0;
    svtme_sb_result *o = dj.out_sb + sb_local;
    // zero the result (uint32 stores; sizeof is a multiple of 4)
    uint32_t *ow = (uint32_t *)o;
    for (int i = tid; i < (int)(sizeof(svtme_sb_result) / 4); i += ME_THREADS) ow[i] = 0;
    __syncthreads();
    const int npus = job.enable_me_16x16 ? (job.enable_me_8x8 ? 85 : 21) : 5;
    const int mode = (nr0 == 1 && nr1 == 0) ? 0 : (nr0 == 1 && nr1 == 1) ? 1 : 2;
    if (mode != 2 && tid < npus)
        o->total_me_candidate_index[tid] = 1; // memset(..., 1, number_of_pus)
    __syncthreads();
    if (tid < SVTME_PU_COUNT) {
        const int n = tid;
        const int use = job.enable_me_16x16 ? (job.enable_me_8x8 || n < 21) : n < 5;
        if (mode == 0) { // construct_me_candidate_array_single_ref
            const int pu            = c_z_to_raster[n];
            st.me_distortion[pu]    = st.best_sad[0][0][n];
            st.cand0[pu]            = 0;
            if (st.do_ref[0][0] && use) {
                o->me_candidate_array[pu][0] = mk_cand(0, 0, 0, 0, 0);
                o->me_mv_array[pu][0]        = st.best_mv[0][0][n];
            }
        } else if (mode == 1) { // construct_me_candidate_array_mrp_off
            const int pu = c_z_to_raster[n];
            uint32_t nlist = nl;
            const uint8_t org0 = st.do_ref[0][0], org1 = nl == 1 ? 0 : st.do_ref[1][0];
            if (nlist < 2 || !st.do_ref[1][0])
                nlist = 1;
            const uint32_t prune_th = (org0 && org1) ? (uint32_t)job.ctrl.prune_me_candidates_th : 0;
            uint8_t off = 0;
            uint8_t blk[2] = {org0, org1};
            const uint32_t s0 = st.best_sad[0][0][n], s1 = st.best_sad[1][0][n];
            const uint32_t best = (org0 && org1) ? min_u32(s0, s1) : org0 ? s0 : s1;
            st.me_distortion[pu] = best;
            int min_list = -1;
            if (job.ctrl.use_best_unipred_cand_only && blk[0] && blk[1])
                min_list = s0 < s1 ? 0 : 1;
            uint8_t c0 = 0;
            for (int li = 0; (uint32_t)li < nlist && (use || off == 0); ++li) {
                if (!blk[li])
                    continue;
                if (prune_th > 0) {
                    const uint32_t dd = (st.best_sad[li][0][n] - best) * 100;
                    if (dd > best * prune_th) {
                        blk[li] = 0;
                        continue;
                    }
                }
                if (min_list != -1 && min_list != li) {
                    if (use)
                        o->me_mv_array[pu][li ? job.max_l0 : 0] = st.best_mv[li][0][n];
                    continue;
                }
                if (use) {
                    const uint8_t cb = mk_cand(li, 0, 0, li == 0 ? li : 24, li == 1 ? li : 24);
                    o->me_candidate_array[pu][off] = cb;
                    if (off == 0)
                        c0 = cb;
                    o->me_mv_array[pu][li ? job.max_l0 : 0] = st.best_mv[li][0][n];
                }
                off++;
            }
            if (blk[0] && blk[1] && use) {
                const uint8_t cb = mk_cand(2, 0, 0, 0, 1);
                o->me_candidate_array[pu][off] = cb;
                if (off == 0)
                    c0 = cb;
                o->total_me_candidate_index[pu] = (uint8_t)(off + 1);
            }
            st.cand0[pu] = c0;
        } else { // construct_me_candidate_array
            const int pu = (n > 4) ? c_z_to_raster[n] : n;
            uint8_t off = 0;
            uint8_t blk[2][4] = {{0}};
            const uint32_t prune_th = (uint32_t)job.ctrl.prune_me_candidates_th;
            uint32_t best = U32MAX;
            for (int li = 0; li < nl; li++)
                for (int r = 0; r < (li ? nr1 : nr0); r++) {
                    blk[li][r] = st.do_ref[li][r];
                    if (!blk[li][r])
                        continue;
                    best = min_u32(best, st.best_sad[li][r][n]);
                }
            st.me_distortion[pu] = best;
            uint8_t c0 = 0;
            for (int li = 0; li < nl && (use || off == 0); ++li)
                for (int r = 0; r < (li ? nr1 : nr0) && (use || off == 0); ++r) {
                    if (!blk[li][r])
                        continue;
                    if (prune_th > 0) {
                        const uint32_t dd = (st.best_sad[li][r][n] - best) * 100;
                        if (dd > best * prune_th) {
                            blk[li][r] = 0;
                            continue;
                        }
                    }
                    if (use) {
                        const uint8_t cb = mk_cand(li, r, r, li == 0 ? li : 24, li == 1 ? li : 24);
                        o->me_candidate_array[pu][off] = cb;
                        if (off == 0)
                            c0 = cb;
                        o->me_mv_array[pu][(li ? job.max_l0 : 0) + r] = st.best_mv[li][r][n];
                    }
                    off++;
                }
            if (nl == 2 && use) {
                for (int a2 = 0; a2 < nr0; a2++)
                    for (int b2 = 0; b2 < nr1; b2++) {
                        if (job.only_l_bwd && (a2 > 0 || b2 > 0))
                            continue;
                        if (blk[0][a2] && blk[1][b2]) {
                            const uint8_t cb = mk_cand(2, a2, b2, 0, 1);
                            if (off == 0)
                                c0 = cb;
                            o->me_candidate_array[pu][off++] = cb;
                        }
                    }
                if (!job.only_l_bwd)
                    for (int a2 = 1; a2 < nr0; a2++)
                        if (blk[0][0] && blk[0][a2]) {
                            const uint8_t cb = mk_cand(2, 0, a2, 0, 0);
                            if (off == 0)
                                c0 = cb;
                            o->me_candidate_array[pu][off++] = cb;
                        }
                if (!job.only_l_bwd && nr1 == 3 && blk[1][0] && blk[1][2]) {
                    const uint8_t cb = mk_cand(2, 0, 2, 1, 1);
                    if (off == 0)
                        c0 = cb;
                    o->me_candidate_array[pu][off++] = cb;
                }
            }
            if (use)
                o->total_me_candidate_index[pu] = off;
            st.cand0[pu] = use ? c0 : 0;
        }
    }
    __syncthreads();
    if (tid < SVTME_PU_COUNT)
        o->me_distortion[tid] = st.me_distortion[tid];
    if (tid == 0) {
        // compute_distortion (motion_estimation.c:2964-3007)
        uint32_t d64 = st.me_distortion[0], d32 = 0, d16 = 0, d8 = 0;
        for (int i = 0; i < 4; i++) d32 += st.me_distortion[1 + i];
        for (int i = 0; i < 16; i++) d16 += st.me_distortion[5 + i];
        for (int i = 0; i < 64; i++) d8 += st.me_distortion[21 + i];
        const uint64_t mean = d8 / 64;
        uint64_t sum_sq = 0;
        for (int i = 0; i < 64; i++) {
            const int64_t diff = (int64_t)st.me_distortion[21 + i] - (int64_t)mean;
            sum_sq += (uint64_t)(diff * diff);
        }
        o->me_8x8_cost_variance = (uint32_t)(sum_sq / 64);
        o->rc_me_distortion     = (job.input_resolution <= 2) ? d8 : d16;
        const uint32_t pix      = bw * bh;
        o->me_64x64_distortion  = (d64 * 4096u) / pix;
        o->me_32x32_distortion  = (d32 * 4096u) / pix;
        o->me_16x16_distortion  = (d16 * 4096u) / pix;
        o->me_8x8_distortion    = (d8 * 4096u) / pix;
        // perform_gm_detection (motion_estimation.c:2838-2961)
        if (job.gm_enabled) {
            uint64_t stationary = 0, tot = 0;
            uint32_t cnt[2][4][2][2];
            for (int a2 = 0; a2 < 2; a2++)
                for (int b2 = 0; b2 < 4; b2++)
                    for (int cc = 0; cc < 2; cc++) cnt[a2][b2][cc][0] = cnt[a2][b2][cc][1] = 0;
            const bool low = job.input_resolution <= 2;
            const int n_blk = low ? 64 : 16;
            for (int i = 0; i < n_blk; i++) {
                uint8_t n = (uint8_t)(low ? 21 + i : 5 + i);
                if (low && !job.enable_me_8x8) {
                    if (n >= 21)
                        n = c_8x8_to_16x16[n - 21];
                    if (!job.enable_me_16x16 && n >= 5)
                        n = c_16x16_to_32x32[n - 5];
                }
                if (!low && !job.enable_me_16x16 && n >= 5)
                    n = c_16x16_to_32x32[n - 5];
                const uint8_t cb = st.cand0[n];
                const int dir = cb & 3, r0 = (cb >> 2) & 3, r1 = (cb >> 4) & 3, l0 = (cb >> 6) & 1, l1 = (cb >> 7) & 1;
                const int li = (dir == 0 || dir == 2) ? l0 : l1;
                const int ri = (dir == 0 || dir == 2) ? r0 : r1;
                int active_th;
                if (low) {
                    const uint64_t a2 = job.picture_number, b2 = job.ref_picture_number[li][ri];
                    const uint16_t dist = (uint16_t)absi((int16_t)((a2 > b2 ? a2 : b2) - (a2 < b2 ? a2 : b2)));
                    active_th = job.gm_use_distance_based_active_th ? max(dist >> 1, 4) : 4;
                } else {
                    const uint16_t dist = (uint16_t)absi((int16_t)(job.picture_number - job.ref_picture_number[li][ri]));
                    active_th = job.gm_use_distance_based_active_th ? max(dist * 16, 32) : 32;
                }
                const uint32_t mv = st.best_mv[li][ri][n];
                const int mx = (int)(int16_t)(mv & 0xFFFF) * 4, my = (int)(int16_t)(mv >> 16) * 4;
                if (mx < -active_th)
                    cnt[li][ri][0][0]++;
                else if (mx > active_th)
                    cnt[li][ri][0][1]++;
                if (my < -active_th)
                    cnt[li][ri][1][0]++;
                else if (my > active_th)
                    cnt[li][ri][1][1]++;
                const int stt = low ? 0 : 4;
                if (absi(mx) <= stt && absi(my) <= stt)
                    stationary++;
                tot++;
            }
            if (stationary > ((tot * 5) / 100))
                o->stationary_block_present = 1;
            for (int a2 = 0; a2 < 2; a2++)
                for (int b2 = 0; b2 < 4; b2++)
                    for (int cc = 0; cc < 2; cc++)
                        for (int s2 = 0; s2 < 2; s2++)
                            if (cnt[a2][b2][cc][s2] > (tot / 2))
                                o->rc_me_allow_gm = 1;
        }
    }
}

// ----------------------------------------------------------------------------
// The per-SB kernel
// ----------------------------------------------------------------------------
template <bool SUB_ME>
__global__ void __launch_bounds__(ME_THREADS) k_me_sb(const DevJob dj) {
    __shared__ SbState st;
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int tid = threadIdx.x, lane = tid & 63;
    // XCD-aware SB order: blocks b and b+8 share an XCD (round-robin dispatch), so give
    // each XCD one contiguous band of SBs; neighbouring SBs share reference windows in
    // that XCD's L2 (bijective for any grid size; placement only affects speed)
    const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const uint32_t sb_local = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t b64      = job.sb_begin + sb_local;
    const uint32_t ox = (b64 % dj.pic_w_b64) * 64, oy = (b64 / dj.pic_w_b64) * 64;
    const uint32_t bw = (job.width - ox) < 64 ? job.width - ox : 64;
    const uint32_t bh = (job.height - oy) < 64 ? job.height - oy : 64;
    const int nl = job.num_lists;
    const int nr0 = job.num_refs[0], nr1 = nl == 2 ? job.num_refs[1] : 0;
    const bool hsub = c.hme_search_method != SVTME_FULL_SAD_SEARCH;
    SVTME_STAMP(0);

    // ---- source blocks -> LDS (me_process.c:183-214)
    {
        const DevPlane &F = dj.cur.lv[0];
        const uint32_t *fp = (const uint32_t *)(F.base + (size_t)oy * F.stride + ox);
        for (int e = tid; e < 64 * 16; e += ME_THREADS) {
            const int r = e >> 4, j = e & 15;
            ((uint32_t *)st.src)[e] = fp[(size_t)r * (F.stride >> 2) + j];
        }
        const DevPlane &Q = dj.cur.lv[1];
        const uint32_t *qp = (const uint32_t *)(Q.base + (size_t)(oy >> 1) * Q.stride + (ox >> 1));
        for (int e = tid; e < 32 * 8; e += ME_THREADS) {
            const int r = e >> 3, j = e & 7;
            ((uint32_t *)(st.src + 4096))[e] = qp[(size_t)r * (Q.stride >> 2) + j];
        }
        const DevPlane &S = dj.cur.lv[2];
        const uint32_t *sp = (const uint32_t *)(S.base + (size_t)(oy >> 2) * S.stride + (ox >> 2));
        if (tid < 64) {
            const int r = tid >> 2, j = tid & 3;
            ((uint32_t *)(st.src + 5120))[tid] = sp[(size_t)r * (S.stride >> 2) + j];
        }
    }
    // ---- init_me_hme_data (motion_estimation.c:3010-3070)
    if (tid == 0) {
        st.b64_w = bw;
        st.b64_h = bh;
        st.ox_sb = ox;
        st.oy_sb = oy;
        for (int l = 0; l < 2; l++)
            for (int r = 0; r < 4; r++) {
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) {
                        st.l0x[l][r][a][b] = st.l0y[l][r][a][b] = 0;
                        st.l1x[l][r][a][b] = st.l1y[l][r][a][b] = 0;
                        st.l2x[l][r][a][b] = st.l2y[l][r][a][b] = 0;
                        st.l0sad[l][r][a][b] = st.l1sad[l][r][a][b] = st.l2sad[l][r][a][b] = 0;
                    }
                st.do_ref[l][r]     = 1;
                st.hme_sad[l][r]    = U32MAX;
                st.hme_sc_x[l][r]   = 0;
                st.hme_sc_y[l][r]   = 0;
                st.reduce_div[l][r] = 1;
                st.zz_sad[l][r]     = U32MAX;
                for (int s = 0; s < 2; s++) {
                    st.prehme[l][r][s].valid    = 0;
                    st.prehme[l][r][s].sad      = 0;
                    st.prehme[l][r][s].col      = 0;
                    st.prehme[l][r][s].row      = 0;
                    st.performed_phme[l][r][s]  = 0;
                }
            }
    }
    for (int e = tid; e < 2 * 4 * SVTME_PU_COUNT; e += ME_THREADS) (&st.best_mv[0][0][0])[e] = 0;
    __syncthreads();
    SVTME_STAMP(1);

    // ---- init_zz_sad (motion_estimation.c:2382-2437)
    if (c.me_early_exit_th || c.me_safe_limit_zz_th) {
        __shared__ NxmReq reqs[8];
        __shared__ int nreq;
        if (tid == 0) {
            nreq = 0;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++)
                    if (tl_or_l0(job, l)) {
                        const DevPlane &P = dj.ref[l][r].lv[0];
                        reqs[nreq++]      = NxmReq{P.base + (size_t)oy * P.stride + ox, P.stride * 2};
                    }
        }
        __syncthreads();
        run_nxm(st, reqs, nreq, (int)(bh >> 1), (int)bw, 128);
        if (tid == 0) {
            uint32_t best_zz = U32MAX;
            int q = 0;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++)
                    if (tl_or_l0(job, l)) {
                        uint32_t zz = st.nxm_sad[q++] << 1;
                        zz          = (zz * 64 * 64) / (bw * bh);
                        st.zz_sad[l][r] = zz;
                        best_zz         = min_u32(best_zz, zz);
                    }
            if (job.temporal_layer_index > 0 && best_zz < c.zz_sad_th) {
                for (int l = 0; l < nl; l++)
                    for (int r = 1; r < (l ? nr1 : nr0); r++)
                        if ((uint32_t)((st.zz_sad[l][r] - best_zz) * 100u) > (uint32_t)(c.zz_sad_pct * best_zz))
                            st.do_ref[l][r] = 0;
            }
            if (c.me_safe_limit_zz_th) {
                const bool safe = job.hierarchical_levels > 0 && nl == 2 &&
                    job.temporal_layer_index >= job.hierarchical_levels && job.similar_brightness_refs &&
                    st.zz_sad[0][0] < c.me_safe_limit_zz_th && st.zz_sad[1][0] < c.me_safe_limit_zz_th;
                if (safe)
                    for (int l = 0; l < nl; l++)
                        for (int r = 1; r < (l ? nr1 : nr0); r++) st.do_ref[l][r] = 0;
            }
        }
        __syncthreads();
    SVTME_STAMP(2);
    }

    // ---- pre-HME (motion_estimation.c:1693-1796); list 1 runs after list 0
    // because its early exit reads list 0's results
    if (c.prehme_enable) {
        const int16_t sox = i16(((int16_t)ox) >> 2), soy = i16(((int16_t)oy) >> 2);
        for (int pass = 0; pass < nl; pass++) {
            if (tid == 0) {
                st.ntasks = st.nitems = 0;
                const int l = pass;
                for (int r = 0; r < (l ? nr1 : nr0); r++) {
                    if (!tl_or_l0(job, l))
                        continue;
                    const uint32_t f = scaled_dist(ref_dist(job, l, r));
                    for (int s = 0; s < 2; s++) {
                        PreHme &d = st.prehme[l][r][s];
                        // check_prehme_early_exit (motion_estimation.c:1693-1719)
                        if (c.me_early_exit_th && st.zz_sad[l][r] < c.me_early_exit_th) {
                            d.col = d.row = 0;
                            d.sad         = 0;
                            d.valid       = 1;
                            continue;
                        }
                        if (c.prehme_l1_early_exit) {
                            const PreHme &z = st.prehme[0][r][s];
                            if (l == 1 && z.valid &&
                                ((z.sad < (32 * 32)) || ((absi(z.col) < 16) && (absi(z.row) < 16)))) {
                                d.col   = (int16_t)-z.col;
                                d.row   = (int16_t)-z.row;
                                d.sad   = z.sad;
                                d.valid = 1;
                                continue;
                            }
                        }
                        if (!st.do_ref[l][r]) {
                            d.col = d.row = 0;
                            d.sad         = U32MAX;
                            continue;
                        }
                        d.sa_w = (uint16_t)min((uint32_t)c.prehme_sa_cfg[s].sa_min.width * f,
                                               (uint32_t)c.prehme_sa_cfg[s].sa_max.width);
                        d.sa_h = (uint16_t)min((uint32_t)c.prehme_sa_cfg[s].sa_min.height * f,
                                               (uint32_t)c.prehme_sa_cfg[s].sa_max.height);
                        const DevPlane &P = dj.ref[l][r].lv[2];
                        int16_t xo, yo, sw, sh2;
                        prehme_prepare(st, P, sox, soy, d, &xo, &yo, &sw, &sh2);
                        st.ox[l][r][s][0] = xo;
                        st.oy[l][r][s][0] = yo;
                        const uint8_t *win = P.base + (ptrdiff_t)(soy + yo) * P.stride + (sox + xo);
                        add_task(st, win, hsub ? P.stride * 2 : P.stride, P.stride, 5120, hsub ? 32 : 16, (int)(bw >> 2),
                                 hsub ? (int)(bh >> 2) >> 1 : (int)(bh >> 2), sw, sh2, c.prehme_skip_search_line);
                        st.tasks[st.ntasks - 1].pad[0] = (uint8_t)(l * 8 + r * 2 + s); // owner
                        st.performed_phme[l][r][s] = 1;
                    }
                }
            }
            __syncthreads();
            run_sad_tasks(st);
            if (tid == 0) {
                for (int t = 0; t < st.ntasks; t++) {
                    const int own = st.tasks[t].pad[0];
                    const int l = own >> 3, r = (own >> 1) & 3, s = own & 1;
                    PreHme &d = st.prehme[l][r][s];
                    uint64_t best;
                    task_result(st, t, &best, &d.col, &d.row);
                    d.sad   = hsub ? best * 2 : best;
                    d.col   = i16(d.col + st.ox[l][r][s][0]);
                    d.col   = i16(d.col * 4);
                    d.row   = i16(d.row + st.oy[l][r][s][0]);
                    d.row   = i16(d.row * 4);
                    d.valid = 1;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            uint32_t best_sad = U32MAX;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++) {
                    if (tl_or_l0(job, l)) {
                        const uint32_t m = (uint32_t)min_u64(st.prehme[l][r][0].sad, st.prehme[l][r][1].sad);
                        best_sad         = min_u32(best_sad, m);
                    } else {
                        for (int s = 0; s < 2; s++) {
                            st.prehme[1][r][s].col = (int16_t)-st.prehme[0][r][s].col;
                            st.prehme[1][r][s].row = (int16_t)-st.prehme[0][r][s].row;
                            st.prehme[1][r][s].sad = st.prehme[0][r][s].sad;
                        }
                    }
                }
            if (job.temporal_layer_index > 0 && best_sad < c.phme_sad_th) {
                for (int l = 0; l < nl; l++)
                    for (int r = 1; r < (l ? nr1 : nr0); r++) {
                        if (!st.do_ref[l][r])
                            continue;
                        const uint32_t psad = (uint32_t)min_u64(st.prehme[l][r][0].sad, st.prehme[l][r][1].sad);
                        if ((uint32_t)((psad - best_sad) * 100u) > (uint32_t)(c.phme_sad_pct * best_sad))
                            st.do_ref[l][r] = 0;
                    }
            }
        }
        __syncthreads();
    SVTME_STAMP(3);
    }

    if (c.enable_hme_flag) {
        // ---- HME level 0 (motion_estimation.c:1906-2036)
        if (c.enable_hme_level0_flag) {
            const int16_t sox = i16(((int16_t)ox) >> 2), soy = i16(((int16_t)oy) >> 2);
            if (tid == 0) {
                st.ntasks = st.nitems = 0;
                for (int l = 0; l < nl; l++)
                    for (int r = 0; r < (l ? nr1 : nr0); r++) {
                        if (c.me_early_exit_th && st.zz_sad[l][r] < (c.me_early_exit_th >> 2)) {
                            for (int a = 0; a < 2; a++)
                                for (int b = 0; b < 2; b++) {
                                    st.l0x[l][r][a][b] = st.l0y[l][r][a][b] = 0;
                                    st.l0sad[l][r][a][b]                    = 0;
                                }
                            continue;
                        }
                        if (c.prev_me_stage_based_exit_th) {
                            const int s = st.prehme[l][r][0].sad <= st.prehme[l][r][1].sad ? 0 : 1;
                            if (st.performed_phme[l][r][s] &&
                                st.prehme[l][r][s].sad < (c.prev_me_stage_based_exit_th >> 4)) {
                                for (int a = 0; a < 2; a++)
                                    for (int b = 0; b < 2; b++) {
                                        st.l0x[l][r][a][b]   = st.prehme[l][r][s].col;
                                        st.l0y[l][r][a][b]   = st.prehme[l][r][s].row;
                                        st.l0sad[l][r][a][b] = st.prehme[l][r][s].sad;
                                    }
                                continue;
                            }
                        }
                        if (!st.do_ref[l][r]) {
                            for (int a = 0; a < 2; a++)
                                for (int b = 0; b < 2; b++) {
                                    st.l0x[l][r][a][b] = st.l0y[l][r][a][b] = 0;
                                    st.l0sad[l][r][a][b]                    = U32MAX;
                                }
                            continue;
                        }
                        if (!tl_or_l0(job, l))
                            continue;
                        int16_t sa_w, sa_h;
                        hme_l0_area(st, c, l, r, ref_dist(job, l, r), &sa_w, &sa_h);
                        const DevPlane &P = dj.ref[l][r].lv[2];
                        for (int sy = 0; sy < 2; sy++)
                            for (int sx = 0; sx < 2; sx++) {
                                int16_t xo, yo, sw, sh2;
                                hme_l0_prepare(c, P, sox, soy, sa_w, sa_h, sx, sy, &xo, &yo, &sw, &sh2);
                                st.ox[l][r][sx][sy] = xo;
                                st.oy[l][r][sx][sy] = yo;
                                const uint8_t *win  = P.base + (ptrdiff_t)(soy + yo) * P.stride + (sox + xo);
                                add_task(st, win, hsub ? P.stride * 2 : P.stride, P.stride, 5120, hsub ? 32 : 16,
                                         (int)(bw >> 2), hsub ? (int)(bh >> 2) >> 1 : (int)(bh >> 2), sw, sh2, 0);
                                st.tasks[st.ntasks - 1].pad[0] = (uint8_t)(l * 16 + r * 4 + sx * 2 + sy);
                            }
                    }
            }
            __syncthreads();
            run_sad_tasks(st);
            if (tid == 0) {
                for (int t = 0; t < st.ntasks; t++) {
                    const int own = st.tasks[t].pad[0];
                    const int l = own >> 4, r = (own >> 2) & 3, sx = (own >> 1) & 1, sy = own & 1;
                    uint64_t best;
                    task_result(st, t, &best, &st.l0x[l][r][sx][sy], &st.l0y[l][r][sx][sy]);
                    st.l0sad[l][r][sx][sy] = hsub ? best * 2 : best;
                    st.l0x[l][r][sx][sy]   = i16(st.l0x[l][r][sx][sy] + st.ox[l][r][sx][sy]);
                    st.l0x[l][r][sx][sy]   = i16(st.l0x[l][r][sx][sy] * 4);
                    st.l0y[l][r][sx][sy]   = i16(st.l0y[l][r][sx][sy] + st.oy[l][r][sx][sy]);
                    st.l0y[l][r][sx][sy]   = i16(st.l0y[l][r][sx][sy] * 4);
                }
                // pre-HME replaces the worst quadrant (motion_estimation.c:2005-2032)
                if (c.prehme_enable) {
                    for (int l = 0; l < nl; l++)
                        for (int r = 0; r < (l ? nr1 : nr0); r++) {
                            if (c.me_early_exit_th && st.zz_sad[l][r] < (c.me_early_exit_th >> 2))
                                continue;
                            if (c.prev_me_stage_based_exit_th) {
                                const int s = st.prehme[l][r][0].sad <= st.prehme[l][r][1].sad ? 0 : 1;
                                if (st.performed_phme[l][r][s] &&
                                    st.prehme[l][r][s].sad < (c.prev_me_stage_based_exit_th >> 4))
                                    continue;
                            }
                            if (!st.do_ref[l][r] || !tl_or_l0(job, l))
                                continue;
                            uint8_t wx = 0, wy = 0;
                            uint64_t mx = 0;
                            if (st.l0sad[l][r][0][0] > mx) { mx = st.l0sad[l][r][0][0]; wx = 0; wy = 0; }
                            if (st.l0sad[l][r][1][0] > mx) { mx = st.l0sad[l][r][1][0]; wx = 1; wy = 0; }
                            if (st.l0sad[l][r][0][1] > mx) { mx = st.l0sad[l][r][0][1]; wx = 0; wy = 1; }
                            if (st.l0sad[l][r][1][1] > mx) { wx = 1; wy = 1; }
                            const int s = st.prehme[l][r][0].sad <= st.prehme[l][r][1].sad ? 0 : 1;
                            if (st.prehme[l][r][s].sad < st.l0sad[l][r][wx][wy]) {
                                st.l0sad[l][r][wx][wy] = st.prehme[l][r][s].sad;
                                st.l0x[l][r][wx][wy]   = st.prehme[l][r][s].col;
                                st.l0y[l][r][wx][wy]   = st.prehme[l][r][s].row;
                            }
                        }
                }
            }
            __syncthreads();
    SVTME_STAMP(4);
        }
        // ---- HME level 1 (motion_estimation.c:2041-2122)
        if (c.enable_hme_level1_flag) {
            const int16_t qox = i16(((int16_t)ox) >> 1), qoy = i16(((int16_t)oy) >> 1);
            if (tid == 0) {
                st.ntasks = st.nitems = 0;
                for (int l = 0; l < nl; l++)
                    for (int r = 0; r < (l ? nr1 : nr0); r++) {
                        if (!tl_or_l0(job, l))
                            continue;
                        if (c.me_early_exit_th && st.zz_sad[l][r] < (c.me_early_exit_th >> 2)) {
                            for (int a = 0; a < 2; a++)
                                for (int b = 0; b < 2; b++) {
                                    st.l1x[l][r][a][b] = st.l1y[l][r][a][b] = 0;
                                    st.l1sad[l][r][a][b]                    = 0;
                                }
                            continue;
                        }
                        if (!st.do_ref[l][r]) {
                            for (int a = 0; a < 2; a++)
                                for (int b = 0; b < 2; b++) {
                                    st.l1x[l][r][a][b] = st.l1y[l][r][a][b] = 0;
                                    st.l1sad[l][r][a][b]                    = U32MAX;
                                }
                            continue;
                        }
                        const DevPlane &P = dj.ref[l][r].lv[1];
                        for (int sy = 0; sy < 2; sy++)
                            for (int sx = 0; sx < 2; sx++) {
                                if (c.prev_me_stage_based_exit_th &&
                                    st.l0sad[l][r][sx][sy] < (c.prev_me_stage_based_exit_th >> 5)) {
                                    st.l1x[l][r][sx][sy]   = st.l0x[l][r][sx][sy];
                                    st.l1y[l][r][sx][sy]   = st.l0y[l][r][sx][sy];
                                    st.l1sad[l][r][sx][sy] = st.l0sad[l][r][sx][sy];
                                    continue;
                                }
                                int16_t xo, yo, sw, sh2;
                                hme_refine_prepare(1, P, qox, qoy, (int16_t)c.hme_l1_sa.width,
                                                   (int16_t)c.hme_l1_sa.height, i16(st.l0x[l][r][sx][sy] >> 1),
                                                   i16(st.l0y[l][r][sx][sy] >> 1), &xo, &yo, &sw, &sh2);
                                st.ox[l][r][sx][sy] = xo;
                                st.oy[l][r][sx][sy] = yo;
                                const uint8_t *win  = P.base + (ptrdiff_t)(qoy + yo) * P.stride + (qox + xo);
                                add_task(st, win, hsub ? P.stride * 2 : P.stride, P.stride, 4096, hsub ? 64 : 32,
                                         (int)(bw >> 1), hsub ? (int)(bh >> 1) >> 1 : (int)(bh >> 1), sw, sh2, 0);
                                st.tasks[st.ntasks - 1].pad[0] = (uint8_t)(l * 16 + r * 4 + sx * 2 + sy);
                            }
                    }
            }
            __syncthreads();
            run_sad_tasks(st);
            if (tid == 0) {
                for (int t = 0; t < st.ntasks; t++) {
                    const int own = st.tasks[t].pad[0];
                    const int l = own >> 4, r = (own >> 2) & 3, sx = (own >> 1) & 1, sy = own & 1;
                    uint64_t best;
                    task_result(st, t, &best, &st.l1x[l][r][sx][sy], &st.l1y[l][r][sx][sy]);
                    st.l1sad[l][r][sx][sy] = hsub ? best * 2 : best;
                    st.l1x[l][r][sx][sy]   = i16(st.l1x[l][r][sx][sy] + st.ox[l][r][sx][sy]);
                    st.l1x[l][r][sx][sy]   = i16(st.l1x[l][r][sx][sy] * 2);
                    st.l1y[l][r][sx][sy]   = i16(st.l1y[l][r][sx][sy] + st.oy[l][r][sx][sy]);
                    st.l1y[l][r][sx][sy]   = i16(st.l1y[l][r][sx][sy] * 2);
                }
            }
            __syncthreads();
    SVTME_STAMP(5);
        }
        // ---- HME level 2 (motion_estimation.c:2127-2177)
        if (c.enable_hme_level2_flag) {
            if (tid == 0) {
                st.ntasks = st.nitems = 0;
                for (int l = 0; l < nl; l++)
                    for (int r = 0; r < (l ? nr1 : nr0); r++) {
                        if (!tl_or_l0(job, l))
                            continue;
                        const DevPlane &P = dj.ref[l][r].lv[0];
                        for (int sy = 0; sy < 2; sy++)
                            for (int sx = 0; sx < 2; sx++) {
                                if (c.prev_me_stage_based_exit_th &&
                                    st.l1sad[l][r][sx][sy] < (c.prev_me_stage_based_exit_th >> 2)) {
                                    st.l2x[l][r][sx][sy]   = st.l1x[l][r][sx][sy];
                                    st.l2y[l][r][sx][sy]   = st.l1y[l][r][sx][sy];
                                    st.l2sad[l][r][sx][sy] = st.l1sad[l][r][sx][sy];
                                    continue;
                                }
                                int16_t xo, yo, sw, sh2;
                                hme_refine_prepare(2, P, (int16_t)ox, (int16_t)oy, (int16_t)c.hme_l2_sa.width,
                                                   (int16_t)c.hme_l2_sa.height, st.l1x[l][r][sx][sy],
                                                   st.l1y[l][r][sx][sy], &xo, &yo, &sw, &sh2);
                                st.ox[l][r][sx][sy] = xo;
                                st.oy[l][r][sx][sy] = yo;
                                const uint8_t *win =
                                    P.base + (ptrdiff_t)((int16_t)oy + yo) * P.stride + ((int16_t)ox + xo);
                                add_task(st, win, hsub ? P.stride * 2 : P.stride, P.stride, 0, hsub ? 128 : 64,
                                         (int)bw, hsub ? (int)bh >> 1 : (int)bh, sw, sh2, 0);
                                st.tasks[st.ntasks - 1].pad[0] = (uint8_t)(l * 16 + r * 4 + sx * 2 + sy);
                            }
                    }
            }
            __syncthreads();
            run_sad_tasks(st);
            if (tid == 0) {
                for (int t = 0; t < st.ntasks; t++) {
                    const int own = st.tasks[t].pad[0];
                    const int l = own >> 4, r = (own >> 2) & 3, sx = (own >> 1) & 1, sy = own & 1;
                    uint64_t best;
                    task_result(st, t, &best, &st.l2x[l][r][sx][sy], &st.l2y[l][r][sx][sy]);
                    st.l2sad[l][r][sx][sy] = hsub ? best * 2 : best;
                    st.l2x[l][r][sx][sy]   = i16(st.l2x[l][r][sx][sy] + st.ox[l][r][sx][sy]);
                    st.l2y[l][r][sx][sy]   = i16(st.l2y[l][r][sx][sy] + st.oy[l][r][sx][sy]);
                }
            }
            __syncthreads();
    SVTME_STAMP(6);
        }
    }

    // ---- set_final_seach_centre_sb (motion_estimation.c:2182-2380) and
    //      hme_prune_ref_and_adjust_sr (motion_estimation.c:2477-2518)
    if (tid == 0) {
        int16_t hx = 0, hy = 0, scx = 0, scy = 0;
        uint64_t hs = 0;
        for (int l = 0; l < nl; l++)
            for (int r = 0; r < (l ? nr1 : nr0); r++) {
                if (tl_or_l0(job, l)) {
                    if (c.enable_hme_flag) {
                        int16_t(*X)[2] = nullptr;
                        int16_t(*Y)[2] = nullptr;
                        uint64_t(*S)[2] = nullptr;
                        if (c.enable_hme_level0_flag && !c.enable_hme_level1_flag && !c.enable_hme_level2_flag) {
                            X = st.l0x[l][r]; Y = st.l0y[l][r]; S = st.l0sad[l][r];
                        }
                        if (c.enable_hme_level1_flag && !c.enable_hme_level2_flag) {
                            X = st.l1x[l][r]; Y = st.l1y[l][r]; S = st.l1sad[l][r];
                        }
                        if (c.enable_hme_level2_flag) {
                            X = st.l2x[l][r]; Y = st.l2y[l][r]; S = st.l2sad[l][r];
                        }
                        if (X) {
                            hx = X[0][0];
                            hy = Y[0][0];
                            hs = S[0][0];
                            uint32_t w = 1, h = 0;
                            while (h < c.num_hme_sa_h) {
                                while (w < c.num_hme_sa_w) {
                                    if (S[w][h] < hs) {
                                        hx = X[w][h];
                                        hy = Y[w][h];
                                        hs = S[w][h];
                                    }
                                    w++;
                                }
                                w = 0;
                                h++;
                            }
                        }
                        scx = hx;
                        scy = hy;
                    }
                } else {
                    scx = 0;
                    scy = 0;
                }
                st.hme_sc_x[l][r] = scx;
                st.hme_sc_y[l][r] = scy;
                st.hme_sad[l][r]  = hs;
            }
        if (c.enable_hme_flag) { /* prune_ref: enable_hme_flag && me_type != ME_MCTF */
            const uint16_t th = c.prune_ref_if_hme_sad_dev_bigger_than_th;
            if (c.enable_me_hme_ref_pruning && th != (uint16_t)~0) {
                uint64_t best = ~0ull;
                for (int i = 0; i < 2; i++)
                    for (int j = 0; j < 4; j++) best = min_u64(best, st.hme_sad[i][j]);
                for (int li = 0; li < 2; li++)
                    for (int ri = 1; ri < 4; ri++)
                        if ((st.hme_sad[li][ri] - best) * 100 > (th * best))
                            st.do_ref[li][ri] = 0;
            }
            if (c.enable_me_sr_adjustment) {
                for (int li = 0; li < 2; li++)
                    for (int ri = 0; ri < 4; ri++) {
                        if (absi(st.hme_sc_x[li][ri]) <= c.reduce_me_sr_based_on_mv_length_th &&
                            absi(st.hme_sc_y[li][ri]) <= c.reduce_me_sr_based_on_mv_length_th &&
                            st.hme_sad[li][ri] < c.stationary_hme_sad_abs_th)
                            st.reduce_div[li][ri] = c.stationary_me_sr_divisor;
                        else if (st.hme_sad[li][ri] < c.reduce_me_sr_based_on_hme_sad_abs_th)
                            st.reduce_div[li][ri] = c.me_sr_divisor_for_low_hme_sad;
                    }
            }
        }
        for (int l = 0; l < 2; l++)
            for (int r = 0; r < 4; r++) st.searched[l][r] = st.do_ref[l][r];
    }
    __syncthreads();
    SVTME_STAMP(7);

    // ---- integer_search_b64 (motion_estimation.c:1249-1516)
    // two rounds when enable_me_sr_adjustment == 2 (other refs read ref (0,0)'s result)
    const int rounds = c.enable_me_sr_adjustment == 2 ? 2 : 1;
    for (int round = 0; round < rounds; round++) {
        // step 1: search-area derivation up to the 8x8-variance decision
        if (tid == 0) {
            st.flag = 0;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++) {
                    if (rounds == 2 && ((l == 0 && r == 0) != (round == 0)))
                        continue;
                    if (!st.do_ref[l][r])
                        continue;
                    int16_t xc = st.hme_sc_x[l][r], yc = st.hme_sc_y[l][r];
                    int16_t w = (int16_t)c.me_sa.sa_min.width, h = (int16_t)c.me_sa.sa_min.height;
                    const uint16_t dist = scaled_dist(ref_dist(job, l, r));
                    w = i16(min((int)(w * dist), (int)c.me_sa.sa_max.width));
                    h = i16(min((int)(h * dist), (int)c.me_sa.sa_max.height));
                    if (c.mv_sa_adj_enabled && (!c.mv_sa_adj_nearest_ref_only || r == 0)) {
                        if (absi(xc) > c.mv_sa_adj_mv_size_th)
                            w = i16(w * c.mv_sa_adj_sa_multiplier);
                        if (absi(yc) > c.mv_sa_adj_mv_size_th)
                            h = i16(h * c.mv_sa_adj_sa_multiplier);
                    }
                    w = i16((max(1u, ((uint32_t)(int32_t)w / st.reduce_div[l][r])) + 7) & ~0x07u);
                    h = i16(max(3u, ((uint32_t)(int32_t)h / st.reduce_div[l][r])));
                    st.is_wb[l][r] = w;
                    st.is_hb[l][r] = h;
                    st.is_best_hme[l][r] = ~0ull;
                    if (c.me_early_exit_th) {
                        if (st.zz_sad[l][r] < (c.me_early_exit_th / 6)) {
                            w = 1;
                            h = 1;
                        }
                    } else if ((xc != 0 || yc != 0) && job.is_ref) {
                        st.flag = 1; // check_00_center needed
                    }
                    st.is_w[l][r]  = w;
                    st.is_h[l][r]  = h;
                    st.is_xc[l][r] = xc;
                    st.is_yc[l][r] = yc;
                }
        }
        __syncthreads();
        // check_00_center (motion_estimation.c:1139-1206), me_early_exit_th == 0 only
        if (st.flag) {
            __shared__ NxmReq reqs[8];
            __shared__ int nreq, owner[8];
            if (tid == 0) {
                nreq = 0;
                const int16_t pad = 63;
                for (int l = 0; l < nl; l++)
                    for (int r = 0; r < (l ? nr1 : nr0); r++) {
                        if (rounds == 2 && ((l == 0 && r == 0) != (round == 0)))
                            continue;
                        if (!st.do_ref[l][r] || c.me_early_exit_th)
                            continue;
                        int16_t xc = st.is_xc[l][r], yc = st.is_yc[l][r];
                        if (!((xc != 0 || yc != 0) && job.is_ref))
                            continue;
                        const DevPlane &P = dj.ref[l][r].lv[0];
                        const int16_t org_x = (int16_t)ox, org_y = (int16_t)oy;
                        const int16_t pw = i16(P.width), ph = i16(P.height);
                        xc = ((org_x + xc) < -pad) ? i16(-pad - org_x) : xc;
                        xc = ((org_x + xc) > pw - 1) ? i16(xc - ((org_x + xc) - (pw - 1))) : xc;
                        yc = ((org_y + yc) < -pad) ? i16(-pad - org_y) : yc;
                        yc = ((org_y + yc) > ph - 1) ? i16(yc - ((org_y + yc) - (ph - 1))) : yc;
                        st.is_xc[l][r] = xc;
                        st.is_yc[l][r] = yc;
                        owner[nreq]    = l * 4 + r;
                        reqs[nreq++]   = NxmReq{P.base + (ptrdiff_t)oy * P.stride + ox, P.stride * 2};
                        owner[nreq]    = l * 4 + r;
                        reqs[nreq++]   = NxmReq{P.base + (ptrdiff_t)((int)oy + yc) * P.stride + ((int)ox + xc),
                                              P.stride * 2};
                    }
            }
            __syncthreads();
            run_nxm(st, reqs, nreq, (int)(bh >> 1), (int)bw, 128);
            if (tid == 0) {
                for (int q = 0; q < nreq; q += 2) {
                    const int l = owner[q] >> 2, r = owner[q] & 3;
                    const uint32_t zero_sad = st.nxm_sad[q] << 1, hme_mv_sad = st.nxm_sad[q + 1] << 1;
                    const uint64_t zc = (uint64_t)zero_sad << 8, hc = (uint64_t)hme_mv_sad << 8;
                    const uint64_t cc = min_u64(zc, hc);
                    if (cc == zc) {
                        st.is_xc[l][r] = 0;
                        st.is_yc[l][r] = 0;
                    }
                    st.is_best_hme[l][r] = hme_mv_sad;
                }
            }
            __syncthreads();
        }
        // sr adjustment level 2 + 8x8-variance centre search setup
        if (tid == 0) {
            st.nfp = st.fp_items = 0;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++) {
                    if (rounds == 2 && ((l == 0 && r == 0) != (round == 0)))
                        continue;
                    if (!st.do_ref[l][r])
                        continue;
                    int16_t w = st.is_w[l][r], h = st.is_h[l][r];
                    if (!c.me_early_exit_th) {
                        const int16_t xc0 = st.hme_sc_x[l][r], yc0 = st.hme_sc_y[l][r];
                        uint8_t accurate  = 1;
                        if ((xc0 != 0 || yc0 != 0) && job.is_ref && st.is_xc[l][r] == 0 && st.is_yc[l][r] == 0)
                            accurate = 0;
                        if (c.enable_me_sr_adjustment == 2) {
                            if ((accurate && (st.is_best_hme[l][r] < (24 * 24))) ||
                                (job.is_ref && st.hme_sad[l][r] < (24 * 24)))
                                h = i16(h / 2);
                        }
                        if (c.enable_me_sr_adjustment == 2) {
                            if (l || r) {
                                if (st.best_sad[0][0][0] < 5000)
                                    if (h == st.is_hb[l][r] && w == st.is_wb[l][r]) {
                                        h = i16(h >> 1);
                                        w = i16(w >> 1);
                                    }
                            }
                        }
                    }
                    st.is_w[l][r] = w;
                    st.is_h[l][r] = h;
                    for (int i = 0; i < SVTME_PU_COUNT; i++) {
                        st.best_sad[l][r][i] = SVTME_MAX_SAD_VALUE;
                        st.pu_key[l * 4 + r][i] = ~0ull;
                    }
                    if (c.me_8x8_var_enabled && (w * h > 24)) {
                        FpRef &F     = st.fp[st.nfp++];
                        F.xo         = st.is_xc[l][r];
                        F.yo         = st.is_yc[l][r];
                        F.w          = 1;
                        F.h          = 1;
                        F.order_base = 0;
                        F.slot       = (uint8_t)(l * 4 + r);
                        F.nq         = 1;
                        F.item_begin = st.fp_items;
                        st.fp_items += 1;
                    }
                }
        }
        __syncthreads();
    SVTME_STAMP(8);
        if (st.nfp) {
            run_fullpel<SUB_ME>(st, job, dj);
            // decode the centre results, then the 8x8-variance resize (motion_estimation.c:1414-1438)
            for (int f = 0; f < st.nfp; f++) {
                const int l = st.fp[f].slot >> 2, r = st.fp[f].slot & 3;
                decode_keys(st, l, r, st.fp[f].xo, st.fp[f].yo, st.fp[f].xo, st.fp[f].yo, 1);
            }
            __syncthreads();
            if (tid == 0) {
                for (int f = 0; f < st.nfp; f++) {
                    const int l = st.fp[f].slot >> 2, r = st.fp[f].slot & 3;
                    int16_t w = st.is_w[l][r], h = st.is_h[l][r];
                    const uint32_t mean = st.best_sad[l][r][0] / 64;
                    uint32_t sum_sq     = 0;
                    for (int i = 0; i < 64; i++) {
                        const int32_t diff = (int32_t)st.best_sad[l][r][21 + i] - (int32_t)mean;
                        sum_sq += (uint32_t)(diff * diff);
                    }
                    const uint32_t var = sum_sq / 64;
                    if (var > c.me_sr_mult2_th) {
                        w = i16((max(1, w * 3 / 2) + 7) & ~0x7);
                        h = i16(max(1, h * 3 / 2));
                    }
                    if (var < c.me_sr_div4_th) {
                        w = i16((max(1, w >> 2) + 7) & ~0x7);
                        h = i16(max(1, h >> 2));
                        h = i16(max(3, (int)h));
                    } else if (var < c.me_sr_div2_th) {
                        w = i16((min((int)w, w >> 1) + 7) & ~0x7);
                        h = i16(min((int)h, h >> 1));
                        h = i16(max(3, (int)h));
                    }
                    st.is_w[l][r] = w;
                    st.is_h[l][r] = h;
                }
            }
            __syncthreads();
    SVTME_STAMP(9);
        }
        // final area clamp + main full-pel search of every searched reference
        if (tid == 0) {
            st.nfp = st.fp_items = 0;
            const int16_t pad = 63, org_x = (int16_t)ox, org_y = (int16_t)oy;
            const int16_t pic_w = (int16_t)job.width, pic_h = (int16_t)job.height;
            for (int l = 0; l < nl; l++)
                for (int r = 0; r < (l ? nr1 : nr0); r++) {
                    if (rounds == 2 && ((l == 0 && r == 0) != (round == 0)))
                        continue;
                    if (!st.do_ref[l][r])
                        continue;
                    int16_t w = st.is_w[l][r], h = st.is_h[l][r];
                    const int16_t xc = st.is_xc[l][r], yc = st.is_yc[l][r];
                    int16_t xo = i16(xc - (w >> 1));
                    int16_t yo = i16(yc - (h >> 1));
                    xo = ((org_x + xo) < -pad) ? i16(-pad - org_x) : xo;
                    w  = ((org_x + xo) < -pad) ? i16(w - (-pad - (org_x + xo))) : w;
                    xo = ((org_x + xo) > pic_w - 1) ? i16(xo - ((org_x + xo) - (pic_w - 1))) : xo;
                    w  = ((org_x + xo + w) > pic_w) ? i16(max(1, w - ((org_x + xo + w) - pic_w))) : w;
                    w  = (w < 8) ? w : i16(w & ~0x07);
                    yo = ((org_y + yo) < -pad) ? i16(-pad - org_y) : yo;
                    h  = ((org_y + yo) < -pad) ? i16(h - (-pad - (org_y + yo))) : h;
                    yo = ((org_y + yo) > pic_h - 1) ? i16(yo - ((org_y + yo) - (pic_h - 1))) : yo;
                    h  = (org_y + yo + h > pic_h) ? i16(max(1, h - ((org_y + yo + h) - pic_h))) : h;
                    FpRef &F     = st.fp[st.nfp++];
                    F.xo         = xo;
                    F.yo         = yo;
                    F.w          = w;
                    F.h          = h;
                    F.order_base = 1;
                    F.slot       = (uint8_t)(l * 4 + r);
                    F.nq         = (uint8_t)((w + 3) / 4);
                    F.item_begin = st.fp_items;
                    st.fp_items += (int)h * F.nq;
                }
        }
        __syncthreads();
        if (st.nfp)
            run_fullpel<SUB_ME>(st, job, dj);
        for (int f = 0; f < st.nfp; f++) {
            const int l = st.fp[f].slot >> 2, r = st.fp[f].slot & 3;
            decode_keys(st, l, r, st.is_xc[l][r], st.is_yc[l][r], st.fp[f].xo, st.fp[f].yo, st.fp[f].w);
        }
        __syncthreads();
    SVTME_STAMP(10);
    }

    // ---- me_prune_ref (motion_estimation.c:1522-1565)
    if (tid == 0 && c.enable_hme_flag && c.enable_me_hme_ref_pruning) {
        for (int l = 0; l < nl; l++)
            for (int r = 0; r < (l ? nr1 : nr0); r++) {
                st.hme_sad[l][r] = 0;
                if (!st.do_ref[l][r]) {
                    st.hme_sad[l][r] = (uint64_t)SVTME_MAX_SAD_VALUE * 64;
                    continue;
                }
                uint64_t s = 0;
                for (int i = 0; i < 64; i++) s += st.best_sad[l][r][21 + i];
                st.hme_sad[l][r] = s;
            }
        const uint16_t th = c.prune_ref_if_me_sad_dev_bigger_than_th;
        if (th != (uint16_t)~0) {
            uint64_t best = ~0ull;
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 4; j++) best = min_u64(best, st.hme_sad[i][j]);
            for (int li = 0; li < 2; li++)
                for (int ri = 1; ri < 4; ri++)
                    if ((st.hme_sad[li][ri] - best) * 100 > (th * best))
                        st.do_ref[li][ri] = 0;
        }
    }
    __syncthreads();
    SVTME_STAMP(11);

    // ---- records
    {
        svtme_ref_record *out = dj.out_records + (size_t)sb_local * dj.R;
        for (int slot = 0, k = 0; slot < 8; slot++) {
            const int l = slot >> 2, r = slot & 3;
            if (l >= nl || r >= (l ? nr1 : nr0))
                continue;
            svtme_ref_record &o = out[k++];
            const bool s = st.searched[l][r];
            for (int i = tid; i < SVTME_PU_COUNT; i += ME_THREADS) {
                o.best_sad[i] = s ? st.best_sad[l][r][i] : U32MAX;
                o.best_mv[i]  = st.best_mv[l][r][i];
            }
            if (tid == 0) {
                o.hme_sad  = st.hme_sad[l][r];
                o.hme_sc_x = st.hme_sc_x[l][r];
                o.hme_sc_y = st.hme_sc_y[l][r];
                o.zz_sad   = st.zz_sad[l][r];
                o.searched = st.searched[l][r];
                o.do_ref   = st.do_ref[l][r];
                for (int p = 0; p < 6; p++) o.pad[p] = 0;
            }
        }
    }
    if (dj.out_sb) {
        __syncthreads();
        finish_sb(st, dj, sb_local, bw, bh);
    }
    SVTME_STAMP(12);
    (void)lane;
}

// ----------------------------------------------------------------------------
// Host-callable launchers
// ----------------------------------------------------------------------------
extern "C" hipError_t svtme_launch_build_full(const void *src, uint32_t src_stride, int w, int h, int ten_bit,
                                              DevPlane dst, int left, int top, int rows, hipStream_t s) {
    const int n = (dst.stride >> 2) * rows;
    if (ten_bit)
        hipLaunchKernelGGL(k_build_full<true>, dim3((n + 255) / 256), dim3(256), 0, s, src, src_stride, w, h, dst,
                           left, top, rows);
    else
        hipLaunchKernelGGL(k_build_full<false>, dim3((n + 255) / 256), dim3(256), 0, s, src, src_stride, w, h, dst,
                           left, top, rows);
    return hipGetLastError();
}

extern "C" hipError_t svtme_launch_build_down(DevPlane prev, DevPlane dst, int left, int top, int rows,
                                              hipStream_t s) {
    const int n = (dst.stride >> 2) * rows;
    hipLaunchKernelGGL(k_build_down, dim3((n + 255) / 256), dim3(256), 0, s, prev, dst, left, top, rows);
    return hipGetLastError();
}

extern "C" hipError_t svtme_launch_me(const DevJob *dj, uint32_t sb_count, hipStream_t s) {
    if (dj->job.ctrl.me_search_method == SVTME_FULL_SAD_SEARCH)
        hipLaunchKernelGGL(k_me_sb<false>, dim3(sb_count), dim3(ME_THREADS), 0, s, *dj);
    else
        hipLaunchKernelGGL(k_me_sb<true>, dim3(sb_count), dim3(ME_THREADS), 0, s, *dj);
    return hipGetLastError();
}
