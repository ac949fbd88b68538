// svtme_me.hip — the per-superblock open-loop ME kernel (k_me_sb), gfx950.
//
// One workgroup = one 64x64 superblock (SB) x all of its references, exactly
// svt_aom_motion_estimation_b64 (reference motion_estimation.c:3076-3153):
//   zz SAD -> pre-HME -> HME L0 / L1 / L2 -> search centre -> HME pruning ->
//   full-pel search with the 85-PU argmin -> ME pruning -> candidates.
//
// Structure (MI355X-first):
//  * Control is lane-parallel: lane i of wave 0 owns one (reference slot,
//    quadrant / search region) pair; cross-reference decisions are wavefront
//    reductions; only the reference's sequential carries run as short loops.
//  * Every search stage stages its reference windows into LDS with bulk,
//    coalesced dword loads (one memory round trip per stage), realigned to
//    dword boundaries so the SAD loops read LDS at fixed byte shifts.
//  * SADs: v_sad_u8 on dword-packed pixels; 4 consecutive search positions per
//    lane (v_alignbyte_b32 rebuilds the shifted runs); block rows split over
//    G adjacent lanes and summed with DPP/shuffles.
//  * Argmins: 64-bit keys (sad << 32 | raster order) min-reduced across the
//    wavefront, then ds_min_u64 across waves; strict-< first-min semantics of
//    compute_sad_c.c:90 and motion_estimation.c:137-425 fall out of the order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svtme_device.h"

#define T2 256                 // threads per workgroup (4 waves)
#define ARENA_BYTES (20 * 1024) // LDS window arena
#define MAXT 40                // tasks per batch
#define U32MAX 0xFFFFFFFFu

#ifdef SVTME_STAMPS
#define STAMP(k)                                                                                                    \
    do {                                                                                                            \
        if (threadIdx.x == 0 && dj.stamps)                                                                          \
            dj.stamps[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime();                               \
    } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

namespace me2 {

__device__ __forceinline__ int16_t i16(int v) { return (int16_t)v; }
__device__ __forceinline__ int absi(int v) { return v < 0 ? -v : v; }
__device__ __forceinline__ uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// motion_estimation.c:1239-1243
__device__ __forceinline__ uint16_t scaled_dist(uint16_t dist) {
    uint8_t round_up = ((dist % 8) == 0) ? 0 : 1;
    return (uint16_t)(((dist * 5) / 8) + round_up);
}
__device__ __forceinline__ uint16_t ref_dist_const(const svtme_job &j, int l, int r) {
    int64_t d = (int64_t)j.picture_number - (int64_t)j.ref_picture_number[l][r];
    return (uint16_t)(int16_t)(d < 0 ? -d : d);
}
__device__ __forceinline__ bool tl_or_l0(const svtme_job &j, int l) { return j.temporal_layer_index > 0 || l == 0; }
__device__ __forceinline__ bool slot_valid(uint32_t vmask, int s) { return s >= 0 && s < 8 && ((vmask >> s) & 1u); }

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long t = __shfl_xor(v, o, 64);
        v                    = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min_u32(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// rank of this lane among lanes with pred set (exclusive prefix count) and the total
__device__ __forceinline__ int wave_compact(bool pred, int *total) {
    const unsigned long long m = __ballot(pred);
    *total                     = __popcll(m);
    const int lane             = threadIdx.x & 63;
    const unsigned long long lt = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
    return __popcll(lt);
}

// ----------------------------------------------------------------------------
// LDS state
// ----------------------------------------------------------------------------
struct Task {             // one sad_loop search (compute_sad_c.c:58-101) with its LDS window
    const uint8_t *g;     // global: first staged row, byte of search column 0
    const uint8_t *gd;    // global: search position (0,0), block row 0 (direct path)
    int32_t gstride;      // global bytes between staged window rows
    int32_t bstride;      // global bytes between block rows (direct path)
    int32_t pstride;      // global bytes between search rows (direct path)
    int32_t nitems;       // (search row, quad, row group) items
    uint32_t mnq, mwdw;   // magic divisors for nq and wdw
    int32_t bytes;
    uint16_t lds_off;     // arena byte offset (16-aligned)
    uint16_t pitch_dw;    // LDS dwords per staged row
    uint16_t wrows;       // staged rows
    uint16_t wdw;         // dwords copied per row
    int16_t sa_w;
    uint16_t src_off, src_stride; // source block in LDS (stride in bytes between block rows)
    uint8_t bw, bh;       // block width (bytes), block rows
    uint8_t ystep;        // staged rows per block row
    uint8_t skip;         // odd search rows only
    uint8_t odd;          // only odd plane rows are staged (skip + sub)
    uint8_t direct;       // window exceeds the arena: read global memory
    uint8_t nq;           // position quads per search row
    uint8_t owner;
    uint8_t lg, per, rpi; // log2 lanes per quad, block rows per lane, staged rows per wave pass
    uint8_t pad[3];
};

struct FpRef {            // full-pel search of one reference slot (or its centre probe)
    const uint8_t *g;     // global: search row 0, search column 0, block (0,0) row 0
    int32_t gstride;
    int32_t nitems;
    uint32_t mnq, mwdw;
    int32_t bytes;
    int16_t xo, yo, w, h;
    int32_t order_base;   // 0: 8x8-variance centre probe, 1: main search
    uint16_t lds_off, pitch_dw, wrows, wdw;
    uint8_t slot, nq, direct, rpi;
};

struct PreHme {
    uint64_t sad;
    int16_t col, row;
    uint16_t sa_w, sa_h;
    uint8_t valid, performed;
    uint8_t pad[2];
};

struct St {
    uint8_t src[64 * 64 + 32 * 32 + 16 * 16]; // full 64x64 | quarter 32x32 | sixteenth 16x16
    // per-slot (slot = list * 4 + ref) search results (SearchResults, me_context.h:348-355)
    uint64_t hme_sad[8];
    uint32_t zz[8];
    uint32_t reduce_div[8];
    int16_t sc_x[8], sc_y[8];
    uint8_t do_ref[8], searched[8];
    PreHme ph[8][2];
    // HME levels 0..2: [level][slot][quadrant q = sx * 2 + sy]
    int16_t lx[3][8][4], ly[3][8][4];
    uint64_t lsad[3][8][4];
    int16_t qox[8][4], qoy[8][4]; // search-area origins of the stage's tasks
    // integer search
    int16_t is_w[8], is_h[8], is_wb[8], is_hb[8], is_xc[8], is_yc[8];
    uint64_t is_best_hme[8];
    uint8_t need00[8];
    uint32_t nxm[16];
    uint32_t best_sad[8][SVTME_PU_COUNT];
    uint32_t best_mv[8][SVTME_PU_COUNT];
    // tasks
    Task tasks[MAXT];
    unsigned long long task_best[MAXT];
    FpRef fp[8];
    int32_t ntasks, nfp, flag, nbatch;
    uint8_t batch_end[MAXT + 1];
    uint8_t in_round[8];
    DevPlane pl[8][3];      // reference planes by slot (copied from the kernel argument)
    uint64_t refpic[8];
    uint16_t dist[8];
    uint32_t gm_cnt[2][4][2][2];
    const uint8_t *req[16]; // n x m SAD requests (zz, check_00_center)
    int32_t req_stride[16];
    int8_t req_slot[8];
    int32_t nreq;
    uint32_t me_distortion[SVTME_PU_COUNT];
    uint8_t cand0[SVTME_PU_COUNT + 3];
    // arena: search windows; the full-pel stage also keeps its PU keys here
    __attribute__((aligned(16))) uint8_t arena[ARENA_BYTES];
};

#define PU_KEY_BYTES (8 * SVTME_PU_COUNT * 8)
#define FP_ARENA (ARENA_BYTES - PU_KEY_BYTES)

// ----------------------------------------------------------------------------
// Search-area derivations (restated per reference function; pure)
// ----------------------------------------------------------------------------
// prehme_core (motion_estimation.c:1568-1636)
__device__ void prehme_area(const DevPlane &p, int16_t org_x, int16_t org_y, int16_t sa_w, int16_t sa_h, int16_t *oxo,
                            int16_t *oyo, int16_t *saw, int16_t *sah) {
    const int16_t pad_w = i16(p.pad - 1), pad_h = i16(p.pad - 1);
    const int16_t pw = i16(p.width), ph = i16(p.height);
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
    *oxo = ox, *oyo = oy, *saw = sa_w, *sah = sa_h;
}

// hme_level_0 (motion_estimation.c:835-889)
__device__ void hme_l0_rect(const svtme_controls &c, const DevPlane &p, int16_t org_x, int16_t org_y, int16_t sa_w,
                            int16_t sa_h, int sr_w, int sr_h, int16_t *oxo, int16_t *oyo, int16_t *saw,
                            int16_t *sah) {
    sa_w = i16((sa_w + 7) & ~0x07);
    const int16_t pad_w = i16(p.pad - 1), pad_h = i16(p.pad - 1);
    const int16_t pw = i16(p.width), ph = i16(p.height);
    const int16_t xd = i16(sa_w * sr_w), yd = i16(sa_h * sr_h);
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
    *oxo = ox, *oyo = oy, *saw = sa_w, *sah = sa_h;
}

// hme_level_1 / hme_level_2 (motion_estimation.c:938-990, 1039-1084)
__device__ void hme_refine_rect(int level, const DevPlane &p, int16_t org_x, int16_t org_y, int16_t sa_w, int16_t sa_h,
                                int16_t scx, int16_t scy, int16_t *oxo, int16_t *oyo, int16_t *saw, int16_t *sah) {
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
    *oxo = ox, *oyo = oy, *saw = sa_w, *sah = sa_h;
}

// get_hme_l0_search_area (motion_estimation.c:1800-1867); the per-ref
// mutate/restore of hme_l0_sa makes it a function of (list, ref, dist)
__device__ void hme_l0_area(const svtme_controls &c, int l, int r, uint16_t dist, int16_t l00x, int16_t l00y,
                            int16_t *sa_w, int16_t *sa_h) {
    uint32_t mnw = c.hme_l0_sa.sa_min.width, mnh = c.hme_l0_sa.sa_min.height;
    uint32_t mxw = c.hme_l0_sa.sa_max.width, mxh = c.hme_l0_sa.sa_max.height;
    if (c.enable_me_sr_adjustment && c.distance_based_hme_resizing) {
        uint8_t is_hor = 1, is_ver = 1, is_still = 0;
        if (c.reduce_hme_l0_sr_th_min && c.reduce_hme_l0_sr_th_max && (l || r)) {
            const int mvx = l00x, mvy = l00y;
            is_ver   = (absi(mvx) < c.reduce_hme_l0_sr_th_min) && (absi(mvy) > c.reduce_hme_l0_sr_th_max);
            is_hor   = (absi(mvx) > c.reduce_hme_l0_sr_th_max) && (absi(mvy) < c.reduce_hme_l0_sr_th_min);
            is_still = (absi(mvx) < (c.reduce_hme_l0_sr_th_min * 3)) && (absi(mvy) < (c.reduce_hme_l0_sr_th_min * 3));
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
    *sa_w = w, *sa_h = h;
}

// ----------------------------------------------------------------------------
// Task construction (one lane per task) and arena planning (wave 0)
// ----------------------------------------------------------------------------
struct TaskArgs { // make_task arguments held in registers until the task's LDS slot is known
    const uint8_t *base;
    int stride, wx, wy, sa_w, sa_h, bw, bh_eff, sub, skip, src_off, src_stride, owner;
};

// exact n / d for n * d < 2^32 with m = magic_u32(d); d == 1 wraps m to 0
__device__ __forceinline__ uint32_t magic_u32(uint32_t d) { return 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ int mdiv(int n, uint32_t m) { return m ? (int)__umulhi((uint32_t)n, m) : n; }

// staging geometry of a window with wdw dwords per row
__device__ __forceinline__ void stage_geometry(int wdw, uint8_t *rpi, uint32_t *mwdw) {
    *rpi  = (uint8_t)(wdw <= 64 ? 64 / wdw : 0);
    *mwdw = magic_u32((uint32_t)wdw);
}

// Fill a sad_loop task: window top-left (plane coords) (wx, wy), search area
// sa_w x sa_h, block bw x bh_eff rows; sub = block rows stride 2.
__device__ void make_task(Task &T, const TaskArgs &a) {
    const int bw = a.bw, bh_eff = a.bh_eff, sa_w = a.sa_w, sa_h = a.sa_h;
    const bool skip = a.skip && bw == 16 && bh_eff <= 16; // compute_sad_c.c:74
    T.sa_w       = (int16_t)sa_w;
    T.bw         = (uint8_t)bw;
    T.bh         = (uint8_t)bh_eff;
    T.skip       = (uint8_t)skip;
    T.owner      = (uint8_t)a.owner;
    T.src_off    = (uint16_t)a.src_off;
    T.src_stride = (uint16_t)a.src_stride;
    const int nrows = (sa_w > 0 && sa_h > 0) ? (skip ? sa_h / 2 : sa_h) : 0;
    const int nq    = sa_w > 0 ? (sa_w + 3) >> 2 : 0;
    T.nq            = (uint8_t)nq;
    T.gd            = a.base + (ptrdiff_t)a.wy * a.stride + a.wx;
    T.bstride       = a.sub ? 2 * a.stride : a.stride;
    T.pstride       = a.stride;
    int wrows;
    if (skip && a.sub) { // odd search rows x odd block rows: stage odd plane rows only
        T.g       = T.gd + a.stride;
        T.gstride = 2 * a.stride;
        T.ystep   = 1;
        T.odd     = 1;
        wrows     = nrows > 0 ? (nrows - 1) + bh_eff : 0;
    } else {
        T.g       = T.gd;
        T.gstride = a.stride;
        T.ystep   = a.sub ? 2 : 1;
        T.odd     = 0;
        const int last_y = nrows > 0 ? (skip ? 2 * nrows - 1 : nrows - 1) : 0;
        wrows            = nrows > 0 ? last_y + (bh_eff - 1) * T.ystep + 1 : 0;
    }
    T.wrows    = (uint16_t)wrows;
    T.wdw      = (uint16_t)(nq + ((bw + 3) >> 2));
    T.pitch_dw = (uint16_t)(T.wdw | 1);
    stage_geometry(T.wdw ? T.wdw : 1, &T.rpi, &T.mwdw);
    // G lanes share one position quad (block rows split G ways); fill one wavefront
    const int quads = nrows * nq;
    int lg = 0;
    while ((2 << lg) <= bh_eff && quads * (2 << lg) <= 64) lg++;
    T.lg     = (uint8_t)lg;
    T.per    = (uint8_t)((bh_eff + (1 << lg) - 1) >> lg);
    T.nitems = quads << lg;
    T.mnq    = magic_u32(nq ? nq : 1);
    const int bytes = ((wrows * T.pitch_dw * 4) + 15) & ~15;
    T.direct = (uint8_t)(bytes > ARENA_BYTES);
    T.bytes  = T.direct ? 0 : bytes;
}

// wave-inclusive prefix sum over lanes (lane order)
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o)
            v += t;
    }
    return v;
}

// wave 0, all lanes: lay the n compacted windows (this lane's at index k when
// mk) into arena batches of at most `cap` bytes; greedy fallback when the
// windows overflow one batch
template <typename W>
__device__ void plan_windows(St &st, W *items, bool mk, int k, int n, int cap) {
    const int lane  = threadIdx.x & 63;
    const int bytes = mk ? (int)items[k].bytes : 0;
    const int incl  = wave_incl_scan(bytes);
    const int total = __shfl(incl, 63, 64);
    if (total <= cap) {
        if (mk)
            items[k].lds_off = (uint16_t)(incl - bytes);
        if (lane == 0) {
            st.batch_end[0] = 0;
            st.batch_end[1] = (uint8_t)n;
            st.nbatch       = n ? 1 : 0;
        }
    } else if (lane == 0) {
        int b = 0, off = 0;
        st.batch_end[0] = 0;
        for (int t = 0; t < n; t++) {
            const int by = items[t].bytes;
            if (off + by > cap && t > (int)st.batch_end[b]) {
                st.batch_end[++b] = (uint8_t)t;
                off = 0;
            }
            items[t].lds_off = (uint16_t)off;
            off += by;
        }
        st.batch_end[b + 1] = (uint8_t)n;
        st.nbatch           = b + 1;
    }
}

// bulk copy of one window, all 4 waves: aligned dword loads realigned to byte 0
// of each LDS row; lane -> (row-in-group, dword) without per-element division
__device__ __forceinline__ void stage_window(uint8_t *arena, const uint8_t *g, int gstride, int wrows, int wdw,
                                             int pitch_dw, int lds_off, int rpi, uint32_t mwdw) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int sh       = (int)((uintptr_t)g & 3);
    const uint8_t *ga  = g - sh;
    uint32_t *dst      = (uint32_t *)(arena + lds_off);
    if (rpi) {
        const int sub = mdiv(lane, mwdw), d = lane - sub * wdw;
        if (sub < rpi) {
            for (int r = wid * rpi + sub; r < wrows; r += 4 * rpi) {
                const uint32_t *src = (const uint32_t *)(ga + (ptrdiff_t)r * gstride) + d;
                dst[r * pitch_dw + d] = __builtin_amdgcn_alignbyte(src[1], src[0], sh);
            }
        }
    } else {
        for (int r = wid; r < wrows; r += 4)
            for (int d = lane; d < wdw; d += 64) {
                const uint32_t *src = (const uint32_t *)(ga + (ptrdiff_t)r * gstride) + d;
                dst[r * pitch_dw + d] = __builtin_amdgcn_alignbyte(src[1], src[0], sh);
            }
    }
}

// SAD partials of positions x0..x0+3 over block rows [k0, k1) from a realigned
// LDS window (position x0 at dword q of each row)
template <bool MASK>
__device__ __forceinline__ void quad_rows_lds(const uint32_t *win, int pitch_dw, int row0, int ystep,
                                              const uint8_t *src, int src_stride, int bw, int k0, int k1,
                                              uint32_t acc[4]) {
    const int nd             = (bw + 3) >> 2;
    const uint32_t last_mask = MASK ? ((1u << (8 * (bw & 3))) - 1u) : 0xFFFFFFFFu;
    for (int k = k0; k < k1; k++) {
        const uint32_t *rd = win + (row0 + k * ystep) * pitch_dw;
        const uint32_t *sd = (const uint32_t *)(src + k * src_stride);
        uint32_t d0        = rd[0];
        for (int j = 0; j < nd; j++) {
            const uint32_t d1 = rd[j + 1];
            const uint32_t m  = (MASK && j == nd - 1) ? last_mask : 0xFFFFFFFFu;
            const uint32_t s  = MASK ? (sd[j] & m) : sd[j];
            const uint32_t r1 = __builtin_amdgcn_alignbyte(d1, d0, 1), r2 = __builtin_amdgcn_alignbyte(d1, d0, 2),
                           r3 = __builtin_amdgcn_alignbyte(d1, d0, 3);
            acc[0] = __builtin_amdgcn_sad_u8(MASK ? d0 & m : d0, s, acc[0]);
            acc[1] = __builtin_amdgcn_sad_u8(MASK ? r1 & m : r1, s, acc[1]);
            acc[2] = __builtin_amdgcn_sad_u8(MASK ? r2 & m : r2, s, acc[2]);
            acc[3] = __builtin_amdgcn_sad_u8(MASK ? r3 & m : r3, s, acc[3]);
            d0 = d1;
        }
    }
}

// v_qsad_pk_u16_u8: 4 SADs of one source dword against the 4 byte shifts of a
// reference dword pair, accumulated in 4 u16 lanes
__device__ __forceinline__ unsigned long long qsad(uint32_t lo, uint32_t hi, uint32_t s, unsigned long long a) {
    return __builtin_amdgcn_qsad_pk_u16_u8(((unsigned long long)hi << 32) | lo, s, a);
}
__device__ __forceinline__ void qsad_unpack(unsigned long long a, uint32_t acc[4]) {
    acc[0] += (uint32_t)a & 0xFFFFu;
    acc[1] += (uint32_t)a >> 16;
    acc[2] += (uint32_t)(a >> 32) & 0xFFFFu;
    acc[3] += (uint32_t)(a >> 48);
}

// quad_rows_lds for whole-dword block widths on v_qsad_pk_u16_u8; the u16
// lanes are widened every 64 / nd rows (nd * 1020 * rows <= 65280)
__device__ __forceinline__ void quad_rows_qsad(const uint32_t *win, int pitch_dw, int row0, int ystep,
                                               const uint8_t *src, int src_stride, int nd, int k0, int k1,
                                               uint32_t acc[4]) {
    const int chunk = 64 / nd;
    for (int kc = k0; kc < k1; kc += chunk) {
        const int ke         = min(k1, kc + chunk);
        unsigned long long a = 0;
        for (int k = kc; k < ke; k++) {
            const uint32_t *rd = win + (row0 + k * ystep) * pitch_dw;
            const uint32_t *sd = (const uint32_t *)(src + k * src_stride);
            uint32_t d0        = rd[0];
            for (int j = 0; j < nd; j++) {
                const uint32_t d1 = rd[j + 1];
                a                 = qsad(d0, d1, sd[j], a);
                d0                = d1;
            }
        }
        qsad_unpack(a, acc);
    }
}

// same from global memory at an arbitrary byte address (oversized windows)
__device__ __forceinline__ void quad_rows_global(const uint8_t *ref, int ref_stride, const uint8_t *src, int src_stride,
                                                 int bw, int k0, int k1, uint32_t acc[4]) {
    const int sh             = (int)((uintptr_t)ref & 3);
    const uint8_t *ra        = ref - sh;
    const int nd             = (bw + 3) >> 2;
    const uint32_t last_mask = (bw & 3) ? ((1u << (8 * (bw & 3))) - 1u) : 0xFFFFFFFFu;
    for (int k = k0; k < k1; k++) {
        const uint32_t *rd = (const uint32_t *)(ra + (ptrdiff_t)k * ref_stride);
        const uint32_t *sd = (const uint32_t *)(src + k * src_stride);
        uint32_t d0 = rd[0], d1 = rd[1];
        for (int j = 0; j < nd; j++) {
            const uint32_t d2 = rd[j + 2];
            const uint32_t m  = (j == nd - 1) ? last_mask : 0xFFFFFFFFu;
            const uint32_t s  = sd[j] & m;
            const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            acc[0] = __builtin_amdgcn_sad_u8(e0 & m, s, acc[0]);
            acc[1] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 1) & m, s, acc[1]);
            acc[2] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 2) & m, s, acc[2]);
            acc[3] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 3) & m, s, acc[3]);
            d0 = d1;
            d1 = d2;
        }
    }
}

#define UNI(x) __builtin_amdgcn_readfirstlane((int)(x))

// Run every planned task; one wavefront per task. Items = (search row, quad,
// row group g) with g innermost; the 2^lg lanes of a quad are adjacent.
__device__ void search_tasks(St &st) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nb = st.nbatch;
    for (int b = 0; b < nb; b++) {
        const int t0 = st.batch_end[b], t1 = st.batch_end[b + 1];
        __syncthreads();
        for (int t = t0; t < t1; t++) {
            const Task &T = st.tasks[t];
            if (!T.direct)
                stage_window(st.arena, T.g, UNI(T.gstride), UNI(T.wrows), UNI(T.wdw), UNI(T.pitch_dw), UNI(T.lds_off),
                             UNI(T.rpi), (uint32_t)UNI(T.mwdw));
        }
        __syncthreads();
        for (int t = t0 + wid; t < t1; t += 4) {
            const Task &T = st.tasks[t];
            const int nitems = UNI(T.nitems), lg = UNI(T.lg), nq = UNI(T.nq), per = UNI(T.per), bh = UNI(T.bh);
            const int bw = UNI(T.bw), sa_w = UNI(T.sa_w), skip = UNI(T.skip), odd = UNI(T.odd);
            const int ystep = UNI(T.ystep), pitch = UNI(T.pitch_dw), direct = UNI(T.direct);
            const uint32_t mnq = (uint32_t)UNI(T.mnq);
            const uint32_t *win = (const uint32_t *)(st.arena + UNI(T.lds_off));
            const uint8_t *src  = st.src + UNI(T.src_off);
            const int sstride   = UNI(T.src_stride);
            const int G = 1 << lg;
            unsigned long long best = ~0ull;
            for (int base = 0; base < nitems; base += 64) {
                const int i  = base + lane;
                const int g  = i & (G - 1), qi = i >> lg;
                const int yy = mdiv(qi, mnq), q = qi - yy * nq;
                const int x0 = 4 * q, y = skip ? 2 * yy + 1 : yy;
                uint32_t acc[4] = {0, 0, 0, 0};
                if (i < nitems) {
                    const int k0 = min(bh, g * per), k1 = min(bh, k0 + per);
                    if (direct)
                        quad_rows_global(T.gd + (ptrdiff_t)y * T.pstride + x0, T.bstride, src, sstride, bw, k0, k1,
                                         acc);
                    else if (bw & 3)
                        quad_rows_lds<true>(win + q, pitch, odd ? yy : y, ystep, src, sstride, bw, k0, k1, acc);
                    else
                        quad_rows_qsad(win + q, pitch, odd ? yy : y, ystep, src, sstride, bw >> 2, k0, k1, acc);
                }
                for (int o = 1; o < G; o <<= 1)
#pragma unroll
                    for (int k = 0; k < 4; k++) acc[k] += __shfl_xor(acc[k], o, 64);
                if (i < nitems && g == 0) {
#pragma unroll
                    for (int s = 0; s < 4; s++)
                        if (x0 + s < sa_w) {
                            const unsigned long long kk =
                                ((unsigned long long)acc[s] << 32) | ((uint32_t)y << 16) | (uint32_t)(x0 + s);
                            best = kk < best ? kk : best;
                        }
                }
            }
            best = wave_min_u64(best);
            if (lane == 0)
                st.task_best[t] = best;
        }
    }
    __syncthreads();
}

// sad_loop result: best_sad starts at 0xffffff and the centre stays put unless
// beaten (compute_sad_c.c:71, :90)
__device__ __forceinline__ void task_result(const St &st, int t, uint64_t *best, int16_t *x, int16_t *y) {
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

// n x m SADs of the 64-wide source (sub rows) vs full-res positions, one
// wavefront per request (compute_sad_c.c:20-37)
__device__ void nxm_requests(St &st, const uint8_t *const *refs, const int32_t *strides, int nreq, int rows,
                             int width) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wd4 = (width + 3) >> 2;
    const uint32_t mwd = magic_u32((uint32_t)wd4);
    for (int q = wid; q < nreq; q += T2 / 64) {
        uint32_t acc       = 0;
        const uint8_t *ref = refs[q];
        const int str      = strides[q];
        const int sh       = (int)((uintptr_t)ref & 3);
        for (int e = lane; e < rows * wd4; e += 64) {
            const int r = mdiv(e, mwd), j = e - r * wd4;
            const uint32_t *da = (const uint32_t *)(ref + (ptrdiff_t)r * str + 4 * j - sh);
            uint32_t run       = __builtin_amdgcn_alignbyte(da[1], da[0], sh);
            uint32_t s         = *(const uint32_t *)(st.src + r * 128 + 4 * j);
            const int valid    = width - 4 * j;
            if (valid < 4) {
                const uint32_t m = (1u << (8 * valid)) - 1u;
                run &= m;
                s &= m;
            }
            acc = __builtin_amdgcn_sad_u8(run, s, acc);
        }
        acc = wave_sum_u32(acc);
        if (lane == 0)
            st.nxm[q] = acc;
    }
}

// ----------------------------------------------------------------------------
// Full-pel search with the 85-PU argmin (motion_estimation.c:98-425, 781-817):
// lane = 8x8 block in Z-order; one item = 4 consecutive x positions of a row;
// 16x16 / 32x32 / 64x64 SADs are DPP lane sums (quad_perm, row_ror, row_bcast).
// Keys: (sad << 12 | order) in 32 bits when every order < 4096 (64x64 SAD <
// 2^20), else (sad << 32 | order).
// ----------------------------------------------------------------------------
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v) {
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}

// Window of one reference: rows h + 63, bytes round4(w) + 64 (16 dwords of 8x8 blocks)
__device__ void make_fp(FpRef &F, const DevPlane &P, uint32_t ox, uint32_t oy, int slot, int16_t xo, int16_t yo,
                        int16_t w, int16_t h, int order_base, bool allow_stage) {
    F.slot       = (uint8_t)slot;
    F.xo = xo, F.yo = yo, F.w = w, F.h = h;
    F.order_base = order_base;
    F.nq         = (uint8_t)((w + 3) >> 2);
    F.mnq        = magic_u32(F.nq ? F.nq : 1);
    F.g          = P.base + (ptrdiff_t)((int)oy + yo) * P.stride + ((int)ox + xo);
    F.gstride    = P.stride;
    F.wrows      = (uint16_t)(h + 63);
    F.wdw        = (uint16_t)(F.nq + 16);
    F.pitch_dw   = (uint16_t)(F.wdw | 1);
    stage_geometry(F.wdw, &F.rpi, &F.mwdw);
    F.nitems     = (int)h * F.nq;
    const int bytes = ((F.wrows * F.pitch_dw * 4) + 15) & ~15;
    F.direct     = (uint8_t)(!allow_stage || bytes > FP_ARENA);
    F.bytes      = F.direct ? 0 : bytes;
}

template <bool SUB, bool K32>
__device__ void fullpel_run(St &st) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int z16 = lane >> 2, k4 = lane & 3;
    const int by = ((z16 >> 3) << 2) | (((z16 >> 1) & 1) << 1) | (k4 >> 1);
    const int bx = (((z16 >> 2) & 1) << 2) | ((z16 & 1) << 1) | (k4 & 1);
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1;
    typedef typename std::conditional<K32, uint32_t, unsigned long long>::type key_t;
    unsigned long long *keys = (unsigned long long *)(st.arena + FP_ARENA);
    for (int e = tid; e < st.nfp * SVTME_PU_COUNT; e += T2) {
        const int f = e / SVTME_PU_COUNT;
        keys[st.fp[f].slot * SVTME_PU_COUNT + (e - f * SVTME_PU_COUNT)] = ~0ull;
    }
    uint32_t src[ROWS][2];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const uint32_t *s = (const uint32_t *)(st.src + (by * 8 + r * RSTEP) * 64 + bx * 8);
        src[r][0] = s[0];
        src[r][1] = s[1];
    }
    const int nb = st.nbatch;
    for (int b = 0; b < nb; b++) {
        const int f0 = st.batch_end[b], f1 = st.batch_end[b + 1];
        __syncthreads();
        for (int f = f0; f < f1; f++) {
            const FpRef &F = st.fp[f];
            if (!F.direct)
                stage_window(st.arena, F.g, UNI(F.gstride), UNI(F.wrows), UNI(F.wdw), UNI(F.pitch_dw), UNI(F.lds_off),
                             UNI(F.rpi), (uint32_t)UNI(F.mwdw));
        }
        __syncthreads();
        for (int f = f0; f < f1; f++) {
            const FpRef &F = st.fp[f];
            const int nitems = UNI(F.nitems);
            if (wid >= nitems)
                continue; // wave-uniform
            const int nq = UNI(F.nq), w = UNI(F.w), obase = UNI(F.order_base), pitch = UNI(F.pitch_dw);
            const int direct = UNI(F.direct), gstride = UNI(F.gstride);
            const uint32_t mnq = (uint32_t)UNI(F.mnq);
            const uint32_t *wbase = (const uint32_t *)(st.arena + UNI(F.lds_off)) + by * 8 * pitch + bx * 2;
            key_t b8 = (key_t)~0ull, b16 = (key_t)~0ull, b32 = (key_t)~0ull, b64 = (key_t)~0ull;
            for (int i = wid; i < nitems; i += T2 / 64) {
                const int y = mdiv(i, mnq), q = i - y * nq, x0 = 4 * q;
                uint32_t acc[4] = {0, 0, 0, 0};
                if (!direct) {
                    const uint32_t *win = wbase + y * pitch + q;
                    unsigned long long a = 0;
#pragma unroll
                    for (int rr = 0; rr < ROWS; rr++) {
                        const uint32_t *rd = win + rr * RSTEP * pitch;
                        const uint32_t d0 = rd[0], d1 = rd[1], d2 = rd[2];
                        a = qsad(d0, d1, src[rr][0], a);
                        a = qsad(d1, d2, src[rr][1], a);
                    }
                    qsad_unpack(a, acc);
                } else {
                    const uint8_t *rp = F.g + (ptrdiff_t)(y + by * 8) * gstride + x0 + bx * 8;
                    const int sh      = (int)((uintptr_t)rp & 3);
                    const uint8_t *ra = rp - sh;
#pragma unroll
                    for (int rr = 0; rr < ROWS; rr++) {
                        const uint32_t *rd = (const uint32_t *)(ra + (ptrdiff_t)(rr * RSTEP) * gstride);
                        const uint32_t e0 = __builtin_amdgcn_alignbyte(rd[1], rd[0], sh);
                        const uint32_t e1 = __builtin_amdgcn_alignbyte(rd[2], rd[1], sh);
                        const uint32_t e2 = __builtin_amdgcn_alignbyte(rd[3], rd[2], sh);
                        const uint32_t s0 = src[rr][0], s1 = src[rr][1];
                        acc[0] = __builtin_amdgcn_sad_u8(e0, s0, acc[0]);
                        acc[0] = __builtin_amdgcn_sad_u8(e1, s1, acc[0]);
                        acc[1] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 1), s0, acc[1]);
                        acc[1] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e2, e1, 1), s1, acc[1]);
                        acc[2] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 2), s0, acc[2]);
                        acc[2] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e2, e1, 2), s1, acc[2]);
                        acc[3] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e1, e0, 3), s0, acc[3]);
                        acc[3] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(e2, e1, 3), s1, acc[3]);
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (x0 + k >= w)
                        break; // wave-uniform
                    const uint32_t s8 = SUB ? acc[k] << 1 : acc[k];
                    const uint32_t s16 = dpp_add<0x4E>(dpp_add<0xB1>(s8));       // xor 1, xor 2
                    const uint32_t s32 = dpp_add<0x128>(dpp_add<0x124>(s16));    // row_ror 4, 8
                    const uint32_t s64 = dpp_add<0x143, 0xC>(dpp_add<0x142, 0xA>(s32)); // valid in row 3
                    const uint32_t o = (uint32_t)(obase + y * w + x0 + k);
                    if (K32) {
                        b8  = min_u32((uint32_t)b8, (s8 << 12) | o);
                        b16 = min_u32((uint32_t)b16, (s16 << 12) | o);
                        b32 = min_u32((uint32_t)b32, (s32 << 12) | o);
                        b64 = min_u32((uint32_t)b64, (s64 << 12) | o);
                    } else {
                        const unsigned long long k8 = ((unsigned long long)s8 << 32) | o;
                        const unsigned long long k16 = ((unsigned long long)s16 << 32) | o;
                        const unsigned long long k32 = ((unsigned long long)s32 << 32) | o;
                        const unsigned long long k64 = ((unsigned long long)s64 << 32) | o;
                        b8  = k8 < b8 ? k8 : b8;
                        b16 = k16 < b16 ? k16 : b16;
                        b32 = k32 < b32 ? k32 : b32;
                        b64 = k64 < b64 ? k64 : b64;
                    }
                }
            }
            // merge into the slot's PU keys (64-bit, sad << 32 | order)
            unsigned long long *pk = keys + UNI(F.slot) * SVTME_PU_COUNT;
            auto wide = [](key_t kk) -> unsigned long long {
                if (K32)
                    return ((unsigned long long)((uint32_t)kk >> 12) << 32) | ((uint32_t)kk & 0xFFFu);
                return (unsigned long long)kk;
            };
            atomicMin(&pk[21 + lane], wide(b8));
            if ((lane & 3) == 0)
                atomicMin(&pk[5 + (lane >> 2)], wide(b16));
            if ((lane & 15) == 0)
                atomicMin(&pk[1 + (lane >> 4)], wide(b32));
            if (lane == 63)
                atomicMin(&pk[0], wide(b64));
        }
    }
    __syncthreads();
    // decode: strict-< update of the running best (motion_estimation.c:1366, :137-205)
    for (int e = tid; e < st.nfp * SVTME_PU_COUNT; e += T2) {
        const int f = e / SVTME_PU_COUNT, pu = e - f * SVTME_PU_COUNT;
        const FpRef &F = st.fp[f];
        const unsigned long long k = keys[F.slot * SVTME_PU_COUNT + pu];
        const uint32_t sad = (uint32_t)(k >> 32);
        if (k != ~0ull && sad < st.best_sad[F.slot][pu]) {
            const int p = (int)(uint32_t)k - F.order_base;
            const int16_t my = (int16_t)(F.yo + p / F.w);
            const int16_t mx = (int16_t)(F.xo + p % F.w);
            st.best_sad[F.slot][pu] = sad;
            st.best_mv[F.slot][pu]  = ((uint32_t)(uint16_t)my << 16) | (uint16_t)mx;
        }
    }
    __syncthreads();
}

template <bool SUB>
__device__ void fullpel(St &st) {
    if (st.flag)
        fullpel_run<SUB, true>(st);
    else
        fullpel_run<SUB, false>(st);
}

// ----------------------------------------------------------------------------
// tables + candidates (motion_estimation.c:2520-3007)
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
__device__ void finish_sb(St &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh) {
    const svtme_job &job = dj.job;
    const int tid = threadIdx.x;
    const int nl = job.num_lists, nr0 = job.num_refs[0], nr1 = nl == 2 ? job.num_refs[1] : 0;
    svtme_sb_result *o = dj.out_sb + sb_local;
    // zero the result (uint32 stores; sizeof is a multiple of 4)
    uint32_t *ow = (uint32_t *)o;
    for (int i = tid; i < (int)(sizeof(svtme_sb_result) / 4); i += T2) ow[i] = 0;
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
            st.me_distortion[pu]    = st.best_sad[(0) * 4 + (0)][n];
            st.cand0[pu]            = 0;
            if (st.do_ref[(0) * 4 + (0)] && use) {
                o->me_candidate_array[pu][0] = mk_cand(0, 0, 0, 0, 0);
                o->me_mv_array[pu][0]        = st.best_mv[(0) * 4 + (0)][n];
            }
        } else if (mode == 1) { // construct_me_candidate_array_mrp_off
            const int pu = c_z_to_raster[n];
            uint32_t nlist = nl;
            const uint8_t org0 = st.do_ref[(0) * 4 + (0)], org1 = nl == 1 ? 0 : st.do_ref[(1) * 4 + (0)];
            if (nlist < 2 || !st.do_ref[(1) * 4 + (0)])
                nlist = 1;
            const uint32_t prune_th = (org0 && org1) ? (uint32_t)job.ctrl.prune_me_candidates_th : 0;
            uint8_t off = 0;
            uint32_t blk = (org0 ? 1u : 0u) | (org1 ? 2u : 0u); // bit li
            const uint32_t s0 = st.best_sad[(0) * 4 + (0)][n], s1 = st.best_sad[(1) * 4 + (0)][n];
            const uint32_t best = (org0 && org1) ? min_u32(s0, s1) : org0 ? s0 : s1;
            st.me_distortion[pu] = best;
            int min_list = -1;
            if (job.ctrl.use_best_unipred_cand_only && (blk & 3u) == 3u)
                min_list = s0 < s1 ? 0 : 1;
            uint8_t c0 = 0;
            for (int li = 0; (uint32_t)li < nlist && (use || off == 0); ++li) {
                if (!((blk >> li) & 1u))
                    continue;
                if (prune_th > 0) {
                    const uint32_t dd = (st.best_sad[(li) * 4 + (0)][n] - best) * 100;
                    if (dd > best * prune_th) {
                        blk &= ~(1u << li);
                        continue;
                    }
                }
                if (min_list != -1 && min_list != li) {
                    if (use)
                        o->me_mv_array[pu][li ? job.max_l0 : 0] = st.best_mv[(li) * 4 + (0)][n];
                    continue;
                }
                if (use) {
                    const uint8_t cb = mk_cand(li, 0, 0, li == 0 ? li : 24, li == 1 ? li : 24);
                    o->me_candidate_array[pu][off] = cb;
                    if (off == 0)
                        c0 = cb;
                    o->me_mv_array[pu][li ? job.max_l0 : 0] = st.best_mv[(li) * 4 + (0)][n];
                }
                off++;
            }
            if ((blk & 3u) == 3u && use) {
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
            uint32_t blk = 0; // bit li * 4 + r
            const uint32_t prune_th = (uint32_t)job.ctrl.prune_me_candidates_th;
            uint32_t best = U32MAX;
            for (int li = 0; li < nl; li++)
                for (int r = 0; r < (li ? nr1 : nr0); r++) {
                    blk |= st.do_ref[(li) * 4 + (r)] ? 1u << (li * 4 + r) : 0u;
                    if (!((blk >> (li * 4 + r)) & 1u))
                        continue;
                    best = min_u32(best, st.best_sad[(li) * 4 + (r)][n]);
                }
            st.me_distortion[pu] = best;
            uint8_t c0 = 0;
            for (int li = 0; li < nl && (use || off == 0); ++li)
                for (int r = 0; r < (li ? nr1 : nr0) && (use || off == 0); ++r) {
                    if (!((blk >> (li * 4 + r)) & 1u))
                        continue;
                    if (prune_th > 0) {
                        const uint32_t dd = (st.best_sad[(li) * 4 + (r)][n] - best) * 100;
                        if (dd > best * prune_th) {
                            blk &= ~(1u << (li * 4 + r));
                            continue;
                        }
                    }
                    if (use) {
                        const uint8_t cb = mk_cand(li, r, r, li == 0 ? li : 24, li == 1 ? li : 24);
                        o->me_candidate_array[pu][off] = cb;
                        if (off == 0)
                            c0 = cb;
                        o->me_mv_array[pu][(li ? job.max_l0 : 0) + r] = st.best_mv[(li) * 4 + (r)][n];
                    }
                    off++;
                }
            if (nl == 2 && use) {
                for (int a2 = 0; a2 < nr0; a2++)
                    for (int b2 = 0; b2 < nr1; b2++) {
                        if (job.only_l_bwd && (a2 > 0 || b2 > 0))
                            continue;
                        if (((blk >> (0 * 4 + a2)) & 1u) && ((blk >> (1 * 4 + b2)) & 1u)) {
                            const uint8_t cb = mk_cand(2, a2, b2, 0, 1);
                            if (off == 0)
                                c0 = cb;
                            o->me_candidate_array[pu][off++] = cb;
                        }
                    }
                if (!job.only_l_bwd)
                    for (int a2 = 1; a2 < nr0; a2++)
                        if (((blk >> (0 * 4 + 0)) & 1u) && ((blk >> (0 * 4 + a2)) & 1u)) {
                            const uint8_t cb = mk_cand(2, 0, a2, 0, 0);
                            if (off == 0)
                                c0 = cb;
                            o->me_candidate_array[pu][off++] = cb;
                        }
                if (!job.only_l_bwd && nr1 == 3 && ((blk >> (1 * 4 + 0)) & 1u) && ((blk >> (1 * 4 + 2)) & 1u)) {
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
            uint32_t(*cnt)[4][2][2] = st.gm_cnt;
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
                    const uint64_t a2 = job.picture_number, b2 = st.refpic[li * 4 + ri];
                    const uint16_t dist = (uint16_t)absi((int16_t)((a2 > b2 ? a2 : b2) - (a2 < b2 ? a2 : b2)));
                    active_th = job.gm_use_distance_based_active_th ? max(dist >> 1, 4) : 4;
                } else {
                    const uint16_t dist = (uint16_t)absi((int16_t)(job.picture_number - st.refpic[li * 4 + ri]));
                    active_th = job.gm_use_distance_based_active_th ? max(dist * 16, 32) : 32;
                }
                const uint32_t mv = st.best_mv[(li) * 4 + (ri)][n];
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
// The kernel
// ----------------------------------------------------------------------------
template <bool SUB_ME>
__global__ void __launch_bounds__(T2) __attribute__((amdgpu_waves_per_eu(4, 8))) k_me_sb(const DevJob dj) {
    __shared__ St st;
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool w0 = wid == 0;
    // XCD-aware SB order: blocks b and b+8 share an XCD, so each XCD gets one
    // contiguous band of SBs whose windows overlap in its L2 (bijective)
    const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const uint32_t sb_local = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t b64 = job.sb_begin + sb_local;
    const uint32_t ox = (b64 % dj.pic_w_b64) * 64, oy = (b64 / dj.pic_w_b64) * 64;
    const uint32_t bw = (job.width - ox) < 64 ? job.width - ox : 64;
    const uint32_t bh = (job.height - oy) < 64 ? job.height - oy : 64;
    const int nl = job.num_lists;
    const bool hsub = c.hme_search_method != SVTME_FULL_SAD_SEARCH;
    STAMP(0);

    // ---- source blocks -> LDS (me_process.c:183-214), 16-byte loads
    {
        const DevPlane &F = dj.cur.lv[0];
        for (int e = tid; e < 64 * 4; e += T2) {
            const int r = e >> 2, j = e & 3;
            ((uint4 *)st.src)[e] = *(const uint4 *)(F.base + (ptrdiff_t)(oy + r) * F.stride + ox + 16 * j);
        }
        const DevPlane &Q = dj.cur.lv[1];
        if (tid < 64) {
            const int r = tid >> 1, j = tid & 1;
            ((uint4 *)(st.src + 4096))[tid] =
                *(const uint4 *)(Q.base + (ptrdiff_t)((oy >> 1) + r) * Q.stride + (ox >> 1) + 16 * j);
        } else if (tid < 80) {
            const DevPlane &S = dj.cur.lv[2];
            const int r = tid - 64;
            ((uint4 *)(st.src + 5120))[r] = *(const uint4 *)(S.base + (ptrdiff_t)((oy >> 2) + r) * S.stride + (ox >> 2));
        }
    }
    // ---- per-slot reference table into LDS (constant-index reads of the argument)
    uint32_t vmask = 0;
#pragma unroll
    for (int s = 0; s < 8; s++)
        if ((s >> 2) < job.num_lists && (s & 3) < job.num_refs[s >> 2])
            vmask |= 1u << s;
    if (tid == 0) {
#pragma unroll
        for (int s = 0; s < 8; s++) {
#pragma unroll
            for (int v = 0; v < 3; v++) st.pl[s][v] = dj.ref[s >> 2][s & 3].lv[v];
            st.refpic[s] = job.ref_picture_number[s >> 2][s & 3];
            st.dist[s]   = ref_dist_const(job, s >> 2, s & 3);
        }
    }
    // ---- init_me_hme_data (motion_estimation.c:3010-3070)
    if (tid < 8) {
        const int s = tid;
        st.do_ref[s] = 1;
        st.hme_sad[s] = U32MAX;
        st.sc_x[s] = st.sc_y[s] = 0;
        st.reduce_div[s] = 1;
        st.zz[s] = U32MAX;
        for (int k = 0; k < 2; k++) {
            st.ph[s][k].valid = 0;
            st.ph[s][k].performed = 0;
            st.ph[s][k].sad = 0;
            st.ph[s][k].col = st.ph[s][k].row = 0;
        }
    }
    if (tid < 96) {
        (&st.lx[0][0][0])[tid] = 0;
        (&st.ly[0][0][0])[tid] = 0;
        (&st.lsad[0][0][0])[tid] = 0;
    }
    for (int e = tid; e < 8 * SVTME_PU_COUNT; e += T2) (&st.best_mv[0][0])[e] = 0;
    __syncthreads();
    STAMP(1);

    // ---- init_zz_sad (motion_estimation.c:2382-2437)
    if (c.me_early_exit_th || c.me_safe_limit_zz_th) {
        if (w0) {
            const int s = lane;
            const bool need = s < 8 && slot_valid(vmask, s) && tl_or_l0(job, s >> 2);
            int tot;
            const int k = wave_compact(need, &tot);
            if (need) {
                const DevPlane &P = st.pl[s][0];
                st.req[k]        = P.base + (ptrdiff_t)oy * P.stride + ox;
                st.req_stride[k] = 2 * P.stride;
                st.req_slot[k]   = (int8_t)s;
            }
            if (lane == 0)
                st.nreq = tot;
        }
        __syncthreads();
        nxm_requests(st, st.req, st.req_stride, st.nreq, (int)(bh >> 1), (int)bw);
        __syncthreads();
        if (w0) {
            uint32_t zz = U32MAX;
            int s = -1;
            if (lane < st.nreq) {
                s  = st.req_slot[lane];
                zz = (st.nxm[lane] << 1);
                zz = (zz * 64 * 64) / (bw * bh);
                st.zz[s] = zz;
            }
            const uint32_t best = wave_min_u32(zz);
            if (s >= 0 && (s & 3) > 0) {
                if (job.temporal_layer_index > 0 && best < c.zz_sad_th &&
                    (uint32_t)((zz - best) * 100u) > (uint32_t)(c.zz_sad_pct * best))
                    st.do_ref[s] = 0;
            }
            if (c.me_safe_limit_zz_th) {
                const bool safe = job.hierarchical_levels > 0 && nl == 2 &&
                    job.temporal_layer_index >= job.hierarchical_levels && job.similar_brightness_refs &&
                    st.zz[0] < c.me_safe_limit_zz_th && st.zz[4] < c.me_safe_limit_zz_th;
                if (safe && lane < 8 && slot_valid(vmask, lane) && (lane & 3) > 0)
                    st.do_ref[lane] = 0;
            }
        }
        __syncthreads();
    }
    STAMP(2);

    // ---- pre-HME (motion_estimation.c:1693-1796)
    if (c.prehme_enable) {
        const int16_t sox = i16(((int16_t)ox) >> 2), soy = i16(((int16_t)oy) >> 2);
        for (int pass = 0; pass < nl; pass++) {
            if (w0) {
                // lane = ref * 2 + region
                const int r = lane >> 1, sr = lane & 1, l = pass, s = l * 4 + r;
                bool mk = false;
                TaskArgs ta;
                if (lane < 8 && slot_valid(vmask, s) && tl_or_l0(job, l)) {
                    PreHme &d = st.ph[s][sr];
                    const uint32_t f = scaled_dist(st.dist[s]);
                    bool done = false;
                    if (c.me_early_exit_th && st.zz[s] < c.me_early_exit_th) { // check_prehme_early_exit
                        d.col = d.row = 0;
                        d.sad = 0;
                        d.valid = 1;
                        done = true;
                    }
                    if (!done && c.prehme_l1_early_exit && l == 1) {
                        const PreHme &z = st.ph[r][sr];
                        if (z.valid && ((z.sad < (32 * 32)) || ((absi(z.col) < 16) && (absi(z.row) < 16)))) {
                            d.col = (int16_t)-z.col;
                            d.row = (int16_t)-z.row;
                            d.sad = z.sad;
                            d.valid = 1;
                            done = true;
                        }
                    }
                    if (!done && !st.do_ref[s]) {
                        d.col = d.row = 0;
                        d.sad = U32MAX;
                        done = true;
                    }
                    if (!done) {
                        d.sa_w = (uint16_t)min((uint32_t)c.prehme_sa_cfg[sr].sa_min.width * f,
                                               (uint32_t)c.prehme_sa_cfg[sr].sa_max.width);
                        d.sa_h = (uint16_t)min((uint32_t)c.prehme_sa_cfg[sr].sa_min.height * f,
                                               (uint32_t)c.prehme_sa_cfg[sr].sa_max.height);
                        const DevPlane &P = st.pl[s][2];
                        int16_t xo, yo, sw, sh2;
                        prehme_area(P, sox, soy, (int16_t)d.sa_w, (int16_t)d.sa_h, &xo, &yo, &sw, &sh2);
                        st.qox[s][sr] = xo;
                        st.qoy[s][sr] = yo;
                        ta = TaskArgs{P.base, P.stride, sox + xo, soy + yo, sw, sh2, (int)(bw >> 2),
                                  hsub ? (int)(bh >> 2) >> 1 : (int)(bh >> 2), hsub, c.prehme_skip_search_line,
                                  5120, hsub ? 32 : 16, s * 2 + sr};
                        d.performed = 1;
                        mk = true;
                    }
                }
                int tot;
                const int k = wave_compact(mk, &tot);
                if (mk)
                    make_task(st.tasks[k], ta);
                plan_windows(st, st.tasks, mk, k, tot, ARENA_BYTES);
                if (lane == 0)
                    st.ntasks = tot;
            }
            __syncthreads();
            search_tasks(st);
            if (w0 && lane < st.ntasks) {
                const int own = st.tasks[lane].owner, s = own >> 1, sr = own & 1;
                PreHme &d = st.ph[s][sr];
                uint64_t best;
                task_result(st, lane, &best, &d.col, &d.row);
                d.sad = hsub ? best * 2 : best;
                d.col = i16((d.col + st.qox[s][sr]) * 4);
                d.row = i16((d.row + st.qoy[s][sr]) * 4);
                d.valid = 1;
            }
            __syncthreads();
        }
        if (w0) {
            uint32_t m = U32MAX;
            const int s = lane;
            if (s < 8 && slot_valid(vmask, s)) {
                if (tl_or_l0(job, s >> 2)) {
                    m = (uint32_t)min_u64(st.ph[s][0].sad, st.ph[s][1].sad);
                } else { // list 1 at the base layer mirrors list 0
                    for (int k = 0; k < 2; k++) {
                        st.ph[s][k].col = (int16_t)-st.ph[s & 3][k].col;
                        st.ph[s][k].row = (int16_t)-st.ph[s & 3][k].row;
                        st.ph[s][k].sad = st.ph[s & 3][k].sad;
                    }
                }
            }
            const uint32_t best = wave_min_u32(m);
            if (job.temporal_layer_index > 0 && best < c.phme_sad_th && s < 8 && slot_valid(vmask, s) && (s & 3) > 0 &&
                st.do_ref[s]) {
                if ((uint32_t)((m - best) * 100u) > (uint32_t)(c.phme_sad_pct * best))
                    st.do_ref[s] = 0;
            }
        }
        __syncthreads();
    }
    STAMP(3);

    // ---- HME levels (motion_estimation.c:1906-2177)
    if (c.enable_hme_flag) {
        for (int level = 0; level < 3; level++) {
            if (level == 0 && !c.enable_hme_level0_flag)
                continue;
            if (level == 1 && !c.enable_hme_level1_flag)
                continue;
            if (level == 2 && !c.enable_hme_level2_flag)
                continue;
            // L0 with reduce_hme_l0_sr_th_*: other refs read ref (0,0)'s result -> two rounds
            const int rounds = (level == 0 && c.enable_me_sr_adjustment && c.distance_based_hme_resizing &&
                                c.reduce_hme_l0_sr_th_min && c.reduce_hme_l0_sr_th_max)
                ? 2
                : 1;
            for (int round = 0; round < rounds; round++) {
                if (w0) {
                    const int s = lane >> 2, q = lane & 3, sx = q >> 1, sy = q & 1;
                    const int l = s >> 2, r = s & 3;
                    bool mk = false;
                    TaskArgs ta;
                    if (lane < 32 && slot_valid(vmask, s) && (rounds == 1 || ((s == 0) == (round == 0)))) {
                        int16_t &X = st.lx[level][s][q], &Y = st.ly[level][s][q];
                        uint64_t &SD = st.lsad[level][s][q];
                        if (level == 0) {
                            bool done = false;
                            if (c.me_early_exit_th && st.zz[s] < (c.me_early_exit_th >> 2)) {
                                X = Y = 0;
                                SD = 0;
                                done = true;
                            }
                            if (!done && c.prev_me_stage_based_exit_th) {
                                const int k = st.ph[s][0].sad <= st.ph[s][1].sad ? 0 : 1;
                                if (st.ph[s][k].performed && st.ph[s][k].sad < (c.prev_me_stage_based_exit_th >> 4)) {
                                    X = st.ph[s][k].col;
                                    Y = st.ph[s][k].row;
                                    SD = st.ph[s][k].sad;
                                    done = true;
                                }
                            }
                            if (!done && !st.do_ref[s]) {
                                X = Y = 0;
                                SD = U32MAX;
                                done = true;
                            }
                            if (!done && tl_or_l0(job, l)) {
                                int16_t sa_w, sa_h;
                                hme_l0_area(c, l, r, st.dist[s], st.lx[0][0][0], st.ly[0][0][0], &sa_w,
                                            &sa_h);
                                const DevPlane &P = st.pl[s][2];
                                const int16_t sox = i16(((int16_t)ox) >> 2), soy = i16(((int16_t)oy) >> 2);
                                int16_t xo, yo, sw, sh2;
                                hme_l0_rect(c, P, sox, soy, sa_w, sa_h, sx, sy, &xo, &yo, &sw, &sh2);
                                st.qox[s][q] = xo;
                                st.qoy[s][q] = yo;
                                ta = TaskArgs{P.base, P.stride, sox + xo, soy + yo, sw, sh2, (int)(bw >> 2),
                                          hsub ? (int)(bh >> 2) >> 1 : (int)(bh >> 2), hsub, false, 5120,
                                          hsub ? 32 : 16, lane};
                                mk = true;
                            }
                        } else if (tl_or_l0(job, l)) {
                            bool done = false;
                            if (level == 1) {
                                if (c.me_early_exit_th && st.zz[s] < (c.me_early_exit_th >> 2)) {
                                    X = Y = 0;
                                    SD = 0;
                                    done = true;
                                }
                                if (!done && !st.do_ref[s]) {
                                    X = Y = 0;
                                    SD = U32MAX;
                                    done = true;
                                }
                                if (!done && c.prev_me_stage_based_exit_th &&
                                    st.lsad[0][s][q] < (c.prev_me_stage_based_exit_th >> 5)) {
                                    X = st.lx[0][s][q];
                                    Y = st.ly[0][s][q];
                                    SD = st.lsad[0][s][q];
                                    done = true;
                                }
                            } else {
                                if (c.prev_me_stage_based_exit_th &&
                                    st.lsad[1][s][q] < (c.prev_me_stage_based_exit_th >> 2)) {
                                    X = st.lx[1][s][q];
                                    Y = st.ly[1][s][q];
                                    SD = st.lsad[1][s][q];
                                    done = true;
                                }
                            }
                            if (!done) {
                                const DevPlane &P = st.pl[s][level == 1 ? 1 : 0];
                                const int16_t cx = level == 1 ? i16(st.lx[0][s][q] >> 1) : st.lx[1][s][q];
                                const int16_t cy = level == 1 ? i16(st.ly[0][s][q] >> 1) : st.ly[1][s][q];
                                const int16_t qx = level == 1 ? i16(((int16_t)ox) >> 1) : (int16_t)ox;
                                const int16_t qy = level == 1 ? i16(((int16_t)oy) >> 1) : (int16_t)oy;
                                const svtme_area sa = level == 1 ? c.hme_l1_sa : c.hme_l2_sa;
                                int16_t xo, yo, sw, sh2;
                                hme_refine_rect(level, P, qx, qy, (int16_t)sa.width, (int16_t)sa.height, cx, cy, &xo,
                                                &yo, &sw, &sh2);
                                st.qox[s][q] = xo;
                                st.qoy[s][q] = yo;
                                const int bwl = level == 1 ? (int)(bw >> 1) : (int)bw;
                                const int bhl = level == 1 ? (int)(bh >> 1) : (int)bh;
                                ta = TaskArgs{P.base, P.stride, qx + xo, qy + yo, sw, sh2, bwl, hsub ? bhl >> 1 : bhl, hsub, false,
                                          level == 1 ? 4096 : 0, (level == 1 ? 32 : 64) * (hsub ? 2 : 1), lane};
                                mk = true;
                            }
                        }
                    }
                    int tot;
                    const int k = wave_compact(mk, &tot);
                    if (mk)
                        make_task(st.tasks[k], ta);
                    plan_windows(st, st.tasks, mk, k, tot, ARENA_BYTES);
                    if (lane == 0)
                        st.ntasks = tot;
                }
                __syncthreads();
                search_tasks(st);
                if (w0 && lane < st.ntasks) {
                    const int own = st.tasks[lane].owner, s = own >> 2, q = own & 3;
                    int16_t &X = st.lx[level][s][q], &Y = st.ly[level][s][q];
                    uint64_t best;
                    task_result(st, lane, &best, &X, &Y);
                    st.lsad[level][s][q] = hsub ? best * 2 : best;
                    const int mul = level == 0 ? 4 : (level == 1 ? 2 : 1);
                    X = i16((X + st.qox[s][q]) * mul);
                    Y = i16((Y + st.qoy[s][q]) * mul);
                }
                __syncthreads();
                // pre-HME replaces the worst L0 quadrant of each searched slot (motion_estimation.c:2005-2032)
                if (level == 0 && c.prehme_enable) {
                    const int s = lane;
                    if (w0 && s < 8 && slot_valid(vmask, s) && (rounds == 1 || ((s == 0) == (round == 0)))) {
                        bool searched = tl_or_l0(job, s >> 2) && st.do_ref[s] &&
                            !(c.me_early_exit_th && st.zz[s] < (c.me_early_exit_th >> 2));
                        const int k = st.ph[s][0].sad <= st.ph[s][1].sad ? 0 : 1;
                        if (searched && c.prev_me_stage_based_exit_th && st.ph[s][k].performed &&
                            st.ph[s][k].sad < (c.prev_me_stage_based_exit_th >> 4))
                            searched = false;
                        if (searched) {
                            uint64_t *S = st.lsad[0][s];
                            int wq      = 0; // get_worst_quadrant: strict > in (0,0),(1,0),(0,1),(1,1) order
                            uint64_t mx = 0;
                            if (S[0] > mx) { mx = S[0]; wq = 0; }
                            if (S[2] > mx) { mx = S[2]; wq = 2; }
                            if (S[1] > mx) { mx = S[1]; wq = 1; }
                            if (S[3] > mx) { wq = 3; }
                            if (st.ph[s][k].sad < S[wq]) {
                                S[wq]           = st.ph[s][k].sad;
                                st.lx[0][s][wq] = st.ph[s][k].col;
                                st.ly[0][s][wq] = st.ph[s][k].row;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
        }
    }
    STAMP(4);

    // ---- set_final_seach_centre_sb (motion_estimation.c:2182-2380) + hme_prune_ref_and_adjust_sr (:2477-2518)
    if (w0) {
        const int s = lane;
        const bool valid = s < 8 && slot_valid(vmask, s);
        // per-slot pick at the highest enabled level; `own` = this slot defines the carried values
        int lvl = -1;
        if (c.enable_hme_level0_flag && !c.enable_hme_level1_flag && !c.enable_hme_level2_flag)
            lvl = 0;
        if (c.enable_hme_level1_flag && !c.enable_hme_level2_flag)
            lvl = 1;
        if (c.enable_hme_level2_flag)
            lvl = 2;
        const bool hme_slot = valid && tl_or_l0(job, s >> 2) && c.enable_hme_flag;
        int16_t hx = 0, hy = 0;
        uint64_t hs = 0;
        const bool own = hme_slot && lvl >= 0;
        if (own) {
            const int16_t *X = st.lx[lvl][s], *Y = st.ly[lvl][s];
            const uint64_t *S = st.lsad[lvl][s];
            hx = X[0], hy = Y[0], hs = S[0];
            // scan order (w, h): (1,0), (0,1), (1,1) = q 2, 1, 3
            if (S[2] < hs) { hx = X[2]; hy = Y[2]; hs = S[2]; }
            if (S[1] < hs) { hx = X[1]; hy = Y[1]; hs = S[1]; }
            if (S[3] < hs) { hx = X[3]; hy = Y[3]; hs = S[3]; }
        }
        // sequential carry over slots in reference order (function-scope variables in the reference)
        int16_t cx = 0, cy = 0, scx = 0, scy = 0;
        uint64_t cs = 0;
        int16_t my_scx = 0, my_scy = 0;
        uint64_t my_hs = 0;
        for (int k = 0; k < 8; k++) {
            const bool vk = __shfl((int)valid, k, 64) != 0;
            if (!vk)
                continue;
            const bool ok = __shfl((int)own, k, 64) != 0;
            const bool hk = __shfl((int)hme_slot, k, 64) != 0;
            const bool tk = __shfl((int)tl_or_l0(job, k >> 2), k, 64) != 0;
            const int16_t kx = (int16_t)__shfl((int)hx, k, 64), ky = (int16_t)__shfl((int)hy, k, 64);
            const uint64_t ks = __shfl(hs, k, 64);
            if (ok) {
                cx = kx, cy = ky, cs = ks;
            }
            if (tk) {
                if (hk) {
                    scx = cx;
                    scy = cy;
                }
            } else {
                scx = 0;
                scy = 0;
            }
            if (lane == k) {
                my_scx = scx, my_scy = scy, my_hs = cs;
            }
        }
        if (valid) {
            st.sc_x[s] = my_scx;
            st.sc_y[s] = my_scy;
            st.hme_sad[s] = my_hs;
        }
        if (c.enable_hme_flag) { // prune_ref = enable_hme_flag && me_type != ME_MCTF
            const uint64_t hsad = s < 8 ? st.hme_sad[s] : ~0ull;
            const uint16_t th = c.prune_ref_if_hme_sad_dev_bigger_than_th;
            if (c.enable_me_hme_ref_pruning && th != (uint16_t)~0) {
                const uint64_t best = wave_min_u64(hsad);
                if (s < 8 && (s & 3) >= 1 && (hsad - best) * 100 > (th * best))
                    st.do_ref[s] = 0;
            }
            if (c.enable_me_sr_adjustment && s < 8) {
                if (absi(st.sc_x[s]) <= c.reduce_me_sr_based_on_mv_length_th &&
                    absi(st.sc_y[s]) <= c.reduce_me_sr_based_on_mv_length_th && hsad < c.stationary_hme_sad_abs_th)
                    st.reduce_div[s] = c.stationary_me_sr_divisor;
                else if (hsad < c.reduce_me_sr_based_on_hme_sad_abs_th)
                    st.reduce_div[s] = c.me_sr_divisor_for_low_hme_sad;
            }
        }
        if (s < 8)
            st.searched[s] = st.do_ref[s];
    }
    __syncthreads();
    STAMP(5);

    // ---- integer_search_b64 (motion_estimation.c:1249-1516); lane s of wave 0 owns slot s.
    // Two rounds when enable_me_sr_adjustment == 2: the other slots read slot 0's 64x64 SAD.
    {
        const int rounds = c.enable_me_sr_adjustment == 2 ? 2 : 1;
        for (int round = 0; round < rounds; round++) {
            // step 1: search area up to the 8x8-variance decision
            if (w0) {
                const int s = lane, l = s >> 2, r = s & 3;
                const bool act = s < 8 && slot_valid(vmask, s) && (rounds == 1 || ((s == 0) == (round == 0))) &&
                    st.do_ref[s];
                bool need = false;
                if (act) {
                    int16_t xc = st.sc_x[s], yc = st.sc_y[s];
                    int16_t w = (int16_t)c.me_sa.sa_min.width, h = (int16_t)c.me_sa.sa_min.height;
                    const uint16_t dist = scaled_dist(st.dist[s]);
                    w = i16(min((int)(w * dist), (int)c.me_sa.sa_max.width));
                    h = i16(min((int)(h * dist), (int)c.me_sa.sa_max.height));
                    if (c.mv_sa_adj_enabled && (!c.mv_sa_adj_nearest_ref_only || r == 0)) {
                        if (absi(xc) > c.mv_sa_adj_mv_size_th)
                            w = i16(w * c.mv_sa_adj_sa_multiplier);
                        if (absi(yc) > c.mv_sa_adj_mv_size_th)
                            h = i16(h * c.mv_sa_adj_sa_multiplier);
                    }
                    w = i16((max(1u, ((uint32_t)(int32_t)w / st.reduce_div[s])) + 7) & ~0x07u);
                    h = i16(max(3u, ((uint32_t)(int32_t)h / st.reduce_div[s])));
                    st.is_wb[s]       = w;
                    st.is_hb[s]       = h;
                    st.is_best_hme[s] = ~0ull;
                    if (c.me_early_exit_th) {
                        if (st.zz[s] < (c.me_early_exit_th / 6)) {
                            w = 1;
                            h = 1;
                        }
                    } else if ((xc != 0 || yc != 0) && job.is_ref) {
                        need = true; // check_00_center (motion_estimation.c:1139-1206): clamp the centre
                        const DevPlane &P = st.pl[s][0];
                        const int16_t pad = 63, org_x = (int16_t)ox, org_y = (int16_t)oy;
                        const int16_t pw = i16(P.width), ph = i16(P.height);
                        xc = ((org_x + xc) < -pad) ? i16(-pad - org_x) : xc;
                        xc = ((org_x + xc) > pw - 1) ? i16(xc - ((org_x + xc) - (pw - 1))) : xc;
                        yc = ((org_y + yc) < -pad) ? i16(-pad - org_y) : yc;
                        yc = ((org_y + yc) > ph - 1) ? i16(yc - ((org_y + yc) - (ph - 1))) : yc;
                    }
                    st.is_w[s]  = w;
                    st.is_h[s]  = h;
                    st.is_xc[s] = xc;
                    st.is_yc[s] = yc;
                }
                if (s < 8)
                    st.in_round[s] = act;
                int tot;
                const int k = wave_compact(need, &tot);
                if (need) { // requests [2k] = (0,0), [2k+1] = clamped centre
                    const DevPlane &P = st.pl[s][0];
                    st.req[2 * k]     = P.base + (ptrdiff_t)oy * P.stride + ox;
                    st.req[2 * k + 1] = P.base + (ptrdiff_t)((int)oy + st.is_yc[s]) * P.stride + ((int)ox + st.is_xc[s]);
                    st.req_stride[2 * k] = st.req_stride[2 * k + 1] = 2 * P.stride;
                    st.req_slot[k] = (int8_t)s;
                }
                if (lane == 0)
                    st.nreq = tot;
            }
            __syncthreads();
            if (st.nreq) {
                nxm_requests(st, st.req, st.req_stride, 2 * st.nreq, (int)(bh >> 1), (int)bw);
                __syncthreads();
                if (w0 && lane < st.nreq) {
                    const int s = st.req_slot[lane];
                    const uint32_t zero_sad = st.nxm[2 * lane] << 1, hme_mv_sad = st.nxm[2 * lane + 1] << 1;
                    const uint64_t zc = (uint64_t)zero_sad << 8, hc = (uint64_t)hme_mv_sad << 8;
                    if (min_u64(zc, hc) == zc) {
                        st.is_xc[s] = 0;
                        st.is_yc[s] = 0;
                    }
                    st.is_best_hme[s] = hme_mv_sad;
                }
            }
            // step 2: sr adjustment level 2, 8x8-variance centre probe setup
            if (w0) {
                const int s = lane, l = s >> 2, r = s & 3;
                const bool act = s < 8 && st.in_round[s];
                bool probe = false;
                if (act) {
                    int16_t w = st.is_w[s], h = st.is_h[s];
                    if (!c.me_early_exit_th) {
                        const int16_t xc0 = st.sc_x[s], yc0 = st.sc_y[s];
                        uint8_t accurate  = 1;
                        if ((xc0 != 0 || yc0 != 0) && job.is_ref && st.is_xc[s] == 0 && st.is_yc[s] == 0)
                            accurate = 0;
                        if (c.enable_me_sr_adjustment == 2) {
                            if ((accurate && (st.is_best_hme[s] < (24 * 24))) ||
                                (job.is_ref && st.hme_sad[s] < (24 * 24)))
                                h = i16(h / 2);
                            if ((l || r) && st.best_sad[0][0] < 5000 && h == st.is_hb[s] && w == st.is_wb[s]) {
                                h = i16(h >> 1);
                                w = i16(w >> 1);
                            }
                        }
                    }
                    st.is_w[s] = w;
                    st.is_h[s] = h;
                    probe      = c.me_8x8_var_enabled && (w * h > 24);
                }
                int tot;
                const int k = wave_compact(probe, &tot);
                if (probe)
                    make_fp(st.fp[k], st.pl[s][0], ox, oy, s, st.is_xc[s], st.is_yc[s], 1, 1, 0, false);
                plan_windows(st, st.fp, probe, k, tot, FP_ARENA);
                if (lane == 0) {
                    st.nfp  = tot;
                    st.flag = 1; // a single position: 32-bit keys
                }
            }
            __syncthreads();
            for (int e = tid; e < 8 * SVTME_PU_COUNT; e += T2) {
                const int s = e / SVTME_PU_COUNT;
                if (st.in_round[s])
                    (&st.best_sad[0][0])[e] = SVTME_MAX_SAD_VALUE;
            }
            STAMP(6);
            if (st.nfp) {
                fullpel<SUB_ME>(st); // centre probe (motion_estimation.c:1414-1417)
                // 8x8-variance resize (motion_estimation.c:1418-1438)
                if (w0 && lane < 8 && st.in_round[lane] && c.me_8x8_var_enabled && (st.is_w[lane] * st.is_h[lane] > 24)) {
                    const int s = lane;
                    int16_t w = st.is_w[s], h = st.is_h[s];
                    const uint32_t mean = st.best_sad[s][0] / 64;
                    uint32_t sum_sq     = 0;
                    for (int i = 0; i < 64; i++) {
                        const int32_t diff = (int32_t)st.best_sad[s][21 + i] - (int32_t)mean;
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
                    st.is_w[s] = w;
                    st.is_h[s] = h;
                }
            }
            STAMP(7);
            // step 3: final area clamp + main full-pel search (motion_estimation.c:1440-1516)
            if (w0) {
                const int s = lane, l = s >> 2, r = s & 3;
                const bool act = s < 8 && st.in_round[s];
                int16_t w = 0, h = 0, xo = 0, yo = 0;
                if (act) {
                    w = st.is_w[s], h = st.is_h[s];
                    const int16_t xc = st.is_xc[s], yc = st.is_yc[s];
                    const int16_t pad = 63, org_x = (int16_t)ox, org_y = (int16_t)oy;
                    const int16_t pic_w = (int16_t)job.width, pic_h = (int16_t)job.height;
                    xo = i16(xc - (w >> 1));
                    yo = i16(yc - (h >> 1));
                    xo = ((org_x + xo) < -pad) ? i16(-pad - org_x) : xo;
                    w  = ((org_x + xo) < -pad) ? i16(w - (-pad - (org_x + xo))) : w;
                    xo = ((org_x + xo) > pic_w - 1) ? i16(xo - ((org_x + xo) - (pic_w - 1))) : xo;
                    w  = ((org_x + xo + w) > pic_w) ? i16(max(1, w - ((org_x + xo + w) - pic_w))) : w;
                    w  = (w < 8) ? w : i16(w & ~0x07);
                    yo = ((org_y + yo) < -pad) ? i16(-pad - org_y) : yo;
                    h  = ((org_y + yo) < -pad) ? i16(h - (-pad - (org_y + yo))) : h;
                    yo = ((org_y + yo) > pic_h - 1) ? i16(yo - ((org_y + yo) - (pic_h - 1))) : yo;
                    h  = (org_y + yo + h > pic_h) ? i16(max(1, h - ((org_y + yo + h) - pic_h))) : h;
                }
                int tot;
                const int k = wave_compact(act, &tot);
                if (act)
                    make_fp(st.fp[k], st.pl[s][0], ox, oy, s, xo, yo, w, h, 1, true);
                plan_windows(st, st.fp, act, k, tot, FP_ARENA);
                const bool k32 = __all(!act || (1 + (int)w * (int)h <= 4096));
                if (lane == 0) {
                    st.nfp  = tot;
                    st.flag = k32;
                }
            }
            __syncthreads();
            STAMP(8);
            if (st.nfp)
                fullpel<SUB_ME>(st);
        }
    }

    // ---- me_prune_ref (motion_estimation.c:1522-1565)
    if (c.enable_hme_flag && c.enable_me_hme_ref_pruning && w0) {
        const int s = lane;
        uint64_t v = ~0ull;
        if (s < 8) {
            v = st.hme_sad[s];
            if (slot_valid(vmask, s)) {
                if (!st.do_ref[s])
                    v = (uint64_t)SVTME_MAX_SAD_VALUE * 64;
                else {
                    uint64_t sum = 0;
                    for (int i = 0; i < 64; i++) sum += st.best_sad[s][21 + i];
                    v = sum;
                }
                st.hme_sad[s] = v;
            }
        }
        const uint16_t th = c.prune_ref_if_me_sad_dev_bigger_than_th;
        if (th != (uint16_t)~0) {
            const uint64_t best = wave_min_u64(v);
            if (s < 8 && (s & 3) >= 1 && (v - best) * 100 > (th * best))
                st.do_ref[s] = 0;
        }
    }
    __syncthreads();
    STAMP(9);

    // ---- records (sb_count x R, slots in list-0-then-list-1 order)
    {
        svtme_ref_record *out = dj.out_records + (size_t)sb_local * dj.R;
        const int R = (int)dj.R;
        for (int k = 0; k < R; k++) { // 704 bytes = 176 dwords per record
            const int s = k < job.num_refs[0] ? k : 4 + (k - job.num_refs[0]);
            const int w = tid;
            if (w >= 176)
                continue;
            uint32_t v;
            if (w < 85)
                v = st.searched[s] ? st.best_sad[s][w] : U32MAX;
            else if (w < 170)
                v = st.best_mv[s][w - 85];
            else if (w == 170)
                v = (uint32_t)st.hme_sad[s];
            else if (w == 171)
                v = (uint32_t)(st.hme_sad[s] >> 32);
            else if (w == 172)
                v = (uint32_t)(uint16_t)st.sc_x[s] | ((uint32_t)(uint16_t)st.sc_y[s] << 16);
            else if (w == 173)
                v = st.zz[s];
            else if (w == 174)
                v = (uint32_t)st.searched[s] | ((uint32_t)st.do_ref[s] << 8);
            else
                v = 0;
            ((uint32_t *)(out + k))[w] = v;
        }
    }
    if (dj.out_sb) {
        __syncthreads();
        finish_sb(st, dj, sb_local, bw, bh);
    }
    STAMP(10);
}

} // namespace me2

extern "C" hipError_t svtme_launch_me2(const DevJob *dj, uint32_t sb_count, hipStream_t s) {
    if (dj->job.ctrl.me_search_method == SVTME_FULL_SAD_SEARCH)
        hipLaunchKernelGGL(me2::k_me_sb<false>, dim3(sb_count), dim3(T2), 0, s, *dj);
    else
        hipLaunchKernelGGL(me2::k_me_sb<true>, dim3(sb_count), dim3(T2), 0, s, *dj);
    return hipGetLastError();
}
