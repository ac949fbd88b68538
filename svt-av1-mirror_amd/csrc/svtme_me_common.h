// svtme_me_common.h — device helpers shared by the open-loop ME stage kernels
// (svtme_stages.hip): reference search-area derivations, wavefront
// reductions, SAD primitives and the candidate tables. gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svtme_device.h"

#define U32MAX 0xFFFFFFFFu

namespace svtme {

#define SVTME_HD __host__ __device__ __forceinline__
SVTME_HD int16_t i16(int v) { return (int16_t)v; }
SVTME_HD int absi(int v) { return v < 0 ? -v : v; }
SVTME_HD int imin(int a, int b) { return a < b ? a : b; }
SVTME_HD uint32_t min_u32(uint32_t a, uint32_t b) { return a < b ? a : b; }
SVTME_HD uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// motion_estimation.c:1239-1243
SVTME_HD uint16_t scaled_dist(uint16_t dist) {
    uint8_t round_up = ((dist % 8) == 0) ? 0 : 1;
    return (uint16_t)(((dist * 5) / 8) + round_up);
}
SVTME_HD uint16_t ref_dist_const(const svtme_job &j, int l, int r) {
    int64_t d = (int64_t)j.picture_number - (int64_t)j.ref_picture_number[l][r];
    return (uint16_t)(int16_t)(d < 0 ? -d : d);
}
// A wave-uniform byte / halfword field of a struct (a job) in global memory, read
// as the dword that holds it: a scalar load (gfx950 has no scalar sub-dword load,
// so the field itself would be a vector-memory round trip). SF(job, max_l0).
template <typename S, typename T>
__device__ __forceinline__ uint32_t sfld_(const S &obj, const T &f) {
    static_assert(sizeof(T) <= 2 && alignof(S) >= 4, "sfld_: a byte / halfword of a dword-aligned struct");
    const uint32_t off = (uint32_t)((const char *)&f - (const char *)&obj);
    const uint32_t v   = ((const uint32_t *)&obj)[off >> 2] >> (8 * (off & 3));
    return sizeof(T) == 1 ? (v & 0xFFu) : (v & 0xFFFFu);
}
#define SF(obj, field) ::svtme::sfld_((obj), (obj).field)
__device__ __forceinline__ bool tl_or_l0(const svtme_job &j, int l) { return j.temporal_layer_index > 0 || l == 0; }
__device__ __forceinline__ bool slot_valid(uint32_t vmask, int s) { return s >= 0 && s < 8 && ((vmask >> s) & 1u); }
__device__ __forceinline__ uint32_t valid_mask(const svtme_job &job) {
    uint32_t m = 0;
#pragma unroll
    for (int s = 0; s < 8; s++)
        if ((s >> 2) < job.num_lists && (s & 3) < job.num_refs[s >> 2])
            m |= 1u << s;
    return m;
}

// Wavefront reductions and scans with DPP (row_shr 1/2/4/8 inside each row of
// 16 lanes, then row_bcast 15/31 across rows): a handful of VALU ops instead of
// ds_bpermute round trips. Every lane of the wavefront must be active.
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143

template <int CTRL, int RM = 0xF>
__device__ __forceinline__ uint32_t dpp_or(uint32_t v, uint32_t id) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, RM, 0xF, false);
}
// inclusive prefix along lanes with op f and identity id; lane 63 ends with the total
template <typename F>
__device__ __forceinline__ uint32_t wave_scan32(uint32_t v, uint32_t id, F f) {
    v = f(v, dpp_or<DPP_ROW_SHR(1)>(v, id));
    v = f(v, dpp_or<DPP_ROW_SHR(2)>(v, id));
    v = f(v, dpp_or<DPP_ROW_SHR(4)>(v, id));
    v = f(v, dpp_or<DPP_ROW_SHR(8)>(v, id));
    v = f(v, dpp_or<DPP_ROW_BCAST15, 0xA>(v, id));
    v = f(v, dpp_or<DPP_ROW_BCAST31, 0xC>(v, id));
    return v;
}
__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    auto step = [&](uint32_t tl, uint32_t th) {
        const unsigned long long t = ((unsigned long long)th << 32) | tl;
        v                          = t < v ? t : v;
    };
#define WMIN64(CTRL, RM)                                                                                              \
    step(dpp_or<CTRL, RM>((uint32_t)v, U32MAX), dpp_or<CTRL, RM>((uint32_t)(v >> 32), U32MAX))
    WMIN64(DPP_ROW_SHR(1), 0xF);
    WMIN64(DPP_ROW_SHR(2), 0xF);
    WMIN64(DPP_ROW_SHR(4), 0xF);
    WMIN64(DPP_ROW_SHR(8), 0xF);
    WMIN64(DPP_ROW_BCAST15, 0xA);
    WMIN64(DPP_ROW_BCAST31, 0xC);
#undef WMIN64
    return ((unsigned long long)lane63((uint32_t)(v >> 32)) << 32) | lane63((uint32_t)v);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return lane63(wave_scan32(v, U32MAX, [](uint32_t a, uint32_t b) { return a < b ? a : b; }));
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return lane63(wave_scan32(v, 0u, [](uint32_t a, uint32_t b) { return a + b; }));
}
// rank of this lane among lanes with pred set (exclusive prefix count) and the total
__device__ __forceinline__ int wave_compact(bool pred, int *total) {
    const unsigned long long m = __ballot(pred);
    *total                     = __popcll(m);
    const int lane             = threadIdx.x & 63;
    const unsigned long long lt = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
    return __popcll(lt);
}

// wave-inclusive prefix sum over lanes (lane order)
__device__ __forceinline__ int wave_incl_scan(int v) {
    return (int)wave_scan32((uint32_t)v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}

// exact n / d for n * d < 2^32 with m = magic_u32(d); d == 1 wraps m to 0
__device__ __forceinline__ uint32_t magic_u32(uint32_t d) { return 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ int mdiv(int n, uint32_t m) { return m ? (int)__umulhi((uint32_t)n, m) : n; }

#define UNI(x) __builtin_amdgcn_readfirstlane((int)(x))
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}

// a pointer known to be wave-uniform, moved to SGPRs (enables base + 32-bit offset addressing)
template <typename T>
__device__ __forceinline__ T *uni_ptr(T *p) {
    const uint64_t v  = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T *)(uintptr_t)(((uint64_t)hi << 32) | lo);
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

// v + DPP-permuted v in one VALU op (quad_perm / row_ror / row_bcast)
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v) {
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}

// a + DPP-permuted b in one VALU op
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ uint32_t dpp_add2(uint32_t a, uint32_t b) {
    return a + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, CTRL, RM, 0xF, false);
}

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
SVTME_HD void hme_l0_area(const svtme_controls &c, int l, int r, uint16_t dist, int16_t l00x, int16_t l00y,
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
    w               = i16(imin((((w * f) + 15) & ~0x0F), (int)(((mxw / c.num_hme_sa_w) + 15) & ~0x0F)));
    int16_t h       = i16(mnh / c.num_hme_sa_h);
    h               = i16(imin((h * f), (int)(mxh / c.num_hme_sa_h)));
    *sa_w = w, *sa_h = h;
}

// ----------------------------------------------------------------------------
// Candidate tables (motion_estimation.c:2520-2531, definitions.h:2613-2632)
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

// c_z_to_raster[n] computed (a per-lane index into __constant__ memory is a vector
// memory load on the critical path): the 16x16 and 8x8 PUs in Z order are bit-
// interleaved (x, y) grid positions, row-major in raster order
__device__ __forceinline__ int z_to_raster(int n) {
    if (n < 5)
        return n;
    if (n < 21) {
        const int z = n - 5;
        return 5 + (((z >> 3) & 1) * 2 + ((z >> 1) & 1)) * 4 + ((z >> 2) & 1) * 2 + (z & 1);
    }
    const int z = n - 21;
    const int x = (z & 1) | ((z >> 1) & 2) | ((z >> 2) & 4);
    const int y = ((z >> 1) & 1) | ((z >> 2) & 2) | ((z >> 3) & 4);
    return 21 + y * 8 + x;
}

__device__ __forceinline__ uint8_t mk_cand(int dir, int r0, int r1, int l0, int l1) {
    return (uint8_t)((dir & 3) | ((r0 & 3) << 2) | ((r1 & 3) << 4) | ((l0 & 1) << 6) | ((l1 & 1) << 7));
}

} // namespace svtme
