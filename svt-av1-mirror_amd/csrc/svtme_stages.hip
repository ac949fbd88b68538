// svtme_stages.hip — open-loop motion estimation as three stage kernels (gfx950).
//
// svt_aom_motion_estimation_b64 (reference motion_estimation.c:3076-3153) runs
// per 64x64 superblock (SB) as a chain of dependent searches. On MI355X the
// chain is executed stage-major over the whole picture so every stage is a
// wide, high-occupancy launch and no workgroup idles on a dependency:
//
//   k_stage_a  one wavefront per independent search of every SB: zz SAD
//              (init_zz_sad), both pre-HME regions of every reference of both
//              lists, and the four HME level-0 quadrants. None of these
//              searches depends on another's result; whether the reference
//              would have skipped one is decided afterwards from the same
//              data (stage B), so skipped searches are simply not read.
//   k_stage_b  one workgroup per SB: the zz / pre-HME / level-0 decisions in
//              reference order, HME level 1 (and 2), search-centre selection
//              and HME pruning (set_final_seach_centre_sb,
//              hme_prune_ref_and_adjust_sr).
//   k_stage_c  one workgroup per SB: integer_search_b64 (check_00_center,
//              8x8-variance probe, full-pel search with the 85-PU argmin),
//              me_prune_ref, the per-reference records and the candidate
//              arrays / distortions / GM detection.
//
// SAD primitive: v_qsad_pk_u16_u8 gives the SADs of 4 consecutive positions
// for one source dword. Positions are grouped in quads aligned to the
// reference plane's dword grid, so every load is a plain aligned dword load
// and no byte realignment is ever needed; positions of a quad outside the
// search area are masked out of the argmin. Argmins use 64-bit keys
// (sad << 32 | y << 16 | x, or sad << 32 | raster order) so the reference's
// strict-< first-minimum scan order (compute_sad_c.c:90,
// motion_estimation.c:137-425) falls out of an integer min.
#include <hip/hip_ext.h>
#include <cstdlib>
#include <type_traits>

#include "svtme_me_common.h"

extern "C" bool svtme_hme_rt(const svtme_controls *c); // (host dispatch, end of file)

namespace svtme {


#define STAGE_A_BUF_DW 1024 // per-wave window buffers (dwords)
#define STAGE_B_BUF_DW 640

// ----------------------------------------------------------------------------
// Wavefront SAD searches (sad_loop, compute_sad_c.c:58-101)
// ----------------------------------------------------------------------------
// rows [k0, k1) of an ND-dword block row for the 4 positions of an aligned quad
template <int ND, typename P>
__device__ __forceinline__ void rows_qsad(P rp, int bstride_dw, const uint8_t *src, int src_stride,
                                          int k0, int k1, uint32_t acc[4]) {
    constexpr int CH = 64 / ND; // u16 lanes: ND * 1020 * CH <= 65280
    for (int kc = k0; kc < k1; kc += CH) {
        const int ke         = min(k1, kc + CH);
        unsigned long long a = 0;
#pragma unroll 2
        for (int k = kc; k < ke; k++) {
            const P rd         = rp + k * bstride_dw;
            const uint32_t *sd = (const uint32_t *)(src + k * src_stride);
            uint32_t d[ND + 1];
#pragma unroll
            for (int j = 0; j <= ND; j++) d[j] = rd[j];
#pragma unroll
            for (int j = 0; j < ND; j++) a = qsad(d[j], d[j + 1], sd[j], a);
        }
        qsad_unpack(a, acc);
    }
}

// any block width (partial last dword masked): v_sad_u8 on the 4 byte shifts
template <typename P>
__device__ __forceinline__ void rows_sad_any(P rp, int bstride_dw, const uint8_t *src, int src_stride,
                                             int bw, int k0, int k1, uint32_t acc[4]) {
    const int nd             = (bw + 3) >> 2;
    const uint32_t last_mask = (bw & 3) ? ((1u << (8 * (bw & 3))) - 1u) : 0xFFFFFFFFu;
    for (int k = k0; k < k1; k++) {
        const P rd        = rp + k * bstride_dw;
        const uint8_t *sb = src + k * src_stride;
        uint32_t d0        = rd[0];
        for (int j = 0; j < nd; j++) {
            const uint32_t d1 = rd[j + 1];
            const uint32_t m  = (j == nd - 1) ? last_mask : 0xFFFFFFFFu;
            const uint32_t s  = *(const uint32_t *)(sb + 4 * j) & m;
            acc[0] = __builtin_amdgcn_sad_u8(d0 & m, s, acc[0]);
            acc[1] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d1, d0, 1) & m, s, acc[1]);
            acc[2] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d1, d0, 2) & m, s, acc[2]);
            acc[3] = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d1, d0, 3) & m, s, acc[3]);
            d0 = d1;
        }
    }
}

// exact-division magics for small divisors (uniform table lookups)
struct MagicTab {
    uint32_t v[256];
};
constexpr MagicTab make_magic_tab() {
    MagicTab t{};
    for (uint32_t d = 1; d < 256; d++) t.v[d] = 0xFFFFFFFFu / d + 1u;
    return t;
}
__constant__ MagicTab c_magic = make_magic_tab();
__device__ __forceinline__ uint32_t magic_of(int d) { return d < 256 ? c_magic.v[d] : magic_u32((uint32_t)d); }

// block widths the SAD loops are specialised for (bit = dwords per row)
#define RW_2 (1 << 2)
#define RW_4 (1 << 4)
#define RW_8 (1 << 8)
#define RW_16 (1 << 16)

template <int ALLOW, typename P>
__device__ __forceinline__ void rows_dispatch(int mode, P rp, int kstride, const uint8_t *src, int src_stride, int bw,
                                              int k0, int k1, uint32_t acc[4]) {
    if ((ALLOW & RW_4) && mode == 4)
        rows_qsad<4>(rp, kstride, src, src_stride, k0, k1, acc);
    else if ((ALLOW & RW_8) && mode == 8)
        rows_qsad<8>(rp, kstride, src, src_stride, k0, k1, acc);
    else if ((ALLOW & RW_16) && mode == 16)
        rows_qsad<16>(rp, kstride, src, src_stride, k0, k1, acc);
    else if ((ALLOW & RW_2) && mode == 2)
        rows_qsad<2>(rp, kstride, src, src_stride, k0, k1, acc);
    else
        rows_sad_any(rp, kstride, src, src_stride, bw, k0, k1, acc);
}

// Wave-uniform geometry of one sad_loop (compute_sad_c.c:58-101): window
// top-left (plane coords) (wx, wy), search area sa_w x sa_h, block bw x bh_eff
// rows (sub: block rows 2 plane rows apart). Positions are grouped in quads
// aligned to the plane's dword grid; the staged window holds odd plane rows
// only for skip + sub, else every row.
struct SadGeo {
    const uint32_t *a0; // dword-aligned address of search row 0's first quad
    const uint32_t *g;  // first staged row
    int gs;             // dwords between staged rows in the plane
    int sdw, sh, nq, bw, bh, per, lg, nitems, mode, sa_w, skip, odd, ystep, wrows, wdw, pitch, staged, sub;
    uint32_t mnq;
};

__device__ __forceinline__ SadGeo sad_geo(const uint8_t *pbase, int pstride, int wx, int wy, int sa_w, int sa_h,
                                          int bw, int bh_eff, bool sub, bool skip_flag, int buf_dw) {
    SadGeo g;
    const bool skip = skip_flag && bw == 16 && bh_eff <= 16; // compute_sad_c.c:74
    const int nrows = (sa_w > 0 && sa_h > 0 && bh_eff > 0) ? (skip ? sa_h / 2 : sa_h) : 0;
    const uint8_t *w0 = pbase + (ptrdiff_t)wy * pstride + wx;
    g.sh     = (int)((uintptr_t)w0 & 3);
    g.a0     = (const uint32_t *)(w0 - g.sh);
    g.nq     = (g.sh + sa_w + 3) >> 2;
    g.bw     = bw;
    g.bh     = bh_eff;
    g.sdw    = pstride >> 2;
    g.sa_w   = sa_w;
    g.skip   = skip;
    g.sub    = sub;
    const int nd    = (bw + 3) >> 2;
    const int quads = nrows > 0 ? nrows * g.nq : 0;
    int lg = 0; // 2^lg lanes share a quad, splitting its block rows
    while ((2 << lg) <= bh_eff && quads * (2 << lg) <= 64) lg++;
    g.lg     = lg;
    g.per    = (bh_eff + (1 << lg) - 1) >> lg;
    g.nitems = quads << lg;
    g.mnq    = magic_of(g.nq > 0 ? g.nq : 1);
    g.mode   = (bw & 3) ? 0 : (bw == 16 ? 4 : (bw == 32 ? 8 : (bw == 64 ? 16 : (bw == 8 ? 2 : 0))));
    g.odd    = skip && sub;
    g.ystep  = g.odd ? 1 : (sub ? 2 : 1);
    const int last_y = skip ? 2 * nrows - 1 : nrows - 1;
    g.wrows  = nrows <= 0 ? 0 : (g.odd ? (nrows - 1) + bh_eff : last_y + (bh_eff - 1) * g.ystep + 1);
    g.wdw    = g.nq + nd;
    g.pitch  = g.wdw | 1;
    g.staged = g.wrows * g.pitch <= buf_dw;
    g.g      = g.a0 + (g.odd ? g.sdw : 0);
    g.gs     = g.odd ? 2 * g.sdw : g.sdw;
    return g;
}

// Wave copy of a window (wrows x wdw dwords from dword-aligned plane rows gs
// dwords apart) into LDS rows `pitch` dwords apart, general form (any width).
__device__ __forceinline__ void wave_stage_generic(uint32_t *buf, int pitch, const uint32_t *g, int gs, int wrows,
                                                   int wdw) {
    const int lane    = threadIdx.x & 63;
    const int n       = wrows * wdw;
    const uint32_t mw = magic_of(wdw);
    for (int base = 0; base < n; base += 512) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = base + u * 64 + lane;
            if (e < n) {
                const int r = mdiv(e, mw);
                v[u]        = g[(ptrdiff_t)r * gs + (e - r * wdw)];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = base + u * 64 + lane;
            if (e < n) {
                const int r                    = mdiv(e, mw);
                buf[r * pitch + (e - r * wdw)] = v[u];
            }
        }
    }
}

// A window to stage (wave-uniform). Windows up to 64 dwords wide are copied
// in passes of 8 row groups: lane -> (row in group, dword) once, rows clamped
// to the last row (duplicate copies are harmless), no per-element division.
struct Win {
    const uint32_t *g; // first row in the plane (dword aligned)
    uint32_t *dst;     // LDS
    int gs, wrows, wdw, pitch, rpi, passes;
};

__device__ __forceinline__ Win make_win(const uint32_t *g, int gs, int wrows, int wdw, int pitch, uint32_t *dst) {
    Win w;
    w.g = g, w.gs = gs, w.wrows = wrows, w.wdw = wdw, w.pitch = pitch, w.dst = dst;
    w.rpi    = wdw <= 64 ? mdiv(64, magic_of(wdw)) : 0;
    w.passes = w.rpi ? (wrows + 8 * w.rpi - 1) / (8 * w.rpi) : 0;
    return w;
}

__device__ __forceinline__ void win_lane(const Win &w, int *sub, int *d) {
    const int lane = threadIdx.x & 63;
    int s          = mdiv(lane, magic_of(w.wdw));
    *d             = lane - s * w.wdw;
    *sub           = s < w.rpi ? s : w.rpi - 1;
}

__device__ __forceinline__ void win_load(const Win &w, int pass, uint32_t v[8]) {
    int sub, d;
    win_lane(w, &sub, &d);
    const char *gb = (const char *)uni_ptr(w.g); // uniform base + 32-bit byte offsets
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int r = min((pass * 8 + u) * w.rpi + sub, w.wrows - 1);
        v[u]        = *(const uint32_t *)(gb + (uint32_t)(r * w.gs + d) * 4u);
    }
}

__device__ __forceinline__ void win_store(const Win &w, int pass, const uint32_t v[8]) {
    int sub, d;
    win_lane(w, &sub, &d);
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int r                 = min((pass * 8 + u) * w.rpi + sub, w.wrows - 1);
        w.dst[r * w.pitch + d]      = v[u];
    }
}

// Stage the windows k of w[] with bit k of `mask` set, every pass's loads of
// all windows in flight together (one memory round trip per pass). No fence
// (see wave_lds_fence).
template <int NW>
__device__ __forceinline__ void stage_windows(const Win (&w)[NW], uint32_t mask) {
    int maxp = 0;
#pragma unroll
    for (int k = 0; k < NW; k++)
        if ((mask >> k) & 1u) {
            if (w[k].rpi)
                maxp = max(maxp, w[k].passes);
            else
                wave_stage_generic(w[k].dst, w[k].pitch, w[k].g, w[k].gs, w[k].wrows, w[k].wdw);
        }
    for (int pass = 0; pass < maxp; pass++) {
        uint32_t v[NW][8];
#pragma unroll
        for (int k = 0; k < NW; k++)
            if (((mask >> k) & 1u) && w[k].rpi && pass < w[k].passes)
                win_load(w[k], pass, v[k]);
#pragma unroll
        for (int k = 0; k < NW; k++)
            if (((mask >> k) & 1u) && w[k].rpi && pass < w[k].passes)
                win_store(w[k], pass, v[k]);
    }
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ Win sad_win(const SadGeo &g, uint32_t *buf) {
    return make_win(g.g, g.gs, g.wrows, g.wdw, g.pitch, buf);
}
__device__ __forceinline__ bool sad_staged(const SadGeo &g) { return g.staged && g.nitems; }

// The search itself; returns the wave-uniform best key (sad << 32 | y << 16 | x),
// ~0 if nothing was searched.
template <int ALLOW>
__device__ __forceinline__ unsigned long long sad_compute(const SadGeo &g, const uint32_t *buf, const uint8_t *src,
                                                          int src_stride) {
    const int lane = threadIdx.x & 63;
    const int G    = 1 << g.lg;
    unsigned long long best = ~0ull;
    for (int base = 0; base < g.nitems; base += 64) {
        const int i  = base + lane;
        const int gi = i & (G - 1), qi = i >> g.lg;
        const int yy = mdiv(qi, g.mnq), q = qi - yy * g.nq;
        const int y  = g.skip ? 2 * yy + 1 : yy;
        uint32_t acc[4] = {0, 0, 0, 0};
        if (i < g.nitems) {
            const int k0 = min(g.bh, gi * g.per), k1 = min(g.bh, k0 + g.per);
            if (g.staged)
                rows_dispatch<ALLOW>(g.mode, buf + (g.odd ? yy : y) * g.pitch + q, g.ystep * g.pitch, src,
                                     src_stride, g.bw, k0, k1, acc);
            else
                rows_dispatch<ALLOW>(g.mode, g.a0 + (ptrdiff_t)y * g.sdw + q, g.sub ? 2 * g.sdw : g.sdw, src,
                                     src_stride, g.bw, k0, k1, acc);
        }
        for (int o = 1; o < G; o <<= 1)
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] += __shfl_xor(acc[k], o, 64);
        if (i < g.nitems && gi == 0) {
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int x = 4 * q - g.sh + s;
                if (x >= 0 && x < g.sa_w) {
                    const unsigned long long kk =
                        ((unsigned long long)acc[s] << 32) | ((uint32_t)y << 16) | (uint32_t)x;
                    best = kk < best ? kk : best;
                }
            }
        }
    }
    return wave_min_u64(best);
}

// sad_loop output: best_sad starts at 0xffffff; the centre stays (0,0) unless
// a position beats it (compute_sad_c.c:71, :90)
__device__ __forceinline__ void key_result(unsigned long long k, uint32_t *best, int *x, int *y) {
    const uint32_t sad = (uint32_t)(k >> 32);
    if (k != ~0ull && sad < 0xffffffu) {
        *best = sad;
        *x    = (int)(int16_t)(k & 0xFFFF);
        *y    = (int)(int16_t)((k >> 16) & 0xFFFF);
    } else {
        *best = 0xffffff;
        *x = *y = 0;
    }
}

// n x m SAD (compute_sad_c.c:20-37) of a width x rows block, by one wavefront;
// ref may be unaligned, cur is dword aligned
__device__ uint32_t wave_nxm(const uint8_t *ref, int rstride, const uint8_t *cur, int cstride, int rows, int width) {
    // an opaque lane index: the per-lane addresses below are not hoisted out of a
    // caller's loop (live across it, they spill at 64 VGPRs)
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const int wd4      = (width + 3) >> 2;
    const uint32_t mwd = magic_u32((uint32_t)wd4);
    const int sh       = (int)((uintptr_t)ref & 3);
    uint32_t acc       = 0;
    for (int e = lane; e < rows * wd4; e += 64) {
        const int r = mdiv(e, mwd), j = e - r * wd4;
        const uint32_t *da = (const uint32_t *)(ref + (ptrdiff_t)r * rstride - sh) + j;
        uint32_t run       = __builtin_amdgcn_alignbyte(da[1], da[0], sh);
        uint32_t s         = *((const uint32_t *)(cur + (ptrdiff_t)r * cstride) + j);
        const int valid    = width - 4 * j;
        if (valid < 4) {
            const uint32_t m = (1u << (8 * valid)) - 1u;
            run &= m;
            s &= m;
        }
        acc = __builtin_amdgcn_sad_u8(run, s, acc);
    }
    return wave_sum_u32(acc);
}

// SB geometry of a picture-local SB index
struct SbGeo {
    uint32_t ox, oy, bw, bh;
};
__device__ __forceinline__ SbGeo sb_geo(const DevJob &dj, uint32_t sb_local) {
    const uint32_t b64 = dj.job.sb_begin + sb_local;
    SbGeo g;
    g.ox = (b64 % dj.pic_w_b64) * 64;
    g.oy = (b64 / dj.pic_w_b64) * 64;
    g.bw = (dj.job.width - g.ox) < 64 ? dj.job.width - g.ox : 64;
    g.bh = (dj.job.height - g.oy) < 64 ? dj.job.height - g.oy : 64;
    return g;
}

// XCD-aware block order: blocks b and b + 8 share an XCD (round-robin
// dispatch), so each XCD gets one contiguous band of work whose reference
// windows overlap in its L2 (bijective for any grid size)
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
    const uint32_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// the job of work unit u of a batch launch, and u's index inside that job. The
// job table is read through the constant address space: it is written before
// the launch and never during it, so the compiler may keep its fields in SGPRs
// (scalar loads, hoisted and CSE'd across the kernel's own stores) exactly as
// it does for a by-value kernel argument.
typedef __attribute__((address_space(4))) const DevJob cjob_t;
__device__ __forceinline__ const DevJob &batch_job(const DevBatch &B, uint32_t u, uint32_t *local) {
    uint32_t j = 0, s0 = 0;
#pragma unroll
    for (int k = 1; k < SVTME_MAX_BATCH; k++)
        if (u >= B.start[k]) {
            j  = (uint32_t)k;
            s0 = B.start[k];
        }
    *local = u - s0;
    cjob_t *t = (cjob_t *)(uintptr_t)B.jobs;
    return *(const DevJob *)(t + UNI(j));
}

// per-slot reference planes into LDS with constant-index argument reads
template <int NLV>
__device__ __forceinline__ void copy_planes(const DevJob &dj, DevPlane (*pl)[NLV], uint16_t *dist) {
#pragma unroll
    for (int s = 0; s < 8; s++) {
#pragma unroll
        for (int v = 0; v < NLV; v++) pl[s][v] = dj.ref[s >> 2][s & 3].lv[v];
        dist[s] = ref_dist_const(dj.job, s >> 2, s & 3);
    }
}

// ----------------------------------------------------------------------------
// Stage A: every independent search of every SB, one wavefront each
// ----------------------------------------------------------------------------
// zz SAD of a full 64x64 SB (sub rows: 32 x 16 dwords), loads issued up front
struct ZzLoads {
    uint32_t r[8], c[8];
};
__device__ __forceinline__ void zz_issue(ZzLoads &z, const uint8_t *ref, int rstride, const uint8_t *cur, int cstride) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int e = u * 64 + lane, row = e >> 4, j = e & 15;
        z.r[u] = *((const uint32_t *)(ref + (ptrdiff_t)row * rstride) + j);
        z.c[u] = *((const uint32_t *)(cur + (ptrdiff_t)row * cstride) + j);
    }
}
__device__ __forceinline__ uint32_t zz_finish(const ZzLoads &z) {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) acc = __builtin_amdgcn_sad_u8(z.r[u], z.c[u], acc);
    return wave_sum_u32(acc);
}

// Stage A wave kinds (DevJob.ta_list entry = kind << 3 | slot)
#define TA_HME 0   // zz SAD + the four HME-L0 quadrants of one slot
#define TA_PH 1    // the two pre-HME regions of one slot
#define TA_ZZ 2    // zz SAD only (real-time tune, slots 1-7: their HME-L0 waits for slot 0's)
#define TA_L0RT 3  // the four HME-L0 quadrants with the area k_stage_d<true> left in BState

template <bool R1> // R1: the real-time tune's second round (DevJob.ta1_list)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_stage_a(const DevBatch B) {
    __shared__ __attribute__((aligned(16))) uint8_t srcb[4][256];
    __shared__ uint32_t wbuf[4][STAGE_A_BUF_DW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const uint32_t tac      = R1 ? dj.ta1_count : dj.ta_count;
    const uint32_t sb_local = UNI(gw / tac);
    const int entry         = UNI((R1 ? dj.ta1_list : dj.ta_list)[gw - sb_local * tac]);
    const int kind = entry >> 3, s = entry & 7, l = s >> 2, r = s & 3;
    const SbGeo G   = sb_geo(dj, sb_local);
    ARes *out       = dj.ares + (size_t)sb_local * SVTME_A_N;
    const bool hsub = c.hme_search_method != SVTME_FULL_SAD_SEARCH;
    const DevPlane &P   = dj.ref[l][r].lv[2];
    const uint16_t dist = ref_dist_const(job, l, r);
    uint32_t *buf       = wbuf[wid];

    // sixteenth-resolution source block (16 x 16): issued first, stored with the windows
    const DevPlane &S = dj.cur.lv[2];
    uint4 sv          = make_uint4(0, 0, 0, 0);
    if (lane < 16)
        sv = *(const uint4 *)(S.base + (ptrdiff_t)((G.oy >> 2) + lane) * S.stride + (G.ox >> 2));
    const int16_t sox = i16(((int16_t)G.ox) >> 2), soy = i16(((int16_t)G.oy) >> 2);
    const int bws = (int)(G.bw >> 2), bhs = hsub ? (int)(G.bh >> 2) >> 1 : (int)(G.bh >> 2);

    if (kind != TA_PH) {
        // real-time tune, second round: only the slots whose HME-L0 runs
        const BState *rb = dj.bst + sb_local;
        if (kind == TA_L0RT && !((rb->rt_need >> s) & 1u))
            return;
        // zz SAD (init_zz_sad, motion_estimation.c:2382-2437)
        const bool zz   = kind != TA_L0RT && (c.me_early_exit_th || c.me_safe_limit_zz_th);
        const bool zz64 = zz && G.bw == 64 && G.bh == 64;
        const DevPlane &F = dj.ref[l][r].lv[0];
        const DevPlane &C = dj.cur.lv[0];
        const uint8_t *zr = F.base + (ptrdiff_t)G.oy * F.stride + G.ox;
        const uint8_t *zc = C.base + (ptrdiff_t)G.oy * C.stride + G.ox;
        ZzLoads zl;
        if (zz64)
            zz_issue(zl, zr, 2 * F.stride, zc, 2 * C.stride);
        // the four HME-L0 quadrants (hme_level_0, motion_estimation.c:835-889), staged as one box
        const bool l0 = kind != TA_ZZ && c.enable_hme_flag && c.enable_hme_level0_flag;
        SadGeo gq[4];
        int16_t qxo[4], qyo[4];
        int boxl = 0x7fff, boxt = 0x7fff, wdwb = 0, wrowsb = 0;
        if (l0) {
            int16_t sa_w, sa_h;
            if (kind == TA_L0RT)
                sa_w = rb->rt_sa[s][0], sa_h = rb->rt_sa[s][1];
            else
                hme_l0_area(c, l, r, dist, 0, 0, &sa_w, &sa_h);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int16_t sw, shh;
                hme_l0_rect(c, P, sox, soy, sa_w, sa_h, q >> 1, q & 1, &qxo[q], &qyo[q], &sw, &shh);
                gq[q] = sad_geo(P.base, P.stride, sox + qxo[q], soy + qyo[q], sw, shh, bws, bhs, hsub, false,
                                0x7fffffff);
                if (gq[q].nitems) {
                    boxl = min(boxl, sox + qxo[q]);
                    boxt = min(boxt, soy + qyo[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (gq[q].nitems) {
                    const int dwo = ((sox + qxo[q]) >> 2) - (boxl >> 2), rwo = soy + qyo[q] - boxt;
                    wdwb   = max(wdwb, dwo + gq[q].wdw);
                    wrowsb = max(wrowsb, rwo + gq[q].wrows);
                }
        }
        const int pitchb  = wdwb | 1;
        const bool staged = l0 && wdwb > 0 && wrowsb * pitchb <= STAGE_A_BUF_DW;
        if (staged) {
            const Win w[1] = {make_win((const uint32_t *)(P.base + (ptrdiff_t)boxt * P.stride) + (boxl >> 2),
                                       P.stride >> 2, wrowsb, wdwb, pitchb, buf)};
            stage_windows<1>(w, 1u);
        }
        if (lane < 16)
            ((uint4 *)srcb[wid])[lane] = sv;
        wave_lds_fence();
        if (zz) {
            const uint32_t v = zz64 ? zz_finish(zl)
                                    : wave_nxm(zr, 2 * F.stride, zc, 2 * C.stride, (int)(G.bh >> 1), (int)G.bw);
            if (lane == 0)
                out[SVTME_A_ZZ + s] = ARes{v, 0, 0};
        }
        if (l0) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                SadGeo g         = gq[q];
                const uint32_t *o = buf;
                if (staged) {
                    g.staged = 1;
                    g.pitch  = pitchb;
                    o        = buf + (soy + qyo[q] - boxt) * pitchb + (((sox + qxo[q]) >> 2) - (boxl >> 2));
                } else {
                    g.staged = 0;
                }
                const unsigned long long k = sad_compute<RW_4>(g, o, srcb[wid], hsub ? 32 : 16);
                if (lane == 0) {
                    uint32_t best;
                    int x, y;
                    key_result(k, &best, &x, &y);
                    out[SVTME_A_L0 + s * 4 + q] =
                        ARes{hsub ? best * 2 : best, i16((x + qxo[q]) * 4), i16((y + qyo[q]) * 4)};
                }
            }
        }
        return;
    }
    // pre-HME: both regions (prehme_core, motion_estimation.c:1568-1636), staged together
    SadGeo gr[2];
    int16_t rxo[2], ryo[2];
    int off = 0;
    Win w[2];
    uint32_t mask = 0;
    const uint32_t f = scaled_dist(dist);
#pragma unroll
    for (int sr = 0; sr < 2; sr++) {
        const uint16_t sa_w = (uint16_t)min((uint32_t)c.prehme_sa_cfg[sr].sa_min.width * f,
                                            (uint32_t)c.prehme_sa_cfg[sr].sa_max.width);
        const uint16_t sa_h = (uint16_t)min((uint32_t)c.prehme_sa_cfg[sr].sa_min.height * f,
                                            (uint32_t)c.prehme_sa_cfg[sr].sa_max.height);
        int16_t sw, shh;
        prehme_area(P, sox, soy, (int16_t)sa_w, (int16_t)sa_h, &rxo[sr], &ryo[sr], &sw, &shh);
        gr[sr] = sad_geo(P.base, P.stride, sox + rxo[sr], soy + ryo[sr], sw, shh, bws, bhs, hsub,
                         c.prehme_skip_search_line, STAGE_A_BUF_DW - off);
        if (sad_staged(gr[sr])) {
            w[sr] = sad_win(gr[sr], buf + off);
            mask |= 1u << sr;
            off += gr[sr].wrows * gr[sr].pitch;
        }
    }
    stage_windows<2>(w, mask);
    if (lane < 16)
        ((uint4 *)srcb[wid])[lane] = sv;
    wave_lds_fence();
    off = 0;
#pragma unroll
    for (int sr = 0; sr < 2; sr++) {
        const unsigned long long k = sad_compute<RW_4>(gr[sr], buf + off, srcb[wid], hsub ? 32 : 16);
        if (sad_staged(gr[sr]))
            off += gr[sr].wrows * gr[sr].pitch;
        if (lane == 0) {
            uint32_t best;
            int x, y;
            key_result(k, &best, &x, &y);
            out[SVTME_A_PH + s * 2 + sr] =
                ARes{hsub ? best * 2 : best, i16((x + rxo[sr]) * 4), i16((y + ryo[sr]) * 4)};
        }
    }
}

// ----------------------------------------------------------------------------
// Stage D: the zz / pre-HME / level-0 decisions of stage A's results in the
// reference's order, one wavefront per SB (lane = slot, or slot x quadrant)
// ----------------------------------------------------------------------------
struct PreHme {
    uint64_t sad;
    int16_t col, row;
    uint8_t valid, performed;
    uint8_t pad[2];
};

struct Dec {
    ARes a[SVTME_A_N];
    uint32_t zz[8];
    uint8_t do_ref[8];
    PreHme ph[8][2];
    int16_t lx[8][4], ly[8][4]; // level 0, [slot][q = sx * 2 + sy]
    uint64_t lsad[8][4];
};

// init_me_hme_data (motion_estimation.c:3010-3070) of the decision state
__device__ __forceinline__ void dec_init(Dec &d) {
    const int lane = threadIdx.x & 63;
    if (lane < 8) {
        d.do_ref[lane] = 1;
        d.zz[lane]     = U32MAX;
        for (int k = 0; k < 2; k++) {
            d.ph[lane][k].valid     = 0;
            d.ph[lane][k].performed = 0;
            d.ph[lane][k].sad       = 0;
            d.ph[lane][k].col = d.ph[lane][k].row = 0;
        }
    }
    if (lane < 32) {
        (&d.lx[0][0])[lane]   = 0;
        (&d.ly[0][0])[lane]   = 0;
        (&d.lsad[0][0])[lane] = 0;
    }
    wave_lds_fence();
}

// init_zz_sad decisions (motion_estimation.c:2382-2437), one wavefront
__device__ __forceinline__ void dec_zz(Dec &d, const svtme_job &job, const SbGeo &G, uint32_t vmask) {
    const svtme_controls &c = job.ctrl;
    const int lane          = threadIdx.x & 63;
    const int nl            = job.num_lists;
    if (c.me_early_exit_th || c.me_safe_limit_zz_th) {
        const int s = lane;
        uint32_t zz = U32MAX;
        const bool have = slot_valid(vmask, s) && tl_or_l0(job, s >> 2);
        if (have) {
            zz      = d.a[SVTME_A_ZZ + s].sad << 1;
            const uint32_t pix = G.bw * G.bh; // (32-bit arithmetic as the reference's; a shift for a whole SB)
            zz                 = pix == 4096u ? (zz * 64 * 64) >> 12 : (zz * 64 * 64) / pix;
            d.zz[s] = zz;
        }
        const uint32_t best = wave_min_u32(zz);
        if (have && (s & 3) > 0 && job.temporal_layer_index > 0 && best < c.zz_sad_th &&
            (uint32_t)((zz - best) * 100u) > (uint32_t)(c.zz_sad_pct * best))
            d.do_ref[s] = 0;
        wave_lds_fence();
        if (c.me_safe_limit_zz_th) {
            const bool safe = job.hierarchical_levels > 0 && nl == 2 &&
                job.temporal_layer_index >= job.hierarchical_levels && job.similar_brightness_refs &&
                d.zz[0] < c.me_safe_limit_zz_th && d.zz[4] < c.me_safe_limit_zz_th;
            if (safe && slot_valid(vmask, lane) && (lane & 3) > 0)
                d.do_ref[lane] = 0;
        }
        wave_lds_fence();
    }
}

// pre-HME decisions (motion_estimation.c:1693-1796), list 0 then list 1, one wavefront
__device__ __forceinline__ void dec_prehme(Dec &d, const svtme_job &job, uint32_t vmask) {
    const svtme_controls &c = job.ctrl;
    const int lane          = threadIdx.x & 63;
    const int nl            = job.num_lists;
    if (c.prehme_enable) {
        for (int l = 0; l < nl; l++) {
            const int r = lane >> 1, sr = lane & 1, s = l * 4 + r;
            if (lane < 8 && slot_valid(vmask, s) && tl_or_l0(job, l)) {
                PreHme &p = d.ph[s][sr];
                bool done = false;
                if (c.me_early_exit_th && d.zz[s] < c.me_early_exit_th) { // check_prehme_early_exit
                    p.col = p.row = 0;
                    p.sad   = 0;
                    p.valid = 1;
                    done    = true;
                }
                if (!done && c.prehme_l1_early_exit && l == 1) {
                    const PreHme &z = d.ph[r][sr];
                    if (z.valid && ((z.sad < (32 * 32)) || ((absi(z.col) < 16) && (absi(z.row) < 16)))) {
                        p.col   = (int16_t)-z.col;
                        p.row   = (int16_t)-z.row;
                        p.sad   = z.sad;
                        p.valid = 1;
                        done    = true;
                    }
                }
                if (!done && !d.do_ref[s]) {
                    p.col = p.row = 0;
                    p.sad = U32MAX;
                    done  = true;
                }
                if (!done) { // searched in stage A
                    const ARes &a = d.a[SVTME_A_PH + s * 2 + sr];
                    p.sad         = a.sad;
                    p.col         = a.x;
                    p.row         = a.y;
                    p.valid       = 1;
                    p.performed   = 1;
                }
            }
            wave_lds_fence();
        }
        uint32_t m  = U32MAX;
        const int s = lane;
        if (slot_valid(vmask, s)) {
            if (tl_or_l0(job, s >> 2)) {
                m = (uint32_t)min_u64(d.ph[s][0].sad, d.ph[s][1].sad);
            } else { // list 1 at the base layer mirrors list 0
                for (int k = 0; k < 2; k++) {
                    d.ph[s][k].col = (int16_t)-d.ph[s & 3][k].col;
                    d.ph[s][k].row = (int16_t)-d.ph[s & 3][k].row;
                    d.ph[s][k].sad = d.ph[s & 3][k].sad;
                }
            }
        }
        const uint32_t best = wave_min_u32(m);
        if (job.temporal_layer_index > 0 && best < c.phme_sad_th && slot_valid(vmask, s) && (s & 3) > 0 &&
            d.do_ref[s] && (uint32_t)((m - best) * 100u) > (uint32_t)(c.phme_sad_pct * best))
            d.do_ref[s] = 0;
        wave_lds_fence();
    }
}

// HME level 0 decisions (motion_estimation.c:1906-2036), one wavefront
__device__ __forceinline__ void dec_l0(Dec &d, const svtme_job &job, uint32_t vmask) {
    const svtme_controls &c = job.ctrl;
    const int lane          = threadIdx.x & 63;
    if (c.enable_hme_flag && c.enable_hme_level0_flag) {
        const int s = lane >> 2, q = lane & 3;
        bool searched = false;
        if (lane < 32 && slot_valid(vmask, s)) {
            int16_t &X = d.lx[s][q], &Y = d.ly[s][q];
            uint64_t &SD = d.lsad[s][q];
            bool done = false;
            if (c.me_early_exit_th && d.zz[s] < (c.me_early_exit_th >> 2)) {
                X = Y = 0;
                SD   = 0;
                done = true;
            }
            if (!done && c.prev_me_stage_based_exit_th) {
                const int k = d.ph[s][0].sad <= d.ph[s][1].sad ? 0 : 1;
                if (d.ph[s][k].performed && d.ph[s][k].sad < (c.prev_me_stage_based_exit_th >> 4)) {
                    X    = d.ph[s][k].col;
                    Y    = d.ph[s][k].row;
                    SD   = d.ph[s][k].sad;
                    done = true;
                }
            }
            if (!done && !d.do_ref[s]) {
                X = Y = 0;
                SD   = U32MAX;
                done = true;
            }
            if (!done && tl_or_l0(job, s >> 2)) {
                const ARes &a = d.a[SVTME_A_L0 + s * 4 + q];
                X             = a.x;
                Y             = a.y;
                SD            = a.sad;
                searched      = true;
            }
        }
        wave_lds_fence();
        // pre-HME replaces the worst quadrant of each searched slot (:2005-2032)
        const unsigned long long sm = __ballot(searched);
        if (c.prehme_enable && lane < 8 && ((sm >> (4 * lane)) & 0xF)) {
            const int s2 = lane;
            uint64_t *S  = d.lsad[s2];
            int wq       = 0; // get_worst_quadrant: strict > in (0,0),(1,0),(0,1),(1,1) order
            uint64_t mx  = 0;
            if (S[0] > mx) { mx = S[0]; wq = 0; }
            if (S[2] > mx) { mx = S[2]; wq = 2; }
            if (S[1] > mx) { mx = S[1]; wq = 1; }
            if (S[3] > mx) { wq = 3; }
            const int k = d.ph[s2][0].sad <= d.ph[s2][1].sad ? 0 : 1;
            if (d.ph[s2][k].sad < S[wq]) {
                S[wq]         = d.ph[s2][k].sad;
                d.lx[s2][wq] = d.ph[s2][k].col;
                d.ly[s2][wq] = d.ph[s2][k].row;
            }
        }
        wave_lds_fence();
    }
}

// RT0 (real-time tune, between the two stage-A rounds): the decisions up to
// slot 0's HME-L0 centre, then the HME-L0 areas of slots 1-7 from it
// (get_hme_l0_search_area, motion_estimation.c:1800-1867) and the slots whose
// HME-L0 runs (dec_l0's exits) into BState for the second round
template <bool RT0>
__global__ void __launch_bounds__(256) k_stage_d(const DevBatch B) {
    __shared__ Dec dec[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t sb_local;
    const DevJob &dj     = batch_job(B, u, &sb_local);
    const svtme_job &job = dj.job;
    Dec &d               = dec[wid];
    const SbGeo G        = sb_geo(dj, sb_local);
    const uint32_t vmask = valid_mask(job);
    if (lane < SVTME_A_N)
        d.a[lane] = dj.ares[(size_t)sb_local * SVTME_A_N + lane];
    dec_init(d);
    dec_zz(d, job, G, vmask);
    dec_prehme(d, job, vmask);
    dec_l0(d, job, vmask);
    BState *b = dj.bst + sb_local;
    if constexpr (RT0) {
        const svtme_controls &c = job.ctrl;
        const int s = lane, l = s >> 2;
        bool run    = s > 0 && s < 8 && slot_valid(vmask, s) && tl_or_l0(job, l) && d.do_ref[s] &&
                   !(c.me_early_exit_th && d.zz[s] < (c.me_early_exit_th >> 2));
        if (run && c.prev_me_stage_based_exit_th) {
            const int k = d.ph[s][0].sad <= d.ph[s][1].sad ? 0 : 1;
            run = !(d.ph[s][k].performed && d.ph[s][k].sad < (c.prev_me_stage_based_exit_th >> 4));
        }
        const uint32_t need = (uint32_t)__ballot(run);
        if (s < 8) {
            int16_t w = 0, h = 0;
            if (slot_valid(vmask, s))
                hme_l0_area(c, l, s & 3, dj.sdist[s], d.lx[0][0], d.ly[0][0], &w, &h);
            b->rt_sa[s][0] = w;
            b->rt_sa[s][1] = h;
        }
        if (lane == 0)
            b->rt_need = (uint8_t)need;
        return;
    }
    if (lane < 32) {
        (&b->lx[0][0])[lane]   = (&d.lx[0][0])[lane];
        (&b->ly[0][0])[lane]   = (&d.ly[0][0])[lane];
        (&b->lsad[0][0])[lane] = (&d.lsad[0][0])[lane];
    }
    if (lane < 8) {
        b->zz[lane]     = d.zz[lane];
        b->do_ref[lane] = d.do_ref[lane];
    }
}

// ----------------------------------------------------------------------------
// Stage B: HME level 1 (and 2) refinement of one (SB, slot, quadrant) per
// wavefront (hme_level1_b64 / hme_level2_b64, motion_estimation.c:2041-2177)
// ----------------------------------------------------------------------------
// one refinement search (hme_level_1 / hme_level_2, :923-1113); the window is
// staged in LDS when it fits, the result is scaled to full-pel units
__device__ __forceinline__ void hme_refine(int level, const DevPlane &P, int16_t qx, int16_t qy, const svtme_area &sa,
                                           int16_t cx, int16_t cy, int bwl, int bhl, bool hsub, const uint8_t *src,
                                           int sst, uint32_t *buf, int16_t *X, int16_t *Y, uint64_t *SD) {
    int16_t xo, yo, sw, sh;
    hme_refine_rect(level, P, qx, qy, (int16_t)sa.width, (int16_t)sa.height, cx, cy, &xo, &yo, &sw, &sh);
    const SadGeo g = sad_geo(P.base, P.stride, qx + xo, qy + yo, sw, sh, bwl, hsub ? bhl >> 1 : bhl, hsub, false,
                             STAGE_B_BUF_DW);
    if (sad_staged(g)) {
        const Win w[1] = {sad_win(g, buf)};
        stage_windows<1>(w, 1u);
    }
    wave_lds_fence();
    const unsigned long long k = sad_compute<RW_8 | RW_16 | RW_4 | RW_2>(g, buf, src, sst);
    uint32_t best;
    int x, y;
    key_result(k, &best, &x, &y);
    const int mul = level == 1 ? 2 : 1;
    *SD           = hsub ? (uint64_t)best * 2 : best;
    *X            = i16((x + xo) * mul);
    *Y            = i16((y + yo) * mul);
}

template <bool L2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(L2 ? 4 : 6, 8))) k_stage_b(const DevBatch B) {
    __shared__ __attribute__((aligned(16))) uint8_t srcb[4][L2 ? 64 * 64 : 32 * 32];
    __shared__ uint32_t wbuf[4][STAGE_B_BUF_DW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const uint32_t sb_local = UNI(gw / dj.tb_count);
    const int e             = UNI(dj.tb_list[gw - sb_local * dj.tb_count]);
    const int s = e >> 2, q = e & 3, l = s >> 2, r = s & 3;
    const SbGeo G   = sb_geo(dj, sb_local);
    const bool hsub = c.hme_search_method != SVTME_FULL_SAD_SEARCH;
    uint8_t *src    = srcb[wid];
    uint32_t *buf   = wbuf[wid];
    BState *b       = dj.bst + sb_local;

    int16_t X = 0, Y = 0; // level-1 result (0 when level 1 is off: init_me_hme_data)
    uint64_t SD = 0;
    if (c.enable_hme_level1_flag) {
        // quarter-resolution source block (32 x 32), issued before the decided state is read
        const DevPlane &Qc = dj.cur.lv[1];
        const uint4 sv     = *(const uint4 *)(Qc.base + (ptrdiff_t)((G.oy >> 1) + (lane >> 1)) * Qc.stride +
                                          (G.ox >> 1) + 16 * (lane & 1));
        const uint32_t zz    = b->zz[s];
        const uint8_t dref   = b->do_ref[s];
        const int16_t X0     = b->lx[s][q], Y0 = b->ly[s][q];
        const uint64_t S0    = b->lsad[s][q];
        ((uint4 *)src)[lane] = sv;
        bool done            = false;
        if (c.me_early_exit_th && zz < (c.me_early_exit_th >> 2)) {
            X = Y = 0;
            SD   = 0;
            done = true;
        }
        if (!done && !dref) {
            X = Y = 0;
            SD   = U32MAX;
            done = true;
        }
        if (!done && c.prev_me_stage_based_exit_th && S0 < (c.prev_me_stage_based_exit_th >> 5)) {
            X = X0, Y = Y0, SD = S0;
            done = true;
        }
        if (!done)
            hme_refine(1, dj.ref[l][r].lv[1], i16(((int16_t)G.ox) >> 1), i16(((int16_t)G.oy) >> 1), c.hme_l1_sa,
                       i16(X0 >> 1), i16(Y0 >> 1), (int)(G.bw >> 1), (int)(G.bh >> 1), hsub, src, hsub ? 64 : 32,
                       buf, &X, &Y, &SD);
    }
    if (L2 && c.enable_hme_level2_flag) {
        if (!(c.prev_me_stage_based_exit_th && SD < (c.prev_me_stage_based_exit_th >> 2))) {
            const DevPlane &F = dj.cur.lv[0]; // full-resolution source block (64 x 64)
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = u * 64 + lane, rr = t >> 2, j = t & 3;
                ((uint4 *)src)[t] = *(const uint4 *)(F.base + (ptrdiff_t)(G.oy + rr) * F.stride + G.ox + 16 * j);
            }
            hme_refine(2, dj.ref[l][r].lv[0], (int16_t)G.ox, (int16_t)G.oy, c.hme_l2_sa, X, Y, (int)G.bw, (int)G.bh,
                       hsub, src, hsub ? 128 : 64, buf, &X, &Y, &SD);
        }
    }
    if (lane == 0) {
        b->hx[s][q]   = X;
        b->hy[s][q]   = Y;
        b->hsad[s][q] = SD;
    }
}

// set_final_seach_centre_sb (motion_estimation.c:2182-2380) and
// hme_prune_ref_and_adjust_sr (:2477-2518) of one SB from the state stages D
// and B left, by one whole wavefront; lane s < 8 returns slot s
struct SlotCentre {
    uint64_t hme_sad;
    uint32_t zz, reduce_div;
    int16_t sc_x, sc_y;
    uint8_t do_ref;
};

// set_final_seach_centre_sb and hme_prune_ref_and_adjust_sr (motion_estimation.c:
// 2182-2380, 2477-2518), lane = slot. Every input is read first, unconditionally,
// in one batch (control values by scalar loads when job is in global memory, the
// slot's BState words): a read under a branch would wait for each in turn
__device__ __forceinline__ SlotCentre final_centre(const svtme_job &job, const BState *b, uint32_t vmask) {
    const svtme_controls &c = job.ctrl;
    const int s             = threadIdx.x & 63;
    const bool hme_on = SF(c, enable_hme_flag) != 0, l0f = SF(c, enable_hme_level0_flag) != 0;
    const bool l1f = SF(c, enable_hme_level1_flag) != 0, l2f = SF(c, enable_hme_level2_flag) != 0;
    const bool mctf  = SF(job, me_type) == SVTME_ME_MCTF;
    const int tli    = (int)SF(job, temporal_layer_index);
    const uint32_t pth = SF(c, prune_ref_if_hme_sad_dev_bigger_than_th);
    const bool prune = SF(c, enable_me_hme_ref_pruning) != 0, sradj = SF(c, enable_me_sr_adjustment) != 0;
    const int mvlen  = (int)SF(c, reduce_me_sr_based_on_mv_length_th);
    const uint32_t stat_th = SF(c, stationary_hme_sad_abs_th), stat_div = SF(c, stationary_me_sr_divisor);
    const uint32_t low_th = SF(c, reduce_me_sr_based_on_hme_sad_abs_th), low_div = SF(c, me_sr_divisor_for_low_hme_sad);
    int lvl = -1;
    if (l0f && !l1f && !l2f)
        lvl = 0;
    if (l1f && !l2f)
        lvl = 1;
    if (l2f)
        lvl = 2;
    const int sl = s & 7;
    const int16_t *X  = lvl > 0 ? b->hx[sl] : b->lx[sl];
    const int16_t *Y  = lvl > 0 ? b->hy[sl] : b->ly[sl];
    const uint64_t *S = lvl > 0 ? b->hsad[sl] : b->lsad[sl];
    // (named values, not arrays: small private arrays are promoted to LDS)
    const int16_t x0 = X[0], x1 = X[1], x2 = X[2], x3 = X[3], y0 = Y[0], y1 = Y[1], y2 = Y[2], y3 = Y[3];
    const uint64_t s0 = S[0], s1 = S[1], s2 = S[2], s3 = S[3];
    const uint8_t dref0 = b->do_ref[sl];
    const uint32_t zz0  = b->zz[sl];
    const bool valid    = slot_valid(vmask, s);
    const bool hme_slot = valid && (tli > 0 || (s >> 2) == 0) && hme_on;
    int16_t hx = 0, hy = 0;
    uint64_t hs    = 0;
    const bool own = hme_slot && lvl >= 0;
    if (own) {
        hx = x0, hy = y0, hs = s0;
        // scan order (w, h): (1,0), (0,1), (1,1) = q 2, 1, 3
        if (s2 < hs) { hx = x2; hy = y2; hs = s2; }
        if (s1 < hs) { hx = x1; hy = y1; hs = s1; }
        if (s3 < hs) { hx = x3; hy = y3; hs = s3; }
    }
    // the reference carries function-scope values across slots
    int16_t cx = 0, cy = 0, scx = 0, scy = 0;
    uint64_t cs = 0;
    int16_t my_scx = 0, my_scy = 0;
    uint64_t my_hs = 0;
    for (int k = 0; k < 8; k++) {
        if (!((vmask >> k) & 1u))
            continue;
        const bool ok = rl32((uint32_t)own, k) != 0;
        const bool hk = rl32((uint32_t)hme_slot, k) != 0;
        const bool tk = tli > 0 || (k >> 2) == 0;
        const int16_t kx = (int16_t)rl32((uint32_t)(int32_t)hx, k), ky = (int16_t)rl32((uint32_t)(int32_t)hy, k);
        const uint64_t ks = rl64(hs, k);
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
        if (s == k) {
            my_scx = scx, my_scy = scy, my_hs = cs;
        }
    }
    uint64_t hsad = U32MAX; // SearchResults init (hme_sad = MAX_U32)
    if (valid)
        hsad = my_hs;
    uint32_t rdiv = 1;
    uint8_t dref  = s < 8 ? dref0 : 0;
    if (hme_on && !mctf) { // prune_ref (motion_estimation.c:3103)
        if (prune && pth != 0xFFFFu) {
            const uint64_t best = wave_min_u64(s < 8 ? hsad : ~0ull);
            if (s < 8 && (s & 3) >= 1 && (hsad - best) * 100 > (pth * best))
                dref = 0;
        }
        if (sradj && s < 8) {
            if (absi(my_scx) <= mvlen && absi(my_scy) <= mvlen && hsad < stat_th)
                rdiv = stat_div;
            else if (hsad < low_th)
                rdiv = low_div;
        }
    }
    SlotCentre o;
    o.hme_sad    = hsad;
    o.zz         = s < 8 ? zz0 : U32MAX;
    o.reduce_div = rdiv;
    o.sc_x       = valid ? my_scx : 0;
    o.sc_y       = valid ? my_scy : 0;
    o.do_ref     = dref;
    return o;
}

// ----------------------------------------------------------------------------
// k_hme: stages A, D and B of one SB fused in one workgroup (4 wavefronts).
// Used when every SB of the job is 64 wide, the HME searches sub-sample rows
// (hme_search_method SUB_SAD) and level 2 is off (svtme_hme_fused); other jobs
// run k_stage_a -> k_stage_d -> k_stage_b. Both write the same BState.
//
//   A0  zz SADs of every slot (init_zz_sad), then the zz decisions, so that
//       pre-HME / level-0 searches the reference provably skips (zz early exit,
//       zz pruning) are never run;
//   A1  the pre-HME regions and HME-L0 quadrants, as register tiles: a lane
//       owns HQ aligned position quads x HT position rows 2 plane rows apart
//       (the sub-sampled block's rows), so each loaded reference row feeds up
//       to 8 block rows x 12 positions; the 16x16 (sub: 16x8) source block
//       sits in SGPRs. Tile minima merge with ds_min_u64 per search;
//   D   the pre-HME and level-0 decisions (dec_prehme, dec_l0);
//   B   HME-L1: a lane owns HQ quads of one position row of one (slot,
//       quadrant) search, the 32x16 (sub) source block in LDS.
// Keys inside a tile are 32-bit (sad << 16 | x, one v_lshl_or / v_and_or and
// a v_min3 per position pair); the row, then the lane's best widen to the
// 64-bit sad << 32 | y << 16 | x order of the reference's scan.
// ----------------------------------------------------------------------------
// Phase hooks of k_hme. The diagnostic builds (scripts/build_diag_lib.sh) force-
// include csrc/diag/svtme_diag.h, which defines them (phase stamps, stop-after
// builds, clock bins); the product build has none of that code.
#ifndef HME_STAMP
#define HME_STAMP(k)
#endif
#ifndef HME_STOP
#define HME_STOP(k)
#endif
#ifndef HME_SUB
#define HME_SUB(k)
#endif
#ifndef HME_WAVE
#define HME_WAVE(k)
#endif

#define HQ 2  // position quads per HME-L2 tile (rows realigned to position 0: 8-wide areas = 2 quads)
#define HQ1 2 // position quads per HME-L1 tile (rows realigned to position 0: 8-wide areas = 2 quads)
#define HQ16 2 // position quads per 1/16 tile (interior windows are dword aligned: 8/16/32 wide = 2/4/8 quads)

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
// 16 bytes at a dword-aligned global address (the planes are global memory)
__device__ __forceinline__ u32x4a4 ldg4(const uint32_t *p) {
    typedef __attribute__((address_space(1))) const u32x4a4 gu4;
    return *(gu4 *)(uintptr_t)p;
}
// raw buffer over a plane from a dword-aligned base (gfx9 descriptor word 3),
// and a 16-byte load at lane offset voff + uniform offset soff (bytes): the
// address adds go to the load unit, none to the VALU
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)0xFFFFFFFF, 0x00020000);
}
__device__ __forceinline__ u32x4a4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    u32x4a4 o;
    o.x = v[0], o.y = v[1], o.z = v[2], o.w = v[3];
    return o;
}
// 16 uniform bytes through the scalar cache (p wave-uniform, 4-byte aligned)
__device__ __forceinline__ uint4 sld4(const uint8_t *p) {
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    cu32 *q = (cu32 *)(uintptr_t)p;
    return make_uint4(q[0], q[1], q[2], q[3]);
}
__device__ __forceinline__ unsigned long long qsad64(unsigned long long ref, uint32_t s, unsigned long long a) {
    return __builtin_amdgcn_qsad_pk_u16_u8(ref, s, a);
}
__device__ __forceinline__ unsigned long long pair(uint32_t lo, uint32_t hi) {
    return ((unsigned long long)hi << 32) | lo;
}

struct HSrch {             // one 1/16-resolution search (pre-HME region or HME-L0 quadrant)
    const uint8_t *a0;     // dword-aligned plane address of window dword 0, position row 0
    int32_t item0;         // first tile of this search in the SB's tile list
    int16_t sa_w, ncols;   // positions per row; tile columns
    int16_t cnt0, cnt1;    // position rows of each tile-row parity (skip: cnt0 = rows, cnt1 = 0)
    int16_t ylast;         // last plane-row offset a tile of this search may read
    uint32_t ncm;          // magic_u32(ncols): tile index / ncols by multiply-high
    uint8_t sh, skip, id;  // byte offset of position 0; odd rows only; ARes index
    uint8_t need;          // bit of HmeSh::need (slot * 2 + (L0 ? 1 : 0))
    uint8_t tt;            // position rows per tile: HT16, or 2 (the HME-L0 group, see k_hme A1)
};
struct HSrch1 {            // one HME-L1 refinement search
    const uint8_t *a0;
    int32_t item0;
    uint32_t ncm;          // magic_u32(ncols)
    int16_t sa_w, ncols;
    uint8_t sh, id;        // id = slot * 4 + quadrant
};


// rows of one 1/16 tile row: the HQ16 + 4 = 6 dwords from quad q0 its position
// quads read (dword-aligned 16- and 8-byte loads)
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
struct Row8 {
    u32x4a4 lo;
    u32x2a4 hi;
};
__device__ __forceinline__ Row8 row8(const uint8_t *a0, int stride, int ro, int q0) {
    typedef __attribute__((address_space(1))) const u32x2a4 gu2;
    const uint32_t *rp = (const uint32_t *)(a0 + (ptrdiff_t)ro * stride) + q0;
    return Row8{ldg4(rp), *(gu2 *)(uintptr_t)(rp + 4)};
}

// SADs of the 16 x kh (sub) source block sr at a T x HQ tile of positions of
// a 1/16 window: quads q0.. of row a0 (sh = byte offset of position 0),
// position rows yf + 2t (t < tv); plane rows are clamped to ylast. Rows are
// loaded two ahead of their use. Returns the tile's minimum key
// (sad << 32 | y << 16 | x), ~0 if no position is valid.
template <int T, bool FULLK = false> // FULLK: a full-height SB (kh == 8), no row checks
__device__ __forceinline__ unsigned long long hme_tile16(const uint8_t *a0, int stride, int q0, int sh, int sa_w,
                                                         int yf, int tv, int ylast, int kh,
                                                         const uint32_t (&sr)[8][4]) {
    constexpr int NR = T + 7;
    kh = UNI(kh); // the block-row checks become scalar compares and branches
    unsigned long long acc[T][HQ16];
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
        for (int qq = 0; qq < HQ16; qq++) acc[t][qq] = 0;
    Row8 buf[3];
    buf[0] = row8(a0, stride, min(yf, ylast), q0);
    buf[1] = row8(a0, stride, min(yf + 2, ylast), q0);
#pragma unroll
    for (int m = 0; m < NR; m++) {
        if (m + 2 < NR)
            buf[(m + 2) % 3] = row8(a0, stride, min(yf + 2 * (m + 2), ylast), q0);
        const Row8 &R = buf[m % 3];
        static_assert(HQ16 + 4 == 6, "Row8 holds 6 dwords");
        const uint32_t d[6] = {R.lo.x, R.lo.y, R.lo.z, R.lo.w, R.hi.x, R.hi.y};
        unsigned long long P[HQ16 + 3];
#pragma unroll
        for (int j = 0; j < HQ16 + 3; j++) P[j] = pair(d[j], d[j + 1]);
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int k = m - t;
            if (k < 0 || k >= 8)
                continue;
            if (!FULLK && k >= kh) // wave-uniform (partial-height SB)
                continue;
#pragma unroll
            for (int qq = 0; qq < HQ16; qq++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[t][qq] = qsad64(P[qq + j], sr[k][j], acc[t][qq]);
        }
    }
    uint32_t xo[HQ16][4];
#pragma unroll
    for (int qq = 0; qq < HQ16; qq++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int x = 4 * (q0 + qq) - sh + e;
            xo[qq][e]   = (x >= 0 && x < sa_w) ? (uint32_t)x : U32MAX;
        }
    unsigned long long best = ~0ull;
    // the key rows from a fresh copy of yf: CSE with the row addresses above keeps
    // yf + 2t live through the loop (a spill at 64 VGPRs)
    uint32_t yk = (uint32_t)yf;
    asm volatile("" : "+v"(yk));
#pragma unroll
    for (int t = 0; t < T; t++) {
        uint32_t mt = U32MAX;
#pragma unroll
        for (int qq = 0; qq < HQ16; qq++) {
            const uint32_t lo = (uint32_t)acc[t][qq], hi = (uint32_t)(acc[t][qq] >> 32);
            const uint32_t k0 = (lo << 16) | xo[qq][0], k1 = (lo & 0xFFFF0000u) | xo[qq][1];
            const uint32_t k2 = (hi << 16) | xo[qq][2], k3 = (hi & 0xFFFF0000u) | xo[qq][3];
            mt = min_u32(mt, min_u32(min_u32(k0, k1), min_u32(k2, k3)));
        }
        if (t < tv && mt != U32MAX) {
            const unsigned long long kk = ((unsigned long long)(mt >> 16) << 32) |
                                          ((unsigned long long)(yk + 2 * t) << 16) | (mt & 0xFFFFu);
            best = kk < best ? kk : best;
        }
    }
    return best;
}

// One quarter of the SADs of the 32 x kh1 (sub) quarter-resolution source
// block (LDS, rows 32 bytes apart) at HQ1 quads of position row y of a 1/4
// window (a0 dword aligned, position 0 at byte sh: the rows are realigned with
// v_alignbyte): block rows [4g, 4g + 4) of lane g = lane & 3, all loads
// issued up front; the 4 lanes of a quad then sum their partial SADs (DPP)
// and every lane returns the row's minimum key.
template <bool FULLK = false> // FULLK: a full-height SB (kh1 == 16), no row checks
__device__ __forceinline__ unsigned long long hme_tile32q(const uint8_t *a0, int stride, int q0, int sh, int sa_w,
                                                          int y, int kh1, const uint8_t (*src)[32]) {
    const int g = threadIdx.x & 3;
    // the HQ1 + 9 = 11 dwords a row's quads read: 16 + 16 + 12 bytes
    static_assert(HQ1 + 9 == 11, "L1 rows hold 11 dwords");
    typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
    typedef __attribute__((address_space(1))) const u32x3a4 gu3;
    struct Row11 {
        u32x4a4 a, b;
        u32x3a4 c;
    };
    auto ld = [&](int kk, Row11 &L) {
        const int k        = min(4 * g + kk, 15);
        const uint32_t *rp = (const uint32_t *)(a0 + (ptrdiff_t)(y + 2 * k) * stride) + q0;
        L.a = ldg4(rp), L.b = ldg4(rp + 4), L.c = *(gu3 *)(uintptr_t)(rp + 8);
    };
    Row11 L[2];
    ld(0, L[0]);
    unsigned long long acc[HQ1] = {};
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
        if (kk + 1 < 4)
            ld(kk + 1, L[(kk + 1) & 1]);
        // every row is summed and rows past the block height (a partial SB, a
        // per-lane test) are dropped by a select: no divergent branch, whose
        // join would wait for the row prefetched above
        const int k = min(4 * g + kk, 15);
        {
            const Row11 &R = L[kk & 1];
            const uint4 s0 = ((const uint4 *)src[k])[0], s1 = ((const uint4 *)src[k])[1];
            const uint32_t sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            uint32_t d[11] = {R.a.x, R.a.y, R.a.z, R.a.w, R.b.x, R.b.y, R.b.z, R.b.w, R.c.x, R.c.y, R.c.z};
#pragma unroll
            for (int j = 0; j < HQ1 + 8; j++) d[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], (uint32_t)sh);
            const bool use = FULLK || 4 * g + kk < kh1;
#pragma unroll
            for (int qq = 0; qq < HQ1; qq++) {
                unsigned long long a = acc[qq];
#pragma unroll
                for (int j = 0; j < 8; j++) a = qsad64(pair(d[qq + j], d[qq + j + 1]), sv[j], a);
                acc[qq] = use ? a : acc[qq];
            }
        }
    }
    uint32_t mt = U32MAX; // sad (< 2^17) << 15 | x (< 2^15)
#pragma unroll
    for (int qq = 0; qq < HQ1; qq++) {
        uint32_t a[4] = {0, 0, 0, 0};
        qsad_unpack(acc[qq], a);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t v = dpp_add<0x4E>(dpp_add<0xB1>(a[e])); // the quad's 4 row groups
            const int x      = 4 * (q0 + qq) + e;
            if (x < sa_w)
                mt = min_u32(mt, (v << 15) | (uint32_t)x);
        }
    }
    if (mt == U32MAX)
        return ~0ull;
    return ((unsigned long long)(mt >> 15) << 32) | ((unsigned long long)(uint32_t)y << 16) | (mt & 0x7FFFu);
}

#define HL2_PITCH 96 // bytes per LDS row of HME-L2's full-resolution source block (64 used)
// One eighth of the SADs of the 64 x kh2 (sub) full-resolution source
// block (LDS, rows HL2_PITCH bytes apart) at HQ quads of position row y of a
// full-resolution window (HME-L2): block rows g + 8j of lane g = lane & 7;
// the 8 lanes of a row then sum their partial SADs (DPP) and every lane
// returns the row's minimum key. Rows are realigned to position 0 of the
// window (a0 = its dword-aligned base, sh = its byte offset; v_alignbyte), so
// an 8-wide area is 2 quads at any alignment: 32 qsads per block row instead
// of the 48 of 3 unaligned quads, for 18 v_alignbyte.
__device__ __forceinline__ unsigned long long hme_tile64(const uint8_t *a0, int stride, int q0, int sh, int sa_w,
                                                         int y, int kh2, const uint8_t (*src)[HL2_PITCH]) {
    const int g = threadIdx.x & 7;
    unsigned long long acc[HQ] = {};
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
        // block rows g, g + 8, g + 16, g + 24: the 8 rows a ds_read_b128 lane group reads at
        // once are HL2_PITCH = 96 bytes (24 banks) apart, 8 disjoint 4-bank sets (rows 4g + kk,
        // 64 bytes apart, all fell on the same 4 banks: 8-way conflicts)
        const int k = g + 8 * kk;
        if (k < kh2) {
            const uint32_t *rp = (const uint32_t *)(a0 + (ptrdiff_t)(y + 2 * k) * stride) + q0;
            u32x4a4 L[5];
#pragma unroll
            for (int v = 0; v < 5; v++) L[v] = ldg4(rp + 4 * v);
            uint32_t d[20];
#pragma unroll
            for (int v = 0; v < 5; v++) d[4 * v] = L[v].x, d[4 * v + 1] = L[v].y, d[4 * v + 2] = L[v].z, d[4 * v + 3] = L[v].w;
            constexpr int ND = HQ + 16; // realigned dwords the qsad pairs read
#pragma unroll
            for (int j = 0; j < ND; j++) d[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], (uint32_t)sh);
#pragma unroll
            for (int j4 = 0; j4 < 4; j4++) {
                const uint4 sv = ((const uint4 *)src[k])[j4];
                const uint32_t s4[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const int j = 4 * j4 + jj;
#pragma unroll
                    for (int qq = 0; qq < HQ; qq++) acc[qq] = qsad64(pair(d[qq + j], d[qq + j + 1]), s4[jj], acc[qq]);
                }
            }
        }
    }
    uint32_t mt = U32MAX; // sad (< 2^19) << 13 | x (< 2^13)
#pragma unroll
    for (int qq = 0; qq < HQ; qq++) {
        uint32_t a[4] = {0, 0, 0, 0};
        qsad_unpack(acc[qq], a);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            // the row's 8 lanes: quad xor 1 / 2, row_half_mirror
            const uint32_t v = dpp_add<0x141>(dpp_add<0x4E>(dpp_add<0xB1>(a[e])));
            const int x      = 4 * (q0 + qq) + e;
            if (x < sa_w)
                mt = min_u32(mt, (v << 13) | (uint32_t)x);
        }
    }
    if (mt == U32MAX)
        return ~0ull;
    return ((unsigned long long)(mt >> 13) << 32) | ((unsigned long long)(uint32_t)y << 16) | (mt & 0x1FFFu);
}

// flat tile index -> search (binary search over item0, n > 0 searches)
template <typename S>
__device__ __forceinline__ int find_search(const S *t, int n, int it) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (t[mid].item0 <= it)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

#define HT16 3 // position rows per 1/16 tile (4K p8: 190 tiles per SB, one pass of the workgroup)


// ----------------------------------------------------------------------------
// Stage C: integer full-pel search with the 85-PU argmin, ME pruning, records,
// candidates; one workgroup per SB
// ----------------------------------------------------------------------------
struct FpRef {        // one full-pel search window of a reference slot
    const uint32_t *a; // dword-aligned address of window row 0 (search row 0)
    int32_t sdw;       // plane stride in dwords
    int32_t nitems;    // rows x aligned quads
    int32_t item_begin;
    uint32_t mnq;
    int16_t xo, yo, w, h;
    int32_t order_base; // 0: 8x8-variance centre probe, 1: main search
    uint8_t slot, nq, sh, pad;
};

struct StC {
    DevPlane pl[8][1];
    uint16_t dist[8];
    uint64_t refpic[8];
    uint64_t hme_sad[8];
    uint32_t zz[8];
    uint32_t reduce_div[8];
    uint32_t sum8[8]; // per slot: the sum of its 64 8x8 best SADs (me_prune_ref), when stage_e_body made it
    int16_t sc_x[8], sc_y[8];
    uint8_t do_ref[8], searched[8], in_round[8];
    uint8_t tf_exit; // MCTF HME-only exit (motion_estimation.c:3109-3113)
    int16_t is_w[8], is_h[8], is_wb[8], is_hb[8], is_xc[8], is_yc[8];
    uint64_t is_best_hme[8];
    const uint8_t *req[16]; // check_00_center n x m requests
    int32_t req_stride[16];
    int8_t req_slot[8];
    uint32_t nxm[16];
    int32_t nreq, nfp, k32, fp_items;
    FpRef fp[8];
    // the 85-PU argmin keys by slot; once decoded into rec, the svtme_sb_result image (finish_sb)
    __attribute__((aligned(16))) unsigned long long keys[8][SVTME_PU_COUNT];
    // per slot, the image of its svtme_ref_record: best_sad [0, 85), best_mv [85, 170),
    // the tail [170, 176) (filled as the record is written): one 16-byte copy per lane
    __attribute__((aligned(16))) uint32_t rec[8][176];
    uint8_t cand0[SVTME_PU_COUNT + 3];
    uint32_t gm_cnt[2][4][2][2];
    uint32_t sink;  // finish_sb's stores that have no target
};

// Window of one reference: rows h, positions w, dword-aligned quads
__device__ void make_fp(FpRef &F, const DevPlane &P, uint32_t ox, uint32_t oy, int slot, int16_t xo, int16_t yo,
                        int16_t w, int16_t h, int order_base) {
    const uint8_t *g = P.base + (ptrdiff_t)((int)oy + yo) * P.stride + ((int)ox + xo);
    F.sh             = (uint8_t)((uintptr_t)g & 3);
    F.a              = (const uint32_t *)(g - F.sh);
    F.sdw            = P.stride >> 2;
    F.slot           = (uint8_t)slot;
    F.xo = xo, F.yo = yo, F.w = w, F.h = h;
    F.order_base = order_base;
    F.nq         = (uint8_t)((F.sh + w + 3) >> 2);
    F.mnq        = magic_u32(F.nq);
    F.nitems     = (int)h * F.nq;
}

// wave 0: item offsets of the compacted FpRefs (this lane's at k when mk)
__device__ __forceinline__ void plan_fp(StC &st, bool mk, int k, int n) {
    const int items = mk ? st.fp[k].nitems : 0;
    const int incl  = wave_incl_scan(items);
    if (mk)
        st.fp[k].item_begin = incl - items;
    if ((threadIdx.x & 63) == 63)
        st.fp_items = incl;
    if ((threadIdx.x & 63) == 0)
        st.nfp = n;
}

// Full-pel search of the planned windows (motion_estimation.c:98-425, 781-817):
// lane = 8x8 block in Z-order; one item = one aligned position quad of a
// search row of one window; the items of all windows are dealt to the 4
// waves DEPTH at a time with their loads issued together. 16x16 / 32x32 /
// 64x64 SADs are DPP lane sums. Keys are (sad << 12 | order) in 32 bits when
// every order < 4096 (64x64 SAD < 2^20), else (sad << 32 | order).
template <bool SUB, bool K32>
__device__ void fullpel_run(StC &st, const DevPlane &C, uint32_t ox, uint32_t oy) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int z16 = lane >> 2, k4 = lane & 3;
    const int by = ((z16 >> 3) << 2) | (((z16 >> 1) & 1) << 1) | (k4 >> 1);
    const int bx = (((z16 >> 2) & 1) << 2) | ((z16 & 1) << 1) | (k4 & 1);
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1, DEPTH = SUB ? 2 : 1;
    typedef typename std::conditional<K32, uint32_t, unsigned long long>::type key_t;
    for (int e = tid; e < st.nfp * SVTME_PU_COUNT; e += 256) {
        const int f = e / SVTME_PU_COUNT;
        st.keys[st.fp[f].slot][e - f * SVTME_PU_COUNT] = ~0ull;
    }
    uint32_t src[ROWS][2];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const uint32_t *sp =
            (const uint32_t *)(C.base + (ptrdiff_t)(oy + by * 8 + r * RSTEP) * C.stride + ox + bx * 8);
        src[r][0] = sp[0];
        src[r][1] = sp[1];
    }
    __syncthreads();
    const int nfp = st.nfp, total = st.fp_items;
    int cur = -1;
    key_t b8 = (key_t)~0ull, b16 = (key_t)~0ull, b32 = (key_t)~0ull, b64 = (key_t)~0ull;
    auto wide = [](key_t kk) -> unsigned long long {
        if (K32) {
            const uint32_t v = (uint32_t)kk;
            return v == 0xFFFFFFFFu ? ~0ull : (((unsigned long long)(v >> 12) << 32) | (v & 0xFFFu));
        }
        return (unsigned long long)kk;
    };
    auto flush = [&](int f) {
        unsigned long long *pk = st.keys[UNI(st.fp[f].slot)];
        atomicMin(&pk[21 + lane], wide(b8));
        if ((lane & 3) == 0)
            atomicMin(&pk[5 + (lane >> 2)], wide(b16));
        if ((lane & 15) == 0)
            atomicMin(&pk[1 + (lane >> 4)], wide(b32));
        if (lane == 63)
            atomicMin(&pk[0], wide(b64));
    };
    for (int base = wid * DEPTH; base < total; base += 4 * DEPTH) {
        uint32_t d[DEPTH][ROWS][3];
        int fi[DEPTH], yi[DEPTH], qi[DEPTH];
#pragma unroll
        for (int u = 0; u < DEPTH; u++) {
            const int i = base + u;
            int f = 0;
            while (f + 1 < nfp && st.fp[f + 1].item_begin <= i) f++;
            fi[u] = UNI(f);
            if (i < total) {
                const FpRef &F = st.fp[fi[u]];
                const int li   = i - UNI(F.item_begin);
                const int nq   = UNI(F.nq);
                yi[u] = mdiv(li, (uint32_t)UNI(F.mnq));
                qi[u] = li - yi[u] * nq;
                const int sdw = UNI(F.sdw);
                const uint32_t *rp = F.a + (ptrdiff_t)(yi[u] + by * 8) * sdw + qi[u] + bx * 2;
#pragma unroll
                for (int rr = 0; rr < ROWS; rr++) {
                    const uint32_t *rd = rp + (ptrdiff_t)(rr * RSTEP) * sdw;
                    d[u][rr][0] = rd[0];
                    d[u][rr][1] = rd[1];
                    d[u][rr][2] = rd[2];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < DEPTH; u++) {
            const int i = base + u;
            if (i >= total)
                break; // wave-uniform
            const int f = fi[u];
            if (f != cur) {
                if (cur >= 0)
                    flush(cur);
                b8 = b16 = b32 = b64 = (key_t)~0ull;
                cur = f;
            }
            const FpRef &F = st.fp[f];
            const int w = UNI(F.w), sh = UNI(F.sh), obase = UNI(F.order_base);
            const int y = yi[u], q = qi[u];
            unsigned long long a = 0;
#pragma unroll
            for (int rr = 0; rr < ROWS; rr++) {
                a = qsad(d[u][rr][0], d[u][rr][1], src[rr][0], a);
                a = qsad(d[u][rr][1], d[u][rr][2], src[rr][1], a);
            }
            uint32_t acc[4] = {0, 0, 0, 0};
            qsad_unpack(a, acc);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int x = 4 * q - sh + k;
                if (x < 0 || x >= w)
                    continue; // wave-uniform
                const uint32_t s8  = SUB ? acc[k] << 1 : acc[k];
                const uint32_t s16 = dpp_add<0x4E>(dpp_add<0xB1>(s8));              // xor 1, xor 2
                const uint32_t s32 = dpp_add<0x128>(dpp_add<0x124>(s16));           // row_ror 4, 8
                const uint32_t s64 = dpp_add<0x143, 0xC>(dpp_add<0x142, 0xA>(s32)); // valid in row 3
                const uint32_t o   = (uint32_t)(obase + y * w + x);
                if (K32) {
                    b8  = min_u32((uint32_t)b8, (s8 << 12) | o);
                    b16 = min_u32((uint32_t)b16, (s16 << 12) | o);
                    b32 = min_u32((uint32_t)b32, (s32 << 12) | o);
                    b64 = min_u32((uint32_t)b64, (s64 << 12) | o);
                } else {
                    const unsigned long long k8  = ((unsigned long long)s8 << 32) | o;
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
    }
    if (cur >= 0)
        flush(cur);
    __syncthreads();
    // decode: strict-< update of the running best (motion_estimation.c:1366, :137-205)
    for (int e = tid; e < st.nfp * SVTME_PU_COUNT; e += 256) {
        const int f = e / SVTME_PU_COUNT, pu = e - f * SVTME_PU_COUNT;
        const FpRef &F             = st.fp[f];
        const unsigned long long k = st.keys[F.slot][pu];
        const uint32_t sad         = (uint32_t)(k >> 32);
        if (k != ~0ull && sad < st.rec[F.slot][pu]) {
            const int p      = (int)(uint32_t)k - F.order_base;
            const int16_t my = (int16_t)(F.yo + p / F.w);
            const int16_t mx = (int16_t)(F.xo + p % F.w);
            st.rec[F.slot][pu] = sad;
            st.rec[F.slot][SVTME_PU_COUNT + pu]  = ((uint32_t)(uint16_t)my << 16) | (uint16_t)mx;
        }
    }
    __syncthreads();
}

template <bool SUB>
__device__ void fullpel(StC &st, const DevPlane &C, uint32_t ox, uint32_t oy) {
    if (st.k32)
        fullpel_run<SUB, true>(st, C, ox, oy);
    else
        fullpel_run<SUB, false>(st, C, ox, oy);
}

// Candidate arrays + distortions + GM detection for one SB (motion_estimation.c:
// 2532-3007), in two parts with a barrier between. finish_sb_cands: thread n < 85
// builds Z-order PU n's candidates, MVs and me_distortion in an LDS image laid over
// st.keys (dead once the keys are decoded into st.rec; stage_c_tail zeroes it).
// finish_sb_out: waves 2-3 store the image up to me_distortion in 16-byte pieces
// while wave 0 (compute_distortion) and wave 1 (GM detection) finish the last words
// and store them themselves: no zero fill of the HBM copy, no scattered byte stores
// to HBM.
__device__ __forceinline__ void finish_sb_cands(StC &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh) {
    static_assert(sizeof(svtme_sb_result) % 4 == 0 && sizeof(svtme_sb_result) <= sizeof(st.keys) &&
                      sizeof(st.keys) % 16 == 0, "svtme_sb_result image over st.keys");
    const svtme_job &job = dj.job;
    const int tid        = threadIdx.x;
    // (the byte fields by scalar dword loads: SF)
    const int nl = (int)SF(job, num_lists), nr0 = (int)SF(job, num_refs[0]), nr1 = nl == 2 ? (int)SF(job, num_refs[1]) : 0;
    const bool mctf = SF(job, me_type) == SVTME_ME_MCTF; // (no candidates / distortions, motion_estimation.c:3126)
    const bool en8 = SF(job, enable_me_8x8) != 0, en16 = SF(job, enable_me_16x16) != 0;
    const int max_l0   = (int)SF(job, max_l0);
    svtme_sb_result *o = (svtme_sb_result *)&st.keys[0][0];
    if (!mctf && tid < SVTME_PU_COUNT) {
        const int npus = en16 ? (en8 ? 85 : 21) : 5;
        const int mode = (nr0 == 1 && nr1 == 0) ? 0 : (nr0 == 1 && nr1 == 1) ? 1 : 2;
        const int n    = tid;
        const int pu   = z_to_raster(n); // (a permutation: thread n owns PU pu's entries)
        const int use  = en16 ? (en8 || n < 21) : n < 5;
        if (mode != 2) // memset(total_me_candidate_index, 1, number_of_pus)
            o->total_me_candidate_index[pu] = pu < npus ? 1 : 0;
        if (mode == 0) { // construct_me_candidate_array_single_ref
            o->me_distortion[pu] = st.rec[0][n];
            st.cand0[pu]         = 0;
            if (st.do_ref[0] && use) {
                o->me_candidate_array[pu][0] = mk_cand(0, 0, 0, 0, 0);
                o->me_mv_array[pu][0]        = st.rec[0][SVTME_PU_COUNT + n];
            }
        } else if (mode == 1) { // construct_me_candidate_array_mrp_off
            uint32_t nlist     = nl;
            const uint8_t org0 = st.do_ref[0], org1 = nl == 1 ? 0 : st.do_ref[4];
            if (nlist < 2 || !st.do_ref[4])
                nlist = 1;
            const uint32_t prune_th = (org0 && org1) ? (uint32_t)job.ctrl.prune_me_candidates_th : 0;
            uint8_t off  = 0;
            uint32_t blk = (org0 ? 1u : 0u) | (org1 ? 2u : 0u); // bit li
            const uint32_t s0 = st.rec[0][n], s1 = st.rec[4][n];
            const uint32_t best = (org0 && org1) ? min_u32(s0, s1) : org0 ? s0 : s1;
            o->me_distortion[pu] = best;
            int min_list         = -1;
            if (SF(job, ctrl.use_best_unipred_cand_only) && (blk & 3u) == 3u)
                min_list = s0 < s1 ? 0 : 1;
            uint8_t c0 = 0;
            for (int li = 0; (uint32_t)li < nlist && (use || off == 0); ++li) {
                if (!((blk >> li) & 1u))
                    continue;
                if (prune_th > 0) {
                    const uint32_t dd = (st.rec[li * 4][n] - best) * 100;
                    if (dd > best * prune_th) {
                        blk &= ~(1u << li);
                        continue;
                    }
                }
                if (min_list != -1 && min_list != li) {
                    if (use)
                        o->me_mv_array[pu][li ? max_l0 : 0] = st.rec[li * 4][SVTME_PU_COUNT + n];
                    continue;
                }
                if (use) {
                    const uint8_t cb               = mk_cand(li, 0, 0, li == 0 ? li : 24, li == 1 ? li : 24);
                    o->me_candidate_array[pu][off] = cb;
                    if (off == 0)
                        c0 = cb;
                    o->me_mv_array[pu][li ? max_l0 : 0] = st.rec[li * 4][SVTME_PU_COUNT + n];
                }
                off++;
            }
            if ((blk & 3u) == 3u && use) {
                const uint8_t cb               = mk_cand(2, 0, 0, 0, 1);
                o->me_candidate_array[pu][off] = cb;
                if (off == 0)
                    c0 = cb;
                o->total_me_candidate_index[pu] = (uint8_t)(off + 1);
            }
            st.cand0[pu] = c0;
        } else { // construct_me_candidate_array (:2532-2835), the slots' SADs in registers
            // slot s = li * 4 + r searched (do_ref) for r < nr[li]; the best SAD over them
            // (a slot without do_ref takes no part)
            static_assert(offsetof(StC, do_ref) % 4 == 0, "StC::do_ref: two dword reads");
            const uint32_t dr0 = ((const uint32_t *)st.do_ref)[0], dr1 = ((const uint32_t *)st.do_ref)[1];
            const uint32_t slots = UNI((0xFu >> (4 - nr0)) | ((0xFu >> (4 - nr1)) << 4)); // r < nr[li]
            // every slot's SAD and MV read at once (one LDS round trip; a read under a
            // per-slot branch waits for each): the slots outside `slots` are masked
            uint32_t sad[8], mvs[8], blk = 0, best = U32MAX;
#pragma unroll
            for (int s2 = 0; s2 < 8; s2++) {
                sad[s2] = st.rec[s2][n];
                mvs[s2] = st.rec[s2][SVTME_PU_COUNT + n];
            }
#pragma unroll
            for (int s2 = 0; s2 < 8; s2++) {
                const int r   = s2 & 3;
                const bool in = ((slots >> s2) & 1u) && (((s2 < 4 ? dr0 : dr1) >> (8 * r)) & 0xFFu) != 0;
                sad[s2]       = in ? sad[s2] : U32MAX;
                blk |= in ? 1u << s2 : 0u;
                best = min_u32(best, sad[s2]);
            }
            o->me_distortion[pu] = best;
            // pruning of the unipred candidates (each against the best alone; a slot
            // outside blk has no bit to clear)
            const uint32_t prune_th = (uint32_t)job.ctrl.prune_me_candidates_th;
            if (prune_th > 0) {
                const uint32_t bt = best * prune_th;
#pragma unroll
                for (int s2 = 0; s2 < 8; s2++)
                    if ((slots >> s2) & 1u) // wave-uniform
                        blk &= (sad[s2] - best) * 100u > bt ? ~(1u << s2) : ~0u;
            }
            // the list as a mask over the potential candidates in the reference's order:
            // bit s2 unipred (list, ref) (:2597-2628), 8 + 4 a + b bipred L0 a x L1 b
            // (:2705-2732), 24 + a - 1 L0-L0 (0, a) (:2737-2760), 27 L1-L1 (0, 2) (:2763-2790)
            const bool lbwd = SF(job, only_l_bwd) != 0;
            const uint32_t m1 = (blk >> 4) & 0xFu;
            uint32_t bip = 0;
#pragma unroll
            for (int a2 = 0; a2 < 4; a2++)
                bip |= (((blk >> a2) & 1u) * m1) << (4 * a2);
            uint32_t cm = blk; // (no list-1 bits with one list)
            if (nl == 2) {
                cm |= (lbwd ? bip & 1u : bip) << 8;
                if (!lbwd)
                    cm |= ((blk & 1u) ? ((blk >> 1) & 7u) << 24 : 0u) |
                          ((nr1 == 3 && ((blk >> 4) & 1u) && ((blk >> 6) & 1u)) ? 1u << 27 : 0u);
            }
            cm = use ? cm : 0u;
            // the first candidate (GM detection reads it; 0 for a PU without candidates)
            const uint32_t f = (uint32_t)__builtin_ctz(blk | 0x100u), fl = f >> 2;
            st.cand0[pu]     = (uint8_t)((use && blk) ? fl | ((f & 3u) * 0x14u) | (fl << 7) : 0u);
            // candidate p goes to position popcount(cm below p): every potential candidate is
            // stored in order, one absent from the list at the position of the next present
            // one (which overwrites it) or at the list's end (cleared after the loop)
            uint32_t can = slots;
            if (nl == 2) {
                uint32_t bp = 0;
                for (int a2 = 0; a2 < nr0; a2++)
                    bp |= (0xFu >> (4 - nr1)) << (4 * a2);
                can |= (lbwd ? bp & 1u : bp) << 8;
                if (!lbwd)
                    can |= (((0xFu >> (4 - nr0)) >> 1) << 24) | (nr1 == 3 ? 1u << 27 : 0u);
            }
            can = UNI(can);
            uint8_t *ca = o->me_candidate_array[pu];
#pragma unroll
            for (int q = 0; q < 28; q++) {
                if (!((can >> q) & 1u))
                    continue; // wave-uniform
                const uint32_t v = q < 4 ? (uint32_t)q * 0x14u : q < 8 ? 0x81u | (uint32_t)(q & 3) * 0x14u
                                   : q < 24 ? 0x82u | (uint32_t)(((q - 8) >> 2) << 2) | (uint32_t)(((q - 8) & 3) << 4)
                                   : q < 27 ? 0x02u | (uint32_t)((q - 23) << 4) : 0xE2u;
                ca[__builtin_popcount(cm & ((1u << q) - 1u))] = (uint8_t)v;
            }
            const uint32_t cnt = (uint32_t)__builtin_popcount(cm);
            if (cnt < SVTME_MAX_PA_ME_CAND)
                ca[cnt] = 0;
            o->total_me_candidate_index[pu] = (uint8_t)cnt;
            // the unipred candidates' MVs (a PU without them writes to st.sink)
#pragma unroll
            for (int s2 = 0; s2 < 8; s2++) {
                if (!((slots >> s2) & 1u))
                    continue; // wave-uniform
                uint32_t *dst = ((cm >> s2) & 1u) ? &o->me_mv_array[pu][(s2 >> 2 ? max_l0 : 0) + (s2 & 3)] : &st.sink;
                *dst          = mvs[s2];
            }
        }
    }
}

__device__ __forceinline__ void finish_sb_out(StC &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh) {
    static_assert(offsetof(svtme_sb_result, me_8x8_cost_variance) ==
                          offsetof(svtme_sb_result, me_distortion) + 4 * SVTME_PU_COUNT &&
                      offsetof(svtme_sb_result, stationary_block_present) ==
                          offsetof(svtme_sb_result, me_8x8_cost_variance) + 24 &&
                      sizeof(svtme_sb_result) == offsetof(svtme_sb_result, stationary_block_present) + 8,
                  "svtme_sb_result tail: 6 distortion words, then the GM flag bytes and padding");
    constexpr int NIMG = (int)(offsetof(svtme_sb_result, me_8x8_cost_variance) / 4); // words stored from the image
    constexpr int WDIST = NIMG, WGM = NIMG + 6;                                         // tail words
    const svtme_job &job = dj.job;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const bool mctf = SF(job, me_type) == SVTME_ME_MCTF; // (no candidates / distortions, motion_estimation.c:3126)
    const bool en8 = SF(job, enable_me_8x8) != 0, en16 = SF(job, enable_me_16x16) != 0;
    uint32_t *img      = (uint32_t *)&st.keys[0][0];
    svtme_sb_result *o = (svtme_sb_result *)img;
    uint32_t *ow       = (uint32_t *)(dj.out_sb + sb_local);
    if (wid >= 2) {
        // the image up to me_distortion: the result is 4-byte aligned (sizeof 4796),
        // so up to 3 head words, 16-byte stores, up to 3 tail words
        const int t     = tid - 128;
        const int head  = (int)((16u - ((uint32_t)(uintptr_t)ow & 15u)) & 15u) >> 2;
        const int n16   = (NIMG - head) >> 2;
        const int tail0 = head + 4 * n16;
        for (int i = t; i < n16; i += 128) {
            const uint32_t *v = img + head + 4 * i;
            *(uint4 *)(ow + head + 4 * i) = make_uint4(v[0], v[1], v[2], v[3]);
        }
        if (t >= 128 - 8) { // head: j < head, tail: tail0 + (j - 4)
            const int j = t - (128 - 8);
            if (j < head)
                ow[j] = img[j];
            else if (j >= 4 && tail0 + (j - 4) < NIMG)
                ow[tail0 + (j - 4)] = img[tail0 + (j - 4)];
        }
    } else if (wid == 0) {
        // compute_distortion (motion_estimation.c:2964-3007): lane-parallel sums; the 6 words to HBM
        uint32_t w6 = 0;
        if (!mctf) {
            const uint32_t d8v  = o->me_distortion[21 + lane];
            const uint32_t d16v = lane < 16 ? o->me_distortion[5 + lane] : 0;
            const uint32_t d32v = lane < 4 ? o->me_distortion[1 + lane] : 0;
            const uint32_t d8 = wave_sum_u32(d8v), d16 = wave_sum_u32(d16v), d32 = wave_sum_u32(d32v);
            const uint32_t d64  = o->me_distortion[0];
            const uint64_t mean = d8 / 64;
            const int64_t diff  = (int64_t)d8v - (int64_t)mean;
            const uint64_t sq1  = (uint64_t)(diff * diff); // < 2^42: 24-bit limbs sum exactly in 32 bits
            const uint64_t sq   = ((uint64_t)wave_sum_u32((uint32_t)(sq1 >> 24)) << 24) +
                                (uint64_t)wave_sum_u32((uint32_t)(sq1 & 0xFFFFFFu));
            const uint32_t pix  = bw * bh;
            // (d * 4096) / pix in 32-bit arithmetic, one division per lane (a shift for a whole SB)
            const uint32_t dd = lane == 2 ? d64 : lane == 3 ? d32 : lane == 4 ? d16 : d8;
            const uint32_t x  = dd * 4096u;
            const uint32_t nd = pix == 4096u ? x >> 12 : x / pix;
            w6 = lane == 0 ? (uint32_t)(sq / 64)                        // me_8x8_cost_variance
                 : lane == 1 ? ((SF(job, input_resolution) <= 2) ? d8 : d16) // rc_me_distortion
                             : nd;                                      // me_{64x64,32x32,16x16,8x8}_distortion
        }
        if (lane < 6)
            ow[WDIST + lane] = w6;
    } else {
        // perform_gm_detection (motion_estimation.c:2838-2961): one lane per block; the
        // direction counters are LDS adds, the stationary count a ballot; the flag
        // bytes (stationary_block_present, rc_me_allow_gm) and the padding to HBM
        uint32_t flags = 0;
        if (!mctf && SF(job, gm_enabled)) {
            uint32_t *cntf = &st.gm_cnt[0][0][0][0];
            if (lane < 32)
                cntf[lane] = 0;
            wave_lds_fence();
            const bool low  = SF(job, input_resolution) <= 2;
            const bool gmd  = SF(job, gm_use_distance_based_active_th) != 0;
            const int n_blk = low ? 64 : 16;
            bool stat       = false;
            if (lane < n_blk) {
                uint8_t n = (uint8_t)(low ? 21 + lane : 5 + lane);
                if (low && !en8) {
                    if (n >= 21)
                        n = c_8x8_to_16x16[n - 21];
                    if (!en16 && n >= 5)
                        n = c_16x16_to_32x32[n - 5];
                }
                if (!low && !en16 && n >= 5)
                    n = c_16x16_to_32x32[n - 5];
                const uint8_t cb = st.cand0[n];
                const int dir = cb & 3, r0 = (cb >> 2) & 3, r1 = (cb >> 4) & 3, l0 = (cb >> 6) & 1, l1 = (cb >> 7) & 1;
                const int li = (dir == 0 || dir == 2) ? l0 : l1;
                const int ri = (dir == 0 || dir == 2) ? r0 : r1;
                int active_th;
                uint64_t rp = 0; // ref_picture_number[li][ri]: uniform loads, a per-lane select
#pragma unroll
                for (int q = 0; q < 8; q++)
                    rp = (li * 4 + ri == q) ? job.ref_picture_number[q >> 2][q & 3] : rp;
                if (low) {
                    const uint64_t a2 = job.picture_number, b2 = rp;
                    const uint16_t dist = (uint16_t)absi((int16_t)((a2 > b2 ? a2 : b2) - (a2 < b2 ? a2 : b2)));
                    active_th = gmd ? max(dist >> 1, 4) : 4;
                } else {
                    const uint16_t dist = (uint16_t)absi((int16_t)(job.picture_number - rp));
                    active_th = gmd ? max(dist * 16, 32) : 32;
                }
                const uint32_t mv = st.rec[li * 4 + ri][SVTME_PU_COUNT + n];
                const int mx = (int)(int16_t)(mv & 0xFFFF) * 4, my = (int)(int16_t)(mv >> 16) * 4;
                uint32_t(*cnt)[4][2][2] = st.gm_cnt;
                if (mx < -active_th)
                    atomicAdd(&cnt[li][ri][0][0], 1u);
                else if (mx > active_th)
                    atomicAdd(&cnt[li][ri][0][1], 1u);
                if (my < -active_th)
                    atomicAdd(&cnt[li][ri][1][0], 1u);
                else if (my > active_th)
                    atomicAdd(&cnt[li][ri][1][1], 1u);
                const int stt = low ? 0 : 4;
                stat          = absi(mx) <= stt && absi(my) <= stt;
            }
            const uint64_t stationary = (uint64_t)__popcll(__ballot(stat)), tot = (uint64_t)n_blk;
            wave_lds_fence();
            const bool over = lane < 32 && cntf[lane] > (tot / 2);
            const bool any  = __ballot(over) != 0ull;
            flags = (stationary > ((tot * 5) / 100) ? 1u : 0u) | (any ? 1u << 8 : 0u);
        }
        if (lane < 2)
            ow[WGM + lane] = lane == 0 ? flags : 0u;
    }}

__device__ __forceinline__ void finish_sb(StC &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh) {
    finish_sb_cands(st, dj, sb_local, bw, bh);
    __syncthreads();
    HME_SUB(20);
    finish_sb_out(st, dj, sb_local, bw, bh);
}

// the records (sb_count x R, slots in list-0-then-list-1 order) by threads [t0, t0 + nt): the
// LDS record images, 44 16-byte pieces each (704 bytes), the tail words and the SADs of an
// unsearched slot patched on the way
__device__ __forceinline__ void write_records(const StC &st, const DevJob &dj, uint32_t sb_local, int t, int nt) {
    static_assert(sizeof(svtme_ref_record) == 176 * 4, "svtme_ref_record: 176 dwords");
    svtme_ref_record *out = dj.out_records + (size_t)sb_local * dj.R;
    const int R = (int)dj.R, nr0 = (int)SF(dj.job, num_refs[0]);
    for (int i = t; i < R * 44; i += nt) {
        const int k = i / 44, q = i - 44 * k;
        const int s = k < nr0 ? k : 4 + (k - nr0);
        uint4 v     = ((const uint4 *)st.rec[s])[q];
        if (q < 22 && !st.searched[s]) { // words 0 .. 87: the SADs (< 85) of an unsearched slot
            if (4 * q + 0 < 85) v.x = U32MAX;
            if (4 * q + 1 < 85) v.y = U32MAX;
            if (4 * q + 2 < 85) v.z = U32MAX;
            if (4 * q + 3 < 85) v.w = U32MAX;
        }
        if (q == 42) { // words 168, 169 (MVs), 170, 171: hme_sad
            v.z = (uint32_t)st.hme_sad[s];
            v.w = (uint32_t)(st.hme_sad[s] >> 32);
        } else if (q == 43) { // 172: search centre, 173: zz SAD, 174: flags, 175: 0
            v.x = (uint32_t)(uint16_t)st.sc_x[s] | ((uint32_t)(uint16_t)st.sc_y[s] << 16);
            v.y = st.zz[s];
            v.z = (uint32_t)st.searched[s] | ((uint32_t)st.do_ref[s] << 8) | ((uint32_t)st.tf_exit << 16);
            v.w = 0;
        }
        ((uint4 *)(out + k))[q] = v;
    }
}

// me_prune_ref, the per-reference records and the candidate arrays /
// distortions / GM detection of one SB from its searched best SADs and MVs
// (motion_estimation.c:1522-1565, 2520-3007); all threads of the workgroup
// SUMS: st.sum8 holds the 8x8 sums of the searched slots (stage_e_body made them),
// and the keys (under the svtme_sb_result image) are dead: waves 1-3 zero the image
// while wave 0 prunes, then waves 0-1 build the candidate arrays while waves 2-3
// write the records (one barrier less, the records off the critical path)
template <bool SUMS>
__device__ __forceinline__ void stage_c_tail(StC &st, const DevJob &dj, uint32_t sb_local, uint32_t bw, uint32_t bh, uint32_t vmask) {
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int tid = threadIdx.x, lane = tid & 63;
    const bool w0 = (tid >> 6) == 0;
    const bool sbr = dj.out_sb != nullptr;
    uint32_t *img  = (uint32_t *)&st.keys[0][0];
    // ---- me_prune_ref (motion_estimation.c:1522-1565)
    if (SF(job, me_type) != SVTME_ME_MCTF && SF(c, enable_hme_flag) && SF(c, enable_me_hme_ref_pruning) && w0) {
        const int s = lane;
        // the 64 8x8 best SADs of every searched slot, summed across the wave
        // (searched == do_ref outside MCTF: each SAD < 2^15, the sum fits 32 bits)
        uint32_t sum8 = 0;
        if (SUMS) {
            if (s < 8)
                sum8 = st.sum8[s];
        } else {
            for (int k = 0; k < 8; k++) {
                if (!(slot_valid(vmask, k) && st.do_ref[k]))
                    continue; // wave-uniform
                const uint32_t t = wave_sum_u32(st.rec[k][21 + lane]);
                if (lane == k)
                    sum8 = t;
            }
        }
        uint64_t v  = ~0ull;
        if (s < 8) {
            v = st.hme_sad[s];
            if (slot_valid(vmask, s)) {
                v             = st.do_ref[s] ? (uint64_t)sum8 : (uint64_t)SVTME_MAX_SAD_VALUE * 64;
                st.hme_sad[s] = v;
            }
        }
        const uint16_t th = (uint16_t)SF(c, prune_ref_if_me_sad_dev_bigger_than_th);
        if (th != (uint16_t)~0) {
            const uint64_t best = wave_min_u64(v);
            if (s < 8 && (s & 3) >= 1 && (v - best) * 100 > (th * best))
                st.do_ref[s] = 0;
        }
    }
    if (SUMS && sbr && !w0) // the svtme_sb_result image (finish_sb) starts zeroed
        for (int i = tid - 64; i < (int)(sizeof(svtme_sb_result) + 15) / 16; i += 192)
            ((uint4 *)img)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    HME_SUB(17);
    if (SUMS && sbr) {
        if (tid < 128)
            finish_sb_cands(st, dj, sb_local, bw, bh);
        else
            write_records(st, dj, sb_local, tid - 128, 128);
        HME_SUB(18);
        __syncthreads();
        HME_SUB(20);
        finish_sb_out(st, dj, sb_local, bw, bh);
        HME_SUB(21);
        return;
    }
    write_records(st, dj, sb_local, tid, 256);
    HME_SUB(18);
    if (sbr) {
        for (int i = tid; i < (int)(sizeof(svtme_sb_result) + 15) / 16; i += 256)
            ((uint4 *)img)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        HME_SUB(19);
        finish_sb(st, dj, sb_local, bw, bh);
        HME_SUB(21);
    }
}

template <bool SUB_ME>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_stage_c(const DevBatch B) {
    __shared__ StC st;
    uint32_t sb_local;
    const DevJob &dj        = batch_job(B, xcd_remap(blockIdx.x, gridDim.x), &sb_local);
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool w0           = wid == 0;
    const SbGeo G           = sb_geo(dj, sb_local);
    const uint32_t ox = G.ox, oy = G.oy, bw = G.bw, bh = G.bh;
    const uint32_t vmask = valid_mask(job);

    const DevPlane &C = dj.cur.lv[0]; // source block read in place (me_process.c:183-214)
    if (tid == 0) {
#pragma unroll
        for (int s = 0; s < 8; s++) {
            st.pl[s][0]  = dj.ref[s >> 2][s & 3].lv[0];
            st.dist[s]   = ref_dist_const(job, s >> 2, s & 3);
            st.refpic[s] = job.ref_picture_number[s >> 2][s & 3];
        }
    }
    if (w0) {
        const SlotCentre sc = final_centre(job, dj.bst + sb_local, vmask);
        const uint64_t h0   = __shfl(sc.hme_sad, 0, 64);
        const bool tf_exit  = job.me_type == SVTME_ME_MCTF && h0 < job.tf_me_exit_th;
        if (lane < 8) {
            st.hme_sad[lane]    = sc.hme_sad;
            st.zz[lane]         = sc.zz;
            st.reduce_div[lane] = sc.reduce_div;
            st.sc_x[lane]       = sc.sc_x;
            st.sc_y[lane]       = sc.sc_y;
            st.do_ref[lane]     = sc.do_ref;
            st.searched[lane]   = tf_exit ? 0 : sc.do_ref;
        }
        if (lane == 0)
            st.tf_exit = tf_exit;
    }
    for (int e = tid; e < 8 * SVTME_PU_COUNT; e += 256) st.rec[e / SVTME_PU_COUNT][SVTME_PU_COUNT + e % SVTME_PU_COUNT] = 0;
    __syncthreads();

    // ---- integer_search_b64 (motion_estimation.c:1249-1516); lane s of wave 0 owns slot s.
    // Two rounds when enable_me_sr_adjustment == 2: the other slots read slot 0's 64x64 SAD.
    const int rounds = c.enable_me_sr_adjustment == 2 ? 2 : 1;
    for (int round = 0; round < rounds; round++) {
        if (w0) { // search area up to the 8x8-variance decision
            const int s = lane, r = s & 3;
            const bool act = slot_valid(vmask, s) && (rounds == 1 || ((s == 0) == (round == 0))) && st.searched[s];
            bool need = false;
            if (act) {
                int16_t xc = st.sc_x[s], yc = st.sc_y[s];
                int16_t w = (int16_t)c.me_sa.sa_min.width, h = (int16_t)c.me_sa.sa_min.height;
                const uint16_t dist = job.me_type == SVTME_ME_MCTF ? st.dist[s] : scaled_dist(st.dist[s]);
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
            for (int q = wid; q < 2 * st.nreq; q += 4) {
                const uint32_t v = wave_nxm(st.req[q], st.req_stride[q], C.base + (ptrdiff_t)oy * C.stride + ox,
                                            2 * C.stride, (int)(bh >> 1), (int)bw);
                if (lane == 0)
                    st.nxm[q] = v;
            }
            __syncthreads();
            if (w0 && lane < st.nreq) {
                const int s             = st.req_slot[lane];
                const uint32_t zero_sad = st.nxm[2 * lane] << 1, hme_mv_sad = st.nxm[2 * lane + 1] << 1;
                const uint64_t zc = (uint64_t)zero_sad << 8, hc = (uint64_t)hme_mv_sad << 8;
                if (min_u64(zc, hc) == zc) {
                    st.is_xc[s] = 0;
                    st.is_yc[s] = 0;
                }
                st.is_best_hme[s] = hme_mv_sad;
            }
        }
        if (w0) { // sr adjustment level 2, 8x8-variance centre probe setup
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
                        if ((l || r) && st.rec[0][0] < 5000 && h == st.is_hb[s] && w == st.is_wb[s]) {
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
                make_fp(st.fp[k], st.pl[s][0], ox, oy, s, st.is_xc[s], st.is_yc[s], 1, 1, 0);
            plan_fp(st, probe, k, tot);
            if (lane == 0)
                st.k32 = 1; // a single position
        }
        __syncthreads();
        for (int e = tid; e < 8 * SVTME_PU_COUNT; e += 256) {
            const int s = e / SVTME_PU_COUNT;
            if (st.in_round[s])
                st.rec[e / SVTME_PU_COUNT][e % SVTME_PU_COUNT] = SVTME_MAX_SAD_VALUE;
        }
        if (st.nfp) {
            fullpel<SUB_ME>(st, C, ox, oy); // centre probe (motion_estimation.c:1414-1417)
            // 8x8-variance resize (motion_estimation.c:1418-1438)
            if (w0 && lane < 8 && st.in_round[lane] && c.me_8x8_var_enabled && (st.is_w[lane] * st.is_h[lane] > 24)) {
                const int s = lane;
                int16_t w = st.is_w[s], h = st.is_h[s];
                const uint32_t mean = st.rec[s][0] / 64;
                uint32_t sum_sq     = 0;
                for (int i = 0; i < 64; i++) {
                    const int32_t diff = (int32_t)st.rec[s][21 + i] - (int32_t)mean;
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
        if (w0) { // final area clamp + main full-pel search (motion_estimation.c:1440-1516)
            const int s = lane;
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
                make_fp(st.fp[k], st.pl[s][0], ox, oy, s, xo, yo, w, h, 1);
            plan_fp(st, act, k, tot);
            const bool k32 = __all(!act || (1 + (int)w * (int)h <= 4096));
            if (lane == 0)
                st.k32 = k32;
        }
        __syncthreads();
        if (st.nfp)
            fullpel<SUB_ME>(st, C, ox, oy);
    }

    stage_c_tail<false>(st, dj, sb_local, bw, bh, vmask);
}

// ----------------------------------------------------------------------------
// Stage C, wide form: one wavefront per (SB, reference slot, band of search
// rows) runs that slot's integer_search_b64 (motion_estimation.c:1249-1516);
// k_stage_e then decodes the 85-PU argmins per SB and runs me_prune_ref, the
// records and the candidate arrays. A slot's search area depends on no other
// slot's search unless enable_me_sr_adjustment == 2 (slot 0's 64x64 SAD,
// :1355-1364), which keeps the per-SB k_stage_c.
// ----------------------------------------------------------------------------
// Running 85-PU minima of one lane (lane = 8x8 block in Z order). The 16x16,
// 32x32 and 64x64 SADs are DPP lane sums (64x64 valid in lanes 48-63). Keys
// are (sad << 12 | order) in 32 bits when every order < 4096 (a 64x64 SAD is
// below 2^20), else (sad << 32 | order).
template <bool K32>
struct PuMin {
    typedef typename std::conditional<K32, uint32_t, unsigned long long>::type key_t;
    key_t b8, b16, b32, b64;
    __device__ __forceinline__ void clear() { b8 = b16 = b32 = b64 = (key_t)~0ull; }
    __device__ __forceinline__ static key_t make(uint32_t sad, uint32_t o) {
        if (K32)
            return (key_t)((sad << 12) | o);
        return (key_t)(((unsigned long long)sad << 32) | o);
    }
    __device__ __forceinline__ void add(uint32_t s8, uint32_t o) {
        const uint32_t s16 = dpp_add<0x4E>(dpp_add<0xB1>(s8));              // xor 1, xor 2
        const uint32_t s32 = dpp_add<0x128>(dpp_add<0x124>(s16));           // row_ror 4, 8
        const uint32_t s64 = dpp_add<0x143, 0xC>(dpp_add<0x142, 0xA>(s32)); // valid in row 3
        const key_t k8 = make(s8, o), k16 = make(s16, o), k32 = make(s32, o), k64 = make(s64, o);
        b8  = k8 < b8 ? k8 : b8;
        b16 = k16 < b16 ? k16 : b16;
        b32 = k32 < b32 ? k32 : b32;
        b64 = k64 < b64 ? k64 : b64;
    }
    // K32 search (fp_rows32): SADs stay raw (SUB: the 8x4 sums, doubled only by
    // out()); b8 keys are (sad << 16 | order) (an 8x8 SAD < 2^15), b16 / b32 / b64
    // (sad << 12 | order). Two aligned position quads, a = x0 + e and b = x0 + 4
    // + e (orders o0 + e, o0 + 4 + e), SADs packed as u16 pairs (l: e = 0, 1;
    // h: e = 2, 3). The 8x8 minima take all 8 positions per lane; the 16x16 /
    // 32x32 minima are lane-specialised: lane g = lane & 3 of each 4-lane group
    // keeps positions = g (mod 4) (16x16 sums on the packed pairs, <= 32640);
    // the 64x64 minima in addition by row: one permlane16_swap sums the 32x32
    // quadrant pairs of both quads, rows with qb = 1 keep quad b. finalize()
    // reduces the classes.
    // INNER: both quads inside the area (the caller's wave-uniform test).
    template <bool INNER>
    __device__ __forceinline__ void add_quads(uint32_t la, uint32_t ha, uint32_t lb, uint32_t hb, uint32_t o0, int x0,
                                              int w, uint32_t qb) {
        const int g = threadIdx.x & 3;
        if (INNER) {
            b8 = min_u32(min_u32((uint32_t)b8, (la << 16) | o0), (la & 0xFFFF0000u) | (o0 + 1));
            b8 = min_u32(min_u32((uint32_t)b8, (ha << 16) | (o0 + 2)), (ha & 0xFFFF0000u) | (o0 + 3));
            b8 = min_u32(min_u32((uint32_t)b8, (lb << 16) | (o0 + 4)), (lb & 0xFFFF0000u) | (o0 + 5));
            b8 = min_u32(min_u32((uint32_t)b8, (hb << 16) | (o0 + 6)), (hb & 0xFFFF0000u) | (o0 + 7));
        } else {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int x = x0 + e;
                if (x < 0 || x >= w)
                    continue; // wave-uniform
                const uint32_t v = e < 2 ? la : e < 4 ? ha : e < 6 ? lb : hb;
                b8 = min_u32((uint32_t)b8, ((e & 1) ? (v & 0xFFFF0000u) : (v << 16)) | (o0 + e));
            }
        }
        // 16x16 by reduce-scatter over the 4 lanes of a group: lanes with g & 2 keep
        // the pair of positions 2, 3 and send 0, 1 (quad_perm xor 2), then both
        // halves of the pair are summed over xor 1; lane g takes position g
        const bool hi2 = (g & 2) != 0;
        const uint32_t A = dpp_add2<0x4E>(hi2 ? ha : la, hi2 ? la : ha);
        const uint32_t B = dpp_add2<0x4E>(hi2 ? hb : lb, hi2 ? lb : hb);
        const uint32_t sel  = (uint32_t)(g & 1) * 16;
        const uint32_t s16a = (dpp_add<0xB1>(A) >> sel) & 0xFFFFu;
        const uint32_t s16b = (dpp_add<0xB1>(B) >> sel) & 0xFFFFu;
        const uint32_t s32a = dpp_add<0x128>(dpp_add<0x124>(s16a)); // row_ror 4, 8: same g
        const uint32_t s32b = dpp_add<0x128>(dpp_add<0x124>(s16b));
        const uint32_t oa = o0 + (uint32_t)g, ob = oa + 4, o64 = oa + 4 * qb;
        const int xa = x0 + g, xb = xa + 4;
        // the 16x16 / 32x32 keys before the swap below consumes s32a / s32b
        if (INNER) {
            b16 = min_u32(min_u32((uint32_t)b16, (s16a << 12) | oa), (s16b << 12) | ob);
            b32 = min_u32(min_u32((uint32_t)b32, (s32a << 12) | oa), (s32b << 12) | ob);
        } else {
            if (xa >= 0 && xa < w) {
                b16 = min_u32((uint32_t)b16, (s16a << 12) | oa);
                b32 = min_u32((uint32_t)b32, (s32a << 12) | oa);
            }
            if (xb >= 0 && xb < w) {
                b16 = min_u32((uint32_t)b16, (s16b << 12) | ob);
                b32 = min_u32((uint32_t)b32, (s32b << 12) | ob);
            }
        }
        // 64x64: rows 2j, 2j + 1 of the swap hold one quad's quadrants 2j + 1 and
        // 2j, which quad is qb; the permlane32_swap of the sum with itself adds
        // the other row pair
        const auto p16     = __builtin_amdgcn_permlane16_swap(s32a, s32b, false, false);
        const uint32_t t   = p16[0] + p16[1];
        const auto p32     = __builtin_amdgcn_permlane32_swap(t, t, false, false);
        const uint32_t s64 = p32[0] + p32[1];
        if (INNER) {
            b64 = min_u32((uint32_t)b64, (s64 << 12) | o64);
        } else {
            const int x64 = xa + 4 * (int)qb;
            if (x64 >= 0 && x64 < w)
                b64 = min_u32((uint32_t)b64, (s64 << 12) | o64);
        }
    }
    // K32: the 8x8-variance centre probe (order 0): this lane's raw 8x8 SAD; every
    // lane class takes the position, so no finalize() is needed before the search
    __device__ __forceinline__ void add_probe(uint32_t s8) {
        const uint32_t s16 = dpp_add<0x4E>(dpp_add<0xB1>(s8));
        const uint32_t s32 = dpp_add<0x128>(dpp_add<0x124>(s16));
        b8  = min_u32((uint32_t)b8, s8 << 16);
        b16 = min_u32((uint32_t)b16, s16 << 12);
        b32 = min_u32((uint32_t)b32, s32 << 12);
        const auto p16     = __builtin_amdgcn_permlane16_swap(s32, s32, false, false);
        const uint32_t t   = p16[0] + p16[1];
        const auto p32     = __builtin_amdgcn_permlane32_swap(t, t, false, false);
        b64 = min_u32((uint32_t)b64, (p32[0] + p32[1]) << 12);
    }
    // the quad of every lane's 64x64 sums in add_quads (the rows permlane16_swap
    // takes from its second operand)
    __device__ __forceinline__ static uint32_t quad_b_rows() {
        return __builtin_amdgcn_permlane16_swap(0u, 1u, false, false)[0];
    }
    // K32 after add_quads: b16 / b32 over the 4 lanes of each group, b64 over
    // the wave (idempotent: the search may go on afterwards)
    __device__ __forceinline__ void finalize() {
        if (K32) {
            b16 = quad_min((uint32_t)b16);
            b32 = quad_min((uint32_t)b32);
            uint32_t v     = quad_min((uint32_t)b64);
            const auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            v              = min_u32(p16[0], p16[1]);
            const auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            b64            = min_u32(p32[0], p32[1]);
        }
    }
    // (sad << 32 | order) of a minimum, ~0 if none: K32 keys converted, SUB
    // SADs doubled (8x4 sums of every other row)
    template <bool SUB>
    __device__ __forceinline__ static unsigned long long out(key_t k, bool is8) {
        if (K32) {
            const uint32_t v = (uint32_t)k;
            if (v == 0xFFFFFFFFu)
                return ~0ull;
            const uint32_t sad = (is8 ? v >> 16 : v >> 12) << (SUB ? 1 : 0);
            return ((unsigned long long)sad << 32) | (is8 ? (v & 0xFFFFu) : (v & 0xFFFu));
        }
        return (unsigned long long)k;
    }
    __device__ __forceinline__ static uint32_t quad_min(uint32_t v) {
        v = min_u32(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
        return min_u32(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    }
};

// Full-pel SADs of this lane's 8x8 block (source rows src) at search rows
// [y0, y1) x columns [0, w) of a window (a = dword-aligned address of window
// row 0, sh = byte offset of column 0, nq = aligned position quads per row),
// in TY x TQ tiles: the reference rows and dwords of a tile are loaded once,
// all in flight together, and shared by its TY x TQ position quads. Orders are
// obase + y * w + x (raster order, motion_estimation.c:781-817).
template <bool SUB, bool K32, int TQ>
__device__ __forceinline__ void fp_rows(PuMin<K32> &M, const uint32_t *a, int sdw, int sh, int w, int nq, int y0,
                                        int y1, uint32_t obase, const uint32_t (&src)[SUB ? 4 : 8][2], int by,
                                        int bx) {
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1, TY = 1; // taller tiles cost registers (aligned qsad pairs)
    constexpr int NR = TY + (ROWS - 1) * RSTEP, ND = TQ + 2;
    // uniform row bases (SGPRs) + one per-lane dword offset: every load is
    // saddr + voffset + immediate
    const uint32_t lo = (uint32_t)((by * 8) * sdw + bx * 2);
    for (int ty = y0; ty < y1; ty += TY) {
        const int ny       = min(TY, y1 - ty);
        const int last_row = ny - 1 + (ROWS - 1) * RSTEP;
        for (int tq = 0; tq < nq; tq += TQ) {
            const int nqq = min(TQ, nq - tq);
            uint32_t T[NR][ND];
#pragma unroll
            for (int i = 0; i < NR; i++) {
                const uint32_t *rowp = uni_ptr(a + (ptrdiff_t)(ty + min(i, last_row)) * sdw + tq);
#pragma unroll
                for (int j = 0; j < ND; j++) T[i][j] = rowp[lo + (uint32_t)min(j, nqq + 1)];
            }
#pragma unroll
            for (int iy = 0; iy < TY; iy++) {
                if (iy >= ny)
                    break; // wave-uniform
#pragma unroll
                for (int iq = 0; iq < TQ; iq++) {
                    if (iq >= nqq)
                        break; // wave-uniform
                    unsigned long long acc = 0;
#pragma unroll
                    for (int rr = 0; rr < ROWS; rr++) {
                        acc = qsad(T[iy + rr * RSTEP][iq], T[iy + rr * RSTEP][iq + 1], src[rr][0], acc);
                        acc = qsad(T[iy + rr * RSTEP][iq + 1], T[iy + rr * RSTEP][iq + 2], src[rr][1], acc);
                    }
                    const int y = ty + iy;
                    static_assert(!K32, "K32 keys: fp_rows32");
                    {
                        uint32_t s4[4] = {0, 0, 0, 0};
                        qsad_unpack(acc, s4);
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            const int x = 4 * (tq + iq) - sh + k;
                            if (x >= 0 && x < w) // wave-uniform
                                M.add(SUB ? s4[k] << 1 : s4[k], obase + (uint32_t)(y * w + x));
                        }
                    }
                }
            }
        }
    }
}

#define FP_TQ 3 // position quads per full-pel tile (sub-sampled rows; 2 for full rows)

// K32 form of fp_rows: position quads in pairs from position 0 of the window
// g at any byte alignment: dword-aligned buffer loads (uniform row offset +
// the lane's offset, no VALU address work) realigned with v_alignbyte, every
// bound wave-uniform. Reads up to 4 bytes right of the window (plane margins /
// allocation slack).
template <bool SUB, int TQ = 2> // TQ: position quads per load set (2: one 16-byte load per row, 6: two)
__device__ __forceinline__ void fp_rows32(PuMin<true> &M, const uint8_t *g, int sdw, int w, int y0, int y1,
                                          uint32_t obase, const uint32_t (&src)[SUB ? 4 : 8][2], int by, int bx) {
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1;
    g     = uni_ptr(g);
    sdw   = UNI(sdw);
    w     = UNI(w);
    const int nq = (w + 3) >> 2; // the quads start at position 0
    y0    = UNI(y0);
    y1    = UNI(y1);
    obase = (uint32_t)UNI(obase);
    static_assert(TQ % 2 == 0, "position quads go in pairs");
    const uint32_t qb = PuMin<true>::quad_b_rows();
    const uint32_t lo = (uint32_t)((by * 8) * sdw + bx * 2);
    // one load set: rows of quads [tq, tq + TQ) of search row ty
    const int sh = (int)((uintptr_t)g & 3); // the loads stay dword aligned
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(g - sh);
    auto set = [&](int ty, int tq, auto inner) {
        const uint32_t rb = (uint32_t)(ty * sdw + tq) * 4u;
        // dword-aligned loads of TQ + 3 dwords, realigned to position 0 (v_alignbyte)
        constexpr int NX = (TQ + 3) / 4, NR = (TQ + 3) - 4 * NX;
        // rows in batches (2 full rows): the 8 full rows of a non-sub-sampled set would hold
        // 8 (TQ + 3) dwords beside the 16 of the source and spill at 64 VGPRs
        constexpr int RB = SUB ? 4 : 2;
        unsigned long long acc[TQ];
#pragma unroll
        for (int iq = 0; iq < TQ; iq++) acc[iq] = 0;
#pragma unroll
        for (int r0 = 0; r0 < ROWS; r0 += RB) {
            uint32_t D[RB][TQ + 3];
#pragma unroll
            for (int rr = 0; rr < RB; rr++) {
                const uint32_t ro = rb + (uint32_t)((r0 + rr) * RSTEP * sdw) * 4u;
#pragma unroll
                for (int v = 0; v < NX; v++) {
                    const u32x4a4 t = bld4(rs, (lo + 4 * v) * 4u, ro);
                    D[rr][4 * v] = t.x, D[rr][4 * v + 1] = t.y, D[rr][4 * v + 2] = t.z, D[rr][4 * v + 3] = t.w;
                }
#pragma unroll
                for (int v = 0; v < NR; v++)
                    D[rr][4 * NX + v] =
                        (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)((lo + 4 * NX + v) * 4u), (int)ro, 0);
#pragma unroll
                for (int j = 0; j < TQ + 2; j++)
                    D[rr][j] = __builtin_amdgcn_alignbyte(D[rr][j + 1], D[rr][j], (uint32_t)sh);
            }
#pragma unroll
            for (int rr = 0; rr < RB; rr++)
#pragma unroll
                for (int iq = 0; iq < TQ; iq++) {
                    acc[iq] = qsad64(pair(D[rr][iq], D[rr][iq + 1]), src[r0 + rr][0], acc[iq]);
                    acc[iq] = qsad64(pair(D[rr][iq + 1], D[rr][iq + 2]), src[r0 + rr][1], acc[iq]);
                }
        }
        const int x0      = 4 * tq;
        const uint32_t ob = obase + (uint32_t)(ty * w + x0);
#pragma unroll
        for (int iq = 0; iq < TQ; iq += 2) {
            if (!decltype(inner)::value && iq > 0 && tq + iq >= nq)
                break; // wave-uniform (a second quad past nq lies right of the area)
            M.template add_quads<decltype(inner)::value>((uint32_t)acc[iq], (uint32_t)(acc[iq] >> 32),
                                                         (uint32_t)acc[iq + 1], (uint32_t)(acc[iq + 1] >> 32),
                                                         ob + 4 * iq, x0 + 4 * iq, w, qb);
        }
    };
    // load sets wholly inside the area: tq < t_out (wave-uniform; every set when
    // w is a multiple of 4 TQ, as the 8-aligned full-pel widths are for TQ = 2)
    const int t_out = w >= 4 * TQ ? (w - 4 * TQ) / (4 * TQ) * TQ + TQ : 0;
    for (int ty = y0; ty < y1; ty++) {
        for (int tq = 0; tq < t_out; tq += TQ)
            set(ty, tq, std::true_type());
        for (int tq = t_out; tq < nq; tq += TQ)
            set(ty, tq, std::false_type()); // the right edge
    }
}




// the whole-area shapes k_hme takes (fp_slot WHOLE bits: 1 full rows 8 x 8, 2 sub-sampled 8 x 3 / 8 x 4)
#define HME_WHOLE 2
// K32, an area 8 wide searched whole (TF-ME level 2: 8 x 8 full rows; the p8
// searches: 8 x 3 / 8 x 4 sub-sampled rows): every reference row of the lane's
// block is loaded and realigned once and feeds each (search row, block row) pair
// it belongs to, instead of once per pair (8 x 8 full rows: 15 row loads instead
// of 64; 8 x 4 sub-sampled: 10 instead of 16). Only search rows of one parity
// share sub-sampled reference rows: fp_whole_class runs the NT search rows
// ty = c + NC j of parity class c (NC = 2 sub-sampled, 1 full rows).
template <bool SUB, int NT>
__device__ __forceinline__ void fp_whole_class(PuMin<true> &M, const __amdgpu_buffer_rsrc_t rs, uint32_t lo, int sdw,
                                               int sh, uint32_t qb, uint32_t obase, int c,
                                               const uint32_t (&src)[SUB ? 4 : 8][2]) {
    constexpr int ROWS = SUB ? 4 : 8, NC = SUB ? 2 : 1;
    unsigned long long acc[NT][2];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j][0] = acc[j][1] = 0;
#pragma unroll
    for (int k = 0; k < NT + ROWS - 1; k++) { // reference row c + NC k: block row k - j of search row j
        const uint32_t ro = (uint32_t)((c + NC * k) * sdw) * 4u;
        const u32x4a4 t4  = bld4(rs, lo, ro);
        const uint32_t t5 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(lo + 16u), (int)ro, 0);
        const uint32_t d0 = __builtin_amdgcn_alignbyte(t4.y, t4.x, (uint32_t)sh);
        const uint32_t d1 = __builtin_amdgcn_alignbyte(t4.z, t4.y, (uint32_t)sh);
        const uint32_t d2 = __builtin_amdgcn_alignbyte(t4.w, t4.z, (uint32_t)sh);
        const uint32_t d3 = __builtin_amdgcn_alignbyte(t5, t4.w, (uint32_t)sh);
#pragma unroll
        for (int j = 0; j < NT; j++) {
            const int r = k - j;
            if (r < 0 || r >= ROWS)
                continue;
            acc[j][0] = qsad64(pair(d0, d1), src[r][0], acc[j][0]);
            acc[j][0] = qsad64(pair(d1, d2), src[r][1], acc[j][0]);
            acc[j][1] = qsad64(pair(d1, d2), src[r][0], acc[j][1]);
            acc[j][1] = qsad64(pair(d2, d3), src[r][1], acc[j][1]);
        }
    }
#pragma unroll
    for (int j = 0; j < NT; j++)
        M.template add_quads<true>((uint32_t)acc[j][0], (uint32_t)(acc[j][0] >> 32), (uint32_t)acc[j][1],
                                   (uint32_t)(acc[j][1] >> 32), obase + (uint32_t)((c + NC * j) * 8), 0, 8, qb);
}

// the whole 8-wide area: full rows h = 8 (one class), sub-sampled h = 3 or 4
// (class 0: search rows 0, 2; class 1: row 1, or rows 1, 3)
template <bool SUB>
__device__ __forceinline__ void fp_rows32_whole(PuMin<true> &M, const uint8_t *g, int sdw, int h, uint32_t obase,
                                                const uint32_t (&src)[SUB ? 4 : 8][2], int by, int bx) {
    g     = uni_ptr(g);
    sdw   = UNI(sdw);
    h     = UNI(h);
    obase = (uint32_t)UNI(obase);
    const uint32_t qb = PuMin<true>::quad_b_rows();
    const int sh      = (int)((uintptr_t)g & 3);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(g - sh);
    const uint32_t lo = (uint32_t)((by * 8) * sdw + bx * 2) * 4u;
    if constexpr (SUB) {
        fp_whole_class<true, 2>(M, rs, lo, sdw, sh, qb, obase, 0, src);
        if (h == 4)
            fp_whole_class<true, 2>(M, rs, lo, sdw, sh, qb, obase, 1, src);
        else
            fp_whole_class<true, 1>(M, rs, lo, sdw, sh, qb, obase, 1, src);
    } else {
        // full rows: search rows 0-3, then 4-7 (11 row loads each instead of 15 for
        // all 8, but half the accumulators live: k_stage_c1 124 -> 104 VGPRs, -4 %)
        fp_whole_class<false, 4>(M, rs, lo, sdw, sh, qb, obase, 0, src);
        fp_whole_class<false, 4>(M, rs, lo, sdw, sh, qb, obase, 4, src);
    }
}

// The 8x8-variance probe of fp_slot (K32): this lane's raw 8x8 SAD at window
// position 0 (dword-aligned buffer loads realigned by v_alignbyte) into M;
// returns it as the reference counts it (SUB: doubled)
template <bool SUB>
__device__ __forceinline__ uint32_t fp_probe32(PuMin<true> &M, const uint8_t *g, int sdw,
                                               const uint32_t (&src)[SUB ? 4 : 8][2], int by, int bx) {
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1;
    g         = uni_ptr(g);
    sdw       = UNI(sdw);
    const int sh = (int)((uintptr_t)g & 3);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(g - sh);
    const uint32_t lo = (uint32_t)((by * 8) * sdw + bx * 2) * 4u;
    u32x4a4 d[ROWS];
#pragma unroll
    for (int rr = 0; rr < ROWS; rr++) d[rr] = bld4(rs, lo, (uint32_t)(rr * RSTEP * sdw) * 4u);
    uint32_t s8 = 0;
#pragma unroll
    for (int rr = 0; rr < ROWS; rr++) {
        s8 = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d[rr].y, d[rr].x, (uint32_t)sh), src[rr][0], s8);
        s8 = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d[rr].z, d[rr].y, (uint32_t)sh), src[rr][1], s8);
    }
    M.add_probe(s8);
    return SUB ? s8 << 1 : s8;
}

// Search area of integer_search_b64 for reference slot s (motion_estimation.c:
// 1282-1482): the area from the centre and the distance, check_00_center
// (:1139-1206), the 8x8-variance centre probe and resize (:1391-1439; probe(g)
// evaluates the centre at g, enters its keys at order 0 and returns the
// variance) and the final clamp to the picture.
struct FpArea {
    int16_t xo, yo, w, h, xc, yc;
    bool probe;
};
template <typename Probe>
__device__ __forceinline__ FpArea fp_area(const DevJob &dj, const SbGeo &G, int s, uint32_t zz, uint32_t rdiv,
                                          int16_t sc_x, int16_t sc_y, Probe probe_var) {
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int l = s >> 2, r = s & 3;
    const uint32_t ox = G.ox, oy = G.oy;
    const bool mctf   = SF(job, me_type) == SVTME_ME_MCTF;
    const DevPlane &C = dj.cur.lv[0];
    const DevPlane &P = dj.ref[l][r].lv[0];
    int16_t xc = sc_x, yc = sc_y;
    uint16_t dist = ref_dist_const(job, l, r);
    if (!mctf) // :1300-1302
        dist = scaled_dist(dist);
    int16_t w = i16(min((int)(SF(c, me_sa.sa_min.width) * dist), (int)SF(c, me_sa.sa_max.width)));
    int16_t h = i16(min((int)(SF(c, me_sa.sa_min.height) * dist), (int)SF(c, me_sa.sa_max.height)));
    if (SF(c, mv_sa_adj_enabled) && (!SF(c, mv_sa_adj_nearest_ref_only) || r == 0)) {
        const int mth = (int)SF(c, mv_sa_adj_mv_size_th), mul = (int)SF(c, mv_sa_adj_sa_multiplier);
        if (absi(xc) > mth)
            w = i16(w * mul);
        if (absi(yc) > mth)
            h = i16(h * mul);
    }
    w = i16((max(1u, ((uint32_t)(int32_t)w / rdiv)) + 7) & ~0x07u);
    h = i16(max(3u, ((uint32_t)(int32_t)h / rdiv)));
    const int16_t pad = 63, org_x = (int16_t)ox, org_y = (int16_t)oy;
    if (c.me_early_exit_th) {
        if (zz < (c.me_early_exit_th / 6)) {
            w = 1;
            h = 1;
        }
    } else if ((xc != 0 || yc != 0) && SF(job, is_ref)) { // check_00_center (:1139-1206)
        const int16_t pw = i16(P.width), ph = i16(P.height);
        xc = ((org_x + xc) < -pad) ? i16(-pad - org_x) : xc;
        xc = ((org_x + xc) > pw - 1) ? i16(xc - ((org_x + xc) - (pw - 1))) : xc;
        yc = ((org_y + yc) < -pad) ? i16(-pad - org_y) : yc;
        yc = ((org_y + yc) > ph - 1) ? i16(yc - ((org_y + yc) - (ph - 1))) : yc;
        const uint8_t *cb = C.base + (ptrdiff_t)oy * C.stride + ox;
        const uint32_t zero_sad =
            wave_nxm(P.base + (ptrdiff_t)oy * P.stride + ox, 2 * P.stride, cb, 2 * C.stride, (int)(G.bh >> 1),
                     (int)G.bw)
            << 1;
        const uint32_t hme_mv_sad = wave_nxm(P.base + (ptrdiff_t)((int)oy + yc) * P.stride + ((int)ox + xc),
                                             2 * P.stride, cb, 2 * C.stride, (int)(G.bh >> 1), (int)G.bw)
            << 1;
        const uint64_t zc = (uint64_t)zero_sad << 8, hc = (uint64_t)hme_mv_sad << 8;
        if (min_u64(zc, hc) == zc) {
            xc = 0;
            yc = 0;
        }
    }
    // 8x8-variance centre probe and search-area resize (:1391-1439); the probe's
    // keys (order 0) stay with the caller, so the centre wins ties against the search
    const bool probe = SF(c, me_8x8_var_enabled) && (w * h > 24);
    if (probe) {
        const uint32_t var = probe_var(P.base + (ptrdiff_t)((int)oy + yc) * P.stride + ((int)ox + xc));
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
    }
    // final area clamp (:1440-1482)
    const int16_t pic_w = (int16_t)job.width, pic_h = (int16_t)job.height;
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
    return FpArea{xo, yo, w, h, xc, yc, probe};
}

// integer_search_b64 of one reference slot s by one wavefront (motion_estimation.c:
// 1249-1516): search area (fp_area) and the full-pel search of search rows
// [h * part / parts, h * (part + 1) / parts); the 85-PU argmin keys go to kp
// (atomic min when parts > 1), the slot state to cs (part 0). src: this lane's
// 8x8 source block rows (lane = block by, bx).
// TF-ME records written by the wavefront that searched them: an ME_MCTF job has
// no me_prune_ref (motion_estimation.c:3103, the records of one SB are
// independent) and no candidate arrays (:3126), so with one band per record and
// no per-SB output the record is the decode of this wavefront's 85 keys
// (stage_e_body / stage_c_tail's record words) and k_stage_e is not launched
__device__ __forceinline__ bool direct_records(const DevJob &dj) {
    return SF(dj.job, me_type) == SVTME_ME_MCTF && dj.parts == 1 && dj.out_sb == nullptr;
}
__device__ __forceinline__ void direct_record(svtme_ref_record *rec, const CSlot &v, unsigned long long k8,
                                              unsigned long long k16, unsigned long long k32, unsigned long long k64) {
    const int lane   = threadIdx.x & 63;
    uint32_t *o      = (uint32_t *)rec;
    const uint32_t wm = magic_u32((uint32_t)max(1, (int)v.w));
    auto put = [&](unsigned long long key, int pu) {
        uint32_t sad = U32MAX, mv = 0;
        if (v.searched) {
            const uint32_t ord = (uint32_t)key;
            sad                = (uint32_t)(key >> 32);
            int16_t mx, my;
            if (v.probe && ord == 0) {
                mx = v.xc;
                my = v.yc;
            } else {
                const int p = (int)ord - (int)v.probe;
                const int q = mdiv(p, wm);
                my          = i16(v.yo + q);
                mx          = i16(v.xo + (p - q * v.w));
            }
            mv = ((uint32_t)(uint16_t)my << 16) | (uint16_t)mx;
        }
        o[pu]      = sad;
        o[85 + pu] = mv;
    };
    put(k8, 21 + lane);
    if ((lane & 3) == 0)
        put(k16, 5 + (lane >> 2));
    if ((lane & 15) == 0)
        put(k32, 1 + (lane >> 4));
    if (lane == 63)
        put(k64, 0);
    if (lane < 6) {
        const uint32_t t[6] = {(uint32_t)v.hme_sad, (uint32_t)(v.hme_sad >> 32),
                               (uint32_t)(uint16_t)v.sc_x | ((uint32_t)(uint16_t)v.sc_y << 16), v.zz,
                               (uint32_t)v.searched | ((uint32_t)v.do_ref << 8) | ((uint32_t)v.tf_exit << 16), 0u};
        o[170 + lane] = t[lane];
    }
}

template <bool SUB, bool K32, int TQ = (SUB ? FP_TQ : 2), bool WIDE = false, int WHOLE = 7>
__device__ __forceinline__ void fp_slot(const DevJob &dj, const SbGeo &G, int s, const uint32_t (&src)[SUB ? 4 : 8][2],
                                        int by, int bx, uint64_t hme_sad, uint32_t zz, uint32_t rdiv, int16_t sc_x,
                                        int16_t sc_y, uint8_t dref, uint8_t tf_exit, int part, uint32_t parts,
                                        unsigned long long *kp, CSlot *cs, svtme_ref_record *rec = nullptr) {
    const int lane = threadIdx.x & 63;
    const int l = s >> 2, r = s & 3;
    const uint32_t ox = G.ox, oy = G.oy;
    if (!dref || tf_exit) {
        const CSlot cv{hme_sad, zz, sc_x, sc_y, 0, 0, 0, 0, 0, 0, dref, 0, tf_exit};
        if (part == 0 && lane == 0)
            *cs = cv;
        if (rec)
            direct_record(rec, cv, 0, 0, 0, 0);
        return;
    }
    const DevPlane &P = dj.ref[l][r].lv[0];
    PuMin<K32> M;
    M.clear();
    const FpArea A = fp_area(dj, G, s, zz, rdiv, sc_x, sc_y, [&](const uint8_t *g) {
        const int sh = (int)((uintptr_t)g & 3);
        uint32_t p8, p64;
        if constexpr (K32) {
            p8  = fp_probe32<SUB>(M, g, P.stride >> 2, src, by, bx);
            p64 = wave_sum_u32(p8); // the 64x64 SAD at the centre
        } else {
            fp_rows<SUB, K32, 1>(M, (const uint32_t *)(g - sh), P.stride >> 2, sh, 1, 1, 0, 1, 0u, src, by, bx);
            M.finalize();
            p8  = (uint32_t)(PuMin<K32>::template out<SUB>(M.b8, true) >> 32);
            p64 = rl32((uint32_t)(PuMin<K32>::template out<SUB>(M.b64, false) >> 32), 63);
        }
        const uint32_t mean = p64 / 64;
        const int32_t diff  = (int32_t)p8 - (int32_t)mean;
        return wave_sum_u32((uint32_t)(diff * diff)) / 64;
    });
    const int16_t xo = A.xo, yo = A.yo, w = A.w, h = A.h, xc = A.xc, yc = A.yc;
    const bool probe = A.probe;
    HME_SUB(22);

    // full-pel search of this part's rows (open_loop_me_fullpel_search_sblock, :781-817)
    const uint8_t *g = P.base + (ptrdiff_t)((int)oy + yo) * P.stride + ((int)ox + xo);
    const int sh     = (int)((uintptr_t)g & 3);
    const int nq     = (sh + w + 3) >> 2;
    const int y0 = (int)(((uint32_t)h * part) / parts), y1 = (int)(((uint32_t)h * (part + 1)) / parts);
    const uint32_t obase = probe ? 1u : 0u; // the centre probe wins ties: order 0
    if constexpr (K32) {
        // an area 8 wide searched whole (wave-uniform)
        const bool whole = !WIDE && w == 8 && parts == 1; // WIDE: areas >= 24 wide
        if ((SUB ? (WHOLE & 2) && (h == 3 || h == 4) : (WHOLE & 1) && h == 8) && whole)
            fp_rows32_whole<SUB>(M, g, P.stride >> 2, h, obase, src, by, bx);
        else
            fp_rows32<SUB, WIDE ? 6 : 2>(M, g, P.stride >> 2, w, y0, y1, obase, src, by, bx);
    }
    else
        fp_rows<SUB, K32, TQ>(M, (const uint32_t *)(g - sh), P.stride >> 2, sh, w, nq, y0, y1, obase, src, by, bx);
    HME_SUB(23);
    M.finalize();
    const unsigned long long k8  = PuMin<K32>::template out<SUB>(M.b8, true);
    const unsigned long long k16 = PuMin<K32>::template out<SUB>(M.b16, false);
    const unsigned long long k32 = PuMin<K32>::template out<SUB>(M.b32, false);
    const unsigned long long k64 = PuMin<K32>::template out<SUB>(M.b64, false);
    if (parts == 1) {
        kp[21 + lane] = k8;
        if ((lane & 3) == 0)
            kp[5 + (lane >> 2)] = k16;
        if ((lane & 15) == 0)
            kp[1 + (lane >> 4)] = k32;
        if (lane == 63)
            kp[0] = k64;
    } else {
        atomicMin(&kp[21 + lane], k8);
        if ((lane & 3) == 0)
            atomicMin(&kp[5 + (lane >> 2)], k16);
        if ((lane & 15) == 0)
            atomicMin(&kp[1 + (lane >> 4)], k32);
        if (lane == 63)
            atomicMin(&kp[0], k64);
    }
    const CSlot cv{hme_sad, zz, sc_x, sc_y, xo, yo, w, xc, yc, 1, dref, (uint8_t)probe, 0};
    if (part == 0 && lane == 0)
        *cs = cv;
    if (rec)
        direct_record(rec, cv, k8, k16, k32, k64);
}


// K32: every order fits 12 bits (the host bounds the area, svtme_fp_k32)
template <bool SUB, bool K32, bool WIDE = false> // WIDE: 6-quad full-pel load sets (areas >= 24 wide)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SUB ? 5 : 4, 8))) k_stage_c1(const DevBatch B) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const uint32_t parts  = dj.parts;
    const uint32_t per_sb = dj.R * parts;
    const uint32_t sb_local = UNI(gw / per_sb);
    const uint32_t rem      = gw - sb_local * per_sb;
    const int k             = UNI(rem / parts);
    const int part          = UNI(rem - (uint32_t)k * parts);
    const int s             = k < job.num_refs[0] ? k : 4 + (k - job.num_refs[0]);
    const SbGeo G     = sb_geo(dj, sb_local);
    const uint32_t ox = G.ox, oy = G.oy;
    const bool mctf   = job.me_type == SVTME_ME_MCTF;
    constexpr int ROWS = SUB ? 4 : 8, RSTEP = SUB ? 2 : 1;
    const int z16 = lane >> 2, k4 = lane & 3;
    const int by  = ((z16 >> 3) << 2) | (((z16 >> 1) & 1) << 1) | (k4 >> 1);
    const int bx  = (((z16 >> 2) & 1) << 2) | ((z16 & 1) << 1) | (k4 & 1);

    // this lane's 8x8 source block, read in place (me_process.c:183-214), issued first
    const DevPlane &C = dj.cur.lv[0];
    uint32_t src[ROWS][2];
#pragma unroll
    for (int rr = 0; rr < ROWS; rr++) {
        const uint32_t *sp =
            (const uint32_t *)(C.base + (ptrdiff_t)(oy + by * 8 + rr * RSTEP) * C.stride + ox + bx * 8);
        src[rr][0] = sp[0];
        src[rr][1] = sp[1];
    }
    // search centre and HME pruning of the SB (lane = slot)
    const SlotCentre scv   = final_centre(job, dj.bst + sb_local, valid_mask(job));
    const uint64_t hme_sad = rl64(scv.hme_sad, s);
    const uint32_t zz = rl32(scv.zz, s), rdiv = rl32(scv.reduce_div, s);
    const int16_t sc_x = (int16_t)rl32((uint32_t)(int32_t)scv.sc_x, s);
    const int16_t sc_y = (int16_t)rl32((uint32_t)(int32_t)scv.sc_y, s);
    const uint8_t dref = (uint8_t)rl32(scv.do_ref, s);
    const uint8_t tf_exit = mctf && rl64(scv.hme_sad, 0) < job.tf_me_exit_th; // motion_estimation.c:3109-3113
    CSlot *cs = dj.cslot + (size_t)sb_local * dj.R + k;
    unsigned long long *kp = dj.keys + ((size_t)sb_local * dj.R + k) * SVTME_PU_COUNT;
    svtme_ref_record *rec = direct_records(dj) ? dj.out_records + (size_t)sb_local * dj.R + k : nullptr;
    fp_slot<SUB, K32, (SUB ? FP_TQ : 2), WIDE>(dj, G, s, src, by, bx, hme_sad, zz, rdiv, sc_x, sc_y, dref, tf_exit, part,
                                             parts, kp, cs, rec);
}

// ============================================================================
// k_fp_wide: the wide full-pel search (areas of 24 positions and more, e.g. the
// 64x64 override; sub-sampled rows, 32-bit keys) with the window in LDS.
//
// A workgroup takes 4 consecutive row bands (parts) of one (SB, reference): it
// stages the window rows of all 4 once, realigned to position 0 (fw_a) and
// shifted by one dword (fw_b[j] = fw_a[j + 1], beside fw_a in the row), so every reference dword pair a
// qsad reads is one 8-byte LDS read, even pairs from fw_a and odd pairs from
// fw_b: no v_alignbyte, no register moves for misaligned pairs, and the L1 /
// TA path idle during the search.
// Lane = by2 * 16 + hr * 8 + bx: the 8x8 blocks (2 by2, bx) and (2 by2 + 1, bx)
// of the SB (an 8x16 column) at search rows of parity hr. The 16x16 SADs are
// summed on packed u16 pairs (no carries: <= 32 640), lane bx & 1 keeping one
// parity of positions; the 32x32 sums (the horizontal halves packed, <= 65 280)
// leave one position per lane through one permlane16_swap (rows by2 even: c,
// odd: c + 4, c = bx < 4 ? bx : 7 - bx, so the row_half_mirror partner in the
// other 32x32 column holds the same position for the 64x64 sum); keys carry
// the position within the set (inline constants), the set's raster order is
// added once per set.
// ============================================================================
#define FPW_PITCH 80 // dwords per LDS row (fw_a then fw_b): the two search rows (hr = 0, 1) of one by2
                     // fall on banks 0-15 / 16-31; the other by2 of a 32-lane ds_read_b64 group reads
                     // rows 16 further (16 x 80 = 0 mod 64 banks): a 2-way conflict
#define FPW_BOFF 40  // fw_b within the row: one base address serves both copies
#define FPW_ROWS 96  // window rows per workgroup (4 bands + 62; the host bounds the band height)
#define FPW_TQ 4 // position quads per set (2 quad pairs, 16 positions; 6 wastes a third of the
               // last set at 64 positions, 8 measures the same as 4)

struct FpW {
    uint32_t b8t, b8b, b16, b32, b64; // K32 keys: 8x8 / 16x16 (sad << 16 | order), 32x32 / 64x64 (sad << 12 | order)
};

// min over lanes l and l ^ 8 (the two search-row halves), in place
__device__ __forceinline__ uint32_t fpw_min_hr(uint32_t v) {
    return min_u32(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false)); // row_ror:8
}

// One quad pair (positions e0 .. e0 + 7 of the set) of both blocks: 8x8 keys of
// each block, then the 16x16 / 32x32 / 64x64 sums and keys into the set minima.
// T / T2 (top), Bq / B2 (bottom): the qsad accumulators of quads a and b.
// MASK: positions >= ev are outside the area (the last, partial pair).
template <bool MASK, bool K8 = true>
__device__ __forceinline__ void fpw_pair(FpW &m, unsigned long long T, unsigned long long T2, unsigned long long Bq,
                                         unsigned long long B2, int e0, int ev, uint32_t sel16, uint32_t sel32,
                                         int p16, int p32) {
    const uint32_t tl = (uint32_t)T, th = (uint32_t)(T >> 32), tl2 = (uint32_t)T2, th2 = (uint32_t)(T2 >> 32);
    const uint32_t bl = (uint32_t)Bq, bh = (uint32_t)(Bq >> 32), bl2 = (uint32_t)B2, bh2 = (uint32_t)(B2 >> 32);
    auto k8 = [&](uint32_t v, int e) { // (sad << 16 | e) of position e of a packed pair
        const uint32_t k = (e & 1) ? ((v & 0xFFFF0000u) | (uint32_t)e) : ((v << 16) | (uint32_t)e);
        return (MASK && e >= ev) ? 0xFFFFFFFFu : k;
    };
    if constexpr (K8) {
        m.b8t = min_u32(min_u32(m.b8t, k8(tl, e0)), k8(tl, e0 + 1));
        m.b8t = min_u32(min_u32(m.b8t, k8(th, e0 + 2)), k8(th, e0 + 3));
        m.b8t = min_u32(min_u32(m.b8t, k8(tl2, e0 + 4)), k8(tl2, e0 + 5));
        m.b8t = min_u32(min_u32(m.b8t, k8(th2, e0 + 6)), k8(th2, e0 + 7));
        m.b8b = min_u32(min_u32(m.b8b, k8(bl, e0)), k8(bl, e0 + 1));
        m.b8b = min_u32(min_u32(m.b8b, k8(bh, e0 + 2)), k8(bh, e0 + 3));
        m.b8b = min_u32(min_u32(m.b8b, k8(bl2, e0 + 4)), k8(bl2, e0 + 5));
        m.b8b = min_u32(min_u32(m.b8b, k8(bh2, e0 + 6)), k8(bh2, e0 + 7));
    }
    // 8x16 columns, then 16x16 over bx ^ 1 (packed: both halves stay below 2^15)
    const uint32_t sl = dpp_add<0xB1>(tl + bl), sh = dpp_add<0xB1>(th + bh);
    const uint32_t sl2 = dpp_add<0xB1>(tl2 + bl2), sh2 = dpp_add<0xB1>(th2 + bh2);
    // lane parity p16 keeps positions e0 + 2i + p16: (half p16 of the pair) << 16 | e0 + 2i
    auto k16 = [&](uint32_t v, int e) {
        const uint32_t k = __builtin_amdgcn_perm(v, (uint32_t)e, sel16);
        return (MASK && e + p16 >= ev) ? 0xFFFFFFFFu : k;
    };
    m.b16 = min_u32(min_u32(m.b16, k16(sl, e0)), k16(sh, e0 + 2));
    m.b16 = min_u32(min_u32(m.b16, k16(sl2, e0 + 4)), k16(sh2, e0 + 6));
    // 32x16 over bx ^ 2 (packed, <= 65 280), then this lane's position of quad a
    // and of quad b (byte select), and the vertical 32x32 sum over by2 ^ 1 (one
    // permlane16_swap: rows by2 even get position c, odd c + 4)
    const uint32_t xl = dpp_add<0x4E>(sl), xh = dpp_add<0x4E>(sh);
    const uint32_t xl2 = dpp_add<0x4E>(sl2), xh2 = dpp_add<0x4E>(sh2);
    const uint32_t va = __builtin_amdgcn_perm(xh, xl, sel32), vb = __builtin_amdgcn_perm(xh2, xl2, sel32);
    const auto sw       = __builtin_amdgcn_permlane16_swap(va, vb, false, false);
    const uint32_t s32  = sw[0] + sw[1];
    const uint32_t k32  = (s32 << 12) | (uint32_t)e0;
    m.b32               = min_u32(m.b32, (MASK && e0 + p32 >= ev) ? 0xFFFFFFFFu : k32);
    // 64x64: the mirrored 32x32 column (bx <-> 7 - bx, same position), then by2 ^ 2
    const uint32_t s64h = dpp_add<0x141>(s32); // row_half_mirror
    const auto sw2      = __builtin_amdgcn_permlane32_swap(s64h, s64h, false, false);
    const uint32_t s64  = sw2[0] + sw2[1];
    const uint32_t k64  = (s64 << 12) | (uint32_t)e0;
    m.b64               = min_u32(m.b64, (MASK && e0 + p32 >= ev) ? 0xFFFFFFFFu : k64);
}

// packed minimum of two u16 pairs (v_pk_min_u16)
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

// set-local minima (orders within the set) into the running minima (raster order)
__device__ __forceinline__ uint32_t fpw_rebase(uint32_t b, uint32_t m, uint32_t base) {
    return min_u32(b, m == 0xFFFFFFFFu ? m : m + base);
}

// The set loop's LDS row reads as ds_read_b64 with immediate offsets from one
// base per set (inline: the compiler pairs them into ds_read2_b64, 8 LDS cycles
// for what two ds_read_b64 move in 4, and adds a base register per row), the
// next row's 5 reads issued before the current row is consumed; the waits are
// explicit, since the compiler does not count these reads. Steady-state A/B at
// the 1080p 64x64 override: k_fp_wide pass 10.39 -> 10.50 M SB/s (3 rounds).
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
struct FpwRow {
    u32x2v v[FPW_TQ + 1]; // v[j] = (A[j], A[j + 1]): even j from fw_a, odd j from fw_b
};
template <int OFF>
__device__ __forceinline__ u32x2v fpw_ds64(uint32_t a) {
    u32x2v r;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
    return r;
}
// row G of the set (block G / 4, sub-sampled row G % 4): rows RSTEP = 2 apart
template <int G>
__device__ __forceinline__ void fpw_row_issue(FpwRow &R, uint32_t lb) {
    constexpr int ROW = (G / 4) * 8 + (G % 4) * 2, O = 4 * ROW * FPW_PITCH;
    R.v[0] = fpw_ds64<O>(lb);
    R.v[2] = fpw_ds64<O + 8>(lb);
    R.v[4] = fpw_ds64<O + 16>(lb);
    R.v[1] = fpw_ds64<O + 4 * FPW_BOFF>(lb);
    R.v[3] = fpw_ds64<O + 4 * FPW_BOFF + 8>(lb);
}
// wait until at most N LDS reads are outstanding (the next row's), tying the row's registers to it
template <int N>
__device__ __forceinline__ void fpw_row_wait(FpwRow &R) {
    asm volatile("s_waitcnt lgkmcnt(%5)" : "+v"(R.v[0]), "+v"(R.v[1]), "+v"(R.v[2]), "+v"(R.v[3]), "+v"(R.v[4]) : "i"(N));
}
template <int B, int E, typename F>
__device__ __forceinline__ void fpw_sfor(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>());
        fpw_sfor<B + 1, E>(f);
    }
}

#define FPW_WAVES 5 // waves per SIMD: 5 workgroups of 30 KB LDS per CU
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FPW_WAVES, FPW_WAVES))) k_fp_wide(const DevBatch B) {
    __shared__ __attribute__((aligned(16))) uint32_t fw[FPW_ROWS * FPW_PITCH]; // rows: fw_a | fw_b
    const uint32_t fw_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)fw;
    constexpr int ROWS = 4, RSTEP = 2; // sub-sampled rows
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total) // the whole workgroup: totals are multiples of 4
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const uint32_t parts    = dj.parts;
    const uint32_t per_sb   = dj.R * parts;
    const uint32_t sb_local = UNI(gw / per_sb);
    const uint32_t rem      = gw - sb_local * per_sb;
    const int k             = UNI(rem / parts);
    const int part          = UNI(rem - (uint32_t)k * parts);
    const int s             = k < job.num_refs[0] ? k : 4 + (k - job.num_refs[0]);
    const SbGeo G           = sb_geo(dj, sb_local);
    const uint32_t ox = G.ox, oy = G.oy;
    const bool mctf   = job.me_type == SVTME_ME_MCTF;
    const int by2 = lane >> 4, hr = (lane >> 3) & 1, bx = lane & 7;
    const int c32 = bx < 4 ? bx : 7 - bx;

    // the lane's two 8x8 source blocks (rows 2 by2 * 8 + blk * 8 + 2 rr), issued first
    const DevPlane &C = dj.cur.lv[0];
    uint32_t src[2][ROWS][2];
#pragma unroll
    for (int blk = 0; blk < 2; blk++)
#pragma unroll
        for (int rr = 0; rr < ROWS; rr++) {
            const uint32_t *sp = (const uint32_t *)(C.base +
                                                    (ptrdiff_t)(oy + (2 * by2 + blk) * 8 + rr * RSTEP) * C.stride +
                                                    ox + bx * 8);
            src[blk][rr][0] = sp[0];
            src[blk][rr][1] = sp[1];
        }
    CSlot *cs              = dj.cslot + (size_t)sb_local * dj.R + k;
    unsigned long long *kp = dj.keys + ((size_t)sb_local * dj.R + k) * SVTME_PU_COUNT;
    const DevPlane &P      = dj.ref[s >> 2][s & 3].lv[0];
    const int sdw          = P.stride >> 2;
    FpW b{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // search centre, area and centre probe: the same for the workgroup's 4 bands,
    // made by wave 0 and handed to the others through LDS
    auto prologue = [&](FpArea &A) -> bool {
        const SlotCentre scv   = final_centre(job, dj.bst + sb_local, valid_mask(job));
        const uint64_t hme_sad = rl64(scv.hme_sad, s);
        const uint32_t zz = rl32(scv.zz, s), rdiv = rl32(scv.reduce_div, s);
        const int16_t sc_x    = (int16_t)rl32((uint32_t)(int32_t)scv.sc_x, s);
        const int16_t sc_y    = (int16_t)rl32((uint32_t)(int32_t)scv.sc_y, s);
        const uint8_t dref    = (uint8_t)rl32(scv.do_ref, s);
        const uint8_t tf_exit = mctf && rl64(scv.hme_sad, 0) < job.tf_me_exit_th; // motion_estimation.c:3109-3113
        if (!dref || tf_exit) {
            if (part == 0 && lane == 0)
                *cs = CSlot{hme_sad, zz, sc_x, sc_y, 0, 0, 0, 0, 0, 0, dref, 0, tf_exit};
            return false;
        }
        A = fp_area(dj, G, s, zz, rdiv, sc_x, sc_y, [&](const uint8_t *g) {
            // the centre: both blocks' raw 8x8 SADs (order 0 in every class)
            g                                 = uni_ptr(g);
            const int sh                      = (int)((uintptr_t)g & 3);
            const __amdgpu_buffer_rsrc_t rs   = plane_rsrc(g - sh);
            uint32_t s8[2];
#pragma unroll
            for (int blk = 0; blk < 2; blk++) {
                const uint32_t lo = (uint32_t)(((2 * by2 + blk) * 8) * sdw + bx * 2) * 4u;
                u32x4a4 d[ROWS];
#pragma unroll
                for (int rr = 0; rr < ROWS; rr++) d[rr] = bld4(rs, lo, (uint32_t)(rr * RSTEP * sdw) * 4u);
                uint32_t a = 0;
#pragma unroll
                for (int rr = 0; rr < ROWS; rr++) {
                    a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d[rr].y, d[rr].x, (uint32_t)sh), src[blk][rr][0], a);
                    a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(d[rr].z, d[rr].y, (uint32_t)sh), src[blk][rr][1], a);
                }
                s8[blk] = a;
            }
            const uint32_t s16 = dpp_add<0xB1>(s8[0] + s8[1]);
            const uint32_t s32h = dpp_add<0x4E>(s16);
            const auto w16 = __builtin_amdgcn_permlane16_swap(s32h, s32h, false, false);
            const uint32_t s32 = w16[0] + w16[1];
            const uint32_t s64h = dpp_add<0x141>(s32);
            const auto w32 = __builtin_amdgcn_permlane32_swap(s64h, s64h, false, false);
            const uint32_t s64 = w32[0] + w32[1];
            b.b8t = s8[0] << 16, b.b8b = s8[1] << 16, b.b16 = s16 << 16, b.b32 = s32 << 12, b.b64 = s64 << 12;
            // the variance of the 64 8x8 SADs as the reference counts them (doubled); every
            // block sits in two lanes (hr = 0, 1)
            const uint32_t p8t = s8[0] << 1, p8b = s8[1] << 1;
            const uint32_t mean = (wave_sum_u32(p8t + p8b) >> 1) / 64;
            const int32_t dt = (int32_t)p8t - (int32_t)mean, db = (int32_t)p8b - (int32_t)mean;
            return (wave_sum_u32((uint32_t)(dt * dt) + (uint32_t)(db * db)) >> 1) / 64;
        });
        if (part == 0 && lane == 0)
            *cs = CSlot{hme_sad, zz, sc_x, sc_y, A.xo, A.yo, A.w, A.xc, A.yc, 1, dref, (uint8_t)A.probe, 0};
        return true;
    };
    FpArea A;
    __shared__ FpArea fx_area;
    __shared__ uint32_t fx_keys[5][64], fx_run;
    if (wid == 0) {
        const bool run = prologue(A);
        if (lane == 0) {
            fx_run  = run;
            fx_area = A;
        }
        fx_keys[0][lane] = b.b8t, fx_keys[1][lane] = b.b8b, fx_keys[2][lane] = b.b16;
        fx_keys[3][lane] = b.b32, fx_keys[4][lane] = b.b64;
    }
    __syncthreads();
    if (!fx_run)
        return;
    A     = fx_area;
    b.b8t = fx_keys[0][lane], b.b8b = fx_keys[1][lane], b.b16 = fx_keys[2][lane];
    b.b32 = fx_keys[3][lane], b.b64 = fx_keys[4][lane];
    const int w = A.w, h = A.h;

    // stage the rows [Y0, Y1 + 62) of the 4 bands: fw_a[row][j] = window dword j
    // (realigned), fw_b[row][j] = fw_a[row][j + 1]
    const uint8_t *g = uni_ptr(P.base + (ptrdiff_t)((int)oy + A.yo) * P.stride + ((int)ox + A.xo));
    const int sh     = (int)((uintptr_t)g & 3);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(g - sh);
    const int part0 = part & ~3;
    const int Y0 = (int)(((uint32_t)h * part0) / parts), Y1 = (int)(((uint32_t)h * (part0 + 4)) / parts);
    const int nq     = (w + 3) >> 2;
    const int nsets  = (nq + FPW_TQ - 1) / FPW_TQ;
    const int ndw    = 14 + (nsets - 1) * FPW_TQ + FPW_TQ + 2; // fw_a dwords a lane's pairs reach
    const int nrows  = Y1 - Y0 + 62;
    {
        // groups of 4 dwords: fw_a[4 g .. 4 g + 3] and fw_b[4 g .. 4 g + 3] from the raw
        // dwords 4 g .. 4 g + 5 of the row (one 16-byte and two 4-byte loads)
        const int ng        = (ndw + 1 + 3) >> 2;
        const uint32_t mg   = magic_u32((uint32_t)ng);
        const int total     = nrows * ng;
        for (int i0 = 0; i0 < total; i0 += 4 * 256) {
            u32x4a4 r[4];
            uint32_t r4[4], r5[4];
            int row[4], gq[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int i = i0 + t * 256 + (int)threadIdx.x;
                row[t]      = mdiv(i, mg);
                gq[t]       = i - row[t] * ng;
                if (i < total) {
                    const uint32_t off = ((uint32_t)(Y0 + row[t]) * (uint32_t)sdw + 4u * (uint32_t)gq[t]) * 4u;
                    r[t]  = bld4(rs, off, 0);
                    r4[t] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + 16u), 0, 0);
                    r5[t] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + 20u), 0, 0);
                }
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int i = i0 + t * 256 + (int)threadIdx.x;
                if (i < total) {
                    const uint32_t a0 = __builtin_amdgcn_alignbyte(r[t].y, r[t].x, (uint32_t)sh);
                    const uint32_t a1 = __builtin_amdgcn_alignbyte(r[t].z, r[t].y, (uint32_t)sh);
                    const uint32_t a2 = __builtin_amdgcn_alignbyte(r[t].w, r[t].z, (uint32_t)sh);
                    const uint32_t a3 = __builtin_amdgcn_alignbyte(r4[t], r[t].w, (uint32_t)sh);
                    const uint32_t a4 = __builtin_amdgcn_alignbyte(r5[t], r4[t], (uint32_t)sh);
                    uint32_t *d = fw + row[t] * FPW_PITCH + 4 * gq[t];
                    *(uint4 *)d              = make_uint4(a0, a1, a2, a3);
                    *(uint4 *)(d + FPW_BOFF) = make_uint4(a1, a2, a3, a4);
                }
            }
        }
    }
    __syncthreads();

    // this band's search rows; the two halves of the wave take rows ty and ty + 1
    const int y0 = (int)(((uint32_t)h * part) / parts), y1 = (int)(((uint32_t)h * (part + 1)) / parts);
    const uint32_t obase = A.probe ? 1u : 0u; // the centre probe wins ties: order 0
    const uint32_t sel16 = (bx & 1) ? 0x07060100u : 0x05040100u;
    const uint32_t sel32 = (c32 & 2) ? ((c32 & 1) ? 0x0C0C0706u : 0x0C0C0504u) : ((c32 & 1) ? 0x0C0C0302u : 0x0C0C0100u);
    const int p16 = bx & 1, p32 = c32 + 4 * (by2 & 1);
    const int L   = 2 * bx;
    const int nwhole = w / (4 * FPW_TQ); // sets with all 16 positions inside the area
    // 8x8 classes in two passes: per set only each block's packed SAD minimum (v_pk_min_u16
    // over the set's 16 positions) and the first set, in scan order, that lowered it; after
    // the loop the position inside that set (one more set of SADs per block). Scan order is
    // raster order and the pass keeps the earliest set, so the reference's tie-break holds
    uint32_t r8t = 0xFFFFu, r8b = 0xFFFFu, rc8t = 0, rc8b = 0;
    for (int ty = y0; ty < y1; ty += 2) {
        const int tyh = min(ty + hr, y1 - 1); // an odd band: half 1 repeats the last row (same keys)
        // one set of 16 positions into the set minima m (orders EOFF + position in the
        // set); WHOLE: all inside the area (every set of a 64-wide area), so the whole
        // sets run one straight loop, two sets per fold into the running minima, and
        // the partial set apart
        auto run_set = [&](const int set, FpW &m, auto EOFF, auto WHOLE) {
            const int tq = set * FPW_TQ;
            unsigned long long acc[2][FPW_TQ];
#pragma unroll
            for (int blk = 0; blk < 2; blk++)
#pragma unroll
                for (int iq = 0; iq < FPW_TQ; iq++) acc[blk][iq] = 0;
            // the 8 rows (2 blocks x 4 sub-sampled rows) of the set, one row ahead
            const uint32_t lb = fw_lds + 4u * (uint32_t)((tyh - Y0 + 2 * by2 * 8) * FPW_PITCH + L + tq);
            FpwRow R[2];
            fpw_row_issue<0>(R[0], lb);
            fpw_sfor<0, 2 * ROWS>([&](auto G) {
                constexpr int g = decltype(G)::value, blk = g / ROWS, rr = g % ROWS;
                if constexpr (g + 1 < 2 * ROWS) {
                    fpw_row_issue<g + 1>(R[(g + 1) & 1], lb);
                    fpw_row_wait<5>(R[g & 1]);
                } else {
                    fpw_row_wait<0>(R[g & 1]);
                }
                const FpwRow &q = R[g & 1];
#pragma unroll
                for (int iq = 0; iq < FPW_TQ; iq++) {
                    acc[blk][iq] = qsad(q.v[iq].x, q.v[iq].y, src[blk][rr][0], acc[blk][iq]);
                    acc[blk][iq] = qsad(q.v[iq + 1].x, q.v[iq + 1].y, src[blk][rr][1], acc[blk][iq]);
                }
            });
            // the SADs exist here: otherwise the compiler sinks the qsads of the
            // later pairs into their (conditional) uses and keeps every row live
#pragma unroll
            for (int blk = 0; blk < 2; blk++)
#pragma unroll
                for (int iq = 0; iq < FPW_TQ; iq++) asm volatile("" : "+v"(acc[blk][iq]));
            const int left = w - 4 * tq; // positions of the area in this set (wave-uniform)
            {
                auto pmin = [&](int blk) -> uint32_t {
                    uint32_t p = 0xFFFFFFFFu;
#pragma unroll
                    for (int iq = 0; iq < FPW_TQ; iq++) {
                        uint32_t lo = (uint32_t)acc[blk][iq], hi = (uint32_t)(acc[blk][iq] >> 32);
                        if constexpr (!decltype(WHOLE)::value) { // positions outside the area
                            lo |= (4 * iq >= left ? 0xFFFFu : 0u) | (4 * iq + 1 >= left ? 0xFFFF0000u : 0u);
                            hi |= (4 * iq + 2 >= left ? 0xFFFFu : 0u) | (4 * iq + 3 >= left ? 0xFFFF0000u : 0u);
                        }
                        p = pk_min_u16(p, pk_min_u16(lo, hi));
                    }
                    return min_u32(p & 0xFFFFu, p >> 16);
                };
                const uint32_t code = ((uint32_t)tyh << 8) | (uint32_t)set;
                const uint32_t st = pmin(0), sb = pmin(1);
                rc8t = st < r8t ? code : rc8t;
                r8t  = min_u32(r8t, st);
                rc8b = sb < r8b ? code : rc8b;
                r8b  = min_u32(r8b, sb);
            }
            if constexpr (decltype(WHOLE)::value) {
#pragma unroll
                for (int pp = 0; pp < FPW_TQ / 2; pp++)
                    fpw_pair<false, false>(m, acc[0][2 * pp], acc[0][2 * pp + 1], acc[1][2 * pp], acc[1][2 * pp + 1],
                                           decltype(EOFF)::value + 8 * pp, 8, sel16, sel32, p16, p32);
            } else {
#pragma unroll
                for (int pp = 0; pp < FPW_TQ / 2; pp++) {
                    const int ev = left - 8 * pp;
                    if (ev <= 0)
                        break;
                    if (ev >= 8)
                        fpw_pair<false, false>(m, acc[0][2 * pp], acc[0][2 * pp + 1], acc[1][2 * pp], acc[1][2 * pp + 1],
                                               8 * pp, 8, sel16, sel32, p16, p32);
                    else
                        fpw_pair<true, false>(m, acc[0][2 * pp], acc[0][2 * pp + 1], acc[1][2 * pp], acc[1][2 * pp + 1],
                                              8 * pp, ev + 8 * pp, sel16, sel32, p16, p32);
                }
            }
        };
        // the set minima (orders from set tq's first position) into the running minima
        auto fold = [&](const FpW &m, const int tq, const bool keyed) {
            const uint32_t ob = obase + (uint32_t)(tyh * w + 4 * tq);
            if (keyed) { // a whole first pair: every class of every lane has a key
                b.b16 = min_u32(b.b16, m.b16 + ob + (uint32_t)p16);
                b.b32 = min_u32(b.b32, m.b32 + ob + (uint32_t)p32);
                b.b64 = min_u32(b.b64, m.b64 + ob + (uint32_t)p32);
            } else {
                b.b16 = fpw_rebase(b.b16, m.b16, ob + (uint32_t)p16);
                b.b32 = fpw_rebase(b.b32, m.b32, ob + (uint32_t)p32);
                b.b64 = fpw_rebase(b.b64, m.b64, ob + (uint32_t)p32);
            }
        };
        using I0  = std::integral_constant<int, 0>;
        using I16 = std::integral_constant<int, 4 * FPW_TQ>;
        int set = 0;
        for (; set + 2 <= nwhole; set += 2) {
            FpW m{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            run_set(set, m, I0(), std::true_type());
            run_set(set + 1, m, I16(), std::true_type());
            fold(m, set * FPW_TQ, true);
        }
        if (set < nwhole) {
            FpW m{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            run_set(set, m, I0(), std::true_type());
            fold(m, set * FPW_TQ, true);
        }
        if (nwhole < nsets) {
            FpW m{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            run_set(nwhole, m, I0(), std::false_type());
            fold(m, nwhole * FPW_TQ, w - 4 * nwhole * FPW_TQ >= 8);
        }
    }
    // 8x8 pass 2: the block's SADs in its recorded set again, the lowest position at the minimum
    auto find8 = [&](auto BLK, const uint32_t rmin, const uint32_t rc, uint32_t &best) {
        constexpr int blk = decltype(BLK)::value;
        if (rmin == 0xFFFFu)
            return; // no position searched
        const int tyr = (int)(rc >> 8), tq = (int)(rc & 0xFFu) * FPW_TQ;
        const uint32_t lb = fw_lds + 4u * (uint32_t)((tyr - Y0 + 2 * by2 * 8) * FPW_PITCH + L + tq);
        unsigned long long acc[FPW_TQ];
#pragma unroll
        for (int iq = 0; iq < FPW_TQ; iq++) acc[iq] = 0;
        FpwRow R[2];
        fpw_row_issue<blk * ROWS>(R[0], lb);
        fpw_sfor<0, ROWS>([&](auto RR) {
            constexpr int rr = decltype(RR)::value, g = blk * ROWS + rr;
            if constexpr (rr + 1 < ROWS) {
                fpw_row_issue<g + 1>(R[(rr + 1) & 1], lb);
                fpw_row_wait<5>(R[rr & 1]);
            } else {
                fpw_row_wait<0>(R[rr & 1]);
            }
            const FpwRow &q = R[rr & 1];
#pragma unroll
            for (int iq = 0; iq < FPW_TQ; iq++) {
                acc[iq] = qsad(q.v[iq].x, q.v[iq].y, src[blk][rr][0], acc[iq]);
                acc[iq] = qsad(q.v[iq + 1].x, q.v[iq + 1].y, src[blk][rr][1], acc[iq]);
            }
        });
        const int left = w - tq * 4;
        uint32_t k = 0xFFFFFFFFu;
#pragma unroll
        for (int iq = 0; iq < FPW_TQ; iq++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int e      = 4 * iq + j;
                const uint32_t v = (uint32_t)(acc[iq] >> (16 * j)) & 0xFFFFu;
                k                = min_u32(k, e >= left ? 0xFFFFFFFFu : (v << 16) | (uint32_t)e);
            }
        best = min_u32(best, k + obase + (uint32_t)(tyr * w + 4 * tq));
    };
    find8(std::integral_constant<int, 0>(), r8t, rc8t, b.b8t);
    find8(std::integral_constant<int, 1>(), r8b, rc8b, b.b8b);
    // both halves, then the lanes of each class
    b.b8t = fpw_min_hr(b.b8t), b.b8b = fpw_min_hr(b.b8b), b.b16 = fpw_min_hr(b.b16);
    b.b32 = fpw_min_hr(b.b32), b.b64 = fpw_min_hr(b.b64);
    // 16x16: the two parities (bx ^ 1); 32x32: the 4 positions of quad a / b (bx ^ 1,
    // bx ^ 2) and the two rows (by2 ^ 1); 64x64: every lane
    b.b16 = min_u32(b.b16, (uint32_t)__builtin_amdgcn_update_dpp((int)b.b16, (int)b.b16, 0xB1, 0xF, 0xF, false));
    b.b32 = PuMin<true>::quad_min(b.b32);
    {
        const auto t = __builtin_amdgcn_permlane16_swap(b.b32, b.b32, false, false);
        b.b32        = min_u32(t[0], t[1]);
    }
    b.b64 = wave_min_u32(b.b64);
    auto out8 = [](uint32_t v) -> unsigned long long { // 16-bit orders; SUB SADs doubled
        return v == 0xFFFFFFFFu ? ~0ull : ((unsigned long long)((v >> 16) << 1) << 32) | (v & 0xFFFFu);
    };
    auto out12 = [](uint32_t v) -> unsigned long long {
        return v == 0xFFFFFFFFu ? ~0ull : ((unsigned long long)((v >> 12) << 1) << 32) | (v & 0xFFFu);
    };
    auto morton = [](int y, int x) { // Z order of the 85-PU table (by bits odd, bx bits even)
        return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2) | ((x & 4) << 2) | ((y & 4) << 3);
    };
    if (hr == 0) {
        atomicMin(&kp[21 + morton(2 * by2, bx)], out8(b.b8t));
        atomicMin(&kp[21 + morton(2 * by2 + 1, bx)], out8(b.b8b));
        if ((bx & 1) == 0)
            atomicMin(&kp[5 + morton(by2, bx >> 1)], out8(b.b16));
        if ((bx & 3) == 0 && (by2 & 1) == 0)
            atomicMin(&kp[1 + morton(by2 >> 1, bx >> 2)], out12(b.b32));
        if (lane == 0)
            atomicMin(&kp[0], out12(b.b64));
    }
}

// ============================================================================
// k_l0_full: stage A of full-SAD HME jobs without pre-HME (TF-ME levels 0-2:
// the zz SAD and hme_level_0, motion_estimation.c:835-889, 2382-2437) with
// HME-L0 quadrants of at most 16 x 16 positions. One wavefront per (SB, slot):
// lanes 16 qq .. 16 qq + 15 take quadrant qq, a lane one aligned position
// quad of PR position rows (each loaded reference row feeds all of them), the
// 16 x 16 sixteenth-resolution source row in SGPRs. u16 accumulators hold the
// whole block (16 x 16 x 255 < 2^16). Partial SBs need a width of a multiple
// of 16 (whole source dwords); k_stage_a otherwise.
// ============================================================================
template <int PR> // position rows per lane: 2 (quadrants up to 8 rows) or 4 (up to 16)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_l0_full(const DevBatch B) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const uint32_t sb_local = UNI(gw / dj.ta_count);
    const int entry         = UNI(dj.ta_list[gw - sb_local * dj.ta_count]); // TA_HME << 3 | slot
    const int s = entry & 7, l = s >> 2, r = s & 3;
    const SbGeo G   = sb_geo(dj, sb_local);
    ARes *out       = dj.ares + (size_t)sb_local * SVTME_A_N;
    const DevPlane &P = dj.ref[l][r].lv[2];
    const int16_t sox = i16(((int16_t)G.ox) >> 2), soy = i16(((int16_t)G.oy) >> 2);
    const int bws = (int)(G.bw >> 2), bhs = (int)(G.bh >> 2), nd = bws >> 2;

    // zz SAD (init_zz_sad, motion_estimation.c:2382-2437): sub-sampled 64 x 32 at full resolution
    const bool zz = c.me_early_exit_th || c.me_safe_limit_zz_th;
    if (zz) {
        const DevPlane &F = dj.ref[l][r].lv[0];
        const DevPlane &Cf = dj.cur.lv[0];
        const uint8_t *zr = F.base + (ptrdiff_t)G.oy * F.stride + G.ox;
        const uint8_t *zc = Cf.base + (ptrdiff_t)G.oy * Cf.stride + G.ox;
        uint32_t v;
        if (G.bw == 64 && G.bh == 64) {
            ZzLoads zl;
            zz_issue(zl, zr, 2 * F.stride, zc, 2 * Cf.stride);
            v = zz_finish(zl);
        } else
            v = wave_nxm(zr, 2 * F.stride, zc, 2 * Cf.stride, (int)(G.bh >> 1), (int)G.bw);
        if (lane == 0)
            out[SVTME_A_ZZ + s] = ARes{v, 0, 0};
    }
    if (!(c.enable_hme_flag && c.enable_hme_level0_flag))
        return;
    // this lane's quadrant (hme_level_0 :835-889)
    const int qq = lane >> 4, qd = lane & 3, rp = (lane >> 2) & 3; // position rows PR rp .. PR rp + PR - 1
    int16_t sa_w, sa_h;
    hme_l0_area(c, l, r, ref_dist_const(job, l, r), 0, 0, &sa_w, &sa_h);
    int16_t xo, yo, sw, shh;
    hme_l0_rect(c, P, sox, soy, sa_w, sa_h, qq >> 1, qq & 1, &xo, &yo, &sw, &shh);
    const uint8_t *w0  = P.base + (ptrdiff_t)(soy + yo) * P.stride + (sox + xo);
    const int sh       = (int)((uintptr_t)w0 & 3);
    const int rowbytes = P.stride;
    const uint8_t *pa  = uni_ptr(P.base - (ptrdiff_t)SVTME_DEV_S_TOP * P.stride - SVTME_DEV_S_LEFT);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(pa); // the slot's sixteenth plane (allocation start)
    const int32_t wofs = (int32_t)((w0 - sh) - pa);
    const int qcol     = 4 * qd < sw ? qd : 0;       // lanes without a position read inside the window
    const int rlast    = (shh > 0 ? shh - 1 : 0) + bhs;
    const DevPlane &Sc = dj.cur.lv[2];
    const uint8_t *sp0 = uni_ptr(Sc.base + (ptrdiff_t)soy * Sc.stride + sox);
    const int sst      = UNI(Sc.stride);
    unsigned long long a[PR] = {}; // position rows PR rp + j
    // reference row PR rp + t feeds block row t - j of position row PR rp + j for every j
    // with 0 <= t - j < bhs (ACT: bit j); the head and tail rows are unrolled so that
    // every condition is a constant (no predicated qsads)
    auto row = [&](int t, auto ACT, auto FW) {
        constexpr uint32_t act = decltype(ACT)::value;
        constexpr bool fw      = decltype(FW)::value;
        const uint32_t off = (uint32_t)(wofs + min(PR * rp + t, rlast) * rowbytes + 4 * qcol);
        const u32x4a4 ra   = bld4(rs, off, 0);
        const uint32_t r4  = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + 16u), 0, 0);
        const uint32_t r5  = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + 20u), 0, 0);
        const uint32_t raw[6] = {ra.x, ra.y, ra.z, ra.w, r4, r5};
        uint32_t d[5];
#pragma unroll
        for (int j = 0; j < 5; j++) d[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], (uint32_t)sh);
#pragma unroll
        for (int j = 0; j < PR; j++) {
            if (!((act >> j) & 1u))
                continue;
            const uint4 sv        = sld4(sp0 + (ptrdiff_t)(t - j) * sst);
            const uint32_t c4[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (fw || k < nd)
                    a[j] = qsad(d[k], d[k + 1], c4[k], a[j]);
        }
    };
    auto rows = [&](auto FW) {
        using A1 = std::integral_constant<uint32_t, 1u>;
        using A3 = std::integral_constant<uint32_t, 3u>;
        using A7 = std::integral_constant<uint32_t, 7u>;
        using AE = std::integral_constant<uint32_t, 14u>;
        using AC = std::integral_constant<uint32_t, 12u>;
        using A8 = std::integral_constant<uint32_t, 8u>;
        using A2 = std::integral_constant<uint32_t, 2u>;
        using AF = std::integral_constant<uint32_t, (1u << PR) - 1u>;
        if constexpr (PR == 4) {
            if (bhs == 2) { // an 8-row SB: block rows t - j in {0, 1} only
                using A6 = std::integral_constant<uint32_t, 6u>;
                row(0, A1(), FW);
                row(1, A3(), FW);
                row(2, A6(), FW);
                row(3, AC(), FW);
                row(4, A8(), FW);
                return;
            }
        }
        // head: t < PR - 1 (position rows j <= t; bhs >= PR - 1 from here)
        row(0, A1(), FW);
        if constexpr (PR == 4) {
            row(1, A3(), FW);
            row(2, A7(), FW);
        }
        for (int t = PR - 1; t < bhs; t++) // every position row
            row(t, AF(), FW);
        // tail: t = bhs + i (position rows j > i)
        if constexpr (PR == 4) {
            row(bhs, AE(), FW);
            row(bhs + 1, AC(), FW);
            row(bhs + 2, A8(), FW);
        } else
            row(bhs, A2(), FW);
    };
    if (nd == 4)
        rows(std::true_type());
    else
        rows(std::false_type());
    // keys (sad << 32 | y << 16 | x) of the lane's positions inside the quadrant's area,
    // then the minimum over the quadrant's 16 lanes (one DPP row)
    unsigned long long best = ~0ull;
#pragma unroll
    for (int j = 0; j < PR; j++) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int x = 4 * qd + e, y = PR * rp + j;
            if (x < sw && y < shh) {
                const uint32_t sad = (uint32_t)(a[j] >> (16 * e)) & 0xFFFFu;
                const unsigned long long k = ((unsigned long long)sad << 32) | ((uint32_t)y << 16) | (uint32_t)x;
                best = k < best ? k : best;
            }
        }
    }
    {
        auto step = [&](uint32_t tl, uint32_t th) {
            const unsigned long long t = ((unsigned long long)th << 32) | tl;
            best                       = t < best ? t : best;
        };
#define L0MIN(CTRL) step(dpp_or<CTRL>((uint32_t)best, U32MAX), dpp_or<CTRL>((uint32_t)(best >> 32), U32MAX))
        L0MIN(DPP_ROW_SHR(1));
        L0MIN(DPP_ROW_SHR(2));
        L0MIN(DPP_ROW_SHR(4));
        L0MIN(DPP_ROW_SHR(8));
#undef L0MIN
    }
    if ((lane & 15) == 15) {
        uint32_t bs;
        int x, y;
        key_result(best, &bs, &x, &y);
        out[SVTME_A_L0 + s * 4 + qq] = ARes{bs, i16((x + xo) * 4), i16((y + yo) * 4)}; // full rows: not doubled
    }
}

#define L1W_PITCH 12                  // dwords per staged window row (16 positions + 31 columns + 1)
#define L1W_HALF (48 * L1W_PITCH + 4) // 48 rows; + 4 dwords: the two halves' rows on different banks
// ============================================================================
// k_l1_full: HME level 1 with full-SAD rows (TF-ME levels 0-2, hme_level1_b64
// :2041-2122 / hme_level_1 :923-1022): the 32x32 quarter-resolution block over
// up to 16 x 16 positions per (slot, quadrant). One wavefront takes two
// quadrants of one slot (lanes 32 h .. 32 h + 31: quadrant 2 qp + h); a lane
// owns one aligned position quad of two position rows (y = 2 i, 2 i + 1), so
// every reference row it loads (16-byte buffer loads, realigned once with
// v_alignbyte) feeds 8 qsads of each of the two rows; the source row, the same
// for the whole wave, sits in SGPRs (scalar loads). Accumulators are flushed
// to 32 bits every 8 block rows (u16 lanes: 8 x 32 x 255 < 2^16).
// Applies when HME-L2 is off and the L1 area is at most 16 x 16 (k_stage_b
// otherwise).
// ============================================================================
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_l1_full(const DevBatch B) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t u = UNI(xcd_remap(blockIdx.x, gridDim.x) * 4 + wid);
    if (u >= B.total)
        return;
    uint32_t gw;
    const DevJob &dj        = batch_job(B, u, &gw);
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const uint32_t npairs   = dj.tb_count >> 1; // the list holds the 4 quadrants of each slot in order
    const uint32_t sb_local = UNI(gw / npairs);
    const int e0            = UNI(dj.tb_list[2 * (gw - sb_local * npairs)]);
    // lane = rh * 32 + half * 16 + pr_lo * 4 + qd: a quadrant (half) takes rows 0 and 2 or 1 and 3 of
    // the wave, so each 32-lane LDS group reads position row pairs 0-3 (rh = 0) or 4-7 of both
    // quadrants: 24 pr + qd (+ the other window's 580 = 4 mod 32) are 32 distinct banks (lanes 0-31
    // of one quadrant had pr and pr + 4 on one bank)
    const int half = (lane >> 4) & 1, s = e0 >> 2, q = (e0 & 3) + half, l = s >> 2, r = s & 3;
    const int qd = lane & 3, pr = ((lane >> 5) << 2) | ((lane >> 2) & 3); // position quad, position row pair
    const SbGeo G = sb_geo(dj, sb_local);
    BState *b     = dj.bst + sb_local;
    const DevPlane &P = dj.ref[l][r].lv[1];
    const int16_t qx = i16(((int16_t)G.ox) >> 1), qy = i16(((int16_t)G.oy) >> 1);
    const int bw = (int)(G.bw >> 1), bh = (int)(G.bh >> 1), nd = bw >> 2;

    // the decisions of hme_level1_b64 (:2058-2083) for this lane's quadrant
    const uint32_t zz   = b->zz[s];
    const uint8_t dref  = b->do_ref[s];
    const int16_t X0    = b->lx[s][q], Y0 = b->ly[s][q];
    const uint64_t S0   = b->lsad[s][q];
    int16_t X = 0, Y = 0;
    uint64_t SD = 0;
    bool search = false;
    if (c.me_early_exit_th && zz < (c.me_early_exit_th >> 2)) {
        X = Y = 0, SD = 0;
    } else if (!dref) {
        X = Y = 0, SD = U32MAX;
    } else if (c.prev_me_stage_based_exit_th && S0 < (c.prev_me_stage_based_exit_th >> 5)) {
        X = X0, Y = Y0, SD = S0;
    } else
        search = true;
    int16_t xo = 0, yo = 0, sw = 0, shh = 0;
    if (search)
        hme_refine_rect(1, P, qx, qy, (int16_t)c.hme_l1_sa.width, (int16_t)c.hme_l1_sa.height, i16(X0 >> 1),
                        i16(Y0 >> 1), &xo, &yo, &sw, &shh);
    // window of this lane: plane position (qx + xo, qy + yo); raw dwords from the aligned base.
    // The buffer starts at the plane's allocation (its top-left margin), so that every
    // window offset is non-negative; lanes with no position of the area read inside it:
    // columns from quad 0, rows clamped to the window's last row
    const uint8_t *w0  = P.base + (ptrdiff_t)(qy + yo) * P.stride + (qx + xo);
    const int sh       = (int)((uintptr_t)w0 & 3);
    const int rowbytes = P.stride;
    const uint8_t *pa  = uni_ptr(P.base - (ptrdiff_t)SVTME_DEV_Q_TOP * P.stride - SVTME_DEV_Q_LEFT);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(pa); // the slot's quarter plane: uniform
    const int32_t wofs = (int32_t)((w0 - sh) - pa);
    const int qcol     = 4 * qd < sw ? qd : 0;
    const int rlast    = (shh > 0 ? shh - 1 : 0) + bh;
    const bool active  = search && sw > 0 && shh > 0;
    const bool any     = __ballot(active) != 0;
    uint32_t acc32[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    // this half's window in LDS, realigned to position 0: rows 0 .. rlast (<= 47) x
    // 12 dwords (positions 0 .. 15 + 31 block columns + 1); every qsad pair is then
    // one 4-byte-aligned 8-byte LDS read (ds_read2_b32), with no v_alignbyte and no
    // register copies for the odd pairs in the row loop
    __shared__ __attribute__((aligned(16))) uint32_t l1w[4][2][L1W_HALF];
    uint32_t *win = l1w[wid][half];
    if (any) {
        if (active) { // 30 lanes of the half: 10 rows x 3 dword groups per pass
            const int l32 = (lane & 15) | ((lane >> 5) << 4), rr = l32 / 3, cg = l32 - 3 * rr;
            for (int r0 = 0; r0 <= rlast; r0 += 10) {
                const int row = r0 + rr;
                if (rr < 10 && row <= rlast) {
                    const uint32_t off = (uint32_t)(wofs + row * rowbytes + 16 * cg);
                    const u32x4a4 t4   = bld4(rs, off, 0);
                    const uint32_t t5  = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off + 16u), 0, 0);
                    *(uint4 *)&win[row * L1W_PITCH + 4 * cg] =
                        make_uint4(__builtin_amdgcn_alignbyte(t4.y, t4.x, (uint32_t)sh),
                                   __builtin_amdgcn_alignbyte(t4.z, t4.y, (uint32_t)sh),
                                   __builtin_amdgcn_alignbyte(t4.w, t4.z, (uint32_t)sh),
                                   __builtin_amdgcn_alignbyte(t5, t4.w, (uint32_t)sh));
                }
            }
        }
        wave_lds_fence();
        const DevPlane &Qc = dj.cur.lv[1];
        const uint8_t *sp0 = uni_ptr(Qc.base + (ptrdiff_t)qy * Qc.stride + qx);
        const int sst      = UNI(Qc.stride);
        unsigned long long a0 = 0, a1 = 0; // position rows 2 pr, 2 pr + 1
        // reference row 2 pr + t of the window: block row t of position row 2 pr (D0)
        // and block row t - 1 of 2 pr + 1 (D1); lanes without a position read row
        // rlast / column quad 0 (their keys are dropped)
        auto row = [&](int t, auto D0, auto D1, auto FW) {
            constexpr bool do0 = decltype(D0)::value, do1 = decltype(D1)::value, fw = decltype(FW)::value;
            const uint32_t *wr = win + min(2 * pr + t, rlast) * L1W_PITCH + qcol;
            // source rows t and t - 1: scalar loads (nothing carried between rows)
            const uint8_t *s0 = sp0 + (ptrdiff_t)(do0 ? t : t - 1) * sst;
            const uint4 c0 = sld4(s0), c1 = sld4(s0 + 16);
            const uint4 p0 = do0 && do1 ? sld4(s0 - sst) : c0, p1 = do0 && do1 ? sld4(s0 - sst + 16) : c1;
            const uint32_t sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
            const uint32_t sp[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (fw || k < nd) {
                    const u32x2a4 v              = *(const u32x2a4 *)(wr + k);
                    const unsigned long long pk = pair(v.x, v.y);
                    if (do0)
                        a0 = qsad64(pk, sc[k], a0);
                    if (do1)
                        a1 = qsad64(pk, do0 ? sp[k] : sc[k], a1);
                }
            }
        };
        auto flush = [&]() { // at most 8 block rows per u16 lane (8 x 32 x 255 < 2^16)
            qsad_unpack(a0, acc32[0]);
            qsad_unpack(a1, acc32[1]);
            a0 = a1 = 0;
        };
        auto rows = [&](auto FW) {
            row(0, std::true_type(), std::false_type(), FW);
            for (int t0 = 1; t0 < bh;) { // chunks [1, 8), [8, 16), ...: position row 2 pr gets 8 rows per flush
                const int t1 = min((t0 | 7) + 1, bh);
                for (int t = t0; t < t1; t++)
                    row(t, std::true_type(), std::true_type(), FW);
                flush();
                t0 = t1;
            }
            row(bh, std::false_type(), std::true_type(), FW);
            flush();
        };
        if (nd == 8)
            rows(std::true_type());
        else
            rows(std::false_type());
    }
    // keys (sad << 32 | y << 16 | x) of this lane's positions inside the area, then
    // the minimum over the 32 lanes of the half (DPP in rows, then rows 0 + 2 / 1 + 3)
    unsigned long long best = ~0ull;
    if (search) {
#pragma unroll
        for (int yy = 0; yy < 2; yy++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int x = 4 * qd + e, y = 2 * pr + yy;
                if (x < sw && y < shh) {
                    const unsigned long long k = ((unsigned long long)acc32[yy][e] << 32) | ((uint32_t)y << 16) | (uint32_t)x;
                    best = k < best ? k : best;
                }
            }
    }
    {
        auto step = [&](uint32_t tl, uint32_t th) {
            const unsigned long long t = ((unsigned long long)th << 32) | tl;
            best                       = t < best ? t : best;
        };
#define L1MIN(CTRL, RM) step(dpp_or<CTRL, RM>((uint32_t)best, U32MAX), dpp_or<CTRL, RM>((uint32_t)(best >> 32), U32MAX))
        L1MIN(DPP_ROW_SHR(1), 0xF);
        L1MIN(DPP_ROW_SHR(2), 0xF);
        L1MIN(DPP_ROW_SHR(4), 0xF);
        L1MIN(DPP_ROW_SHR(8), 0xF);
#undef L1MIN
    }
    auto rowmin = [&](int ln) {
        return ((unsigned long long)rl32((uint32_t)(best >> 32), ln) << 32) | rl32((uint32_t)best, ln);
    };
    const unsigned long long kb0 = rowmin(15), kb1 = rowmin(47), kt0 = rowmin(31), kt1 = rowmin(63);
    const unsigned long long kb = kb0 < kb1 ? kb0 : kb1, kt = kt0 < kt1 ? kt0 : kt1;
    if (search) {
        uint32_t bs;
        int x, y;
        key_result(half ? kt : kb, &bs, &x, &y);
        SD = bs; // full-SAD rows: not doubled
        X  = i16((x + xo) * 2);
        Y  = i16((y + yo) * 2);
    }
    if ((lane & 47) == 0) { // lanes 0 and 16
        b->hx[s][q]   = X;
        b->hy[s][q]   = Y;
        b->hsad[s][q] = SD;
    }
}

// Per SB: decode the argmin keys kb[k][85] of the R records (slot state cin[k])
// into best SAD / MV per PU (strict-< first minimum in search order), then
// stage_c_tail; all threads of the workgroup. reset: leave kb at ~0 (banded
// jobs merge into it with atomic min). Wavefront w decodes the records w, w + 4
// whole (its lanes the 64 8x8 PUs, then 21 the larger ones) and sums the 8x8
// best SADs of each for me_prune_ref on the way (st.sum8): no serial sums later.
__device__ __forceinline__ void stage_e_body(StC &st, const DevJob &dj, uint32_t sb_local,
                                             const SbGeo &G, uint32_t vmask, const CSlot *cin,
                                             unsigned long long *kb, bool reset) {
    const svtme_job &job = dj.job;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const int R = (int)dj.R, nr0 = (int)SF(job, num_refs[0]);
    // the slot state in one pass: slot tid's record (k), or the defaults of a slot without one
    if (tid < 8) {
        const int s    = tid;
        const int k    = s < 4 ? s : nr0 + (s - 4);
        const bool has = s < 4 ? s < nr0 : k < R;
        CSlot v{};
        if (has)
            v = cin[k];
        st.hme_sad[s]  = has ? v.hme_sad : U32MAX;
        st.zz[s]       = has ? v.zz : U32MAX;
        st.sc_x[s]     = has ? v.sc_x : 0;
        st.sc_y[s]     = has ? v.sc_y : 0;
        st.searched[s] = has ? v.searched : 0;
        st.do_ref[s]   = has ? v.do_ref : 0;
        if (!(has && v.searched)) // (a searched slot's sum: its record's decode below)
            st.sum8[s] = 0;
        if (s == (nr0 > 0 ? 0 : 4)) // record 0's
            st.tf_exit = has ? v.tf_exit : 0;
    }
    // the records' decode reads its record's state straight from cin (not the slot
    // state above): no barrier between the two
    for (int kk = wid; kk < R; kk += 4) {
        const int s      = kk < nr0 ? kk : 4 + (kk - nr0);
        const CSlot &v   = cin[kk];
        const bool srch  = v.searched != 0;
        const uint32_t wm = srch ? magic_u32((uint32_t)max(1, (int)v.w)) : 0u;
        auto decode = [&](int pu, uint32_t &sad, uint32_t &mv) {
            sad = U32MAX, mv = 0;
            if (srch) {
                const size_t e                = (size_t)kk * SVTME_PU_COUNT + pu;
                const unsigned long long key = kb[e];
                if (reset)
                    kb[e] = ~0ull; // keys rest at ~0 for the next banded job
                const uint32_t o = (uint32_t)key;
                sad              = (uint32_t)(key >> 32);
                int16_t mx, my;
                if (v.probe && o == 0) {
                    mx = v.xc;
                    my = v.yc;
                } else { // p / w by multiply-high (p * w < 2^32)
                    const int p = (int)o - (int)v.probe;
                    const int q = mdiv(p, wm);
                    my          = i16(v.yo + q);
                    mx          = i16(v.xo + (p - q * v.w));
                }
                mv = ((uint32_t)(uint16_t)my << 16) | (uint16_t)mx;
            }
            st.rec[s][pu]                  = sad;
            st.rec[s][SVTME_PU_COUNT + pu] = mv;
        };
        uint32_t sad, mv;
        decode(21 + lane, sad, mv); // the 8x8 PUs
        if (srch) {                 // me_prune_ref's sum (searched == do_ref outside MCTF; < 2^21)
            const uint32_t t = wave_sum_u32(sad);
            if (lane == 0)
                st.sum8[s] = t;
        }
        if (lane < 21)
            decode(lane, sad, mv); // 64x64, 32x32, 16x16
    }
    __syncthreads();
    stage_c_tail<true>(st, dj, sb_local, G.bw, G.bh, vmask);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_stage_e(const DevBatch B) {
    __shared__ StC st;
    uint32_t sb_local;
    const DevJob &dj     = batch_job(B, xcd_remap(blockIdx.x, gridDim.x), &sb_local);
    const SbGeo G        = sb_geo(dj, sb_local);
    const uint32_t vmask = valid_mask(dj.job);
    stage_e_body(st, dj, sb_local, G, vmask, dj.cslot + (size_t)sb_local * dj.R,
                 dj.keys + (size_t)sb_local * dj.R * SVTME_PU_COUNT, dj.parts > 1);
}

struct HmeA { // state of phases A0 .. B
    Dec d;
    unsigned long long key[SVTME_A_N]; // search minima by ARes index
    int16_t kxo[SVTME_A_N], kyo[SVTME_A_N];
    uint32_t need;                     // bit slot * 2: pre-HME searched, slot * 2 + 1: HME-L0 searched
    HSrch srch[48];
    int32_t nsrch, nitems;
    int32_t nitems3, base2; // end of the HT16-row tiles; first item of the 2-row group (64-aligned)
    int32_t end1, base3;    // end of the first A1 round; first item of the gated list-1 pre-HME group
    unsigned long long key1[32];
    int16_t x1o[32], y1o[32];
    HSrch1 s1[32];
    int32_t nsrch1, nitems1;
    int16_t hx[32], hy[32];
    uint64_t hsad[32];
    __attribute__((aligned(16))) uint8_t src4[16][32]; // quarter-resolution source, sub rows
    __attribute__((aligned(16))) uint8_t src1[32][HL2_PITCH]; // full-resolution source, sub rows (HME-L2)
};

// A1 search table (wave 0): lane = slot * 6 + k, k < 2 pre-HME region k, else
// HME-L0 quadrant k - 2. RND 0: every search the slots may need. The real-time
// tune's HME-L0 reduction (reduce_hme_l0_sr_th, enc_mode_config.c:692-704) makes
// the HME-L0 areas of slots 1-7 depend on slot 0's HME-L0 centre after its
// worst-quadrant replacement (get_hme_l0_search_area, motion_estimation.c:
// 1800-1867, called in slot order by hme_level0_b64 :1974-2036); then RND 1
// has every search but those, and RND 2 those alone: the slots of bit set
// l0need, areas from the centre (l00x, l00y)
// GATE (RND 0): the list-1 pre-HME regions form a group of their own after the
// others, searched in a second round only where check_prehme_early_exit
// (motion_estimation.c:1693-1719) does not mirror list 0's result (a1_gated)
template <int RND>
__device__ __forceinline__ void a1_table(HmeA &A, const DevJob &dj, uint32_t vmask, int16_t sox, int16_t soy, int kh,
                                         uint32_t l0need = 0, int16_t l00x = 0, int16_t l00y = 0,
                                         bool gate = false) {
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const int lane          = threadIdx.x & 63;
    // lane = slot * 6 + k: k < 2 pre-HME region k, else HME-L0 quadrant k - 2
    const int s = lane / 6, k = lane - 6 * (lane / 6), l = s >> 2;
    bool on = lane < 48 && slot_valid(vmask, s) && tl_or_l0(job, l) &&
              (k < 2 ? c.prehme_enable != 0 : (c.enable_hme_flag && c.enable_hme_level0_flag));
    if (RND == 1)
        on = on && (k < 2 || s == 0);
    if (RND == 2)
        on = on && k >= 2 && s > 0 && ((l0need >> s) & 1u);
    bool mk    = false;
    int items3 = 0, items2 = 0;
    HSrch e;
    if (on) {
        const DevPlane &P = dj.ref[l][s & 3].lv[2];
        int16_t aw = k < 2 ? dj.ph_sa[s][k][0] : dj.l0_sa[s][0];
        int16_t ah = k < 2 ? dj.ph_sa[s][k][1] : dj.l0_sa[s][1];
        if (RND == 2) // get_hme_l0_search_area from the first slot's centre (:1800-1867)
            hme_l0_area(c, l, s & 3, dj.sdist[s], l00x, l00y, &aw, &ah);
        int16_t xo, yo, sw, shh;
        bool skip;
        if (k < 2) { // prehme_core (motion_estimation.c:1568-1636)
            prehme_area(P, sox, soy, aw, ah, &xo, &yo, &sw, &shh);
            skip   = c.prehme_skip_search_line != 0; // compute_sad_c.c:74 (16 wide, <= 16 rows)
            e.id   = (uint8_t)(SVTME_A_PH + s * 2 + k);
            e.need = (uint8_t)(s * 2);
        } else { // hme_level_0 (motion_estimation.c:835-889)
            hme_l0_rect(c, P, sox, soy, aw, ah, (k - 2) >> 1, (k - 2) & 1, &xo, &yo, &sw, &shh);
            skip   = false;
            e.id   = (uint8_t)(SVTME_A_L0 + s * 4 + (k - 2));
            e.need = (uint8_t)(s * 2 + 1);
        }
        A.kxo[e.id]    = xo;
        A.kyo[e.id]    = yo;
        const int nrows = (sw > 0 && shh > 0) ? (skip ? shh / 2 : shh) : 0;
        if (nrows > 0) {
            const uint8_t *w0 = P.base + (ptrdiff_t)(soy + yo) * P.stride + (sox + xo);
            e.sh              = (uint8_t)((uintptr_t)w0 & 3);
            e.a0              = w0 - e.sh;
            e.sa_w            = sw;
            e.skip            = skip;
            const int nq      = (e.sh + sw + 3) >> 2;
            e.ncols           = (int16_t)((nq + HQ16 - 1) / HQ16);
            e.ncm             = magic_u32((uint32_t)e.ncols);
            if (skip) {
                e.cnt0  = (int16_t)nrows;
                e.cnt1  = 0;
                e.ylast = (int16_t)(2 * nrows - 1 + 2 * (kh - 1));
                items3  = e.ncols * ((nrows + HT16 - 1) / HT16);
                items2  = e.ncols * ((nrows + 1) / 2);
            } else {
                e.cnt0  = (int16_t)((nrows + 1) >> 1);
                e.cnt1  = (int16_t)(nrows >> 1);
                e.ylast = (int16_t)(nrows - 1 + 2 * (kh - 1));
                items3  = e.ncols * 2 * ((e.cnt0 + HT16 - 1) / HT16);
                items2  = e.ncols * 2 * ((e.cnt0 + 1) / 2);
            }
            mk = true;
        }
    }
    // Tile shapes: a wavefront's qsad count is its tiles' row count x 64 lanes, so
    // the HME-L0 quadrants (few rows per parity, e.g. 2 at p8, wasting a third of
    // a 3-row tile) take 2-row tiles in wavefronts of their own when that needs
    // fewer wavefront-rows: the 3-row group first, the 2-row group from the next
    // multiple of 64 items
    const bool l0    = k >= 2;
    const bool g     = RND == 0 && gate && mk && !l0 && l == 1; // the gated group (second round)
    const int n3_pre = (int)wave_sum_u32(mk && !l0 && !g ? (uint32_t)items3 : 0u);
    const int n3_l0  = (int)wave_sum_u32(mk && l0 ? (uint32_t)items3 : 0u);
    const int n2_l0  = (int)wave_sum_u32(mk && l0 ? (uint32_t)items2 : 0u);
    const bool split = ((n3_pre + 63) / 64) * HT16 + ((n2_l0 + 63) / 64) * 2 < ((n3_pre + n3_l0 + 63) / 64) * HT16;
    const bool t2    = mk && split && l0;
    const int items  = t2 ? items2 : items3;
    e.tt             = (uint8_t)(t2 ? 2 : HT16);
    int n3s, n2s, ngs;
    const int k3 = wave_compact(mk && !t2 && !g, &n3s), k2 = wave_compact(t2, &n2s), kg = wave_compact(g, &ngs);
    const int i3 = wave_incl_scan(mk && !t2 && !g ? items : 0), i2 = wave_incl_scan(t2 ? items : 0);
    const int ig = wave_incl_scan(g ? items : 0);
    const int N3 = (int)lane63((uint32_t)i3), N2 = (int)lane63((uint32_t)i2), NG = (int)lane63((uint32_t)ig);
    const int base2 = (N3 + 63) & ~63;
    const int end1  = N2 ? base2 + N2 : N3;
    const int base3 = (end1 + 63) & ~63;
    if (mk) {
        e.item0 = g ? base3 + ig - items : t2 ? base2 + i2 - items : i3 - items;
        A.srch[g ? n3s + n2s + kg : t2 ? n3s + k2 : k3] = e;
    }
    if (lane == 0) {
        A.nsrch   = n3s + n2s + ngs;
        A.nitems3 = N3;
        A.base2   = base2;
        A.end1    = end1;
        A.base3   = NG ? base3 : end1;
        A.nitems  = NG ? base3 + NG : end1;
    }
}

// A1's second round: does check_prehme_early_exit (motion_estimation.c:1693-1719)
// search list-1 pre-HME region e? Its mirror of list 0's region (l1_early_exit:
// sad < 32 x 32 or |mv| < 16 in both components) needs list 0's result, final
// after the first round: zz early exit of the list-0 slot (valid, sad 0), or its
// search's key decoded as phase D decodes it. Only a certain mirror skips the
// search (dec_prehme then takes the mirror without reading the key).
__device__ __forceinline__ bool a1_mirrored(const HmeA &A, const svtme_controls &c, uint32_t need, int id) {
    const int r = ((id - SVTME_A_PH) >> 1) & 3, k = (id - SVTME_A_PH) & 1;
    if (c.me_early_exit_th && A.d.zz[r] < c.me_early_exit_th)
        return true;
    if (!((need >> (2 * r)) & 1u))
        return false;
    const int id0 = SVTME_A_PH + 2 * r + k;
    uint32_t best;
    int x, y;
    key_result(A.key[id0], &best, &x, &y);
    const uint32_t sad = best * 2; // sub-sampled rows (the gated layout is SUB_SAD HME only)
    const int16_t col = i16((x + A.kxo[id0]) * 4), row = i16((y + A.kyo[id0]) * 4); // as phase D stores them
    return sad < 32 * 32 || (absi(col) < 16 && absi(row) < 16);
}

// k_hme shared memory: the job copy, the SB's HME state, the per-record
// full-pel results, and the phase-A..B state overlaid by the stage-C/E state
// (dead by then)
struct HmeSh {
    DevJob dj; // the job, copied once: every later job / control read is an LDS read
    BState bs;
    CSlot cin[8]; // by record
    SlotCentre cen[8]; // final search centre / pruning by slot
    uint8_t tf_exit;
    union U {
        HmeA a;
        StC st;
    } u;
};

// FP: the whole ME pass of the SB in this workgroup (k_stage_c1 with one band
// per record, then k_stage_e); else the HME state goes to BState for them.
// wave 0's serial phases (decisions, search tables, final centre) run at raised
// issue priority: the workgroup's other waves wait for them at a barrier
#define HME_PRIO_HI() __builtin_amdgcn_s_setprio(2)
#define HME_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#define HME_WAVES_PER_EU 8 // 64 VGPRs: 8 workgroups per CU
template <bool FP, bool SUB_ME, bool K32, bool RT = false> // RT: the real-time tune's HME-L0 reduction (a1_table)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HME_WAVES_PER_EU, HME_WAVES_PER_EU))) k_hme(const DevBatch B) {
    __shared__ HmeSh sh;
    const int tid = threadIdx.x, lane = tid & 63, wid = UNI(tid >> 6);
    uint32_t sb_local;
    // the job in the job table (scalar loads where the reads are wave-uniform: the
    // full-pel and decode phases) and its LDS copy (per-lane reads of the HME phases)
    const DevJob &gj = batch_job(B, xcd_remap(blockIdx.x, gridDim.x), &sb_local);
    {
        // one 16-byte load per thread (a loop of dword loads waited for each round trip)
        static_assert(sizeof(DevJob) % 16 == 0 && sizeof(DevJob) / 16 <= 256, "DevJob: one uint4 per thread");
        if (tid < (int)(sizeof(DevJob) / 16))
            ((uint4 *)&sh.dj)[tid] = ((const uint4 *)&gj)[tid];
    }
    __syncthreads();
    const DevJob &dj        = sh.dj;
    const svtme_job &job    = dj.job;
    const svtme_controls &c = job.ctrl;
    const SbGeo G           = sb_geo(dj, sb_local);
    const uint32_t vmask    = valid_mask(job);
    Dec &d                  = sh.u.a.d;
    const int16_t sox = i16(((int16_t)G.ox) >> 2), soy = i16(((int16_t)G.oy) >> 2);
    const int kh  = (int)(G.bh >> 2) >> 1; // 1/16 block rows (sub)
    const int kh1 = (int)(G.bh >> 2);      // 1/4 block rows (sub): (bh / 2) / 2
    const bool zz_on = c.me_early_exit_th || c.me_safe_limit_zz_th;
    HME_STAMP(0);

    // ---- phase 0 (independent work of all waves):
    //   wave 0: zz SADs of every slot (init_zz_sad, motion_estimation.c:2382-2437), lane = sub
    //           row x half row, two batches of loads in flight, then the zz decisions in the same
    //           wave (which searches the reference performs): no barrier between the two
    //   wave 1: A1 search table of every search the slots may need (geometry only)
    //   waves 2-3: the full- and quarter-resolution source blocks of HME-L2 / HME-L1
    if (wid == 0) {
        dec_init(d);
        uint32_t accv = 0; // lane s: slot s's zz sum
        if (zz_on) {
            // the current rows loaded once
            const int r = lane >> 1, h = lane & 1; // sub row r, half row h
            const bool row_in = r < (int)(G.bh >> 1);
            const DevPlane &C = dj.cur.lv[0];
            u32x4a4 b0{}, b1{};
            if (row_in) {
                const uint32_t *cr = (const uint32_t *)(C.base + (ptrdiff_t)(G.oy + 2 * r) * C.stride + G.ox) + 8 * h;
                b0 = ldg4(cr), b1 = ldg4(cr + 4);
            }
            // every slot's plane address first, then the slots' reference
            // rows in three batches (3, 3, 2 slots), each batch's loads issued before the
            // previous batch's SADs: two batches in flight, not one round trip per batch
            // (from the job in global memory: scalar loads into SGPRs)
            const uint8_t *fb[8];
            int fs[8];
#pragma unroll
            for (int sl = 0; sl < 8; sl++) {
                fb[sl] = gj.ref[sl >> 2][sl & 3].lv[0].base;
                fs[sl] = gj.ref[sl >> 2][sl & 3].lv[0].stride;
            }
            u32x4a4 a[8][2];
            bool sv[8];
            auto issue = [&](int sl) {
                sv[sl]    = slot_valid(vmask, sl) && tl_or_l0(job, sl >> 2);
                a[sl][0] = a[sl][1] = u32x4a4{};
                if (sv[sl] && row_in) {
                    const uint32_t *rr =
                        (const uint32_t *)(fb[sl] + (ptrdiff_t)(G.oy + 2 * r) * fs[sl] + G.ox) + 8 * h;
                    a[sl][0] = ldg4(rr), a[sl][1] = ldg4(rr + 4);
                }
            };
            auto sum = [&](int sl) {
                if (!sv[sl])
                    return;
                uint32_t acc = 0;
                if (row_in) {
                    acc = __builtin_amdgcn_sad_u8(a[sl][0].x, b0.x, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][0].y, b0.y, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][0].z, b0.z, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][0].w, b0.w, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][1].x, b1.x, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][1].y, b1.y, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][1].z, b1.z, acc);
                    acc = __builtin_amdgcn_sad_u8(a[sl][1].w, b1.w, acc);
                }
                const uint32_t t = wave_sum_u32(acc);
                accv             = lane == sl ? t : accv;
            };
            issue(0), issue(1), issue(2);
            issue(3), issue(4), issue(5);
            sum(0), sum(1), sum(2);
            issue(6), issue(7);
            sum(3), sum(4), sum(5);
            sum(6), sum(7);
        }
        HME_PRIO_HI();
        // dec_zz's decisions (init_zz_sad, motion_estimation.c:2382-2437) with the state in
        // registers, lane = slot: every input read in one batch, cross-lane values by
        // readlane / ds_bpermute, one LDS write of the results (no LDS round trips)
        const uint32_t eet = c.me_early_exit_th, slz = c.me_safe_limit_zz_th;
        const uint32_t zth = c.zz_sad_th;
        const uint32_t zpct = c.zz_sad_pct;
        const int tli = job.temporal_layer_index, hl = job.hierarchical_levels, nl = job.num_lists;
        const bool sbr = job.similar_brightness_refs != 0;
        const uint32_t acc = accv;
        const bool have    = slot_valid(vmask, lane) && tl_or_l0(job, lane >> 2);
        uint32_t zz = U32MAX; // (dec_init's state)
        bool dref   = true;
        if (eet || slz) {
            if (have) {
                zz                 = acc << 1;
                const uint32_t pix = G.bw * G.bh; // (32-bit arithmetic as the reference's; a shift for a whole SB)
                zz                 = pix == 4096u ? (zz * 64 * 64) >> 12 : (zz * 64 * 64) / pix;
            }
            const uint32_t best = wave_min_u32(zz);
            if (have && (lane & 3) > 0 && tli > 0 && best < zth && (uint32_t)((zz - best) * 100u) > (uint32_t)(zpct * best))
                dref = false;
            if (slz) {
                const uint32_t z0 = rl32(zz, 0), z4 = rl32(zz, 4);
                const bool safe = hl > 0 && nl == 2 && tli >= hl && sbr && z0 < slz && z4 < slz;
                if (safe && slot_valid(vmask, lane) && (lane & 3) > 0)
                    dref = false;
            }
        }
        if (lane < 8) {
            d.zz[lane]     = zz;
            d.do_ref[lane] = dref ? 1 : 0;
        }
        // the searches the reference performs: lane 2s pre-HME, 2s + 1 HME-L0 of slot s
        const int s       = lane >> 1;
        const uint32_t zs = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * s, (int)zz);
        const uint32_t ds = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * s, dref ? 1 : 0);
        const bool act    = lane < 16 && slot_valid(vmask, s) && tl_or_l0(job, s >> 2) && ds;
        const bool nd     = act && ((lane & 1) ? !(eet && zs < (eet >> 2)) : !(eet && zs < eet));
        const unsigned long long m = __ballot(nd);
        if (lane == 0)
            sh.u.a.need = (uint32_t)m;
        HME_PRIO_LO();
    } else if (wid == 1) {
        if (lane < SVTME_A_N)
            sh.u.a.key[lane] = ~0ull;
        // list-1 pre-HME regions in a second, gated A1 round (a1_mirrored)
        const bool gate = !RT && c.prehme_enable && c.prehme_l1_early_exit && job.num_lists == 2 &&
                          c.hme_search_method != SVTME_FULL_SAD_SEARCH && !(dj.paths & SVTME_PATH_NO_A1_GATE);
        a1_table<RT ? 1 : 0>(sh.u.a, dj, vmask, sox, soy, kh, 0, 0, 0, gate);
    } else {
        // full-resolution source block (64 x 64, even rows) for HME-L2: waves 2-3
        if (c.enable_hme_level2_flag) {
            const DevPlane &F = dj.cur.lv[0];
            const int row = (tid - 128) >> 2, part = tid & 3;
            const u32x4a4 v = ldg4((const uint32_t *)(F.base + (ptrdiff_t)(G.oy + 2 * row) * F.stride + G.ox + 16 * part));
            ((uint4 *)sh.u.a.src1[row])[part] = make_uint4(v.x, v.y, v.z, v.w);
        }
        // quarter-resolution source block (32 x 32, even rows) for HME-L1: threads 128-159
        if (c.enable_hme_level1_flag && tid < 160) {
            const DevPlane &Q = dj.cur.lv[1];
            const int row = (tid - 128) >> 1, half = tid & 1;
            const u32x4a4 v = ldg4((const uint32_t *)(Q.base + (ptrdiff_t)((G.oy >> 1) + 2 * row) * Q.stride +
                                                      (G.ox >> 1) + 16 * half));
            ((uint4 *)sh.u.a.src4[row])[half] = make_uint4(v.x, v.y, v.z, v.w);
        }
    }
    HME_WAVE(0);
    __syncthreads();
    HME_STAMP(1);
    HME_STAMP(2); // (the zz decisions are part of phase 0)
    // ---- A1: pre-HME regions and HME-L0 quadrants, one HT16 x HQ tile per thread
    auto a1_tiles = [&]() {
        // source block of the 1/16 searches (16 x 8 sub rows) into SGPRs (live in A1 only)
        uint32_t sr[8][4];
        {
            const uint8_t *sp = uni_ptr(dj.cur.lv[2].base + (ptrdiff_t)soy * dj.cur.lv[2].stride + sox);
            const int sst     = UNI(dj.cur.lv[2].stride);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint4 v = sld4(sp + (ptrdiff_t)(2 * k) * sst);
                sr[k][0] = v.x, sr[k][1] = v.y, sr[k][2] = v.z, sr[k][3] = v.w;
            }
        }
        const int nitems = sh.u.a.nitems, nsrch = sh.u.a.nsrch;
        const uint32_t need = sh.u.a.need;
        const int pstride = dj.cur.lv[2].stride; // every plane of one level shares the geometry
        const int nitems3 = sh.u.a.nitems3, base2 = sh.u.a.base2, end1 = sh.u.a.end1, base3 = sh.u.a.base3;
        // round 1: items [0, end1); round 2 (gated list-1 pre-HME): [base3, nitems), after a barrier
        auto tiles = [&](auto fullk, int lo, int hi, bool gated) {
            for (int it = lo + tid; it < hi; it += 256) {
                if (it >= nitems3 && it < base2)
                    continue; // the padding before the 2-row group
                const HSrch &e = sh.u.a.srch[find_search(sh.u.a.srch, nsrch, it)];
                if (!((need >> e.need) & 1u))
                    continue;
                if (gated && a1_mirrored(sh.u.a, c, need, e.id))
                    continue; // phase D mirrors list 0's result (check_prehme_early_exit)
                const int local = it - e.item0;
                const int rt = mdiv(local, e.ncm), col = local - rt * e.ncols;
                // the wavefront's tiles all have e.tt rows (the groups are 64-aligned)
                auto run = [&](auto TT) {
                    constexpr int T = decltype(TT)::value;
                    int yf, tv;
                    if (e.skip) {
                        yf = 2 * T * rt + 1;
                        tv = min(T, e.cnt0 - T * rt);
                    } else {
                        const int p = rt & 1, i = rt >> 1;
                        yf = 2 * T * i + p;
                        tv = min(T, (p ? e.cnt1 : e.cnt0) - T * i);
                    }
                    if (tv <= 0)
                        return;
                    const unsigned long long kk = hme_tile16<T, decltype(fullk)::value>(
                        e.a0, pstride, HQ16 * col, e.sh, e.sa_w, yf, tv, e.ylast, kh, sr);
                    if (kk != ~0ull)
                        atomicMin(&sh.u.a.key[e.id], kk);
                };
                if (UNI(it >= base2 && it < base3))
                    run(std::integral_constant<int, 2>());
                else
                    run(std::integral_constant<int, HT16>());
            }
        };
        tiles(std::false_type(), 0, end1, false); // (a kh == 8 specialisation spills: the scheduler hoists every row)
        if (base3 < nitems) { // (workgroup-uniform)
            __syncthreads();
            tiles(std::false_type(), base3, nitems, true);
        }
    };
    a1_tiles();
    if constexpr (RT) {
        // the real-time tune: slot 0's HME-L0 centre after its worst-quadrant
        // replacement (the pre-HME decisions and dec_l0 of slot 0), then the
        // HME-L0 quadrants of slots 1-7 with the areas it selects
        __syncthreads();
        if (wid == 0) {
            HME_PRIO_HI();
            if (lane < SVTME_A_N && lane >= SVTME_A_PH) {
                uint32_t best;
                int x, y;
                key_result(sh.u.a.key[lane], &best, &x, &y);
                d.a[lane] = ARes{best * 2, i16((x + sh.u.a.kxo[lane]) * 4), // (sub-sampled rows)
                                 i16((y + sh.u.a.kyo[lane]) * 4)};
            }
            wave_lds_fence();
            dec_prehme(d, job, vmask);
            dec_l0(d, job, vmask); // slots 1-7 read unsearched keys here: D redoes them
            // the slots whose HME-L0 runs (dec_l0's order of exits)
            const int s = lane;
            bool run    = s > 0 && s < 8 && slot_valid(vmask, s) && tl_or_l0(job, s >> 2) && d.do_ref[s] &&
                       !(c.me_early_exit_th && d.zz[s] < (c.me_early_exit_th >> 2));
            if (run && c.prev_me_stage_based_exit_th) {
                const int k = d.ph[s][0].sad <= d.ph[s][1].sad ? 0 : 1;
                run = !(d.ph[s][k].performed && d.ph[s][k].sad < (c.prev_me_stage_based_exit_th >> 4));
            }
            const uint32_t l0need = (uint32_t)__ballot(run);
            a1_table<2>(sh.u.a, dj, vmask, sox, soy, kh, l0need, d.lx[0][0], d.ly[0][0]);
            if (lane == 0)
                sh.u.a.need = ~0u; // the table holds only searches that run
        }
        __syncthreads();
        HME_PRIO_LO();
        a1_tiles();
    }
    __syncthreads();
    HME_STAMP(3);
    // ---- D: pre-HME and level-0 decisions, then the HME-L1 table (wave 0)
    const bool hsub = c.hme_search_method != SVTME_FULL_SAD_SEARCH; // true on this path
    if (wid == 0) {
        HME_PRIO_HI();
        // lane = slot * 4 + q (lane < 32): the slot's HME-L0 quadrant q (X, Y, SD), its zz SAD and do_ref
        // (the lane id from mbcnt: the compiler would keep lane >> 2 live into the full-pel phase and spill it)
        const int mlane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int s = mlane >> 2, q = mlane & 3, l = s >> 2;
        int16_t X0 = 0, Y0 = 0;
        uint32_t S0 = 0, zzs, drs;
        if constexpr (RT) {
            if (lane < SVTME_A_N && lane >= SVTME_A_PH) {
                uint32_t best;
                int x, y;
                key_result(sh.u.a.key[lane], &best, &x, &y);
                d.a[lane] = ARes{hsub ? best * 2 : best, i16((x + sh.u.a.kxo[lane]) * 4), i16((y + sh.u.a.kyo[lane]) * 4)};
            }
            wave_lds_fence(); // (RT: dec_prehme ran before the second A1 round; its pruning is not idempotent)
            dec_l0(d, job, vmask);
            if (lane < 32) {
                X0 = d.lx[s][q], Y0 = d.ly[s][q], S0 = (uint32_t)d.lsad[s][q];
            }
            zzs = d.zz[s & 7], drs = d.do_ref[s & 7];
        } else {
            // dec_prehme and dec_l0 (motion_estimation.c:1693-1796, 1906-2036) with the state in
            // registers: every input read in one batch, the slot's two pre-HME regions in lanes
            // q = 0, 1 of its quad, cross-lane values by DPP / permlane16_swap (no LDS round trips)
            const svtme_controls &gc = gj.job.ctrl; // (uniform control values: scalar loads)
            const uint32_t eet = gc.me_early_exit_th, pmse = gc.prev_me_stage_based_exit_th;
            const uint32_t phth = gc.phme_sad_th, phpct = SF(gc, phme_sad_pct);
            const bool ph_on = SF(gc, prehme_enable) != 0, l1ee = SF(gc, prehme_l1_early_exit) != 0;
            const bool l0_on = SF(gc, enable_hme_flag) && SF(gc, enable_hme_level0_flag);
            const int tli    = (int)SF(gj.job, temporal_layer_index);
            const int i32    = lane & 31;
            const unsigned long long kph = sh.u.a.key[SVTME_A_PH + ((2 * (i32 >> 2) + (q & 1)) & 15)];
            const int pxo = sh.u.a.kxo[SVTME_A_PH + ((2 * (i32 >> 2) + (q & 1)) & 15)];
            const int pyo = sh.u.a.kyo[SVTME_A_PH + ((2 * (i32 >> 2) + (q & 1)) & 15)];
            const unsigned long long kl0 = sh.u.a.key[SVTME_A_L0 + i32];
            const int lxo = sh.u.a.kxo[SVTME_A_L0 + i32], lyo = sh.u.a.kyo[SVTME_A_L0 + i32];
            zzs = d.zz[s & 7];
            drs = d.do_ref[s & 7];
            const bool sv   = lane < 32 && slot_valid(vmask, s);
            const bool tl   = tli > 0 || l == 0;
            // pre-HME region q of slot s (q < 2): psad, pcr (col | row << 16), valid, performed
            uint32_t psad = 0, pcr = 0;
            bool pval = false, pperf = false;
            if (ph_on) {
                const bool have = sv && q < 2 && tl;
                uint32_t kb;
                int kx, ky;
                key_result(kph, &kb, &kx, &ky);
                if (have) {
                    if (eet && zzs < eet) { // check_prehme_early_exit
                        pval = true;
                    } else if (!drs) {
                        psad = U32MAX;
                    } else { // searched in A1
                        psad  = hsub ? kb * 2 : kb;
                        pcr   = (uint32_t)(uint16_t)i16((kx + pxo) * 4) | ((uint32_t)(uint16_t)i16((ky + pyo) * 4) << 16);
                        pval  = true;
                        pperf = true;
                    }
                }
                // list 1 mirrors list 0's region (lane - 16) when it is certain (:1693-1719)
                const auto zs = __builtin_amdgcn_permlane16_swap(psad, psad, false, false);
                const auto zc = __builtin_amdgcn_permlane16_swap(pcr, pcr, false, false);
                const auto zv = __builtin_amdgcn_permlane16_swap(pval ? 1u : 0u, pval ? 1u : 0u, false, false);
                const uint32_t zsad = zs[0], zcr = zc[0];
                const int zcol = (int)(int16_t)(zcr & 0xFFFFu), zrow = (int)(int16_t)(zcr >> 16);
                if (have && l == 1 && l1ee && !(eet && zzs < eet) && zv[0] &&
                    (zsad < 32 * 32 || (absi(zcol) < 16 && absi(zrow) < 16))) {
                    psad  = zsad;
                    pcr   = (uint32_t)(uint16_t)(int16_t)-zcol | ((uint32_t)(uint16_t)(int16_t)-zrow << 16);
                    pval  = true;
                    pperf = false;
                }
                // the slot's best pre-HME SAD against the best slot's (:1773-1796)
                const uint32_t p0 = dpp_or<0x00>(psad, 0u), p1 = dpp_or<0x55>(psad, 0u); // quad lanes 0, 1
                const uint32_t m  = sv && tl ? min_u32(p0, p1) : U32MAX;
                const uint32_t bm = wave_min_u32(m);
                if (tli > 0 && bm < phth && sv && (s & 3) > 0 && drs && (uint32_t)((m - bm) * 100u) > (uint32_t)(phpct * bm))
                    drs = 0;
            }
            // level 0 of quadrant q (dec_l0)
            bool srch = false;
            if (l0_on) {
                // the slot's pre-HME region with the lower SAD (quad lanes 0, 1)
                const uint32_t s0 = dpp_or<0x00>(psad, 0u), s1 = dpp_or<0x55>(psad, 0u);
                const uint32_t c0 = dpp_or<0x00>(pcr, 0u), c1 = dpp_or<0x55>(pcr, 0u);
                const uint32_t f0 = dpp_or<0x00>(pperf ? 1u : 0u, 0u), f1 = dpp_or<0x55>(pperf ? 1u : 0u, 0u);
                const bool k1     = !(s0 <= s1);
                const uint32_t bs = k1 ? s1 : s0, bcr = k1 ? c1 : c0;
                const bool bperf  = (k1 ? f1 : f0) != 0;
                uint32_t kb;
                int kx, ky;
                key_result(kl0, &kb, &kx, &ky);
                if (sv) {
                    if (eet && zzs < (eet >> 2)) {
                    } else if (pmse && bperf && bs < (pmse >> 4)) {
                        X0 = (int16_t)(bcr & 0xFFFFu), Y0 = (int16_t)(bcr >> 16), S0 = bs;
                    } else if (!drs) {
                        S0 = U32MAX;
                    } else if (tl) {
                        X0   = i16((kx + lxo) * 4);
                        Y0   = i16((ky + lyo) * 4);
                        S0   = hsub ? kb * 2 : kb;
                        srch = true;
                    }
                }
                // pre-HME replaces the worst quadrant of each searched slot (:2005-2032)
                const unsigned long long sm = __ballot(srch);
                if (ph_on && lane < 32 && ((sm >> (4 * s)) & 0xFu)) {
                    const uint32_t q0 = dpp_or<0x00>(S0, 0u), q1 = dpp_or<0x55>(S0, 0u);
                    const uint32_t q2 = dpp_or<0xAA>(S0, 0u), q3 = dpp_or<0xFF>(S0, 0u);
                    int wq = 0; // get_worst_quadrant: strict > in (0,0),(1,0),(0,1),(1,1) order
                    uint32_t mx = 0;
                    if (q0 > mx) { mx = q0; wq = 0; }
                    if (q2 > mx) { mx = q2; wq = 2; }
                    if (q1 > mx) { mx = q1; wq = 1; }
                    if (q3 > mx) { wq = 3; }
                    const uint32_t sw = wq == 0 ? q0 : wq == 1 ? q1 : wq == 2 ? q2 : q3;
                    if (q == wq && bs < sw) {
                        S0 = bs;
                        X0 = (int16_t)(bcr & 0xFFFFu);
                        Y0 = (int16_t)(bcr >> 16);
                    }
                }
            }
            // the decisions' state for phase B's copy to BState
            if (lane < 32) {
                d.lx[s][q]   = X0;
                d.ly[s][q]   = Y0;
                d.lsad[s][q] = S0;
            }
            if (lane < 32 && q == 0)
                d.do_ref[s] = (uint8_t)drs;
        }
        // HME-L1 per (slot, quadrant), lane = slot * 4 + q (hme_level1_b64, :2041-2122)
        bool mk   = false;
        int items = 0;
        HSrch1 e;
        if (lane < 32) {
            int16_t X = 0, Y = 0;
            uint64_t SD = 0;
            sh.u.a.key1[lane] = ~0ull;
            const bool listed = c.enable_hme_flag && c.enable_hme_level1_flag && slot_valid(vmask, s) &&
                                tl_or_l0(job, l);
            if (listed) { // hme_level1_b64 (motion_estimation.c:2041-2122)
                bool done = false;
                if (c.me_early_exit_th && zzs < (c.me_early_exit_th >> 2)) {
                    X = Y = 0;
                    SD   = 0;
                    done = true;
                }
                if (!done && !drs) {
                    X = Y = 0;
                    SD   = U32MAX;
                    done = true;
                }
                if (!done && c.prev_me_stage_based_exit_th && S0 < (c.prev_me_stage_based_exit_th >> 5)) {
                    X = X0, Y = Y0, SD = S0;
                    done = true;
                }
                if (!done) { // hme_level_1 (motion_estimation.c:923-1022)
                    const DevPlane &P = dj.ref[l][s & 3].lv[1];
                    const int16_t qx = i16(((int16_t)G.ox) >> 1), qy = i16(((int16_t)G.oy) >> 1);
                    int16_t xo, yo, sw, shh;
                    hme_refine_rect(1, P, qx, qy, (int16_t)c.hme_l1_sa.width, (int16_t)c.hme_l1_sa.height,
                                    i16(X0 >> 1), i16(Y0 >> 1), &xo, &yo, &sw, &shh);
                    sh.u.a.x1o[lane] = xo;
                    sh.u.a.y1o[lane] = yo;
                    SD           = ~0ull; // searched: resolved from key1 below
                    if (sw > 0 && shh > 0 && kh1 > 0) {
                        const uint8_t *w0 = P.base + (ptrdiff_t)(qy + yo) * P.stride + (qx + xo);
                        e.sh              = (uint8_t)((uintptr_t)w0 & 3);
                        e.a0              = w0 - e.sh;
                        e.sa_w            = sw;
                        e.ncols           = (int16_t)((((sw + 3) >> 2) + HQ1 - 1) / HQ1); // realigned rows
                        e.ncm             = magic_u32((uint32_t)e.ncols);
                        e.id              = (uint8_t)lane;
                        items             = e.ncols * shh;
                        mk                = true;
                    }
                }
            }
            sh.u.a.hx[lane]   = X;
            sh.u.a.hy[lane]   = Y;
            sh.u.a.hsad[lane] = SD;
        }
        int tot;
        const int kpos = wave_compact(mk, &tot);
        const int incl = wave_incl_scan(items);
        if (mk) {
            e.item0     = incl - items;
            sh.u.a.s1[kpos] = e;
        }
        if (lane == 63)
            sh.u.a.nitems1 = incl;
        if (lane == 0)
            sh.u.a.nsrch1 = tot;
    }
    __syncthreads();
    HME_PRIO_LO();
    HME_STAMP(4);
    // ---- B: HME-L1 tiles, 4 lanes (block-row quarters) per tile
    {
        const int nlanes = 4 * sh.u.a.nitems1, nsrch = sh.u.a.nsrch1;
        const int pstride = dj.cur.lv[1].stride;
        auto tiles = [&](auto fullk) {
            for (int it4 = tid; it4 < nlanes; it4 += 256) {
                const int it    = it4 >> 2;
                const HSrch1 &e = sh.u.a.s1[find_search(sh.u.a.s1, nsrch, it)];
                const int local = it - e.item0;
                const int y = mdiv(local, e.ncm), col = local - y * e.ncols;
                const unsigned long long kk = hme_tile32q<decltype(fullk)::value>(e.a0, pstride, HQ1 * col, e.sh,
                                                                                  e.sa_w, y, kh1, sh.u.a.src4);
                if ((it4 & 3) == 0 && kk != ~0ull)
                    atomicMin(&sh.u.a.key1[e.id], kk);
            }
        };
        tiles(std::false_type()); // (a kh1 == 16 specialisation measured slower)
    }
    __syncthreads();
    // resolve the searched level-1 refinements (full-pel units: x 2)
    if (wid == 0 && lane < 32 && sh.u.a.hsad[lane] == ~0ull) {
        uint32_t best;
        int x, y;
        key_result(sh.u.a.key1[lane], &best, &x, &y);
        sh.u.a.hsad[lane] = hsub ? (uint64_t)best * 2 : best;
        sh.u.a.hx[lane]   = i16((x + sh.u.a.x1o[lane]) * 2);
        sh.u.a.hy[lane]   = i16((y + sh.u.a.y1o[lane]) * 2);
    }
    if (c.enable_hme_level2_flag) { // hme_level2_b64 (motion_estimation.c:2127-2177), every listed (slot, quadrant)
        if (wid == 0) {
            const int s = lane >> 2, l = s >> 2;
            bool mk   = false;
            int items = 0;
            HSrch1 e;
            if (lane < 32) {
                sh.u.a.key1[lane] = ~0ull;
                const bool listed = c.enable_hme_flag && slot_valid(vmask, s) && tl_or_l0(job, l);
                const bool keep   = c.prev_me_stage_based_exit_th &&
                                  sh.u.a.hsad[lane] < (c.prev_me_stage_based_exit_th >> 2);
                if (listed && !keep) { // hme_level_2 (:1025-1113) around the level-1 centre
                    const DevPlane &P = dj.ref[l][s & 3].lv[0];
                    int16_t xo, yo, sw, shh;
                    hme_refine_rect(2, P, (int16_t)G.ox, (int16_t)G.oy, (int16_t)c.hme_l2_sa.width,
                                    (int16_t)c.hme_l2_sa.height, sh.u.a.hx[lane], sh.u.a.hy[lane], &xo, &yo, &sw, &shh);
                    sh.u.a.x1o[lane]  = xo;
                    sh.u.a.y1o[lane]  = yo;
                    sh.u.a.hsad[lane] = ~0ull; // searched: resolved from key1 below
                    if (sw > 0 && shh > 0) {
                        const uint8_t *w0 = P.base + (ptrdiff_t)((int16_t)G.oy + yo) * P.stride + ((int16_t)G.ox + xo);
                        e.sh              = (uint8_t)((uintptr_t)w0 & 3);
                        e.a0              = w0 - e.sh;
                        e.sa_w            = sw;
                        e.ncols           = (int16_t)((((sw + 3) >> 2) + HQ - 1) / HQ); // realigned rows
                        e.ncm             = magic_u32((uint32_t)e.ncols);
                        e.id              = (uint8_t)lane;
                        items             = e.ncols * shh;
                        mk                = true;
                    }
                }
            }
            int tot;
            const int kpos = wave_compact(mk, &tot);
            const int incl = wave_incl_scan(items);
            if (mk) {
                e.item0            = incl - items;
                sh.u.a.s1[kpos] = e;
            }
            if (lane == 63)
                sh.u.a.nitems1 = incl;
            if (lane == 0)
                sh.u.a.nsrch1 = tot;
        }
        __syncthreads();
        {
            const int nlanes = 8 * sh.u.a.nitems1, nsrch = sh.u.a.nsrch1;
            const int pstride = dj.cur.lv[0].stride;
            const int kh2     = (int)(G.bh >> 1);
            for (int it8 = tid; it8 < nlanes; it8 += 256) {
                const int it    = it8 >> 3;
                const HSrch1 &e = sh.u.a.s1[find_search(sh.u.a.s1, nsrch, it)];
                const int local = it - e.item0;
                const int y = mdiv(local, e.ncm), col = local - y * e.ncols;
                const unsigned long long kk = hme_tile64(e.a0, pstride, HQ * col, e.sh, e.sa_w, y, kh2, sh.u.a.src1);
                if ((it8 & 7) == 0 && kk != ~0ull)
                    atomicMin(&sh.u.a.key1[e.id], kk);
            }
        }
        __syncthreads();
        if (wid == 0 && lane < 32 && sh.u.a.hsad[lane] == ~0ull) {
            uint32_t best;
            int x, y;
            key_result(sh.u.a.key1[lane], &best, &x, &y);
            sh.u.a.hsad[lane] = hsub ? (uint64_t)best * 2 : best;
            sh.u.a.hx[lane]   = i16(x + sh.u.a.x1o[lane]);
            sh.u.a.hy[lane]   = i16(y + sh.u.a.y1o[lane]);
        }
    }
    HME_STAMP(5);
    BState *b = FP ? &sh.bs : dj.bst + sb_local;
    if (wid == 0) {
        if (lane < 32) {
            b->hx[0][lane]         = sh.u.a.hx[lane];
            b->hy[0][lane]         = sh.u.a.hy[lane];
            b->hsad[0][lane]       = sh.u.a.hsad[lane];
            (&b->lx[0][0])[lane]   = (&d.lx[0][0])[lane];
            (&b->ly[0][0])[lane]   = (&d.ly[0][0])[lane];
            (&b->lsad[0][0])[lane] = (&d.lsad[0][0])[lane];
        }
        if (lane < 8) {
            b->zz[lane]     = d.zz[lane];
            b->do_ref[lane] = d.do_ref[lane];
        }
    }
    if (!FP) {
        HME_STAMP(6);
        return;
    }
    // (no barrier: wave 0 alone reads the phase A..B state above and then the BState in
    // LDS; the other waves write nothing before the barrier after the final centre, from
    // which StC overlays the A..B state)
    // ---- C: set_final_seach_centre_sb / hme_prune_ref_and_adjust_sr once (wave 0), then
    // integer_search_b64 of every record, one wavefront each (k_stage_c1, one band)
    if (wid == 0) {
        HME_PRIO_HI();
        wave_lds_fence(); // (the BState other lanes of this wave just wrote)
        const SlotCentre scv = final_centre(gj.job, &sh.bs, vmask); // lane = slot (controls by scalar loads)
        if (lane < 8)
            sh.cen[lane] = scv;
        if (lane == 0)
            sh.tf_exit = job.me_type == SVTME_ME_MCTF && scv.hme_sad < job.tf_me_exit_th; // :3109-3113
    }
    __syncthreads();
    HME_PRIO_LO();
    HME_STOP(55);
    for (int k = wid; k < (int)dj.R; k += 4) {
        constexpr int ROWS = SUB_ME ? 4 : 8, RSTEP = SUB_ME ? 2 : 1;
        // an opaque lane index: the block's address terms are made per record, not hoisted
        // out of this loop (live across it, they spill at 64 VGPRs)
        int fl = lane;
        asm volatile("" : "+v"(fl));
        const int z16 = fl >> 2, k4 = fl & 3;
        const int by  = ((z16 >> 3) << 2) | (((z16 >> 1) & 1) << 1) | (k4 >> 1);
        const int bx  = (((z16 >> 2) & 1) << 2) | ((z16 & 1) << 1) | (k4 & 1);
        // this lane's 8x8 source block: buffer loads from the SB origin (a 32-bit
        // lane offset; 64-bit per-lane row pointers hoisted out of this loop spill)
        const DevPlane &C = gj.cur.lv[0];
        const int cst     = UNI(C.stride);
        const __amdgpu_buffer_rsrc_t crs = plane_rsrc(uni_ptr(C.base + (ptrdiff_t)G.oy * cst + G.ox));
        const uint32_t coff = (uint32_t)(by * 8 * cst + bx * 8);
        uint32_t src[ROWS][2];
#pragma unroll
        for (int rr = 0; rr < ROWS; rr++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(crs, (int)coff, rr * RSTEP * cst, 0);
            src[rr][0] = v[0];
            src[rr][1] = v[1];
        }
        const int nr0       = (int)SF(gj.job, num_refs[0]);
        const int s         = k < nr0 ? k : 4 + (k - nr0);
        const SlotCentre &v = sh.cen[s];
        fp_slot<SUB_ME, K32, 2, false, HME_WHOLE>(gj, G, s, src, by, bx, rl64(v.hme_sad, 0), (uint32_t)UNI(v.zz), (uint32_t)UNI(v.reduce_div),
                                (int16_t)UNI(v.sc_x), (int16_t)UNI(v.sc_y), (uint8_t)UNI(v.do_ref),
                                (uint8_t)UNI(sh.tf_exit), 0, 1u, &sh.u.st.keys[k][0], &sh.cin[k]);
    }
    HME_WAVE(1);
    __syncthreads();
    HME_STAMP(6);
    // ---- E: decode, me_prune_ref, records, candidates / distortions / GM detection
    stage_e_body(sh.u.st, gj, sb_local, G, vmask, sh.cin, &sh.u.st.keys[0][0], false);
    HME_STAMP(7);
}

} // namespace svtme

// Stage-A search list of a job: every independent search the reference may
// perform for a valid slot (see k_stage_a). Host-side, pure.
extern "C" void svtme_stage_a_list(const svtme_job *job, uint8_t *list, uint32_t *count) {
    const svtme_controls &c = job->ctrl;
    uint32_t n = 0;
    for (int s = 0; s < 8; s++) {
        const int l = s >> 2, r = s & 3;
        if (l >= job->num_lists || r >= job->num_refs[l])
            continue;
        if (!(job->temporal_layer_index > 0 || l == 0))
            continue;
        const bool zz = c.me_early_exit_th || c.me_safe_limit_zz_th;
        const bool l0 = c.enable_hme_flag && c.enable_hme_level0_flag;
        if (svtme_hme_rt(&c) && s > 0) { // HME-L0 in the second round (svtme_stage_a1_list)
            if (zz)
                list[n++] = (uint8_t)((TA_ZZ << 3) | s);
        } else if (zz || l0)
            list[n++] = (uint8_t)((TA_HME << 3) | s);
        if (c.prehme_enable)
            list[n++] = (uint8_t)((TA_PH << 3) | s);
    }
    *count = n;
}

// Real-time tune on the split path: the second stage-A round, the HME-L0
// quadrants of slots 1-7 (areas from slot 0's centre, k_stage_d<true>).
extern "C" void svtme_stage_a1_list(const svtme_job *job, uint8_t *list, uint32_t *count) {
    const svtme_controls &c = job->ctrl;
    uint32_t n = 0;
    if (svtme_hme_rt(&c) && c.enable_hme_flag && c.enable_hme_level0_flag)
        for (int s = 1; s < 8; s++) {
            const int l = s >> 2, r = s & 3;
            if (l >= job->num_lists || r >= job->num_refs[l])
                continue;
            if (!(job->temporal_layer_index > 0 || l == 0))
                continue;
            list[n++] = (uint8_t)((TA_L0RT << 3) | s);
        }
    *count = n;
}

// Stage-B refinement list of a job: every (slot, quadrant) HME level 1/2
// refines (hme_level1_b64 / hme_level2_b64 loop over valid slots with
// temporal_layer_index > 0 || list 0). Host-side, pure.
extern "C" void svtme_stage_b_list(const svtme_job *job, uint8_t *list, uint32_t *count) {
    const svtme_controls &c = job->ctrl;
    uint32_t n = 0;
    if (c.enable_hme_flag && (c.enable_hme_level1_flag || c.enable_hme_level2_flag))
        for (int s = 0; s < 8; s++) {
            const int l = s >> 2, r = s & 3;
            if (l >= job->num_lists || r >= job->num_refs[l])
                continue;
            if (!(job->temporal_layer_index > 0 || l == 0))
                continue;
            for (int q = 0; q < 4; q++) list[n++] = (uint8_t)((s << 2) | q);
        }
    *count = n;
}

// Wide full-pel stage geometry, host-side and pure. The largest search area
// integer_search_b64 can reach (me_sa max, x mv multiplier, x 3/2 variance
// growth, rounded up to 8 columns) decides 32-bit argmin keys, and the number
// of search-row bands per (SB, reference).
static void fp_area_bound(const svtme_controls *c, uint32_t *w, uint32_t *h) {
    // min(sa_min x distance, sa_max) (:1303-1304), x mv multiplier (:1305-1310),
    // rounded up to 8 (:1318), then x 3/2 and rounded again by the variance
    // growth (:1424-1427) when its threshold can be passed
    uint32_t mw = c->me_sa.sa_max.width, mh = c->me_sa.sa_max.height;
    if (c->mv_sa_adj_enabled) {
        mw *= c->mv_sa_adj_sa_multiplier;
        mh *= c->mv_sa_adj_sa_multiplier;
    }
    mw = (mw + 7) & ~7u;
    mh = mh < 3 ? 3 : mh;
    if (c->me_8x8_var_enabled && c->me_sr_mult2_th != 0xFFFFFFFFu) {
        mw = ((mw * 3 / 2) + 7) & ~7u;
        mh = mh * 3 / 2;
    }
    *w = mw;
    *h = mh;
}

// Per-slot search parameters of k_hme that do not depend on the SB: the
// distance, get_hme_l0_search_area (motion_estimation.c:1800-1867, here with
// l00 = (0, 0); with the real-time reduction, svtme_hme_rt, k_hme recomputes
// slots 1-7 per SB) and the pre-HME areas (prehme_core :1580-1587).
extern "C" void svtme_hme_prepare(DevJob *dj) {
    const svtme_job &job    = dj->job;
    const svtme_controls &c = job.ctrl;
    for (int s = 0; s < 8; s++) {
        const int l = s >> 2, r = s & 3;
        const bool valid = l < job.num_lists && r < job.num_refs[l];
        const uint16_t dist = valid ? svtme::ref_dist_const(job, l, r) : 1;
        dj->sdist[s] = dist;
        int16_t w = 0, h = 0;
        if (valid)
            svtme::hme_l0_area(c, l, r, dist, 0, 0, &w, &h);
        dj->l0_sa[s][0] = w;
        dj->l0_sa[s][1] = h;
        const uint32_t f = svtme::scaled_dist(dist);
        for (int k = 0; k < 2; k++) {
            const uint32_t mw = (uint32_t)c.prehme_sa_cfg[k].sa_min.width * f, xw = c.prehme_sa_cfg[k].sa_max.width;
            const uint32_t mh = (uint32_t)c.prehme_sa_cfg[k].sa_min.height * f, xh = c.prehme_sa_cfg[k].sa_max.height;
            dj->ph_sa[s][k][0] = (int16_t)(uint16_t)(mw < xw ? mw : xw);
            dj->ph_sa[s][k][1] = (int16_t)(uint16_t)(mh < xh ? mh : xh);
        }
    }
}

// k_hme applies: every SB 64 wide, sub-sampled HME rows
extern "C" bool svtme_hme_fused(const svtme_job *job) {
    const svtme_controls &c = job->ctrl;
    return (job->width % 64) == 0 && c.hme_search_method != SVTME_FULL_SAD_SEARCH;
}
// the same with the context's path selection (svtme_set_paths) applied
static bool hme_fused(const DevJob &dj) { return svtme_hme_fused(&dj.job) && !(dj.paths & SVTME_PATH_NO_FUSED_HME); }

// the real-time tune's HME-L0 reduction is on (get_hme_l0_search_area,
// motion_estimation.c:1811-1819): k_hme<..., RT = true> only
extern "C" bool svtme_hme_rt(const svtme_controls *c) {
    return c->enable_me_sr_adjustment && c->distance_based_hme_resizing && c->reduce_hme_l0_sr_th_min &&
           c->reduce_hme_l0_sr_th_max;
}

// k_l1_full applies: full-SAD HME rows, HME-L1 without L2, an L1 area of at most
// 16 x 16 positions (TF-ME levels 0-2)
extern "C" bool svtme_l1_full(const svtme_controls *c) {
    return c->hme_search_method == SVTME_FULL_SAD_SEARCH && c->enable_hme_flag && c->enable_hme_level1_flag &&
           !c->enable_hme_level2_flag && c->hme_l1_sa.width <= 16 && c->hme_l1_sa.height <= 16;
}
static bool l1_full(const DevJob &dj) { return svtme_l1_full(&dj.job.ctrl) && !(dj.paths & SVTME_PATH_NO_L1_FULL); }

// k_l0_full applies: full-SAD HME rows, HME-L0 on, no pre-HME, HME-L0 quadrants of
// at most 16 x 8 positions for every slot, whole source dwords on partial SBs
extern "C" bool svtme_l0_full(const DevJob *dj) {
    const svtme_controls &c = dj->job.ctrl;
    if (c.hme_search_method != SVTME_FULL_SAD_SEARCH || c.prehme_enable || !c.enable_hme_flag ||
        !c.enable_hme_level0_flag || svtme_hme_rt(&c) || (dj->job.width % 64) % 16 != 0 ||
        (dj->paths & SVTME_PATH_NO_L0_FULL))
        return false;
    for (int s = 0; s < 8; s++)
        if (dj->l0_sa[s][0] > 16 || dj->l0_sa[s][1] > 16)
            return false;
    return true;
}

// the same test on a job (bench / diagnostics: which kernel runs stage A)
extern "C" bool svtme_l0_full_job(const svtme_job *job) {
    DevJob dj{};
    dj.job = *job;
    svtme_hme_prepare(&dj);
    return svtme_l0_full(&dj);
}

// position rows per lane of k_l0_full: 2 when every quadrant has at most 8 rows
static bool l0_full_short(const DevJob *dj) {
    for (int s = 0; s < 8; s++)
        if (dj->l0_sa[s][1] > 8)
            return false;
    return true;
}

extern "C" bool svtme_fp_k32(const svtme_controls *c) {
    uint32_t w, h;
    fp_area_bound(c, &w, &h);
    return (c->me_8x8_var_enabled ? 1u : 0u) + w * h <= 4096u; // order 0 is the variance probe
}

// the full-pel area's minimum width reaches 24 positions: 6-quad load sets pay
extern "C" bool svtme_fp_wide(const svtme_controls *c) {
    return c->me_sa.sa_min.width >= 24 && c->me_sa.sa_max.width >= 24;
}

// k_fp_wide applies: sub-sampled rows, 32-bit keys, a wide area of more than one
// band, and the window of 4 bands in its LDS rows (FPW_PITCH dwords, bands of
// at most 8 rows with up to 16 parts)
extern "C" bool svtme_fp_wide_lds(const svtme_controls *c) {
    if (c->me_search_method == SVTME_FULL_SAD_SEARCH || c->enable_me_sr_adjustment == 2 || !svtme_fp_k32(c) ||
        !svtme_fp_wide(c))
        return false;
    uint32_t w, h;
    fp_area_bound(c, &w, &h);
    const uint32_t nsets = ((w + 3) / 4 + FPW_TQ - 1) / FPW_TQ;
    return (w * h) / 512 >= 2 && 14 + nsets * FPW_TQ + 2 + 1 <= FPW_BOFF && h <= 8 * 16;
}

static bool fp_wide_lds(const svtme_controls *c, uint32_t paths) {
    return svtme_fp_wide_lds(c) && !(paths & SVTME_PATH_NO_FP_WIDE);
}
static bool fp_wide_lds(const DevJob &dj) { return fp_wide_lds(&dj.job.ctrl, dj.paths); }

// search-row bands per (SB, reference) of the wide full-pel stage under path selection `paths`
extern "C" uint32_t svtme_fp_parts_paths(const svtme_controls *c, uint32_t paths) {
    if (c->enable_me_sr_adjustment == 2)
        return 0; // slot 0's 64x64 SAD feeds the other slots' areas: per-SB k_stage_c
    uint32_t w, h;
    fp_area_bound(c, &w, &h);
    uint32_t parts = (w * h) / 512;
    if (fp_wide_lds(c, paths)) { // workgroups of 4 bands of <= 8 rows
        parts = parts > (h + 7) / 8 ? parts : (h + 7) / 8;
        parts = (parts + 3) & ~3u;
    }
    return parts < 1 ? 1 : (parts > 16 ? 16 : parts);
}
extern "C" uint32_t svtme_fp_parts(const svtme_controls *c) { return svtme_fp_parts_paths(c, 0); }

// Batch launch key: jobs launched together must agree on it (svtme_host.cpp
// splits a batch into groups by it).
extern "C" uint32_t svtme_launch_key(const DevJob *dj) {
    const bool full = dj->job.ctrl.me_search_method == SVTME_FULL_SAD_SEARCH;
    return (uint32_t)full | (uint32_t)(dj->parts != 0) << 1 | (uint32_t)svtme_fp_k32(&dj->job.ctrl) << 2 |
           (uint32_t)(dj->job.ctrl.enable_hme_level2_flag != 0) << 3 | (uint32_t)hme_fused(*dj) << 4 |
           (uint32_t)(dj->parts == 1) << 5 | (uint32_t)svtme_fp_wide(&dj->job.ctrl) << 6 |
           (uint32_t)svtme_hme_rt(&dj->job.ctrl) << 7 | (uint32_t)fp_wide_lds(*dj) << 8 |
           (uint32_t)l1_full(*dj) << 9 | (uint32_t)svtme_l0_full(dj) << 10 |
           (uint32_t)((dj->paths & SVTME_PATH_SPLIT_PASS) != 0) << 11;
}

static DevBatch make_batch(const DevJob *d_jobs, const DevJob *h, uint32_t n, uint32_t (*units)(const DevJob &)) {
    DevBatch b;
    b.jobs     = d_jobs;
    b.n        = n;
    uint32_t t = 0;
    for (uint32_t k = 0; k < SVTME_MAX_BATCH; k++) {
        b.start[k] = k < n ? t : 0xFFFFFFFFu;
        if (k < n)
            t += units(h[k]);
    }
    b.total = t;
    return b;
}

// One launch of every stage over a batch of n jobs sharing svtme_launch_key.
// d_jobs: the jobs in device memory; h_jobs: the same jobs on the host (unit
// counts). ev (optional, timing): ten events, start / stop of stage k in
// ev[2k], ev[2k+1] (k = A, D, B, C1|C, E), attached to the dispatch packets
// themselves (hipExtLaunchKernelGGL: no extra packets, no gaps); *mask gets
// bit k for every stage launched. With the real-time tune on the split path,
// stage A spans both stage-A rounds and the k_stage_d<true> between them.
#define SVTME_LAUNCH(K, grid, k, ...)                                                                               \
    do {                                                                                                           \
        if (ev) {                                                                                                  \
            hipExtLaunchKernelGGL(K, grid, dim3(256), 0, s, ev[2 * (k)], ev[2 * (k) + 1], 0, __VA_ARGS__);           \
            *mask |= 1u << (k);                                                                                    \
        } else                                                                                                     \
            hipLaunchKernelGGL(K, grid, dim3(256), 0, s, __VA_ARGS__);                                             \
    } while (0)

extern "C" hipError_t svtme_prime_stages(void) { // (see svtme_prime_pyramid): every kernel a job can launch
    const void *k[] = {
        (const void *)svtme::k_hme<true, true, true, false>,   (const void *)svtme::k_hme<true, true, true, true>,
        (const void *)svtme::k_hme<false, true, true, false>,  (const void *)svtme::k_hme<true, true, false, false>,
        (const void *)svtme::k_stage_a<false>,                 (const void *)svtme::k_stage_a<true>,
        (const void *)svtme::k_stage_d<false>,                 (const void *)svtme::k_stage_d<true>,
        (const void *)svtme::k_stage_b<false>,                 (const void *)svtme::k_stage_b<true>,
        (const void *)svtme::k_stage_c<false>,                 (const void *)svtme::k_stage_c<true>,
        (const void *)svtme::k_stage_c1<true, true, true>,     (const void *)svtme::k_stage_c1<true, true>,
        (const void *)svtme::k_stage_c1<true, false>,          (const void *)svtme::k_stage_c1<false, true, true>,
        (const void *)svtme::k_stage_c1<false, true>,          (const void *)svtme::k_stage_c1<false, false>,
        (const void *)svtme::k_l0_full<2>,                     (const void *)svtme::k_l0_full<4>,
        (const void *)svtme::k_l1_full,                        (const void *)svtme::k_fp_wide,
        (const void *)svtme::k_stage_e};
    hipFuncAttributes a;
    for (const void *f : k) {
        const hipError_t e = hipFuncGetAttributes(&a, f);
        if (e != hipSuccess)
            return e;
    }
    return hipSuccess;
}

extern "C" hipError_t svtme_launch_stages(const DevJob *d_jobs, const DevJob *h_jobs, uint32_t n, hipStream_t s,
                                          hipEvent_t *ev, uint32_t *mask) {
    if (n == 0 || n > SVTME_MAX_BATCH)
        return hipErrorInvalidValue;
    const DevJob &h0 = h_jobs[0];
    if (mask)
        *mask = 0;
    const DevBatch bd = make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count; });
    const bool full = h0.job.ctrl.me_search_method == SVTME_FULL_SAD_SEARCH;
    const bool k32  = svtme_fp_k32(&h0.job.ctrl);
    // the whole pass in one launch; SVTME_PATH_SPLIT_PASS keeps k_hme -> k_stage_c1 -> k_stage_e (diagnostics)
    const bool rt = svtme_hme_rt(&h0.job.ctrl); // the real-time tune's HME-L0 reduction
#define SVTME_HME(FP, SUB, K32)                                                                                     \
    do {                                                                                                           \
        if (rt)                                                                                                    \
            SVTME_LAUNCH((svtme::k_hme<FP, SUB, K32, true>), dim3(bd.total), 0, bd);                               \
        else                                                                                                       \
            SVTME_LAUNCH((svtme::k_hme<FP, SUB, K32, false>), dim3(bd.total), 0, bd);                              \
    } while (0)
    if (hme_fused(h0) && h0.parts == 1 && !(h0.paths & SVTME_PATH_SPLIT_PASS)) {
        if (full && k32)
            SVTME_HME(true, false, true);
        else if (full)
            SVTME_HME(true, false, false);
        else if (k32)
            SVTME_HME(true, true, true);
        else
            SVTME_HME(true, true, false);
        return hipGetLastError();
    }
    if (hme_fused(h0)) {
        SVTME_HME(false, true, true);
    } else {
    const DevBatch ba = make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count * j.ta_count; });
    bool short_l0 = true;
    for (uint32_t k = 0; k < n; k++)
        short_l0 = short_l0 && l0_full_short(&h_jobs[k]);
    if (ba.total && svtme_l0_full(&h0) && short_l0)
        SVTME_LAUNCH(svtme::k_l0_full<2>, dim3((ba.total + 3) / 4), 0, ba);
    else if (ba.total && svtme_l0_full(&h0))
        SVTME_LAUNCH(svtme::k_l0_full<4>, dim3((ba.total + 3) / 4), 0, ba);
    else if (ba.total)
        SVTME_LAUNCH(svtme::k_stage_a<false>, dim3((ba.total + 3) / 4), 0, ba);
    if (rt) { // the real-time tune: slot 0's HME-L0 centre, then the other slots' HME-L0
        const DevBatch ba1 =
            make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count * j.ta1_count; });
        // timed as part of stage 0: the last of these launches re-records stage 0's stop event
        hipEvent_t stop_d = ev && !ba1.total ? ev[1] : nullptr, stop_a = ev ? ev[1] : nullptr;
        hipExtLaunchKernelGGL(svtme::k_stage_d<true>, dim3((bd.total + 3) / 4), dim3(256), 0, s, nullptr, stop_d, 0, bd);
        if (ba1.total)
            hipExtLaunchKernelGGL(svtme::k_stage_a<true>, dim3((ba1.total + 3) / 4), dim3(256), 0, s, nullptr, stop_a, 0,
                                  ba1);
        if (ev)
            *mask |= 1u;
    }
    SVTME_LAUNCH(svtme::k_stage_d<false>, dim3((bd.total + 3) / 4), 1, bd);
    const DevBatch bb = make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count * j.tb_count; });
    if (bb.total && l1_full(h0)) { // two quadrants per wavefront
        const DevBatch b2 =
            make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count * (j.tb_count / 2); });
        SVTME_LAUNCH(svtme::k_l1_full, dim3((b2.total + 3) / 4), 2, b2);
    } else if (bb.total) {
        if (h0.job.ctrl.enable_hme_level2_flag)
            SVTME_LAUNCH(svtme::k_stage_b<true>, dim3((bb.total + 3) / 4), 2, bb);
        else
            SVTME_LAUNCH(svtme::k_stage_b<false>, dim3((bb.total + 3) / 4), 2, bb);
    }
    }
    const DevBatch be = make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count; });
    if (h0.parts) { // wide full-pel stage + per-SB decode
        const DevBatch bc = make_batch(d_jobs, h_jobs, n, [](const DevJob &j) { return j.job.sb_count * j.R * j.parts; });
        const dim3 grid((bc.total + 3) / 4);
        const bool wide = svtme_fp_wide(&h0.job.ctrl);
        if (fp_wide_lds(h0))
            SVTME_LAUNCH(svtme::k_fp_wide, grid, 3, bc);
        else if (full && k32 && wide)
            SVTME_LAUNCH((svtme::k_stage_c1<false, true, true>), grid, 3, bc);
        else if (full && k32)
            SVTME_LAUNCH((svtme::k_stage_c1<false, true>), grid, 3, bc);
        else if (full)
            SVTME_LAUNCH((svtme::k_stage_c1<false, false>), grid, 3, bc);
        else if (k32 && wide)
            SVTME_LAUNCH((svtme::k_stage_c1<true, true, true>), grid, 3, bc);
        else if (k32)
            SVTME_LAUNCH((svtme::k_stage_c1<true, true>), grid, 3, bc);
        else
            SVTME_LAUNCH((svtme::k_stage_c1<true, false>), grid, 3, bc);
        bool direct = true; // every record made by k_stage_c1 (direct_records)
        for (uint32_t k = 0; k < n; k++)
            direct = direct && h_jobs[k].job.me_type == SVTME_ME_MCTF && h_jobs[k].parts == 1 && !h_jobs[k].out_sb &&
                     !fp_wide_lds(h_jobs[k]);
        if (!direct)
            SVTME_LAUNCH(svtme::k_stage_e, dim3(be.total), 4, be);
    } else if (full)
        SVTME_LAUNCH(svtme::k_stage_c<false>, dim3(be.total), 3, be);
    else
        SVTME_LAUNCH(svtme::k_stage_c<true>, dim3(be.total), 3, be);
    return hipGetLastError();
}
