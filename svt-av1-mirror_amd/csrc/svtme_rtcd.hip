// svtme_rtcd.hip — per-kernel rtcd variants (`*_hip`) with the exact
// signatures of the reference's dispatch pointers (Source/Lib/Codec/aom_dsp_rtcd.h,
// lines cited per function). Host memory in and out, synchronous.
//
// They exist so an encoder can register a HIP variant set exactly where the
// AVX2 one is registered (aom_dsp_rtcd.c:501-515) and so each kernel's
// semantics can be checked in isolation. One call is microseconds of CPU work,
// far below a launch: the performance boundary is the picture job API.
//
// Each call: copy the bytes the kernel reads into the calling thread's device
// scratch, run one kernel on the calling thread's stream, copy the outputs
// back. Reentrant: the reference calls these from up to 25 ME threads at once
// (enc_handle.c:731-773), so every thread owns its stream and scratch and no
// lock is taken. On any HIP error the call reports through svtme_last_error()
// and stderr, leaves outputs untouched and raises the thread's failure flag
// (svtme_rtcd_failed()); the library has no CPU path of its own -- the
// encoder glue (integration/svtme_svt_glue.c) re-runs the call on the C
// variant it replaced, so the encoder never consumes stale outputs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "svtme_device.h"

extern "C" void svtme_set_error_internal(const char *msg);

namespace {

struct Scratch {
    hipStream_t stream = nullptr;
    uint8_t *d         = nullptr;
    size_t cap         = 0;
    bool init          = false;
    bool failed        = false;
    ~Scratch() {
        if (d)
            (void)hipFree(d);
        if (stream)
            (void)hipStreamDestroy(stream);
    }
};
thread_local Scratch g_rt;

bool report(hipError_t e, const char *what) {
    if (e == hipSuccess)
        return true;
    g_rt.failed = true;
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    svtme_set_error_internal(buf);
    return false;
}

// device scratch of at least `need` bytes (+64 slack for dword over-reads)
uint8_t *scratch(size_t need) {
    if (!g_rt.init) {
        if (!report(hipStreamCreateWithFlags(&g_rt.stream, hipStreamNonBlocking), "rtcd stream"))
            return nullptr;
        g_rt.init = true;
    }
    need += 64;
    if (g_rt.cap < need) {
        if (g_rt.d)
            (void)hipFree(g_rt.d);
        g_rt.d   = nullptr;
        g_rt.cap = 0;
        if (!report(hipMalloc((void **)&g_rt.d, need), "rtcd scratch"))
            return nullptr;
        g_rt.cap = need;
    }
    return g_rt.d;
}

__device__ __forceinline__ uint32_t absd(uint32_t a, uint32_t b) { return a > b ? a - b : b - a; }

// --------------------------------------------------------------------------
// svt_sad_loop_kernel (compute_sad_c.c:58-101): one thread per position,
// block-level argmin by (sad, y, x) key.
// --------------------------------------------------------------------------
__global__ void k_sad_loop(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                           uint32_t bh, uint32_t bw, uint32_t stride_raw, int skip, int sa_w, int sa_h,
                           unsigned long long *best) {
    __shared__ unsigned long long sbest;
    if (threadIdx.x == 0)
        sbest = ~0ull;
    __syncthreads();
    unsigned long long k = ~0ull;
    for (int p = threadIdx.x; p < sa_w * sa_h; p += blockDim.x) {
        const int y = p / sa_w, x = p - y * sa_w;
        if (skip && (y & 1) == 0)
            continue;
        const uint8_t *r = ref + (size_t)y * stride_raw + x;
        uint32_t sad     = 0;
        for (uint32_t i = 0; i < bh; i++)
            for (uint32_t j = 0; j < bw; j++) sad += absd(src[i * src_stride + j], r[(size_t)i * ref_stride + j]);
        const unsigned long long kk = ((unsigned long long)sad << 32) | ((uint32_t)y << 16) | (uint32_t)x;
        k                           = kk < k ? kk : k;
    }
    atomicMin(&sbest, k);
    __syncthreads();
    if (threadIdx.x == 0)
        *best = sbest;
}

// n x m SAD, 8 or 16 bit
template <typename T>
__global__ void k_nxm(const T *src, uint32_t src_stride, const T *ref, uint32_t ref_stride, uint32_t h, uint32_t w,
                      uint32_t *out) {
    __shared__ uint32_t s;
    if (threadIdx.x == 0)
        s = 0;
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t e = threadIdx.x; e < h * w; e += blockDim.x) {
        const uint32_t i = e / w, j = e - i * w;
        acc += absd(src[(size_t)i * src_stride + j], ref[(size_t)i * ref_stride + j]);
    }
    atomicAdd(&s, acc);
    __syncthreads();
    if (threadIdx.x == 0)
        *out = s;
}

// 8x8 SAD (or 8x4 sub <<1) of block (bx, by) of a 16/64-wide source at ref offset
__device__ uint32_t sad8(const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs, bool sub) {
    uint32_t s = 0;
    if (sub) {
        for (int i = 0; i < 8; i += 2)
            for (int j = 0; j < 8; j++) s += absd(src[i * ss + j], ref[(size_t)i * rs + j]);
        return s << 1;
    }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) s += absd(src[i * ss + j], ref[(size_t)i * rs + j]);
    return s;
}

// sum over the 2^k lanes of an aligned group (butterfly: every lane of the group holds it)
template <int K>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
#pragma unroll
    for (int m = 1; m < (1 << K); m <<= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// svt_ext_sad_calculation_8x8_16x16 (motion_estimation.c:98-164): io[0..3] best 8x8 sad,
// io[4] best 16x16 sad, io[5..8] mv8x8, io[9] mv16x16, io[10] sad16x16, io[11..14] sad8x8.
// One wave: lane = block b (lane >> 4, raster in the 16x16) x row (lane >> 1 & 7) x
// 4-pixel half (lane & 1); the 16 lanes of a block sum its SAD.
__global__ void k_ext_8x8_16x16(const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs, uint32_t mv,
                                int sub, uint32_t *io) {
    const int lane = threadIdx.x, b = lane >> 4, r = (lane >> 1) & 7, h = lane & 1;
    const int y = (b >> 1) * 8 + r, x = (b & 1) * 8 + h * 4;
    uint32_t a = 0;
    if (!sub || (r & 1) == 0)
        for (int j = 0; j < 4; j++) a += absd(src[y * ss + x + j], ref[(size_t)y * rs + x + j]);
    const uint32_t s8  = group_sum<4>(a) << (sub ? 1 : 0);
    const uint32_t s16 = s8 + __shfl_xor(s8, 16, 64) + __shfl_xor(s8, 32, 64) + __shfl_xor(s8, 48, 64);
    if ((lane & 15) == 0) {
        io[11 + b] = s8;
        if (s8 < io[b]) {
            io[b]     = s8;
            io[5 + b] = mv;
        }
    }
    if (lane == 0) {
        if (s16 < io[4]) {
            io[4] = s16;
            io[9] = mv;
        }
        io[10] = s16;
    }
}

// svt_ext_sad_calculation_32x32_64x64 (motion_estimation.c:171-205):
// io[0..15] sad16x16, [16..19] best32, [20] best64, [21..24] mv32, [25] mv64, [26..29] sad32.
// Lane q < 4: quadrant q's sum of its four 16x16 SADs; the 64x64 sum over the 4 lanes.
__global__ void k_ext_32x32_64x64(uint32_t mv, uint32_t *io) {
    const int q = threadIdx.x & 3;
    const uint32_t s   = io[4 * q] + io[4 * q + 1] + io[4 * q + 2] + io[4 * q + 3];
    const uint32_t s64 = group_sum<2>(s);
    if (threadIdx.x < 4) {
        io[26 + q] = s;
        if (s < io[16 + q]) {
            io[16 + q] = s;
            io[21 + q] = mv;
        }
    }
    if (threadIdx.x == 0 && s64 < io[20]) {
        io[20] = s64;
        io[25] = mv;
    }
}

// svt_ext_all_sad_calculation_8x8_16x16 (motion_estimation.c:210-362): 8 positions,
// io: [0..63] best8x8, [64..79] best16x16, [80..143] mv8x8, [144..159] mv16x16,
// [160..287] eight_sad16x16[16][8]. One wave; lane = 8x8 block in the 16x16 Z-order.
__global__ void k_ext_all_8x8_16x16(const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs, uint32_t mv,
                                    int sub, uint32_t *io) {
    const int lane = threadIdx.x; // 0..63 = 16x16 block (lane >> 2, Z-order) x 8x8 child
    const int z16 = lane >> 2, k4 = lane & 3;
    // Z-order 16x16 index -> raster (y, x) in 16-pixel units (offsets table, motion_estimation.c:341)
    const int y16 = ((z16 >> 3) << 1) | ((z16 >> 1) & 1), x16 = (((z16 >> 2) & 1) << 1) | (z16 & 1);
    const int py = y16 * 16 + (k4 >> 1) * 8, px = x16 * 16 + (k4 & 1) * 8;
    for (int si = 0; si < 8; si++) {
        uint32_t s8  = sad8(src + py * ss + px, ss, ref + (size_t)py * rs + px + si, rs, sub != 0);
        uint32_t s16 = s8 + __shfl_xor(s8, 1, 64);
        s16 += __shfl_xor(s16, 2, 64);
        const int16_t xm   = (int16_t)((int16_t)(mv & 0xFFFF) + si);
        const int16_t ym   = (int16_t)(mv >> 16);
        const uint32_t nmv = ((uint32_t)(uint16_t)ym << 16) | (uint16_t)xm;
        if (s8 < io[lane]) {
            io[lane]      = s8;
            io[80 + lane] = nmv;
        }
        if (k4 == 0) {
            io[160 + z16 * 8 + si] = s16;
            if (s16 < io[64 + z16]) {
                io[64 + z16]  = s16;
                io[144 + z16] = nmv;
            }
        }
    }
}

// svt_ext_eight_sad_calculation_32x32_64x64 (motion_estimation.c:369-425):
// io [0..127] sad16x16[16][8], [128..131] best32, [132] best64, [133..136] mv32, [137] mv64, [138..169] sad32[4][8].
// Lane = quadrant q (lane >> 3) x position si (lane & 7), 32 lanes. The reference
// updates each best in position order with a strict <, so its result is the
// lowest position of the minimum, taken only if below the incoming best: a
// (sad << 3 | si) minimum over the 8 lanes of a quadrant.
__global__ void k_ext_eight_32x32_64x64(uint32_t mv, uint32_t *io) {
    const int lane = threadIdx.x & 31, q = lane >> 3, si = lane & 7;
    const uint32_t s = io[(4 * q) * 8 + si] + io[(4 * q + 1) * 8 + si] + io[(4 * q + 2) * 8 + si] +
        io[(4 * q + 3) * 8 + si];
    const uint32_t s64 = s + __shfl_xor(s, 8, 64) + __shfl_xor(s, 16, 64) + __shfl_xor(s, 24, 64);
    auto min8 = [](unsigned long long k) { // over the 8 lanes of a group
        for (int m = 1; m < 8; m <<= 1) {
            const unsigned long long o = __shfl_xor(k, m, 64);
            k = o < k ? o : k;
        }
        return k;
    };
    const unsigned long long k32 = min8(((unsigned long long)s << 3) | (uint32_t)si);
    const unsigned long long k64 = min8(((unsigned long long)s64 << 3) | (uint32_t)si);
    auto mv_at = [&](uint32_t p) {
        const int16_t xm = (int16_t)((int16_t)(mv & 0xFFFF) + (int)p), ym = (int16_t)(mv >> 16);
        return ((uint32_t)(uint16_t)ym << 16) | (uint16_t)xm;
    };
    if (threadIdx.x < 32) {
        io[138 + q * 8 + si] = s;
        if (si == 0 && (uint32_t)(k32 >> 3) < io[128 + q]) {
            io[128 + q] = (uint32_t)(k32 >> 3);
            io[133 + q] = mv_at((uint32_t)k32 & 7);
        }
    }
    if (threadIdx.x == 0 && (uint32_t)(k64 >> 3) < io[132]) {
        io[132] = (uint32_t)(k64 >> 3);
        io[137] = mv_at((uint32_t)k64 & 7);
    }
}

__global__ void k_fill32(uint32_t *p, uint32_t n, uint32_t v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        p[i] = v;
}

// downsample_2d (pic_analysis_process.c:130-158), any decim_step
__global__ void k_downsample(const uint8_t *in, uint32_t in_stride, uint32_t w, uint32_t h, uint8_t *out,
                             uint32_t out_stride, uint32_t step, uint32_t ow, uint32_t oh) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ow * oh)
        return;
    const uint32_t oy = i / ow, ox = i - oy * ow;
    const uint32_t half = step >> 1;
    const uint32_t vy = half + oy * step, hx = half + ox * step;
    const uint8_t *cur = in + (size_t)vy * in_stride, *prev = cur - in_stride;
    const uint32_t s   = (uint32_t)prev[hx - 1] + prev[hx] + cur[hx - 1] + cur[hx];
    out[(size_t)oy * out_stride + ox] = (uint8_t)((s + 2) >> 2);
}

// --------------------------------------------------------------------------
// svt_pme_sad_loop_kernel (product_coding_loop.c:1811-1860): one thread per
// visited position (the host lists them in the reference's visit order with
// their MV rate); block-level argmin by (sad + rate, visit index).
// --------------------------------------------------------------------------
__global__ void k_pme(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride, uint32_t bh,
                      uint32_t bw, const int16_t *px, const int16_t *py, const uint32_t *rate, int n,
                      unsigned long long *best) {
    __shared__ unsigned long long sbest;
    if (threadIdx.x == 0)
        sbest = ~0ull;
    __syncthreads();
    unsigned long long k = ~0ull;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint8_t *r = ref + (size_t)py[i] * ref_stride + px[i];
        uint32_t sad     = 0;
        for (uint32_t y = 0; y < bh; y++)
            for (uint32_t x = 0; x < bw; x++) sad += absd(src[y * src_stride + x], r[(size_t)y * ref_stride + x]);
        const unsigned long long kk = ((unsigned long long)(sad + rate[i]) << 32) | (uint32_t)i;
        k                           = kk < k ? kk : k;
    }
    atomicMin(&sbest, k);
    __syncthreads();
    if (threadIdx.x == 0)
        *best = sbest;
}

} // namespace

// --------------------------------------------------------------------------
// host wrappers
// --------------------------------------------------------------------------
// 1 if an rtcd call of this thread failed since the last query (then cleared)
extern "C" int svtme_rtcd_failed(void) {
    const int f = g_rt.failed ? 1 : 0;
    g_rt.failed = false;
    return f;
}

#define RT_CHECK(expr, what)                                                                                        \
    do {                                                                                                            \
        if (!report((expr), what))                                                                                  \
            return;                                                                                                 \
    } while (0)
#define RT_CHECK_V(expr, what, val)                                                                                 \
    do {                                                                                                            \
        if (!report((expr), what))                                                                                  \
            return val;                                                                                             \
    } while (0)

static size_t span(size_t rows, size_t stride, size_t width) { return rows ? (rows - 1) * stride + width : 0; }

extern "C" void svt_sad_loop_kernel_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                        uint32_t block_height, uint32_t block_width, uint64_t *best_sad,
                                        int16_t *x_search_center, int16_t *y_search_center, uint32_t src_stride_raw,
                                        uint8_t skip_search_line, int16_t search_area_width,
                                        int16_t search_area_height) {
    *best_sad = 0xffffff;
    if (search_area_width <= 0 || search_area_height <= 0 || block_height == 0 || block_width == 0)
        return;
    const size_t sspan = span(block_height, src_stride, block_width);
    const size_t rspan = span(search_area_height, src_stride_raw, 0) + span(block_height, ref_stride, 0) +
        search_area_width + block_width;
    uint8_t *d = scratch(sspan + rspan + 8 + 64);
    if (!d)
        return;
    uint8_t *ds = d, *dr = d + ((sspan + 15) & ~(size_t)15);
    unsigned long long *db = (unsigned long long *)(dr + ((rspan + 15) & ~(size_t)15));
    const int skip = block_width == 16 && block_height <= 16 && skip_search_line;
    RT_CHECK(hipMemcpyAsync(ds, src, sspan, hipMemcpyHostToDevice, g_rt.stream), "sad_loop H2D");
    RT_CHECK(hipMemcpyAsync(dr, ref, rspan - 1, hipMemcpyHostToDevice, g_rt.stream), "sad_loop H2D");
    hipLaunchKernelGGL(k_sad_loop, dim3(1), dim3(256), 0, g_rt.stream, ds, src_stride, dr, ref_stride, block_height,
                       block_width, src_stride_raw, skip, (int)search_area_width, (int)search_area_height, db);
    RT_CHECK(hipGetLastError(), "k_sad_loop");
    unsigned long long k = ~0ull;
    RT_CHECK(hipMemcpyAsync(&k, db, 8, hipMemcpyDeviceToHost, g_rt.stream), "sad_loop D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "sad_loop sync");
    const uint32_t sad = (uint32_t)(k >> 32);
    if (k != ~0ull && sad < 0xffffffu) {
        *best_sad        = sad;
        *x_search_center = (int16_t)(k & 0xFFFF);
        *y_search_center = (int16_t)((k >> 16) & 0xFFFF);
    }
}

template <typename T>
static uint32_t nxm_hip(const T *src, uint32_t src_stride, const T *ref, uint32_t ref_stride, uint32_t h, uint32_t w) {
    if (h == 0 || w == 0)
        return 0;
    const size_t ss = span(h, src_stride, w) * sizeof(T), rs = span(h, ref_stride, w) * sizeof(T);
    uint8_t *d = scratch(ss + rs + 64);
    if (!d)
        return 0;
    T *ds = (T *)d, *dr = (T *)(d + ((ss + 15) & ~(size_t)15));
    uint32_t *dout = (uint32_t *)((uint8_t *)dr + ((rs + 15) & ~(size_t)15));
    RT_CHECK_V(hipMemcpyAsync(ds, src, ss, hipMemcpyHostToDevice, g_rt.stream), "nxm H2D", 0);
    RT_CHECK_V(hipMemcpyAsync(dr, ref, rs, hipMemcpyHostToDevice, g_rt.stream), "nxm H2D", 0);
    hipLaunchKernelGGL(k_nxm<T>, dim3(1), dim3(256), 0, g_rt.stream, ds, src_stride, dr, ref_stride, h, w, dout);
    RT_CHECK_V(hipGetLastError(), "k_nxm", 0);
    uint32_t out = 0;
    RT_CHECK_V(hipMemcpyAsync(&out, dout, 4, hipMemcpyDeviceToHost, g_rt.stream), "nxm D2H", 0);
    RT_CHECK_V(hipStreamSynchronize(g_rt.stream), "nxm sync", 0);
    return out;
}

extern "C" uint32_t svt_nxm_sad_kernel_hip(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                           uint32_t ref_stride, uint32_t height, uint32_t width) {
    return nxm_hip<uint8_t>(src, src_stride, ref, ref_stride, height, width);
}

extern "C" uint32_t svt_aom_sad_16b_kernel_hip(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                                               uint32_t height, uint32_t width) {
    return nxm_hip<uint16_t>(src, src_stride, ref, ref_stride, height, width);
}

extern "C" void svt_ext_sad_calculation_8x8_16x16_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref,
                                                      uint32_t ref_stride, uint32_t *p_best_sad_8x8,
                                                      uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                                      uint32_t *p_best_mv16x16, uint32_t mv, uint32_t *p_sad16x16,
                                                      uint32_t *p_sad8x8, bool sub_sad) {
    const size_t ss = span(16, src_stride, 16), rs = span(16, ref_stride, 16);
    uint8_t *d = scratch(ss + rs + 64 + 16 * 4);
    if (!d)
        return;
    uint8_t *ds = d, *dr = d + ((ss + 15) & ~(size_t)15);
    uint32_t *io = (uint32_t *)(dr + ((rs + 15) & ~(size_t)15));
    uint32_t h[15];
    for (int i = 0; i < 4; i++) h[i] = p_best_sad_8x8[i], h[5 + i] = p_best_mv8x8[i];
    h[4] = p_best_sad_16x16[0];
    h[9] = p_best_mv16x16[0];
    RT_CHECK(hipMemcpyAsync(ds, src, ss, hipMemcpyHostToDevice, g_rt.stream), "ext8 H2D");
    RT_CHECK(hipMemcpyAsync(dr, ref, rs, hipMemcpyHostToDevice, g_rt.stream), "ext8 H2D");
    RT_CHECK(hipMemcpyAsync(io, h, sizeof(h), hipMemcpyHostToDevice, g_rt.stream), "ext8 H2D");
    hipLaunchKernelGGL(k_ext_8x8_16x16, dim3(1), dim3(64), 0, g_rt.stream, ds, src_stride, dr, ref_stride, mv,
                       sub_sad ? 1 : 0, io);
    RT_CHECK(hipGetLastError(), "k_ext_8x8_16x16");
    RT_CHECK(hipMemcpyAsync(h, io, sizeof(h), hipMemcpyDeviceToHost, g_rt.stream), "ext8 D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "ext8 sync");
    for (int i = 0; i < 4; i++) p_best_sad_8x8[i] = h[i], p_best_mv8x8[i] = h[5 + i], p_sad8x8[i] = h[11 + i];
    p_best_sad_16x16[0] = h[4];
    p_best_mv16x16[0]   = h[9];
    *p_sad16x16         = h[10];
}

extern "C" void svt_ext_sad_calculation_32x32_64x64_hip(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                                        uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                        uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32) {
    uint32_t *io = (uint32_t *)scratch(30 * 4);
    if (!io)
        return;
    uint32_t h[30];
    for (int i = 0; i < 16; i++) h[i] = p_sad16x16[i];
    for (int i = 0; i < 4; i++) h[16 + i] = p_best_sad_32x32[i], h[21 + i] = p_best_mv32x32[i];
    h[20] = p_best_sad_64x64[0];
    h[25] = p_best_mv64x64[0];
    RT_CHECK(hipMemcpyAsync(io, h, sizeof(h), hipMemcpyHostToDevice, g_rt.stream), "ext32 H2D");
    hipLaunchKernelGGL(k_ext_32x32_64x64, dim3(1), dim3(64), 0, g_rt.stream, mv, io);
    RT_CHECK(hipGetLastError(), "k_ext_32x32_64x64");
    RT_CHECK(hipMemcpyAsync(h, io, sizeof(h), hipMemcpyDeviceToHost, g_rt.stream), "ext32 D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "ext32 sync");
    for (int i = 0; i < 4; i++) p_best_sad_32x32[i] = h[16 + i], p_best_mv32x32[i] = h[21 + i], p_sad32x32[i] = h[26 + i];
    p_best_sad_64x64[0] = h[20];
    p_best_mv64x64[0]   = h[25];
}

extern "C" void svt_ext_all_sad_calculation_8x8_16x16_hip(uint8_t *src, uint32_t src_stride, uint8_t *ref,
                                                          uint32_t ref_stride, uint32_t mv, uint32_t *p_best_sad_8x8,
                                                          uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                                          uint32_t *p_best_mv16x16, uint32_t p_eight_sad16x16[16][8],
                                                          uint32_t p_eight_sad8x8[64][8], bool sub_sad) {
    (void)p_eight_sad8x8; // not written by the C reference either (motion_estimation.c:218)
    const size_t ss = span(64, src_stride, 64), rs = span(64, ref_stride, 64 + 7);
    uint8_t *d = scratch(ss + rs + 64 + 288 * 4);
    if (!d)
        return;
    uint8_t *ds = d, *dr = d + ((ss + 15) & ~(size_t)15);
    uint32_t *io = (uint32_t *)(dr + ((rs + 15) & ~(size_t)15));
    static thread_local uint32_t h[288];
    memcpy(h, p_best_sad_8x8, 64 * 4);
    memcpy(h + 64, p_best_sad_16x16, 16 * 4);
    memcpy(h + 80, p_best_mv8x8, 64 * 4);
    memcpy(h + 144, p_best_mv16x16, 16 * 4);
    memcpy(h + 160, p_eight_sad16x16, 128 * 4);
    RT_CHECK(hipMemcpyAsync(ds, src, ss, hipMemcpyHostToDevice, g_rt.stream), "extall H2D");
    RT_CHECK(hipMemcpyAsync(dr, ref, rs, hipMemcpyHostToDevice, g_rt.stream), "extall H2D");
    RT_CHECK(hipMemcpyAsync(io, h, sizeof(h), hipMemcpyHostToDevice, g_rt.stream), "extall H2D");
    hipLaunchKernelGGL(k_ext_all_8x8_16x16, dim3(1), dim3(64), 0, g_rt.stream, ds, src_stride, dr, ref_stride, mv,
                       sub_sad ? 1 : 0, io);
    RT_CHECK(hipGetLastError(), "k_ext_all_8x8_16x16");
    RT_CHECK(hipMemcpyAsync(h, io, sizeof(h), hipMemcpyDeviceToHost, g_rt.stream), "extall D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "extall sync");
    memcpy(p_best_sad_8x8, h, 64 * 4);
    memcpy(p_best_sad_16x16, h + 64, 16 * 4);
    memcpy(p_best_mv8x8, h + 80, 64 * 4);
    memcpy(p_best_mv16x16, h + 144, 16 * 4);
    memcpy(p_eight_sad16x16, h + 160, 128 * 4);
}

extern "C" void svt_ext_eight_sad_calculation_32x32_64x64_hip(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                              uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                              uint32_t *p_best_mv64x64, uint32_t mv,
                                                              uint32_t p_sad32x32[4][8]) {
    uint32_t *io = (uint32_t *)scratch(170 * 4);
    if (!io)
        return;
    uint32_t h[170];
    memcpy(h, p_sad16x16, 128 * 4);
    for (int i = 0; i < 4; i++) h[128 + i] = p_best_sad_32x32[i], h[133 + i] = p_best_mv32x32[i];
    h[132] = p_best_sad_64x64[0];
    h[137] = p_best_mv64x64[0];
    RT_CHECK(hipMemcpyAsync(io, h, sizeof(h), hipMemcpyHostToDevice, g_rt.stream), "ext8x32 H2D");
    hipLaunchKernelGGL(k_ext_eight_32x32_64x64, dim3(1), dim3(64), 0, g_rt.stream, mv, io);
    RT_CHECK(hipGetLastError(), "k_ext_eight_32x32_64x64");
    RT_CHECK(hipMemcpyAsync(h, io, sizeof(h), hipMemcpyDeviceToHost, g_rt.stream), "ext8x32 D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "ext8x32 sync");
    for (int i = 0; i < 4; i++) p_best_sad_32x32[i] = h[128 + i], p_best_mv32x32[i] = h[133 + i];
    p_best_sad_64x64[0] = h[132];
    p_best_mv64x64[0]   = h[137];
    memcpy(p_sad32x32, h + 138, 32 * 4);
}

extern "C" void svt_initialize_buffer_32bits_hip(uint32_t *pointer, uint32_t count128, uint32_t count32,
                                                 uint32_t value) {
    const uint32_t n = count128 * 4 + count32;
    if (!n)
        return;
    uint32_t *d = (uint32_t *)scratch((size_t)n * 4);
    if (!d)
        return;
    hipLaunchKernelGGL(k_fill32, dim3((n + 255) / 256), dim3(256), 0, g_rt.stream, d, n, value);
    RT_CHECK(hipGetLastError(), "k_fill32");
    RT_CHECK(hipMemcpyAsync(pointer, d, (size_t)n * 4, hipMemcpyDeviceToHost, g_rt.stream), "init D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "init sync");
}

extern "C" void svt_aom_downsample_2d_hip(uint8_t *input_samples, uint32_t input_stride, uint32_t input_area_width,
                                          uint32_t input_area_height, uint8_t *decim_samples, uint32_t decim_stride,
                                          uint32_t decim_step) {
    const uint32_t half = decim_step >> 1;
    if (decim_step < 2 || input_area_width <= half || input_area_height <= half)
        return;
    const uint32_t ow = (input_area_width - half + decim_step - 1) / decim_step;
    const uint32_t oh = (input_area_height - half + decim_step - 1) / decim_step;
    // rows half-1 .. last sampled row, all columns of the area
    const uint32_t last_row = half + (oh - 1) * decim_step;
    const size_t in_bytes   = span(last_row - (half - 1) + 1, input_stride, input_area_width);
    const size_t out_bytes  = span(oh, decim_stride, ow);
    uint8_t *d = scratch(in_bytes + out_bytes + 32);
    if (!d)
        return;
    uint8_t *din = d, *dout = d + ((in_bytes + 15) & ~(size_t)15);
    const uint8_t *hin = input_samples + (size_t)(half - 1) * input_stride;
    RT_CHECK(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, g_rt.stream), "ds H2D");
    RT_CHECK(hipMemcpyAsync(dout, decim_samples, out_bytes, hipMemcpyHostToDevice, g_rt.stream), "ds H2D");
    const uint32_t n = ow * oh;
    // the kernel addresses rows relative to the original input pointer
    hipLaunchKernelGGL(k_downsample, dim3((n + 255) / 256), dim3(256), 0, g_rt.stream,
                       din - (ptrdiff_t)(half - 1) * input_stride, input_stride, input_area_width, input_area_height,
                       dout, decim_stride, decim_step, ow, oh);
    RT_CHECK(hipGetLastError(), "k_downsample");
    RT_CHECK(hipMemcpyAsync(decim_samples, dout, out_bytes, hipMemcpyDeviceToHost, g_rt.stream), "ds D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "ds sync");
}

// MV rate of a full-pel candidate (svt_mv_err_cost, mcomp.c:44-68; svt_mv_cost,
// mcomp.h:134; svt_av1_get_mv_joint, rd_cost.c:55), read through the
// MV_COST_PARAMS layout of include/svtme.h
static uint32_t pme_rate(const uint8_t *p, int16_t row, int16_t col) {
    const int16_t *ref_mv = *(const int16_t *const *)(p + SVTME_MVCOST_OFF_REF_MV);
    // diff and abs_diff are int16 MVs in the reference (mcomp.c:46-47)
    const int dr = (int16_t)(row - ref_mv[0]), dc = (int16_t)(col - ref_mv[1]);
    const int ar = (int16_t)(dr < 0 ? -dr : dr), ac = (int16_t)(dc < 0 ? -dc : dc);
    const int epb = *(const int *)(p + SVTME_MVCOST_OFF_ERROR_PER_BIT);
    const int shift = 7 + 9 - 6 + 4; // RDDIV_BITS + AV1_PROB_COST_SHIFT - RD_EPB_SHIFT + PIXEL_TRANSFORM_ERROR_SCALE
    switch (p[SVTME_MVCOST_OFF_TYPE]) {
    case 0: { // MV_COST_ENTROPY (`if (mvcost)` tests the array parameter: always taken)
        const int *jc = *(const int *const *)(p + SVTME_MVCOST_OFF_MVJCOST);
        const int *const *cc = (const int *const *)(p + SVTME_MVCOST_OFF_MVCOST); // the reference's
        const int joint = dr == 0 ? (dc == 0 ? 0 : 1) : (dc == 0 ? 2 : 3);
        const int cr = dr < -(1 << 14) ? -(1 << 14) : dr > (1 << 14) ? (1 << 14) : dr;
        const int ccl = dc < -(1 << 14) ? -(1 << 14) : dc > (1 << 14) ? (1 << 14) : dc;
        const int64_t c = (int64_t)(jc[joint] + cc[0][cr] + cc[1][ccl]) * epb;
        return (uint32_t)(int)((c + (((int64_t)1 << shift) >> 1)) >> shift);
    }
    case 1: return (uint32_t)((2 * (ar + ac)) >> 3); // MV_COST_L1_LOWRES
    case 2: return 0;                                // MV_COST_L1_MIDRES (lambda 0)
    case 3: return (uint32_t)((ar + ac) >> 3);       // MV_COST_L1_HDRES
    case 4: {                                        // MV_COST_OPT
        const int64_t c = (int64_t)((ar + ac) << 8) * epb;
        return (uint32_t)(int)((c + (((int64_t)1 << shift) >> 1)) >> shift);
    }
    default: return 0; // MV_COST_NONE
    }
}

extern "C" void svt_pme_sad_loop_kernel_hip(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src,
                                            uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                            uint32_t block_height, uint32_t block_width, uint32_t *best_cost,
                                            int16_t *best_mvx, int16_t *best_mvy, int16_t search_position_start_x,
                                            int16_t search_position_start_y, int16_t search_area_width,
                                            int16_t search_area_height, int16_t search_step, int16_t mvx,
                                            int16_t mvy) {
    if (search_area_width <= 0 || search_area_height <= 0 || search_step <= 0)
        return;
    // the reference's visit order (product_coding_loop.c:1823-1836): col_num and
    // the x step persist across rows; a column whose remaining width is below 8
    // is skipped while col_num == 0 (the step of the previous column applies)
    std::vector<int16_t> px, py;
    std::vector<uint32_t> rate;
    const uint8_t *cp = (const uint8_t *)mv_cost_params;
    int16_t col_num = 0, step_x = 1;
    int maxx = 0, maxy = 0;
    for (int16_t y = 0; y < search_area_height; y = (int16_t)(y + search_step)) {
        for (int16_t x = 0; x < search_area_width; x = (int16_t)(x + step_x)) {
            if ((search_area_width - x) < 8 && col_num == 0)
                continue;
            if (col_num == 7) {
                col_num = 0;
                step_x  = search_step;
            } else {
                col_num++;
                step_x = 1;
            }
            const uint32_t rx = (uint32_t)(search_position_start_x + x), ry = (uint32_t)(search_position_start_y + y);
            const int16_t mvc = (int16_t)(mvx + (rx * 8)), mvr = (int16_t)(mvy + (ry * 8));
            px.push_back(x);
            py.push_back(y);
            rate.push_back(pme_rate(cp, mvr, mvc));
            maxx = x > maxx ? x : maxx;
            maxy = y > maxy ? y : maxy;
        }
    }
    const int n = (int)px.size();
    if (n == 0 || block_height == 0 || block_width == 0)
        return;
    const size_t sspan = span(block_height, src_stride, block_width);
    const size_t rspan = (size_t)(maxy + block_height - 1) * ref_stride + maxx + block_width;
    const size_t pos   = (size_t)n * (2 + 2 + 4);
    uint8_t *d = scratch(sspan + rspan + pos + 64);
    if (!d)
        return;
    uint8_t *ds = d, *dr = d + ((sspan + 15) & ~(size_t)15);
    uint8_t *dp = dr + ((rspan + 15) & ~(size_t)15);
    int16_t *dx = (int16_t *)dp, *dy = dx + n;
    uint32_t *drate = (uint32_t *)(dp + (((size_t)n * 4 + 15) & ~(size_t)15));
    unsigned long long *db = (unsigned long long *)((uint8_t *)drate + (((size_t)n * 4 + 15) & ~(size_t)15));
    RT_CHECK(hipMemcpyAsync(ds, src, sspan, hipMemcpyHostToDevice, g_rt.stream), "pme H2D");
    RT_CHECK(hipMemcpyAsync(dr, ref, rspan, hipMemcpyHostToDevice, g_rt.stream), "pme H2D");
    RT_CHECK(hipMemcpyAsync(dx, px.data(), (size_t)n * 2, hipMemcpyHostToDevice, g_rt.stream), "pme H2D");
    RT_CHECK(hipMemcpyAsync(dy, py.data(), (size_t)n * 2, hipMemcpyHostToDevice, g_rt.stream), "pme H2D");
    RT_CHECK(hipMemcpyAsync(drate, rate.data(), (size_t)n * 4, hipMemcpyHostToDevice, g_rt.stream), "pme H2D");
    hipLaunchKernelGGL(k_pme, dim3(1), dim3(256), 0, g_rt.stream, ds, src_stride, dr, ref_stride, block_height,
                       block_width, dx, dy, drate, n, db);
    RT_CHECK(hipGetLastError(), "k_pme");
    unsigned long long k = ~0ull;
    RT_CHECK(hipMemcpyAsync(&k, db, 8, hipMemcpyDeviceToHost, g_rt.stream), "pme D2H");
    RT_CHECK(hipStreamSynchronize(g_rt.stream), "pme sync");
    const uint32_t cost = (uint32_t)(k >> 32);
    const int i         = (int)(uint32_t)k;
    if (k != ~0ull && cost < *best_cost) {
        const uint32_t rx = (uint32_t)(search_position_start_x + px[i]), ry = (uint32_t)(search_position_start_y + py[i]);
        *best_mvx  = (int16_t)(mvx + (rx * 8));
        *best_mvy  = (int16_t)(mvy + (ry * 8));
        *best_cost = cost;
    }
}
