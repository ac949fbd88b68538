// svtme_pyramid.hip — the padded three-level luma pyramid of one picture.
//
//   k_build_full<TEN_BIT> : full-resolution plane, pad-to-8 + edge replication
//                           (10-bit input reduced to its MSB plane, enc_handle.c:4964-4972)
//   k_build_down          : 1/4 and 1/16 planes, (a+b+c+d+2)>>2 of the level above
//                           (svt_aom_downsample_2d_c, pic_analysis_process.c:130-158;
//                            svt_aom_downsample_filtering_input_picture :1945-2002;
//                            svt_aom_generate_padding, pic_operators.c:338-383)
//
// One thread writes one dword of the padded plane (margins included), so every
// store is a full coalesced dword; margins are produced by clamping the source
// coordinate, which is the reference's edge replication.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svtme_device.h"

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// level 0: from the caller's picture (8-bit or 10-bit MSB), pad-to-8 + edge replicate.
// One thread writes 4 bytes of the padded plane (margins included). pad_only: src
// is the plane's own interior (k_host_rows wrote it in place), so the dwords
// wholly inside it are left alone and only the margins are written (src aliases
// dst: no __restrict__).
template <bool TEN_BIT>
__global__ void __launch_bounds__(256) k_build_full(const void *src, uint32_t src_stride, int w, int h, DevPlane dst,
                                                    int left, int top, int rows, int pad_only) {
    const int dw_per_row = dst.stride >> 2;
    const int idx        = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= dw_per_row * rows)
        return;
    const int ry = idx / dw_per_row, rx4 = (idx - ry * dw_per_row) * 4;
    const int y  = clampi(ry - top, 0, h - 1);
    const int x0 = rx4 - left;
    const bool in_x = x0 >= 0 && x0 + 3 < w;
    if (pad_only && in_x && ry >= top && ry - top < h)
        return;
    uint32_t v   = 0;
    const uint8_t *p8 = (const uint8_t *)src + (size_t)y * src_stride + x0;
    if (!TEN_BIT && in_x && ((uintptr_t)p8 & 3) == 0) {
        v = *(const uint32_t *)p8; // interior: one dword (a plane read over PCIe moves a quarter of the requests)
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int x = clampi(x0 + k, 0, w - 1);
            uint32_t p;
            if (TEN_BIT)
                p = (uint32_t)(((const uint16_t *)src)[(size_t)y * src_stride + x] >> 2);
            else
                p = ((const uint8_t *)src)[(size_t)y * src_stride + x];
            v |= p << (8 * k);
        }
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

// level 0's interior straight from a page-locked host plane (read over PCIe):
// a few workgroups stream the rows in 16-byte chunks (two chunks in flight per
// thread), so the upload holds a handful of the GPU's workgroup slots while it
// waits on PCIe instead of a grid's worth; k_build_full then pads the plane from
// its own interior. src, src_stride, dst and dst_stride are 4-byte aligned.
#ifndef HOST_ROWS_WGS
#define HOST_ROWS_WGS 128
#endif
__global__ void __launch_bounds__(256) k_host_rows(const uint8_t *__restrict__ src, uint32_t src_stride, int w, int h,
                                                   uint8_t *__restrict__ dst, uint32_t dst_stride) {
    const int chunks  = (w + 15) >> 4;
    const int total   = chunks * h;
    const int step    = (int)gridDim.x * 256;
    auto copy = [&](int i, uint32_t (&v)[4], bool load) {
        const int y = i / chunks, x = (i - y * chunks) * 16;
        const uint32_t *s = (const uint32_t *)(src + (size_t)y * src_stride + x);
        uint32_t *d       = (uint32_t *)(dst + (size_t)y * dst_stride + x);
        const int nb      = min(16, w - x);
        if (nb == 16) {
            if (load) {
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = s[k];
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) d[k] = v[k];
            }
        } else if (!load) { // the row's last partial chunk, bytewise
            const uint8_t *sb = (const uint8_t *)s;
            uint8_t *db       = (uint8_t *)d;
            for (int k = 0; k < nb; k++) db[k] = sb[k];
        }
    };
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += 2 * step) {
        uint32_t a[4], b[4];
        const bool two = i + step < total;
        copy(i, a, true);
        if (two)
            copy(i + step, b, true);
        copy(i, a, false);
        if (two)
            copy(i + step, b, false);
    }
}

extern "C" hipError_t svtme_launch_host_rows(const uint8_t *src, uint32_t src_stride, int w, int h, uint8_t *dst,
                                             uint32_t dst_stride, hipStream_t s) {
    hipLaunchKernelGGL(k_host_rows, dim3(HOST_ROWS_WGS), dim3(256), 0, s, src, src_stride, w, h, dst, dst_stride);
    return hipGetLastError();
}

extern "C" hipError_t svtme_launch_build_full(const void *src, uint32_t src_stride, int w, int h, int ten_bit,
                                              DevPlane dst, int left, int top, int rows, hipStream_t s) {
    const int n = (dst.stride >> 2) * rows;
    // in place (the interior already in the plane): margins only
    const int pad_only = !ten_bit && (const uint8_t *)src == dst.base && src_stride == (uint32_t)dst.stride;
    if (ten_bit)
        hipLaunchKernelGGL(k_build_full<true>, dim3((n + 255) / 256), dim3(256), 0, s, src, src_stride, w, h, dst,
                           left, top, rows, 0);
    else
        hipLaunchKernelGGL(k_build_full<false>, dim3((n + 255) / 256), dim3(256), 0, s, src, src_stride, w, h, dst,
                           left, top, rows, pad_only);
    return hipGetLastError();
}

extern "C" hipError_t svtme_launch_build_down(DevPlane prev, DevPlane dst, int left, int top, int rows,
                                              hipStream_t s) {
    const int n = (dst.stride >> 2) * rows;
    hipLaunchKernelGGL(k_build_down, dim3((n + 255) / 256), dim3(256), 0, s, prev, dst, left, top, rows);
    return hipGetLastError();
}

// The job table from pinned host memory into the device ring: a kernel read over
// PCIe instead of a DMA, so it never queues behind a picture upload's copy on
// the DMA engine (svtme_picture_upload_async)
__global__ void __launch_bounds__(256) k_copy_words(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                    uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

extern "C" hipError_t svtme_launch_copy_words(const void *src, void *dst, uint32_t nwords, hipStream_t s) {
    const uint32_t blocks = (nwords + 255) / 256 < 16 ? (nwords + 255) / 256 : 16;
    hipLaunchKernelGGL(k_copy_words, dim3(blocks), dim3(256), 0, s, (const uint32_t *)src, (uint32_t *)dst, nwords);
    return hipGetLastError();
}

// Load this translation unit's code object now (HIP loads it lazily at the first
// launch of one of its kernels, which would otherwise land in a job's latency)
extern "C" hipError_t svtme_prime_pyramid(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_build_down);
}
