// svtme_pack.hip — packed host output of a picture job (include/svtme.h,
// svtme_pack_layout): per SB only the bytes the encoder's ME consumer reads,
// sized by its MeSbResults allocation (pcs.c:91-117). The device-to-host copy
// of a 4K p8 picture with 4 references drops from 15.5 MB (whole records and
// SB results) to about 5.5 MB (record tails and the allocated candidate slots).
//
// One workgroup per SB. The SB's packed bytes are assembled in LDS (byte-wise
// gathers from the job's own record / SB-result buffers, still in L2) and
// written out as 16-byte stores.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "svtme_device.h"

#define PACK_MAX_BYTES 12288 // >= svtme_packed_sb_bytes of the largest layout (R = 8, full records, 85 PUs)

__global__ void __launch_bounds__(256) k_pack(const svtme_ref_record *__restrict__ recs,
                                              const svtme_sb_result *__restrict__ sbr, uint32_t R,
                                              svtme_pack_layout L, uint32_t stride, uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[PACK_MAX_BYTES];
    const uint32_t sb = blockIdx.x, tid = threadIdx.x;
    const uint8_t *rb = (const uint8_t *)(recs + (size_t)sb * R);
    // records: whole, or the tail of each (the 24 bytes from offsetof(hme_sad))
    const uint32_t tail0 = (uint32_t)offsetof(svtme_ref_record, hme_sad);
    const uint32_t rsz   = L.full_records ? (uint32_t)sizeof(svtme_ref_record) : (uint32_t)sizeof(svtme_record_tail);
    const uint32_t rbytes = R * rsz;
    if (L.full_records) {
        const uint32_t *rw = (const uint32_t *)rb;
        for (uint32_t i = tid; i < rbytes / 4; i += 256) ((uint32_t *)buf)[i] = rw[i];
    } else {
        for (uint32_t i = tid; i < rbytes / 4; i += 256) {
            const uint32_t r = i / (rsz / 4), k = i - r * (rsz / 4);
            ((uint32_t *)buf)[i] = ((const uint32_t *)(rb + (size_t)r * sizeof(svtme_ref_record) + tail0))[k];
        }
    }
    uint32_t o = rbytes;
    if (L.sb_results) {
        const svtme_sb_result *s = sbr + sb;
        const uint32_t np = L.n_pus, mc = L.max_cand, mr = L.max_refs;
        uint32_t *w = (uint32_t *)(buf + o);
        if (tid < 6) {
            const uint32_t v[6] = {s->me_8x8_cost_variance, s->rc_me_distortion, s->me_64x64_distortion,
                                   s->me_32x32_distortion, s->me_16x16_distortion, s->me_8x8_distortion};
            w[tid] = v[tid];
        }
        if (tid < SVTME_PU_COUNT)
            w[6 + tid] = s->me_distortion[tid];
        for (uint32_t i = tid; i < np * mr; i += 256) {
            const uint32_t pu = i / mr;
            w[6 + SVTME_PU_COUNT + i] = s->me_mv_array[pu][i - pu * mr];
        }
        o += 4u * (6u + SVTME_PU_COUNT + np * mr);
        if (tid < 4)
            buf[o + tid] = tid == 0 ? s->stationary_block_present : tid == 1 ? s->rc_me_allow_gm : 0;
        o += 4;
        for (uint32_t i = tid; i < np; i += 256) buf[o + i] = s->total_me_candidate_index[i];
        o += np;
        for (uint32_t i = tid; i < np * mc; i += 256) {
            const uint32_t pu = i / mc;
            buf[o + i] = s->me_candidate_array[pu][i - pu * mc];
        }
        o += np * mc;
    }
    for (uint32_t i = o + tid; i < stride; i += 256) buf[i] = 0;
    __syncthreads();
    uint4 *dst = (uint4 *)(out + (size_t)sb * stride);
    for (uint32_t i = tid; i < stride / 16; i += 256) dst[i] = ((const uint4 *)buf)[i];
}

extern "C" hipError_t svtme_launch_pack(const svtme_ref_record *d_recs, const svtme_sb_result *d_sb, uint32_t n_sb,
                                        uint32_t R, const svtme_pack_layout *L, void *d_out, hipStream_t s) {
    const uint32_t stride = svtme_packed_sb_bytes(L, R);
    if (stride > PACK_MAX_BYTES || (L->sb_results && !d_sb))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pack, dim3(n_sb), dim3(256), 0, s, d_recs, d_sb, R, *L, stride, (uint8_t *)d_out);
    return hipGetLastError();
}

extern "C" hipError_t svtme_prime_pack(void) { // (see svtme_prime_pyramid)
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_pack);
}
