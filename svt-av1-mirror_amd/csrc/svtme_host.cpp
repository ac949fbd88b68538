// svtme_host.cpp — C ABI of include/svtme.h on HIP (gfx950 / MI355X).
//
// Picture-level job API: a context owns one HIP stream, a cache of resident
// picture pyramids keyed by picture_number (the PA reference pyramids of
// reference_object.c:243-305, built on the GPU), and the device record
// buffers of the last job. One job = one launch of k_me_sb over the SB range
// (+ k_me_post for candidate arrays / distortions).
//
// Per-kernel rtcd variants (svt_*_hip): synchronous, caller-owned host memory,
// copied to a per-process device scratch, one small kernel, copied back.
//
// No CPU fallback anywhere: HIP failures return an error status (job API) or
// set svtme_last_error() and print to stderr (void rtcd variants).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "svtme_device.h"

extern "C" hipError_t svtme_launch_build_full(const void *src, uint32_t src_stride, int w, int h, int ten_bit,
                                              DevPlane dst, int left, int top, int rows, hipStream_t s);
extern "C" hipError_t svtme_launch_build_down(DevPlane prev, DevPlane dst, int left, int top, int rows,
                                              hipStream_t s);
extern "C" hipError_t svtme_launch_stages(const DevJob *dj, uint32_t sb_count, hipStream_t s, hipEvent_t *mid);
extern "C" void svtme_stage_a_list(const svtme_job *job, uint8_t *list, uint32_t *count);
extern "C" void svtme_stage_b_list(const svtme_job *job, uint8_t *list, uint32_t *count);
extern "C" uint32_t svtme_fp_parts(const svtme_controls *c);

// ----------------------------------------------------------------------------
// errors
// ----------------------------------------------------------------------------
static thread_local std::string g_last_error;

static svtme_status fail(svtme_status st, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    fprintf(stderr, "[svtme] %s\n", buf);
    return st;
}

#define HIP_TRY(expr)                                                                                               \
    do {                                                                                                            \
        hipError_t _e = (expr);                                                                                     \
        if (_e != hipSuccess)                                                                                       \
            return fail(SVTME_ERR_UNDEFINED, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__,      \
                        __LINE__);                                                                                  \
    } while (0)

extern "C" const char *svtme_last_error(void) { return g_last_error.c_str(); }

// used by the rtcd variants (svtme_rtcd.hip), which return void
extern "C" void svtme_set_error_internal(const char *msg) {
    g_last_error = msg;
    fprintf(stderr, "[svtme] %s\n", msg);
}

// ----------------------------------------------------------------------------
// context
// ----------------------------------------------------------------------------
struct PicBuf {
    uint8_t *mem = nullptr;
    size_t bytes = 0;
    uint32_t W = 0, H = 0;
    DevPyramid pyr{};
};

struct svtme_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::map<uint64_t, PicBuf> pics;
    void *staging      = nullptr;
    size_t staging_cap = 0;
    svtme_ref_record *d_records = nullptr;
    size_t records_cap          = 0;
    svtme_sb_result *d_sb       = nullptr;
    size_t sb_cap               = 0;
    uint32_t last_count = 0, last_R = 0;
    bool last_has_sb    = false;
    bool timing         = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_mid[3] = {nullptr, nullptr, nullptr}; // after stages A, D, B
    ARes *d_ares    = nullptr; // stage-A results [count][SVTME_A_N]
    size_t ares_cap = 0;
    BState *d_bst   = nullptr; // stage-B state [count]
    size_t bst_cap  = 0;
    unsigned long long *d_keys = nullptr; // wide full-pel argmin keys [count][R][85]
    size_t keys_cap            = 0;
    bool keys_rest             = false; // every key is ~0 (banded jobs accumulate with atomic min)
    CSlot *d_cslot             = nullptr; // [count][R]
    size_t cslot_cap           = 0;
#ifdef SVTME_STAMPS
    unsigned long long *d_stamps = nullptr;
    size_t stamps_cap            = 0;
    double stamp_sum[16]         = {0};
    uint64_t stamp_n             = 0;
#endif
    std::mutex mu;
};

extern "C" uint32_t svtme_sb_total(uint32_t width, uint32_t height) {
    return ((width + 63) / 64) * ((height + 63) / 64);
}

extern "C" uint32_t svtme_job_ref_slots(const svtme_job *job) {
    return job->num_refs[0] + (job->num_lists == 2 ? job->num_refs[1] : 0);
}

extern "C" svtme_status svtme_ctx_create(int device, svtme_ctx **out) {
    if (!out)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_ctx_create: null out");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_ctx_create: device %d of %d", device, n);
    HIP_TRY(hipSetDevice(device));
    svtme_ctx *c = new svtme_ctx();
    c->device    = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(SVTME_ERR_INSUFFICIENT_RESOURCES, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return SVTME_OK;
}

extern "C" void svtme_ctx_destroy(svtme_ctx *c) {
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto &kv : c->pics) (void)hipFree(kv.second.mem);
    if (c->staging)
        (void)hipFree(c->staging);
    if (c->d_records)
        (void)hipFree(c->d_records);
    if (c->d_sb)
        (void)hipFree(c->d_sb);
    if (c->ev0)
        (void)hipEventDestroy(c->ev0);
    if (c->ev1)
        (void)hipEventDestroy(c->ev1);
    for (auto &e : c->ev_mid)
        if (e)
            (void)hipEventDestroy(e);
#ifdef SVTME_STAMPS
    if (c->stamp_n) {
        fprintf(stderr, "[svtme stamps] %llu SBs, mean cycles per phase (from previous stamp):",
                (unsigned long long)c->stamp_n);
        for (int k = 1; k < 16; k++)
            if (c->stamp_sum[k] > 0)
                fprintf(stderr, " p%d=%.0f", k, c->stamp_sum[k] / c->stamp_n);
        fprintf(stderr, "\n");
    }
    if (c->d_stamps)
        (void)hipFree(c->d_stamps);
#endif
    if (c->d_ares)
        (void)hipFree(c->d_ares);
    if (c->d_bst)
        (void)hipFree(c->d_bst);
    if (c->d_keys)
        (void)hipFree(c->d_keys);
    if (c->d_cslot)
        (void)hipFree(c->d_cslot);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" void *svtme_stream(svtme_ctx *c) { return c ? (void *)c->stream : nullptr; }

static svtme_status ensure_buf(void **p, size_t *cap, size_t need) {
    if (*cap >= need)
        return SVTME_OK;
    if (*p)
        HIP_TRY(hipFree(*p));
    *p   = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, need));
    *cap = need;
    return SVTME_OK;
}

// allocate the three planes of a W x H picture in one buffer
static svtme_status alloc_pic(svtme_ctx *c, uint64_t pn, uint32_t W, uint32_t H, PicBuf **out) {
    auto it = c->pics.find(pn);
    if (it != c->pics.end() && (it->second.W != W || it->second.H != H)) {
        HIP_TRY(hipFree(it->second.mem));
        c->pics.erase(it);
        it = c->pics.end();
    }
    size_t offs[3], total = 0;
    uint32_t w[3], h[3], left[3], top[3], stride[3], rows[3], pad[3];
    for (int lv = 0; lv < 3; lv++) {
        svtme_plane_geometry(lv, W, H, &w[lv], &h[lv], &left[lv], &top[lv], &stride[lv], &rows[lv], &pad[lv]);
        offs[lv] = total;
        total += (size_t)stride[lv] * rows[lv];
        total = (total + 255) & ~(size_t)255;
    }
    if (it == c->pics.end()) {
        PicBuf pb;
        HIP_TRY(hipMalloc((void **)&pb.mem, total));
        pb.bytes = total;
        pb.W = W, pb.H = H;
        it = c->pics.emplace(pn, pb).first;
    }
    PicBuf &pb = it->second;
    for (int lv = 0; lv < 3; lv++) {
        DevPlane &p = pb.pyr.lv[lv];
        p.base      = pb.mem + offs[lv] + (size_t)top[lv] * stride[lv] + left[lv];
        p.stride    = (int32_t)stride[lv];
        p.width     = (int32_t)w[lv];
        p.height    = (int32_t)h[lv];
        p.pad       = (int32_t)pad[lv];
    }
    *out = &pb;
    return SVTME_OK;
}

static svtme_status build_pyramid(svtme_ctx *c, PicBuf *pb, const void *dsrc, uint32_t src_stride, uint32_t w,
                                  uint32_t h, int ten_bit) {
    uint32_t pw, ph, left, top, stride, rows, pad;
    svtme_plane_geometry(0, pb->W, pb->H, &pw, &ph, &left, &top, &stride, &rows, &pad);
    HIP_TRY(svtme_launch_build_full(dsrc, src_stride, (int)w, (int)h, ten_bit, pb->pyr.lv[0], (int)left, (int)top,
                                    (int)rows, c->stream));
    for (int lv = 1; lv < 3; lv++) {
        svtme_plane_geometry(lv, pb->W, pb->H, &pw, &ph, &left, &top, &stride, &rows, &pad);
        HIP_TRY(svtme_launch_build_down(pb->pyr.lv[lv - 1], pb->pyr.lv[lv], (int)left, (int)top, (int)rows,
                                        c->stream));
    }
    return SVTME_OK;
}

static svtme_status upload_host(svtme_ctx *c, uint64_t pn, const void *y, uint32_t stride, uint32_t w, uint32_t h,
                                int ten_bit) {
    if (!c || !y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t bpp = ten_bit ? 2 : 1;
    svtme_status st    = ensure_buf(&c->staging, &c->staging_cap, (size_t)w * h * bpp);
    if (st)
        return st;
    HIP_TRY(hipMemcpy2DAsync(c->staging, (size_t)w * bpp, y, (size_t)stride * bpp, (size_t)w * bpp, h,
                             hipMemcpyHostToDevice, c->stream));
    PicBuf *pb;
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    if ((st = build_pyramid(c, pb, c->staging, w, w, h, ten_bit)))
        return st;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

extern "C" svtme_status svtme_picture_upload(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride, uint32_t w,
                                             uint32_t h) {
    return upload_host(c, pn, y, stride, w, h, 0);
}

extern "C" svtme_status svtme_picture_upload_10bit(svtme_ctx *c, uint64_t pn, const uint16_t *y, uint32_t stride,
                                                   uint32_t w, uint32_t h) {
    return upload_host(c, pn, y, stride, w, h, 1);
}

extern "C" svtme_status svtme_picture_upload_device(svtme_ctx *c, uint64_t pn, const uint8_t *d_y, uint32_t stride,
                                                    uint32_t w, uint32_t h) {
    if (!c || !d_y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload_device: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    PicBuf *pb;
    svtme_status st;
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    if ((st = build_pyramid(c, pb, d_y, stride, w, h, 0)))
        return st;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

extern "C" svtme_status svtme_picture_release(svtme_ctx *c, uint64_t pn) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_release: null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->pics.find(pn);
    if (it == c->pics.end())
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_release: picture %llu not resident",
                    (unsigned long long)pn);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(it->second.mem));
    c->pics.erase(it);
    return SVTME_OK;
}

// Copy one level back in the reference's geometry: (h + 2 pad) rows of (w + 2 pad) bytes
extern "C" svtme_status svtme_picture_download(svtme_ctx *c, uint64_t pn, int level, uint8_t *dst, uint32_t *stride,
                                               uint32_t *width, uint32_t *height, uint32_t *pad) {
    if (!c || level < 0 || level > 2)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_download: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->pics.find(pn);
    if (it == c->pics.end())
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_download: picture %llu not resident",
                    (unsigned long long)pn);
    const DevPlane &p = it->second.pyr.lv[level];
    const uint32_t S  = (uint32_t)(p.width + 2 * p.pad);
    if (stride)
        *stride = S;
    if (width)
        *width = (uint32_t)p.width;
    if (height)
        *height = (uint32_t)p.height;
    if (pad)
        *pad = (uint32_t)p.pad;
    if (!dst)
        return SVTME_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy2D(dst, S, p.base - (ptrdiff_t)p.pad * p.stride - p.pad, (size_t)p.stride, S,
                        (size_t)(p.height + 2 * p.pad), hipMemcpyDeviceToHost));
    return SVTME_OK;
}

// ----------------------------------------------------------------------------
// jobs
// ----------------------------------------------------------------------------
static svtme_status validate_job(svtme_ctx *c, const svtme_job *job, DevJob *dj, uint32_t *count) {
    if (!job)
        return fail(SVTME_ERR_BAD_PARAMETER, "null job");
    if ((job->width & 7) || (job->height & 7) || job->width == 0 || job->height == 0)
        return fail(SVTME_ERR_BAD_PARAMETER, "job size %ux%u must be a non-zero multiple of 8", job->width,
                    job->height);
    if (job->num_lists < 1 || job->num_lists > 2 || job->num_refs[0] > 4 || job->num_refs[1] > 4)
        return fail(SVTME_ERR_BAD_PARAMETER, "bad reference counts");
    if (job->ctrl.num_hme_sa_w != 2 || job->ctrl.num_hme_sa_h != 2)
        return fail(SVTME_ERR_BAD_PARAMETER, "only 2x2 HME-L0 search regions are supported "
                                             "(motion_estimation.c:1875)");
    if (job->ctrl.enable_me_sr_adjustment && job->ctrl.distance_based_hme_resizing &&
        job->ctrl.reduce_hme_l0_sr_th_min && job->ctrl.reduce_hme_l0_sr_th_max)
        return fail(SVTME_ERR_BAD_PARAMETER, "reduce_hme_l0_sr_th_min/max (real-time tune, enc_mode_config.c:690-703) "
                                             "are not supported");
    if (job->me_type != 0 && job->me_type != SVTME_ME_OPEN_LOOP && job->me_type != SVTME_ME_MCTF)
        return fail(SVTME_ERR_BAD_PARAMETER, "me_type %u is neither SVTME_ME_OPEN_LOOP nor SVTME_ME_MCTF",
                    job->me_type);
    if (job->width > 16384 || job->height > 16384)
        return fail(SVTME_ERR_BAD_PARAMETER, "picture too large for int16 search arithmetic");
    const uint32_t total = svtme_sb_total(job->width, job->height);
    const uint32_t n     = job->sb_count ? job->sb_count : total - job->sb_begin;
    if (job->sb_begin >= total || job->sb_begin + n > total)
        return fail(SVTME_ERR_BAD_PARAMETER, "SB range [%u, %u) outside the picture's %u SBs", job->sb_begin,
                    job->sb_begin + n, total);
    auto find = [&](uint64_t pn, DevPyramid *out) -> svtme_status {
        auto it = c->pics.find(pn);
        if (it == c->pics.end())
            return fail(SVTME_ERR_BAD_PARAMETER, "picture %llu is not resident (svtme_picture_upload it first)",
                        (unsigned long long)pn);
        if (it->second.W != job->width || it->second.H != job->height)
            return fail(SVTME_ERR_BAD_PARAMETER, "picture %llu is %ux%u, job is %ux%u", (unsigned long long)pn,
                        it->second.W, it->second.H, job->width, job->height);
        *out = it->second.pyr;
        return SVTME_OK;
    };
    memset(dj, 0, sizeof(*dj));
    dj->job = *job;
    svtme_status st;
    if ((st = find(job->picture_number, &dj->cur)))
        return st;
    for (int l = 0; l < job->num_lists; l++)
        for (int r = 0; r < job->num_refs[l]; r++)
            if ((st = find(job->ref_picture_number[l][r], &dj->ref[l][r])))
                return st;
    dj->R         = svtme_job_ref_slots(job);
    dj->pic_w_b64 = (job->width + 63) / 64;
    *count        = n;
    dj->job.sb_count = n;
    if (dj->R == 0)
        return fail(SVTME_ERR_BAD_PARAMETER, "job has no references");
    return SVTME_OK;
}

static svtme_status submit_locked(svtme_ctx *c, const svtme_job *job, bool with_sb, svtme_ref_record *d_out,
                                  svtme_sb_result *d_out_sb) {
    HIP_TRY(hipSetDevice(c->device));
    DevJob dj;
    uint32_t count;
    svtme_status st = validate_job(c, job, &dj, &count);
    if (st)
        return st;
    if (d_out) {
        dj.out_records = d_out;
        dj.out_sb      = d_out_sb;
    } else {
        if ((st = ensure_buf((void **)&c->d_records, &c->records_cap,
                             (size_t)count * dj.R * sizeof(svtme_ref_record))))
            return st;
        dj.out_records = c->d_records;
        if (with_sb) {
            if ((st = ensure_buf((void **)&c->d_sb, &c->sb_cap, (size_t)count * sizeof(svtme_sb_result))))
                return st;
            dj.out_sb = c->d_sb;
        }
    }
#ifdef SVTME_STAMPS
    if ((st = ensure_buf((void **)&c->d_stamps, &c->stamps_cap, (size_t)count * 16 * 8)))
        return st;
    HIP_TRY(hipMemsetAsync(c->d_stamps, 0, (size_t)count * 16 * 8, c->stream));
    dj.stamps = c->d_stamps;
#endif
    if (c->timing)
        HIP_TRY(hipEventRecord(c->ev0, c->stream));
    if ((st = ensure_buf((void **)&c->d_ares, &c->ares_cap, (size_t)count * SVTME_A_N * sizeof(ARes))))
        return st;
    if ((st = ensure_buf((void **)&c->d_bst, &c->bst_cap, (size_t)count * sizeof(BState))))
        return st;
    dj.ares = c->d_ares;
    dj.bst  = c->d_bst;
    dj.parts = svtme_fp_parts(&dj.job.ctrl);
    if (dj.parts) { // wide full-pel stage (k_stage_c1 + k_stage_e)
        const size_t kb = (size_t)count * dj.R * SVTME_PU_COUNT * sizeof(unsigned long long);
        if (c->keys_cap < kb) {
            if ((st = ensure_buf((void **)&c->d_keys, &c->keys_cap, kb)))
                return st;
            c->keys_rest = false;
        }
        if ((st = ensure_buf((void **)&c->d_cslot, &c->cslot_cap, (size_t)count * dj.R * sizeof(CSlot))))
            return st;
        if (dj.parts > 1 && !c->keys_rest) {
            HIP_TRY(hipMemsetAsync(c->d_keys, 0xFF, c->keys_cap, c->stream));
            c->keys_rest = true;
        }
        if (dj.parts == 1)
            c->keys_rest = false; // plain stores leave keys behind
        dj.keys  = c->d_keys;
        dj.cslot = c->d_cslot;
    }
    svtme_stage_a_list(&dj.job, dj.ta_list, &dj.ta_count);
    svtme_stage_b_list(&dj.job, dj.tb_list, &dj.tb_count);
    HIP_TRY(svtme_launch_stages(&dj, count, c->stream, c->timing ? c->ev_mid : nullptr));
#ifdef SVTME_STAMPS
    {
        std::vector<unsigned long long> h((size_t)count * 16);
        HIP_TRY(hipMemcpyAsync(h.data(), c->d_stamps, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (uint32_t b = 0; b < count; b++) {
            unsigned long long prev = h[b * 16];
            for (int k = 1; k < 16; k++) {
                const unsigned long long v = h[b * 16 + k];
                if (v) {
                    c->stamp_sum[k] += (double)(v - prev);
                    prev = v;
                }
            }
        }
        c->stamp_n += count;
    }
#endif
    if (c->timing)
        HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->last_count  = count;
    c->last_R      = dj.R;
    c->last_has_sb = with_sb && !d_out;
    return SVTME_OK;
}

extern "C" svtme_status svtme_submit_picture_device(svtme_ctx *c, const svtme_job *job, svtme_ref_record *d_recs,
                                                    svtme_sb_result *d_sb) {
    if (!c || !d_recs)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_picture_device: null ctx or output");
    std::lock_guard<std::mutex> lk(c->mu);
    return submit_locked(c, job, d_sb != nullptr, d_recs, d_sb);
}

extern "C" svtme_status svtme_set_timing(svtme_ctx *c, int enable) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    if (enable && !c->ev0) {
        HIP_TRY(hipEventCreate(&c->ev0));
        HIP_TRY(hipEventCreate(&c->ev1));
        for (auto &e : c->ev_mid)
            HIP_TRY(hipEventCreate(&e));
    }
    c->timing = enable != 0;
    return SVTME_OK;
}

extern "C" float svtme_kernel_ms(svtme_ctx *c) {
    if (!c || !c->timing)
        return -1.0f;
    float ms = -1.0f;
    if (hipEventSynchronize(c->ev1) != hipSuccess || hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess)
        return -1.0f;
    return ms;
}

extern "C" float svtme_stage_ms(svtme_ctx *c, int stage) {
    if (!c || !c->timing || stage < 0 || stage > 3 || !c->ev_mid[0])
        return -1.0f;
    hipEvent_t a = stage == 0 ? c->ev0 : c->ev_mid[stage - 1];
    hipEvent_t b = stage == 3 ? c->ev1 : c->ev_mid[stage];
    float ms = -1.0f;
    if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess)
        return -1.0f;
    return ms;
}

extern "C" svtme_status svtme_submit_picture_async(svtme_ctx *c, const svtme_job *job) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    return submit_locked(c, job, true, nullptr, nullptr);
}

extern "C" svtme_status svtme_sync(svtme_ctx *c) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

extern "C" svtme_status svtme_fetch(svtme_ctx *c, svtme_ref_record *recs, svtme_sb_result *sb) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    if (recs)
        HIP_TRY(hipMemcpyAsync(recs, c->d_records, (size_t)c->last_count * c->last_R * sizeof(svtme_ref_record),
                               hipMemcpyDeviceToHost, c->stream));
    if (sb) {
        if (!c->last_has_sb)
            return fail(SVTME_ERR_BAD_PARAMETER, "last job produced no SB results");
        HIP_TRY(hipMemcpyAsync(sb, c->d_sb, (size_t)c->last_count * sizeof(svtme_sb_result), hipMemcpyDeviceToHost,
                               c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

extern "C" svtme_status svtme_submit_picture(svtme_ctx *c, const svtme_job *job, svtme_ref_record *recs,
                                             svtme_sb_result *sb) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    {
        std::lock_guard<std::mutex> lk(c->mu);
        svtme_status st = submit_locked(c, job, sb != nullptr, nullptr, nullptr);
        if (st)
            return st;
    }
    return svtme_fetch(c, recs, sb);
}

extern "C" void *svtme_device_records(svtme_ctx *c, uint64_t *bytes) {
    if (!c)
        return nullptr;
    if (bytes)
        *bytes = (uint64_t)c->last_count * c->last_R * sizeof(svtme_ref_record);
    return c->d_records;
}

// ----------------------------------------------------------------------------
// svt_aom_sig_deriv_me restatement, non-RTC, non-screen-content
// (enc_mode_config.c:136-212 set_hme_search_params, :213-340 set_me_search_params,
//  :341-529 prune / sr / 8x8-var / mv-adj controls, :532-589 pre-HME, :671-808)
// ----------------------------------------------------------------------------
static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

extern "C" void svtme_derive_controls(int enc_mode, int qp, int res, int tl, int hierarchical_levels,
                                      int frame_rate_q16, svtme_controls *c) {
    memset(c, 0, sizeof(*c));
    const bool is_base = tl == 0;
    // set_me_search_params (enc_mode_config.c:213-340), rtc_tune = 0, sc_class1 = 0
    int q_mult = 0;
    auto sa = [](svtme_area_minmax &a, int w0, int h0, int w1, int h1) {
        a.sa_min = {(uint16_t)w0, (uint16_t)h0};
        a.sa_max = {(uint16_t)w1, (uint16_t)h1};
    };
    if (enc_mode <= 1)
        sa(c->me_sa, 64, 64, 256, 256);
    else if (enc_mode <= 2)
        sa(c->me_sa, 32, 32, 128, 128);
    else if (enc_mode <= 4)
        sa(c->me_sa, 24, 24, 104, 104);
    else if (enc_mode <= 6) {
        sa(c->me_sa, 16, 16, 64, 32);
        q_mult = 7;
    } else if (enc_mode <= 9) {
        if (hierarchical_levels <= 3) {
            if (res < 5)
                sa(c->me_sa, 8, 5, 16, 9);
            else
                sa(c->me_sa, 8, 1, 8, 1);
        } else if (res < 4)
            sa(c->me_sa, 16, 16, 32, 16);
        else
            sa(c->me_sa, 16, 6, 16, 9);
        q_mult = 7;
    } else {
        sa(c->me_sa, 16, 6, 16, 6);
        q_mult = 6;
    }
    if (q_mult) {
        const int qw = clip3(500, 1000, (int)(q_mult * ((31 * qp) - 700)) >> 3);
        c->me_sa.sa_min.width  = (uint16_t)std::max(8, (c->me_sa.sa_min.width * qw) / 1000);
        c->me_sa.sa_min.height = (uint16_t)std::max(3, (c->me_sa.sa_min.height * qw) / 1000);
        c->me_sa.sa_max.width  = (uint16_t)std::max(8, (c->me_sa.sa_max.width * qw) / 1000);
        c->me_sa.sa_max.height = (uint16_t)std::max(3, (c->me_sa.sa_max.height * qw) / 1000);
    }
    if (frame_rate_q16 >> 16) { // low_frame_rate_flag (enc_mode_config.c:334-339)
        c->me_sa.sa_min.width  = (uint16_t)((c->me_sa.sa_min.width * 3) >> 1);
        c->me_sa.sa_min.height = (uint16_t)((c->me_sa.sa_min.height * 3) >> 1);
    }
    // set_hme_search_params (enc_mode_config.c:136-212)
    c->num_hme_sa_w = 2;
    c->num_hme_sa_h = 2;
    q_mult          = 0;
    if (enc_mode <= 1) {
        if (res < 5)
            sa(c->hme_l0_sa, 32, 32, 192, 192);
        else
            sa(c->hme_l0_sa, 240, 240, 480, 480);
    } else if (enc_mode <= 3)
        sa(c->hme_l0_sa, 32, 32, 192, 192);
    else if (enc_mode <= 6) {
        sa(c->hme_l0_sa, 32, 32, 192, 192);
        q_mult = 3;
    } else if (enc_mode <= 7) {
        if (res >= 5)
            sa(c->hme_l0_sa, 32, 32, 192, 192);
        else
            sa(c->hme_l0_sa, 16, 16, 192, 192);
        q_mult = 3;
    } else if (enc_mode <= 9) {
        sa(c->hme_l0_sa, 16, 16, 192, 192);
        q_mult = 3;
    } else {
        if (res < 5)
            sa(c->hme_l0_sa, 8, 8, 96, 96);
        else
            sa(c->hme_l0_sa, 16, 16, 96, 96);
        q_mult = 3;
    }
    if (q_mult) {
        const int qw = clip3(500, 1000, (int)(q_mult * ((8 * qp) - 125)));
        c->hme_l0_sa.sa_min.width  = (uint16_t)std::max(8, (c->hme_l0_sa.sa_min.width * qw) / 1000);
        c->hme_l0_sa.sa_min.height = (uint16_t)std::max(8, (c->hme_l0_sa.sa_min.height * qw) / 1000);
        c->hme_l0_sa.sa_max.width  = (uint16_t)std::max(96, (c->hme_l0_sa.sa_max.width * qw) / 1000);
        c->hme_l0_sa.sa_max.height = (uint16_t)std::max(96, (c->hme_l0_sa.sa_max.height * qw) / 1000);
    }
    if (enc_mode <= -1) {
        c->hme_l1_sa = {16, 16};
        c->hme_l2_sa = {16, 16};
    } else {
        c->hme_l1_sa = {8, 3};
        c->hme_l2_sa = {8, 3};
    }
    // HME level flags (enc_mode_config.c:1608-1619) and methods (:687-689)
    c->enable_hme_flag        = 1;
    c->enable_hme_level0_flag = 1;
    c->enable_hme_level1_flag = 1;
    c->enable_hme_level2_flag = enc_mode <= 6 ? 1 : 0;
    c->hme_search_method      = SVTME_SUB_SAD_SEARCH;
    c->me_search_method       = SVTME_SUB_SAD_SEARCH;
    c->reduce_hme_l0_sr_th_min = 0;
    c->reduce_hme_l0_sr_th_max = 0;
    // pre-HME level (enc_mode_config.c:707-722, :532-589)
    const int prehme_level = enc_mode <= 7 ? 2 : 4;
    c->prehme_enable = 1;
    if (prehme_level == 2) {
        sa(c->prehme_sa_cfg[0], 8, 100, 8, 400);
        sa(c->prehme_sa_cfg[1], 96, 3, 384, 3);
        c->prehme_skip_search_line = 0;
        c->prehme_l1_early_exit    = 0;
    } else {
        sa(c->prehme_sa_cfg[0], 8, 100, 8, 350);
        sa(c->prehme_sa_cfg[1], 32, 7, 128, 7);
        c->prehme_skip_search_line = 1;
        c->prehme_l1_early_exit    = 1;
    }
    // hme/me reference pruning (enc_mode_config.c:729-744, :341-410)
    int prune_level;
    if (enc_mode <= 0)
        prune_level = is_base ? 1 : 2;
    else if (enc_mode <= 1)
        prune_level = is_base ? 1 : 4;
    else if (enc_mode <= 3)
        prune_level = is_base ? 1 : 5;
    else if (enc_mode <= 9)
        prune_level = is_base ? 1 : 6;
    else
        prune_level = 6;
    static const uint16_t hme_th[7] = {0xFFFF, 80, 50, 30, 15, 5, 5};
    static const uint16_t me_th[7]  = {0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF, 60, 60, 60};
    c->enable_me_hme_ref_pruning               = prune_level ? 1 : 0;
    c->prune_ref_if_hme_sad_dev_bigger_than_th = hme_th[prune_level];
    c->prune_ref_if_me_sad_dev_bigger_than_th  = me_th[prune_level];
    if (prune_level == 6) {
        c->zz_sad_th    = 20 * 64 * 64;
        c->zz_sad_pct   = 5;
        c->phme_sad_th  = 10 * 64 * 64;
        c->phme_sad_pct = 5;
    }
    // hme-based ME search-area adjustment (enc_mode_config.c:747-757, :446-509)
    const int sr_level = enc_mode <= -1 ? 0 : (enc_mode <= 0 ? 1 : 3);
    if (sr_level) {
        c->enable_me_sr_adjustment              = 1;
        c->reduce_me_sr_based_on_mv_length_th   = 4;
        c->stationary_hme_sad_abs_th            = 12000;
        c->stationary_me_sr_divisor             = 8;
        c->reduce_me_sr_based_on_hme_sad_abs_th = sr_level == 3 ? 12000 : 6000;
        c->me_sr_divisor_for_low_hme_sad        = 8;
        c->distance_based_hme_resizing          = sr_level == 3 ? 1 : 0;
        if (!c->enable_hme_level2_flag) { // :500-508
            c->stationary_hme_sad_abs_th            = (uint16_t)(c->stationary_hme_sad_abs_th / 4);
            c->reduce_me_sr_based_on_hme_sad_abs_th = (uint16_t)(c->reduce_me_sr_based_on_hme_sad_abs_th / 4);
        }
    }
    // mv-based search-area adjustment (enc_mode_config.c:759-764, :411-431)
    if (enc_mode <= 3) {
        c->mv_sa_adj_enabled          = 1;
        c->mv_sa_adj_nearest_ref_only = 1;
        c->mv_sa_adj_mv_size_th       = 25;
        c->mv_sa_adj_sa_multiplier    = 2;
    }
    // 8x8-variance search-area adjustment, level 2 (enc_mode_config.c:766-767, :511-529)
    c->me_8x8_var_enabled = 1;
    c->me_sr_div4_th      = 80000;
    c->me_sr_div2_th      = 150000;
    c->me_sr_mult2_th     = 0xFFFFFFFFu;
    c->prune_me_candidates_th     = enc_mode <= 6 ? 0 : 65;
    c->use_best_unipred_cand_only = enc_mode <= 3 ? 0 : 1; // enc_mode_config.c:1802-1805
    c->me_early_exit_th           = enc_mode <= 4 ? 0 : 64 * 64 * 8;
    c->me_safe_limit_zz_th        = 0; // safe_limit_nref == 2 at mrp levels 9-10 (enc_handle.c:3542-3543)
    c->prev_me_stage_based_exit_th = 0;
}

// ----------------------------------------------------------------------------
// TF-ME (ME_MCTF) controls: the tf HME enables by tf_ctrls.hme_me_level
// (enc_mode_config.c:1620-1645), svt_aom_sig_deriv_me_tf (:814-854) with
// tf_set_me_hme_params_oq (:588-665), and set_hme_search_params_mctf(ctx, 0)
// (temporal_filtering.c:2759-2767)
// ----------------------------------------------------------------------------
extern "C" void svtme_derive_controls_tf(int hme_me_level, int qp_opt, int qp, int res, svtme_controls *c) {
    memset(c, 0, sizeof(*c));
    auto sa = [](svtme_area_minmax &a, int w0, int h0, int w1, int h1) {
        a.sa_min = {(uint16_t)w0, (uint16_t)h0};
        a.sa_max = {(uint16_t)w1, (uint16_t)h1};
    };
    c->num_hme_sa_w = 2;
    c->num_hme_sa_h = 2;
    switch (hme_me_level) {
    case 0:
        sa(c->hme_l0_sa, 30, 30, 60, 60);
        c->hme_l1_sa = {16, 16};
        c->hme_l2_sa = {16, 16};
        sa(c->me_sa, 60, 60, 120, 120);
        break;
    case 1:
        sa(c->hme_l0_sa, 16, 16, 32, 32);
        c->hme_l1_sa = {16, 16};
        c->hme_l2_sa = {16, 16};
        sa(c->me_sa, 16, 16, 32, 32);
        break;
    case 2:
        if (res <= 1) { // INPUT_SIZE_360p_RANGE
            sa(c->hme_l0_sa, 8, 8, 8, 8);
            c->hme_l1_sa = {8, 8};
        } else if (res <= 2) { // INPUT_SIZE_480p_RANGE
            sa(c->hme_l0_sa, 8, 8, 16, 16);
            c->hme_l1_sa = {8, 8};
        } else {
            sa(c->hme_l0_sa, 16, 16, 32, 32);
            c->hme_l1_sa = {16, 16};
        }
        c->hme_l2_sa = {16, 16};
        sa(c->me_sa, 8, 8, 8, 8);
        break;
    case 3:
        sa(c->hme_l0_sa, 8, 8, 8, 8);
        c->hme_l1_sa = {8, 8};
        c->hme_l2_sa = {8, 8};
        sa(c->me_sa, 8, 8, 8, 8);
        break;
    default: // 4
        sa(c->hme_l0_sa, 4, 4, 4, 4);
        c->hme_l1_sa = {8, 8};
        c->hme_l2_sa = {8, 8};
        sa(c->me_sa, 8, 8, 8, 8);
        break;
    }
    if (qp_opt) {
        const int qw = clip3(250, 1000, (int)((8 * qp) - 125));
        c->me_sa.sa_min.width  = (uint16_t)std::max(8, (c->me_sa.sa_min.width * qw) / 1000);
        c->me_sa.sa_min.height = (uint16_t)std::max(8, (c->me_sa.sa_min.height * qw) / 1000);
        c->me_sa.sa_max.width  = (uint16_t)std::max(8, (c->me_sa.sa_max.width * qw) / 1000);
        c->me_sa.sa_max.height = (uint16_t)std::max(8, (c->me_sa.sa_max.height * qw) / 1000);
    }
    c->enable_hme_flag        = 1;
    c->enable_hme_level0_flag = 1;
    c->enable_hme_level1_flag = hme_me_level <= 2 ? 1 : 0;
    c->enable_hme_level2_flag = hme_me_level == 0 ? 1 : 0;
    c->hme_search_method = c->me_search_method = hme_me_level <= 2 ? SVTME_FULL_SAD_SEARCH : SVTME_SUB_SAD_SEARCH;
    // pre-HME, reference pruning, sr adjustment, mv-based area and 8x8 variance: level 0 (off)
    c->prune_ref_if_hme_sad_dev_bigger_than_th = 0xFFFF;
    c->prune_ref_if_me_sad_dev_bigger_than_th  = 0xFFFF;
    c->me_early_exit_th            = hme_me_level <= 1 ? 0 : 64 * 64 * 4;
    c->prev_me_stage_based_exit_th = hme_me_level <= 1 ? 0 : 64 * 64 * 4;
}
