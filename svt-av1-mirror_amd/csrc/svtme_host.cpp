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
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "svtme_device.h"

extern "C" hipError_t svtme_launch_build_full(const void *src, uint32_t src_stride, int w, int h, int ten_bit,
                                              DevPlane dst, int left, int top, int rows, hipStream_t s);
extern "C" hipError_t svtme_launch_copy_words(const void *src, void *dst, uint32_t nwords, hipStream_t s);
extern "C" hipError_t svtme_launch_pack(const svtme_ref_record *d_recs, const svtme_sb_result *d_sb, uint32_t n_sb,
                                        uint32_t R, const svtme_pack_layout *L, void *d_out, hipStream_t s);
extern "C" hipError_t svtme_launch_build_down(DevPlane prev, DevPlane dst, int left, int top, int rows,
                                              hipStream_t s);
extern "C" hipError_t svtme_launch_stages(const DevJob *d_jobs, const DevJob *h_jobs, uint32_t n, hipStream_t s,
                                          hipEvent_t *ev, uint32_t *mask);
extern "C" uint32_t svtme_launch_key(const DevJob *dj);
extern "C" hipError_t svtme_prime_pyramid(void);
extern "C" hipError_t svtme_launch_host_rows(const uint8_t *src, uint32_t src_stride, int w, int h, uint8_t *dst,
                                             uint32_t dst_stride, hipStream_t s);
extern "C" hipError_t svtme_prime_pack(void);
extern "C" hipError_t svtme_prime_stages(void);
extern "C" void svtme_stage_a_list(const svtme_job *job, uint8_t *list, uint32_t *count);
extern "C" void svtme_stage_b_list(const svtme_job *job, uint8_t *list, uint32_t *count);
extern "C" void svtme_stage_a1_list(const svtme_job *job, uint8_t *list, uint32_t *count);
extern "C" uint32_t svtme_fp_parts_paths(const svtme_controls *c, uint32_t paths);
extern "C" void svtme_hme_prepare(DevJob *dj);
extern "C" bool svtme_hme_fused(const svtme_job *job);
extern "C" bool svtme_hme_rt(const svtme_controls *c);

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
    hipEvent_t ready = nullptr;           // end of an asynchronous upload on the upload stream
    uint32_t pending = 0;                 // lanes whose stream has not waited on `ready` yet
    hipEvent_t used[SVTME_LANES] = {};    // end of the last submission of each lane that reads the
                                          // picture (a lane's submission event, not owned)
};

// A submission lane: a stream and the inter-stage scratch of the jobs running
// on it. Submissions on different lanes overlap on the GPU (the next one's
// workgroups fill the CUs while the previous one drains); lane 0's stream is
// the context's stream.
struct Lane {
    hipStream_t s = nullptr;
    static constexpr int kEv = 64;  // submission events, recorded round-robin: one per submission
    hipEvent_t ev[kEv] = {};
    int ev_next        = 0;
    ARes *d_ares    = nullptr; // stage-A results [count][SVTME_A_N]
    size_t ares_cap = 0;
    BState *d_bst   = nullptr; // stage-B state [count]
    size_t bst_cap  = 0;
    unsigned long long *d_keys = nullptr; // wide full-pel argmin keys [count][R][85]
    size_t keys_cap            = 0;
    bool keys_rest             = false; // every key is ~0 (banded jobs accumulate with atomic min)
    CSlot *d_cslot             = nullptr; // [count][R]
    size_t cslot_cap           = 0;
};

// An outstanding packed host-output job (svtme_submit_picture_packed_async):
// its device outputs stay allocated with the ticket slot and are reused by the
// next job that takes the slot after svtme_ticket_wait retired it.
struct Ticket {
    uint64_t id = 0;               // 0: the slot is free
    bool waiting = false;          // a thread is blocked on `done`
    hipEvent_t queued = nullptr;   // the job's turn on its lane (timing: svtme_ticket_wait_timed)
    hipEvent_t launched = nullptr; // end of the job's launches on its lane
    hipEvent_t done = nullptr;     // end of the copy into host memory (download stream)
    void *d_mem = nullptr;         // records | SB results | packed bytes
    size_t d_cap = 0;
};

struct svtme_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t ustream = nullptr; // asynchronous uploads (copy + pyramid build), created on first use
    void *ustaging = nullptr;      // their device staging plane (reused in upload-stream order)
    size_t ustaging_cap = 0;
    std::map<uint64_t, PicBuf> pics;
    // released pictures whose memory queued work may still read: freed (or reused by
    // a picture of the same size) once their upload and last readers have completed
    std::vector<PicBuf> graves;
    // idle picture buffers (released pictures whose readers have run, and those
    // svtme_reserve_pictures made), reused for pictures of the same size: no
    // hipMalloc / hipFree on the steady path
    std::vector<std::pair<size_t, uint8_t *>> freebufs;
    static constexpr size_t kMaxFree = 256;
    // page-locked staging of svtme_picture_upload_copy_async, reused in rotation
    struct UpSlot {
        void *h = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr; // the slot's last DMA has run
        bool busy = false;         // a thread is filling it
        bool queued = false;       // `done` marks a DMA
    };
    UpSlot up[SVTME_UPLOAD_SLOTS];
    uint32_t up_next = 0;
    void *staging      = nullptr;
    size_t staging_cap = 0;
    svtme_ref_record *d_records = nullptr;
    size_t records_cap          = 0;
    svtme_sb_result *d_sb       = nullptr;
    size_t sb_cap               = 0;
    uint32_t last_count = 0, last_R = 0;
    bool last_has_sb    = false;
    // job tables: a ring of device slots of SVTME_MAX_BATCH DevJobs, copied from
    // pinned host memory on the job stream (in order: a slot is only rewritten
    // after every kernel queued before has read it); a table identical to the
    // last one published is reused without a copy
    static constexpr int kRing = 16;
    DevJob *d_table = nullptr, *h_table = nullptr, *h_table_dev = nullptr;
    hipEvent_t ring_copied[kRing] = {}; // the copy out of the pinned slot has run
    hipEvent_t ring_read[kRing] = {};   // end of the last submission that read the slot (not owned)
    bool ring_used[kRing] = {};
    uint32_t ring_n[kRing] = {};
    int ring_next = 0;
    // timing: start/stop events of every stage launch of every launch group
    // while enabled (attached to the dispatch packets: hipExtLaunchKernelGGL)
    static constexpr int kTimeSets = 256;
    bool timing = false;
    // uploads from page-locked host memory build the pyramid from the host plane itself
    // over PCIe (no DMA into a staging plane); SVTME_UPLOAD_ZERO_COPY=0: DMA + build
    bool zero_copy = true;
    hipEvent_t tev[kTimeSets][10] = {};
    uint32_t tmask[kTimeSets] = {};
    int t_pending = 0;
    uint32_t t_dropped = 0;
    Lane lanes[SVTME_LANES]; // lanes[0].s == stream
    uint32_t paths = 0;      // SVTME_PATH_* (svtme_set_paths; the environment at creation)
    Ticket tickets[SVTME_MAX_TICKETS];
    uint64_t ticket_seq = 0;
    hipStream_t dstream = nullptr; // packed outputs to host memory, created on first use
    std::mutex mu;
    std::condition_variable retired; // a ticket was retired (svtme_ticket_wait)
    std::condition_variable up_free; // a staging slot of svtme_picture_upload_copy_async was released
};

extern "C" uint32_t svtme_sb_total(uint32_t width, uint32_t height) {
    return ((width + 63) / 64) * ((height + 63) / 64);
}

extern "C" uint32_t svtme_job_ref_slots(const svtme_job *job) {
    return job->num_refs[0] + (job->num_lists == 2 ? job->num_refs[1] : 0);
}

static svtme_status prepare(svtme_ctx *c);

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
    c->lanes[0].s = c->stream;
    // the code objects of the kernels, loaded now rather than at a first job's launches
    if ((e = svtme_prime_pyramid()) != hipSuccess || (e = svtme_prime_pack()) != hipSuccess ||
        (e = svtme_prime_stages()) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fail(SVTME_ERR_UNDEFINED, "svtme_ctx_create: loading the kernels: %s", hipGetErrorString(e));
    }
    // kernel-path selection from the environment, read once (diagnostic A/B runs)
    static const struct {
        const char *var;
        uint32_t bit;
    } env_paths[] = {{"SVTME_NO_FUSED_HME", SVTME_PATH_NO_FUSED_HME}, {"SVTME_NO_L1_FULL", SVTME_PATH_NO_L1_FULL},
                     {"SVTME_NO_L0_FULL", SVTME_PATH_NO_L0_FULL},       {"SVTME_NO_FP_WIDE", SVTME_PATH_NO_FP_WIDE},
                     {"SVTME_SPLIT_PASS", SVTME_PATH_SPLIT_PASS},     {"SVTME_NO_A1_GATE", SVTME_PATH_NO_A1_GATE}};
    for (const auto &e : env_paths)
        if (const char *v = getenv(e.var))
            if (*v && strcmp(v, "0") != 0)
                c->paths |= e.bit;
    if (const char *v = getenv("SVTME_UPLOAD_ZERO_COPY"))
        c->zero_copy = !(*v && strcmp(v, "0") == 0);
    const svtme_status ps = prepare(c);
    if (ps) {
        svtme_ctx_destroy(c);
        return ps;
    }
    *out = c;
    return SVTME_OK;
}

extern "C" svtme_status svtme_set_paths(svtme_ctx *c, uint32_t paths) {
    if (!c || (paths & ~63u))
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_set_paths: null ctx or unknown path bits 0x%x", paths);
    std::lock_guard<std::mutex> lk(c->mu);
    c->paths = paths;
    return SVTME_OK;
}

extern "C" void svtme_ctx_destroy(svtme_ctx *c) {
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    for (auto &L : c->lanes)
        if (L.s)
            (void)hipStreamSynchronize(L.s);
    if (c->ustream)
        (void)hipStreamSynchronize(c->ustream);
    for (auto &kv : c->pics) {
        (void)hipFree(kv.second.mem);
        if (kv.second.ready)
            (void)hipEventDestroy(kv.second.ready);
    }
    for (auto &g : c->graves) {
        (void)hipFree(g.mem);
        if (g.ready)
            (void)hipEventDestroy(g.ready);
    }
    for (auto &f : c->freebufs)
        (void)hipFree(f.second);
    for (auto &u : c->up) {
        if (u.h)
            (void)hipHostFree(u.h);
        if (u.done)
            (void)hipEventDestroy(u.done);
    }
    if (c->staging)
        (void)hipFree(c->staging);
    if (c->ustaging)
        (void)hipFree(c->ustaging);
    if (c->d_records)
        (void)hipFree(c->d_records);
    if (c->d_sb)
        (void)hipFree(c->d_sb);
    for (auto &set : c->tev)
        for (auto &e : set)
            if (e)
                (void)hipEventDestroy(e);
    for (int k = 0; k < svtme_ctx::kRing; k++)
        if (c->ring_copied[k])
            (void)hipEventDestroy(c->ring_copied[k]);
    if (c->dstream)
        (void)hipStreamSynchronize(c->dstream);
    for (auto &t : c->tickets) {
        if (t.d_mem)
            (void)hipFree(t.d_mem);
        if (t.launched)
            (void)hipEventDestroy(t.launched);
        if (t.queued)
            (void)hipEventDestroy(t.queued);
        if (t.done)
            (void)hipEventDestroy(t.done);
    }
    if (c->dstream)
        (void)hipStreamDestroy(c->dstream);
    if (c->d_table)
        (void)hipFree(c->d_table);
    if (c->h_table)
        (void)hipHostFree(c->h_table);
    for (int l = 0; l < SVTME_LANES; l++) {
        Lane &L = c->lanes[l];
        if (L.d_ares)
            (void)hipFree(L.d_ares);
        if (L.d_bst)
            (void)hipFree(L.d_bst);
        if (L.d_keys)
            (void)hipFree(L.d_keys);
        if (L.d_cslot)
            (void)hipFree(L.d_cslot);
        for (auto &e : L.ev)
            if (e)
                (void)hipEventDestroy(e);
        if (l > 0 && L.s)
            (void)hipStreamDestroy(L.s);
    }
    (void)hipStreamDestroy(c->stream);
    if (c->ustream)
        (void)hipStreamDestroy(c->ustream);
    delete c;
}

// lane `lane`'s stream waits for a picture's asynchronous upload (once per upload)
static svtme_status join_upload(svtme_ctx *c, PicBuf &pb, int lane) {
    if ((pb.pending >> lane) & 1u) {
        HIP_TRY(hipStreamWaitEvent(c->lanes[lane].s, pb.ready, 0));
        pb.pending &= ~(1u << lane);
    }
    return SVTME_OK;
}
// `s` waits for every launch of the other lanes already queued that reads the picture
static svtme_status after_readers(svtme_ctx *c, PicBuf &pb, hipStream_t s) {
    for (int l = 0; l < SVTME_LANES; l++)
        if (pb.used[l] && c->lanes[l].s != s)
            HIP_TRY(hipStreamWaitEvent(s, pb.used[l], 0));
    return SVTME_OK;
}
// no stream still uses the picture's memory
static svtme_status quiesce(svtme_ctx *c) {
    for (auto &L : c->lanes)
        if (L.s)
            HIP_TRY(hipStreamSynchronize(L.s));
    if (c->ustream)
        HIP_TRY(hipStreamSynchronize(c->ustream));
    return SVTME_OK;
}
static svtme_status ensure_lane(svtme_ctx *c, uint32_t lane) {
    if (lane >= SVTME_LANES)
        return fail(SVTME_ERR_BAD_PARAMETER, "lane %u (0..%d)", lane, SVTME_LANES - 1);
    Lane &L = c->lanes[lane];
    if (!L.s)
        HIP_TRY(hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking));
    if (!L.ev[0])
        for (auto &e : L.ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return SVTME_OK;
}

extern "C" void *svtme_stream(svtme_ctx *c) { return c ? (void *)c->stream : nullptr; }

extern "C" void *svtme_lane_stream(svtme_ctx *c, uint32_t lane) {
    if (!c)
        return nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    if (hipSetDevice(c->device) != hipSuccess || ensure_lane(c, lane))
        return nullptr;
    return (void *)c->lanes[lane].s;
}

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

// a released picture's memory is idle: its upload and its lanes' last readers have run
// (a lane's event may since mark a later submission: later, never early)
static bool grave_idle(const PicBuf &g) {
    if (g.ready && hipEventQuery(g.ready) != hipSuccess)
        return false;
    for (int l = 0; l < SVTME_LANES; l++)
        if (g.used[l] && hipEventQuery(g.used[l]) != hipSuccess)
            return false;
    return true;
}
// an idle buffer of exactly `bytes` from the free pool, or nullptr
static uint8_t *take_free(svtme_ctx *c, size_t bytes) {
    for (size_t i = 0; i < c->freebufs.size(); i++)
        if (c->freebufs[i].first == bytes) {
            uint8_t *m     = c->freebufs[i].second;
            c->freebufs[i] = c->freebufs.back();
            c->freebufs.pop_back();
            return m;
        }
    return nullptr;
}
// move the idle released pictures' memory to the free pool (beyond kMaxFree
// buffers it goes back to HIP); with want > 0, return one idle buffer of
// exactly `want` bytes instead
static uint8_t *sweep_graves(svtme_ctx *c, size_t want) {
    uint8_t *keep = nullptr;
    for (size_t i = 0; i < c->graves.size();) {
        PicBuf &g = c->graves[i];
        if (!grave_idle(g)) {
            i++;
            continue;
        }
        if (g.ready)
            (void)hipEventDestroy(g.ready);
        if (!keep && want && g.bytes == want)
            keep = g.mem;
        else if (c->freebufs.size() < svtme_ctx::kMaxFree)
            c->freebufs.emplace_back(g.bytes, g.mem);
        else
            (void)hipFree(g.mem);
        c->graves[i] = c->graves.back();
        c->graves.pop_back();
    }
    return keep;
}

// bytes of a W x H picture's three padded planes in one buffer, and their offsets
static size_t pic_bytes(uint32_t W, uint32_t H, size_t offs[3] = nullptr) {
    size_t total = 0;
    for (int lv = 0; lv < 3; lv++) {
        uint32_t w, h, left, top, stride, rows, pad;
        svtme_plane_geometry(lv, W, H, &w, &h, &left, &top, &stride, &rows, &pad);
        if (offs)
            offs[lv] = total;
        total += (size_t)stride * rows;
        total = (total + 255) & ~(size_t)255;
    }
    return total + 1024; // slack: search-window loads may read a few dwords past the last row
}

// device memory for a picture: the free pool, an idle released picture, or HIP;
// when HIP is out of memory, wait for the released pictures' readers, give every
// idle buffer back and try once more
static svtme_status pic_mem(svtme_ctx *c, size_t total, uint8_t **out) {
    if ((*out = take_free(c, total)) || (*out = sweep_graves(c, total)))
        return SVTME_OK;
    if (hipMalloc((void **)out, total) == hipSuccess)
        return SVTME_OK;
    (void)hipGetLastError();
    for (auto &g : c->graves) {
        if (g.ready)
            HIP_TRY(hipEventSynchronize(g.ready));
        for (int l = 0; l < SVTME_LANES; l++)
            if (g.used[l])
                HIP_TRY(hipEventSynchronize(g.used[l]));
    }
    (void)sweep_graves(c, 0);
    for (auto &f : c->freebufs)
        HIP_TRY(hipFree(f.second));
    c->freebufs.clear();
    HIP_TRY(hipMalloc((void **)out, total));
    return SVTME_OK;
}

// allocate the three planes of a W x H picture in one buffer
static svtme_status alloc_pic(svtme_ctx *c, uint64_t pn, uint32_t W, uint32_t H, PicBuf **out) {
    auto it = c->pics.find(pn);
    if (it != c->pics.end() && (it->second.W != W || it->second.H != H)) {
        // a new size: the old buffer goes to the graves (freed for reuse once its readers ran)
        c->graves.push_back(it->second);
        c->pics.erase(it);
        it = c->pics.end();
    }
    size_t offs[3];
    const size_t total = pic_bytes(W, H, offs);
    uint32_t w[3], h[3], left[3], top[3], stride[3], rows[3], pad[3];
    for (int lv = 0; lv < 3; lv++)
        svtme_plane_geometry(lv, W, H, &w[lv], &h[lv], &left[lv], &top[lv], &stride[lv], &rows[lv], &pad[lv]);
    if (it == c->pics.end()) {
        PicBuf pb;
        svtme_status ms = pic_mem(c, total, &pb.mem);
        if (ms)
            return ms;
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
                                  uint32_t h, int ten_bit, hipStream_t st = nullptr) {
    if (!st)
        st = c->stream;
    uint32_t pw, ph, left, top, stride, rows, pad;
    svtme_plane_geometry(0, pb->W, pb->H, &pw, &ph, &left, &top, &stride, &rows, &pad);
    HIP_TRY(svtme_launch_build_full(dsrc, src_stride, (int)w, (int)h, ten_bit, pb->pyr.lv[0], (int)left, (int)top,
                                    (int)rows, st));
    for (int lv = 1; lv < 3; lv++) {
        svtme_plane_geometry(lv, pb->W, pb->H, &pw, &ph, &left, &top, &stride, &rows, &pad);
        HIP_TRY(svtme_launch_build_down(pb->pyr.lv[lv - 1], pb->pyr.lv[lv], (int)left, (int)top, (int)rows, st));
    }
    return SVTME_OK;
}

// The device address of a page-locked host range (hipHostMalloc / hipHostRegister),
// or null for pageable memory (then a DMA through a staging plane is needed)
static const uint8_t *device_view(const svtme_ctx *c, const void *y) {
    if (!c->zero_copy)
        return nullptr;
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, y) != hipSuccess) {
        (void)hipGetLastError(); // (pageable memory reads as an error)
        return nullptr;
    }
    if (pa.type != hipMemoryTypeHost || !pa.devicePointer)
        return nullptr;
    return (const uint8_t *)pa.devicePointer + (pa.hostPointer ? ((const uint8_t *)y - (const uint8_t *)pa.hostPointer) : 0);
}

// the pyramid of an 8-bit plane the device reads in page-locked host memory: the
// interior of level 0 streamed over PCIe by a few workgroups (svtme_launch_host_rows),
// then the padding and the lower levels from it, on device
static svtme_status build_pyramid_host(svtme_ctx *c, PicBuf *pb, const uint8_t *dv, uint32_t stride, uint32_t w,
                                       uint32_t h, hipStream_t st) {
    const DevPlane &p0 = pb->pyr.lv[0];
    HIP_TRY(svtme_launch_host_rows(dv, stride, (int)w, (int)h, p0.base, (uint32_t)p0.stride, st));
    return build_pyramid(c, pb, p0.base, (uint32_t)p0.stride, w, h, 0, st);
}
// zero-copy needs dword-aligned rows (the stream kernel's loads and stores)
static bool zero_copy_ok(const void *y, uint32_t stride, const PicBuf *pb) {
    return (((uintptr_t)y | stride | (uintptr_t)pb->pyr.lv[0].base | (uint32_t)pb->pyr.lv[0].stride) & 3) == 0;
}

static svtme_status upload_host(svtme_ctx *c, uint64_t pn, const void *y, uint32_t stride, uint32_t w, uint32_t h,
                                int ten_bit) {
    if (!c || !y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t bpp = ten_bit ? 2 : 1;
    const uint8_t *dv  = ten_bit ? nullptr : device_view(c, y); // page-locked: read in place
    svtme_status st;
    PicBuf *pb;
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    if (dv && !zero_copy_ok(y, stride, pb))
        dv = nullptr;
    if (!dv) {
        if ((st = ensure_buf(&c->staging, &c->staging_cap, (size_t)w * h * bpp)))
            return st;
        HIP_TRY(hipMemcpy2DAsync(c->staging, (size_t)w * bpp, y, (size_t)stride * bpp, (size_t)w * bpp, h,
                                 hipMemcpyHostToDevice, c->stream));
    }
    if ((st = join_upload(c, *pb, 0)) || (st = after_readers(c, *pb, c->stream)))
        return st;
    if ((st = dv ? build_pyramid_host(c, pb, dv, stride, w, h, c->stream)
                 : build_pyramid(c, pb, c->staging, w, w, h, ten_bit)))
        return st;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

// Asynchronous 8-bit upload: one linear DMA of the rows into a device staging
// plane on the upload stream (a pitched copy straight into the padded plane
// runs as a slow blit), which then builds the padded pyramid from it; the
// first job that reads the picture waits for it on the job stream. Jobs
// already queued that read an earlier version of the picture finish before
// its planes are rewritten.
static svtme_status ensure_ustream(svtme_ctx *c) {
    if (!c->ustream) { // high priority: its small pyramid kernels go ahead of queued search workgroups
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, hi));
    }
    return SVTME_OK;
}

extern "C" void *svtme_upload_stream(svtme_ctx *c) {
    if (!c)
        return nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    if (hipSetDevice(c->device) != hipSuccess || ensure_ustream(c))
        return nullptr;
    return (void *)c->ustream;
}

// Device-resident form of svtme_picture_upload_async: the pyramid is built from
// d_y on the upload stream (the caller orders d_y's producer before it, e.g. an
// RCCL broadcast of the plane, and keeps d_y until the build has run).
extern "C" svtme_status svtme_picture_upload_device_async(svtme_ctx *c, uint64_t pn, const uint8_t *d_y,
                                                          uint32_t stride, uint32_t w, uint32_t h) {
    if (!c || !d_y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload_device_async: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    svtme_status st;
    if ((st = ensure_ustream(c)))
        return st;
    const bool resident = c->pics.count(pn) != 0;
    PicBuf *pb;
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    if (resident && (st = after_readers(c, *pb, c->ustream))) // queued jobs may still read the old planes
        return st;
    if (!pb->ready)
        HIP_TRY(hipEventCreateWithFlags(&pb->ready, hipEventDisableTiming));
    if ((st = build_pyramid(c, pb, d_y, stride, w, h, 0, c->ustream)))
        return st;
    HIP_TRY(hipEventRecord(pb->ready, c->ustream));
    pb->pending = (1u << SVTME_LANES) - 1u;
    return SVTME_OK;
}

extern "C" svtme_status svtme_picture_upload_async(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride,
                                                   uint32_t w, uint32_t h) {
    if (!c || !y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload_async: bad arguments");
    // SVTME_SLOW_UPLOAD_MS=t: a call over t ms prints where its time went (stderr)
    static const double slow_ms = getenv("SVTME_SLOW_UPLOAD_MS") ? atof(getenv("SVTME_SLOW_UPLOAD_MS")) : 0.0;
    using clk     = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::lock_guard<std::mutex> lk(c->mu);
    const auto t1 = clk::now();
    HIP_TRY(hipSetDevice(c->device));
    {
        const svtme_status us = ensure_ustream(c);
        if (us)
            return us;
    }
    const bool resident = c->pics.count(pn) != 0;
    PicBuf *pb;
    svtme_status st;
    const size_t nfree = c->freebufs.size();
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    const auto t2 = clk::now();
    if (resident && (st = after_readers(c, *pb, c->ustream))) // queued jobs may still read the old planes
        return st;
    struct SlowLog {
        double lim;
        std::chrono::steady_clock::time_point t0, t1, t2;
        uint64_t pn;
        size_t nfree;
        bool resident;
        ~SlowLog() {
            if (lim <= 0.0)
                return;
            const auto t3 = std::chrono::steady_clock::now();
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            if (ms(t0, t3) > lim)
                fprintf(stderr, "[svtme] slow upload pn %llu: %.3f ms (lock %.3f, alloc %.3f, rest %.3f; free bufs %zu, %s)\n",
                        (unsigned long long)pn, ms(t0, t3), ms(t0, t1), ms(t1, t2), ms(t2, t3), nfree,
                        resident ? "resident" : "new");
        }
    } slow_log{slow_ms, t0, t1, t2, pn, nfree, resident};
    if (!pb->ready)
        HIP_TRY(hipEventCreateWithFlags(&pb->ready, hipEventDisableTiming));
    // a page-locked plane the device can read: the pyramid build reads it over PCIe
    // itself (no DMA into a staging plane, no second pass over it)
    const uint8_t *dy = device_view(c, y);
    if (dy && zero_copy_ok(y, stride, pb)) {
        if ((st = build_pyramid_host(c, pb, dy, stride, w, h, c->ustream)))
            return st;
        HIP_TRY(hipEventRecord(pb->ready, c->ustream));
        pb->pending = (1u << SVTME_LANES) - 1u;
        return SVTME_OK;
    }
    // one linear copy of the span from the first to the last sample (rows keep their
    // stride; a padded encoder plane's margins ride along): a 2D copy out of
    // pageable memory goes row by row
    const size_t need = (size_t)(h - 1) * stride + w;
    if (c->ustaging_cap < need) { // only between uploads: nothing queued reads the old buffer
        HIP_TRY(hipStreamSynchronize(c->ustream));
        if ((st = ensure_buf(&c->ustaging, &c->ustaging_cap, need)))
            return st;
    }
    HIP_TRY(hipMemcpyAsync(c->ustaging, y, need, hipMemcpyHostToDevice, c->ustream));
    if ((st = build_pyramid(c, pb, c->ustaging, stride, w, h, 0, c->ustream)))
        return st;
    HIP_TRY(hipEventRecord(pb->ready, c->ustream));
    pb->pending = (1u << SVTME_LANES) - 1u;
    return SVTME_OK;
}

// Upload from pageable memory through the context's page-locked staging ring:
// take a slot (wait for its last DMA), copy the rows into it with no lock held,
// then queue the DMA and the pyramid build like svtme_picture_upload_async.
extern "C" svtme_status svtme_picture_upload_copy_async(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride,
                                                        uint32_t w, uint32_t h) {
    if (!c || !y || w == 0 || h == 0 || stride < w)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload_copy_async: bad arguments");
    svtme_ctx::UpSlot *u = nullptr;
    {
        std::unique_lock<std::mutex> lk(c->mu);
        HIP_TRY(hipSetDevice(c->device));
        const svtme_status us = ensure_ustream(c);
        if (us)
            return us;
        // every slot being filled by other threads: wait for one (each is released
        // once its rows are staged and its DMA queued, a bounded time)
        c->up_free.wait(lk, [&] {
            for (int k = 0; k < SVTME_UPLOAD_SLOTS && !u; k++) {
                svtme_ctx::UpSlot &x = c->up[(c->up_next + k) % SVTME_UPLOAD_SLOTS];
                if (!x.busy)
                    u = &x;
            }
            return u != nullptr;
        });
        c->up_next = (uint32_t)(u - c->up + 1) % SVTME_UPLOAD_SLOTS;
        u->busy    = true;
        if (!u->done)
            HIP_TRY(hipEventCreateWithFlags(&u->done, hipEventDisableTiming));
    }
    // outside the context lock: other threads submit jobs meanwhile
    const size_t need = (size_t)w * h;
    hipError_t e      = hipSetDevice(c->device);
    if (e == hipSuccess && u->queued)
        e = hipEventSynchronize(u->done); // the slot's previous DMA has read it
    if (e == hipSuccess && u->cap < need) {
        if (u->h)
            e = hipHostFree(u->h);
        u->h   = nullptr;
        u->cap = 0;
        if (e == hipSuccess && (e = hipHostMalloc(&u->h, need, hipHostMallocDefault)) == hipSuccess)
            u->cap = need;
    }
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(c->mu);
        u->busy = false;
        c->up_free.notify_all();
        return fail(SVTME_ERR_INSUFFICIENT_RESOURCES, "svtme_picture_upload_copy_async: staging: %s",
                    hipGetErrorString(e));
    }
    for (uint32_t r = 0; r < h; r++)
        memcpy((uint8_t *)u->h + (size_t)r * w, y + (size_t)r * stride, w);
    std::lock_guard<std::mutex> lk(c->mu);
    struct Release { // the slot is free again however this returns (c->mu held)
        svtme_ctx *c;
        svtme_ctx::UpSlot *u;
        ~Release() {
            u->busy = false;
            c->up_free.notify_all();
        }
    } rel{c, u};
    const bool resident = c->pics.count(pn) != 0;
    PicBuf *pb;
    svtme_status st;
    if ((st = alloc_pic(c, pn, svtme_align8_u(w), svtme_align8_u(h), &pb)))
        return st;
    if (resident && (st = after_readers(c, *pb, c->ustream))) // queued jobs may still read the old planes
        return st;
    if (!pb->ready)
        HIP_TRY(hipEventCreateWithFlags(&pb->ready, hipEventDisableTiming));
    if (c->ustaging_cap < need) { // only between uploads: nothing queued reads the old buffer
        HIP_TRY(hipStreamSynchronize(c->ustream));
        if ((st = ensure_buf(&c->ustaging, &c->ustaging_cap, need)))
            return st;
    }
    HIP_TRY(hipMemcpyAsync(c->ustaging, u->h, need, hipMemcpyHostToDevice, c->ustream));
    HIP_TRY(hipEventRecord(u->done, c->ustream));
    u->queued = true;
    if ((st = build_pyramid(c, pb, c->ustaging, w, w, h, 0, c->ustream)))
        return st;
    HIP_TRY(hipEventRecord(pb->ready, c->ustream));
    pb->pending = (1u << SVTME_LANES) - 1u;
    return SVTME_OK;
}

extern "C" svtme_status svtme_reserve_pictures(svtme_ctx *c, uint32_t width, uint32_t height, uint32_t count) {
    if (!c || width == 0 || height == 0 || count > 4096)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_reserve_pictures: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = pic_bytes(svtme_align8_u(width), svtme_align8_u(height));
    uint32_t have      = 0;
    for (auto &f : c->freebufs)
        have += f.first == bytes;
    for (; have < count && c->freebufs.size() < svtme_ctx::kMaxFree; have++) {
        uint8_t *m = nullptr;
        HIP_TRY(hipMalloc((void **)&m, bytes));
        c->freebufs.emplace_back(bytes, m);
    }
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
    if ((st = join_upload(c, *pb, 0)) || (st = after_readers(c, *pb, c->stream)))
        return st;
    if ((st = build_pyramid(c, pb, d_y, stride, w, h, 0)))
        return st;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVTME_OK;
}

extern "C" svtme_status svtme_picture_invalidate(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride,
                                                 uint32_t w, uint32_t h) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_invalidate: null ctx");
    {
        std::lock_guard<std::mutex> lk(c->mu);
        auto it = c->pics.find(pn);
        if (it == c->pics.end())
            return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_invalidate: picture %llu not resident",
                        (unsigned long long)pn);
        if (it->second.W != svtme_align8_u(w) || it->second.H != svtme_align8_u(h))
            return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_invalidate: picture %llu is %ux%u, new planes %ux%u",
                        (unsigned long long)pn, it->second.W, it->second.H, w, h);
    }
    // same stream as the jobs: the rebuild runs after every job already queued
    return upload_host(c, pn, y, stride, w, h, 0);
}

extern "C" svtme_status svtme_picture_release(svtme_ctx *c, uint64_t pn) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_release: null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->pics.find(pn);
    if (it == c->pics.end())
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_release: picture %llu not resident",
                    (unsigned long long)pn);
    HIP_TRY(hipSetDevice(c->device));
    // no device-wide wait: the memory goes to the graves until the work queued
    // before the release (its upload, the lanes' readers) has run
    c->graves.push_back(it->second);
    c->pics.erase(it);
    (void)sweep_graves(c, 0);
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
    svtme_status qs = quiesce(c);
    if (qs)
        return qs;
    HIP_TRY(hipMemcpy2D(dst, S, p.base - (ptrdiff_t)p.pad * p.stride - p.pad, (size_t)p.stride, S,
                        (size_t)(p.height + 2 * p.pad), hipMemcpyDeviceToHost));
    return SVTME_OK;
}

// ----------------------------------------------------------------------------
// jobs
// ----------------------------------------------------------------------------
static svtme_status validate_job(svtme_ctx *c, const svtme_job *job, DevJob *dj, uint32_t *count, int lane) {
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
        svtme_status js = join_upload(c, it->second, lane);
        if (js)
            return js;
        *out = it->second.pyr;
        return SVTME_OK;
    };
    memset(dj, 0, sizeof(*dj));
    dj->job   = *job;
    dj->paths = c->paths;
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

static svtme_status ensure_ring(svtme_ctx *c) {
    if (c->d_table)
        return SVTME_OK;
    const size_t bytes = sizeof(DevJob) * SVTME_MAX_BATCH * svtme_ctx::kRing;
    HIP_TRY(hipMalloc((void **)&c->d_table, bytes));
    HIP_TRY(hipHostMalloc((void **)&c->h_table, bytes, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void **)&c->h_table_dev, c->h_table, 0)); // read by k_copy_words
    for (int k = 0; k < svtme_ctx::kRing; k++)
        HIP_TRY(hipEventCreateWithFlags(&c->ring_copied[k], hipEventDisableTiming));
    return SVTME_OK;
}

// The streams, events and job-table ring of a context, made at creation so
// that no job's latency carries them
static svtme_status prepare(svtme_ctx *c) {
    svtme_status st;
    for (uint32_t l = 0; l < SVTME_LANES; l++)
        if ((st = ensure_lane(c, l)))
            return st;
    if ((st = ensure_ustream(c)) || (st = ensure_ring(c)))
        return st;
    HIP_TRY(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
    for (auto &t : c->tickets) { // timing events: svtme_ticket_wait_timed
        HIP_TRY(hipEventCreate(&t.queued));
        HIP_TRY(hipEventCreate(&t.launched));
        HIP_TRY(hipEventCreate(&t.done));
    }
    // The first work on a stream and the first large copy in each direction cost
    // milliseconds of one-time runtime setup (the first packed job's D2H copy call
    // took 6.8 ms in a HIP API trace, later ones 10 us; small copies take another
    // path and do not set it up): a fill on every stream and a 4 MB copy each way
    // on the upload and download streams happen here, at context creation.
    void *d = nullptr, *h = nullptr;
    const size_t wb = (size_t)4 << 20;
    HIP_TRY(hipMalloc(&d, wb));
    HIP_TRY(hipHostMalloc(&h, wb, hipHostMallocDefault));
    for (uint32_t l = 0; l < SVTME_LANES; l++) HIP_TRY(hipMemsetAsync(d, 0, 256, c->lanes[l].s));
    HIP_TRY(hipMemsetAsync(d, 0, 256, c->ustream));
    HIP_TRY(hipMemcpyAsync(d, h, wb, hipMemcpyHostToDevice, c->ustream));
    HIP_TRY(hipStreamSynchronize(c->ustream));
    HIP_TRY(hipMemcpyAsync(h, d, wb, hipMemcpyDeviceToHost, c->dstream));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(d));
    HIP_TRY(hipHostFree(h));
    return SVTME_OK;
}

// Validate, lay out and launch n jobs. out[k] / out_sb[k]: device outputs of
// job k; null out => the context's own record buffer (single job only).
static svtme_status submit_batch_locked(svtme_ctx *c, const svtme_job *jobs, uint32_t n,
                                        svtme_ref_record *const *out, svtme_sb_result *const *out_sb,
                                        bool with_sb, uint32_t lane = 0) {
    HIP_TRY(hipSetDevice(c->device));
    svtme_status st;
    if ((st = ensure_lane(c, lane)))
        return st;
    Lane &L = c->lanes[lane];
    if (!out && lane != 0)
        return fail(SVTME_ERR_BAD_PARAMETER, "context-owned outputs are lane 0's");
    if (n == 0 || n > SVTME_MAX_BATCH)
        return fail(SVTME_ERR_BAD_PARAMETER, "batch of %u jobs (1..%d)", n, SVTME_MAX_BATCH);
    DevJob hj[SVTME_MAX_BATCH];
    uint32_t count[SVTME_MAX_BATCH];
    size_t sbs = 0, slots = 0;
    for (uint32_t k = 0; k < n; k++) {
        if ((st = validate_job(c, &jobs[k], &hj[k], &count[k], (int)lane)))
            return st;
        sbs += count[k];
        slots += (size_t)count[k] * hj[k].R;
    }
    if (!out && n != 1)
        return fail(SVTME_ERR_BAD_PARAMETER, "context-owned outputs hold one job");
    if (out) {
        for (uint32_t k = 0; k < n; k++) {
            if (!out[k])
                return fail(SVTME_ERR_BAD_PARAMETER, "null record buffer for job %u", k);
            hj[k].out_records = out[k];
            hj[k].out_sb      = out_sb ? out_sb[k] : nullptr;
        }
    } else {
        if ((st = ensure_buf((void **)&c->d_records, &c->records_cap, slots * sizeof(svtme_ref_record))))
            return st;
        hj[0].out_records = c->d_records;
        if (with_sb) {
            if ((st = ensure_buf((void **)&c->d_sb, &c->sb_cap, sbs * sizeof(svtme_sb_result))))
                return st;
            hj[0].out_sb = c->d_sb;
        }
    }
    // inter-stage scratch of the whole batch, per-job offsets
    // a lane's scratch grows only between its submissions: the old buffers are idle
    if (L.ares_cap < sbs * SVTME_A_N * sizeof(ARes) || L.bst_cap < sbs * sizeof(BState))
        HIP_TRY(hipStreamSynchronize(L.s));
    if ((st = ensure_buf((void **)&L.d_ares, &L.ares_cap, sbs * SVTME_A_N * sizeof(ARes))))
        return st;
    if ((st = ensure_buf((void **)&L.d_bst, &L.bst_cap, sbs * sizeof(BState))))
        return st;
    bool any_banded = false, any_single = false, any_wide = false;
    for (uint32_t k = 0; k < n; k++) {
        hj[k].parts = svtme_fp_parts_paths(&hj[k].job.ctrl, hj[k].paths);
        any_wide |= hj[k].parts != 0;
        any_banded |= hj[k].parts > 1;
        any_single |= hj[k].parts == 1;
    }
    if (any_wide) { // wide full-pel stage (k_stage_c1 + k_stage_e)
        const size_t kb = slots * SVTME_PU_COUNT * sizeof(unsigned long long);
        if (L.keys_cap < kb || L.cslot_cap < slots * sizeof(CSlot))
            HIP_TRY(hipStreamSynchronize(L.s));
        if (L.keys_cap < kb) {
            if ((st = ensure_buf((void **)&L.d_keys, &L.keys_cap, kb)))
                return st;
            L.keys_rest = false;
        }
        if ((st = ensure_buf((void **)&L.d_cslot, &L.cslot_cap, slots * sizeof(CSlot))))
            return st;
        // banded jobs merge with atomic min into keys that must all be ~0; k_stage_e
        // resets what it consumed, plain-store (single band) jobs leave keys behind
        if (any_banded && !L.keys_rest)
            HIP_TRY(hipMemsetAsync(L.d_keys, 0xFF, L.keys_cap, L.s));
        L.keys_rest = !any_single;
    }
    size_t sb_off = 0, slot_off = 0;
    for (uint32_t k = 0; k < n; k++) {
        hj[k].ares  = L.d_ares + sb_off * SVTME_A_N;
        hj[k].bst   = L.d_bst + sb_off;
        hj[k].keys  = hj[k].parts ? L.d_keys + slot_off * SVTME_PU_COUNT : nullptr;
        hj[k].cslot = hj[k].parts ? L.d_cslot + slot_off : nullptr;
        svtme_stage_a_list(&hj[k].job, hj[k].ta_list, &hj[k].ta_count);
        svtme_stage_a1_list(&hj[k].job, hj[k].ta1_list, &hj[k].ta1_count);
        svtme_stage_b_list(&hj[k].job, hj[k].tb_list, &hj[k].tb_count);
        svtme_hme_prepare(&hj[k]);
        sb_off += count[k];
        slot_off += (size_t)count[k] * hj[k].R;
    }
    // group by kernel variant (stable), publish the table, launch each group
    DevJob ordered[SVTME_MAX_BATCH];
    uint32_t keys[SVTME_MAX_BATCH], m = 0;
    for (uint32_t k = 0; k < n; k++) keys[k] = svtme_launch_key(&hj[k]);
    bool taken[SVTME_MAX_BATCH] = {};
    uint32_t group_start[SVTME_MAX_BATCH + 1], groups = 0;
    for (uint32_t k = 0; k < n; k++) {
        if (taken[k])
            continue;
        group_start[groups++] = m;
        for (uint32_t q = k; q < n; q++)
            if (!taken[q] && keys[q] == keys[k]) {
                ordered[m++] = hj[q];
                taken[q]     = true;
            }
    }
    group_start[groups] = m;
    if ((st = ensure_ring(c)))
        return st;
    int slot = -1;
    for (int k = 0; k < svtme_ctx::kRing && slot < 0; k++)
        if (c->ring_used[k] && c->ring_n[k] == n &&
            memcmp(c->h_table + (size_t)k * SVTME_MAX_BATCH, ordered, sizeof(DevJob) * n) == 0)
            slot = k; // already resident (device copy of this exact table)
    if (slot < 0) {
        slot         = c->ring_next;
        c->ring_next = (slot + 1) % svtme_ctx::kRing;
        DevJob *h    = c->h_table + (size_t)slot * SVTME_MAX_BATCH;
        if (c->ring_used[slot]) { // its pinned copy and the launches that read it (any lane) are done
            HIP_TRY(hipEventSynchronize(c->ring_copied[slot]));
            if (c->ring_read[slot])
                HIP_TRY(hipEventSynchronize(c->ring_read[slot]));
        }
        memcpy(h, ordered, sizeof(DevJob) * n);
        static_assert(sizeof(DevJob) % 4 == 0, "DevJob copied in dwords");
        HIP_TRY(svtme_launch_copy_words(c->h_table_dev + (size_t)slot * SVTME_MAX_BATCH,
                                        c->d_table + (size_t)slot * SVTME_MAX_BATCH,
                                        (uint32_t)(sizeof(DevJob) * n / 4), L.s));
        HIP_TRY(hipEventRecord(c->ring_copied[slot], L.s));
        c->ring_used[slot] = true;
        c->ring_n[slot]    = n;
    }
    DevJob *d = c->d_table + (size_t)slot * SVTME_MAX_BATCH;
    for (uint32_t g = 0; g < groups; g++) {
        hipEvent_t *ev = nullptr;
        uint32_t *mask = nullptr;
        if (c->timing && c->t_pending < svtme_ctx::kTimeSets) {
            ev   = c->tev[c->t_pending];
            mask = &c->tmask[c->t_pending++];
        } else if (c->timing) {
            c->t_dropped++;
        }
        HIP_TRY(svtme_launch_stages(d + group_start[g], ordered + group_start[g], group_start[g + 1] - group_start[g],
                                    L.s, ev, mask));
    }
    // one event per submission: the slot and the pictures it read point at it
    // (a re-upload / rebuild waits for these launches only)
    hipEvent_t done = L.ev[L.ev_next];
    L.ev_next       = (L.ev_next + 1) % Lane::kEv;
    HIP_TRY(hipEventRecord(done, L.s));
    c->ring_read[slot] = done;
    for (uint32_t k = 0; k < n; k++) {
            const svtme_job &j = jobs[k];
            auto mark          = [&](uint64_t pn) -> svtme_status {
                c->pics.find(pn)->second.used[lane] = done; // resident: validate_job checked
                return SVTME_OK;
            };
            if ((st = mark(j.picture_number)))
                return st;
            for (int l = 0; l < j.num_lists; l++)
                for (int r = 0; r < j.num_refs[l]; r++)
                    if ((st = mark(j.ref_picture_number[l][r])))
                        return st;
        }
    // svtme_fetch / svtme_device_records describe the context-owned buffers only:
    // a submission into caller buffers leaves them as they were
    if (!out) {
        c->last_count  = (uint32_t)sbs;
        c->last_R      = hj[0].R;
        c->last_has_sb = with_sb;
    }
    return SVTME_OK;
}

static svtme_status submit_locked(svtme_ctx *c, const svtme_job *job, bool with_sb, svtme_ref_record *d_out,
                                  svtme_sb_result *d_out_sb) {
    if (d_out)
        return submit_batch_locked(c, job, 1, &d_out, &d_out_sb, d_out_sb != nullptr);
    return submit_batch_locked(c, job, 1, nullptr, nullptr, with_sb);
}

extern "C" svtme_status svtme_submit_picture_device(svtme_ctx *c, const svtme_job *job, svtme_ref_record *d_recs,
                                                    svtme_sb_result *d_sb) {
    if (!c || !d_recs)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_picture_device: null ctx or output");
    std::lock_guard<std::mutex> lk(c->mu);
    return submit_locked(c, job, d_sb != nullptr, d_recs, d_sb);
}

extern "C" svtme_status svtme_submit_batch_device(svtme_ctx *c, const svtme_job *jobs, uint32_t n,
                                                  svtme_ref_record *const *d_recs, svtme_sb_result *const *d_sb) {
    if (!c || !jobs || !d_recs)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_batch_device: null ctx, jobs or outputs");
    std::lock_guard<std::mutex> lk(c->mu);
    return submit_batch_locked(c, jobs, n, d_recs, d_sb, d_sb != nullptr);
}

extern "C" svtme_status svtme_submit_batch_device_lane(svtme_ctx *c, uint32_t lane, const svtme_job *jobs,
                                                       uint32_t n, svtme_ref_record *const *d_recs,
                                                       svtme_sb_result *const *d_sb) {
    if (!c || !jobs || !d_recs)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_batch_device_lane: null ctx, jobs or outputs");
    std::lock_guard<std::mutex> lk(c->mu);
    return submit_batch_locked(c, jobs, n, d_recs, d_sb, d_sb != nullptr, lane);
}

// ----------------------------------------------------------------------------
// packed host output, asynchronous (tickets)
// ----------------------------------------------------------------------------
extern "C" void *svtme_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? (size_t)bytes : 1, hipHostMallocDefault) != hipSuccess) {
        svtme_set_error_internal("svtme_host_alloc: hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

extern "C" void svtme_host_free(void *p) {
    if (p)
        (void)hipHostFree(p);
}

extern "C" svtme_status svtme_host_register(void *p, uint64_t bytes) {
    if (!p || !bytes)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_host_register: bad arguments");
    HIP_TRY(hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault));
    return SVTME_OK;
}

extern "C" svtme_status svtme_host_unregister(void *p) {
    if (!p)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_host_unregister: null pointer");
    HIP_TRY(hipHostUnregister(p));
    return SVTME_OK;
}

// Worst-case device bytes of one packed job over sbs SBs with R slots: records,
// SB results and the packed copy (the layout of svtme_submit_picture_packed_async)
static size_t packed_job_bytes(size_t sbs, uint32_t R, const svtme_pack_layout *L) {
    const size_t rb = sbs * R * sizeof(svtme_ref_record);
    const size_t sbb = L->sb_results ? sbs * sizeof(svtme_sb_result) : 0;
    const size_t o_sb = (rb + 255) & ~(size_t)255, o_pk = (o_sb + sbb + 255) & ~(size_t)255;
    return o_pk + sbs * svtme_packed_sb_bytes(L, R);
}

extern "C" svtme_status svtme_reserve(svtme_ctx *c, uint32_t width, uint32_t height, uint32_t max_refs,
                                      uint32_t tickets) {
    if (!c || width == 0 || height == 0 || max_refs == 0 || max_refs > 8 || tickets > SVTME_MAX_TICKETS)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_reserve: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    // one picture with max_refs slots, or a batch of SVTME_MAX_BATCH_JOBS pictures of one
    // slot each (a TF window): the per-SB scratch covers the batch's SBs
    const size_t pic_sbs = svtme_sb_total(width, height);
    const size_t sbs     = pic_sbs * SVTME_MAX_BATCH_JOBS;
    const size_t slots   = pic_sbs * std::max<size_t>(max_refs, SVTME_MAX_BATCH_JOBS);
    svtme_status st;
    for (uint32_t l = 0; l < SVTME_LANES; l++) {
        if ((st = ensure_lane(c, l)))
            return st;
        Lane &L = c->lanes[l];
        const size_t kb = slots * SVTME_PU_COUNT * sizeof(unsigned long long);
        if (L.ares_cap < sbs * SVTME_A_N * sizeof(ARes) || L.bst_cap < sbs * sizeof(BState) || L.keys_cap < kb ||
            L.cslot_cap < slots * sizeof(CSlot))
            HIP_TRY(hipStreamSynchronize(L.s)); // (the lane's queued work reads the old buffers)
        if ((st = ensure_buf((void **)&L.d_ares, &L.ares_cap, sbs * SVTME_A_N * sizeof(ARes))) ||
            (st = ensure_buf((void **)&L.d_bst, &L.bst_cap, sbs * sizeof(BState))))
            return st;
        if (L.keys_cap < kb) {
            if ((st = ensure_buf((void **)&L.d_keys, &L.keys_cap, kb)))
                return st;
            L.keys_rest = false; // new keys are not ~0 yet
        }
        if ((st = ensure_buf((void **)&L.d_cslot, &L.cslot_cap, slots * sizeof(CSlot))))
            return st;
    }
    const svtme_pack_layout pa = {SVTME_PU_COUNT, SVTME_MAX_PA_ME_CAND, SVTME_MAX_PA_ME_MV, 0, 1, {0, 0}};
    const svtme_pack_layout tf = {0, 0, 0, 1, 0, {0, 0}};
    const size_t need = std::max(packed_job_bytes(pic_sbs, max_refs, &pa), packed_job_bytes(pic_sbs, max_refs, &tf));
    uint32_t k = 0;
    for (auto &t : c->tickets) {
        if (k == tickets)
            break;
        if (t.id) // outstanding: its buffer is in use
            continue;
        if ((st = ensure_buf(&t.d_mem, &t.d_cap, need)))
            return st;
        k++;
    }
    return SVTME_OK;
}

extern "C" svtme_status svtme_submit_pictures_packed_async(svtme_ctx *c, uint32_t lane, uint32_t n,
                                                           const svtme_job *jobs, const svtme_pack_layout *layouts,
                                                           void *const *host_outs, uint64_t *tickets) {
    if (!c || !jobs || !layouts || !host_outs || !tickets)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_pictures_packed_async: null argument");
    if (n == 0 || n > SVTME_MAX_BATCH_JOBS)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_pictures_packed_async: %u jobs (1..%d)", n,
                    SVTME_MAX_BATCH_JOBS);
    for (uint32_t k = 0; k < n; k++) {
        const svtme_pack_layout *L = &layouts[k];
        if (!host_outs[k])
            return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_pictures_packed_async: null host_out %u", k);
        if (L->sb_results && (L->n_pus == 0 || L->n_pus > SVTME_PU_COUNT || L->max_cand == 0 ||
                              L->max_cand > SVTME_MAX_PA_ME_CAND || L->max_refs == 0 ||
                              L->max_refs > SVTME_MAX_PA_ME_MV))
            return fail(SVTME_ERR_BAD_PARAMETER, "pack layout: %u PUs, %u candidates, %u MVs", L->n_pus,
                        L->max_cand, L->max_refs);
    }
    std::unique_lock<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    // n free ticket slots; with too few free, wait for other threads' svtme_ticket_wait
    // to retire some (up to 100 ms while nobody waits on a ticket: then the caller
    // holds them itself and is refused)
    Ticket *t[SVTME_MAX_BATCH_JOBS];
    auto free_slots = [&]() {
        uint32_t k = 0;
        for (auto &x : c->tickets)
            if (!x.id && k < n)
                t[k++] = &x;
        return k == n;
    };
    auto someone_waits = [&]() {
        for (auto &x : c->tickets)
            if (x.waiting)
                return true;
        return false;
    };
    const auto grace = std::chrono::steady_clock::now() + std::chrono::milliseconds(100);
    while (!free_slots()) {
        if (!someone_waits() && std::chrono::steady_clock::now() >= grace)
            return fail(SVTME_ERR_INSUFFICIENT_RESOURCES,
                        "%d packed jobs outstanding and none being waited on (svtme_ticket_wait retires them)",
                        SVTME_MAX_TICKETS);
        c->retired.wait_for(lk, std::chrono::milliseconds(5));
    }
    if (!c->dstream)
        HIP_TRY(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
    svtme_ref_record *d_recs[SVTME_MAX_BATCH_JOBS];
    svtme_sb_result *d_sb[SVTME_MAX_BATCH_JOBS];
    void *d_pack[SVTME_MAX_BATCH_JOBS];
    size_t pbytes[SVTME_MAX_BATCH_JOBS];
    uint32_t counts[SVTME_MAX_BATCH_JOBS], Rs[SVTME_MAX_BATCH_JOBS];
    bool any_sb = false;
    svtme_status st;
    for (uint32_t k = 0; k < n; k++) {
        const svtme_job *job       = &jobs[k];
        const svtme_pack_layout *L = &layouts[k];
        const uint32_t total = svtme_sb_total(job->width, job->height);
        counts[k] = job->sb_count ? job->sb_count : (job->sb_begin < total ? total - job->sb_begin : 0);
        Rs[k]     = svtme_job_ref_slots(job);
        const size_t rb  = (size_t)counts[k] * Rs[k] * sizeof(svtme_ref_record);
        const size_t sbb = L->sb_results ? (size_t)counts[k] * sizeof(svtme_sb_result) : 0;
        pbytes[k]        = (size_t)counts[k] * svtme_packed_sb_bytes(L, Rs[k]);
        const size_t o_sb = (rb + 255) & ~(size_t)255, o_pk = (o_sb + sbb + 255) & ~(size_t)255;
        if ((st = ensure_buf(&t[k]->d_mem, &t[k]->d_cap, o_pk + pbytes[k]))) // free slot: nothing reads it
            return st;
        d_recs[k] = (svtme_ref_record *)t[k]->d_mem;
        d_sb[k]   = L->sb_results ? (svtme_sb_result *)((uint8_t *)t[k]->d_mem + o_sb) : nullptr;
        d_pack[k] = (uint8_t *)t[k]->d_mem + o_pk;
        any_sb |= d_sb[k] != nullptr;
    }
    if ((st = ensure_lane(c, lane)))
        return st;
    for (uint32_t k = 0; k < n; k++)
        HIP_TRY(hipEventRecord(t[k]->queued, c->lanes[lane].s));
    // one launch over every job (the stage kernels take up to SVTME_MAX_BATCH jobs)
    if ((st = submit_batch_locked(c, jobs, n, d_recs, d_sb, any_sb, lane)))
        return st;
    hipStream_t ls = c->lanes[lane].s;
    for (uint32_t k = 0; k < n; k++) {
        HIP_TRY(svtme_launch_pack(d_recs[k], d_sb[k], counts[k], Rs[k], &layouts[k], d_pack[k], ls));
        HIP_TRY(hipEventRecord(t[k]->launched, ls));
        HIP_TRY(hipStreamWaitEvent(c->dstream, t[k]->launched, 0));
        HIP_TRY(hipMemcpyAsync(host_outs[k], d_pack[k], pbytes[k], hipMemcpyDeviceToHost, c->dstream));
        HIP_TRY(hipEventRecord(t[k]->done, c->dstream));
        t[k]->id   = ++c->ticket_seq;
        tickets[k] = t[k]->id;
    }
    return SVTME_OK;
}

extern "C" svtme_status svtme_submit_picture_packed_async(svtme_ctx *c, uint32_t lane, const svtme_job *job,
                                                          const svtme_pack_layout *L, void *host_out,
                                                          uint64_t *ticket) {
    if (!c || !job || !L || !host_out || !ticket)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_picture_packed_async: null argument");
    return svtme_submit_pictures_packed_async(c, lane, 1, job, L, &host_out, ticket);
}

extern "C" svtme_status svtme_ticket_wait_timed(svtme_ctx *c, uint64_t ticket, float *gpu_ms, float *copy_ms) {
    if (!c || !ticket)
        return fail(SVTME_ERR_BAD_PARAMETER, "svtme_ticket_wait: null ctx or ticket");
    hipEvent_t done = nullptr;
    Ticket *t       = nullptr;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        for (auto &x : c->tickets)
            if (x.id == ticket && !x.waiting) {
                t = &x;
                break;
            }
        if (!t)
            return fail(SVTME_ERR_BAD_PARAMETER, "svtme_ticket_wait: ticket %llu is not outstanding",
                        (unsigned long long)ticket);
        t->waiting = true;
        done       = t->done;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipError_t e = hipEventSynchronize(done); // without the context lock: other threads submit meanwhile
    // GPU-side times: the job's turn on its lane -> its packed output ready; -> in host memory
    if (e == hipSuccess && gpu_ms)
        e = hipEventElapsedTime(gpu_ms, t->queued, t->launched);
    if (e == hipSuccess && copy_ms)
        e = hipEventElapsedTime(copy_ms, t->launched, t->done);
    std::lock_guard<std::mutex> lk(c->mu);
    t->waiting = false;
    t->id      = 0;
    c->retired.notify_all();
    if (e != hipSuccess)
        return fail(SVTME_ERR_UNDEFINED, "svtme_ticket_wait: %s", hipGetErrorString(e));
    return SVTME_OK;
}

extern "C" svtme_status svtme_ticket_wait(svtme_ctx *c, uint64_t ticket) {
    return svtme_ticket_wait_timed(c, ticket, nullptr, nullptr);
}

extern "C" svtme_status svtme_set_timing(svtme_ctx *c, int enable) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    if (enable && !c->tev[0][0])
        for (auto &set : c->tev)
            for (auto &e : set) HIP_TRY(hipEventCreate(&e));
    c->timing = enable != 0;
    return SVTME_OK;
}

extern "C" uint32_t svtme_timing_read(svtme_ctx *c, float stage_ms[5]) {
    if (!c || !stage_ms)
        return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    double sum[5] = {0, 0, 0, 0, 0};
    uint32_t launches[5] = {0, 0, 0, 0, 0};
    const int n = c->t_pending;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 5; k++) {
            if (!((c->tmask[i] >> k) & 1u))
                continue;
            float ms = 0.0f;
            if (hipEventSynchronize(c->tev[i][2 * k + 1]) != hipSuccess ||
                hipEventElapsedTime(&ms, c->tev[i][2 * k], c->tev[i][2 * k + 1]) != hipSuccess)
                return 0;
            sum[k] += ms;
            launches[k]++;
        }
    // each stage is averaged over the launch groups that ran it
    for (int k = 0; k < 5; k++) stage_ms[k] = launches[k] ? (float)(sum[k] / launches[k]) : 0.0f;
    if (c->t_dropped)
        svtme_set_error_internal("svtme_timing_read: launch groups beyond the timing capacity were not recorded");
    c->t_pending = 0;
    c->t_dropped = 0;
    return (uint32_t)n;
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
    return quiesce(c);
}

static svtme_status fetch_locked(svtme_ctx *c, svtme_ref_record *recs, svtme_sb_result *sb) {
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

extern "C" svtme_status svtme_fetch(svtme_ctx *c, svtme_ref_record *recs, svtme_sb_result *sb) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    return fetch_locked(c, recs, sb);
}

// Submit and fetch under one hold of the context lock: the encoder's ME threads
// call this concurrently, and another thread's submission must not replace the
// context-owned records between this job's launch and its copy-out.
extern "C" svtme_status svtme_submit_picture(svtme_ctx *c, const svtme_job *job, svtme_ref_record *recs,
                                             svtme_sb_result *sb) {
    if (!c)
        return fail(SVTME_ERR_BAD_PARAMETER, "null ctx");
    std::lock_guard<std::mutex> lk(c->mu);
    svtme_status st = submit_locked(c, job, sb != nullptr, nullptr, nullptr);
    if (st)
        return st;
    return fetch_locked(c, recs, sb);
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
