/*
 * svtme_oraclejob.c — TEST INFRASTRUCTURE ONLY.
 *
 * The picture-level job API of include/svtme.h (svtme_ctx_create,
 * svtme_picture_upload / _invalidate / _release / _download,
 * svtme_submit_picture, svtme_last_error) implemented over the CPU oracle
 * (svtora_build_pyramid, svtora_me in svtme_oracle.c). It exists so that the
 * encoder-side glue (integration/svtme_svt_glue.c) can be linked into the
 * reference encoder in the build container, which has no GPU, and its field
 * mapping pinned by a byte-identical bitstream (tests/test_encoder.py). The
 * GPU's job results equal the oracle's (tests/test_gpu_parity.py and the golden
 * fixtures), so the same encode with libsvtme.so must give the same bytes.
 * It is never shipped and libsvtme.so never links it.
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "svtme_oracle.h"

struct svtme_ctx {
    pthread_mutex_t mu;
    struct OraPic {
        uint64_t pn;
        uint32_t W, H;
        svtme_pyr pyr;
        int used;
    } *pics;
    size_t n, cap;
    int nthreads;
};

static __thread char t_err[256];

static svtme_status ora_fail(svtme_status st, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_err, sizeof(t_err), fmt, ap);
    va_end(ap);
    fprintf(stderr, "svtme(oracle backend): %s\n", t_err);
    return st;
}

const char *svtme_last_error(void) { return t_err; }

svtme_status svtme_ctx_create(int device, svtme_ctx **out) {
    (void)device;
    svtme_ctx *c = (svtme_ctx *)calloc(1, sizeof(*c));
    if (!c)
        return SVTME_ERR_INSUFFICIENT_RESOURCES;
    pthread_mutex_init(&c->mu, NULL);
    const char *e = getenv("SVTME_ORACLE_THREADS");
    c->nthreads   = e ? atoi(e) : 4;
    *out          = c;
    return SVTME_OK;
}

static void free_pic(struct OraPic *p) {
    free(p->pyr.full);
    free(p->pyr.quarter);
    free(p->pyr.sixteenth);
}

void svtme_ctx_destroy(svtme_ctx *c) {
    if (!c)
        return;
    for (size_t i = 0; i < c->n; i++) free_pic(&c->pics[i]);
    free(c->pics);
    pthread_mutex_destroy(&c->mu);
    free(c);
}

static struct OraPic *find(svtme_ctx *c, uint64_t pn) {
    for (size_t i = 0; i < c->n; i++)
        if (c->pics[i].used && c->pics[i].pn == pn)
            return &c->pics[i];
    return NULL;
}

static svtme_status upload_locked(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride, uint32_t w,
                                  uint32_t h) {
    const uint32_t W = svtme_align8(w), H = svtme_align8(h);
    struct OraPic *p = find(c, pn);
    if (p && (p->W != W || p->H != H)) {
        free_pic(p);
        p->used = 0;
        p       = NULL;
    }
    if (!p) {
        for (size_t i = 0; i < c->n && !p; i++)
            if (!c->pics[i].used)
                p = &c->pics[i];
        if (!p) {
            if (c->n == c->cap) {
                size_t nc             = c->cap ? 2 * c->cap : 16;
                struct OraPic *grown = (struct OraPic *)realloc(c->pics, nc * sizeof(*grown));
                if (!grown)
                    return ora_fail(SVTME_ERR_INSUFFICIENT_RESOURCES, "out of memory");
                c->pics = grown;
                c->cap  = nc;
            }
            p = &c->pics[c->n++];
        }
        memset(p, 0, sizeof(*p));
        p->pyr.full      = (uint8_t *)malloc((size_t)(W + 2 * SVTME_PAD_FULL) * (H + 2 * SVTME_PAD_FULL));
        p->pyr.quarter   = (uint8_t *)malloc((size_t)(W / 2 + 2 * SVTME_PAD_QUARTER) * (H / 2 + 2 * SVTME_PAD_QUARTER));
        p->pyr.sixteenth = (uint8_t *)malloc((size_t)(W / 4 + 2 * SVTME_PAD_SIXTEENTH) * (H / 4 + 2 * SVTME_PAD_SIXTEENTH));
        if (!p->pyr.full || !p->pyr.quarter || !p->pyr.sixteenth) {
            free_pic(p);
            return ora_fail(SVTME_ERR_INSUFFICIENT_RESOURCES, "out of memory");
        }
        p->pn = pn, p->W = W, p->H = H, p->used = 1;
    }
    svtora_build_pyramid(y, stride, w, h, &p->pyr);
    return SVTME_OK;
}

svtme_status svtme_picture_upload(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride, uint32_t width,
                                  uint32_t height) {
    if (!c || !y || !width || !height || stride < width)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_upload: bad arguments");
    pthread_mutex_lock(&c->mu);
    svtme_status st = upload_locked(c, pn, y, stride, width, height);
    pthread_mutex_unlock(&c->mu);
    return st;
}

svtme_status svtme_picture_invalidate(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride, uint32_t width,
                                      uint32_t height) {
    if (!c)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_invalidate: null ctx");
    pthread_mutex_lock(&c->mu);
    svtme_status st = find(c, pn) ? upload_locked(c, pn, y, stride, width, height)
                                  : ora_fail(SVTME_ERR_BAD_PARAMETER, "picture %llu not resident", (unsigned long long)pn);
    pthread_mutex_unlock(&c->mu);
    return st;
}

svtme_status svtme_picture_release(svtme_ctx *c, uint64_t pn) {
    if (!c)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_release: null ctx");
    pthread_mutex_lock(&c->mu);
    struct OraPic *p = find(c, pn);
    if (p) {
        free_pic(p);
        p->used = 0;
    }
    pthread_mutex_unlock(&c->mu);
    return p ? SVTME_OK : ora_fail(SVTME_ERR_BAD_PARAMETER, "picture %llu not resident", (unsigned long long)pn);
}

svtme_status svtme_picture_download(svtme_ctx *c, uint64_t pn, int level, uint8_t *dst, uint32_t *stride,
                                    uint32_t *width, uint32_t *height, uint32_t *pad) {
    if (!c || level < 0 || level > 2)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_picture_download: bad arguments");
    pthread_mutex_lock(&c->mu);
    struct OraPic *p = find(c, pn);
    if (!p) {
        pthread_mutex_unlock(&c->mu);
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "picture %llu not resident", (unsigned long long)pn);
    }
    const uint32_t pd = level == 0 ? SVTME_PAD_FULL : level == 1 ? SVTME_PAD_QUARTER : SVTME_PAD_SIXTEENTH;
    const uint32_t w = p->W >> level, h = p->H >> level, S = w + 2 * pd;
    if (stride)
        *stride = S;
    if (width)
        *width = w;
    if (height)
        *height = h;
    if (pad)
        *pad = pd;
    if (dst)
        memcpy(dst, level == 0 ? p->pyr.full : level == 1 ? p->pyr.quarter : p->pyr.sixteenth,
               (size_t)S * (h + 2 * pd));
    pthread_mutex_unlock(&c->mu);
    return SVTME_OK;
}

svtme_status svtme_submit_picture(svtme_ctx *c, const svtme_job *job, svtme_ref_record *ref_records,
                                  svtme_sb_result *sb_results) {
    if (!c || !job || !ref_records)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_picture: null argument");
    pthread_mutex_lock(&c->mu);
    svtme_status st = SVTME_OK;
    const struct OraPic *cur = find(c, job->picture_number);
    svtme_pyr refs[8];
    memset(refs, 0, sizeof(refs));
    if (!cur || cur->W != job->width || cur->H != job->height)
        st = ora_fail(SVTME_ERR_BAD_PARAMETER, "current picture %llu not resident at %ux%u",
                      (unsigned long long)job->picture_number, job->width, job->height);
    for (int l = 0; !st && l < job->num_lists; l++)
        for (int r = 0; !st && r < job->num_refs[l]; r++) {
            const struct OraPic *p = find(c, job->ref_picture_number[l][r]);
            if (!p || p->W != job->width || p->H != job->height)
                st = ora_fail(SVTME_ERR_BAD_PARAMETER, "reference picture %llu not resident at %ux%u",
                              (unsigned long long)job->ref_picture_number[l][r], job->width, job->height);
            else
                refs[l * 4 + r] = p->pyr;
        }
    if (!st)
        st = svtora_me(job, &cur->pyr, refs, ref_records, sb_results, c->nthreads);
    pthread_mutex_unlock(&c->mu);
    return st;
}

/* ---- asynchronous forms, run synchronously here (the glue's fast path) ---- */
svtme_status svtme_picture_upload_async(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride, uint32_t width,
                                        uint32_t height) {
    return svtme_picture_upload(c, pn, y, stride, width, height);
}

svtme_status svtme_picture_upload_copy_async(svtme_ctx *c, uint64_t pn, const uint8_t *y, uint32_t stride,
                                             uint32_t width, uint32_t height) {
    return svtme_picture_upload(c, pn, y, stride, width, height);
}

void *svtme_upload_stream(svtme_ctx *c) { return c; } // (no streams here: a non-null handle)
svtme_status svtme_reserve_pictures(svtme_ctx *c, uint32_t width, uint32_t height, uint32_t count) {
    return c && width && height && count <= 4096 ? SVTME_OK : SVTME_ERR_BAD_PARAMETER;
}

void *svtme_host_alloc(uint64_t bytes) { return malloc(bytes ? (size_t)bytes : 1); }
void svtme_host_free(void *p) { free(p); }
svtme_status svtme_host_register(void *p, uint64_t bytes) { return p && bytes ? SVTME_OK : SVTME_ERR_BAD_PARAMETER; }
svtme_status svtme_host_unregister(void *p) { return p ? SVTME_OK : SVTME_ERR_BAD_PARAMETER; }
svtme_status svtme_reserve(svtme_ctx *c, uint32_t width, uint32_t height, uint32_t max_refs, uint32_t tickets) {
    return c && width && height && max_refs >= 1 && max_refs <= 8 && tickets <= SVTME_MAX_TICKETS ? SVTME_OK
                                                                                                : SVTME_ERR_BAD_PARAMETER;
}

/* the packed layout of include/svtme.h (svtme_pack_layout), as svtme_pack.hip writes it */
static void pack_sb(const svtme_ref_record *rec, const svtme_sb_result *s, uint32_t R, const svtme_pack_layout *L,
                    uint8_t *o) {
    const uint32_t stride = svtme_packed_sb_bytes(L, R);
    uint8_t *p = o;
    memset(o, 0, stride);
    for (uint32_t r = 0; r < R; r++) {
        if (L->full_records) {
            memcpy(p, &rec[r], sizeof(svtme_ref_record));
            p += sizeof(svtme_ref_record);
        } else {
            memcpy(p, &rec[r].hme_sad, sizeof(svtme_record_tail));
            p += sizeof(svtme_record_tail);
        }
    }
    if (!L->sb_results)
        return;
    const uint32_t v[6] = {s->me_8x8_cost_variance, s->rc_me_distortion, s->me_64x64_distortion,
                           s->me_32x32_distortion, s->me_16x16_distortion, s->me_8x8_distortion};
    memcpy(p, v, sizeof(v));
    p += sizeof(v);
    memcpy(p, s->me_distortion, sizeof(s->me_distortion));
    p += sizeof(s->me_distortion);
    for (uint32_t pu = 0; pu < L->n_pus; pu++) {
        memcpy(p, s->me_mv_array[pu], 4u * L->max_refs);
        p += 4u * L->max_refs;
    }
    p[0] = s->stationary_block_present;
    p[1] = s->rc_me_allow_gm;
    p += 4;
    memcpy(p, s->total_me_candidate_index, L->n_pus);
    p += L->n_pus;
    for (uint32_t pu = 0; pu < L->n_pus; pu++) {
        memcpy(p, s->me_candidate_array[pu], L->max_cand);
        p += L->max_cand;
    }
}

svtme_status svtme_submit_picture_packed_async(svtme_ctx *c, uint32_t lane, const svtme_job *job,
                                               const svtme_pack_layout *L, void *host_out, uint64_t *ticket) {
    (void)lane;
    if (!c || !job || !L || !host_out || !ticket)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_picture_packed_async: null argument");
    const uint32_t total = svtme_sb_total(job->width, job->height);
    const uint32_t count = job->sb_count ? job->sb_count : total - job->sb_begin;
    const uint32_t R     = svtme_job_ref_slots(job);
    svtme_ref_record *recs = (svtme_ref_record *)malloc((size_t)count * R * sizeof(svtme_ref_record));
    svtme_sb_result *sbr   = L->sb_results ? (svtme_sb_result *)malloc((size_t)count * sizeof(svtme_sb_result)) : NULL;
    svtme_status st        = (!recs || (L->sb_results && !sbr))
        ? ora_fail(SVTME_ERR_INSUFFICIENT_RESOURCES, "out of memory")
        : svtme_submit_picture(c, job, recs, sbr);
    if (!st) {
        const uint32_t stride = svtme_packed_sb_bytes(L, R);
        for (uint32_t k = 0; k < count; k++)
            pack_sb(recs + (size_t)k * R, sbr ? sbr + k : NULL, R, L, (uint8_t *)host_out + (size_t)k * stride);
        *ticket = 1;
    }
    free(recs);
    free(sbr);
    return st;
}

svtme_status svtme_submit_pictures_packed_async(svtme_ctx *c, uint32_t lane, uint32_t n, const svtme_job *jobs,
                                                const svtme_pack_layout *layouts, void *const *host_outs,
                                                uint64_t *tickets) {
    if (!c || !jobs || !layouts || !host_outs || !tickets || n == 0 || n > SVTME_MAX_BATCH_JOBS)
        return ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_submit_pictures_packed_async: bad arguments");
    for (uint32_t k = 0; k < n; k++) {
        const svtme_status st = svtme_submit_picture_packed_async(c, lane, &jobs[k], &layouts[k], host_outs[k],
                                                                  &tickets[k]);
        if (st)
            return st;
    }
    return SVTME_OK;
}

svtme_status svtme_sync(svtme_ctx *c) { return c ? SVTME_OK : SVTME_ERR_BAD_PARAMETER; }

svtme_status svtme_ticket_wait_timed(svtme_ctx *c, uint64_t ticket, float *gpu_ms, float *copy_ms) {
    if (gpu_ms)
        *gpu_ms = 0;
    if (copy_ms)
        *copy_ms = 0;
    return svtme_ticket_wait(c, ticket);
}

svtme_status svtme_ticket_wait(svtme_ctx *c, uint64_t ticket) {
    return c && ticket ? SVTME_OK : ora_fail(SVTME_ERR_BAD_PARAMETER, "svtme_ticket_wait: bad arguments");
}
