/*
 * synth.c — deterministic, integer-exact synthetic luma generator.
 *
 * Test/bench input infrastructure shared by the GPU path, the CPU oracle and the
 * reference harness so all three see identical pictures:
 *   texture: PCG32(seed 0x5EED0001, stream 1) bytes (top 8 bits) on a
 *            (W/8+48) x (H/8+48) grid, nearest-upsampled x8, then a 9-tap box
 *            filter horizontally then vertically, (sum + 4) / 9, edges clamped;
 *   frame t: texture window offset by (5t, 3t) (global pan) plus per-pixel noise
 *            (pcg() % 9) - 4 from PCG32(seed 0x5EED0001 + t + 1, stream 2) in
 *            raster order, clamped to [0, 255];
 *   10-bit : p10 = (y8 << 2) | ((x + y) & 3), so the MSB plane equals y8.
 *   mixed  : (svtme_synth_frame_mixed_from_texture) the picture is tiled in
 *            256x256 regions, each with its own motion of the same texture
 *            (static, slow, the global pan, other directions, fast, beyond the
 *            search range) or fresh noise every frame, so early exits, pruning
 *            and search centres vary across the picture (bench --workload
 *            4k_p8_mixed); the +-4 noise as above.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct pcg32 {
    uint64_t state, inc;
} pcg32;

static uint32_t pcg32_next(pcg32 *r) {
    uint64_t old = r->state;
    r->state     = old * 6364136223846793005ULL + r->inc;
    uint32_t xs  = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

static void pcg32_seed(pcg32 *r, uint64_t seed, uint64_t seq) {
    r->state = 0;
    r->inc   = (seq << 1u) | 1u;
    pcg32_next(r);
    r->state += seed;
    pcg32_next(r);
}

#define SYNTH_SEED 0x5EED0001ull

void svtme_synth_texture_size(uint32_t w, uint32_t h, uint32_t *tw, uint32_t *th) {
    *tw = (w / 8 + 48) * 8;
    *th = (h / 8 + 48) * 8;
}

static uint32_t clampi(int64_t v, int64_t lo, int64_t hi) { return (uint32_t)(v < lo ? lo : v > hi ? hi : v); }

/* tex must hold tw * th bytes */
void svtme_synth_texture(uint32_t w, uint32_t h, uint8_t *tex) {
    uint32_t tw, th;
    svtme_synth_texture_size(w, h, &tw, &th);
    const uint32_t gw = tw / 8, gh = th / 8;
    uint8_t *grid = (uint8_t *)malloc((size_t)gw * gh);
    pcg32 rng;
    pcg32_seed(&rng, SYNTH_SEED, 1);
    for (size_t i = 0; i < (size_t)gw * gh; i++) grid[i] = (uint8_t)(pcg32_next(&rng) >> 24);
    uint8_t *tmp = (uint8_t *)malloc((size_t)tw * th);
    /* nearest upsample x8 fused with the horizontal 9-tap box */
    for (uint32_t y = 0; y < th; y++) {
        const uint8_t *g = grid + (size_t)(y / 8) * gw;
        for (uint32_t x = 0; x < tw; x++) {
            uint32_t s = 0;
            for (int k = -4; k <= 4; k++) s += g[clampi((int64_t)x + k, 0, tw - 1) / 8];
            tmp[(size_t)y * tw + x] = (uint8_t)((s + 4) / 9);
        }
    }
    for (uint32_t y = 0; y < th; y++)
        for (uint32_t x = 0; x < tw; x++) {
            uint32_t s = 0;
            for (int k = -4; k <= 4; k++) s += tmp[(size_t)clampi((int64_t)y + k, 0, th - 1) * tw + x];
            tex[(size_t)y * tw + x] = (uint8_t)((s + 4) / 9);
        }
    free(tmp);
    free(grid);
}

/* frame t of the pan, 8-bit, into out (stride bytes per row) */
void svtme_synth_frame_from_texture(const uint8_t *tex, uint32_t w, uint32_t h, uint32_t t, uint8_t *out,
                                    uint32_t stride) {
    uint32_t tw, th;
    svtme_synth_texture_size(w, h, &tw, &th);
    pcg32 rng;
    pcg32_seed(&rng, SYNTH_SEED + t + 1, 2);
    const uint32_t dx = 5 * t, dy = 3 * t;
    for (uint32_t y = 0; y < h; y++) {
        const uint8_t *row = tex + (size_t)((y + dy) % th) * tw;
        for (uint32_t x = 0; x < w; x++) {
            int v = row[(x + dx) % tw] + (int)(pcg32_next(&rng) % 9) - 4;
            out[(size_t)y * stride + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
}

void svtme_synth_frame(uint32_t w, uint32_t h, uint32_t t, uint8_t *out, uint32_t stride) {
    uint32_t tw, th;
    svtme_synth_texture_size(w, h, &tw, &th);
    uint8_t *tex = (uint8_t *)malloc((size_t)tw * th);
    svtme_synth_texture(w, h, tex);
    svtme_synth_frame_from_texture(tex, w, h, t, out, stride);
    free(tex);
}

/* 10-bit variant: uint16 samples, stride in samples */
void svtme_synth_frame10_from_texture(const uint8_t *tex, uint32_t w, uint32_t h, uint32_t t, uint16_t *out,
                                      uint32_t stride) {
    uint8_t *y8 = (uint8_t *)malloc((size_t)w * h);
    svtme_synth_frame_from_texture(tex, w, h, t, y8, w);
    for (uint32_t y = 0; y < h; y++)
        for (uint32_t x = 0; x < w; x++)
            out[(size_t)y * stride + x] = (uint16_t)((y8[(size_t)y * w + x] << 2) | ((x + y) & 3));
    free(y8);
}

/* region motion classes of the mixed content: (vx, vy) per frame; 0x7FFF = noise */
static const int16_t k_mixed_motion[8][2] = {{0, 0}, {1, 1}, {5, 3}, {-6, 2}, {14, -8}, {36, 20}, {-72, 40},
                                             {0x7FFF, 0}};

static uint32_t mix32(uint32_t v) { /* integer hash of a region index */
    v ^= v >> 16;
    v *= 0x7FEB352Du;
    v ^= v >> 15;
    v *= 0x846CA68Bu;
    v ^= v >> 16;
    return v;
}

static uint32_t wrap(int64_t v, uint32_t n) { return (uint32_t)(((v % (int64_t)n) + (int64_t)n) % (int64_t)n); }

/* frame t of the mixed-motion content, 8-bit */
void svtme_synth_frame_mixed_from_texture(const uint8_t *tex, uint32_t w, uint32_t h, uint32_t t, uint8_t *out,
                                          uint32_t stride) {
    uint32_t tw, th;
    svtme_synth_texture_size(w, h, &tw, &th);
    pcg32 rng, nrng;
    pcg32_seed(&rng, SYNTH_SEED + t + 1, 2);
    pcg32_seed(&nrng, SYNTH_SEED ^ (0x9E3779B9u * (t + 1)), 3);
    for (uint32_t y = 0; y < h; y++)
        for (uint32_t x = 0; x < w; x++) {
            const uint32_t k = mix32((x >> 8) * 131u + (y >> 8) * 7919u + 17u) & 7u;
            const uint32_t n = pcg32_next(&rng) % 9, z = pcg32_next(&nrng) >> 24;
            int v;
            if (k_mixed_motion[k][0] == 0x7FFF)
                v = (int)z;
            else
                v = tex[(size_t)wrap((int64_t)y + (int64_t)k_mixed_motion[k][1] * t, th) * tw +
                        wrap((int64_t)x + (int64_t)k_mixed_motion[k][0] * t, tw)] + (int)n - 4;
            out[(size_t)y * stride + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
}
