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
