/*
 * synth.c -- deterministic synthetic camera stream.
 *
 * The reference's datasets (TUM/EuRoC/KITTI) and mono_tum are absent, so every config runs
 * on a textured synthetic scene of the same geometry. Integer-only, so the CPU container,
 * the GPU box and every rank produce identical bytes.
 *
 * Texture of agent a: (W+640) x (H+32) = low-frequency background (bilinear upsample of a
 * 20x15 random grid, values 40..215) + rectangles (8..64 px, intensity 0..255; 400 per
 * 640x480 of texture area) + per-pixel noise in [-3,3]; seed 0x5EED0000 + 1000003*a.
 * Frame t = W x H crop at (16 + (2t mod 600), 8 + (t mod 7)): a slow pan, so consecutive
 * frames share most features (realistic work for the triangulation matcher). Shared-scene
 * mode (orbx_synth_scene_frames): every agent views one texture from its own crop offset, as
 * the reference's two agents map one environment (the bench's default at N > 1).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/orbslam_amd.h"

static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint8_t* make_texture(int agent, int tw, int th) {
    uint64_t s = 0x5EED0000ull + 1000003ull * (uint64_t)agent;
    enum { GX = 20, GY = 15 };
    int g[GY + 1][GX + 1];
    for (int y = 0; y <= GY; y++)
        for (int x = 0; x <= GX; x++) g[y][x] = 40 + (int)(splitmix64(&s) % 176);
    uint8_t* t = (uint8_t*)malloc((size_t)tw * th);
    if (!t) return NULL;
    for (int y = 0; y < th; y++) {
        int64_t fy = ((int64_t)y * GY << 16) / th;
        int iy = (int)(fy >> 16);
        int64_t wy = fy & 0xFFFF;
        for (int x = 0; x < tw; x++) {
            int64_t fx = ((int64_t)x * GX << 16) / tw;
            int ix = (int)(fx >> 16);
            int64_t wx = fx & 0xFFFF;
            int64_t top = g[iy][ix] * (65536 - wx) + g[iy][ix + 1] * wx;
            int64_t bot = g[iy + 1][ix] * (65536 - wx) + g[iy + 1][ix + 1] * wx;
            int64_t v = (top * (65536 - wy) + bot * wy + (1ll << 31)) >> 32;
            t[(size_t)y * tw + x] = (uint8_t)v;
        }
    }
    int64_t nrect = (int64_t)400 * tw * th / (640 * 480);
    for (int64_t r = 0; r < nrect; r++) {
        uint64_t a = splitmix64(&s), b = splitmix64(&s);
        int rw = 8 + (int)(a % 57), rh = 8 + (int)((a >> 16) % 57);
        int x0 = (int)((a >> 32) % (uint64_t)tw), y0 = (int)(b % (uint64_t)th);
        uint8_t val = (uint8_t)((b >> 32) & 0xFF);
        for (int y = y0; y < y0 + rh && y < th; y++) memset(t + (size_t)y * tw + x0, val, (size_t)((x0 + rw < tw ? x0 + rw : tw) - x0));
    }
    for (size_t i = 0; i < (size_t)tw * th; i += 16) {
        uint64_t a = splitmix64(&s), b = splitmix64(&s);
        for (int k = 0; k < 16 && i + k < (size_t)tw * th; k++) {
            uint64_t bits = k < 8 ? (a >> (8 * k)) : (b >> (8 * (k - 8)));
            int v = t[i + k] + (int)((bits & 0xFF) % 7) - 3;
            t[i + k] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
    return t;
}

/* frame t of view `view` of the texture of `scene`: the crop of view v starts kViewStep*v pixels further along the
 * pan (modulo the pan's 600 px), so the views of one scene are agents looking at one environment from places a
 * few dozen pixels apart; view 0 is the scene's own stream (orbx_synth_frames_shifted(scene, ...)) */
enum { kViewStep = 12 };

int orbx_synth_scene_frames(int scene, int view, int t0, int count, int width, int height, int dx, uint8_t* out) {
    if (width <= 0 || height <= 0 || count < 0 || !out || scene < 0 || view < 0 || view > 4096 || t0 < 0 || dx < 0 ||
        dx > 26)
        return ORBX_EARG;
    const int tw = width + 640, th = height + 32;
    uint8_t* tex = make_texture(scene, tw, th);
    if (!tex) return ORBX_EARG;
    for (int f = 0; f < count; f++) {
        int t = t0 + f;
        int ox = 16 + (int)((2ll * t + (long long)kViewStep * view) % 600) + dx, oy = 8 + t % 7;
        for (int y = 0; y < height; y++)
            memcpy(out + ((size_t)f * height + y) * width, tex + (size_t)(oy + y) * tw + ox, (size_t)width);
    }
    free(tex);
    return ORBX_OK;
}

int orbx_synth_frames_shifted(int agent, int t0, int count, int width, int height, int dx, uint8_t* out) {
    return orbx_synth_scene_frames(agent, 0, t0, count, width, height, dx, out);
}

int orbx_synth_frames(int agent, int t0, int count, int width, int height, uint8_t* out) {
    return orbx_synth_frames_shifted(agent, t0, count, width, height, 0, out);
}

int orbx_synth_frame(int agent, int t, int width, int height, uint8_t* out) {
    return orbx_synth_frames(agent, t, 1, width, height, out);
}
