// Fragment program 7: `hill` (reference csrc/shaders.cpp:123-554, op csrc/hill.cpp) for the raster
// kernel's resolve.  Same rules as oceanic.h: float32 in the GLSL operation order, no contraction, IEEE
// division and sqrt, the fixed sin / pow of namespace ocean.  The terrain lookup texture (GL_LINEAR,
// CLAMP_TO_EDGE, hill.cpp:232-236) is the op's background tensor, read in place: bilinear in float32 at
// texel centres (the oracle's hill_sample).  Mirrors oracle/dirt_oracle.c hill_* line by line.
#pragma once
#include "oceanic.h"

namespace hill {

using ocean::clamp01;
using ocean::dot3;
using ocean::fract;
using ocean::mixf;
using ocean::pow_pos;
using ocean::sgn;

struct Tex {
    const float *tex;  // one frame [H][W][C], rows top-first (GL row j = tensor row H-1-j)
    int H, W, C;
};

__device__ __forceinline__ const float *texel_ptr(const Tex &T, int i, int j)
{
    i = i < 0 ? 0 : (i > T.W - 1 ? T.W - 1 : i);
    j = j < 0 ? 0 : (j > T.H - 1 ? T.H - 1 : j);
    return T.tex + ((int64_t)(T.H - 1 - j) * T.W + i) * T.C;
}

__device__ __forceinline__ float4 texel4(const Tex &T, const float *p)
{
    // background upload channel fill (rasterise_egl.cu:33-47)
    if (T.C == 1) return make_float4(p[0], p[0], p[0], 1.0f);
    if (T.C == 3) return make_float4(p[0], p[1], p[2], 1.0f);
    return make_float4(p[0], p[1], p[2], p[3]);
}

__device__ __forceinline__ float lerp2(float t00, float t10, float t01, float t11, float a, float b)
{
    const float r0 = t00 * (1.0f - a) + t10 * a;
    const float r1 = t01 * (1.0f - a) + t11 * a;
    return r0 * (1.0f - b) + r1 * b;
}

// Terrain(p.xz).x (shaders.cpp:219-227)
__device__ __forceinline__ float terrain(const Tex &T, float px, float pz)
{
    const float sx = (px - -14.0f) / 28.0f, sz = (pz - 5.0f) / 20.0f;
    const float u = clamp01(sz), v = clamp01(sx);
    const float x = u * (float)T.W - 0.5f, y = v * (float)T.H - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, b = y - fy;
    const int i0 = (int)fx, j0 = (int)fy;
    const float t00 = texel_ptr(T, i0, j0)[0], t10 = texel_ptr(T, i0 + 1, j0)[0];
    const float t01 = texel_ptr(T, i0, j0 + 1)[0], t11 = texel_ptr(T, i0 + 1, j0 + 1)[0];
    return lerp2(t00, t10, t01, t11, a, b) * 10.3f - 6.1f;
}

// Terrain_normal(p.xz) (:229-237)
__device__ __forceinline__ float3 terrain_normal(const Tex &T, float px, float pz)
{
    const float sx = (px - -14.0f) / 28.0f, sz = (pz - 5.0f) / 20.0f;
    const float u = clamp01(sz), v = clamp01(sx);
    const float x = u * (float)T.W - 0.5f, y = v * (float)T.H - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, b = y - fy;
    const int i0 = (int)fx, j0 = (int)fy;
    const float4 t00 = texel4(T, texel_ptr(T, i0, j0)), t10 = texel4(T, texel_ptr(T, i0 + 1, j0));
    const float4 t01 = texel4(T, texel_ptr(T, i0, j0 + 1)), t11 = texel4(T, texel_ptr(T, i0 + 1, j0 + 1));
    return make_float3(lerp2(t00.y, t10.y, t01.y, t11.y, a, b) * 2.0f - 1.0f,
                       lerp2(t00.z, t10.z, t01.z, t11.z, a, b) * 2.0f - 1.0f,
                       lerp2(t00.w, t10.w, t01.w, t11.w, a, b) * 2.0f - 1.0f);
}

// Hash(float) / Hash(vec2), MOD2 = (3.07965, 7.4235) (:160-175)
__device__ __forceinline__ float hash1(float p)
{
    float x = fract(p / 3.07965f), y = fract(p / 7.4235f);
    const float d = y * (x + 19.19f) + x * (y + 19.19f);
    x = x + d; y = y + d;
    return fract(x * y);
}
__device__ __forceinline__ float hash2(float px, float py)
{
    float x = fract(px / 3.07965f), y = fract(py / 7.4235f);
    const float d = x * (y + 19.19f) + y * (x + 19.19f);
    x = x + d; y = y + d;
    return fract(x * y);
}

// Noise(vec2) (:179-189)
__device__ __forceinline__ float noise(float x, float y)
{
    const float px = floorf(x), py = floorf(y);
    float fx = fract(x), fy = fract(y);
    fx = (fx * fx) * (3.0f - 2.0f * fx);
    fy = (fy * fy) * (3.0f - 2.0f * fy);
    const float n = px + py * 57.0f;
    return mixf(mixf(hash1(n + 0.0f), hash1(n + 1.0f), fx), mixf(hash1(n + 57.0f), hash1(n + 58.0f), fx), fy);
}

// Voronoi (:191-209)
__device__ __forceinline__ float2 voronoi(float x, float y)
{
    const float px = floorf(x), py = floorf(y);
    const float fx = fract(x), fy = fract(y);
    float res = 100.0f, id = 0.0f;
#pragma unroll
    for (int j = -1; j <= 1; ++j)
#pragma unroll
        for (int i = -1; i <= 1; ++i) {
            const float bx = (float)i, by = (float)j;
            const float h = hash2(px + bx, py + by);
            const float rx = (bx - fx) + h, ry = (by - fy) + h;
            const float d = rx * rx + ry * ry;
            if (d < res) {
                res = d;
                id = h;
            }
        }
    return make_float2(fmaxf(0.4f - sqrtf(res), 0.0f), id);
}

// DE(p) (:287-300), iTime = 0
__device__ __noinline__ float3 de(const Tex T, float px, float py, float pz)
{
    const float iTime = 0.0f;
    const float base = terrain(T, px, pz) - 1.3f;
    const float qx = px * 4.0f, qz = pz * 4.0f;
    const float height = (noise(qx * 2.0f, qz * 2.0f) * 0.75f + noise(qx, qz) * 0.35f) + noise(qx * 0.5f, qz * 0.5f) * 0.2f;
    float y = (py - base) - height;
    y = y * y;
    const float s0 = ocean::sin_fixed(y * 4.0f + qz * 12.3f), s1 = ocean::sin_fixed(y * 4.0f + qx * 12.3f);
    const float w0 = ocean::sin_fixed(iTime * 2.3f + 1.5f * qz), w1 = ocean::sin_fixed(iTime * 3.6f + 1.5f * qx);
    const float ax = (qx * 2.5f + s0 * 0.12f) + (w0 * y) * 0.5f;
    const float ay = (qz * 2.5f + s1 * 0.12f) + (w1 * y) * 0.5f;
    const float2 v = voronoi(ax, ay);
    const float f = v.x * 0.6f + y * 0.58f;
    return make_float3(y - f * 1.4f, clamp01(f * 1.5f), v.y);
}

// GetSky (:254-263)
__device__ __forceinline__ float3 sky(float rx, float ry, float rz, float sx, float sy, float sz)
{
    const float sunAmount = fmaxf(dot3(rx, ry, rz, sx, sy, sz), 0.0f);
    const float v = pow_pos(1.0f - fmaxf(ry, 0.0f), 6.0f);
    const float p800 = fminf(pow_pos(sunAmount, 800.0f) * 1.5f, 0.3f);
    const float sunc[3] = {1.0f, 0.75f, 0.6f}, lo[3] = {0.1f, 0.2f, 0.3f};
    float out[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float s = mixf(lo[k], 0.32f, v);
        s = s + ((sunc[k] * sunAmount) * sunAmount) * 0.25f;
        s = s + sunc[k] * p800;
        out[k] = clamp01(s);
    }
    return make_float3(out[0], out[1], out[2]);
}

// main() (:453-551) at texCoordV (tx, ty); cam: 12 floats, [9..11] = o0, o1, o2
__device__ __noinline__ float4 shade(const Tex T, float tx, float ty, const float *cam)
{
    const float width = (float)T.W, height = (float)T.H;
    const float xyx = (tx + 1.0f) / 2.0f, xyy = (ty * -1.0f + 1.0f) / 2.0f;
    if (fabsf(xyy * height - height / 2.0f) / (width / 2.0f) >= 0.5625f) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float sx = 0.35f, sy = 0.2f, sz = 0.3f;
    {
        const float l = sqrtf(dot3(sx, sy, sz, sx, sy, sz));
        sx = sx / l; sy = sy / l; sz = sz / l;
    }
    float vx = xyx * width - width / 2.0f, vy = xyy * height - height / 2.0f, vz = 0.85f * width;
    {
        const float l = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
        vx = vx / l; vy = vy / l; vz = vz / l;
    }
    const float rox = -cam[9], roy = cam[11], roz = cam[10];
    const float r00 = 0.999999573f, r01 = -0.0000933038802f, r02 = 0.000919791287f;
    const float r10 = 0.000918443273f, r11 = -0.0135434586f, r12 = -0.999907861f;
    const float r20 = 0.000105752439f, r21 = 0.999908279f, r22 = -0.0135433672f;
    const float dx = -((r00 * vx + r10 * vy) + r20 * vz);
    const float dz = (r01 * vx + r11 * vy) + r21 * vz;
    const float dy = (r02 * vx + r12 * vy) + r22 * vz;
    // Scene (:393-428)
    float t = -(roy + 1.0f) / dy;
    float t_inc = 0.0f;
    if (dy > -0.015f) t = 80.0f;
    float h = 0.0f, st = 1.0f, old_h = 0.0f;
    for (int j = 0; j < 100; ++j) {
        t = t + t_inc;
        const float p0 = rox + t * dx, p1 = roy + t * dy, p2 = roz + t * dz;
        h = p1 - terrain(T, p0, p2);
        t_inc = (fmaxf(1.0f, fabsf(h)) * sgn(h)) * st;
        if (h * old_h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    const float dist = t;
    float col[3];
    if (!(fabsf(h) < 0.05f)) {
        const float3 s = sky(dx, dy, dz, sx, sy, sz);
        col[0] = s.x; col[1] = s.y; col[2] = s.z;
    } else {
        const float px = rox + dist * dx, py = roy + dist * dy, pz = roz + dist * dz;
        const float3 nor = terrain_normal(T, px, pz);
        // TerrainColour (:363-377), type 0
        float mat[3];
        const float nz = noise(px * 0.025f, pz * 0.025f);
        const float m0[3] = {0.0f, 0.3f, 0.0f}, m1[3] = {0.2f, 0.3f, 0.0f};
#pragma unroll
        for (int k = 0; k < 3; ++k) mat[k] = mixf(m0[k], m1[k], nz);
        float fn = 0.0f, w = 0.7f, nx = px * 0.1f, ny = pz * 0.1f;  // FractalNoise (:242-252)
        for (int i = 0; i < 3; ++i) {
            fn = fn + noise(nx, ny) * w;
            w = w * 0.6f;
            nx = 2.0f * nx;
            ny = 2.0f * ny;
        }
        const float tsh = fn + 0.5f;
        {  // GrassBlades (:317-346)
            const float rCoC = fmaxf((dist * 0.3f) * 0.04f, (2.0f / height) * (1.0f + dist * 0.3f));
            float d = 0.0f, alpha = 0.0f;
            float cw[4] = {mat[0] * 0.15f, mat[1] * 0.15f, mat[2] * 0.15f, 0.0f};
            for (int i = 0; i < 15; ++i) {
                if (cw[3] > 0.99f) break;
                float3 ret = de(T, px + dx * d, py + dy * d, pz + dz * d);
                ret.x = ret.x + 0.5f * rCoC;
                if (ret.x < rCoC) {
                    alpha = (1.0f - cw[1]) * clamp01((-ret.x - -rCoC) / (rCoC - -rCoC));
                    const float tip[3] = {0.35f, 0.35f, fminf(pow_pos(ret.z, 4.0f) * 35.0f, 0.35f)};
                    const float wt = pow_pos(ret.y, 9.0f) * 0.7f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const float gra = mixf(mat[k], tip[k], wt) * ret.y;
                        cw[k] = cw[k] + gra * alpha;
                    }
                    cw[3] = cw[3] + alpha;
                }
                d = d + fmaxf(ret.x * 0.7f, 0.1f);
            }
            if (cw[3] < 0.2f) { cw[0] = 0.1f; cw[1] = 0.15f; cw[2] = 0.05f; }
#pragma unroll
            for (int k = 0; k < 3; ++k) mat[k] = cw[k] * tsh;
        }
        // DoLighting (:351-356)
        const float sl = dot3(sx, sy, sz, nor.x, nor.y, nor.z);
        const float hl = (sl * sl) * 4.0f;
        const float sunc[3] = {1.0f, 0.75f, 0.6f};
#pragma unroll
        for (int k = 0; k < 3; ++k) mat[k] = (mat[k] * sunc[k]) * hl;
        // ApplyFog (:267-271)
        const float fog = clamp01((dist * dist) * 0.0000012f);
        const float3 s = sky(dx, dy, dz, sx, sy, sz);
        col[0] = mixf(mat[0], s.x, fog);
        col[1] = mixf(mat[1], s.y, fog);
        col[2] = mixf(mat[2], s.z, fog);
    }
    // PostEffects (:437-451)
    float rgb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) rgb[k] = pow_pos(col[k], 0.45f) * 1.3f;
    const float lum = (0.2125f * rgb[0] + 0.7154f * rgb[1]) + 0.0721f * rgb[2];
    const float vig = 0.4f + 0.5f * pow_pos((((40.0f * xyx) * xyy) * (1.0f - xyx)) * (1.0f - xyy), 0.2f);
    float o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = mixf(0.5f, mixf(lum, rgb[k], 1.3f), 1.1f) * vig;
    return make_float4(o[0], o[1], o[2], 1.0f);
}

}  // namespace hill
