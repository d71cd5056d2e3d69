// Fragment program 1: the fork's `oceanic_horizon` (reference csrc/shaders.cpp:1668-1919) for the
// raster kernel's resolve.  float32 in the GLSL source's operation order, no contraction
// (-ffp-contract=off), IEEE division and sqrt; GLSL's driver-defined sin/cos/pow are replaced by fixed
// algorithms that the CPU oracle (oracle/dirt_oracle.c, ocn_*) states identically, so
// the two agree bit for bit.  Terms scaled by small_waveheight = 0.0 (shaders.cpp:1690,1776-1785) are
// exact zeros and omitted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ocean {

__device__ __forceinline__ float sincos_fixed(float x, bool want_cos)
{
    if (!(fabsf(x) < 1.0e30f)) return x - x;  // NaN for inf / NaN
    const float k = __builtin_rintf(x * 0.636619772f);
    float r = x - k * 1.5703125f;  // pi/2 = 1.5703125 + 4.8375129699707031e-4 + 7.549790126e-8
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.549790126404332e-8f;
    float q = k - 4.0f * floorf(k * 0.25f);
    if (want_cos) q = q + 1.0f;
    if (q >= 4.0f) q = q - 4.0f;
    const float z = r * r;
    const float s = r + (r * z) * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
    const float c = (1.0f - 0.5f * z) +
                    (z * z) * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    return q == 0.0f ? s : q == 1.0f ? c : q == 2.0f ? -s : -c;
}
__device__ __forceinline__ float sin_fixed(float x) { return sincos_fixed(x, false); }

// sin for water() (the hot loop): one reduction by pi, odd Taylor polynomial to x^11 on [-pi/2, pi/2],
// sign by the parity of k (the oracle's ocn_sin_pi)
__device__ __forceinline__ float sin_pi_fixed(float x)
{
    if (!(fabsf(x) < 1.0e30f)) return x - x;
    const float k = __builtin_rintf(x * 0.318309873f);
    float r = fmaf(-k, 3.140625f, x);  // explicit fused multiply-adds, as the oracle's fmaf
    r = fmaf(-k, 9.675025939941406e-4f, r);
    r = fmaf(-k, 1.5099580252808664e-7f, r);
    const float z = r * r;
    float p = fmaf(z, -2.5052107943679403e-8f, 2.7557318844628753e-6f);
    p = fmaf(z, p, -1.9841270113829523e-4f);
    p = fmaf(z, p, 8.333333767950535e-3f);
    p = fmaf(z, p, -1.666666716337204e-1f);
    const float sn = fmaf(r * z, p, r);
    const float parity = k - 2.0f * floorf(k * 0.5f);
    return parity == 1.0f ? -sn : sn;
}
__device__ __forceinline__ float cos_fixed(float x) { return sincos_fixed(x, true); }

__device__ __forceinline__ float log2_fixed(float x)  // normal x > 0
{
    const uint32_t u = __builtin_bit_cast(uint32_t, x);
    float e = (float)((int)((u >> 23) & 0xffu) - 126);
    float m = __builtin_bit_cast(float, (u & 0x807fffffu) | 0x3f000000u);  // [0.5, 1)
    if (m < 0.70710678f) {
        m = m * 2.0f;
        e = e - 1.0f;
    }
    const float t = (m - 1.0f) / (m + 1.0f);
    const float t2 = t * t;
    const float l = t * (2.885390082f + t2 * (0.9617966939f + t2 * (0.5770780164f + t2 * (0.4121985831f +
                                                                                         t2 * 0.3205988980f))));
    return e + l;
}

__device__ __forceinline__ float exp2_fixed(float z)  // z <= 0
{
    if (!(z >= -125.0f)) return 0.0f;
    const float n = floorf(z + 0.5f);
    const float f = z - n;
    const float p = 1.0f + f * (0.6931471806f + f * (0.2402265070f + f * (0.05550410866f + f * (0.009618129108f +
                    f * (0.001333355815f + f * 0.0001540353039f)))));
    return ldexpf(p, (int)n);
}

__device__ __forceinline__ float pow01(float x, float y)  // GLSL pow, x in [0,1], y > 0
{
    if (!(x >= 1.17549435e-38f)) return 0.0f;
    if (x >= 1.0f) return 1.0f;
    return exp2_fixed(y * log2_fixed(x));
}

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
__device__ __forceinline__ float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz)
{
    return (ax * bx + ay * by) + az * bz;
}

// water(p), shaders.cpp:1760-1791
__device__ __forceinline__ float water(float px, float py, float shift2x)
{
    float wave = 0.0f;
    wave = wave + sin_pi_fixed(px * 0.021f + shift2x) * 4.5f;
    wave = wave + sin_pi_fixed((px * 0.0172f + py * 0.010f) + shift2x * 1.121f) * 4.0f;
    wave = wave - sin_pi_fixed((px * 0.00104f + py * 0.005f) + shift2x * 0.121f) * 4.0f;
    wave = wave + sin_pi_fixed((px * 0.02221f + py * 0.01233f) + shift2x * 3.437f) * 5.0f;
    wave = wave + sin_pi_fixed((px * 0.03112f + py * 0.01122f) + shift2x * 4.269f) * 2.5f;
    wave = wave * 1.0f;  // large_waveheight
    return 70.0f + wave;
}

struct Camera {
    float x, y, z, ang1, ang2, ang3, time, light_z;
};

// main() of shaders.cpp:1858-1917 at the jittered texCoordV (xx, xy): returns (col.x, col.y)
__device__ __noinline__ float2 shade(float xx, float xy, const Camera cam, float width, float height)
{
    const float shift2x = 0.001f * ((cam.time * 190.0f) * 2.0f);
    float lx = 0.1f, ly = 0.25f, lz = cam.light_z;
    {
        const float l = sqrtf(dot3(lx, ly, lz, lx, ly, lz));
        lx = lx / l; ly = ly / l; lz = lz / l;
    }
    float vx = (xx + 1.0f) * width / 2.0f - width / 2.0f;
    float vy = (xy + 1.0f) * height / 2.0f - height / 2.0f;
    float vz = 1.73f * width / 2.0f;
    {
        const float l = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
        vx = vx / l; vy = vy / l; vz = vz / l;
    }
    const float sin1 = sin_fixed(cam.ang1), cos1 = cos_fixed(cam.ang1);
    const float sin2 = sin_fixed(cam.ang2), cos2 = cos_fixed(cam.ang2);
    const float sin3 = sin_fixed(cam.ang3), cos3 = cos_fixed(cam.ang3);
    const float rx = ((cos2 * cos3) * vx + (-cos1 * sin3 + (sin1 * sin2) * cos3) * vy) +
                     (sin1 * sin3 + (cos1 * sin2) * cos3) * vz;
    const float ry = ((cos2 * sin3) * vx + (cos1 * cos3 + (sin1 * sin2) * sin3) * vy) +
                     (-sin1 * cos3 + (cos1 * sin2) * sin3) * vz;
    const float rz = (-sin2 * vx + (sin1 * cos2) * vy) + (cos1 * cos2) * vz;
    float sundot = clamp01(dot3(rx, ry, rz, lx, ly, lz));
    // sky: trace() returns false for rd.y > 0 and its march result is unused
    if (ry > 0.0f) return make_float2(1.0f, pow01(sundot, 350.0f));
    // trace(), shaders.cpp:1817-1856 (RENDER_GODRAYS undefined)
    float t = -cam.y / ry;
    float st = 0.5f, old_h = 0.0f;
    for (int j = 1000; j < 1020; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p0 = cam.x + t * rx, p1 = cam.y + t * ry, p2 = cam.z + t * rz;
        const float h = p1 - water(p0, p2, shift2x);
        t = t + (fmaxf(1.0f, fabsf(h)) * sgn(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    const float wx = cam.x + t * rx, wz = cam.z + t * rz;
    const float d = 0.1f * 1.0f * 4.0f;
    float nx = water(wx - d, wz, shift2x) - water(wx + d, wz, shift2x), ny = 1.0f;
    float nz = water(wx, wz - d, shift2x) - water(wx, wz + d, shift2x);
    {
        const float l = sqrtf(dot3(nx, ny, nz, nx, ny, nz));
        nx = nx / l; ny = ny / l; nz = nz / l;
    }
    const float dn = 2.0f * dot3(nx, ny, nz, rx, ry, rz);
    const float qx = rx - dn * nx, qy = ry - dn * ny, qz = rz - dn * nz;
    sundot = clamp01(dot3(qx, qy, qz, lx, ly, lz));
    const float refl = (0.5f * pow01(sundot, 10.0f) + 0.25f * pow01(sundot, 3.5f)) + 0.75f * pow01(sundot, 300.0f);
    return make_float2(0.0f, refl);
}


// ------------------------------------------------------------------------------------------------
// The oceanic family (shader ids 2..5): `oceanic` (bound by RasteriseGrad, shaders.cpp:556-864),
// `oceanic_still_cloud` (:866-1176), `oceanic_no_cloud` (:1402-1666), `oceanic_simple_proxy`
// (:1921-2185) -- one program with per-member constants.  Mirrors the oracle's ocn_family_* line by
// line (GLSL operation order, fixed transcendentals, column-major mat*vec, row-vector v *= M).

struct Family {
    float wavegain, large_wh, small_wh;
    float fogcolor[3], skybottom[3], skytop[3], reflskycolor[3], watercolor[3];
    float s1x, s1y, s2x, s2y;
    int wave_cos, small_iters, march_steps, clouds;
};

__device__ __forceinline__ Family family_params(int sid)
{
    Family P{1.0f, 1.0f, 1.0f, {0.5f, 0.7f, 1.1f}, {0.6f, 0.8f, 1.2f}, {0.05f, 0.2f, 0.5f},
             {0.025f, 0.10f, 0.20f}, {0.2f, 0.25f, 0.3f}, 160.0f, 120.0f, 190.0f, 130.0f, 0, 7, 20, 1};
    if (sid == DIRT_SHADER_OCEANIC_STILL_CLOUD) P.clouds = 2;
    if (sid == DIRT_SHADER_OCEANIC_NO_CLOUD) P.clouds = 0;
    if (sid == DIRT_SHADER_OCEANIC_SIMPLE_PROXY)
        P = Family{0.75f, 0.75f, 1.5f, {0.4f, 0.4f, 1.2f}, {0.5f, 0.5f, 1.3f}, {0.15f, 0.1f, 0.7f},
                   {0.1f, 0.1f, 0.15f}, {0.1f, 0.2f, 0.5f}, 260.0f, 100.0f, 150.0f, 230.0f, 1, 3, 10, 0};
    return P;
}

__device__ __forceinline__ float fract(float x) { return x - floorf(x); }
__device__ __forceinline__ float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
__device__ __forceinline__ float smoothstepf(float e0, float e1, float x)
{
    const float t = clamp01((x - e0) / (e1 - e0));
    return t * t * (3.0f - 2.0f * t);
}
__device__ __forceinline__ float exp2_any(float z)
{
    if (!(z >= -125.0f)) return 0.0f;
    if (z > 128.0f) return __builtin_inff();
    const float n = floorf(z + 0.5f);
    const float f = z - n;
    const float p = 1.0f + f * (0.6931471806f + f * (0.2402265070f + f * (0.05550410866f + f * (0.009618129108f +
                    f * (0.001333355815f + f * 0.0001540353039f)))));
    return ldexpf(p, (int)n);
}
__device__ __forceinline__ float pow_pos(float x, float y)
{
    if (!(x >= 1.17549435e-38f)) return 0.0f;
    if (x == 1.0f) return 1.0f;
    if (!(x < __builtin_inff())) return __builtin_inff();
    return exp2_any(y * log2_fixed(x));
}
__device__ __forceinline__ float expf_fixed(float x) { return exp2_any(x * 1.44269504f); }

__device__ __forceinline__ float hashf(float n) { return fract(cos_fixed(n) * 41415.92653f); }
__device__ __forceinline__ float rand2(float nx, float ny)
{
    return fract(sin_pi_fixed(nx * 12.9898f + ny * 4.1414f) * 43758.5453f);
}

__device__ __forceinline__ float noise2(float px, float py)
{
    const float ix = floorf(px), iy = floorf(py);
    float ux = fract(px), uy = fract(py);
    ux = ux * ux * (3.0f - 2.0f * ux);
    uy = uy * uy * (3.0f - 2.0f * uy);
    return mixf(mixf(rand2(ix, iy), rand2(ix + 1.0f, iy + 0.0f), ux),
                mixf(rand2(ix + 0.0f, iy + 1.0f), rand2(ix + 1.0f, iy + 1.0f), ux), uy);
}

__device__ __forceinline__ float noise3(float x, float y, float z)
{
    const float px = floorf(x), py = floorf(y), pz = floorf(z);
    const float fx = smoothstepf(0.0f, 1.0f, fract(x));
    const float fy = smoothstepf(0.0f, 1.0f, fract(y));
    const float fz = smoothstepf(0.0f, 1.0f, fract(z));
    const float n = (px + py * 57.0f) + 113.0f * pz;
    return mixf(mixf(mixf(hashf(n + 0.0f), hashf(n + 1.0f), fx), mixf(hashf(n + 57.0f), hashf(n + 58.0f), fx), fy),
                mixf(mixf(hashf(n + 113.0f), hashf(n + 114.0f), fx), mixf(hashf(n + 170.0f), hashf(n + 171.0f), fx), fy),
                fz);
}

__device__ __forceinline__ void m3(float &x, float &y, float &z)
{
    const float a = x, b = y, c = z;
    x = (0.00f * a + -1.60f * b) + -1.20f * c;
    y = (1.60f * a + 0.72f * b) + -0.96f * c;
    z = (1.20f * a + -0.96f * b) + 1.28f * c;
}

__device__ __noinline__ float fbm3(float x, float y, float z)
{
    float f = 0.5000f * noise3(x, y, z);
    m3(x, y, z); x = x * 1.1f; y = y * 1.1f; z = z * 1.1f;
    f = f + 0.2500f * noise3(x, y, z);
    m3(x, y, z); x = x * 1.2f; y = y * 1.2f; z = z * 1.2f;
    f = f + 0.1666f * noise3(x, y, z);
    m3(x, y, z);
    f = f + 0.0834f * noise3(x, y, z);
    return f;
}

__device__ __forceinline__ float fbm2(float x, float y)
{
    float f = 0.5000f * noise2(x, y);
    float nx = 1.6f * x + 1.2f * y, ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.2500f * noise2(x, y);
    nx = 1.6f * x + 1.2f * y; ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.1666f * noise2(x, y);
    nx = 1.6f * x + 1.2f * y; ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.0834f * noise2(x, y);
    return f;
}

__device__ __noinline__ float family_water(const Family &P, float px, float py, float time)
{
    float height = 70.0f;
    float s1x = 0.001f * ((time * P.s1x) * 2.0f), s1y = 0.001f * ((time * P.s1y) * 2.0f);
    const float s2x = 0.001f * ((time * P.s2x) * 2.0f), s2y = 0.001f * ((-time * P.s2y) * 2.0f);
    float wave = 0.0f;
    if (P.wave_cos) {
        wave = wave + cos_fixed(px * 0.021f + s2x) * 4.5f;
        wave = wave + cos_fixed((px * 0.0172f + py * 0.010f) + s2x * 1.121f) * 4.0f;
        wave = wave - cos_fixed((px * 0.00104f + py * 0.005f) + s2x * 0.121f) * 4.0f;
        wave = wave + cos_fixed((px * 0.02221f + py * 0.01233f) + s2x * 3.437f) * 5.0f;
        wave = wave + cos_fixed((px * 0.03112f + py * 0.01122f) + s2x * 4.269f) * 2.5f;
    } else {
        wave = wave + sin_pi_fixed(px * 0.021f + s2x) * 4.5f;
        wave = wave + sin_pi_fixed((px * 0.0172f + py * 0.010f) + s2x * 1.121f) * 4.0f;
        wave = wave - sin_pi_fixed((px * 0.00104f + py * 0.005f) + s2x * 0.121f) * 4.0f;
        wave = wave + sin_pi_fixed((px * 0.02221f + py * 0.01233f) + s2x * 3.437f) * 5.0f;
        wave = wave + sin_pi_fixed((px * 0.03112f + py * 0.01122f) + s2x * 4.269f) * 2.5f;
    }
    wave = wave * P.large_wh;
    wave = wave - (fbm2(px * 0.004f - s2x * 0.5f, py * 0.004f - s2y * 0.5f) * P.small_wh) * 24.0f;
    float amp = 6.0f * P.small_wh;
    s1x = s1x * 0.3f; s1y = s1y * 0.3f;
    const float m00 = 1.6f * 0.9331f, m01 = -1.2f * 0.9331f, m10 = 1.2f * 0.9331f, m11 = 1.6f * 0.9331f;
    for (int i = 0; i < P.small_iters; ++i) {
        wave = wave - fabsf(sin_pi_fixed((noise2(px * 0.01f + s1x, py * 0.01f + s1y) - 0.5f) * 3.14f)) * amp;
        amp = amp * 0.51f;
        s1x = s1x * 1.841f; s1y = s1y * 1.841f;
        const float nx = px * m00 + py * m01, ny = px * m10 + py * m11;
        px = nx; py = ny;
    }
    height = height + wave;
    return height;
}

__device__ __forceinline__ void cloud_pos(const Family &P, float rox, float roy, float roz, float c, float rdx, float rdy,
                                          float rdz, float q3, float shx, float shy, float &cx, float &cy, float &cz)
{
    if (P.clouds == 1) {
        cx = (rox + c * rdx) + 831.0f;
        cy = (roy + c * rdy) + ((321.0f + q3) - shx * 0.2f);
        cz = (roz + c * rdz) + (1330.0f + shy * 3.0f);
    } else {
        cx = c * rdx + 831.0f;
        cy = c * rdy + ((321.0f + q3) - shx * 0.2f);
        cz = c * rdz + (1330.0f + shy * 3.0f);
    }
}

// main() of the family at the jittered texCoordV; cam: 9 floats (cloud_t at [8] for still_cloud)
__device__ __noinline__ float3 shade_family(const Family P, float xx, float xy, const float *cam, float width,
                                            float height)
{
    const float rox = cam[0], roy = cam[1], roz = cam[2], time = cam[6];
    const float ct = P.clouds == 2 ? cam[8] : time;
    const float shx = ct * 80.0f, shy = ct * 60.0f;
    float lx = 0.1f, ly = 0.25f, lz = cam[7];
    {
        const float l = sqrtf(dot3(lx, ly, lz, lx, ly, lz));
        lx = lx / l; ly = ly / l; lz = lz / l;
    }
    float vx = (xx + 1.0f) * width / 2.0f - width / 2.0f;
    float vy = (xy + 1.0f) * height / 2.0f - height / 2.0f;
    float vz = 1.73f * width / 2.0f;
    {
        const float l = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
        vx = vx / l; vy = vy / l; vz = vz / l;
    }
    const float sin1 = sin_fixed(cam[3]), cos1 = cos_fixed(cam[3]);
    const float sin2 = sin_fixed(cam[4]), cos2 = cos_fixed(cam[4]);
    const float sin3 = sin_fixed(cam[5]), cos3 = cos_fixed(cam[5]);
    const float rx = ((cos2 * cos3) * vx + (-cos1 * sin3 + (sin1 * sin2) * cos3) * vy) +
                     (sin1 * sin3 + (cos1 * sin2) * cos3) * vz;
    const float ry = ((cos2 * sin3) * vx + (cos1 * cos3 + (sin1 * sin2) * sin3) * vy) +
                     (-sin1 * cos3 + (cos1 * sin2) * sin3) * vz;
    const float rz = (-sin2 * vx + (sin1 * cos2) * vy) + (cos1 * cos2) * vz;
    const float sundot = clamp01(dot3(rx, ry, rz, lx, ly, lz));
    if (ry > 0.0f) {
        const float t = pow_pos(1.0f - 0.7f * ry, 15.0f);
        const float p350 = pow_pos(sundot, 350.0f), p2 = pow_pos(sundot, 2.0f);
        const float sunc[3] = {0.47f * 1.6f, 0.47f * 1.4f, 0.47f * 1.0f}, haze[3] = {0.4f * 0.8f, 0.4f * 0.9f, 0.4f * 1.0f};
        float col[3];
        for (int k = 0; k < 3; ++k) {
            col[k] = 0.8f * (P.skybottom[k] * t + P.skytop[k] * (1.0f - t));
            col[k] = col[k] + sunc[k] * p350;
            col[k] = col[k] + haze[k] * p2;
        }
        if (P.clouds != 0) {
            float sum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            const float dense[3] = {0.7f * 0.4f, 0.7f * 0.4f, 0.7f * 0.3f}, light_c[3] = {1.1f, 1.05f, 1.0f};
            for (int q = 1000; q < 1100; ++q) {
                const float fq = (float)(q - 1000);
                const float c = P.clouds == 1 ? ((fq * 12.0f + 350.0f) - roy) / ry : (fq * 12.0f + 350.0f) / ry;
                float cx, cy, cz;
                cloud_pos(P, rox, roy, roz, c, rx, ry, rz, fq * 0.15f, shx, shy, cx, cy, cz);
                float alpha = smoothstepf(0.5f, 1.0f, fbm3(cx * 0.0015f, cy * 0.0015f, cz * 0.0015f)) * 0.9f;
                float lc[3];
                for (int k = 0; k < 3; ++k) lc[k] = mixf(light_c[k], dense[k], alpha);
                alpha = (1.0f - sum[3]) * alpha;
                for (int k = 0; k < 3; ++k) sum[k] = sum[k] + lc[k] * alpha;
                sum[3] = sum[3] + alpha;
                if (sum[3] > 0.98f) break;
            }
            const float alpha = smoothstepf(0.7f, 1.0f, sum[3]);
            const float p13 = pow_pos(sundot, 13.0f), p5 = pow_pos(sundot, 5.0f);
            const float shade_c[3] = {0.6f * 0.8f, 0.6f * 0.75f, 0.6f * 0.7f}, scat[3] = {0.2f * 1.3f, 0.2f * 1.2f, 0.2f * 1.0f};
            for (int k = 0; k < 3; ++k) {
                sum[k] = sum[k] / (sum[3] + 0.0001f);
                sum[k] = sum[k] - (shade_c[k] * p13) * alpha;
                sum[k] = sum[k] + (scat[k] * p5) * (1.0f - alpha);
                col[k] = mixf(col[k], sum[k], sum[3] * (1.0f - t));
            }
        }
        return make_float3(col[0], col[1], col[2]);
    }
    float t = -roy / ry;
    float st = 0.5f, old_h = 0.0f;
    for (int j = 0; j < P.march_steps; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p0 = rox + t * rx, p1 = roy + t * ry, p2 = roz + t * rz;
        const float h = p1 - family_water(P, p0, p2, time);
        t = t + (fmaxf(1.0f, fabsf(h)) * sgn(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    const float dist = t;
    const float wx = rox + dist * rx, wy = roy + dist * ry, wz = roz + dist * rz;
    const float d = 0.1f * P.wavegain * 4.0f;
    float nx = family_water(P, wx - d, wz, time) - family_water(P, wx + d, wz, time), ny = 1.0f;
    float nz = family_water(P, wx, wz - d, time) - family_water(P, wx, wz + d, time);
    {
        const float l = sqrtf(dot3(nx, ny, nz, nx, ny, nz));
        nx = nx / l; ny = ny / l; nz = nz / l;
    }
    const float dn = 2.0f * dot3(nx, ny, nz, rx, ry, rz);
    const float qx = rx - dn * nx, qy = ry - dn * ny, qz = rz - dn * nz;
    const float refl = 1.0f - clamp01(dot3(qx, qy, qz, 0.0f, 1.0f, 0.0f));
    float fogv = 1.0f;
    if (P.clouds != 0) {
        const float fx = wx + 20.0f * qx, fy = wy + 20.0f * qy, fz = wz + 20.0f * qz;
        float sum = 0.0f, q2 = 0.0f, q3 = 0.0f;
        for (int q = 0; q < 10; ++q) {
            const float c = P.clouds == 1 ? ((q2 + 350.0f) - fy) / qy : (q2 + 350.0f) / qy;
            float cx, cy, cz;
            cloud_pos(P, fx, fy, fz, c, qx, qy, qz, q3, shx, shy, cx, cy, cz);
            const float alpha = smoothstepf(0.5f, 1.0f, fbm3(cx * 0.0015f, cy * 0.0015f, cz * 0.0015f));
            sum = sum + (1.0f - sum) * alpha;
            if (sum > 0.98f) break;
            q2 = q2 + 120.0f;
            q3 = q3 + 0.15f;
        }
        fogv = clamp01(1.0f - sum);
    }
    const float sh = smoothstepf(0.2f, 1.0f, fogv) * 0.7f + 0.3f;
    const float wsky = refl * sh, wwater = (1.0f - refl) * sh;
    const float sd = clamp01(dot3(qx, qy, qz, lx, ly, lz));
    const float lift = (wy - 70.0f) + 30.0f;
    const float tint[3] = {0.003f, 0.005f, 0.005f};
    const float wsunrefl = wsky * ((0.5f * pow_pos(sd, 10.0f) + 0.25f * pow_pos(sd, 3.5f)) + 0.75f * pow_pos(sd, 300.0f));
    const float sunw[3] = {1.5f, 1.3f, 1.0f};
    const float fo = 1.0f - expf_fixed(-pow_pos(0.0003f * dist, 1.5f));
    const float p4 = pow_pos(sd, 4.0f);
    const float fogc[3] = {0.6f * 0.6f, 0.6f * 0.5f, 0.6f * 0.4f};
    float out[3];
    for (int k = 0; k < 3; ++k) {
        float c = wsky * P.reflskycolor[k];
        c = c + wwater * P.watercolor[k];
        c = c + tint[k] * lift;
        c = c + sunw[k] * wsunrefl;
        const float fco = P.fogcolor[k] + fogc[k] * p4;
        out[k] = mixf(c, fco, fo);
    }
    return make_float3(out[0], out[1], out[2]);
}

// oceanic_opt_flow (shader id 6), shaders.cpp:1178-1398: flat sea (water() = 58), no jitter; cam: 16
// floats ([9] dt, [10..12] dx,dy,dz, [13..15] dang1..3, oceanic_opt_flow.cpp:399-414).  Returns
// new_coord; mirrors the oracle's oracle_opt_flow_pixel.
__device__ __noinline__ float2 opt_flow(float xx, float xy, const float *cam, float width, float height)
{
    const float rox = cam[0], roy = cam[1], roz = cam[2], dt = cam[9];
    float vx = (xx + 1.0f) * width / 2.0f - width / 2.0f;
    float vy = (xy + 1.0f) * height / 2.0f - height / 2.0f;
    float vz = 1.73f * width / 2.0f;
    {
        const float l = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
        vx = vx / l; vy = vy / l; vz = vz / l;
    }
    float sin1 = sin_fixed(cam[3]), cos1 = cos_fixed(cam[3]);
    float sin2 = sin_fixed(cam[4]), cos2 = cos_fixed(cam[4]);
    float sin3 = sin_fixed(cam[5]), cos3 = cos_fixed(cam[5]);
    const float rx = ((cos2 * cos3) * vx + (-cos1 * sin3 + (sin1 * sin2) * cos3) * vy) +
                     (sin1 * sin3 + (cos1 * sin2) * cos3) * vz;
    const float ry = ((cos2 * sin3) * vx + (cos1 * cos3 + (sin1 * sin2) * sin3) * vy) +
                     (-sin1 * cos3 + (cos1 * sin2) * sin3) * vz;
    const float rz = (-sin2 * vx + (sin1 * cos2) * vy) + (cos1 * cos2) * vz;
    sin1 = sin_fixed(cam[3] - cam[13] * dt); cos1 = cos_fixed(cam[3] - cam[13] * dt);
    sin2 = sin_fixed(cam[4] - cam[14] * dt); cos2 = cos_fixed(cam[4] - cam[14] * dt);
    sin3 = sin_fixed(cam[5] - cam[15] * dt); cos3 = cos_fixed(cam[5] - cam[15] * dt);
    float t = -roy / ry;
    float st = 0.5f, old_h = 0.0f;
    for (int j = 1000; j < 1020; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p1 = roy + t * ry;
        const float h = p1 - 58.0f;
        t = t + (fmaxf(1.0f, fabsf(h)) * sgn(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    float odx = rx, ody = ry, odz = rz;
    if (!(ry > 0.0f)) {
        odx = (rox + t * rx) - (rox - cam[10] * dt);
        ody = (roy + t * ry) - (roy - cam[11] * dt);
        odz = (roz + t * rz) - (roz - cam[12] * dt);
    }
    float ox = ((cos2 * cos3) * odx + (cos2 * sin3) * ody) - sin2 * odz;
    float oy = ((-cos1 * sin3 + (sin1 * sin2) * cos3) * odx + (cos1 * cos3 + (sin1 * sin2) * sin3) * ody) +
               (sin1 * cos2) * odz;
    const float oz = ((sin1 * sin3 + (cos1 * sin2) * cos3) * odx + (-sin1 * cos3 + (cos1 * sin2) * sin3) * ody) +
                     (cos1 * cos2) * odz;
    ox = ox / oz;
    oy = oy / oz;
    const float s = 1.73f * width / 2.0f;
    ox = ox * s;
    oy = oy * s;
    return make_float2(ox + width / 2.0f, oy + height / 2.0f);
}

}  // namespace ocean
