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

}  // namespace ocean
