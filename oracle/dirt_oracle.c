/*
 * dirt_oracle.c -- CPU ORACLE for the dirt rasterise hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path (dirt_amd/) never links it.
 *
 * It restates, as plain single-pass C loops, what the reference's `Rasterise` op computes
 * through the OpenGL fixed-function pipeline:
 *   - op signature / shapes / batching     : csrc/rasterise_egl.cpp:33-53, 309-339
 *   - per-frame draw in face index order   : csrc/rasterise_egl.cpp:440-458 (glDrawElementsBaseVertex,
 *                                             base vertex b*V -> faces index the frame's own vertices)
 *   - depth test LESS on a DEPTH24 buffer   : csrc/rasterise_egl.cpp:194 (GL_DEPTH_TEST), :248 (DEPTH24_STENCIL8),
 *     cleared to 1.0 per frame               : csrc/rasterise_egl.cpp:449
 *   - vertex stage = clip-space passthrough : csrc/shaders.cpp:16-34
 *   - Gouraud colour (perspective-correct)  : README.md:134-137, dirt/rasterise_ops.py:25-26
 *   - background where uncovered, rows flipped to top-row-first:
 *                                             csrc/rasterise_egl.cu:16-51 (upload), :78-104 (download)
 *   - no face culling, no blending          : (no glEnable(GL_CULL_FACE)/GL_BLEND anywhere in csrc/)
 * and the gradient contract of csrc/rasterise_grad_common.h:19-24 (grad_vertices, grad_vertex_colors,
 * grad_background from pixels + grad_pixels), whose algorithm the fork lost; the
 * backward rule is DIRT's filter-based derivative (README.md:146-147) as specified in DESIGN.md §4.
 *
 * PARITY STATUS: the GL driver's exact rasterisation arithmetic is closed source and the reference
 * ships no golden vectors, so the driver-level rules below are *chosen*  and
 * pinned by analytic known-answer tests derived from the reference (README.md:27-70 square, the
 * rasterise_tests.py cylinder invariants) -- "parity pinned by KATs; driver arithmetic unpinned".
 *
 * Raster rules (identical in the HIP path):
 *   R1 vertex: iw=1/w; window xw=(x*iw+1)*(W/2), yw=(y*iw+1)*(H/2) (GL y up), zw=(z*iw)*0.5+0.5
 *   R2 snap:   X=rint(xw*256), Y=rint(yw*256)   (8 sub-pixel bits)
 *   R3 edges:  E_k(P) = A_k*Px + B_k*Py + C_k, exact int64, sample at pixel centre (256i+128, 256j+128);
 *              orientation normalised so the interior is positive; top-left rule: an E_k==0 sample is
 *              inside iff edge k is "left" (A_k>0) or "top" (A_k==0 && B_k<0).
 *   R4 depth:  plane through the snapped vertices, float32, zw in [0,1]; d=(uint)(zw*(2^24-1)+0.5),
 *              passes iff d < 2^24-1 and ((d<<32)|face) is the minimum so far (LESS, first face wins ties)
 *   R5 clip:   faces with every vertex strictly inside the guard band (w>0, |x|<=gx*w, |y|<=gy*w,
 *              gx=32768/W, gy=32768/H) are rasterised directly (near/far by the per-sample zw test);
 *              others are clipped (Sutherland-Hodgman, float32) against z>=-w and the guard planes and
 *              fan-triangulated; sub-triangle s>0 of face f lives at record index F+5f+(s-1).
 *   R6 colour: lambda_k = a_k/((a_0+a_1)+a_2), a_k=float(E_k)*iw_k, mapped through the clip basis;
 *              colour = (l0*c0 + l1*c1) + l2*c2.
 *
 * Compile with -ffp-contract=off (Makefile): every float operation above is one IEEE op, so the HIP
 * kernels (also built with -ffp-contract=off) reproduce coverage, depth and face ids bit-exactly.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define SUBPIX 256
#define MAX_SUB 6 /* a triangle clipped by 5 planes has <= 8 vertices -> <= 6 fan triangles */
#define MAX_POLY 9
#define DEPTH_MAX 16777215u
/* g-buffer word: visible record index, bit 30 set when the face took the R5 clipping path */
#define GBUF_MULTI (1 << 30)
#define GBUF_INDEX_MASK (GBUF_MULTI - 1)

typedef struct {
    int32_t A[3], B[3];
    int64_t C[3];
    int32_t i0, j0, i1, j1; /* inclusive pixel bbox; empty if i0>i1 */
    int32_t face;
    float fx0, fy0, z0, za, zb;
    float iw[3];
    float basis[9]; /* row k = parent barycentric of sub-vertex k */
} orc_rec;

static int64_t floor_div256(int64_t v) { return v >= 0 ? v / 256 : -((-v + 255) / 256); }

/* R1-R4 for one (sub-)triangle given clip coords (x,y,z,w) of three vertices and their parent basis.
 * Returns 1 if the triangle produces a non-empty record. */
/* R5 sub-vertex clamp: a clipped face's sub-vertex x/w is clamped to [-2 gx, 2 gx] (NaN to
 * 2 gx), y/w likewise -- Sutherland-Hodgman keeps them inside the guard band only up to rounding, which near
 * w = 0 is unbounded; ordinary rounding never reaches twice the band, and the snapped integers stay below 2^24. */
static float guard_clamp(float xn, float g) { return xn <= g ? (xn >= -g ? xn : -g) : g; }

/* clamp_g: NULL on the fast path; twice the guard band (2 gx, 2 gy) for a clipped face's sub-triangles */
static int make_record(const float v[3][4], const float basis[3][3], int W, int H, int face, orc_rec *r,
                       const float *clamp_g)
{
    const float hw = 0.5f * (float)W, hh = 0.5f * (float)H;
    int32_t X[3], Y[3];
    float zw[3];
    for (int k = 0; k < 3; ++k) {
        float iw = 1.0f / v[k][3];
        float xn = v[k][0] * iw, yn = v[k][1] * iw, zn = v[k][2] * iw;
        if (clamp_g) {
            xn = guard_clamp(xn, clamp_g[0]);
            yn = guard_clamp(yn, clamp_g[1]);
        }
        float xw = (xn + 1.0f) * hw, yw = (yn + 1.0f) * hh;
        zw[k] = zn * 0.5f + 0.5f;
        X[k] = (int32_t)rintf(xw * 256.0f);
        Y[k] = (int32_t)rintf(yw * 256.0f);
        r->iw[k] = iw;
        for (int i = 0; i < 3; ++i) r->basis[k * 3 + i] = basis[k][i];
    }
    int64_t A[3], B[3], C[3];
    for (int k = 0; k < 3; ++k) {
        int a = (k + 1) % 3, b = (k + 2) % 3;
        A[k] = (int64_t)Y[a] - Y[b];
        B[k] = (int64_t)X[b] - X[a];
        C[k] = -(A[k] * X[a] + B[k] * Y[a]);
    }
    int64_t D = A[0] * X[0] + B[0] * Y[0] + C[0];
    if (D == 0) return 0;
    int64_t Dsigned = D;
    if (D < 0) {
        for (int k = 0; k < 3; ++k) { A[k] = -A[k]; B[k] = -B[k]; C[k] = -C[k]; }
    }
    for (int k = 0; k < 3; ++k) { r->A[k] = (int32_t)A[k]; r->B[k] = (int32_t)B[k]; r->C[k] = C[k]; }
    int32_t xmin = X[0], xmax = X[0], ymin = Y[0], ymax = Y[0];
    for (int k = 1; k < 3; ++k) {
        if (X[k] < xmin) xmin = X[k];
        if (X[k] > xmax) xmax = X[k];
        if (Y[k] < ymin) ymin = Y[k];
        if (Y[k] > ymax) ymax = Y[k];
    }
    int64_t i0 = floor_div256((int64_t)xmin - 128 + 255), i1 = floor_div256((int64_t)xmax - 128);
    int64_t j0 = floor_div256((int64_t)ymin - 128 + 255), j1 = floor_div256((int64_t)ymax - 128);
    if (i0 < 0) i0 = 0;
    if (j0 < 0) j0 = 0;
    if (i1 > W - 1) i1 = W - 1;
    if (j1 > H - 1) j1 = H - 1;
    if (i0 > i1 || j0 > j1) return 0;
    r->i0 = (int32_t)i0; r->i1 = (int32_t)i1; r->j0 = (int32_t)j0; r->j1 = (int32_t)j1;
    r->face = face;
    /* depth plane through the snapped vertices (R4) */
    float fx0 = (float)X[0] * 0.00390625f, fy0 = (float)Y[0] * 0.00390625f;
    float dx1 = (float)X[1] * 0.00390625f - fx0, dy1 = (float)Y[1] * 0.00390625f - fy0;
    float dx2 = (float)X[2] * 0.00390625f - fx0, dy2 = (float)Y[2] * 0.00390625f - fy0;
    float dz1 = zw[1] - zw[0], dz2 = zw[2] - zw[0];
    float det = (float)Dsigned * (1.0f / 65536.0f);
    r->za = (dz1 * dy2 - dz2 * dy1) / det;
    r->zb = (dx1 * dz2 - dx2 * dz1) / det;
    r->fx0 = fx0; r->fy0 = fy0; r->z0 = zw[0];
    return 1;
}

static int finite4(const float *v) { return isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]) && isfinite(v[3]); }

/* plane distances for R5 clipping, in fixed order */
static float plane_dist(int p, const float *v, float gx, float gy)
{
    switch (p) {
    case 0: return v[2] + v[3];
    case 1: return gx * v[3] + v[0];
    case 2: return gx * v[3] - v[0];
    case 3: return gy * v[3] + v[1];
    default: return gy * v[3] - v[1];
    }
}

/* Set up face f of one frame: fills recs[0..nsub-1] (empty ones have i0>i1). Returns nsub (0 = culled);
 * *clipped = 1 if the face took the R5 clipping path. */
static int setup_face(const float *verts, const int32_t *face3, int V, int W, int H, int f, orc_rec recs[MAX_SUB],
                      int *clipped)
{
    *clipped = 0;
    for (int s = 0; s < MAX_SUB; ++s) { recs[s].i0 = 1; recs[s].i1 = 0; recs[s].face = f; }
    float v[3][4];
    for (int k = 0; k < 3; ++k) {
        int32_t vi = face3[k];
        if (vi < 0 || vi >= V) return 0;
        for (int c = 0; c < 4; ++c) v[k][c] = verts[(int64_t)vi * 4 + c];
        if (!finite4(v[k])) return 0;
    }
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    int fast = 1;
    for (int k = 0; k < 3; ++k) {
        float w = v[k][3];
        if (!(w > 0.0f && fabsf(v[k][0]) <= gx * w && fabsf(v[k][1]) <= gy * w)) fast = 0;
    }
    if (fast) {
        const float id[3][3] = {{1.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, {0.f, 0.f, 1.f}};
        make_record((const float(*)[4])v, id, W, H, f, &recs[0], NULL);
        return 1;
    }
    /* R5: Sutherland-Hodgman against near + 4 guard planes, carrying the parent basis */
    *clipped = 1;
    float poly[MAX_POLY][7], tmp[MAX_POLY][7];
    int n = 3;
    for (int k = 0; k < 3; ++k) {
        for (int c = 0; c < 4; ++c) poly[k][c] = v[k][c];
        for (int i = 0; i < 3; ++i) poly[k][4 + i] = (i == k) ? 1.0f : 0.0f;
    }
    for (int p = 0; p < 5; ++p) {
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const float *a = poly[i], *c = poly[(i + 1) % n];
            float da = plane_dist(p, a, gx, gy), dc = plane_dist(p, c, gx, gy);
            int ina = da >= 0.0f, inc = dc >= 0.0f;
            /* R5 vertex cap: more than 8 vertices -- only when rounding near w = 0 makes the
             * polygon non-convex -- culls the face */
            if (ina + (ina != inc) > 8 - m) return 0;
            if (ina) { memcpy(tmp[m], a, sizeof(tmp[m])); ++m; }
            if (ina != inc) {
                float t = da / (da - dc);
                for (int q = 0; q < 7; ++q) tmp[m][q] = a[q] + t * (c[q] - a[q]);
                ++m;
            }
        }
        n = m;
        if (n < 3) return 0;
        memcpy(poly, tmp, sizeof(float) * 7 * (size_t)n);
    }
    for (int i = 0; i < n; ++i)
        if (!(poly[i][3] > 0.0f)) return 0;
    int nsub = n - 2;
    for (int s = 0; s < nsub; ++s) {
        float sv[3][4], sb[3][3];
        const int idx[3] = {0, s + 1, s + 2};
        for (int k = 0; k < 3; ++k) {
            for (int c = 0; c < 4; ++c) sv[k][c] = poly[idx[k]][c];
            for (int i = 0; i < 3; ++i) sb[k][i] = poly[idx[k]][4 + i];
        }
        const float g2[2] = {2.0f * gx, 2.0f * gy};
        make_record((const float(*)[4])sv, (const float(*)[3])sb, W, H, f, &recs[s], g2);
    }
    return nsub;
}

static inline int rec_nonempty(const orc_rec *r) { return r->i0 <= r->i1; }

static inline void edge_values(const orc_rec *r, int i, int j, int64_t E[3])
{
    int64_t px = (int64_t)i * 256 + 128, py = (int64_t)j * 256 + 128;
    for (int k = 0; k < 3; ++k) E[k] = (int64_t)r->A[k] * px + (int64_t)r->B[k] * py + r->C[k];
}

static inline int inside(const orc_rec *r, const int64_t E[3])
{
    for (int k = 0; k < 3; ++k) {
        if (E[k] > 0) continue;
        if (E[k] == 0 && (r->A[k] > 0 || (r->A[k] == 0 && r->B[k] < 0))) continue;
        return 0;
    }
    return 1;
}

/* R4: returns 1 and the 24-bit depth if the sample passes the depth-range test */
static inline int sample_depth(const orc_rec *r, int i, int j, uint32_t *d)
{
    float fx = (float)i + 0.5f, fy = (float)j + 0.5f;
    float zw = fmaf(r->za, fx - r->fx0, fmaf(r->zb, fy - r->fy0, r->z0));
    if (!(zw >= 0.0f && zw <= 1.0f)) return 0;
    uint32_t q = (uint32_t)fmaf(zw, 16777215.0f, 0.5f);
    if (q >= DEPTH_MAX) return 0;
    *d = q;
    return 1;
}

/* R4 without the depth comparison (hill: GL_DEPTH_TEST off): inside the near/far range */
static inline int sample_in_range(const orc_rec *r, int i, int j)
{
    float fx = (float)i + 0.5f, fy = (float)j + 0.5f;
    float zw = fmaf(r->za, fx - r->fx0, fmaf(r->zb, fy - r->fy0, r->z0));
    return zw >= 0.0f && zw <= 1.0f;
}

/* R6: perspective-correct parent barycentrics from (possibly doubled) edge values */
static inline int parent_lambda(const orc_rec *r, const int64_t E[3], float lam[3])
{
    float a0 = (float)E[0] * r->iw[0], a1 = (float)E[1] * r->iw[1], a2 = (float)E[2] * r->iw[2];
    float s = (a0 + a1) + a2;
    if (s == 0.0f) return 0;
    float rs = 1.0f / s;
    float m0 = a0 * rs, m1 = a1 * rs, m2 = a2 * rs;
    for (int i = 0; i < 3; ++i) lam[i] = (m0 * r->basis[0 * 3 + i] + m1 * r->basis[1 * 3 + i]) + m2 * r->basis[2 * 3 + i];
    return 1;
}

static inline int64_t rec_index(int F, int f, int s) { return s == 0 ? f : (int64_t)F + 5 * (int64_t)f + (s - 1); }

/* ------------------------------------------------------------------------------------------------ */
/* Setup for a whole frame: recs has 6F slots, nsub F entries */
static int setup_frame(const float *verts, const int32_t *faces, int V, int F, int W, int H, orc_rec *recs, int32_t *nsub,
                       int32_t *clipped)
{
    int bad = 0;
    for (int64_t i = 0; i < 6 * (int64_t)F; ++i) { recs[i].i0 = 1; recs[i].i1 = 0; recs[i].face = -1; }
    for (int f = 0; f < F; ++f) {
        orc_rec tmp[MAX_SUB];
        const int32_t *f3 = faces + 3 * (int64_t)f;
        for (int k = 0; k < 3; ++k)
            if (f3[k] < 0 || f3[k] >= V) bad = 1;
        int cl = 0;
        int n = setup_face(verts, f3, V, W, H, f, tmp, &cl);
        nsub[f] = n;
        if (clipped) clipped[f] = cl;
        for (int s = 0; s < n; ++s) recs[rec_index(F, f, s)] = tmp[s];
    }
    return bad;
}

/* Forward: pixels [B,H,W,C] (rows top-first), gbuffer [B,H,W] record index or -1.
 * Returns 0, or 2 if a face index was out of range (such faces are culled). */
/* ------------------------------------------------------------------------------------------------ */
/* Fragment program 1: the fork's `oceanic_horizon` (csrc/shaders.cpp:1668-1919), restated in float32
 * with the operation order of the GLSL source and no contraction.  GLSL's sin/cos/pow are the driver's
 * (NVIDIA, unpinned); here they are fixed algorithms (OCEANIC.md-style spec in DESIGN.md §3b), written
 * identically in the HIP path, so oracle and GPU agree bit for bit.
 *   - sin/cos: 3-part Cody-Waite reduction by pi/2 (11+11+24-bit constants), cephes minimax polynomials;
 *   - pow(x,y), x in [0,1]: exp2(y*log2(x)); log2 via atanh series on m in [sqrt(1/2), sqrt(2)),
 *     exp2 via degree-6 polynomial, results below 2^-125 flush to 0 (as fp32 GLSL on the reference GPU);
 *   - normalize(v) = v / sqrt(dot(v,v)) (IEEE sqrt and division), dot = (x*x' + y*y') + z*z'.
 *   - water()'s sines: one reduction by pi and an odd degree-11 polynomial, written with explicit fmaf
 *     (correctly rounded on both sides, so still bit-identical) (ocn_sin_pi);
 * The water() terms multiplied by small_waveheight = 0.0 (shaders.cpp:1690,1776-1785) are exact zeros
 * (finite * 0) and are omitted. */

static float ocn_sincos(float x, int want_cos)
{
    if (!(fabsf(x) < 1.0e30f)) return x - x; /* NaN for inf / NaN */
    const float k = rintf(x * 0.636619772f);
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.549790126404332e-8f;
    float q = k - 4.0f * floorf(k * 0.25f); /* quadrant 0..3 (exact while |k| < 2^24) */
    if (want_cos) q = q + 1.0f;
    if (q >= 4.0f) q = q - 4.0f;
    const float z = r * r;
    const float s = r + (r * z) * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
    const float c = (1.0f - 0.5f * z) +
                    (z * z) * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    if (q == 0.0f) return s;
    if (q == 1.0f) return c;
    if (q == 2.0f) return -s;
    return -c;
}
static float ocn_sin(float x) { return ocn_sincos(x, 0); }

/* sin for water(): one reduction by pi (3.140625 + 9.675025939941406e-4 + 1.509958025e-7) and the odd
 * Taylor polynomial to x^11 on [-pi/2, pi/2] (1.5e-7 absolute error for |x| < 3000), sign by parity */
static float ocn_sin_pi(float x)
{
    if (!(fabsf(x) < 1.0e30f)) return x - x;
    const float k = rintf(x * 0.318309873f);
    float r = fmaf(-k, 3.140625f, x); /* explicit fused multiply-adds (correctly rounded in C and on the GPU) */
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
static float ocn_cos(float x) { return ocn_sincos(x, 1); }

static float ocn_bits_to_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ocn_f_to_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* log2(x) for normal x > 0 */
static float ocn_log2(float x)
{
    const uint32_t u = ocn_f_to_bits(x);
    float e = (float)((int)((u >> 23) & 0xffu) - 126);
    float m = ocn_bits_to_f((u & 0x807fffffu) | 0x3f000000u); /* [0.5, 1) */
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

/* 2^z for z <= 0 (pow of [0,1] by a positive exponent) */
static float ocn_exp2(float z)
{
    if (!(z >= -125.0f)) return 0.0f; /* also NaN -> 0 */
    const float n = floorf(z + 0.5f);
    const float f = z - n; /* [-0.5, 0.5] */
    const float p = 1.0f + f * (0.6931471806f + f * (0.2402265070f + f * (0.05550410866f + f * (0.009618129108f +
                    f * (0.001333355815f + f * 0.0001540353039f)))));
    return ldexpf(p, (int)n);
}

/* GLSL pow(x, y) for x = clamp(...) in [0,1], y > 0 */
static float ocn_pow01(float x, float y)
{
    if (!(x >= 1.17549435e-38f)) return 0.0f; /* 0, denormal (flushed) or NaN */
    if (x >= 1.0f) return 1.0f;
    return ocn_exp2(y * ocn_log2(x));
}

static float ocn_clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
static float ocn_sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
static float ocn_dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static void ocn_normalize(float v[3])
{
    const float l = sqrtf(ocn_dot3(v, v));
    v[0] = v[0] / l; v[1] = v[1] / l; v[2] = v[2] / l;
}

/* water(p), shaders.cpp:1760-1791 with small_waveheight = 0 */
static float ocn_water(float px, float py, float time)
{
    float height = 70.0f;
    const float shift2x = 0.001f * ((time * 190.0f) * 2.0f);
    float wave = 0.0f;
    wave = wave + ocn_sin_pi(px * 0.021f + shift2x) * 4.5f;
    wave = wave + ocn_sin_pi((px * 0.0172f + py * 0.010f) + shift2x * 1.121f) * 4.0f;
    wave = wave - ocn_sin_pi((px * 0.00104f + py * 0.005f) + shift2x * 0.121f) * 4.0f;
    wave = wave + ocn_sin_pi((px * 0.02221f + py * 0.01233f) + shift2x * 3.437f) * 5.0f;
    wave = wave + ocn_sin_pi((px * 0.03112f + py * 0.01122f) + shift2x * 4.269f) * 2.5f;
    wave = wave * 1.0f; /* large_waveheight */
    height = height + wave;
    return height;
}

/* trace(), shaders.cpp:1817-1856 (RENDER_GODRAYS undefined -> fog stays 0) */
static int ocn_trace(const float ro[3], const float rd[3], float time, float *dist)
{
    float t = -ro[1] / rd[1];
    float st = 0.5f;
    float old_h = 0.0f;
    for (int j = 1000; j < 1020; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p0 = ro[0] + t * rd[0], p1 = ro[1] + t * rd[1], p2 = ro[2] + t * rd[2];
        const float h = p1 - ocn_water(p0, p2, time);
        t = t + (fmaxf(1.0f, fabsf(h)) * ocn_sign(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    *dist = t;
    return !(rd[1] > 0.0f);
}

/* main(), shaders.cpp:1858-1917: xy = texCoordV + jitter; writes (col.x, col.y) */
static void ocn_shade(float xyx, float xyy, const float *cam, float width, float height, float out[2])
{
    const float ro[3] = {cam[0], cam[1], cam[2]};
    const float time = cam[6];
    float light[3] = {0.1f, 0.25f, cam[7]};
    ocn_normalize(light);
    float rdv[3];
    rdv[0] = (xyx + 1.0f) * width / 2.0f - width / 2.0f;
    rdv[1] = (xyy + 1.0f) * height / 2.0f - height / 2.0f;
    rdv[2] = 1.73f * width / 2.0f;
    ocn_normalize(rdv);
    const float sin1 = ocn_sin(cam[3]), cos1 = ocn_cos(cam[3]);
    const float sin2 = ocn_sin(cam[4]), cos2 = ocn_cos(cam[4]);
    const float sin3 = ocn_sin(cam[5]), cos3 = ocn_cos(cam[5]);
    float rd[3];
    rd[0] = ((cos2 * cos3) * rdv[0] + (-cos1 * sin3 + (sin1 * sin2) * cos3) * rdv[1]) +
            (sin1 * sin3 + (cos1 * sin2) * cos3) * rdv[2];
    rd[1] = ((cos2 * sin3) * rdv[0] + (cos1 * cos3 + (sin1 * sin2) * sin3) * rdv[1]) +
            (-sin1 * cos3 + (cos1 * sin2) * sin3) * rdv[2];
    rd[2] = (-sin2 * rdv[0] + (sin1 * cos2) * rdv[1]) + (cos1 * cos2) * rdv[2];
    float sundot = ocn_clamp01(ocn_dot3(rd, light));
    float dist = 0.0f;
    if (!ocn_trace(ro, rd, time, &dist)) {
        out[0] = 1.0f;
        out[1] = ocn_pow01(sundot, 350.0f);
        return;
    }
    out[0] = 0.0f;
    const float wx = ro[0] + dist * rd[0], wz = ro[2] + dist * rd[2];
    const float d = 0.1f * 1.0f * 4.0f; /* 0.1 * wavegain * 4 */
    float n[3] = {ocn_water(wx - d, wz, time) - ocn_water(wx + d, wz, time), 1.0f,
                  ocn_water(wx, wz - d, time) - ocn_water(wx, wz + d, time)};
    ocn_normalize(n);
    const float dn = 2.0f * ocn_dot3(n, rd); /* reflect(I, N) = I - 2 dot(N, I) N */
    const float rr[3] = {rd[0] - dn * n[0], rd[1] - dn * n[1], rd[2] - dn * n[2]};
    sundot = ocn_clamp01(ocn_dot3(rr, light));
    out[1] = (0.5f * ocn_pow01(sundot, 10.0f) + 0.25f * ocn_pow01(sundot, 3.5f)) + 0.75f * ocn_pow01(sundot, 300.0f);
}

/* ------------------------------------------------------------------------------------------------ */
/* The `oceanic` family: `oceanic` (bound by RasteriseGrad, shaders.cpp:556-864),
 * `oceanic_still_cloud` (:866-1176), `oceanic_no_cloud` (:1402-1666) and `oceanic_simple_proxy`
 * (:1921-2185) are one program with different constants, wave function, loop counts and cloud mode
 * (the diffs of those four GLSL sources).  Same rules as above: GLSL operation order in float32, no
 * contraction, the fixed transcendentals; mat*vec as (c0*x + c1*y) + c2*z over the columns; v *= M as
 * the row-vector product; mix(a,b,t) = a*(1-t) + b*t; smoothstep per the GLSL definition; fract(x) =
 * x - floor(x); exp(x) = exp2(x * log2(e)); pow(x,y) = exp2(y * log2(x)) for x > 0, 0 for x <= 0.  The
 * god-ray term (RENDER_GODRAYS undefined) is the exact zero `vec3(..)*fog` and is omitted. */

typedef struct {
    float wavegain, large_wh, small_wh;
    float fogcolor[3], skybottom[3], skytop[3], reflskycolor[3], watercolor[3];
    float s1x, s1y, s2x, s2y; /* shift1 = 0.001*vec2(time*s1x*2, time*s1y*2), shift2 = 0.001*vec2(time*s2x*2, -time*s2y*2) */
    int wave_cos;             /* large waves use cos (simple_proxy) instead of sin */
    int small_iters;          /* 7, or 3 (simple_proxy) */
    int march_steps;          /* 20, or 10 (simple_proxy) */
    int clouds;               /* 0 none (trace_fog = 1), 1 moving with the camera (time), 2 still (cloud_t) */
} ocn_family;

static const ocn_family OCN_OCEANIC = {1.0f, 1.0f, 1.0f, {0.5f, 0.7f, 1.1f}, {0.6f, 0.8f, 1.2f}, {0.05f, 0.2f, 0.5f},
                                       {0.025f, 0.10f, 0.20f}, {0.2f, 0.25f, 0.3f}, 160.0f, 120.0f, 190.0f, 130.0f,
                                       0, 7, 20, 1};
static const ocn_family OCN_STILL = {1.0f, 1.0f, 1.0f, {0.5f, 0.7f, 1.1f}, {0.6f, 0.8f, 1.2f}, {0.05f, 0.2f, 0.5f},
                                     {0.025f, 0.10f, 0.20f}, {0.2f, 0.25f, 0.3f}, 160.0f, 120.0f, 190.0f, 130.0f,
                                     0, 7, 20, 2};
static const ocn_family OCN_NOCLOUD = {1.0f, 1.0f, 1.0f, {0.5f, 0.7f, 1.1f}, {0.6f, 0.8f, 1.2f}, {0.05f, 0.2f, 0.5f},
                                       {0.025f, 0.10f, 0.20f}, {0.2f, 0.25f, 0.3f}, 160.0f, 120.0f, 190.0f, 130.0f,
                                       0, 7, 20, 0};
static const ocn_family OCN_PROXY = {0.75f, 0.75f, 1.5f, {0.4f, 0.4f, 1.2f}, {0.5f, 0.5f, 1.3f}, {0.15f, 0.1f, 0.7f},
                                     {0.1f, 0.1f, 0.15f}, {0.1f, 0.2f, 0.5f}, 260.0f, 100.0f, 150.0f, 230.0f,
                                     1, 3, 10, 0};

static float ocn_fract(float x) { return x - floorf(x); }
static float ocn_mix(float a, float b, float t) { return a * (1.0f - t) + b * t; }
static float ocn_smoothstep(float e0, float e1, float x)
{
    const float t = ocn_clamp01((x - e0) / (e1 - e0));
    return t * t * (3.0f - 2.0f * t);
}
static float ocn_exp2_any(float z)
{
    if (!(z >= -125.0f)) return 0.0f; /* also NaN */
    if (z > 128.0f) return INFINITY;
    const float n = floorf(z + 0.5f);
    const float f = z - n;
    const float p = 1.0f + f * (0.6931471806f + f * (0.2402265070f + f * (0.05550410866f + f * (0.009618129108f +
                    f * (0.001333355815f + f * 0.0001540353039f)))));
    return ldexpf(p, (int)n);
}
static float ocn_pow_pos(float x, float y) /* GLSL pow for any x (0 for x <= 0) */
{
    if (!(x >= 1.17549435e-38f)) return 0.0f;
    if (x == 1.0f) return 1.0f;
    if (!(x < INFINITY)) return INFINITY;
    return ocn_exp2_any(y * ocn_log2(x));
}
static float ocn_exp(float x) { return ocn_exp2_any(x * 1.44269504f); }

static float ocn_hash(float n) { return ocn_fract(ocn_cos(n) * 41415.92653f); }
static float ocn_rand2(float nx, float ny) { return ocn_fract(ocn_sin_pi(nx * 12.9898f + ny * 4.1414f) * 43758.5453f); }

static float ocn_noise2(float px, float py)
{
    const float ix = floorf(px), iy = floorf(py);
    float ux = ocn_fract(px), uy = ocn_fract(py);
    ux = ux * ux * (3.0f - 2.0f * ux);
    uy = uy * uy * (3.0f - 2.0f * uy);
    return ocn_mix(ocn_mix(ocn_rand2(ix, iy), ocn_rand2(ix + 1.0f, iy + 0.0f), ux),
                   ocn_mix(ocn_rand2(ix + 0.0f, iy + 1.0f), ocn_rand2(ix + 1.0f, iy + 1.0f), ux), uy);
}

static float ocn_noise3(float x, float y, float z)
{
    const float px = floorf(x), py = floorf(y), pz = floorf(z);
    const float fx = ocn_smoothstep(0.0f, 1.0f, ocn_fract(x));
    const float fy = ocn_smoothstep(0.0f, 1.0f, ocn_fract(y));
    const float fz = ocn_smoothstep(0.0f, 1.0f, ocn_fract(z));
    const float n = (px + py * 57.0f) + 113.0f * pz;
    return ocn_mix(ocn_mix(ocn_mix(ocn_hash(n + 0.0f), ocn_hash(n + 1.0f), fx),
                           ocn_mix(ocn_hash(n + 57.0f), ocn_hash(n + 58.0f), fx), fy),
                   ocn_mix(ocn_mix(ocn_hash(n + 113.0f), ocn_hash(n + 114.0f), fx),
                           ocn_mix(ocn_hash(n + 170.0f), ocn_hash(n + 171.0f), fx), fy), fz);
}

/* mat3 m = mat3(0.00,1.60,1.20, -1.60,0.72,-0.96, -1.20,-0.96,1.28) (columns), m*p */
static void ocn_m3(float p[3])
{
    const float x = p[0], y = p[1], z = p[2];
    p[0] = (0.00f * x + -1.60f * y) + -1.20f * z;
    p[1] = (1.60f * x + 0.72f * y) + -0.96f * z;
    p[2] = (1.20f * x + -0.96f * y) + 1.28f * z;
}

static float ocn_fbm3(float x, float y, float z)
{
    float p[3] = {x, y, z};
    float f = 0.5000f * ocn_noise3(p[0], p[1], p[2]);
    ocn_m3(p); p[0] = p[0] * 1.1f; p[1] = p[1] * 1.1f; p[2] = p[2] * 1.1f;
    f = f + 0.2500f * ocn_noise3(p[0], p[1], p[2]);
    ocn_m3(p); p[0] = p[0] * 1.2f; p[1] = p[1] * 1.2f; p[2] = p[2] * 1.2f;
    f = f + 0.1666f * ocn_noise3(p[0], p[1], p[2]);
    ocn_m3(p);
    f = f + 0.0834f * ocn_noise3(p[0], p[1], p[2]);
    return f;
}

/* mat2 m2 = mat2(1.6,-1.2, 1.2,1.6) (columns), m2*p */
static float ocn_fbm2(float x, float y)
{
    float f = 0.5000f * ocn_noise2(x, y);
    float nx = 1.6f * x + 1.2f * y, ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.2500f * ocn_noise2(x, y);
    nx = 1.6f * x + 1.2f * y; ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.1666f * ocn_noise2(x, y);
    nx = 1.6f * x + 1.2f * y; ny = -1.2f * x + 1.6f * y; x = nx; y = ny;
    f = f + 0.0834f * ocn_noise2(x, y);
    return f;
}

static float ocn_family_water(const ocn_family *P, float px, float py, float time)
{
    float height = 70.0f;
    float s1x = 0.001f * ((time * P->s1x) * 2.0f), s1y = 0.001f * ((time * P->s1y) * 2.0f);
    const float s2x = 0.001f * ((time * P->s2x) * 2.0f), s2y = 0.001f * ((-time * P->s2y) * 2.0f);
    float wave = 0.0f;
    if (P->wave_cos) {
        wave = wave + ocn_cos(px * 0.021f + s2x) * 4.5f;
        wave = wave + ocn_cos((px * 0.0172f + py * 0.010f) + s2x * 1.121f) * 4.0f;
        wave = wave - ocn_cos((px * 0.00104f + py * 0.005f) + s2x * 0.121f) * 4.0f;
        wave = wave + ocn_cos((px * 0.02221f + py * 0.01233f) + s2x * 3.437f) * 5.0f;
        wave = wave + ocn_cos((px * 0.03112f + py * 0.01122f) + s2x * 4.269f) * 2.5f;
    } else {
        wave = wave + ocn_sin_pi(px * 0.021f + s2x) * 4.5f;
        wave = wave + ocn_sin_pi((px * 0.0172f + py * 0.010f) + s2x * 1.121f) * 4.0f;
        wave = wave - ocn_sin_pi((px * 0.00104f + py * 0.005f) + s2x * 0.121f) * 4.0f;
        wave = wave + ocn_sin_pi((px * 0.02221f + py * 0.01233f) + s2x * 3.437f) * 5.0f;
        wave = wave + ocn_sin_pi((px * 0.03112f + py * 0.01122f) + s2x * 4.269f) * 2.5f;
    }
    wave = wave * P->large_wh;
    wave = wave - (ocn_fbm2(px * 0.004f - s2x * 0.5f, py * 0.004f - s2y * 0.5f) * P->small_wh) * 24.0f;
    float amp = 6.0f * P->small_wh;
    s1x = s1x * 0.3f; s1y = s1y * 0.3f;
    const float m00 = 1.6f * 0.9331f, m01 = -1.2f * 0.9331f, m10 = 1.2f * 0.9331f, m11 = 1.6f * 0.9331f;
    for (int i = 0; i < P->small_iters; ++i) {
        wave = wave - fabsf(ocn_sin_pi((ocn_noise2(px * 0.01f + s1x, py * 0.01f + s1y) - 0.5f) * 3.14f)) * amp;
        amp = amp * 0.51f;
        s1x = s1x * 1.841f; s1y = s1y * 1.841f;
        const float nx = px * m00 + py * m01, ny = px * m10 + py * m11; /* p *= m2*0.9331 (row vector) */
        px = nx; py = ny;
    }
    height = height + wave;
    return height;
}
/* trace_fog (cloud cover along a ray, 10 layers; 1 without clouds) */
static float ocn_family_trace_fog(const ocn_family *P, const float ro[3], const float rd[3], const float *cam)
{
    if (P->clouds == 0) return 1.0f;
    const float ct = P->clouds == 2 ? cam[8] : cam[6];
    const float shx = ct * 80.0f, shy = ct * 60.0f;
    float sum = 0.0f, q2 = 0.0f, q3 = 0.0f;
    for (int q = 0; q < 10; ++q) {
        float cx, cy, cz;
        if (P->clouds == 1) {
            const float c = ((q2 + 350.0f) - ro[1]) / rd[1];
            cx = (ro[0] + c * rd[0]) + 831.0f;
            cy = (ro[1] + c * rd[1]) + ((321.0f + q3) - shx * 0.2f);
            cz = (ro[2] + c * rd[2]) + (1330.0f + shy * 3.0f);
        } else {
            const float c = (q2 + 350.0f) / rd[1];
            cx = c * rd[0] + 831.0f;
            cy = c * rd[1] + ((321.0f + q3) - shx * 0.2f);
            cz = c * rd[2] + (1330.0f + shy * 3.0f);
        }
        const float alpha = ocn_smoothstep(0.5f, 1.0f, ocn_fbm3(cx * 0.0015f, cy * 0.0015f, cz * 0.0015f));
        sum = sum + (1.0f - sum) * alpha;
        if (sum > 0.98f) break;
        q2 = q2 + 120.0f;
        q3 = q3 + 0.15f;
    }
    return ocn_clamp01(1.0f - sum);
}

/* main() of the family: writes col.xyz */
static void ocn_family_shade(const ocn_family *P, float xyx, float xyy, const float *cam, float width, float height,
                             float out[3])
{
    const float ro[3] = {cam[0], cam[1], cam[2]};
    const float time = cam[6];
    float light[3] = {0.1f, 0.25f, cam[7]};
    ocn_normalize(light);
    float rdv[3];
    rdv[0] = (xyx + 1.0f) * width / 2.0f - width / 2.0f;
    rdv[1] = (xyy + 1.0f) * height / 2.0f - height / 2.0f;
    rdv[2] = 1.73f * width / 2.0f;
    ocn_normalize(rdv);
    const float sin1 = ocn_sin(cam[3]), cos1 = ocn_cos(cam[3]);
    const float sin2 = ocn_sin(cam[4]), cos2 = ocn_cos(cam[4]);
    const float sin3 = ocn_sin(cam[5]), cos3 = ocn_cos(cam[5]);
    float rd[3];
    rd[0] = ((cos2 * cos3) * rdv[0] + (-cos1 * sin3 + (sin1 * sin2) * cos3) * rdv[1]) +
            (sin1 * sin3 + (cos1 * sin2) * cos3) * rdv[2];
    rd[1] = ((cos2 * sin3) * rdv[0] + (cos1 * cos3 + (sin1 * sin2) * sin3) * rdv[1]) +
            (-sin1 * cos3 + (cos1 * sin2) * sin3) * rdv[2];
    rd[2] = (-sin2 * rdv[0] + (sin1 * cos2) * rdv[1]) + (cos1 * cos2) * rdv[2];
    const float sundot = ocn_clamp01(ocn_dot3(rd, light));
    if (rd[1] > 0.0f) {
        /* sky (trace() returns false; its march is not read) */
        const float t = ocn_pow_pos(1.0f - 0.7f * rd[1], 15.0f);
        float col[3];
        const float p350 = ocn_pow_pos(sundot, 350.0f), p2 = ocn_pow_pos(sundot, 2.0f);
        const float sunc[3] = {0.47f * 1.6f, 0.47f * 1.4f, 0.47f * 1.0f}, haze[3] = {0.4f * 0.8f, 0.4f * 0.9f, 0.4f * 1.0f};
        for (int k = 0; k < 3; ++k) {
            col[k] = 0.8f * (P->skybottom[k] * t + P->skytop[k] * (1.0f - t));
            col[k] = col[k] + sunc[k] * p350;
            col[k] = col[k] + haze[k] * p2;
        }
        if (P->clouds != 0) {
            const float ct = P->clouds == 2 ? cam[8] : time;
            const float shx = ct * 80.0f, shy = ct * 60.0f;
            float sum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            const float dense[3] = {0.7f * 0.4f, 0.7f * 0.4f, 0.7f * 0.3f}, light_c[3] = {1.1f, 1.05f, 1.0f};
            for (int q = 1000; q < 1100; ++q) {
                const float fq = (float)(q - 1000);
                float cx, cy, cz;
                if (P->clouds == 1) {
                    const float c = ((fq * 12.0f + 350.0f) - cam[1]) / rd[1];
                    cx = (ro[0] + c * rd[0]) + 831.0f;
                    cy = (ro[1] + c * rd[1]) + ((321.0f + fq * 0.15f) - shx * 0.2f);
                    cz = (ro[2] + c * rd[2]) + (1330.0f + shy * 3.0f);
                } else {
                    const float c = (fq * 12.0f + 350.0f) / rd[1];
                    cx = c * rd[0] + 831.0f;
                    cy = c * rd[1] + ((321.0f + fq * 0.15f) - shx * 0.2f);
                    cz = c * rd[2] + (1330.0f + shy * 3.0f);
                }
                float alpha = ocn_smoothstep(0.5f, 1.0f, ocn_fbm3(cx * 0.0015f, cy * 0.0015f, cz * 0.0015f)) * 0.9f;
                float lc[3];
                for (int k = 0; k < 3; ++k) lc[k] = ocn_mix(light_c[k], dense[k], alpha);
                alpha = (1.0f - sum[3]) * alpha;
                for (int k = 0; k < 3; ++k) sum[k] = sum[k] + lc[k] * alpha;
                sum[3] = sum[3] + alpha;
                if (sum[3] > 0.98f) break;
            }
            const float alpha = ocn_smoothstep(0.7f, 1.0f, sum[3]);
            const float p13 = ocn_pow_pos(sundot, 13.0f), p5 = ocn_pow_pos(sundot, 5.0f);
            const float shade_c[3] = {0.6f * 0.8f, 0.6f * 0.75f, 0.6f * 0.7f}, scat[3] = {0.2f * 1.3f, 0.2f * 1.2f, 0.2f * 1.0f};
            for (int k = 0; k < 3; ++k) {
                sum[k] = sum[k] / (sum[3] + 0.0001f);
                sum[k] = sum[k] - (shade_c[k] * p13) * alpha;
                sum[k] = sum[k] + (scat[k] * p5) * (1.0f - alpha);
                col[k] = ocn_mix(col[k], sum[k], sum[3] * (1.0f - t));
            }
        }
        out[0] = col[0]; out[1] = col[1]; out[2] = col[2];
        return;
    }
    /* trace(), shaders.cpp:700-744 */
    float t = -ro[1] / rd[1];
    float st = 0.5f, old_h = 0.0f;
    for (int j = 0; j < P->march_steps; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p0 = ro[0] + t * rd[0], p1 = ro[1] + t * rd[1], p2 = ro[2] + t * rd[2];
        const float h = p1 - ocn_family_water(P, p0, p2, time);
        t = t + (fmaxf(1.0f, fabsf(h)) * ocn_sign(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    const float dist = t;
    const float wpos[3] = {ro[0] + dist * rd[0], ro[1] + dist * rd[1], ro[2] + dist * rd[2]};
    const float d = 0.1f * P->wavegain * 4.0f;
    float n[3] = {ocn_family_water(P, wpos[0] - d, wpos[2], time) - ocn_family_water(P, wpos[0] + d, wpos[2], time), 1.0f,
                  ocn_family_water(P, wpos[0], wpos[2] - d, time) - ocn_family_water(P, wpos[0], wpos[2] + d, time)};
    ocn_normalize(n);
    const float dn = 2.0f * ocn_dot3(n, rd);
    const float rr[3] = {rd[0] - dn * n[0], rd[1] - dn * n[1], rd[2] - dn * n[2]};
    const float up[3] = {0.0f, 1.0f, 0.0f};
    const float refl = 1.0f - ocn_clamp01(ocn_dot3(rr, up));
    const float fro[3] = {wpos[0] + 20.0f * rr[0], wpos[1] + 20.0f * rr[1], wpos[2] + 20.0f * rr[2]};
    const float sh = ocn_smoothstep(0.2f, 1.0f, ocn_family_trace_fog(P, fro, rr, cam)) * 0.7f + 0.3f;
    const float wsky = refl * sh, wwater = (1.0f - refl) * sh;
    const float sd = ocn_clamp01(ocn_dot3(rr, light));
    const float lift = (wpos[1] - 70.0f) + 30.0f;
    const float tint[3] = {0.003f, 0.005f, 0.005f};
    const float wsunrefl = wsky * ((0.5f * ocn_pow_pos(sd, 10.0f) + 0.25f * ocn_pow_pos(sd, 3.5f)) +
                                   0.75f * ocn_pow_pos(sd, 300.0f));
    const float sunw[3] = {1.5f, 1.3f, 1.0f};
    const float fo = 1.0f - ocn_exp(-ocn_pow_pos(0.0003f * dist, 1.5f));
    const float p4 = ocn_pow_pos(sd, 4.0f);
    const float fogc[3] = {0.6f * 0.6f, 0.6f * 0.5f, 0.6f * 0.4f};
    for (int k = 0; k < 3; ++k) {
        float c = wsky * P->reflskycolor[k];
        c = c + wwater * P->watercolor[k];
        c = c + tint[k] * lift;
        c = c + sunw[k] * wsunrefl;
        const float fco = P->fogcolor[k] + fogc[k] * p4;
        out[k] = ocn_mix(c, fco, fo);
    }
}

/* texCoordV = perspective-correct interpolation of the vertices' clip xy (shaders.cpp:19,21 alias
 * texCoord to position); jitter = background texel at (texCoordV+1)/2 (NEAREST; at texel centres the
 * reference's LINEAR magnification returns the same texel), channels x,y (C=1 broadcast,
 * rasterise_egl.cu:39-47) divided by (width, height) (shaders.cpp:1865-1867) */
void oracle_oceanic_horizon_pixel(const float *bgframe, int H, int W, int C, float tx, float ty, const float *cam,
                                  float out[2])
{
    const float u = (tx + 1.0f) / 2.0f, v = (ty + 1.0f) / 2.0f;
    int ix = (int)floorf(u * (float)W), iy = (int)floorf(v * (float)H);
    if (!(u * (float)W >= 0.0f)) ix = 0;
    if (!(v * (float)H >= 0.0f)) iy = 0;
    ix = ix < 0 ? 0 : (ix > W - 1 ? W - 1 : ix);
    iy = iy < 0 ? 0 : (iy > H - 1 ? H - 1 : iy);
    const float *texel = bgframe + (((int64_t)(H - 1 - iy)) * W + ix) * C;
    const float sx = texel[0], sy = C >= 2 ? texel[1] : texel[0];
    ocn_shade(tx + sx / (float)W, ty + sy / (float)H, cam, (float)W, (float)H, out);
}

/* shader ids 2..5 (include/dirt_mi355x.h): the oceanic family; writes col.xyz */
void oracle_oceanic_family_pixel(int shader_id, const float *bgframe, int H, int W, int C, float tx, float ty,
                                 const float *cam, float out[3])
{
    const ocn_family *P = shader_id == 2 ? &OCN_OCEANIC : shader_id == 3 ? &OCN_STILL
                          : shader_id == 4 ? &OCN_NOCLOUD : &OCN_PROXY;
    const float u = (tx + 1.0f) / 2.0f, v = (ty + 1.0f) / 2.0f;
    int ix = (int)floorf(u * (float)W), iy = (int)floorf(v * (float)H);
    if (!(u * (float)W >= 0.0f)) ix = 0;
    if (!(v * (float)H >= 0.0f)) iy = 0;
    ix = ix < 0 ? 0 : (ix > W - 1 ? W - 1 : ix);
    iy = iy < 0 ? 0 : (iy > H - 1 ? H - 1 : iy);
    const float *texel = bgframe + (((int64_t)(H - 1 - iy)) * W + ix) * C;
    const float sx = texel[0], sy = C >= 2 ? texel[1] : texel[0];
    ocn_family_shade(P, tx + sx / (float)W, ty + sy / (float)H, cam, (float)W, (float)H, out);
}

/* ------------------------------------------------------------------------------------------------ */
/* oceanic_opt_flow (shader id 6), shaders.cpp:1178-1398, op csrc/oceanic_opt_flow.cpp.  Optical flow
 * of a flat sea: water() is the constant waterlevel - 12 = 58 (:1283-1286), no jitter (:1323-1325 are
 * commented out).  camera_pos (oceanic_opt_flow.cpp:399-414): [0..7] as the family, [9] dt, [10..12]
 * dx,dy,dz, [13..15] dang1..3 ([8] is not read).  Writes new_coord = the pixel position of the same
 * world point in the previous frame (:1376-1395; fragColor.xy, z = 0, w = 1). */
void oracle_opt_flow_pixel(float xyx, float xyy, const float *cam, float width, float height, float out[2])
{
    const float ro[3] = {cam[0], cam[1], cam[2]};
    const float dt = cam[9];
    float rdv[3];
    rdv[0] = (xyx + 1.0f) * width / 2.0f - width / 2.0f;
    rdv[1] = (xyy + 1.0f) * height / 2.0f - height / 2.0f;
    rdv[2] = 1.73f * width / 2.0f;
    ocn_normalize(rdv);
    float sin1 = ocn_sin(cam[3]), cos1 = ocn_cos(cam[3]);
    float sin2 = ocn_sin(cam[4]), cos2 = ocn_cos(cam[4]);
    float sin3 = ocn_sin(cam[5]), cos3 = ocn_cos(cam[5]);
    float rd[3];
    rd[0] = ((cos2 * cos3) * rdv[0] + (-cos1 * sin3 + (sin1 * sin2) * cos3) * rdv[1]) +
            (sin1 * sin3 + (cos1 * sin2) * cos3) * rdv[2];
    rd[1] = ((cos2 * sin3) * rdv[0] + (cos1 * cos3 + (sin1 * sin2) * sin3) * rdv[1]) +
            (-sin1 * cos3 + (cos1 * sin2) * sin3) * rdv[2];
    rd[2] = (-sin2 * rdv[0] + (sin1 * cos2) * rdv[1]) + (cos1 * cos2) * rdv[2];
    /* the previous frame's angles (:1337-1342) */
    sin1 = ocn_sin(cam[3] - cam[13] * dt); cos1 = ocn_cos(cam[3] - cam[13] * dt);
    sin2 = ocn_sin(cam[4] - cam[14] * dt); cos2 = ocn_cos(cam[4] - cam[14] * dt);
    sin3 = ocn_sin(cam[5] - cam[15] * dt); cos3 = ocn_cos(cam[5] - cam[15] * dt);
    /* trace(), :1288-1321, against the constant water height */
    float t = -ro[1] / rd[1];
    float st = 0.5f, old_h = 0.0f;
    for (int j = 1000; j < 1020; ++j) {
        if (t > 500.0f) st = 1.0f;
        if (t > 800.0f) st = 2.0f;
        if (t > 1500.0f) st = 3.0f;
        const float p1 = ro[1] + t * rd[1];
        const float h = p1 - 58.0f;
        t = t + (fmaxf(1.0f, fabsf(h)) * ocn_sign(h)) * st;
        if (old_h * h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    float od[3];
    if (rd[1] > 0.0f) {
        od[0] = rd[0]; od[1] = rd[1]; od[2] = rd[2];
    } else {
        const float dv[3] = {cam[10], cam[11], cam[12]};
        for (int k = 0; k < 3; ++k) {
            const float wpos = ro[k] + t * rd[k];
            const float old_cam = ro[k] - dv[k] * dt;
            od[k] = wpos - old_cam;
        }
    }
    /* inverse rotation at the previous angles, projection (:1376-1393) */
    float ox = ((cos2 * cos3) * od[0] + (cos2 * sin3) * od[1]) - sin2 * od[2];
    float oy = ((-cos1 * sin3 + (sin1 * sin2) * cos3) * od[0] + (cos1 * cos3 + (sin1 * sin2) * sin3) * od[1]) +
               (sin1 * cos2) * od[2];
    const float oz = ((sin1 * sin3 + (cos1 * sin2) * cos3) * od[0] + (-sin1 * cos3 + (cos1 * sin2) * sin3) * od[1]) +
                     (cos1 * cos2) * od[2];
    ox = ox / oz;
    oy = oy / oz;
    const float s = 1.73f * width / 2.0f;
    ox = ox * s;
    oy = oy * s;
    out[0] = ox + width / 2.0f;
    out[1] = oy + height / 2.0f;
}

/* ------------------------------------------------------------------------------------------------ */
/* hill (shader id 7), shaders.cpp:123-554, op csrc/hill.cpp.  David Hoskins' "rolling hills" over a
 * terrain lookup texture: the background tensor (any of 1/3/4 channels, hill.cpp:310 does not check the
 * channel count) uploaded like every background (rasterise_egl.cu:16-47: rows flipped, C=1 broadcast,
 * alpha 1 for C<4) into a GL_LINEAR / CLAMP_TO_EDGE texture (hill.cpp:232-236); .x = terrain height,
 * .yzw = normal.  camera_pos: 12 floats (hill.cpp:395-407); r00..r22 are shadowed by main()'s local
 * constants (shaders.cpp:473-481), so only o0,o1,o2 = [9],[10],[11] are read.  Same float32 rules as the
 * oceanic programs; additionally: texture() = bilinear in float32 at texel centres (i+0.5)/W, with
 * weights a = x - floor(x) (the driver's fixed-point filter weights are not emulated); pow(x, 2.0) with a
 * possibly negative x (DoLighting) = x*x; uninitialised old_h in Scene() = 0. */
typedef struct {
    const float *tex; /* one frame, [H][W][C], rows top-first */
    int H, W, C;
} hill_tex;

static void hill_texel(const hill_tex *T, int i, int j, int nch, float out[4])
{
    i = i < 0 ? 0 : (i > T->W - 1 ? T->W - 1 : i);
    j = j < 0 ? 0 : (j > T->H - 1 ? T->H - 1 : j);
    const float *p = T->tex + ((int64_t)(T->H - 1 - j) * T->W + i) * T->C;
    out[0] = p[0];
    if (nch == 1) return;
    if (T->C == 1) { out[1] = p[0]; out[2] = p[0]; out[3] = 1.0f; }
    else if (T->C == 3) { out[1] = p[1]; out[2] = p[2]; out[3] = 1.0f; }
    else { out[1] = p[1]; out[2] = p[2]; out[3] = p[3]; }
}

/* texture(TerrainLookup, (u,v)) for u,v in [0,1]; nch = 1 (.x only) or 4 */
static void hill_sample(const hill_tex *T, float u, float v, int nch, float out[4])
{
    const float x = u * (float)T->W - 0.5f, y = v * (float)T->H - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, b = y - fy;
    const int i0 = (int)fx, j0 = (int)fy;
    float t00[4], t10[4], t01[4], t11[4];
    hill_texel(T, i0, j0, nch, t00);
    hill_texel(T, i0 + 1, j0, nch, t10);
    hill_texel(T, i0, j0 + 1, nch, t01);
    hill_texel(T, i0 + 1, j0 + 1, nch, t11);
    for (int k = 0; k < nch; ++k) {
        const float r0 = t00[k] * (1.0f - a) + t10[k] * a;
        const float r1 = t01[k] * (1.0f - a) + t11[k] * a;
        out[k] = r0 * (1.0f - b) + r1 * b;
    }
}

/* Terrain(p.xz).x (:219-227): texture coordinate clamp(scaled_p.yx, 0, 1) */
static float hill_terrain(const hill_tex *T, float px, float pz)
{
    const float sx = (px - -14.0f) / 28.0f, sz = (pz - 5.0f) / 20.0f;
    float t[4];
    hill_sample(T, ocn_clamp01(sz), ocn_clamp01(sx), 1, t);
    return t[0] * 10.3f - 6.1f;
}

/* Terrain_normal(p.xz) (:229-237) */
static void hill_terrain_normal(const hill_tex *T, float px, float pz, float n[3])
{
    const float sx = (px - -14.0f) / 28.0f, sz = (pz - 5.0f) / 20.0f;
    float t[4];
    hill_sample(T, ocn_clamp01(sz), ocn_clamp01(sx), 4, t);
    n[0] = t[1] * 2.0f - 1.0f; n[1] = t[2] * 2.0f - 1.0f; n[2] = t[3] * 2.0f - 1.0f;
}

/* Hash(float) / Hash(vec2), MOD2 = (3.07965, 7.4235) (:160-175) */
static float hill_hash1(float p)
{
    float x = ocn_fract(p / 3.07965f), y = ocn_fract(p / 7.4235f);
    const float d = y * (x + 19.19f) + x * (y + 19.19f);
    x = x + d; y = y + d;
    return ocn_fract(x * y);
}
static float hill_hash2(float px, float py)
{
    float x = ocn_fract(px / 3.07965f), y = ocn_fract(py / 7.4235f);
    const float d = x * (y + 19.19f) + y * (x + 19.19f);
    x = x + d; y = y + d;
    return ocn_fract(x * y);
}

/* Noise(vec2) (:179-189) */
static float hill_noise(float x, float y)
{
    const float px = floorf(x), py = floorf(y);
    float fx = ocn_fract(x), fy = ocn_fract(y);
    fx = (fx * fx) * (3.0f - 2.0f * fx);
    fy = (fy * fy) * (3.0f - 2.0f * fy);
    const float n = px + py * 57.0f;
    return ocn_mix(ocn_mix(hill_hash1(n + 0.0f), hill_hash1(n + 1.0f), fx),
                   ocn_mix(hill_hash1(n + 57.0f), hill_hash1(n + 58.0f), fx), fy);
}

/* Voronoi (:191-209); returns (max(.4 - sqrt(res), 0), id) */
static void hill_voronoi(float x, float y, float out[2])
{
    const float px = floorf(x), py = floorf(y);
    const float fx = ocn_fract(x), fy = ocn_fract(y);
    float res = 100.0f, id = 0.0f;
    for (int j = -1; j <= 1; ++j)
        for (int i = -1; i <= 1; ++i) {
            const float bx = (float)i, by = (float)j;
            const float h = hill_hash2(px + bx, py + by);
            const float rx = (bx - fx) + h, ry = (by - fy) + h;
            const float d = rx * rx + ry * ry;
            if (d < res) {
                res = d;
                id = h;
            }
        }
    out[0] = fmaxf(0.4f - sqrtf(res), 0.0f);
    out[1] = id;
}

/* DE(p) (:287-300), iTime = 0 */
static void hill_de(const hill_tex *T, float px, float py, float pz, float out[3])
{
    const float iTime = 0.0f;
    const float base = hill_terrain(T, px, pz) - 1.3f;
    const float qx = px * 4.0f, qz = pz * 4.0f;
    const float height = (hill_noise(qx * 2.0f, qz * 2.0f) * 0.75f + hill_noise(qx, qz) * 0.35f) +
                         hill_noise(qx * 0.5f, qz * 0.5f) * 0.2f;
    float y = (py - base) - height;
    y = y * y;
    const float s0 = ocn_sin(y * 4.0f + qz * 12.3f), s1 = ocn_sin(y * 4.0f + qx * 12.3f);
    const float w0 = ocn_sin(iTime * 2.3f + 1.5f * qz), w1 = ocn_sin(iTime * 3.6f + 1.5f * qx);
    const float ax = (qx * 2.5f + s0 * 0.12f) + (w0 * y) * 0.5f;
    const float ay = (qz * 2.5f + s1 * 0.12f) + (w1 * y) * 0.5f;
    float v[2];
    hill_voronoi(ax, ay, v);
    const float f = v[0] * 0.6f + y * 0.58f;
    out[0] = y - f * 1.4f;
    out[1] = ocn_clamp01(f * 1.5f);
    out[2] = v[1];
}

/* GetSky (:254-263) */
static void hill_sky(const float rd[3], const float sun[3], float out[3])
{
    const float sunc[3] = {1.0f, 0.75f, 0.6f};
    const float lo[3] = {0.1f, 0.2f, 0.3f};
    const float sunAmount = fmaxf(ocn_dot3(rd, sun), 0.0f);
    const float v = ocn_pow_pos(1.0f - fmaxf(rd[1], 0.0f), 6.0f);
    const float p800 = fminf(ocn_pow_pos(sunAmount, 800.0f) * 1.5f, 0.3f);
    for (int k = 0; k < 3; ++k) {
        float s = ocn_mix(lo[k], 0.32f, v);
        s = s + ((sunc[k] * sunAmount) * sunAmount) * 0.25f;
        s = s + sunc[k] * p800;
        out[k] = ocn_clamp01(s);
    }
}

/* Scene (:393-428); returns hit, *resT */
static int hill_scene(const hill_tex *T, const float ro[3], const float rd[3], float *resT)
{
    float t = -(ro[1] + 1.0f) / rd[1];
    float t_inc = 0.0f;
    if (rd[1] > -0.015f) t = 80.0f;
    float h = 0.0f, st = 1.0f, old_h = 0.0f;
    for (int j = 0; j < 100; ++j) {
        t = t + t_inc;
        const float p0 = ro[0] + t * rd[0], p1 = ro[1] + t * rd[1], p2 = ro[2] + t * rd[2];
        h = p1 - hill_terrain(T, p0, p2);
        t_inc = (fmaxf(1.0f, fabsf(h)) * ocn_sign(h)) * st;
        if (h * old_h < 0.0f) st = st / 2.0f;
        old_h = h;
    }
    *resT = t;
    return fabsf(h) < 0.05f;
}

/* main() (:453-551) at texCoordV (tx, ty); writes fragColor (4 floats) */
void oracle_hill_pixel(const float *tex_frame, int H, int W, int Ct, float tx, float ty, const float *cam,
                       float out[4])
{
    const hill_tex T = {tex_frame, H, W, Ct};
    const float width = (float)W, height = (float)H;
    const float xyx = (tx + 1.0f) / 2.0f, xyy = (ty * -1.0f + 1.0f) / 2.0f;
    if (fabsf(xyy * height - height / 2.0f) / (width / 2.0f) >= 0.5625f) {
        out[0] = out[1] = out[2] = out[3] = 0.0f;
        return;
    }
    float sun[3] = {0.35f, 0.2f, 0.3f};
    ocn_normalize(sun);
    float rv[3] = {xyx * width - width / 2.0f, xyy * height - height / 2.0f, 0.85f * width};
    ocn_normalize(rv);
    const float ro[3] = {-cam[9], cam[11], cam[10]};
    const float r00 = 0.999999573f, r01 = -0.0000933038802f, r02 = 0.000919791287f;
    const float r10 = 0.000918443273f, r11 = -0.0135434586f, r12 = -0.999907861f;
    const float r20 = 0.000105752439f, r21 = 0.999908279f, r22 = -0.0135433672f;
    float dir[3];
    dir[0] = -((r00 * rv[0] + r10 * rv[1]) + r20 * rv[2]);
    dir[2] = (r01 * rv[0] + r11 * rv[1]) + r21 * rv[2];
    dir[1] = (r02 * rv[0] + r12 * rv[1]) + r22 * rv[2];
    float col[3], dist;
    if (!hill_scene(&T, ro, dir, &dist)) {
        hill_sky(dir, sun, col);
    } else {
        const float pos[3] = {ro[0] + dist * dir[0], ro[1] + dist * dir[1], ro[2] + dist * dir[2]};
        float nor[3];
        hill_terrain_normal(&T, pos[0], pos[2], nor);
        /* TerrainColour (:363-377), type 0 */
        float mat[3];
        const float nz = hill_noise(pos[0] * 0.025f, pos[2] * 0.025f);
        const float m0[3] = {0.0f, 0.3f, 0.0f}, m1[3] = {0.2f, 0.3f, 0.0f};
        for (int k = 0; k < 3; ++k) mat[k] = ocn_mix(m0[k], m1[k], nz);
        float fn = 0.0f, w = 0.7f, nx = pos[0] * 0.1f, ny = pos[2] * 0.1f; /* FractalNoise (:242-252) */
        for (int i = 0; i < 3; ++i) {
            fn = fn + hill_noise(nx, ny) * w;
            w = w * 0.6f;
            nx = 2.0f * nx;
            ny = 2.0f * ny;
        }
        const float tsh = fn + 0.5f;
        /* GrassBlades (:317-346) */
        {
            const float rCoC = fmaxf((dist * 0.3f) * 0.04f, (2.0f / height) * (1.0f + dist * 0.3f));
            float d = 0.0f, alpha = 0.0f;
            float cw[4] = {mat[0] * 0.15f, mat[1] * 0.15f, mat[2] * 0.15f, 0.0f};
            for (int i = 0; i < 15; ++i) {
                if (cw[3] > 0.99f) break;
                float ret[3];
                hill_de(&T, pos[0] + dir[0] * d, pos[1] + dir[1] * d, pos[2] + dir[2] * d, ret);
                ret[0] = ret[0] + 0.5f * rCoC;
                if (ret[0] < rCoC) {
                    alpha = (1.0f - cw[1]) * ocn_clamp01((-ret[0] - -rCoC) / (rCoC - -rCoC));
                    const float tip[3] = {0.35f, 0.35f, fminf(ocn_pow_pos(ret[2], 4.0f) * 35.0f, 0.35f)};
                    const float wt = ocn_pow_pos(ret[1], 9.0f) * 0.7f;
                    for (int k = 0; k < 3; ++k) {
                        const float gra = ocn_mix(mat[k], tip[k], wt) * ret[1];
                        cw[k] = cw[k] + gra * alpha;
                    }
                    cw[3] = cw[3] + alpha;
                }
                d = d + fmaxf(ret[0] * 0.7f, 0.1f);
            }
            if (cw[3] < 0.2f) { cw[0] = 0.1f; cw[1] = 0.15f; cw[2] = 0.05f; }
            for (int k = 0; k < 3; ++k) mat[k] = cw[k] * tsh;
        }
        /* DoLighting (:351-356) */
        const float sl = ocn_dot3(sun, nor);
        const float hl = (sl * sl) * 4.0f;
        const float sunc[3] = {1.0f, 0.75f, 0.6f};
        for (int k = 0; k < 3; ++k) mat[k] = (mat[k] * sunc[k]) * hl;
        /* ApplyFog (:267-271) */
        const float fog = ocn_clamp01((dist * dist) * 0.0000012f);
        float sky[3];
        hill_sky(dir, sun, sky);
        for (int k = 0; k < 3; ++k) col[k] = ocn_mix(mat[k], sky[k], fog);
    }
    /* PostEffects (:437-451) */
    float rgb[3];
    for (int k = 0; k < 3; ++k) rgb[k] = ocn_pow_pos(col[k], 0.45f) * 1.3f;
    const float lum = (0.2125f * rgb[0] + 0.7154f * rgb[1]) + 0.0721f * rgb[2];
    const float vig = 0.4f + 0.5f * ocn_pow_pos((((40.0f * xyx) * xyy) * (1.0f - xyx)) * (1.0f - xyy), 0.2f);
    for (int k = 0; k < 3; ++k) out[k] = ocn_mix(0.5f, ocn_mix(lum, rgb[k], 1.3f), 1.1f) * vig;
    out[3] = 1.0f;
}

static int fwd_core(const float *background, int Cb, const float *vertices, const float *vertex_colors,
                    const int32_t *faces, int B, int H, int W, int C, int V, int F, int shader_id,
                    const float *camera_pos, float *pixels, int32_t *gbuffer, int nthreads,
                    float *depth, float *bary, int32_t *face_ids);

int oracle_rasterise_fwd_shader(const float *background, const float *vertices, const float *vertex_colors,
                                const int32_t *faces, int B, int H, int W, int C, int V, int F, int shader_id,
                                const float *camera_pos, float *pixels, int32_t *gbuffer, int nthreads)
{
    return fwd_core(background, C, vertices, vertex_colors, faces, B, H, W, C, V, F, shader_id, camera_pos, pixels,
                    gbuffer, nthreads, NULL, NULL, NULL);
}

/* the Hill op (csrc/hill.cpp): terrain lookup [B,H,W,Ct] (Ct in {1,3,4}) in place of the background */
int oracle_hill_fwd(const float *terrain, int Ct, const float *vertices, const int32_t *faces, int B, int H, int W,
                    int C, int V, int F, const float *camera_pos, float *pixels, int32_t *gbuffer, int nthreads)
{
    return fwd_core(terrain, Ct, vertices, NULL, faces, B, H, W, C, V, F, 7, camera_pos, pixels, gbuffer, nthreads,
                    NULL, NULL, NULL);
}

int oracle_rasterise_fwd(const float *background, const float *vertices, const float *vertex_colors,
                         const int32_t *faces, int B, int H, int W, int C, int V, int F,
                         float *pixels, int32_t *gbuffer, int nthreads)
{
    return oracle_rasterise_fwd_shader(background, vertices, vertex_colors, faces, B, H, W, C, V, F, 0, NULL,
                                       pixels, gbuffer, nthreads);
}

/* Gouraud forward plus the deferred-shading G-buffer of dirt_rasterise_fwd_gbuffer (include/dirt_mi355x.h):
 * depth = the DEPTH24 value read back as float, d / (2^24 - 1) (1.0 uncovered, the clear value,
 * csrc/rasterise_egl.cpp:248,449); barycentrics = the R6 perspective-correct lambdas of the visible face's
 * vertices (0 uncovered); face_ids = the visible face (-1 uncovered).  Each output may be NULL. */
int oracle_rasterise_fwd_gbuffer(const float *background, const float *vertices, const float *vertex_colors,
                                 const int32_t *faces, int B, int H, int W, int C, int V, int F, float *pixels,
                                 int32_t *gbuffer, float *depth, float *bary, int32_t *face_ids, int nthreads)
{
    return fwd_core(background, C, vertices, vertex_colors, faces, B, H, W, C, V, F, 0, NULL, pixels, gbuffer,
                    nthreads, depth, bary, face_ids);
}

/* shader_id (include/dirt_mi355x.h): 0 Gouraud, 1 oceanic_horizon, 2..5 the oceanic family,
 * 6 oceanic_opt_flow, 7 hill (no depth test: the last face in draw order wins, hill.cpp:194;
 * uncovered pixels 0, hill never writes its colour attachment there); camera_pos: host floats.
 * background has Cb channels (Cb == C except for hill's terrain lookup). */
static int fwd_core(const float *background, int Cb, const float *vertices, const float *vertex_colors,
                    const int32_t *faces, int B, int H, int W, int C, int V, int F, int shader_id,
                    const float *camera_pos, float *pixels, int32_t *gbuffer, int nthreads,
                    float *depth, float *bary, int32_t *face_ids)
{
    int status = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    orc_rec *recs = (orc_rec *)malloc(sizeof(orc_rec) * 6 * (size_t)(F > 0 ? F : 1));
    int32_t *nsub = (int32_t *)malloc(sizeof(int32_t) * (size_t)(F > 0 ? F : 1));
    int32_t *clipped = (int32_t *)malloc(sizeof(int32_t) * (size_t)(F > 0 ? F : 1));
    uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)H * W);
    int32_t *rbuf = (int32_t *)malloc(sizeof(int32_t) * (size_t)H * W);
    for (int b = 0; b < B; ++b) {
        const float *vb = vertices + (int64_t)b * V * 4;
        const float *cb = vertex_colors ? vertex_colors + (int64_t)b * V * C : NULL;
        const int32_t *fb = faces + (int64_t)b * F * 3;
        if (setup_frame(vb, fb, V, F, W, H, recs, nsub, clipped)) status = 2;
        /* raster: parallel over bands of window rows; key-min is order independent */
#pragma omp parallel for schedule(dynamic, 1)
        for (int band = 0; band < (H + 7) / 8; ++band) {
            int jb0 = band * 8, jb1 = jb0 + 7 < H - 1 ? jb0 + 7 : H - 1;
            for (int j = jb0; j <= jb1; ++j)
                for (int i = 0; i < W; ++i) { keys[(int64_t)j * W + i] = ~0ull; rbuf[(int64_t)j * W + i] = -1; }
            for (int f = 0; f < F; ++f) {
                for (int s = 0; s < nsub[f]; ++s) {
                    int64_t ri = rec_index(F, f, s);
                    const orc_rec *r = &recs[ri];
                    if (!rec_nonempty(r)) continue;
                    int j0 = r->j0 > jb0 ? r->j0 : jb0, j1 = r->j1 < jb1 ? r->j1 : jb1;
                    for (int j = j0; j <= j1; ++j)
                        for (int i = r->i0; i <= r->i1; ++i) {
                            int64_t E[3];
                            edge_values(r, i, j, E);
                            if (!inside(r, E)) continue;
                            uint64_t key;
                            if (shader_id == 7) {
                                /* depth test off; near/far clipping still applies (zw in [0,1]) */
                                if (!sample_in_range(r, i, j)) continue;
                                key = (uint64_t)(0xffffffffu - (uint32_t)f);
                            } else {
                                uint32_t d;
                                if (!sample_depth(r, i, j, &d)) continue;
                                key = ((uint64_t)d << 32) | (uint32_t)f;
                            }
                            int64_t p = (int64_t)j * W + i;
                            if (key < keys[p]) { keys[p] = key; rbuf[p] = (int32_t)ri; }
                        }
                }
            }
            /* resolve (R6) + background, rows flipped to top-first */
            for (int j = jb0; j <= jb1; ++j) {
                int row = H - 1 - j;
                for (int i = 0; i < W; ++i) {
                    int64_t p = (int64_t)j * W + i;
                    int64_t o = (((int64_t)b * H + row) * W + i);
                    float *out = pixels + o * C;
                    const float *bg = background + o * Cb;
                    int32_t ri = rbuf[p];
                    if (gbuffer) gbuffer[o] = ri < 0 ? -1 : (ri | (clipped[recs[ri].face] ? GBUF_MULTI : 0));
                    if (ri < 0) {
                        for (int c = 0; c < C; ++c) out[c] = shader_id == 7 ? 0.0f : bg[c];
                        if (depth) depth[o] = 1.0f;
                        if (bary) bary[o * 3] = bary[o * 3 + 1] = bary[o * 3 + 2] = 0.0f;
                        if (face_ids) face_ids[o] = -1;
                        continue;
                    }
                    const orc_rec *r = &recs[ri];
                    int64_t E[3];
                    edge_values(r, i, j, E);
                    float lam[3] = {0.0f, 0.0f, 0.0f};
                    parent_lambda(r, E, lam);
                    if (depth) depth[o] = (float)(uint32_t)(keys[p] >> 32) / 16777215.0f;
                    if (bary) { bary[o * 3] = lam[0]; bary[o * 3 + 1] = lam[1]; bary[o * 3 + 2] = lam[2]; }
                    if (face_ids) face_ids[o] = r->face;
                    const int32_t *f3 = fb + 3 * (int64_t)r->face;
                    if (shader_id == 6 || shader_id == 7) {
                        const float tx = (lam[0] * vb[(int64_t)f3[0] * 4] + lam[1] * vb[(int64_t)f3[1] * 4]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4];
                        const float ty = (lam[0] * vb[(int64_t)f3[0] * 4 + 1] + lam[1] * vb[(int64_t)f3[1] * 4 + 1]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4 + 1];
                        float col[4];
                        if (shader_id == 6) {
                            oracle_opt_flow_pixel(tx, ty, camera_pos, (float)W, (float)H, col);
                            col[2] = 0.0f;
                            col[3] = 1.0f;
                        } else {
                            oracle_hill_pixel(background + (int64_t)b * H * W * Cb, H, W, Cb, tx, ty, camera_pos, col);
                        }
                        for (int c = 0; c < C; ++c) out[c] = c < 4 ? col[c] : 0.0f;
                        continue;
                    }
                    if (shader_id >= 2) {
                        const float tx = (lam[0] * vb[(int64_t)f3[0] * 4] + lam[1] * vb[(int64_t)f3[1] * 4]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4];
                        const float ty = (lam[0] * vb[(int64_t)f3[0] * 4 + 1] + lam[1] * vb[(int64_t)f3[1] * 4 + 1]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4 + 1];
                        float col[3];
                        oracle_oceanic_family_pixel(shader_id, background + (int64_t)b * H * W * C, H, W, C, tx, ty,
                                                    camera_pos, col);
                        for (int c = 0; c < C; ++c) out[c] = c < 3 ? col[c] : c == 3 ? 1.0f : 0.0f;
                        continue;
                    }
                    if (shader_id == 1) {
                        /* fragColor = (col.x, col.y, 0, 1) (shaders.cpp:1860-1862,1916) */
                        const float tx = (lam[0] * vb[(int64_t)f3[0] * 4] + lam[1] * vb[(int64_t)f3[1] * 4]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4];
                        const float ty = (lam[0] * vb[(int64_t)f3[0] * 4 + 1] + lam[1] * vb[(int64_t)f3[1] * 4 + 1]) +
                                         lam[2] * vb[(int64_t)f3[2] * 4 + 1];
                        float col[2];
                        oracle_oceanic_horizon_pixel(background + (int64_t)b * H * W * C, H, W, C, tx, ty,
                                                     camera_pos, col);
                        for (int c = 0; c < C; ++c) out[c] = c == 0 ? col[0] : c == 1 ? col[1] : c == 3 ? 1.0f : 0.0f;
                        continue;
                    }
                    for (int c = 0; c < C; ++c)
                        out[c] = (lam[0] * cb[(int64_t)f3[0] * C + c] + lam[1] * cb[(int64_t)f3[1] * C + c]) +
                                 lam[2] * cb[(int64_t)f3[2] * C + c];
                }
            }
        }
    }
    free(recs); free(nsub); free(clipped); free(keys); free(rbuf);
    return status;
}

/* ------------------------------------------------------------------------------------------------ */
/* Backward.  Contributions are computed in float exactly as the HIP kernel computes
 * them; sums are accumulated in double (the GPU sums in float with atomics -> tolerance). */

static int covers_face(const orc_rec *recs, const int32_t *nsub, int F, int f, int i, int j)
{
    for (int s = 0; s < nsub[f]; ++s) {
        const orc_rec *r = &recs[rec_index(F, f, s)];
        if (!rec_nonempty(r)) continue;
        if (i < r->i0 || i > r->i1 || j < r->j0 || j > r->j1) continue;
        int64_t E[3];
        edge_values(r, i, j, E);
        if (inside(r, E)) return 1;
    }
    return 0;
}

/* owner h (record r), pair midpoint between samples (i,j) and (i2,j2), axis 0=x 1=y.
 * dL/dx_k += omega s (W/2) lambda_k / Wm with lambda the perspective-correct parent barycentrics
 * at the pair midpoint and Wm = sum_k lambda_k w_k (the clip w there).  Evaluated without normalising:
 * a_k = E_k(mid) / w_k of the record's own vertices, and the edge functions at the midpoint sum to 2D exactly
 * (E_0 + E_1 + E_2 = D at every sample, an int64 identity), so lambda_k / Wm = a_k / (2D) for a face that did not
 * take the clipping path; a clipped face's sub-triangle has vertices that are convex combinations of the
 * parent's (basis rows; w_sub = basis . w_parent), so the parent's lambda_i / Wm = sum_k a_k basis_ki / (2D).
 * The normalised form (lambda = a / sum a, Wm = sum lambda w) cancels catastrophically on slivers, whose E_k
 * are ~10^3 x D: the fuzz scene of seed 37851 (a 1811-unit sliver) lost 4e-4 relative that way against a
 * float64 evaluation (tests/backward_f64.py pins both kinds of face at 1e-6 of the gradient scale). */
static void add_pair_owner(const orc_rec *r, const float *vb, const int32_t *fb, int W, int H,
                           int i, int j, int i2, int j2, int axis, float s, float omega, int identity, double *gv)
{
    (void)vb;
    int64_t E1[3], E2[3], E[3];
    edge_values(r, i, j, E1);
    edge_values(r, i2, j2, E2);
    for (int k = 0; k < 3; ++k) E[k] = E1[k] + E2[k];
    const int32_t *f3 = fb + 3 * (int64_t)r->face;
    float half = axis == 0 ? 0.5f * (float)W : 0.5f * (float)H;
    float mid = axis == 0 ? (float)(i + 1) : (float)(j + 1);
    float ndc = mid / half - 1.0f;
    const int64_t twoD = E[0] + E[1] + E[2];
    if (twoD == 0) return;
    const float t = ((omega * s) * half) / (float)twoD;
    float a[3], g3[3];
    for (int k = 0; k < 3; ++k) a[k] = (float)E[k] * r->iw[k];
    for (int k = 0; k < 3; ++k)
        g3[k] = identity ? t * a[k] : t * ((a[0] * r->basis[k] + a[1] * r->basis[3 + k]) + a[2] * r->basis[6 + k]);
    for (int k = 0; k < 3; ++k) {
        float g = g3[k];
        double *d = gv + (int64_t)f3[k] * 4;
        d[axis] += (double)g;
        d[3] += (double)(-(g * ndc));
    }
}

static int all_finite(const float *x, int C)
{
    for (int c = 0; c < C; ++c)
        if (!isfinite(x[c])) return 0;
    return 1;
}

int oracle_rasterise_bwd(const float *vertices, const float *vertex_colors, const int32_t *faces,
                         const float *pixels, const float *grad_pixels, const int32_t *gbuffer,
                         int B, int H, int W, int C, int V, int F,
                         float *grad_vertices, float *grad_vertex_colors, float *grad_background, int nthreads)
{
    (void)vertex_colors;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int status = 0;
    orc_rec *recs = (orc_rec *)malloc(sizeof(orc_rec) * 6 * (size_t)(F > 0 ? F : 1));
    int32_t *nsub = (int32_t *)malloc(sizeof(int32_t) * (size_t)(F > 0 ? F : 1));
    int32_t *clipped = (int32_t *)malloc(sizeof(int32_t) * (size_t)(F > 0 ? F : 1));
    int nthr = 1;
#ifdef _OPENMP
    nthr = omp_get_max_threads();
#endif
    double *accv = (double *)malloc(sizeof(double) * (size_t)nthr * V * 4);
    double *accc = (double *)malloc(sizeof(double) * (size_t)nthr * V * C);
    for (int b = 0; b < B; ++b) {
        const float *vb = vertices + (int64_t)b * V * 4;
        const int32_t *fb = faces + (int64_t)b * F * 3;
        if (setup_frame(vb, fb, V, F, W, H, recs, nsub, clipped)) status = 2;
        memset(accv, 0, sizeof(double) * (size_t)nthr * V * 4);
        memset(accc, 0, sizeof(double) * (size_t)nthr * V * C);
#pragma omp parallel
        {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            double *gv = accv + (size_t)tid * V * 4, *gc = accc + (size_t)tid * V * C;
#pragma omp for schedule(static)
            for (int j = 0; j < H; ++j) {
                for (int i = 0; i < W; ++i) {
                    int row = H - 1 - j;
                    int64_t o = ((int64_t)b * H + row) * W + i;
                    const float *G = grad_pixels + o * C, *I = pixels + o * C;
                    int32_t rp = gbuffer[o] < 0 ? -1 : (gbuffer[o] & GBUF_INDEX_MASK);
                    const int undef_p = rp < 0 && !all_finite(I, C);
                    float *gbg = grad_background + o * C;
                    if (rp < 0) {
                        for (int c = 0; c < C; ++c) gbg[c] = G[c];
                    } else {
                        for (int c = 0; c < C; ++c) gbg[c] = 0.0f;
                        const orc_rec *r = &recs[rp];
                        int64_t E[3];
                        edge_values(r, i, j, E);
                        float lam[3];
                        if (parent_lambda(r, E, lam)) {
                            const int32_t *f3 = fb + 3 * (int64_t)r->face;
                            for (int k = 0; k < 3; ++k)
                                for (int c = 0; c < C; ++c) gc[(int64_t)f3[k] * C + c] += (double)(lam[k] * G[c]);
                        }
                    }
                    for (int axis = 0; axis < 2; ++axis) {
                        int i2 = i + (axis == 0), j2 = j + (axis == 1);
                        if (i2 >= W || j2 >= H) continue;
                        int64_t o2 = ((int64_t)b * H + (H - 1 - j2)) * W + i2;
                        int32_t rq = gbuffer[o2] < 0 ? -1 : (gbuffer[o2] & GBUF_INDEX_MASK);
                        if (rp < 0 && rq < 0) continue;
                        const float *G2 = grad_pixels + o2 * C, *I2 = pixels + o2 * C;
                        /* a background pixel with a non-finite value (samples/deferred.py:67,81 renders
                         * G-buffers over -inf) defines no image difference: its pairs carry no vertex
                         * gradient */
                        if (undef_p || (rq < 0 && !all_finite(I2, C))) continue;
                        float acc = 0.0f;
                        for (int c = 0; c < C; ++c) acc += (G[c] + G2[c]) * (I2[c] - I[c]);
                        float s = -0.5f * acc;
                        if (s == 0.0f) continue;
                        int fp = rp >= 0 ? recs[rp].face : -1, fq = rq >= 0 ? recs[rq].face : -1;
                        const int idp = fp >= 0 && !clipped[fp], idq = fq >= 0 && !clipped[fq];
                        if (fp == fq || fq < 0) {
                            add_pair_owner(&recs[rp], vb, fb, W, H, i, j, i2, j2, axis, s, 1.0f, idp, gv);
                        } else if (fp < 0) {
                            add_pair_owner(&recs[rq], vb, fb, W, H, i, j, i2, j2, axis, s, 1.0f, idq, gv);
                        } else {
                            int cfq = covers_face(recs, nsub, F, fp, i2, j2);
                            int cgp = covers_face(recs, nsub, F, fq, i, j);
                            if (!cfq && cgp) {
                                add_pair_owner(&recs[rp], vb, fb, W, H, i, j, i2, j2, axis, s, 1.0f, idp, gv);
                            } else if (cfq && !cgp) {
                                add_pair_owner(&recs[rq], vb, fb, W, H, i, j, i2, j2, axis, s, 1.0f, idq, gv);
                            } else {
                                add_pair_owner(&recs[rp], vb, fb, W, H, i, j, i2, j2, axis, s, 0.5f, idp, gv);
                                add_pair_owner(&recs[rq], vb, fb, W, H, i, j, i2, j2, axis, s, 0.5f, idq, gv);
                            }
                        }
                    }
                }
            }
        }
        for (int64_t v = 0; v < (int64_t)V * 4; ++v) {
            double a = 0.0;
            for (int t = 0; t < nthr; ++t) a += accv[(size_t)t * V * 4 + v];
            grad_vertices[(int64_t)b * V * 4 + v] = (float)a;
        }
        for (int64_t v = 0; v < (int64_t)V * C; ++v) {
            double a = 0.0;
            for (int t = 0; t < nthr; ++t) a += accc[(size_t)t * V * C + v];
            grad_vertex_colors[(int64_t)b * V * C + v] = (float)a;
        }
    }
    free(recs); free(nsub); free(clipped); free(accv); free(accc);
    return status;
}

int oracle_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
