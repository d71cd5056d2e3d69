// raster_rules.h -- device-side raster rules R1..R6 of DESIGN.md section 3 (gfx950).
//
// These functions are the GPU statement of the rules the CPU oracle (oracle/dirt_oracle.c) states
// independently.  Both are compiled with -ffp-contract=off and IEEE-correct division so that
// coverage, 24-bit depth and the visible face are bit-identical; see DESIGN.md section 3.
//
// Reference semantics restated: csrc/shaders.cpp:16-34 (clip-space passthrough vertex stage),
// csrc/rasterise_egl.cpp:194,248,449 (depth test LESS, DEPTH24 cleared to 1.0), :440-458 (faces drawn
// in index order with base vertex b*V), README.md:134-137 (Gouraud = perspective-correct interpolation).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dirt {

constexpr int kTile = 16;          // raster tile edge (pixels); one 256-thread workgroup per tile
constexpr int kMaxSub = 6;         // fan triangles of a triangle clipped by 5 planes
constexpr int kExtraPerFace = 5;   // record slots F + 5f + (s-1) for sub-triangles s>0
constexpr uint32_t kDepthMax = 16777215u;  // 2^24-1 == cleared depth 1.0 (rasterise_egl.cpp:449)
// g-buffer word: visible record index (< 2^29 since F <= 2^26), bit 30 set when the face went through
// the R5 clipping path (non-identity basis, possibly several records), -1 for background
constexpr int32_t kGbufMulti = 1 << 30;
constexpr int32_t kGbufIndexMask = kGbufMulti - 1;

// Per (sub-)triangle setup record, 128 B in two 64-B halves.  The first half is everything the tile raster
// stages and every coverage test reads (edge functions relative to vertex 0, bbox, depth plane), so a
// non-clipped face's record is written and read as one 64-B piece; the second half (1/w of the three
// sub-vertices, parent barycentric basis) is written and read for clipped faces only -- a non-clipped
// face's 1/w travels in its FaceData (below) and its basis is the identity.
//   E_k(px, py) = A_k (px - X0) + B_k (py - Y0) + (k == 0 ? D : 0)
// equals the usual A_k px + B_k py + C_k exactly (vertex 0 lies on edges 1 and 2, and E_0 there is D).
struct alignas(16) Rec {
    int32_t A[3];
    int32_t B[3];
    int32_t X0, Y0;           // snapped vertex 0 (1/256 px)
    int64_t D;                // E_0 at vertex 0 = E_0 + E_1 + E_2 everywhere (twice the signed area, > 0)
    uint16_t i0, i1, j0, j1;  // inclusive pixel bbox (window coords, j from the bottom); empty if i0 > i1
    float z0, za, zb;         // depth plane relative to vertex 0 (R4); fx0, fy0 = X0, Y0 / 256 exactly
    int32_t face;
    // second half: clipped records only
    float iw[3];              // 1/w of the three (sub-)vertices
    float basis[9];           // row k = parent barycentric of sub-vertex k (identity on the fast path)
    int32_t pad[4];
};
static_assert(sizeof(Rec) == 128, "Rec must be 128 B");

struct alignas(8) EdgePart {  // first 48 B of Rec: what a coverage test needs
    int32_t A[3];
    int32_t B[3];
    int32_t X0, Y0;
    int64_t D;
    uint16_t i0, i1, j0, j1;
};
static_assert(sizeof(EdgePart) == 48, "EdgePart must be 48 B");

struct alignas(16) RasterPart {  // first 64 B of Rec
    int32_t A[3];
    int32_t B[3];
    int32_t X0, Y0;
    int64_t D;
    uint16_t i0, i1, j0, j1;
    float z0, za, zb;
    int32_t face;
};
static_assert(sizeof(RasterPart) == 64, "RasterPart must be 64 B");
constexpr int kRecBboxOffset = 40;  // offsetof(Rec, i0): the packed bbox as one 8-B load

__host__ __device__ inline float rec_fx0(int32_t X0) { return (float)X0 * 0.00390625f; }  // exact: |X0| < 2^23

// Per-face data written by setup, read by the resolve and the backward (one 32-B load instead of a
// faces[] -> vertices[] dependent chain).
struct alignas(16) FaceData {
    int32_t v[3];  // vertex indices (frame-local)
    float q[3];    // non-clipped face: 1/w of its three vertices (its record's interpolation data);
                   // clipped face: clip w of the three parent vertices
    int32_t nsub;     // number of (sub-)triangle records, 0 = culled
    int32_t clipped;  // 1 if set up by the R5 clipping path
};
static_assert(sizeof(FaceData) == 32, "FaceData must be 32 B");

// Clip-space triangle passed by value (keeps it in registers across the non-inlined clip path).
struct Tri {
    float v[3][4];
};

// record indices are < 6F <= 6 * 2^26 < 2^31: 32-bit arithmetic (a 64-bit division by 5 is ~15 VALU)
__host__ __device__ inline int face_of_record(int32_t ri, int F)
{
    return ri < F ? ri : (int)((uint32_t)(ri - F) / (uint32_t)kExtraPerFace);
}

__host__ __device__ inline int64_t rec_index(int F, int f, int s)
{
    return s == 0 ? (int64_t)f : (int64_t)F + (int64_t)kExtraPerFace * f + (s - 1);
}

__device__ inline void set_empty(Rec &r, int face)
{
    r.i0 = 1; r.i1 = 0; r.j0 = 1; r.j1 = 0;
    r.face = face;
}

// Store a non-clipped face's record: its first 64 B only (the second half -- 1/w, identity basis -- is
// never read for such faces: the 1/w are in its FaceData, and every basis use takes the identity branch from
// FaceData.clipped / the g-buffer's multi bit)
__device__ __forceinline__ void store_record_fast(Rec *dst, const Rec &r)
{
    const int4 *s4 = reinterpret_cast<const int4 *>(&r);
    int4 *d4 = reinterpret_cast<int4 *>(dst);
#pragma unroll
    for (int k = 0; k < 4; ++k) d4[k] = s4[k];
}

// R5 sub-vertex clamp: x/w of a clipped face's sub-vertex to [-2 gx, 2 gx] (NaN to 2 gx), y/w likewise.
// R5's guard planes keep a sub-vertex inside the guard band only up to float rounding, and near w = 0 that
// rounding is unbounded (an intersection computed after the x planes can land at x / w = -4.7e6 with w = 7e-12,
// fuzz seed 167059); clamped at twice the band, which ordinary rounding never reaches, every snapped
// coordinate stays below 2^24 (W, H <= 8192), so A, B and the offsets to X0, Y0 stay exact in int32.
__device__ __forceinline__ float guard_clamp(float xn, float g) { return xn <= g ? (xn >= -g ? xn : -g) : g; }

// R1..R4 for one (sub-)triangle: fills `out` (a register-resident local), returns true if non-empty.
// Clamp: a clipped face's sub-triangle (R5 sub-vertex clamp to gx2, gy2 = twice the guard band).
template <bool Clamp = false>
__device__ inline bool make_record(const float v[3][4], const float basis[3][3], int W, int H, int face, Rec &out,
                                   float gx2 = 0.0f, float gy2 = 0.0f)
{
    const float hw = 0.5f * (float)W, hh = 0.5f * (float)H;
    int32_t X[3], Y[3];
    float zw[3], iwv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float iw = 1.0f / v[k][3];
        float xn = v[k][0] * iw, yn = v[k][1] * iw, zn = v[k][2] * iw;
        if (Clamp) {
            xn = guard_clamp(xn, gx2);
            yn = guard_clamp(yn, gy2);
        }
        float xw = (xn + 1.0f) * hw, yw = (yn + 1.0f) * hh;
        zw[k] = zn * 0.5f + 0.5f;
        X[k] = (int32_t)__builtin_rintf(xw * 256.0f);
        Y[k] = (int32_t)__builtin_rintf(yw * 256.0f);
        iwv[k] = iw;
    }
    // |X|, |Y| < 2^24 (the guard band is 16384 px beyond the frame centre, twice that for a clamped sub-vertex;
    // 256 sub-pixels per pixel, W, H <= 8192): A, B < 2^25 fit int32
    // and every product is one 32 x 32 -> 64-bit multiply-add (no 64 x 64 multiplies)
    int32_t A[3], B[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int a = (k + 1) % 3, b = (k + 2) % 3;
        A[k] = Y[a] - Y[b];
        B[k] = X[b] - X[a];
    }
    // D = E_0 at vertex 0 = A_0 (X0 - X1) + B_0 (Y0 - Y1) (edge 0 runs through vertex 1)
    int64_t D = (int64_t)A[0] * (X[0] - X[1]) + (int64_t)B[0] * (Y[0] - Y[1]);
    // (no early exits: the emptiness tests select at the end, so the divisions below can start while the
    // integer path is still running -- setup runs one wave per SIMD, where only ILP hides latency)
    const bool neg = D < 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) { A[k] = neg ? -A[k] : A[k]; B[k] = neg ? -B[k] : B[k]; }
    const int64_t Dn = neg ? -D : D;
    int32_t xmin = min(X[0], min(X[1], X[2])), xmax = max(X[0], max(X[1], X[2]));
    int32_t ymin = min(Y[0], min(Y[1], Y[2])), ymax = max(Y[0], max(Y[1], Y[2]));
    int32_t i0 = (xmin - 128 + 255) >> 8, i1 = (xmax - 128) >> 8;  // arithmetic shift = floor
    int32_t j0 = (ymin - 128 + 255) >> 8, j1 = (ymax - 128) >> 8;
    i0 = i0 < 0 ? 0 : i0;
    j0 = j0 < 0 ? 0 : j0;
    i1 = i1 > W - 1 ? W - 1 : i1;
    j1 = j1 > H - 1 ? H - 1 : j1;
    const bool nonempty = D != 0 && i0 <= i1 && j0 <= j1;
    const float fx0 = rec_fx0(X[0]), fy0 = rec_fx0(Y[0]);
    const float dx1 = (float)X[1] * 0.00390625f - fx0, dy1 = (float)Y[1] * 0.00390625f - fy0;
    const float dx2 = (float)X[2] * 0.00390625f - fx0, dy2 = (float)Y[2] * 0.00390625f - fy0;
    const float dz1 = zw[1] - zw[0], dz2 = zw[2] - zw[0];
    // (float)D: one conversion when every lane's D fits int32 (the same integer, so the same float)
    float fD;
    if (__builtin_amdgcn_ballot_w64(D != (int64_t)(int32_t)D) == 0)
        fD = (float)(int32_t)D;
    else
        fD = (float)D;
    const float det = fD * (1.0f / 65536.0f);
#pragma unroll
    for (int k = 0; k < 3; ++k) { out.A[k] = A[k]; out.B[k] = B[k]; }
    out.X0 = X[0]; out.Y0 = Y[0]; out.D = Dn;
    out.i0 = (uint16_t)i0; out.i1 = (uint16_t)i1; out.j0 = (uint16_t)j0; out.j1 = (uint16_t)j1;
    out.face = face;
    out.z0 = zw[0];
    out.za = (dz1 * dy2 - dz2 * dy1) / det;
    out.zb = (dx1 * dz2 - dx2 * dz1) / det;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        out.iw[k] = iwv[k];
#pragma unroll
        for (int i = 0; i < 3; ++i) out.basis[k * 3 + i] = basis[k][i];
    }
    if (!nonempty) set_empty(out, face);
    return nonempty;
}

// R3: exact edge values at pixel centre (i,j)
// (32 x 32 -> 64-bit signed multiplies: one v_mad_i64_i32 each; pixel coordinates fit in 22 bits)
// (relative to vertex 0: |px - X0|, |py - Y0| < 2^24, so the offsets are int32 and each product is one
// 32 x 32 -> 64-bit multiply-add)
template <typename R>
__device__ __forceinline__ void edge_values(const R &r, int i, int j, int64_t E[3])
{
    const int32_t dx = i * 256 + 128 - r.X0, dy = j * 256 + 128 - r.Y0;
#pragma unroll
    for (int k = 0; k < 3; ++k) E[k] = (int64_t)r.A[k] * (int64_t)dx + ((int64_t)r.B[k] * (int64_t)dy + (k == 0 ? r.D : 0));
}

// R3 top-left rule: E > 0, or E == 0 on an owned (left or top) edge  <=>  E + owned > 0
template <typename R>
__device__ __forceinline__ bool inside(const R &r, const int64_t E[3])
{
    bool in = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t owned = (r.A[k] > 0 || (r.A[k] == 0 && r.B[k] < 0)) ? 1 : 0;
        in = in && (E[k] + owned > 0);
    }
    return in;
}

// R4: depth at the pixel centre, zw = fma(za, fx - fx0, fma(zb, fy - fy0, z0)) (fx - fx0 is exact: both
// are multiples of 2^-8 below 2^15), in range iff 0 <= zw <= 1; quantised q = (uint)fma(zw, 2^24-1, 0.5)
__device__ __forceinline__ float depth_at(float za, float zb, float z0, float dx, float dy)
{
    return __builtin_fmaf(za, dx, __builtin_fmaf(zb, dy, z0));
}

__device__ __forceinline__ uint32_t depth_q24(float zw) { return (uint32_t)__builtin_fmaf(zw, 16777215.0f, 0.5f); }

// R4: 24-bit depth of the sample, false if outside [0,1] or not nearer than the cleared depth
template <typename R>
__device__ __forceinline__ bool sample_depth(const R &r, int i, int j, uint32_t &d)
{
    const float fx = (float)i + 0.5f, fy = (float)j + 0.5f;
    const float zw = depth_at(r.za, r.zb, r.z0, fx - rec_fx0(r.X0), fy - rec_fx0(r.Y0));
    if (!(zw >= 0.0f && zw <= 1.0f)) return false;
    const uint32_t q = depth_q24(zw);
    if (q >= kDepthMax) return false;
    d = q;
    return true;
}

// R6 from the edge values already converted to float (fE[k] == (float)E[k]) and the record's 1/w (`iw`:
// FaceData.q of a non-clipped face, Rec.iw of a clipped one); `identity`: the record's basis is the identity
// (non-clipped face), where (m0*1 + m1*0) + m2*0 == m0 exactly since m_k >= +0
__device__ __forceinline__ bool parent_lambda_f(const Rec &r, const float iw[3], const float fE[3], bool identity,
                                                float lam[3])
{
    const float a0 = fE[0] * iw[0], a1 = fE[1] * iw[1], a2 = fE[2] * iw[2];
    const float s = (a0 + a1) + a2;
    if (s == 0.0f) return false;
    const float rs = 1.0f / s;
    const float m0 = a0 * rs, m1 = a1 * rs, m2 = a2 * rs;
    if (identity) {
        lam[0] = m0; lam[1] = m1; lam[2] = m2;
        return true;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) lam[i] = (m0 * r.basis[i] + m1 * r.basis[3 + i]) + m2 * r.basis[6 + i];
    return true;
}

}  // namespace dirt
