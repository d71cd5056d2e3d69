// dirt_raster.hip -- MI355X (gfx950) software rasteriser behind the C ABI of include/dirt_mi355x.h.
//
// CDNA4 has no graphics pipeline, so the reference's GL fixed-function raster
// (csrc/rasterise_egl.cpp:440-487 + the NVIDIA driver) becomes a compute pipeline:
//
//   K1 setup_kernel    one thread per (frame, face): fetch 3 clip vertices, project + snap (R1/R2),
//                      edge equations (R3), depth plane (R4), guard-band clipping (R5, rare slow path);
//                      writes 128-B setup records + 32-B FaceData, counts (tile, triangle) bin entries.
//   K2 scan_kernel     exclusive scan of per-tile counts.
//   K3 fill_kernel     scatter each record index into the bins of the 16x16 tiles its bbox overlaps.
//   K4 raster_kernel   one 256-thread workgroup per 16x16 tile (a wave per 16x4 strip): stages the
//                      tile's records in LDS with strip-relative 32-bit edge values (exact), each lane
//                      owns one pixel and keeps the min (depth24<<32 | face) key, then resolves
//                      in-kernel: perspective-correct Gouraud colour (R6) or background, coalesced
//                      [B,H,W,C] writes + the int32 g-buffer.  This fuses the reference's
//                      upload_background + raster + second pass + download_pixels
//                      (csrc/rasterise_egl.cu:16-129, rasterise_egl.cpp:370-503) into one HBM pass.
//   K5 grad_kernel     backward: dL/dbackground, dL/dvertex_colors and the
//                      filter-based dL/dvertices (README.md:146-147) for the gradient contract of
//                      csrc/rasterise_grad_common.h:19-24.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dirt_mi355x.h"
#include "raster_rules.h"

using namespace dirt;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *msg)
{
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            char _b[256];                                                               \
            snprintf(_b, sizeof(_b), "%s failed: %s", #expr, hipGetErrorString(_e));    \
            return fail(DIRT_EHIP, _b);                                                 \
        }                                                                               \
    } while (0)

// ------------------------------------------------------------------------------------------------
// Optional per-kernel event timing (bench.py roofline); off by default, host-side only.
enum KernelId { K_SETUP = 0, K_SCAN, K_FILL, K_RASTER, K_GRAD, K_COUNT };
const char *const kKernelNames[K_COUNT] = {"setup_kernel", "scan_kernel", "fill_kernel", "raster_kernel",
                                           "grad_kernel"};
struct Profiler {
    bool enabled = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[K_COUNT];
} g_prof;

struct ProfScope {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s;
    int id;
    ProfScope(int id_, hipStream_t s_) : s(s_), id(id_)
    {
        if (!g_prof.enabled) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { a = b = nullptr; return; }
        (void)hipEventRecord(a, s);
    }
    ~ProfScope()
    {
        if (!a) return;
        (void)hipEventRecord(b, s);
        g_prof.ev[id].emplace_back(a, b);
    }
};

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------
// Workspace layout.  saved = records [B][6F] (128 B) + FaceData [B][F] (32 B): what the backward reads.
// scratch = per-tile counts, cursors, offsets and the bins (forward only).
struct Layout {
    int ntx, nty, ntiles;
    int64_t nrec;
    size_t saved_recs, saved_fdata, saved_total;
    size_t off_count, off_cursor, off_offset, off_flag, off_bins, scratch_total;
    int64_t bin_capacity;
};

int64_t default_capacity(int B, int F, int ntiles)
{
    int64_t c = 16 * (int64_t)B * (int64_t)F + 4 * (int64_t)B * ntiles;
    if (c < (1 << 20)) c = 1 << 20;
    if (c > 0x7fffffffLL) c = 0x7fffffffLL;
    return c;
}

int make_layout(int B, int H, int W, int F, int64_t bin_capacity, Layout &L)
{
    L.ntx = (W + kTile - 1) / kTile;
    L.nty = (H + kTile - 1) / kTile;
    L.ntiles = L.ntx * L.nty;
    L.nrec = (int64_t)(1 + kExtraPerFace) * F;
    L.bin_capacity = bin_capacity > 0 ? (bin_capacity > 0x7fffffffLL ? 0x7fffffffLL : bin_capacity)
                                      : default_capacity(B, F, L.ntiles);
    L.saved_recs = 0;
    L.saved_fdata = (size_t)align_up((int64_t)B * L.nrec * (int64_t)sizeof(Rec), 256);
    L.saved_total = L.saved_fdata + (size_t)align_up((int64_t)B * F * (int64_t)sizeof(FaceData), 256);
    const int64_t nt = (int64_t)B * L.ntiles;
    size_t o = 0;
    L.off_count = o;  o += (size_t)align_up(nt * 4, 256);
    L.off_cursor = o; o += (size_t)align_up(nt * 4, 256);
    L.off_offset = o; o += (size_t)align_up(nt * 8, 256);
    L.off_flag = o;   o += 256;
    L.off_bins = o;   o += (size_t)align_up(L.bin_capacity * 4, 256);
    L.scratch_total = o;
    return DIRT_OK;
}

int validate(int B, int H, int W, int C, int V, int F)
{
    if (B < 0 || V < 0 || F < 0) return fail(DIRT_EINVAL, "Rasterise expects non-negative batch, vertex and face counts");
    if (H <= 0 || W <= 0 || H > DIRT_MAX_DIM || W > DIRT_MAX_DIM)
        return fail(DIRT_EINVAL, "Rasterise expects 0 < height, width <= 8192");
    if (C < 1 || C > DIRT_MAX_CHANNELS) return fail(DIRT_EINVAL, "Rasterise expects 1 <= channels <= 8");
    if ((int64_t)B * F > 0x0fffffffLL || (int64_t)B * V > 0x7fffffffLL)
        return fail(DIRT_EINVAL, "Rasterise batch too large");
    return DIRT_OK;
}

// ------------------------------------------------------------------------------------------------
// K1: setup

__device__ inline bool finite4(const float *v)
{
    return __builtin_isfinite(v[0]) && __builtin_isfinite(v[1]) && __builtin_isfinite(v[2]) && __builtin_isfinite(v[3]);
}

__device__ inline float plane_dist(int p, const float *v, float gx, float gy)
{
    switch (p) {
    case 0: return v[2] + v[3];
    case 1: return gx * v[3] + v[0];
    case 2: return gx * v[3] - v[0];
    case 3: return gy * v[3] + v[1];
    default: return gy * v[3] - v[1];
    }
}

// R5 slow path: clip against z>=-w and the guard planes, fan-triangulate, write the sub-records.
// Not inlined so that its stack arrays do not inflate the fast path.  Returns nsub.
__device__ __noinline__ int clip_face(Tri tri, int W, int H, int F, int f, Rec *frame_recs)
{
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    float poly[9][7], tmp[9][7];
    int n = 3;
    for (int k = 0; k < 3; ++k) {
        for (int c = 0; c < 4; ++c) poly[k][c] = tri.v[k][c];
        for (int i = 0; i < 3; ++i) poly[k][4 + i] = (i == k) ? 1.0f : 0.0f;
    }
    for (int p = 0; p < 5; ++p) {
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const float *a = poly[i];
            const float *c = poly[(i + 1) % n];
            const float da = plane_dist(p, a, gx, gy), dc = plane_dist(p, c, gx, gy);
            const bool ina = da >= 0.0f, inc = dc >= 0.0f;
            if (ina) {
                for (int q = 0; q < 7; ++q) tmp[m][q] = a[q];
                ++m;
            }
            if (ina != inc) {
                const float t = da / (da - dc);
                for (int q = 0; q < 7; ++q) tmp[m][q] = a[q] + t * (c[q] - a[q]);
                ++m;
            }
        }
        n = m;
        if (n < 3) return 0;
        for (int i = 0; i < n; ++i)
            for (int q = 0; q < 7; ++q) poly[i][q] = tmp[i][q];
    }
    for (int i = 0; i < n; ++i)
        if (!(poly[i][3] > 0.0f)) return 0;
    const int nsub = n - 2;
    for (int s = 0; s < nsub; ++s) {
        float sv[3][4], sb[3][3];
        const int idx[3] = {0, s + 1, s + 2};
        for (int k = 0; k < 3; ++k) {
            for (int c = 0; c < 4; ++c) sv[k][c] = poly[idx[k]][c];
            for (int i = 0; i < 3; ++i) sb[k][i] = poly[idx[k]][4 + i];
        }
        Rec r;
        make_record(sv, sb, W, H, f, r);
        frame_recs[rec_index(F, f, s)] = r;
    }
    return nsub;
}

__device__ inline void count_tiles(int i0, int i1, int j0, int j1, int ntx, uint32_t *tile_count_frame)
{
    if (i0 > i1) return;
    const int tx0 = i0 / kTile, tx1 = i1 / kTile, ty0 = j0 / kTile, ty1 = j1 / kTile;
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&tile_count_frame[ty * ntx + tx], 1u);
}

constexpr int kSetupThreads = 64;  // 50k faces -> 784 workgroups: spread over all 256 CUs

__global__ __launch_bounds__(kSetupThreads) void setup_kernel(const float *__restrict__ verts,
                                                              const int32_t *__restrict__ faces, int B, int V, int F,
                                                              int W, int H, int ntx, int ntiles, int64_t nrec,
                                                              Rec *__restrict__ recs, FaceData *__restrict__ fdata,
                                                              uint32_t *__restrict__ tile_count, uint32_t *__restrict__ flag)
{
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)B * F) return;
    const int b = (int)(gid / F), f = (int)(gid - (int64_t)b * F);
    Rec *frame_recs = recs + (int64_t)b * nrec;
    const float *vb = verts + (int64_t)b * V * 4;
    const int32_t i0 = faces[gid * 3], i1 = faces[gid * 3 + 1], i2 = faces[gid * 3 + 2];
    const int32_t vidx[3] = {i0, i1, i2};
    Tri tri;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int32_t vi = vidx[k];
        if (vi < 0 || vi >= V) {
            ok = false;
            tri.v[k][0] = tri.v[k][1] = tri.v[k][2] = 0.0f;
            tri.v[k][3] = 1.0f;
        } else {
            const float4 p = *reinterpret_cast<const float4 *>(vb + (int64_t)vi * 4);
            tri.v[k][0] = p.x; tri.v[k][1] = p.y; tri.v[k][2] = p.z; tri.v[k][3] = p.w;
            ok = ok && finite4(tri.v[k]);
        }
    }
    if (!(i0 >= 0 && i0 < V && i1 >= 0 && i1 < V && i2 >= 0 && i2 < V)) atomicOr(flag, 1u);
    uint32_t *tc = tile_count + (int64_t)b * ntiles;
    FaceData fd;
    fd.v[0] = i0; fd.v[1] = i1; fd.v[2] = i2;
    fd.w[0] = tri.v[0][3]; fd.w[1] = tri.v[1][3]; fd.w[2] = tri.v[2][3];
    fd.pad = 0;
    Rec r;
    set_empty(r, f);
    int nsub = 0;
    if (ok) {
        const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
        bool fast = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float w = tri.v[k][3];
            fast = fast && (w > 0.0f && fabsf(tri.v[k][0]) <= gx * w && fabsf(tri.v[k][1]) <= gy * w);
        }
        if (fast) {
            const float id[3][3] = {{1.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, {0.f, 0.f, 1.f}};
            make_record(tri.v, id, W, H, f, r);
            nsub = 1;
            frame_recs[f] = r;
            count_tiles(r.i0, r.i1, r.j0, r.j1, ntx, tc);
        } else {
            frame_recs[f] = r;  // empty unless clip_face overwrites it
            nsub = clip_face(tri, W, H, F, f, frame_recs);
            for (int s = 0; s < nsub; ++s) {
                const Rec &q = frame_recs[rec_index(F, f, s)];
                count_tiles(q.i0, q.i1, q.j0, q.j1, ntx, tc);
            }
        }
    } else {
        frame_recs[f] = r;
    }
    fd.nsub = nsub;
    fdata[gid] = fd;
}

// ------------------------------------------------------------------------------------------------
// K2: exclusive scan of the per-tile counts (one workgroup; B*ntiles is 4096 per 1024^2 frame)

constexpr int kScanThreads = 1024;
constexpr int kScanPerThread = 4;

__global__ __launch_bounds__(kScanThreads) void scan_kernel(const uint32_t *__restrict__ in, uint64_t *__restrict__ out,
                                                            int64_t n)
{
    __shared__ uint64_t wave_sums[kScanThreads / 64];
    __shared__ uint64_t carry_s;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint64_t carry = 0;
    for (int64_t base = 0; base < n; base += (int64_t)kScanThreads * kScanPerThread) {
        const int64_t k0 = base + (int64_t)t * kScanPerThread;
        uint32_t v[kScanPerThread];
        uint64_t local = 0;
        if (k0 + kScanPerThread <= n) {
            const uint4 q = *reinterpret_cast<const uint4 *>(in + k0);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int q = 0; q < kScanPerThread; ++q) v[q] = (k0 + q < n) ? in[k0 + q] : 0u;
        }
#pragma unroll
        for (int q = 0; q < kScanPerThread; ++q) local += v[q];
        uint64_t x = local;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) wave_sums[wave] = x;
        __syncthreads();
        if (wave == 0) {
            uint64_t w = lane < kScanThreads / 64 ? wave_sums[lane] : 0;
#pragma unroll
            for (int d = 1; d < kScanThreads / 64; d <<= 1) {
                const uint64_t y = __shfl_up(w, d, 64);
                if (lane >= d) w += y;
            }
            if (lane < kScanThreads / 64) wave_sums[lane] = w;
            if (lane == kScanThreads / 64 - 1) carry_s = w;
        }
        __syncthreads();
        uint64_t run = carry + (wave > 0 ? wave_sums[wave - 1] : 0) + (x - local);
#pragma unroll
        for (int q = 0; q < kScanPerThread; ++q) {
            if (k0 + q < n) out[k0 + q] = run;
            run += v[q];
        }
        carry += carry_s;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// K3: fill bins (order inside a bin is irrelevant: the depth resolve is a commutative min).
// The common <= 3x3-tile case issues all its returning atomics back to back (one latency, not n).

__device__ inline void fill_one(int64_t ri, int i0, int i1, int j0, int j1, int b, int ntx, int ntiles,
                                const uint64_t *__restrict__ tile_offset, uint32_t *__restrict__ tile_cursor,
                                int32_t *__restrict__ bins, int64_t capacity)
{
    if (i0 > i1) return;
    const int tx0 = i0 / kTile, tx1 = i1 / kTile, ty0 = j0 / kTile, ty1 = j1 / kTile;
    const int nx = tx1 - tx0 + 1, ny = ty1 - ty0 + 1;
    const int64_t base = (int64_t)b * ntiles;
    if (nx <= 3 && ny <= 3) {
        uint32_t pos[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int qx = q % 3, qy = q / 3;
            if (qx < nx && qy < ny) pos[q] = atomicAdd(&tile_cursor[base + (ty0 + qy) * ntx + tx0 + qx], 1u);
        }
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int qx = q % 3, qy = q / 3;
            if (qx < nx && qy < ny) {
                const int64_t t = base + (ty0 + qy) * ntx + tx0 + qx;
                const uint64_t dst = tile_offset[t] + pos[q];
                if (dst < (uint64_t)capacity) bins[dst] = (int32_t)ri;
            }
        }
        return;
    }
    for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
            const int64_t t = base + ty * ntx + tx;
            const uint32_t pos = atomicAdd(&tile_cursor[t], 1u);
            const uint64_t dst = tile_offset[t] + pos;
            if (dst < (uint64_t)capacity) bins[dst] = (int32_t)ri;
        }
}

__global__ __launch_bounds__(kSetupThreads) void fill_kernel(const Rec *__restrict__ recs,
                                                             const FaceData *__restrict__ fdata, int B, int F, int ntx,
                                                             int ntiles, int64_t nrec,
                                                             const uint64_t *__restrict__ tile_offset,
                                                             uint32_t *__restrict__ tile_cursor,
                                                             int32_t *__restrict__ bins, int64_t capacity)
{
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)B * F) return;
    const int b = (int)(gid / F), f = (int)(gid - (int64_t)b * F);
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const int n = fdata[gid].nsub;
    for (int s = 0; s < n; ++s) {
        const int64_t ri = rec_index(F, f, s);
        const Rec &r = frame_recs[ri];
        fill_one(ri, r.i0, r.i1, r.j0, r.j1, b, ntx, ntiles, tile_offset, tile_cursor, bins, capacity);
    }
}

// ------------------------------------------------------------------------------------------------
// K4: tile raster + resolve
//
// Exactness with 32-bit lanes: per (entry, strip) the staging thread evaluates the int64 edge
// functions at the strip's first pixel, folds in the top-left bias (E + owned > 0  <=>  inside), and
// classifies each edge over the 16x4 strip: all-outside (entry culled for this strip), all-inside
// (value pinned to 2^30), or straddling.  For "small" triangles (|A|,|B| < 2^16) a straddling edge
// satisfies |E| < 2^29 over the strip, so lanes step it with 24-bit multiply-adds exactly; larger
// triangles fall back to per-lane int64 evaluation.  Results are bit-identical to R3 either way.

constexpr int kStrips = 4;           // waves per tile; a strip is 16 x 4 pixels
constexpr int kChunk = 256;          // entries staged per round
constexpr int kSmallEdge = 1 << 16;  // |A|,|B| bound for the 32-bit path
constexpr uint32_t kStripCulled = 1u, kStripLarge = 2u;

struct alignas(16) StripEdges {
    int32_t e[3];
    uint32_t flags;
};
struct alignas(16) RasterEntry {  // 128 B of LDS per staged entry
    StripEdges strip[kStrips];     // 64 B
    int32_t A[3], B[3];            // 24 B
    float fx0, fy0, z0, za, zb;    // 20 B
    int32_t face, ri;              // 8 B
    int32_t pad[3];
};
static_assert(sizeof(RasterEntry) == 128, "RasterEntry must be 128 B");

struct PixelState {
    uint64_t best;
    int32_t best_rec;
};

__device__ __forceinline__ void depth_update(float za, float zb, float fx0, float fy0, float z0, int32_t face,
                                             int32_t ri, float fxl, float fyl, PixelState &st)
{
    // R4, same operation order as sample_depth()
    const float zw = (za * (fxl - fx0) + zb * (fyl - fy0)) + z0;
    if (!(zw >= 0.0f && zw <= 1.0f)) return;
    const uint32_t q = (uint32_t)(zw * 16777215.0f + 0.5f);
    if (q >= kDepthMax) return;
    const uint64_t key = ((uint64_t)q << 32) | (uint32_t)face;
    if (key < st.best) {
        st.best = key;
        st.best_rec = ri;
    }
}

__device__ inline void stage_entry(const Rec *__restrict__ frame_recs, int32_t ri, int tx, int ty, RasterEntry &E)
{
    const RasterPart R = *reinterpret_cast<const RasterPart *>(&frame_recs[ri]);
    bool small = true;
    int64_t owned[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        owned[k] = (R.A[k] > 0 || (R.A[k] == 0 && R.B[k] < 0)) ? 1 : 0;
        small = small && R.A[k] > -kSmallEdge && R.A[k] < kSmallEdge && R.B[k] > -kSmallEdge && R.B[k] < kSmallEdge;
    }
#pragma unroll
    for (int w = 0; w < kStrips; ++w) {
        const int si0 = tx * kTile, si1 = si0 + kTile - 1, sj0 = ty * kTile + w * 4, sj1 = sj0 + 3;
        uint32_t flags = 0;
        int32_t ev[3] = {0, 0, 0};
        if (R.i1 < si0 || R.i0 > si1 || R.j1 < sj0 || R.j0 > sj1) {
            flags = kStripCulled;
        } else if (!small) {
            flags = kStripLarge;
        } else {
            const int64_t px0 = (int64_t)si0 * 256 + 128, py0 = (int64_t)sj0 * 256 + 128;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int64_t e0 = (int64_t)R.A[k] * px0 + (int64_t)R.B[k] * py0 + R.C[k] + owned[k];
                const int64_t sx = (int64_t)R.A[k] * (15 * 256), sy = (int64_t)R.B[k] * (3 * 256);
                const int64_t emin = e0 + (sx < 0 ? sx : 0) + (sy < 0 ? sy : 0);
                const int64_t emax = e0 + (sx > 0 ? sx : 0) + (sy > 0 ? sy : 0);
                if (emax <= 0) flags = kStripCulled;
                ev[k] = emin > 0 ? (1 << 30) : (int32_t)e0;
            }
        }
        E.strip[w].e[0] = ev[0]; E.strip[w].e[1] = ev[1]; E.strip[w].e[2] = ev[2];
        E.strip[w].flags = flags;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { E.A[k] = R.A[k]; E.B[k] = R.B[k]; }
    E.fx0 = R.fx0; E.fy0 = R.fy0; E.z0 = R.z0; E.za = R.za; E.zb = R.zb;
    E.face = R.face;
    E.ri = ri;
}

template <int CC>
__global__ __launch_bounds__(256) void raster_kernel(const float *__restrict__ background, const float *__restrict__ colors,
                                                     const Rec *__restrict__ recs, const FaceData *__restrict__ fdata,
                                                     const uint32_t *__restrict__ tile_count,
                                                     const uint64_t *__restrict__ tile_offset,
                                                     const int32_t *__restrict__ bins, int64_t capacity,
                                                     int B, int H, int W, int Cdyn, int V, int F, int ntx, int ntiles,
                                                     int64_t nrec, float *__restrict__ pixels, int32_t *__restrict__ gbuffer)
{
    const int C = CC > 0 ? CC : Cdyn;
    __shared__ RasterEntry lds[kChunk];
    const int tile = blockIdx.x, b = blockIdx.y;
    const int tx = tile % ntx, ty = tile / ntx;
    const int t = threadIdx.x, lx = t & 15, ly = t >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int i = tx * kTile + lx, j = ty * kTile + ly;
    const int dx = lx * 256, dy = (ly & 3) * 256;
    const float fxl = (float)i + 0.5f, fyl = (float)j + 0.5f;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    PixelState st{~0ull, -1};

    const int64_t tt = (int64_t)b * ntiles + tile;
    const uint32_t cnt = tile_count[tt];
    const uint64_t off = tile_offset[tt];
    if (off + cnt <= (uint64_t)capacity) {
        for (uint32_t base = 0; base < cnt; base += kChunk) {
            const int n = (int)min((uint32_t)kChunk, cnt - base);
            __syncthreads();
            if (t < n) stage_entry(frame_recs, bins[off + base + t], tx, ty, lds[t]);
            __syncthreads();
            for (int e = 0; e < n; ++e) {
                const RasterEntry &R = lds[e];
                const StripEdges se = R.strip[wave];
                const uint32_t flags = __builtin_amdgcn_readfirstlane(se.flags);
                if (flags & kStripCulled) continue;
                bool in;
                if (!(flags & kStripLarge)) {
                    const int32_t e0 = se.e[0] + __mul24(R.A[0], dx) + __mul24(R.B[0], dy);
                    const int32_t e1 = se.e[1] + __mul24(R.A[1], dx) + __mul24(R.B[1], dy);
                    const int32_t e2 = se.e[2] + __mul24(R.A[2], dx) + __mul24(R.B[2], dy);
                    in = min(e0, min(e1, e2)) > 0;
                } else {
                    const Rec &r = frame_recs[R.ri];
                    int64_t E[3];
                    edge_values(r, i, j, E);
                    in = inside(r, E);
                }
                if (in) depth_update(R.za, R.zb, R.fx0, R.fy0, R.z0, R.face, R.ri, fxl, fyl, st);
            }
        }
    } else {
        // bin overflow (capacity too small for this input): test every record of the frame
        for (int f = 0; f < F; ++f) {
            const int ns = fdata[(int64_t)b * F + f].nsub;
            for (int s = 0; s < ns; ++s) {
                const int64_t ri = rec_index(F, f, s);
                const Rec &r = frame_recs[ri];
                if (r.i0 > r.i1) continue;
                int64_t E[3];
                edge_values(r, i, j, E);
                if (!inside(r, E)) continue;
                depth_update(r.za, r.zb, r.fx0, r.fy0, r.z0, r.face, (int32_t)ri, fxl, fyl, st);
            }
        }
    }

    if (i >= W || j >= H) return;
    const int row = H - 1 - j;
    const int64_t o = ((int64_t)b * H + row) * W + i;
    gbuffer[o] = st.best_rec;
    float *out = pixels + o * C;
    if (st.best_rec < 0) {
        const float *bg = background + o * C;
        for (int c = 0; c < C; ++c) out[c] = bg[c];
        return;
    }
    const Rec &r = frame_recs[st.best_rec];
    const FaceData fd = fdata[(int64_t)b * F + face_of_record(st.best_rec, F)];
    int64_t E[3];
    edge_values(r, i, j, E);
    float lam[3] = {0.0f, 0.0f, 0.0f};
    parent_lambda(r, E, lam);
    const float *cb = colors + (int64_t)b * V * C;
    const float *c0 = cb + (int64_t)fd.v[0] * C, *c1 = cb + (int64_t)fd.v[1] * C, *c2 = cb + (int64_t)fd.v[2] * C;
    for (int c = 0; c < C; ++c) out[c] = (lam[0] * c0[c] + lam[1] * c1[c]) + lam[2] * c2[c];
}

// ------------------------------------------------------------------------------------------------
// K5: backward
//
// One 256-thread workgroup per 16x16 tile, one lane per pixel.  Every contribution of a lane goes to
// the face visible at its own pixel: colour gradients lambda_k * G, and the share of the four
// neighbour pairs around the pixel that this face owns (a pair's other owner is handled by the lane
// on the other side, same-face pairs by the lower lane only).  Reduction without global contention:
//   1. DPP segmented scan along each 16-pixel row (one DPP row == one pixel row) sums runs of equal
//      record index into the run's last lane;
//   2. run tails ds_add into a per-tile LDS hash table keyed by record index (vertex ids cached);
//   3. one wave-instruction of global float atomics per (tile, record): <= 9+3C lanes, ~3 cache lines.

// Does face f cover pixel (i,j)?  `hint` is a record of f to try first (the one covering a nearby pixel).
__device__ bool covers_face(const Rec *frame_recs, const FaceData *fdata_frame, int F, int f, int64_t hint, int i, int j)
{
    {
        const Rec &r = frame_recs[hint];
        if (!(r.i0 > r.i1 || i < r.i0 || i > r.i1 || j < r.j0 || j > r.j1)) {
            int64_t E[3];
            edge_values(r, i, j, E);
            if (inside(r, E)) return true;
        }
    }
    const int n = fdata_frame[f].nsub;
    if (n <= 1) return false;
    for (int s = 0; s < n; ++s) {
        const int64_t ri = rec_index(F, f, s);
        if (ri == hint) continue;
        const Rec &r = frame_recs[ri];
        if (r.i0 > r.i1 || i < r.i0 || i > r.i1 || j < r.j0 || j > r.j1) continue;
        int64_t E[3];
        edge_values(r, i, j, E);
        if (inside(r, E)) return true;
    }
    return false;
}

template <int D>
__device__ __forceinline__ float dpp_shr_f(float v)  // lane l <- lane l-D of the same 16-lane row, 0 if none
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x110 + D, 0xF, 0xF, false));
}
template <int D>
__device__ __forceinline__ int dpp_shr_i(int v, int fill)
{
    return __builtin_amdgcn_update_dpp(fill, v, 0x110 + D, 0xF, 0xF, false);
}
template <int D>
__device__ __forceinline__ int dpp_shl_i(int v, int fill)  // lane l <- lane l+D of the same row
{
    return __builtin_amdgcn_update_dpp(fill, v, 0x100 + D, 0xF, 0xF, false);
}

constexpr int kHalo = kTile + 2;   // staged tile with a one-pixel border
constexpr int kHashSlots = 256;    // >= distinct records a 256-pixel tile can hold

template <int CC>
__global__ __launch_bounds__(256) void grad_kernel(const float *__restrict__ pixels, const float *__restrict__ grad_pixels,
                                                   const int32_t *__restrict__ gbuffer, const Rec *__restrict__ recs,
                                                   const FaceData *__restrict__ fdata, int B, int H, int W, int Cdyn,
                                                   int V, int F, int ntx, int64_t nrec, float *__restrict__ grad_verts,
                                                   float *__restrict__ grad_colors, float *__restrict__ grad_bg)
{
    constexpr int CM = CC > 0 ? CC : DIRT_MAX_CHANNELS;
    constexpr int NVM = 9 + 3 * CM;
    const int C = CC > 0 ? CC : Cdyn;
    const int NV = 9 + 3 * C;
    __shared__ int32_t s_rec[kHalo * kHalo];
    __shared__ float s_G[kHalo * kHalo * CM];
    __shared__ float s_I[kHalo * kHalo * CM];
    __shared__ int32_t s_keys[kHashSlots];
    __shared__ int32_t s_list[kHashSlots];
    __shared__ int32_t s_vid[kHashSlots * 3];
    __shared__ float s_vals[kHashSlots * NVM];
    __shared__ int32_t s_n;

    const int tile = blockIdx.x, b = blockIdx.y;
    const int tx = tile % ntx, ty = tile / ntx;
    const int t = threadIdx.x, lx = t & 15, ly = t >> 4;
    const int i = tx * kTile + lx, j = ty * kTile + ly;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const FaceData *fdata_frame = fdata + (int64_t)b * F;

    for (int k = t; k < kHashSlots; k += 256) s_keys[k] = -1;
    for (int k = t; k < kHashSlots * NVM; k += 256) s_vals[k] = 0.0f;
    if (t == 0) s_n = 0;
    // stage gbuffer / G / I of the tile plus a one-pixel halo (window coords, j from the bottom)
    const int hi0 = tx * kTile - 1, hj0 = ty * kTile - 1;
    for (int k = t; k < kHalo * kHalo; k += 256) {
        const int hi = hi0 + k % kHalo, hj = hj0 + k / kHalo;
        if (hi < 0 || hj < 0 || hi >= W || hj >= H) {
            s_rec[k] = -2;
            continue;
        }
        const int64_t o = ((int64_t)b * H + (H - 1 - hj)) * W + hi;
        s_rec[k] = gbuffer[o];
        for (int c = 0; c < C; ++c) {
            s_G[k * CM + c] = grad_pixels[o * C + c];
            s_I[k * CM + c] = pixels[o * C + c];
        }
    }
    __syncthreads();

    const bool in_frame = i < W && j < H;
    const int kme = (ly + 1) * kHalo + (lx + 1);
    const int32_t rp = in_frame ? s_rec[kme] : -2;
    if (in_frame) {
        const int64_t o = ((int64_t)b * H + (H - 1 - j)) * W + i;
        for (int c = 0; c < C; ++c) grad_bg[o * C + c] = rp < 0 ? s_G[kme * CM + c] : 0.0f;
    }

    float acc[NVM];
#pragma unroll
    for (int v = 0; v < NVM; ++v) acc[v] = 0.0f;
    int key = -1;
    FaceData fd;
    if (rp >= 0) {
        const Rec &r = frame_recs[rp];
        const int f = face_of_record(rp, F);
        fd = fdata_frame[f];
        int64_t Ep[3];
        edge_values(r, i, j, Ep);
        {
            float lam[3];
            if (parent_lambda(r, Ep, lam)) {
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < C; ++c) acc[9 + k * C + c] = lam[k] * s_G[kme * CM + c];
            }
        }
        // the four pairs around the pixel: dir 0 right, 1 left (x axis); 2 up, 3 down (y axis, window)
#pragma unroll
        for (int dir = 0; dir < 4; ++dir) {
            const int axis = dir >> 1;
            const bool me_low = (dir & 1) == 0;
            const int di = axis == 0 ? (me_low ? 1 : -1) : 0, dj = axis == 1 ? (me_low ? 1 : -1) : 0;
            const int kq = kme + dj * kHalo + di;
            const int32_t rq = s_rec[kq];
            if (rq == -2) continue;
            const int klo = me_low ? kme : kq, kup = me_low ? kq : kme;
            float a = 0.0f;
            for (int c = 0; c < C; ++c)
                a += (s_G[klo * CM + c] + s_G[kup * CM + c]) * (s_I[kup * CM + c] - s_I[klo * CM + c]);
            const float s = -0.5f * a;
            if (s == 0.0f) continue;
            const int iq = i + di, jq = j + dj;
            const int fq = rq >= 0 ? face_of_record(rq, F) : -1;
            float omega;
            if (fq == f) {
                omega = me_low ? 1.0f : 0.0f;
            } else if (fq < 0) {
                omega = 1.0f;
            } else {
                const bool mine_covers_other = covers_face(frame_recs, fdata_frame, F, f, rp, iq, jq);
                const bool other_covers_me = covers_face(frame_recs, fdata_frame, F, fq, rq, i, j);
                omega = (!mine_covers_other && other_covers_me) ? 1.0f
                        : (mine_covers_other && !other_covers_me) ? 0.0f : 0.5f;
            }
            if (omega == 0.0f) continue;
            int64_t Eq[3], E[3];
            edge_values(r, iq, jq, Eq);
#pragma unroll
            for (int k = 0; k < 3; ++k) E[k] = Ep[k] + Eq[k];
            float lam[3];
            if (!parent_lambda(r, E, lam)) continue;
            const float Wm = (lam[0] * fd.w[0] + lam[1] * fd.w[1]) + lam[2] * fd.w[2];
            if (Wm == 0.0f) continue;
            const int ilo = me_low ? i : iq, jlo = me_low ? j : jq;
            const float half = axis == 0 ? 0.5f * (float)W : 0.5f * (float)H;
            const float mid = axis == 0 ? (float)(ilo + 1) : (float)(jlo + 1);
            const float ndc = mid / half - 1.0f;
            const float tt = ((omega * s) * half) / Wm;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float g = tt * lam[k];
                acc[k * 3 + axis] += g;
                acc[k * 3 + 2] += -(g * ndc);
            }
        }
        key = rp;
    }

    // 1. segmented sum over runs of equal key along the 16-lane row
    const int kl = dpp_shr_i<1>(key, -3);
    int start = (lx == 0 || kl != key) ? lx : -1;
    start = max(start, dpp_shr_i<1>(start, -1));
    start = max(start, dpp_shr_i<2>(start, -1));
    start = max(start, dpp_shr_i<4>(start, -1));
    start = max(start, dpp_shr_i<8>(start, -1));
#pragma unroll
    for (int v = 0; v < NVM; ++v) {
        float x = acc[v];
        float y;
        y = dpp_shr_f<1>(x); if (lx - 1 >= start) x += y;
        y = dpp_shr_f<2>(x); if (lx - 2 >= start) x += y;
        y = dpp_shr_f<4>(x); if (lx - 4 >= start) x += y;
        y = dpp_shr_f<8>(x); if (lx - 8 >= start) x += y;
        acc[v] = x;
    }
    const int kr = dpp_shl_i<1>(key, -3);
    const bool tail = key >= 0 && (lx == 15 || kr != key);

    // 2. run tails accumulate into the tile's LDS hash table
    if (tail) {
        int slot = (int)(((uint32_t)key * 2654435761u) >> 24) & (kHashSlots - 1);
        while (true) {
            const int old = atomicCAS(&s_keys[slot], -1, key);
            if (old == -1) {
                s_list[atomicAdd(&s_n, 1)] = slot;
                s_vid[slot * 3 + 0] = fd.v[0];
                s_vid[slot * 3 + 1] = fd.v[1];
                s_vid[slot * 3 + 2] = fd.v[2];
                break;
            }
            if (old == key) break;
            slot = (slot + 1) & (kHashSlots - 1);
        }
        for (int v = 0; v < NV; ++v)
            if (acc[v] != 0.0f) atomicAdd(&s_vals[slot * NVM + v], acc[v]);
    }
    __syncthreads();

    // 3. flush: one wave-instruction of global atomics per (tile, record)
    const int n = s_n, wave = t >> 6, lane = t & 63;
    float *gvb = grad_verts + (int64_t)b * V * 4;
    float *gcb = grad_colors + (int64_t)b * V * C;
    if (lane < NV) {
        const int k = lane < 9 ? lane / 3 : (lane - 9) / C;
        const int comp = lane < 9 ? ((lane % 3) == 2 ? 3 : lane % 3) : (lane - 9) % C;
        for (int e = wave; e < n; e += 4) {
            const int slot = s_list[e];
            const float val = s_vals[slot * NVM + lane];
            if (val == 0.0f) continue;
            const int vtx = s_vid[slot * 3 + k];
            if (lane < 9) atomicAdd(gvb + (int64_t)vtx * 4 + comp, val);
            else atomicAdd(gcb + (int64_t)vtx * C + comp, val);
        }
    }
}

__global__ void check_faces_kernel(const int32_t *__restrict__ faces, int64_t n, int V, uint32_t *flag)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        if (faces[k] < 0 || faces[k] >= V) atomicOr(flag, 1u);
}

}  // namespace

// ================================================================================================
// C ABI

extern "C" {

int dirt_abi_version(void) { return 2; }

const char *dirt_last_error(void) { return g_last_error.c_str(); }

int dirt_workspace_sizes(int B, int H, int W, int C, int V, int F, int64_t bin_capacity, size_t *saved_bytes,
                         size_t *scratch_bytes)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    Layout L;
    rc = make_layout(B, H, W, F, bin_capacity, L);
    if (rc) return rc;
    if (saved_bytes) *saved_bytes = L.saved_total;
    if (scratch_bytes) *scratch_bytes = L.scratch_total;
    return DIRT_OK;
}

int dirt_rasterise_fwd(const float *background, const float *vertices, const float *vertex_colors,
                       const int32_t *faces, const float *camera_pos, int B, int H, int W, int C, int V, int F,
                       int shader_id, float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes, void *scratch,
                       size_t scratch_bytes, int64_t bin_capacity, void *stream_)
{
    (void)camera_pos;
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (shader_id != DIRT_SHADER_GOURAUD) return fail(DIRT_EINVAL, "Rasterise: unsupported shader_id");
    if (B == 0) return DIRT_OK;
    if (!background || !pixels || !gbuffer || !saved || !scratch || (F > 0 && (!faces || !vertices)) ||
        (V > 0 && (!vertices || !vertex_colors)))
        return fail(DIRT_EINVAL, "Rasterise: null tensor pointer");
    Layout L;
    rc = make_layout(B, H, W, F, bin_capacity, L);
    if (rc) return rc;
    if (saved_bytes < L.saved_total || scratch_bytes < L.scratch_total)
        return fail(DIRT_EINVAL, "Rasterise: workspace smaller than dirt_workspace_sizes()");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    char *sv = static_cast<char *>(saved), *sc = static_cast<char *>(scratch);
    Rec *recs = reinterpret_cast<Rec *>(sv + L.saved_recs);
    FaceData *fdata = reinterpret_cast<FaceData *>(sv + L.saved_fdata);
    uint32_t *tile_count = reinterpret_cast<uint32_t *>(sc + L.off_count);
    uint32_t *tile_cursor = reinterpret_cast<uint32_t *>(sc + L.off_cursor);
    uint64_t *tile_offset = reinterpret_cast<uint64_t *>(sc + L.off_offset);
    uint32_t *flag = reinterpret_cast<uint32_t *>(sc + L.off_flag);
    int32_t *bins = reinterpret_cast<int32_t *>(sc + L.off_bins);
    const int64_t nt = (int64_t)B * L.ntiles;

    // counts and cursors are adjacent: one memset
    HIP_TRY(hipMemsetAsync(tile_count, 0, L.off_offset - L.off_count, stream));
    const int64_t nf = (int64_t)B * F;
    const unsigned setup_blocks = (unsigned)((nf + kSetupThreads - 1) / kSetupThreads);
    if (nf > 0) {
        ProfScope ps(K_SETUP, stream);
        setup_kernel<<<dim3(setup_blocks), dim3(kSetupThreads), 0, stream>>>(
            vertices, faces, B, V, F, W, H, L.ntx, L.ntiles, L.nrec, recs, fdata, tile_count, flag);
        HIP_TRY(hipGetLastError());
    }
    {
        ProfScope ps(K_SCAN, stream);
        scan_kernel<<<dim3(1), dim3(kScanThreads), 0, stream>>>(tile_count, tile_offset, nt);
    }
    HIP_TRY(hipGetLastError());
    if (nf > 0) {
        ProfScope ps(K_FILL, stream);
        fill_kernel<<<dim3(setup_blocks), dim3(kSetupThreads), 0, stream>>>(
            recs, fdata, B, F, L.ntx, L.ntiles, L.nrec, tile_offset, tile_cursor, bins, L.bin_capacity);
        HIP_TRY(hipGetLastError());
    }
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
    ProfScope ps(K_RASTER, stream);
#define LAUNCH_RASTER(CC)                                                                                        \
    raster_kernel<CC><<<grid, dim3(256), 0, stream>>>(background, vertex_colors, recs, fdata, tile_count,         \
                                                      tile_offset, bins, L.bin_capacity, B, H, W, C, V, F, L.ntx, \
                                                      L.ntiles, L.nrec, pixels, gbuffer)
    if (C == 1) LAUNCH_RASTER(1);
    else if (C == 3) LAUNCH_RASTER(3);
    else LAUNCH_RASTER(0);
#undef LAUNCH_RASTER
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_rasterise_bwd(const float *vertices, const float *vertex_colors, const int32_t *faces, const float *pixels,
                       const float *grad_pixels, const int32_t *gbuffer, const void *saved, int B, int H, int W, int C,
                       int V, int F, float *grad_vertices, float *grad_vertex_colors, float *grad_background,
                       void *stream_)
{
    // vertices / vertex_colors / faces are part of the contract (rasterise_grad_common.h:19-24); the
    // forward's FaceData in `saved` already holds what the kernel needs from them.
    (void)vertex_colors;
    (void)vertices;
    (void)faces;
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (B == 0) return DIRT_OK;
    if (!pixels || !grad_pixels || !gbuffer || !saved || !grad_background ||
        (V > 0 && (!grad_vertices || !grad_vertex_colors)))
        return fail(DIRT_EINVAL, "RasteriseGrad: null tensor pointer");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const char *sv = static_cast<const char *>(saved);
    const Rec *recs = reinterpret_cast<const Rec *>(sv + L.saved_recs);
    const FaceData *fdata = reinterpret_cast<const FaceData *>(sv + L.saved_fdata);
    if (V > 0) {
        HIP_TRY(hipMemsetAsync(grad_vertices, 0, (size_t)B * V * 4 * sizeof(float), stream));
        HIP_TRY(hipMemsetAsync(grad_vertex_colors, 0, (size_t)B * V * C * sizeof(float), stream));
    }
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
    ProfScope ps(K_GRAD, stream);
#define LAUNCH_GRAD(CC)                                                                                       \
    grad_kernel<CC><<<grid, dim3(256), 0, stream>>>(pixels, grad_pixels, gbuffer, recs, fdata, B, H, W, C, V, F, \
                                                    L.ntx, L.nrec, grad_vertices, grad_vertex_colors,            \
                                                    grad_background)
    if (C == 1) LAUNCH_GRAD(1);
    else if (C == 3) LAUNCH_GRAD(3);
    else LAUNCH_GRAD(0);
#undef LAUNCH_GRAD
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_profile_enable(int enable)
{
    for (int k = 0; k < K_COUNT; ++k) {
        for (auto &p : g_prof.ev[k]) {
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
        g_prof.ev[k].clear();
    }
    g_prof.enabled = enable != 0;
    return DIRT_OK;
}

int dirt_profile_read(int kernel_id, const char **name, int *launches, double *total_ms)
{
    if (kernel_id < 0 || kernel_id >= K_COUNT) return fail(DIRT_EINVAL, "dirt_profile_read: bad kernel id");
    double tot = 0.0;
    for (auto &p : g_prof.ev[kernel_id]) {
        HIP_TRY(hipEventSynchronize(p.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.first, p.second));
        tot += ms;
    }
    if (name) *name = kKernelNames[kernel_id];
    if (launches) *launches = (int)g_prof.ev[kernel_id].size();
    if (total_ms) *total_ms = tot;
    return DIRT_OK;
}

int dirt_check_faces(const int32_t *faces, int B, int V, int F, void *scratch, size_t scratch_bytes, void *stream_)
{
    if (B < 0 || F < 0 || V < 0) return fail(DIRT_EINVAL, "dirt_check_faces: negative size");
    if (!scratch || scratch_bytes < 256) return fail(DIRT_EINVAL, "dirt_check_faces: scratch too small");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    uint32_t *flag = reinterpret_cast<uint32_t *>(scratch);
    HIP_TRY(hipMemsetAsync(flag, 0, 4, stream));
    const int64_t n = (int64_t)B * F * 3;
    if (n > 0) {
        check_faces_kernel<<<dim3(1024), dim3(256), 0, stream>>>(faces, n, V, flag);
        HIP_TRY(hipGetLastError());
    }
    uint32_t h = 0;
    HIP_TRY(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (h) return fail(DIRT_EFACE, "Rasterise: face index out of range [0, vertex count)");
    return DIRT_OK;
}

}  // extern "C"
