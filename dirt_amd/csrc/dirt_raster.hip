// dirt_raster.hip -- MI355X (gfx950) software rasteriser behind the C ABI of include/dirt_mi355x.h.
//
// CDNA4 has no graphics pipeline, so the reference's GL fixed-function raster
// (csrc/rasterise_egl.cpp:440-487 + the NVIDIA driver) becomes a compute pipeline:
//
//   K1 setup_kernel    one thread per (frame, face): fetch 3 clip vertices, project + snap (R1/R2),
//                      edge equations (R3), depth plane (R4), guard-band clipping (R5, rare slow path);
//                      writes 128-B setup records + 32-B FaceData, counts (coarse tile, record) pairs
//                      (one fire-and-forget device atomic per touched (workgroup, coarse tile)).
//   K3 fill_kernel     every workgroup scans its frame's per-tile totals into bin offsets (frame-local
//                      bin regions), then scatters each record index into the coarse bins it overlaps.
//                      (K2, a separate scan launch, no longer exists; its profile slot stays empty.)
//   K4 raster_kernel   one 256-thread workgroup per 16x16 tile (a wave per 8x8 block): stages the
//                      tile's records in LDS with tile-relative 32-bit edge values (exact), each lane
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
#include <algorithm>

#include "../../include/dirt_mi355x.h"
#include "raster_rules.h"
#include "oceanic.h"
#include "hill.h"

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
enum KernelId { K_SETUP = 0, K_RASTER, K_GRAD, K_COUNT };
const char *const kKernelNames[K_COUNT] = {"setup_kernel", "raster_kernel", "grad_kernel"};
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
// Workspace layout.  saved = records [B][6F] (128 B) + FaceData [B][F] (32 B) + 4 neighbour-coverage
// bits per pixel: what the backward reads.  scratch = two sets of per-coarse-tile counts (alternating
// forwards: see kParP), a flag area, and the coarse bins: one fixed-capacity slab per (frame, coarse tile).
//
// Binning is two-level.  Coarse tiles (64x64 px, 128x128 above 4096 px) are binned by the setup kernel
// itself: each workgroup of 256 faces counts its (record, coarse tile) pairs in LDS, reserves its range
// of every touched slab with one returning device atomic per (workgroup, coarse tile), and writes the
// entries -- no separate count/scan/fill passes (a dependent kernel boundary costs ~1.7 us, and the
// fill pass had to re-read every record).  HBM is plentiful (288 GB), so the default slab holds as many
// entries as the frame has faces (+25 % for clipped sub-triangles): a tile overflows only under that
// budget or an explicit small bin_capacity, and an overflowed tile's raster workgroup then filters every
// record of the frame itself (slow, exact).  The fine 16x16-tile binning happens inside the raster
// kernel, in LDS.
struct Layout {
    int ntx, nty, ntiles;     // fine tiles per frame
    int cshift, csize;        // coarse tile edge = 1 << cshift pixels
    int nctx, ncty, ncoarse;  // coarse tiles per frame (<= kMaxCoarse)
    int64_t nrec;
    size_t saved_recs, saved_fdata, saved_cov, saved_total;
    size_t off_count, off_flag, off_bins, scratch_total;
    int64_t bin_capacity;     // entries in all slabs
    uint32_t slab;            // entries per (frame, coarse tile) slab
};

constexpr int kMaxCoarse = 4096;   // LDS histogram size in setup
constexpr int kFacesPerThread = 1;
#ifndef DIRT_BIN_THREADS
#define DIRT_BIN_THREADS 256
#endif
constexpr int kBinThreads = DIRT_BIN_THREADS;
constexpr int kFacesPerBlock = kFacesPerThread * kBinThreads;
constexpr int64_t kDefaultBinBudget = 1ll << 27;  // entries (1 GiB) above which the default slab shrinks
// Count-set parity, so that no kernel has to return the counts it read to zero.  Words of the flag area
// (separate 64-B lines): [0] out-of-range-face flag, [kParP] P, [kParQ] Q.  The setup kernel reads p = Q,
// publishes P = p, accumulates into counts[p] and zeroes counts[p ^ 1] (read by the previous forward's
// raster, which has completed); the raster kernel bins from counts[0] + counts[1] (= counts[p], the
// other set being zero) and publishes Q = P ^ 1 for the next forward.  Each word is only read by one kernel and only written (one workgroup,
// one value) by the other, so no launch reads a word it writes.  Zeroed scratch = a valid state.
constexpr int kParP = 16, kParQ = 32;
// Words between two bin counters: the setup's reservation atomics execute at the memory side, and ~200
// workgroups reserving in the same few lines serialise there, so every counter gets a line of its own.
#ifndef DIRT_COUNT_STRIDE
#define DIRT_COUNT_STRIDE 64
#endif
constexpr int kCountStride = DIRT_COUNT_STRIDE;

int64_t default_capacity(int B, int F, int ncoarse)
{
    const int64_t slabs = (int64_t)B * ncoarse;
    int64_t per = (int64_t)F + F / 4 + 64;
    if (slabs * per > kDefaultBinBudget) per = std::max<int64_t>(kDefaultBinBudget / std::max<int64_t>(slabs, 1), 256);
    return slabs * per;
}

int make_layout(int B, int H, int W, int F, int64_t bin_capacity, Layout &L)
{
    L.ntx = (W + kTile - 1) / kTile;
    L.nty = (H + kTile - 1) / kTile;
    L.ntiles = L.ntx * L.nty;
#ifndef DIRT_COARSE_SHIFT
#define DIRT_COARSE_SHIFT 6  // coarse tile edge 64 px (grown until the frame has <= kMaxCoarse of them)
#endif
    for (L.cshift = DIRT_COARSE_SHIFT;; ++L.cshift) {
        L.csize = 1 << L.cshift;
        L.nctx = (W + L.csize - 1) >> L.cshift;
        L.ncty = (H + L.csize - 1) >> L.cshift;
        L.ncoarse = L.nctx * L.ncty;
        if (L.ncoarse <= kMaxCoarse) break;
    }
    L.nrec = (int64_t)(1 + kExtraPerFace) * F;
    const int64_t slabs = std::max<int64_t>((int64_t)B * L.ncoarse, 1);
    L.bin_capacity = bin_capacity > 0 ? bin_capacity : default_capacity(B, F, L.ncoarse);
    L.slab = (uint32_t)std::min<int64_t>(std::max<int64_t>(L.bin_capacity / slabs, 1), 0x7fffffffLL);
    L.bin_capacity = (int64_t)L.slab * slabs;
    L.saved_recs = 0;
    L.saved_fdata = (size_t)align_up((int64_t)B * L.nrec * (int64_t)sizeof(Rec), 256);
    L.saved_cov = L.saved_fdata + (size_t)align_up((int64_t)B * F * (int64_t)sizeof(FaceData), 256);
    L.saved_total = L.saved_cov + (size_t)align_up((int64_t)B * H * W, 256);  // 4 coverage bits per pixel
    const int64_t nc = (int64_t)B * L.ncoarse;
    size_t o = 0;
    L.off_count = o;  o += (size_t)align_up(2 * nc * 4 * kCountStride, 256);  // counts[2][B][ncoarse] (strided)
    L.off_flag = o;   o += 256;
    L.off_bins = o;   o += (size_t)align_up(L.bin_capacity * 8, 256);
    L.scratch_total = o;
    return DIRT_OK;
}

int validate(int B, int H, int W, int C, int V, int F)
{
    if (B < 0 || V < 0 || F < 0) return fail(DIRT_EINVAL, "Rasterise expects non-negative batch, vertex and face counts");
    if (H <= 0 || W <= 0 || H > DIRT_MAX_DIM || W > DIRT_MAX_DIM)
        return fail(DIRT_EINVAL, "Rasterise expects 0 < height, width <= 8192");
    if (C < 1 || C > DIRT_MAX_CHANNELS) return fail(DIRT_EINVAL, "Rasterise expects 1 <= channels <= 8");
    if (F > (1 << 26) || (int64_t)B * F > 0x0fffffffLL || (int64_t)B * V > 0x7fffffffLL)
        return fail(DIRT_EINVAL, "Rasterise batch too large (at most 2^26 faces per frame, 2^28 per batch)");
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

// bbox (pixels) packed as i0 | i1<<16 and j0 | j1<<16; empty when i0 > i1
__device__ __forceinline__ void coarse_range(uint32_t bx, uint32_t by, int cshift, int &cx0, int &cx1, int &cy0, int &cy1)
{
    cx0 = (int)(bx & 0xffff) >> cshift;
    cx1 = (int)(bx >> 16) >> cshift;
    cy0 = (int)(by & 0xffff) >> cshift;
    cy1 = (int)(by >> 16) >> cshift;
}

__device__ __forceinline__ void load_bbox(const Rec &r, uint32_t &bx, uint32_t &by)
{
    const uint2 q = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(&r) + 48);
    // Rec stores i0, i1, j0, j1 as consecutive uint16
    bx = q.x;
    by = q.y;
}

// Records that span many coarse tiles (large triangles) would serialise one thread over all their
// tiles; they are queued in LDS and their (record, coarse tile) pairs are spread over the whole
// workgroup instead.  Small records (<= kSmallPairs tiles) stay with their thread.
constexpr int kSmallPairs = 8;
constexpr int kBigCap = 64;
struct BigQueue {
    int32_t ri[kBigCap];
    uint32_t bx[kBigCap], by[kBigCap];
    int32_t cx0[kBigCap], cy0[kBigCap], w[kBigCap], start[kBigCap + 1];
    int32_t n;
};

// Call op(ri, bx, by, cx, cy) for every coarse tile of a record: inline when small or when the queue is
// full, else queue it for coarse_pairs_flush.
template <class Op>
__device__ __forceinline__ void coarse_pairs_add(BigQueue &Q, int32_t ri, uint32_t bx, uint32_t by, int cshift, Op op)
{
    if ((bx & 0xffff) > (bx >> 16)) return;
    int cx0, cx1, cy0, cy1;
    coarse_range(bx, by, cshift, cx0, cx1, cy0, cy1);
    const int w = cx1 - cx0 + 1, n = w * (cy1 - cy0 + 1);
    if (n > kSmallPairs) {
        const int q = atomicAdd(&Q.n, 1);
        if (q < kBigCap) {
            Q.ri[q] = ri; Q.bx[q] = bx; Q.by[q] = by; Q.cx0[q] = cx0; Q.cy0[q] = cy0; Q.w[q] = w;
            Q.start[q + 1] = n;
            return;
        }
    }
    for (int cy = cy0; cy <= cy1; ++cy)
        for (int cx = cx0; cx <= cx1; ++cx) op(ri, bx, by, cx, cy);
}

// Whole workgroup (converged): expand the queued records' pairs over all threads; resets the queue.
// Returns the number of queued records; an empty queue costs one barrier.
template <int NT, class Op>
__device__ __forceinline__ int coarse_pairs_flush(BigQueue &Q, Op op)
{
    __syncthreads();
    const int nq = min(Q.n, kBigCap);
    if (nq == 0) return 0;  // (uniform; Q.n is already 0)
    if (threadIdx.x == 0) {
        Q.start[0] = 0;
        for (int q = 0; q < nq; ++q) Q.start[q + 1] += Q.start[q];
    }
    __syncthreads();
    const int total = Q.start[nq];
    int q = 0;
    for (int k = threadIdx.x; k < total; k += NT) {
        while (Q.start[q + 1] <= k) ++q;  // k only grows: a forward walk over the (short) queue
        const int local = k - Q.start[q];
        const int cy = Q.cy0[q] + local / Q.w[q], cx = Q.cx0[q] + local % Q.w[q];
        op(Q.ri[q], Q.bx[q], Q.by[q], cx, cy);
    }
    __syncthreads();
    if (threadIdx.x == 0) Q.n = 0;
    __syncthreads();
    return nq;
}

// per-workgroup phase timestamps of the instrumented backward (AB & 128, dirt_debug_bwd_variant 128)
constexpr int kTsMaxWG = 1 << 16;
constexpr int kTsStride = 13;  // 8 phase timestamps, HW_ID, XCC_ID, 3 inside phase B (wave 0)
__device__ uint64_t g_phase_ts[kTsMaxWG * kTsStride];
#define PHASE_TS(n)                                                                                           \
    do {                                                                                                      \
        if ((AB & 128) && threadIdx.x == 0) {                                                                 \
            const int wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                              \
            if (wg_ < kTsMaxWG) {                                                                             \
                g_phase_ts[wg_ * kTsStride + (n)] = __builtin_amdgcn_s_memtime();                             \
                if ((n) == 0) {                                                                               \
                    g_phase_ts[wg_ * kTsStride + 8] = __builtin_amdgcn_s_getreg((4) | (31 << 11));            \
                    g_phase_ts[wg_ * kTsStride + 9] = __builtin_amdgcn_s_getreg((20) | (31 << 11));           \
                }                                                                                             \
            }                                                                                                 \
        }                                                                                                     \
    } while (0)

__device__ __forceinline__ uint32_t rel_bbox(uint32_t bx, uint32_t by, int cx, int cy, int cshift)
{
    const int lim = (1 << cshift) - 1;
    const int ox = cx << cshift, oy = cy << cshift;
    const int a0 = max((int)(bx & 0xffff) - ox, 0), a1 = min((int)(bx >> 16) - ox, lim);
    const int b0 = max((int)(by & 0xffff) - oy, 0), b1 = min((int)(by >> 16) - oy, lim);
    return (uint32_t)a0 | ((uint32_t)a1 << 8) | ((uint32_t)b0 << 16) | ((uint32_t)b1 << 24);
}

// Zero-fill of two float arrays by a range of workgroups (16-B stores where the buffer is 16-B aligned --
// torch allocations are -- else scalar)
struct ZeroFill {
    float *a, *b;
    int64_t na, nb;
    int nfb;  // workgroups before the fillers (blockIdx.x < nfb do the kernel's own work)
    __device__ void run(int64_t blk, int64_t nblk) const
    {
        const int64_t gt = blk * blockDim.x + threadIdx.x, gs = nblk * blockDim.x;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a) {
            const int64_t n4 = (reinterpret_cast<uintptr_t>(a) & 15) == 0 ? (na >> 2) : 0;
            for (int64_t k = gt; k < n4; k += gs) reinterpret_cast<float4 *>(a)[k] = z4;
            for (int64_t k = 4 * n4 + gt; k < na; k += gs) a[k] = 0.f;
        }
        if (b) {
            const int64_t n4 = (reinterpret_cast<uintptr_t>(b) & 15) == 0 ? (nb >> 2) : 0;
            for (int64_t k = gt; k < n4; k += gs) reinterpret_cast<float4 *>(b)[k] = z4;
            for (int64_t k = 4 * n4 + gt; k < nb; k += gs) b[k] = 0.f;
        }
    }
};

// K1: setup + coarse binning.  Bin entry = {record index, bbox clamped to the coarse tile, 8 bits per
// side}; order inside a slab is irrelevant (the depth resolve is a commutative min).
// AB & 128: per-workgroup phase timestamps (dirt_debug_setup_ts, tools/setup_ts.py)
template <int AB = 0>
__global__ __launch_bounds__(kBinThreads) void setup_kernel(const float *__restrict__ verts,
                                                            const int32_t *__restrict__ faces, int V, int F, int W,
                                                            int H, int cshift, int nctx, int ncoarse, int64_t nrec,
                                                            Rec *__restrict__ recs, FaceData *__restrict__ fdata,
                                                            uint32_t *__restrict__ counts, uint32_t *__restrict__ flag,
                                                            uint2 *__restrict__ bins, uint32_t slab, int B,
                                                            const ZeroFill zf)
{
    // workgroups past the faces zero-fill the caller's gradient accumulators (DIRT_FWD zero_grad_*): the
    // setup grid leaves most CUs idle (196 workgroups at config 3), so the fill costs the raster nothing
    if ((int)blockIdx.x >= zf.nfb) {
        zf.run((int64_t)blockIdx.y * (gridDim.x - zf.nfb) + (blockIdx.x - zf.nfb), (int64_t)(gridDim.x - zf.nfb) * gridDim.y);
        return;
    }
    __shared__ uint32_t hist[kMaxCoarse];
    __shared__ uint32_t base[kMaxCoarse];
    __shared__ BigQueue Q;
    const int b = blockIdx.y, t = threadIdx.x;
    PHASE_TS(0);
    const int64_t ncount = (int64_t)B * ncoarse;
    const uint32_t par = flag[kParQ] & 1u;
    uint32_t *ccount = counts + par * ncount * kCountStride;
    {
        // publish this forward's parity for the raster; zero the other count set for the next forward
        const int64_t g = (int64_t)blockIdx.y * zf.nfb + blockIdx.x, ng = (int64_t)zf.nfb * gridDim.y;  // face workgroups
        if (g == 0 && t == 0) flag[kParP] = par;
        uint32_t *other = counts + (par ^ 1u) * ncount * kCountStride;
        for (int64_t k = g * kBinThreads + t; k < ncount; k += ng * kBinThreads) other[k * kCountStride] = 0;
    }
    for (int c = t; c < ncoarse; c += kBinThreads) hist[c] = 0;
    if (t == 0) Q.n = 0;
    __syncthreads();
    auto count = [&](int32_t, uint32_t, uint32_t, int cx, int cy) { atomicAdd(&hist[cy * nctx + cx], 1u); };
    Rec *frame_recs = recs + (int64_t)b * nrec;
    const float *vb = verts + (int64_t)b * V * 4;
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    const int f = blockIdx.x * kFacesPerBlock + t;
    // what the placement pass needs again: the fast-path record's packed bbox, or the sub-record count
    int nsub = 0;
    bool fast = false;
    uint32_t fbx = 1, fby = 0;
    if (f < F) {
        const int64_t gid = (int64_t)b * F + f;
        const int32_t i0 = faces[gid * 3], i1 = faces[gid * 3 + 1], i2 = faces[gid * 3 + 2];
        const int32_t vidx[3] = {i0, i1, i2};
        PHASE_TS(10 + (i0 == 0x7fffffff));
        Tri tri;
        bool ok = true;
        // the three vertex loads are issued together (clamped indices, no per-vertex branch: one
        // memory round trip instead of three); out-of-range vertices are replaced afterwards
        float4 pv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int32_t vi = vidx[k];
            const bool in = vi >= 0 && vi < V;
            pv[k] = V > 0 ? *reinterpret_cast<const float4 *>(vb + (int64_t)(in ? vi : 0) * 4) : make_float4(0.f, 0.f, 0.f, 1.f);
            if (!in) pv[k] = make_float4(0.f, 0.f, 0.f, 1.f);
            ok = ok && in;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            tri.v[k][0] = pv[k].x; tri.v[k][1] = pv[k].y; tri.v[k][2] = pv[k].z; tri.v[k][3] = pv[k].w;
            ok = ok && finite4(tri.v[k]);
        }
        PHASE_TS(11 + (tri.v[0][0] == 12345.f));
        if (!(i0 >= 0 && i0 < V && i1 >= 0 && i1 < V && i2 >= 0 && i2 < V)) atomicOr(flag, 1u);
        FaceData fd;
        fd.v[0] = i0; fd.v[1] = i1; fd.v[2] = i2;
        fd.w[0] = tri.v[0][3]; fd.w[1] = tri.v[1][3]; fd.w[2] = tri.v[2][3];
        fd.clipped = 0;
        Rec r;
        set_empty(r, f);
        fast = ok;
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
            fbx = (uint32_t)r.i0 | ((uint32_t)r.i1 << 16);
            fby = (uint32_t)r.j0 | ((uint32_t)r.j1 << 16);
            coarse_pairs_add(Q, f, fbx, fby, cshift, count);
        } else {
            frame_recs[f] = r;  // empty unless clip_face overwrites it
#ifndef DIRT_SETUP_NO_CLIP
            if (ok) {
                nsub = clip_face(tri, W, H, F, f, frame_recs);
                fd.clipped = 1;
            }
#endif
            for (int s = 0; s < nsub; ++s) {
                uint32_t bx, by;
                const int64_t ri = rec_index(F, f, s);
                load_bbox(frame_recs[ri], bx, by);
                coarse_pairs_add(Q, (int32_t)ri, bx, by, cshift, count);
            }
        }
        fd.nsub = nsub;
        fdata[gid] = fd;
    }
    PHASE_TS(1);
    // (the placement pass queues the same records again: with none queued here, it needs no flush)
    const int nbig = coarse_pairs_flush<kBinThreads>(Q, count);
    PHASE_TS(2);
    // reserve this workgroup's range of every touched slab: one returning device atomic per (workgroup,
    // coarse tile), all in flight together
    uint32_t *cc = ccount + (int64_t)b * ncoarse * kCountStride;
    for (int c = t; c < ncoarse; c += kBinThreads) {
        const uint32_t n = hist[c];
        base[c] = (AB & 1) ? 0u : n ? atomicAdd(&cc[c * kCountStride], n) : 0u;  // (AB & 1: ablation, no reservation)
        hist[c] = 0;
    }
    __syncthreads();
    PHASE_TS(3);
    uint2 *fb = bins + (int64_t)b * ncoarse * slab;
    auto place = [&](int32_t ri, uint32_t bx, uint32_t by, int cx, int cy) {
        const int c = cy * nctx + cx;
        const uint32_t pos = base[c] + atomicAdd(&hist[c], 1u);
        if (pos < slab) fb[(int64_t)c * slab + pos] = make_uint2((uint32_t)ri, rel_bbox(bx, by, cx, cy, cshift));
    };
    if (fast) {
        coarse_pairs_add(Q, f, fbx, fby, cshift, place);
    } else {
        for (int s = 0; s < nsub; ++s) {
            uint32_t bx, by;
            const int64_t ri = rec_index(F, f, s);
            load_bbox(frame_recs[ri], bx, by);
            coarse_pairs_add(Q, (int32_t)ri, bx, by, cshift, place);
        }
    }
    if (nbig > 0) coarse_pairs_flush<kBinThreads>(Q, place);
    if (AB & 128) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        PHASE_TS(7);
    }
}

__device__ __forceinline__ void wave_lds_sync()
{
    // LDS ops of one wave execute in order; this only stops the compiler from reordering across it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// launch the setup (and binning) of B frames x F faces
template <int AB = 0>
void launch_setup(const float *vertices, const int32_t *faces, int B, int H, int W, int V, int F, const Layout &L,
                  Rec *recs, FaceData *fdata, uint32_t *ccount, uint32_t *flag, uint2 *bins, hipStream_t stream,
                  float *zero_a = nullptr, int64_t nzero_a = 0, float *zero_b = nullptr, int64_t nzero_b = 0)
{
    ZeroFill zf{zero_a, zero_b, zero_a ? nzero_a : 0, zero_b ? nzero_b : 0, (F + kFacesPerBlock - 1) / kFacesPerBlock};
    // filler workgroups per frame row: ~16 float4 stores per thread, at most 64 in all
    const int64_t z4 = (zf.na + zf.nb) / 4, want = std::min<int64_t>((z4 + 4095) / 4096, 64);
    const int nzb = z4 > 0 ? (int)std::max<int64_t>(1, (want + B - 1) / B) : 0;
    const dim3 grid((unsigned)(zf.nfb + nzb), (unsigned)B);
    setup_kernel<AB><<<grid, dim3(kBinThreads), 0, stream>>>(vertices, faces, V, F, W, H, L.cshift, L.nctx, L.ncoarse,
                                                             L.nrec, recs, fdata, ccount, flag, bins, L.slab, B, zf);
}

// ------------------------------------------------------------------------------------------------
// K4: tile raster + resolve
//
// One workgroup per 16x16 tile; each of its 4 waves owns an 8x8 block of it:
//   a. the workgroup filters its coarse slab once (a quarter of every 512-entry chunk per wave) by the
//      packed bbox against the tile, compacting survivors into per-wave LDS segments (ballot);
//   b. the survivors are staged once, an entry per thread: int64 edge functions at the tile origin with
//      the top-left bias folded in (E + owned > 0 <=> inside), pinned to 2^30 where an edge holds over
//      the whole tile, else exact int32; packed i16 (A, B); the depth plane; the exact mask of the
//      blocks the record can cover;
//   c. each wave walks the entries of its block: three v_dot2_i32_i16 edge steps (exact for records with
//      |A|, |B| < 2^15; larger ones use per-lane int64, flagged), two FMAs of depth and a branch-free
//      min of the 64-bit (depth24 << 32 | face << 3 | s) key.
// Results are bit-identical to R3/R4 (oracle) by construction.

constexpr int kStrips = 4;
// The pixels a wave owns inside its 16x16 tile: an 8x8 block (DIRT_RASTER_STRIPS=0, default) or a 16x4
// strip.  A block is the more compact shape: fewer triangles overlap it (Steiner: the overlap area of a
// region and a triangle grows with the region's perimeter, 32 vs 40 px), so fewer entries per wave.
#ifndef DIRT_RASTER_STRIPS
#define DIRT_RASTER_STRIPS 0
#endif
constexpr int kWaveW = DIRT_RASTER_STRIPS ? 16 : 8, kWaveH = DIRT_RASTER_STRIPS ? 4 : 8;
__host__ __device__ constexpr int wave_ox(int w) { return DIRT_RASTER_STRIPS ? 0 : 8 * (w & 1); }
__host__ __device__ constexpr int wave_oy(int w) { return DIRT_RASTER_STRIPS ? 4 * w : 8 * (w >> 1); }
// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8 shares an L2),
// so give each residue class a contiguous band of tiles; neighbouring tiles then share halo pixels and
// records in one L2.  A bijection on [0, n); speed only, never correctness.
__device__ __forceinline__ int xcd_tile(int x, int n)
{
    const int q = n >> 3, r = n & 7, g = x & 7, k = x >> 3;
    return g * q + min(g, r) + k;
}

// Tiles per row with a host-computed reciprocal: tile / ntx = umulhi(tile, ceil(2^32 / ntx)), exact for
// tile < 2^18 and ntx <= 2^9 (the error term tile * (m - 2^32/ntx) / 2^32 < 2^-14 never reaches the next
// integer) -- two scalar instructions instead of a ~25-instruction division in every wave's prologue.
struct TileGrid {
    int ntx;
    uint32_t inv;
    __device__ __forceinline__ void split(int tile, int &tx, int &ty) const
    {
        ty = (int)__umulhi((uint32_t)tile, inv);
        tx = tile - ty * ntx;
    }
};
static_assert((DIRT_MAX_DIM / kTile) <= 512 && (DIRT_MAX_DIM / kTile) * (DIRT_MAX_DIM / kTile) <= (1 << 18),
              "TileGrid reciprocal range");
inline TileGrid tile_grid(int ntx) { return TileGrid{ntx, (uint32_t)(((1ull << 32) + (uint64_t)ntx - 1) / (uint64_t)ntx)}; }

#ifndef DIRT_RASTER_LISTS
#define DIRT_RASTER_LISTS 1  // per-wave entry lists (1) or the scalar bit-mask walk (0)
#endif
// Hierarchical depth culling (depth-tested programs): a wave whose list holds at least DIRT_RASTER_HZ_MIN
// entries walks it in groups of 16 and skips every entry whose depth lower bound over the tile exceeds
// the farthest depth its 64 pixels already hold -- such an entry can win no pixel.  Pays where depth
// complexity is high (large overlapping triangles); short lists keep the plain loop.
#ifndef DIRT_RASTER_HZ
#define DIRT_RASTER_HZ 1
#endif
#ifndef DIRT_RASTER_HZ_MIN
#define DIRT_RASTER_HZ_MIN 32
#endif
constexpr int kWaveList = 256 + 2;  // a staging round's entries + the even pad
constexpr int kFilterBlock = 128;  // coarse-bin entries filtered per wave and chunk (2 loads per lane in flight)
// A staged record is "small" when every |A|, |B| < 2^15: its edge steps inside a strip are one
// v_dot2_i32_i16 of the packed (A, B) with the lane's packed (dx, dy) offsets (<= 15*256, 3*256).
constexpr int kDotEdge = 1 << 15;
constexpr uint32_t kLargeAB = 0x80008000u;  // ab[0] of a large entry (A = B = -2^15 never occurs in a small one)

struct alignas(16) StripEntry {  // 48 B of wave-private LDS per staged (sub-)triangle: three ds_read_b128
    int32_t e[3];    // small: E + owned at the strip origin (2^30 when the edge holds over the whole strip);
                     // large: e[0] = record index
    uint32_t ab[3];  // small: (uint16)A | B << 16; large: ab[0] = kLargeAB
    float za, zb, fx0, fy0;  // fx0, fy0 8-byte aligned: one register pair for v_pk_add_f32
    uint32_t key;    // face << 3 | sub-triangle: the low word of the depth key (the lower face wins ties);
                     // an even register once loaded, so the quantised depth lands beside it (no move)
    float z0;
};
static_assert(sizeof(StripEntry) == 48, "StripEntry must be 48 B");

typedef short short2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));

// low word of the depth key of record ri: face << 3 | sub-triangle index (rec_index inverse)
__device__ __forceinline__ uint32_t rec_key(int32_t ri, int F)
{
    if (ri < F) return (uint32_t)ri << 3;
    const int32_t d = ri - F, f = d / kExtraPerFace;
    return ((uint32_t)f << 3) | (uint32_t)(d - f * kExtraPerFace + 1);
}
__device__ __forceinline__ int32_t key_rec(uint32_t key, int F) { return (int32_t)rec_index(F, (int)(key >> 3), (int)(key & 7)); }

// R4 key: (q24 << 32 | face << 3 | s), minimum wins -- GL LESS with draw order = face index
// (rasterise_egl.cpp:451-457).  NoDepth (hill.cpp:194, GL_DEPTH_TEST off): the last face in draw order
// wins, near/far clipping stays.  The initial value rejects q >= 2^24-1 (cleared depth 1.0) by itself.
template <bool NoDepth>
__device__ __forceinline__ uint64_t depth_key(uint32_t q, uint32_t key)
{
    return NoDepth ? (uint64_t)(0xffffffffu - key) : (((uint64_t)q << 32) | key);
}
template <bool NoDepth>
constexpr uint64_t kKeyInit = NoDepth ? ~0ull : ((uint64_t)kDepthMax << 32);
template <bool NoDepth>
__device__ __forceinline__ uint32_t key_low(uint64_t best) { return NoDepth ? 0xffffffffu - (uint32_t)best : (uint32_t)best; }

// overflow / large-record path: one record against this lane's pixel (R3 + R4)
template <bool NoDepth>
__device__ __forceinline__ void depth_update(const Rec &r, uint32_t key, float fxl, float fyl, bool in, uint64_t &best)
{
    const float zw = depth_at(r.za, r.zb, r.z0, fxl - r.fx0, fyl - r.fy0);
    const float zc = __builtin_amdgcn_fmed3f(zw, 0.0f, 1.0f);
    const uint64_t k = depth_key<NoDepth>(depth_q24(zc), key);
    const bool win = in && zc == zw && k < best;
    best = win ? k : best;
}

// stage_tile's block mask of a large record (some |A|, |B| >= 2^15) in int64, out of line (rare)
__device__ __noinline__ uint32_t large_block_mask(const Rec *rp, int32_t px0, int32_t py0, uint32_t mask)
{
    const RasterPart R = *reinterpret_cast<const RasterPart *>(rp);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t owned = (R.A[k] > 0 || (R.A[k] == 0 && R.B[k] < 0)) ? 1 : 0;
        const int64_t e0 = (int64_t)R.A[k] * (int64_t)px0 + ((int64_t)R.B[k] * (int64_t)py0 + R.C[k]) + owned;
        const int64_t a = (int64_t)R.A[k] * 256, bb = (int64_t)R.B[k] * 256;
        // over a wave's rectangle [ox, ox + kWaveW) x [oy, oy + kWaveH): max of E at its origin + the
        // positive parts of the steps across it
        const int64_t wx = a * (kWaveW - 1), wy = bb * (kWaveH - 1);
        const int64_t wmax = (wx > 0 ? wx : 0) + (wy > 0 ? wy : 0);
#pragma unroll
        for (int st = 0; st < kStrips; ++st)
            if (e0 + a * wave_ox(st) + bb * wave_oy(st) + wmax <= 0) mask &= ~(1u << st);
    }
    return mask;
}

// Stage one tile survivor (record ri) for the 16x16 tile at pixel (ti0, tj0): edge values at the tile
// origin (E + owned, exact int32, pinned to 2^30 where the edge holds over the whole tile), the packed
// (A, B) steps, depth plane and key.  Returns the mask of the tile's four wave rectangles (8x8 blocks) the
// record can cover (its bbox overlaps the block and no edge excludes the whole block; exact int64 tests) and sets
// `large` when the record needs the per-lane int64 path (some |A|, |B| >= 2^15).
__device__ __forceinline__ uint32_t stage_tile(const Rec *__restrict__ frame_recs, int32_t ri, int ti0, int tj0, int F,
                                               StripEntry &E, bool &large)
{
    const RasterPart R = *reinterpret_cast<const RasterPart *>(&frame_recs[ri]);
    bool small = true;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        small = small && R.A[k] > -kDotEdge && R.A[k] < kDotEdge && R.B[k] > -kDotEdge && R.B[k] < kDotEdge;
    uint32_t mask = 0;
#pragma unroll
    for (int st = 0; st < kStrips; ++st) {
        const int x0 = ti0 + wave_ox(st), y0 = tj0 + wave_oy(st);
        if ((int)R.i0 <= x0 + kWaveW - 1 && (int)R.i1 >= x0 && (int)R.j0 <= y0 + kWaveH - 1 && (int)R.j1 >= y0)
            mask |= 1u << st;
    }
    const int32_t px0 = ti0 * 256 + 128, py0 = tj0 * 256 + 128;
    // E at the tile origin in int64, clamped to +-2^30; for a small record (|A|, |B| < 2^15: steps
    // across the tile < 2^23) that keeps every block decision and the pinning exact, so the rest is
    // int32.  A large record's block mask is redone in int64 out of line (rare).
    const uint32_t bbox_mask = mask;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int32_t owned = (R.A[k] > 0 || (R.A[k] == 0 && R.B[k] < 0)) ? 1 : 0;
        const int64_t e64 = (int64_t)R.A[k] * (int64_t)px0 + ((int64_t)R.B[k] * (int64_t)py0 + R.C[k]) + owned;
        const int32_t e0 = e64 > (1 << 30) ? (1 << 30) : e64 < -(1 << 30) ? -(1 << 30) : (int32_t)e64;
        // (wrapping uint32 arithmetic: a large record's values may wrap here -- its mask is redone below
        // and its edge values are unused -- a small record's never do)
        const uint32_t a = (uint32_t)R.A[k] << 8, bb = (uint32_t)R.B[k] << 8;
        const int32_t wx = (int32_t)(a * (kWaveW - 1)), wy = (int32_t)(bb * (kWaveH - 1));
        const uint32_t wmax = (uint32_t)(wx > 0 ? wx : 0) + (uint32_t)(wy > 0 ? wy : 0);
#pragma unroll
        for (int st = 0; st < kStrips; ++st)
            if ((int32_t)((uint32_t)e0 + a * wave_ox(st) + bb * wave_oy(st) + wmax) <= 0) mask &= ~(1u << st);
        const int32_t tx = (int32_t)(a * (kTile - 1)), ty = (int32_t)(bb * (kTile - 1));
        E.e[k] = (int32_t)((uint32_t)e0 + (uint32_t)(tx < 0 ? tx : 0) + (uint32_t)(ty < 0 ? ty : 0)) > 0 ? (1 << 30) : e0;
        E.ab[k] = ((uint32_t)R.A[k] & 0xffffu) | ((uint32_t)R.B[k] << 16);
    }
    if (__builtin_amdgcn_ballot_w64(!small) != 0 && !small) mask = large_block_mask(&frame_recs[ri], px0, py0, bbox_mask);
    if (!small) {
        E.e[0] = ri;
        E.ab[0] = kLargeAB;
    }
    E.za = R.za; E.zb = R.zb; E.z0 = R.z0; E.fx0 = R.fx0; E.fy0 = R.fy0;
    E.key = rec_key(ri, F);
    large = !small;
    return mask;
}

// R3 + R4 of staged entries (LDS, three 16-B broadcast reads each) against this lane's pixel
typedef __attribute__((address_space(3))) const volatile int4v lds_int4v;
struct EntryRegs {
    int4v q0, q1, q2;
};
// volatile + LDS address space: keeps the reads whole ds_read_b128s (4 LDS cycles each)
__device__ __forceinline__ EntryRegs load_entry(const StripEntry *ent, int e)
{
    lds_int4v *ve = (lds_int4v *)(ent) + 3 * e;
    return EntryRegs{ve[0], ve[1], ve[2]};
}

// the same at a byte offset into the staging array (a per-wave list element)
__device__ __forceinline__ EntryRegs load_entry_at(const StripEntry *ent, uint32_t off)
{
    lds_int4v *ve = (lds_int4v *)((const char *)ent + off);
    return EntryRegs{ve[0], ve[1], ve[2]};
}

// rank of this lane among the set lanes of `mask` below it
__device__ __forceinline__ int lane_rank(uint64_t mask)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// maximum of v over the wave, wave-uniform: row_shr 1/2/4/8 leave each 16-lane row's maximum in its
// last lane, four readlanes combine the rows (lanes shifted in from outside a row keep their own value)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));
    const uint32_t a = __builtin_amdgcn_readlane(v, 15), b = __builtin_amdgcn_readlane(v, 31);
    const uint32_t c = __builtin_amdgcn_readlane(v, 47), d = __builtin_amdgcn_readlane(v, 63);
    return max(max(a, b), max(c, d));
}

#if DIRT_RASTER_HZ
// Conservative lower bound of the quantised depth a staged small entry can reach in the wave's pixel
// rectangle at (x0, y0): the plane's minimum over the rectangle is at the corner its slopes point away
// from; every zw the raster computes is within 2^-23 (|za||dx| + |zb||dy| + |z0|) of the exact plane
// (two roundings), so twice that margin, and two more quanta, keep the bound below every key the
// entry can produce there.  NaN planes give 0 (never culled).
__device__ __forceinline__ uint32_t entry_qmin(const StripEntry *ent, uint32_t off, int x0, int y0)
{
    lds_int4v *ve = (lds_int4v *)((const char *)ent + off);
    const int4v q1 = ve[1], q2 = ve[2];
    const float za = __int_as_float(q1.z), zb = __int_as_float(q1.w), z0 = __int_as_float(q2.w);
    const float xa = (float)x0 + 0.5f - __int_as_float(q2.x), xb = (float)(x0 + kWaveW - 1) + 0.5f - __int_as_float(q2.x);
    const float ya = (float)y0 + 0.5f - __int_as_float(q2.y), yb = (float)(y0 + kWaveH - 1) + 0.5f - __int_as_float(q2.y);
    const float zc = depth_at(za, zb, z0, za > 0.0f ? xa : xb, zb > 0.0f ? ya : yb);
    const float s = fabsf(za) * fmaxf(fabsf(xa), fabsf(xb)) + fabsf(zb) * fmaxf(fabsf(ya), fabsf(yb)) + fabsf(z0);
    const float zq = __builtin_fmaf(__builtin_fmaf(-s, 0x1p-21f, zc), 16777215.0f, -2.0f);
    return zq > 0.0f ? (uint32_t)fminf(zq, 16777215.0f) : 0u;
}
#endif

template <bool NoDepth, bool Large>
__device__ __forceinline__ void raster_entry(const EntryRegs &q, const Rec *__restrict__ frame_recs, short2v pix,
                                             float2v pxy, int i, int j, uint64_t &best)
{
    bool in;
    if (!Large) {
        // R3 on tile-relative exact int32 values: E + owned > 0 for all three edges
        // (scalars first: clang's __builtin_bit_cast of an ext_vector component reads component 0)
        const int ab0 = q.q0.w, ab1 = q.q1.x, ab2 = q.q1.y;
        const int e0 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, ab0), pix, q.q0.x, false);
        const int e1 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, ab1), pix, q.q0.y, false);
        const int e2 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, ab2), pix, q.q0.z, false);
        in = min(e0, min(e1, e2)) > 0;
    } else {
        const Rec &r = frame_recs[__builtin_amdgcn_readfirstlane(q.q0.x)];
        int64_t E[3];
        edge_values(r, i, j, E);
        in = inside(r, E);
    }
    const float2v d = pxy - float2v{__int_as_float(q.q2.x), __int_as_float(q.q2.y)};
    const float zw = depth_at(__int_as_float(q.q1.z), __int_as_float(q.q1.w), __int_as_float(q.q2.w), d.x, d.y);
    if constexpr (NoDepth) {
        // R4 range test without branches: in range iff the clamp leaves zw unchanged (false for NaN)
        const float zc = __builtin_amdgcn_fmed3f(zw, 0.0f, 1.0f);
        const uint64_t k = depth_key<NoDepth>(depth_q24(zc), (uint32_t)q.q2.z);
        const bool win = in && zc == zw && k < best;
        best = win ? k : best;
    } else {
        // R4 with the far test folded into the key: zw >= 1 quantises to q >= 2^24-1 (v_cvt_u32 saturates),
        // a key that never beats the initial one (cleared depth), so only zw >= 0 needs a test (false for
        // NaN).  Inside [0, 1] q is depth_q24(zw): the same keys as the clamped form, one VALU less.
        uint32_t qd;
        asm("v_cvt_u32_f32 %0, %1" : "=v"(qd) : "v"(__builtin_fmaf(zw, 16777215.0f, 0.5f)));
        const uint64_t k = ((uint64_t)qd << 32) | (uint32_t)q.q2.z;
        const bool win = in && zw >= 0.0f && k < best;
        best = win ? k : best;
    }
}

__device__ __noinline__ bool covers_face_multi(int64_t hint_ri, const Rec *frame_recs, const FaceData *fdata_frame,
                                               int F, int f, int i, int j);

// correctly rounded int64 -> float of three values, out of line (rare: |E| >= 2^31)
__device__ __noinline__ float3 i64x3_to_f32(int64_t a, int64_t b, int64_t c)
{
    return make_float3((float)a, (float)b, (float)c);
}

// neighbour_coverage() without the int32 shortcut: int64 edge values, out of line (rare)
__device__ __noinline__ uint32_t neighbour_bits_i64(const EdgePart &r, int64_t E0, int64_t E1, int64_t E2)
{
    const int64_t E[3] = {E0, E1, E2};
    uint32_t bits = 0;
#pragma unroll
    for (int dir = 0; dir < 4; ++dir) {
        const int axis = dir >> 1, sg = (dir & 1) ? -1 : 1;
        int64_t Eq[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) Eq[k] = E[k] + (int64_t)(axis == 0 ? r.A[k] : r.B[k]) * (256 * sg);
        bits |= (inside(r, Eq) ? 1u : 0u) << dir;
    }
    return bits;
}

// Bit d of the result: the face visible at pixel (i, j) (record r, E = its edge values there) also
// covers the neighbour in direction d (0 right, 1 left, 2 up, 3 down; window coordinates) -- exactly
// the coverage tests of the backward's pairs, computed once here for every pixel, so the
// backward reads them (its own face at p: bit d of p; the neighbour's face at p: bit opposite(d) of q)
// instead of re-testing records per pair.
__device__ __forceinline__ uint32_t neighbour_coverage(const Rec &r, const int64_t E[3], bool multi, int32_t ri,
                                                       const Rec *frame_recs, const FaceData *fdata_frame, int F, int f,
                                                       int i, int j)
{
    // int32 when every lane's |E| < 2^30 and |A|, |B| < 2^22 (a one-pixel step stays inside int32);
    // otherwise the out-of-line int64 version (a real branch, not both paths)
    bool small = true;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        small = small && (uint64_t)(E[k] + (1ll << 30)) < (2ull << 30) && (uint32_t)(r.A[k] + (1 << 22)) < (2u << 22) &&
                (uint32_t)(r.B[k] + (1 << 22)) < (2u << 22);
    uint32_t bits = 0;
    if (__builtin_amdgcn_ballot_w64(!small) == 0) {
        int32_t eo[3];  // E + owned
#pragma unroll
        for (int k = 0; k < 3; ++k) eo[k] = (int32_t)E[k] + ((r.A[k] > 0 || (r.A[k] == 0 && r.B[k] < 0)) ? 1 : 0);
#pragma unroll
        for (int dir = 0; dir < 4; ++dir) {
            const int axis = dir >> 1, sg = (dir & 1) ? -256 : 256;
            const int32_t q0 = eo[0] + (axis == 0 ? r.A[0] : r.B[0]) * sg;
            const int32_t q1 = eo[1] + (axis == 0 ? r.A[1] : r.B[1]) * sg;
            const int32_t q2 = eo[2] + (axis == 0 ? r.A[2] : r.B[2]) * sg;
            bits |= (min(q0, min(q1, q2)) > 0 ? 1u : 0u) << dir;
        }
    } else {
        bits = neighbour_bits_i64(*reinterpret_cast<const EdgePart *>(&r), E[0], E[1], E[2]);
    }
    if (multi) {
#pragma unroll
        for (int dir = 0; dir < 4; ++dir) {
            const int axis = dir >> 1, sg = (dir & 1) ? -1 : 1;
            if (!((bits >> dir) & 1u) &&
                covers_face_multi(ri, frame_recs, fdata_frame, F, f, i + (axis == 0 ? sg : 0), j + (axis == 1 ? sg : 0)))
                bits |= 1u << dir;
        }
    }
    return bits;
}

// AB: ablation mask for tools/ablate.py (0 in the product): 1 skip the per-pixel loop, 2 skip
// staging + loop (bin filter only), 4 skip the resolve (g-buffer only), 8 skip the bin filter too,
// 32 no neighbour-coverage bits, 64 no colour loads (lambda written), 128 phase timestamps
#ifndef DIRT_RASTER_WAVES
#define DIRT_RASTER_WAVES 7  // min waves per SIMD the register allocation must allow (Gouraud, C = 1 or 3;
                             // the procedural programs and the generic-C path keep their natural allocation)
#endif
template <int CC, int AB = 0, int SH = DIRT_SHADER_GOURAUD>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256), amdgpu_waves_per_eu(SH == DIRT_SHADER_GOURAUD && CC > 0 ? DIRT_RASTER_WAVES : 1))) void raster_kernel(const float *__restrict__ background, const float *__restrict__ colors,
                                                     const Rec *__restrict__ recs, const FaceData *__restrict__ fdata,
                                                     const uint32_t *__restrict__ counts, uint32_t *__restrict__ flag,
                                                     const uint2 *__restrict__ bins, uint32_t slab,
                                                     int B, int H, int W, int Cdyn, int V, int F, TileGrid tg, int cshift,
                                                     int nctx, int ncoarse, int64_t nrec, float *__restrict__ pixels,
                                                     int32_t *__restrict__ gbuffer, uint8_t *__restrict__ covbits,
                                                     float *__restrict__ zero_a,
                                                     int64_t nzero_a, float *__restrict__ zero_b, int64_t nzero_b,
                                                     const float *__restrict__ verts, const float *__restrict__ cam,
                                                     int sid, int tcb)
{
    constexpr bool kNoDepth = SH == DIRT_SHADER_HILL;
#if defined(DIRT_RASTER_LDS_PAD) && DIRT_RASTER_LDS_PAD > 0
    __shared__ volatile char occupancy_probe[DIRT_RASTER_LDS_PAD];  // experiment: caps workgroups per CU
    if (threadIdx.x == 1023) occupancy_probe[0] = 0;
#endif
    PHASE_TS(0);
    constexpr int CM = CC > 0 ? CC : DIRT_MAX_CHANNELS;
    const int C = CC > 0 ? CC : Cdyn;
    __shared__ int32_t t_list[kStrips][kFilterBlock];  // per-wave segments of the tile's survivors
    __shared__ int32_t t_nw[2][kStrips];                // segment lengths, double-buffered by chunk parity
    __shared__ StripEntry t_ent[257];                   // one staging round: an entry per thread (+ sentinel)
    __shared__ uint8_t t_mask[256];                     // strips the entry can cover; bit 4: large
#if DIRT_RASTER_LISTS
    // per-wave entry lists of a staging round: byte offsets into t_ent of the small entries from the
    // front (padded to even with the sentinel), indices of the large ones from the back
    __shared__ uint32_t t_wl[kStrips][kWaveList];
    if (threadIdx.x == 0) {
        // sentinel t_ent[256]: ab = 0 so every edge value stays -2^30 (never covers)
        int4 *d = reinterpret_cast<int4 *>(&t_ent[256]);
        d[0] = make_int4(-(1 << 30), -(1 << 30), -(1 << 30), 0);
        d[1] = make_int4(0, 0, 0, 0);
        d[2] = make_int4(0, 0, 0, 0);
    }
#endif
    // Gouraud: XCD bands (L2 sharing of bins / records between neighbouring tiles); a procedural
    // program is compute-bound and its cost follows the image content (sky vs water), so its tiles are
    // interleaved over the XCDs instead (round-robin dispatch order) for balance
    const int tile = SH == DIRT_SHADER_GOURAUD ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x, b = blockIdx.y;
    int tx, ty;
    tg.split(tile, tx, ty);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int lx = wave_ox(wave) + lane % kWaveW, ly = wave_oy(wave) + lane / kWaveW;
    const int i = tx * kTile + lx, j = ty * kTile + ly;
    const int dx = lx * 256, dy = ly * 256;  // offset from the tile origin (sub-pixels)
    const float fxl = (float)i + 0.5f, fyl = (float)j + 0.5f;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const bool in_frame = i < W && j < H;
    const int64_t o = ((int64_t)b * H + (H - 1 - j)) * W + i;


    uint64_t best = kKeyInit<kNoDepth>;
    const short2v pix = {(short)dx, (short)dy};  // lane offset from the tile origin in sub-pixels
    const float2v pxy = {fxl, fyl};
    const int ti0 = tx * kTile, tj0 = ty * kTile;
    const int cx = ti0 >> cshift, cy = tj0 >> cshift;
    const int c = cy * nctx + cx;
    const int64_t cc = (int64_t)b * ncoarse + c;
    // The parity word, both count sets and the first chunk of the slab are loaded together (one memory
    // round trip instead of three dependent ones): slab entries are loaded before the count is known,
    // unconditionally (index clamped to the slab), and those past the count are masked afterwards.
    const uint2 *slab_bins = bins + cc * slab;
    constexpr int U = kFilterBlock / 64;
    uint2 ev[U];
    auto load_chunk = [&](uint32_t chunk) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = chunk + wave * kFilterBlock + u * 64 + lane;
            ev[u] = slab_bins[min(idx, slab - 1u)];
        }
    };
    if (slab > 0 && !(AB & 8)) load_chunk(0);
    // This forward's setup zeroed the other count set, so the count is the sum of both (no dependent
    // parity load); F == 0: setup did not run
    const uint32_t raw = F > 0 ? counts[cc * kCountStride] + counts[((int64_t)B * ncoarse + cc) * kCountStride] : 0u;
    if (blockIdx.x == 0 && blockIdx.y == 0 && t == 0 && !(AB & 16)) flag[kParQ] = (flag[kParP] & 1u) ^ 1u;
    if (!(AB & 16)) {
        // housekeeping spread over all blocks (a few KB each): zero-fill the caller's gradient
        // accumulators if it passed them (after the slab loads are in flight)
        const int64_t nblk = (int64_t)gridDim.x * gridDim.y;
        const int64_t gt = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x, gs = nblk * 256;
        // (16-B stores where the caller's buffer is 16-B aligned -- torch allocations are -- else scalar)
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (zero_a) {
            const int64_t n4 = (reinterpret_cast<uintptr_t>(zero_a) & 15) == 0 ? (nzero_a >> 2) : 0;
            for (int64_t k = gt; k < n4; k += gs) reinterpret_cast<float4 *>(zero_a)[k] = z4;
            for (int64_t k = 4 * n4 + gt; k < nzero_a; k += gs) zero_a[k] = 0.f;
        }
        if (zero_b) {
            const int64_t n4 = (reinterpret_cast<uintptr_t>(zero_b) & 15) == 0 ? (nzero_b >> 2) : 0;
            for (int64_t k = gt; k < n4; k += gs) reinterpret_cast<float4 *>(zero_b)[k] = z4;
            for (int64_t k = 4 * n4 + gt; k < nzero_b; k += gs) zero_b[k] = 0.f;
        }
    }
    // an overflowed slab (more pairs than its capacity): filter every record of the frame instead
    const bool overflow = raw > slab;
    const uint32_t n_items = overflow ? (uint32_t)nrec : raw;
    const FaceData *fdata_frame = fdata + (int64_t)b * F;
    // tile rectangle relative to the coarse tile
    const uint32_t rx0 = (uint32_t)(ti0 - (cx << cshift)), rx1 = rx0 + kTile - 1;
    const uint32_t ry0 = (uint32_t)(tj0 - (cy << cshift)), ry1 = ry0 + kTile - 1;

    if (AB & 8) {
        best = raw;
    } else {
        // The workgroup reads its coarse bin once: each wave filters a quarter of every 512-entry chunk
        // against the tile into its own list segment; the tile's survivors are staged once (an entry per
        // thread, with the mask of strips it can cover) and every wave rasterises the entries that reach
        // its strip.  Chunks and rounds are workgroup-uniform, so every thread meets every barrier.
        int par = 0;
        for (uint32_t chunk = 0; chunk == 0 || chunk < n_items; chunk += kStrips * kFilterBlock, par ^= 1) {
            uint32_t rid[U];
            bool keep_u[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t idx = chunk + wave * kFilterBlock + u * 64 + lane;
                const bool ok = idx < n_items;
                if (!overflow) {
                    const uint32_t bb = ev[u].y;
                    rid[u] = ev[u].x;
                    keep_u[u] = ok && (bb & 0xff) <= rx1 && ((bb >> 8) & 0xff) >= rx0 && ((bb >> 16) & 0xff) <= ry1 &&
                                (bb >> 24) >= ry0;
                } else {
                    // record slot idx: sub-triangle 0 of face idx, or slot F + 5f + s - 1 (valid if s < nsub)
                    bool valid = ok;
                    if (valid && idx >= (uint32_t)F) {
                        const uint32_t d = idx - (uint32_t)F, fq = d / kExtraPerFace;
                        valid = fdata_frame[fq].nsub > (int)(d - fq * kExtraPerFace + 1);
                    }
                    uint32_t bx = 1, by = 0;
                    if (valid) load_bbox(frame_recs[idx], bx, by);
                    rid[u] = idx;
                    keep_u[u] = valid && (bx & 0xffff) <= (bx >> 16) && (int)(bx & 0xffff) <= ti0 + kTile - 1 &&
                                (int)(bx >> 16) >= ti0 && (int)(by & 0xffff) <= tj0 + kTile - 1 && (int)(by >> 16) >= tj0;
                }
            }
            int n_w = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool keep = keep_u[u];
                const uint64_t mask = __ballot(keep);
                if (keep)
                    t_list[wave][n_w + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] =
                        (int32_t)rid[u];
                n_w += __popcll(mask);
            }
            if (lane == 0) t_nw[par][wave] = n_w;
            __syncthreads();
            if (chunk == 0) PHASE_TS(1);
            int pre[kStrips + 1];
            pre[0] = 0;
#pragma unroll
            for (int w = 0; w < kStrips; ++w) pre[w + 1] = pre[w] + t_nw[par][w];
            const int n_list = pre[kStrips];
            if (AB & 2) {
                best += (uint64_t)n_list;
                __syncthreads();
            }
            for (int from = 0; from < ((AB & 2) ? 0 : n_list); from += 256) {
                const int g = from + t;
                uint32_t m = 0;
                if (g < n_list) {
                    int w = 0;
#pragma unroll
                    for (int q = 1; q < kStrips; ++q) w += g >= pre[q] ? 1 : 0;
                    const int32_t ri = t_list[w][g - pre[w]];
                    StripEntry E;
                    bool large;
                    m = stage_tile(frame_recs, ri, ti0, tj0, F, E, large);
                    int4 *d = reinterpret_cast<int4 *>(&t_ent[t]);
                    d[0] = make_int4(E.e[0], E.e[1], E.e[2], (int)E.ab[0]);
                    d[1] = make_int4((int)E.ab[1], (int)E.ab[2], __float_as_int(E.za), __float_as_int(E.zb));
                    d[2] = make_int4(__float_as_int(E.fx0), __float_as_int(E.fy0), (int)E.key, __float_as_int(E.z0));
                    m |= large ? 16u : 0u;
                }
                t_mask[t] = (uint8_t)m;
                __syncthreads();
                if (chunk == 0 && from == 0) PHASE_TS(2);
                const int nst = min(256, n_list - from);
#if DIRT_RASTER_LISTS
                if (!(AB & 1)) {
                    // this wave's entries as a list (ballot compaction of the round's masks): the loop then
                    // walks offsets read two at a time instead of scanning a bit mask on the scalar unit
                    int ns = 0, nl = 0;
                    for (int c0 = 0; c0 < nst; c0 += 64) {
                        const uint32_t mm = c0 + lane < nst ? t_mask[c0 + lane] : 0u;
                        const bool mine = (mm >> wave) & 1u, big = (mm >> 4) & 1u;
                        const uint64_t bs = __ballot(mine && !big), bl = __ballot(mine && big);
                        if (mine && !big) t_wl[wave][ns + lane_rank(bs)] = (uint32_t)(c0 + lane) * sizeof(StripEntry);
                        if (mine && big) t_wl[wave][kWaveList - 1 - (nl + lane_rank(bl))] = (uint32_t)(c0 + lane);
                        ns += __popcll(bs);
                        nl += __popcll(bl);
                    }
                    if (lane == 0) t_wl[wave][ns] = 256u * sizeof(StripEntry);  // pad / sentinel
                    wave_lds_sync();
                    // two entries per iteration; the next pair's offsets are read before this pair is
                    // tested (reads at k + 2 <= ns + 1 stay inside the list)
                    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                    typedef const volatile __attribute__((address_space(3))) u32x2 lds_u32x2;
                    // Depth-tested programs with long lists (DIRT_RASTER_HZ): the list runs in segments -- the
                    // first DIRT_RASTER_HZ_MIN entries as they are, then each following group of 64 compacted in
                    // place (to its front) to the entries whose depth lower bound over the tile does not exceed
                    // the farthest depth the wave's pixels hold; the others can win no pixel.  A segment starts
                    // even (aligned pair reads); the second read of an odd segment's last pair lands on a
                    // valid entry (stale or next) or the sentinel, and an entry run twice changes nothing (min).
                    int base = 0;
                    int seg = (!kNoDepth && DIRT_RASTER_HZ) ? min(ns, DIRT_RASTER_HZ_MIN) : ns;
                    int rp = seg;  // first list position not yet run or culled
                    for (;;) {
                        u32x2 oo = *(lds_u32x2 *)&t_wl[wave][base];
                        for (int k = base; k < base + seg; k += 2) {
                            const EntryRegs qa = load_entry_at(t_ent, oo.x), qb = load_entry_at(t_ent, oo.y);
                            oo = *(lds_u32x2 *)&t_wl[wave][k + 2];
                            raster_entry<kNoDepth, false>(qa, frame_recs, pix, pxy, i, j, best);
                            raster_entry<kNoDepth, false>(qb, frame_recs, pix, pxy, i, j, best);
                        }
                        if (kNoDepth || !DIRT_RASTER_HZ || rp >= ns) break;
#if DIRT_RASTER_HZ
                        const uint32_t wmax = wave_max_u32((uint32_t)(best >> 32));
                        const int kk = rp + lane;
                        const bool tst = kk < ns;
                        const uint32_t off = tst ? t_wl[wave][kk] : 0u;
                        const bool live = tst && entry_qmin(t_ent, off, ti0 + wave_ox(wave), tj0 + wave_oy(wave)) <= wmax;
                        const uint64_t lm = __ballot(live);
                        if (live) t_wl[wave][rp + lane_rank(lm)] = off;
                        wave_lds_sync();
                        base = rp;
                        seg = __popcll(lm);
                        rp = min(rp + 64, ns);
#endif
                    }
                    for (int k = 0; k < nl; ++k)
                        raster_entry<kNoDepth, true>(load_entry(t_ent, (int)t_wl[wave][kWaveList - 1 - k]), frame_recs, pix,
                                                     pxy, i, j, best);
                } else if (nst > 0) {
                    best += t_ent[lane % nst].key;
                }
#else
                if (!(AB & 1)) {
                    for (int c0 = 0; c0 < nst; c0 += 64) {
                        const uint32_t mm = c0 + lane < nst ? t_mask[c0 + lane] : 0u;
                        uint64_t mine = __ballot((mm >> wave) & 1u);
                        const uint64_t big = __ballot((mm >> 4) & 1u) & mine;
                        if (big == 0) {
                            // two entries per iteration: both sets of reads in flight before either test
                            while (mine) {
                                const int e0 = c0 + (int)__builtin_ctzll(mine);
                                mine &= mine - 1;
                                if (mine) {
                                    const int e1 = c0 + (int)__builtin_ctzll(mine);
                                    mine &= mine - 1;
                                    const EntryRegs qa = load_entry(t_ent, e0), qb = load_entry(t_ent, e1);
                                    raster_entry<kNoDepth, false>(qa, frame_recs, pix, pxy, i, j, best);
                                    raster_entry<kNoDepth, false>(qb, frame_recs, pix, pxy, i, j, best);
                                } else {
                                    raster_entry<kNoDepth, false>(load_entry(t_ent, e0), frame_recs, pix, pxy, i, j, best);
                                }
                            }
                        } else {
                            while (mine) {
                                const int bit = (int)__builtin_ctzll(mine);
                                mine &= mine - 1;
                                const EntryRegs q = load_entry(t_ent, c0 + bit);
                                if ((big >> bit) & 1)
                                    raster_entry<kNoDepth, true>(q, frame_recs, pix, pxy, i, j, best);
                                else
                                    raster_entry<kNoDepth, false>(q, frame_recs, pix, pxy, i, j, best);
                            }
                        }
                    }
                } else if (nst > 0) {
                    best += t_ent[lane % nst].key;
                }
#endif
                // t_ent / t_mask are rewritten by the next round of this chunk; a next chunk rewrites
                // them only after its own filter barrier, and the last round needs no barrier at all
                if (from + 256 < n_list) __syncthreads();
            }
            // next chunk's slab entries (its filter runs after the next barrier-free LDS writes; t_list
            // is rewritten only after this chunk's last staging round)
            if (!overflow && chunk + kStrips * kFilterBlock < n_items) {
                load_chunk(chunk + kStrips * kFilterBlock);
            } else {
                // (no next chunk: defining ev on both paths ends its live range at the filter instead of
                // keeping the stale entries in registers through the staging rounds)
#pragma unroll
                for (int u = 0; u < U; ++u) ev[u] = make_uint2(0u, 0u);
            }
        }
    }
    PHASE_TS(3);
    if (!in_frame) return;
    float *out = pixels + o * C;
    if (AB & 15) {
        gbuffer[o] = (int32_t)best;
        return;
    }
    const int32_t best_rec = best != kKeyInit<kNoDepth> ? key_rec(key_low<kNoDepth>(best), F) : -1;
    if (best_rec < 0) {
        gbuffer[o] = -1;
        if constexpr (SH == DIRT_SHADER_GOURAUD) covbits[o] = 0;
#pragma unroll
        for (int c2 = 0; c2 < CM; ++c2)
            if (c2 < C) out[c2] = kNoDepth ? 0.0f : background[o * C + c2];  // (hill: no background copy)
        PHASE_TS(4);
        PHASE_TS(5);
        return;
    }
    const Rec &r = frame_recs[best_rec];
    const FaceData fd = fdata[(int64_t)b * F + face_of_record(best_rec, F)];
    gbuffer[o] = best_rec | (fd.clipped ? kGbufMulti : 0);
    int64_t E[3];
    edge_values(r, i, j, E);
    float lam[3] = {0.0f, 0.0f, 0.0f};
    // R6 with the int64 -> float conversions done in int32 when every value of the wave fits (the same
    // integers, so the same floats); non-clipped faces skip the identity basis (m_k >= +0 are exact)
    bool fits = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) fits = fits && E[k] == (int64_t)(int32_t)E[k];
    float fE[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fE[k] = (float)(int32_t)E[k];
    if (__builtin_amdgcn_ballot_w64(!fits) != 0) {  // (a real branch: the int64 conversions are not inlined)
        const float3 w = i64x3_to_f32(E[0], E[1], E[2]);
        fE[0] = w.x; fE[1] = w.y; fE[2] = w.z;
    }
    parent_lambda_f(r, fE, fd.clipped == 0, lam);
    PHASE_TS(4);
    if constexpr (SH == DIRT_SHADER_OCEANIC_HORIZON) {
        // texCoordV = perspective-correct clip xy (shaders.cpp:19,21 alias texCoord to position); jitter by
        // the background texel at (texCoordV+1)/2 (NEAREST), channels x,y (C=1 broadcast)
        const float *vb = verts + (int64_t)b * V * 4;
        const float *p0 = vb + (int64_t)fd.v[0] * 4, *p1 = vb + (int64_t)fd.v[1] * 4, *p2 = vb + (int64_t)fd.v[2] * 4;
        const float tx = (lam[0] * p0[0] + lam[1] * p1[0]) + lam[2] * p2[0];
        const float ty = (lam[0] * p0[1] + lam[1] * p1[1]) + lam[2] * p2[1];
        const float u = (tx + 1.0f) / 2.0f, v = (ty + 1.0f) / 2.0f;
        int ix = (int)floorf(u * (float)W), iy = (int)floorf(v * (float)H);
        if (!(u * (float)W >= 0.0f)) ix = 0;
        if (!(v * (float)H >= 0.0f)) iy = 0;
        ix = ix < 0 ? 0 : (ix > W - 1 ? W - 1 : ix);
        iy = iy < 0 ? 0 : (iy > H - 1 ? H - 1 : iy);
        const float *texel = background + (((int64_t)b * H + (H - 1 - iy)) * W + ix) * C;
        const float sx = texel[0], sy = C >= 2 ? texel[1] : texel[0];
        const ocean::Camera camv{cam[0], cam[1], cam[2], cam[3], cam[4], cam[5], cam[6], cam[7]};
        const float2 col = ocean::shade(tx + sx / (float)W, ty + sy / (float)H, camv, (float)W, (float)H);
        for (int k = 0; k < C; ++k) out[k] = k == 0 ? col.x : k == 1 ? col.y : k == 3 ? 1.0f : 0.0f;
    } else if constexpr (SH == DIRT_SHADER_HILL) {
        // hill: texCoordV without jitter; the op's background tensor is the terrain lookup (tcb channels)
        const float *vb = verts + (int64_t)b * V * 4;
        const float *p0 = vb + (int64_t)fd.v[0] * 4, *p1 = vb + (int64_t)fd.v[1] * 4, *p2 = vb + (int64_t)fd.v[2] * 4;
        const float tx = (lam[0] * p0[0] + lam[1] * p1[0]) + lam[2] * p2[0];
        const float ty = (lam[0] * p0[1] + lam[1] * p1[1]) + lam[2] * p2[1];
        const hill::Tex T{background + (int64_t)b * H * W * tcb, H, W, tcb};
        const float4 col = hill::shade(T, tx, ty, cam);
        for (int k = 0; k < C; ++k) out[k] = k == 0 ? col.x : k == 1 ? col.y : k == 2 ? col.z : k == 3 ? col.w : 0.0f;
    } else if constexpr (SH == DIRT_SHADER_OCEANIC) {
        // the oceanic family (shader ids 2..6, `sid` at run time), same texCoordV and jitter as above
        const float *vb = verts + (int64_t)b * V * 4;
        const float *p0 = vb + (int64_t)fd.v[0] * 4, *p1 = vb + (int64_t)fd.v[1] * 4, *p2 = vb + (int64_t)fd.v[2] * 4;
        const float tx = (lam[0] * p0[0] + lam[1] * p1[0]) + lam[2] * p2[0];
        const float ty = (lam[0] * p0[1] + lam[1] * p1[1]) + lam[2] * p2[1];
        if (sid == DIRT_SHADER_OCEANIC_OPT_FLOW) {
            // no jitter (shaders.cpp:1323-1325 commented out); fragColor = (new_coord, 0, 1)
            const float2 nc = ocean::opt_flow(tx, ty, cam, (float)W, (float)H);
            for (int k = 0; k < C; ++k) out[k] = k == 0 ? nc.x : k == 1 ? nc.y : k == 3 ? 1.0f : 0.0f;
            return;
        }
        const float u = (tx + 1.0f) / 2.0f, v = (ty + 1.0f) / 2.0f;
        int ix = (int)floorf(u * (float)W), iy = (int)floorf(v * (float)H);
        if (!(u * (float)W >= 0.0f)) ix = 0;
        if (!(v * (float)H >= 0.0f)) iy = 0;
        ix = ix < 0 ? 0 : (ix > W - 1 ? W - 1 : ix);
        iy = iy < 0 ? 0 : (iy > H - 1 ? H - 1 : iy);
        const float *texel = background + (((int64_t)b * H + (H - 1 - iy)) * W + ix) * C;
        const float sx = texel[0], sy = C >= 2 ? texel[1] : texel[0];
        const float3 col = ocean::shade_family(ocean::family_params(sid), tx + sx / (float)W, ty + sy / (float)H, cam,
                                               (float)W, (float)H);
        for (int k = 0; k < C; ++k) out[k] = k == 0 ? col.x : k == 1 ? col.y : k == 2 ? col.z : k == 3 ? 1.0f : 0.0f;
    } else {
        if (AB & 64) {
            for (int k = 0; k < C; ++k) out[k] = lam[k % 3];
        } else {
            const float *cb = colors + (int64_t)b * V * C;
            const float *c0 = cb + (int64_t)fd.v[0] * C, *c1 = cb + (int64_t)fd.v[1] * C, *c2 = cb + (int64_t)fd.v[2] * C;
            for (int k = 0; k < C; ++k) out[k] = (lam[0] * c0[k] + lam[1] * c1[k]) + lam[2] * c2[k];
        }
        covbits[o] = (AB & 32) ? (uint8_t)0
                               : (uint8_t)neighbour_coverage(r, E, fd.clipped != 0, best_rec, frame_recs,
                                                             fdata + (int64_t)b * F, F, face_of_record(best_rec, F), i, j);
        PHASE_TS(5);
    }
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
//   2. run tails write their partial sums into their record's contiguous LDS range (records kept in a
//      per-tile LDS hash table keyed by record index, vertex ids cached);
//   3. one wave-instruction of global float atomics per (tile, record): <= 9+3C lanes, ~3 cache lines.

// Does face f cover pixel (i,j)?  `hint` is the record of f covering a neighbouring pixel; the other
// sub-records of f are only consulted when f was clipped into several (`multi`).
__device__ __forceinline__ bool edge_covers(const EdgePart &r, int i, int j)
{
    // empty records have i0 > i1 and are rejected by the bbox test
    if (r.i0 > r.i1 || i < r.i0 || i > r.i1 || j < r.j0 || j > r.j1) return false;
    int64_t E[3];
    edge_values(r, i, j, E);
    return inside(r, E);
}

__device__ __noinline__ bool covers_face_multi(int64_t hint_ri, const Rec *frame_recs, const FaceData *fdata_frame,
                                               int F, int f, int i, int j)
{
    const int n = fdata_frame[f].nsub;
    for (int s = 0; s < n; ++s) {
        const int64_t ri = rec_index(F, f, s);
        if (ri == hint_ri) continue;
        if (edge_covers(*reinterpret_cast<const EdgePart *>(&frame_recs[ri]), i, j)) return true;
    }
    return false;
}

__device__ __forceinline__ bool covers_face(const EdgePart &hint, int64_t hint_ri, bool multi, const Rec *frame_recs,
                            const FaceData *fdata_frame, int F, int f, int i, int j)
{
    if (edge_covers(hint, i, j)) return true;
    if (!multi) return false;
    return covers_face_multi(hint_ri, frame_recs, fdata_frame, F, f, i, j);
}

template <int D>
__device__ __forceinline__ float dpp_shr_f(float v)  // lane l <- lane l-D of the same 16-lane row, 0 if none
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x110 + D, 0xF, 0xF, true));
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

// int64 -> f32 with two conversions (may double-round: backward-only, tolerance-level)
__device__ __forceinline__ float fast_i64_to_f32(int64_t v)
{
    const int32_t hi = (int32_t)(v >> 32);
    const uint32_t lo = (uint32_t)v;
    return fmaf((float)hi, 4294967296.0f, (float)lo);
}

// perspective-correct barycentrics from a_k = E_k / w_k (R6) with one fast reciprocal
__device__ __forceinline__ bool fast_lambda(const Rec &r, bool multi, float a0, float a1, float a2, float lam[3])
{
    const float s = (a0 + a1) + a2;
    if (s == 0.0f) return false;
    const float rs = __builtin_amdgcn_rcpf(s);
    const float m0 = a0 * rs, m1 = a1 * rs, m2 = a2 * rs;
    if (!multi) {
        lam[0] = m0; lam[1] = m1; lam[2] = m2;
        return true;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) lam[i] = (m0 * r.basis[i] + m1 * r.basis[3 + i]) + m2 * r.basis[6 + i];
    return true;
}

#ifndef DIRT_GRAD_WAVES
#define DIRT_GRAD_WAVES 6  // min waves per SIMD the register allocation must allow
#endif
#ifndef DIRT_GRAD_WAVES_C3
#define DIRT_GRAD_WAVES_C3 8  // C = 3: 64 VGPRs without spills (then 7 workgroups per CU, LDS-bound);
                              // C = 1 spills at 8, the generic paths are LDS-bound at 5
#endif
#ifndef DIRT_GRAD_ATTR
#define DIRT_GRAD_ATTR
#endif

// window-transform constants of the chain rule, computed on the host (IEEE, as the oracle)
struct NdcScale {
    float inv_hw, inv_hh, half_w, half_h;
};

constexpr int kHalo = kTile + 2;   // staged tile with a one-pixel border
constexpr int kHaloPix = kHalo * kHalo;
constexpr int kSlots = 64;         // distinct records per tile+halo kept in LDS (typ. 10-40)
constexpr int kNoSlot = -3;        // record not in the slot table: read it from global memory
static_assert(kSlots <= 128, "slot ids (0 .. kSlots-1) are stored as int8");

// LDS-resident copy of the edge part of the records seen in a tile + halo (for coverage tests of a
// neighbour's face) and of their vertex ids (for the flush).
struct SlotTable {
    int32_t key[kSlots];     // g-buffer word (record index | clipped flag), -1 = free
    int8_t list[kSlots];     // occupied slots in insertion order
    int32_t A[3][kSlots], B[3][kSlots];
    int32_t e[3][kSlots];      // small records: E + owned at the halo origin pixel (see kGradSmallEdge)
    uint32_t bx[kSlots], by[kSlots];  // i0 | i1 << 16 (bit 31: large record, use the global Rec)
    int32_t v[3][kSlots];    // vertex ids, indexed by list position
    float iw[3][kSlots], w[3][kSlots];  // interpolation data of the record (own-pixel path)
    float h2d[kSlots];                  // 1 / (2 D), D = E0 + E1 + E2 (constant over the plane)
    int32_t n;
};

// A record is "small" for the backward when every |A|, |B| < 2^14 (edges shorter than 64 px).  Such a
// record is visible somewhere in the 18x18 tile + halo region, so at every region pixel its edge values
// satisfy |E| < 2^28 (E at a covered pixel) + 2 * 2^14 * 17 * 256 < 2^30: exact in int32, and a
// coverage test is E0 + A*256*hx + B*256*hy with 24-bit multiplies (hx, hy in 0..17).
constexpr int32_t kGradSmallEdge = 1 << 14;
constexpr uint32_t kSlotLarge = 0x80000000u;

__device__ __forceinline__ bool slot_is_large(const SlotTable &T, int s) { return (T.bx[s] & kSlotLarge) != 0; }

// exact coverage of region pixel (hx, hy) = absolute (i, j) by small slot s (bbox + R2/R3 edge test)
__device__ __forceinline__ bool slot_covers_small(const SlotTable &T, int s, int hx, int hy, int i, int j)
{
    const uint32_t bx = T.bx[s], by = T.by[s];
    if (i < (int)(bx & 0xffff) || i > (int)((bx >> 16) & 0x7fff) || j < (int)(by & 0xffff) || j > (int)(by >> 16))
        return false;
    const int32_t x = hx * 256, y = hy * 256;
    const int32_t e0 = T.e[0][s] + __mul24(T.A[0][s], x) + __mul24(T.B[0][s], y);
    const int32_t e1 = T.e[1][s] + __mul24(T.A[1][s], x) + __mul24(T.B[1][s], y);
    const int32_t e2 = T.e[2][s] + __mul24(T.A[2][s], x) + __mul24(T.B[2][s], y);
    return min(e0, min(e1, e2)) > 0;
}

__device__ __forceinline__ int32_t owned_bit(int32_t A, int32_t B) { return (A > 0 || (A == 0 && B < 0)) ? 1 : 0; }

__device__ __forceinline__ int slot_hash(int32_t key) { return (int)(((uint32_t)key * 2654435761u) >> 25) & (kSlots - 1); }

// Insert `key` for every lane with `want` (called by the whole wave, converged): probes advance in
// lockstep, and the lanes that created a slot append it to the slot list with one atomic per wave.
// Returns the slot, kNoSlot if the table is full, -1 where !want.
__device__ __forceinline__ int slot_insert_wave(SlotTable &T, int32_t key, bool want)
{
    int slot = slot_hash(key);
    int result = want ? kNoSlot : -1;
    bool pending = want, fresh = false;
    for (int probe = 0; probe < kSlots; ++probe) {
        if (!__any(pending)) break;
        if (pending) {
            const int old = atomicCAS(&T.key[slot], -1, key);
            if (old == -1 || old == key) {
                result = slot;
                fresh = old == -1;
                pending = false;
            } else {
                slot = (slot + 1) & (kSlots - 1);
            }
        }
    }
    const uint64_t mask = __ballot(fresh);
    if (mask) {
        int base = 0;
        if ((threadIdx.x & 63) == 0) base = atomicAdd(&T.n, __popcll(mask));
        base = __shfl(base, 0, 64);
        if (fresh)
            T.list[base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] = (int8_t)result;
    }
    return result;
}

// pair scalar s = -0.5 sum_c (G(p)+G(q)) (I(q)-I(p)) of staged pixels p = k, q = k2 (same operand order
// as the oracle), 0 when either is outside the frame; every operand read unconditionally (no branches
// between the LDS reads)
template <int CP, int CM>
__device__ __forceinline__ float pair_scalar(const int32_t *s_gb, const float *s_G, const float *s_I, int k, int k2, int C)
{
    const int32_t g1 = s_gb[k], g2 = s_gb[k2];
    float a = 0.0f;
    if (CP == 4 && CM == 3) {
        typedef float f3v __attribute__((ext_vector_type(3)));  // ds_read_b96: 3 registers per operand
        const f3v Gp = *reinterpret_cast<const f3v *>(&s_G[k * 4]), Gq = *reinterpret_cast<const f3v *>(&s_G[k2 * 4]);
        const f3v Ip = *reinterpret_cast<const f3v *>(&s_I[k * 4]), Iq = *reinterpret_cast<const f3v *>(&s_I[k2 * 4]);
        a = (Gp.x + Gq.x) * (Iq.x - Ip.x);
        a = a + (Gp.y + Gq.y) * (Iq.y - Ip.y);
        a = a + (Gp.z + Gq.z) * (Iq.z - Ip.z);
    } else {
        for (int c = 0; c < C; ++c) a += (s_G[k * CP + c] + s_G[k2 * CP + c]) * (s_I[k2 * CP + c] - s_I[k * CP + c]);
    }
    return (g1 != -2 && g2 != -2) ? -0.5f * a : 0.0f;
}

// Index (0..15) of the first lane of this lane's run of equal `key` in its 16-lane DPP row.
__device__ __forceinline__ int run_start(int key, int lx)
{
    const int kl = dpp_shr_i<1>(key, -3);
    int start = (lx == 0 || kl != key) ? lx : -1;
    start = max(start, dpp_shr_i<1>(start, -1));
    start = max(start, dpp_shr_i<2>(start, -1));
    start = max(start, dpp_shr_i<4>(start, -1));
    start = max(start, dpp_shr_i<8>(start, -1));
    return start;
}

// AB: ablation mask for tools/ablate.py (0 in the product): 1 skip pairs, 2 skip colour weights,
// 4 skip the whole reduction, 8 skip only the global flush, 16 skip neighbour coverage tests,
// 32 skip the DPP run scan (every lane adds into LDS), 128 phase timestamps, 256 flush sums without
// the global atomics
template <int CC, int AB = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256),
                          amdgpu_waves_per_eu(CC == 3 ? DIRT_GRAD_WAVES_C3 : DIRT_GRAD_WAVES))) DIRT_GRAD_ATTR void grad_kernel(const float *__restrict__ pixels, const float *__restrict__ grad_pixels,
                                                   const int32_t *__restrict__ gbuffer, const uint8_t *__restrict__ covbits,
                                                   const Rec *__restrict__ recs,
                                                   const FaceData *__restrict__ fdata, int B, int H, int W, int Cdyn,
                                                   int V, int F, TileGrid tg, int64_t nrec, float *__restrict__ grad_verts,
                                                   float *__restrict__ grad_colors, float *__restrict__ grad_bg,
                                                   const NdcScale ns)
{
    constexpr int CM = CC > 0 ? CC : DIRT_MAX_CHANNELS;
    constexpr int CP = CM == 3 ? 4 : CM;  // LDS pixel stride (float4 for RGB)
    constexpr int NVM = 9 + 3 * CM;
    const int C = CC > 0 ? CC : Cdyn;
    const int NV = 9 + 3 * C;
#if defined(DIRT_GRAD_LDS_PAD) && DIRT_GRAD_LDS_PAD > 0
    __shared__ volatile char occupancy_probe[DIRT_GRAD_LDS_PAD];  // experiment: caps workgroups per CU
    if (threadIdx.x == 1023) occupancy_probe[0] = 0;
#endif
    __shared__ int32_t s_gb[kHaloPix];
    __shared__ uint8_t s_cov[kHaloPix];  // neighbour_coverage() bits of the pixel's face (forward)
    __shared__ int8_t s_slot[kHaloPix];  // slot of the pixel's record, -1 none, kNoSlot table full
#ifndef DIRT_GRAD_PAIR_RECOMPUTE
#define DIRT_GRAD_PAIR_RECOMPUTE 1
#endif
    // RGB: each lane recomputes the pair scalars of its four pairs in phase B instead of staging them
    // (LDS 22 -> 19 KiB: 8 workgroups per CU instead of 7); other channel counts stage them in phase A
    constexpr bool kRecompute = DIRT_GRAD_PAIR_RECOMPUTE && CM == 3;
    __shared__ float s_sx[kRecompute ? 1 : kHaloPix];  // pair scalar s of (k, k+x) and (k, k+y), DESIGN.md 4
    __shared__ float s_sy[kRecompute ? 1 : kHaloPix];
    // G / I of the staged pixels (phases A-B), then reused for the run-tail partial sums (C-D):
    // keeps the workgroup at ~26 KB of LDS (6 per CU)
    constexpr int kUnion = 2 * kHaloPix * CP;
    constexpr int kTailCap = kUnion / NVM;
    __shared__ __attribute__((aligned(16))) float s_u[kUnion];
    float *const s_G = s_u;
    float *const s_I = s_u + kHaloPix * CP;
    float *const s_part = s_u;
    // pair scalar of the pair (klo, klo + x) (axis 0) or (klo, klo + kHalo) (axis 1)
    auto pair_s = [&](int axis, int klo) -> float {
        if constexpr (kRecompute)
            return pair_scalar<CP, CM>(s_gb, s_G, s_I, klo, klo + (axis == 0 ? 1 : kHalo), C);
        else
            return axis == 0 ? s_sx[klo] : s_sy[klo];
    };
    __shared__ SlotTable T;
    // per slot: its number of row runs (= run tails), then the start (a cursor during the tail phase)
    // of its contiguous range of tail partials in s_part
    __shared__ int32_t s_tcnt[kSlots];
    __shared__ int32_t s_toff[kSlots];
    __shared__ int32_t s_lbeg[kSlots], s_lcnt[kSlots];  // the same ranges by list position (flush)

    const int tile = xcd_tile(blockIdx.x, gridDim.x), b = blockIdx.y;
    int tx, ty;
    tg.split(tile, tx, ty);
    const int t = threadIdx.x, lx = t & 15, ly = t >> 4;
    const int i = tx * kTile + lx, j = ty * kTile + ly;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const FaceData *fdata_frame = fdata + (int64_t)b * F;
    // uniform: readfirstlane (convergent) keeps the divisions at the top instead of in every pair branch
    const float inv_hw = ns.inv_hw, inv_hh = ns.inv_hh;  // 2/W, 2/H from the host (no division in the kernel)
    const int kme = (ly + 1) * kHalo + (lx + 1);
    const bool in_frame = i < W && j < H;

    // ---- phase A: stage g-buffer / G / I of the tile + one-pixel halo, pair scalars, slot table
    PHASE_TS(0);
    for (int k = t; k < kSlots; k += 256) {
        T.key[k] = -1;
        s_tcnt[k] = 0;
    }
    if (t == 0) T.n = 0;
    const int hi0 = tx * kTile - 1, hj0 = ty * kTile - 1;
    {
        // every load of both passes in flight before the first LDS store (kHaloPix <= 2 * 256)
        static_assert(kHaloPix <= 512, "two staging passes");
        // frame base pointers (64-bit, uniform) + 32-bit per-lane offsets: H * W * C < 2^29
        const int64_t fpix = (int64_t)b * H * W;
        const int32_t *gb_f = gbuffer + fpix;
        const uint8_t *cov_f = covbits + fpix;
        const float *gp_f = grad_pixels + fpix * C, *px_f = pixels + fpix * C;
        int32_t gbv[2];
        uint32_t cvv[2];
        float Gv[2][CM], Iv[2][CM];
        bool ok[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = t + 256 * u;
            const int hi = hi0 + k % kHalo, hj = hj0 + k / kHalo;
            ok[u] = k < kHaloPix && hi >= 0 && hj >= 0 && hi < W && hj < H;
            gbv[u] = -2;
            cvv[u] = 0;
            if (ok[u]) {
                const uint32_t o = (uint32_t)((H - 1 - hj) * W + hi);
                gbv[u] = gb_f[o];
                cvv[u] = cov_f[o];
                // one pixel's channels from one base address (o * C < 2^29): RGB becomes one
                // global_load_dwordx3 per operand instead of three dword loads
                const float *gq = gp_f + o * (uint32_t)C, *pq = px_f + o * (uint32_t)C;
#pragma unroll
                for (int c = 0; c < CM; ++c)
                    if (c < C) {
                        Gv[u][c] = gq[c];
                        Iv[u][c] = pq[c];
                    }
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = t + 256 * u;
            if (k >= kHaloPix) continue;
            s_gb[k] = gbv[u];
            s_cov[k] = (uint8_t)cvv[u];
            if (!ok[u]) continue;
            if constexpr (CM == 3) {
                *reinterpret_cast<float4 *>(&s_G[k * CP]) = make_float4(Gv[u][0], Gv[u][1], Gv[u][2], 0.0f);
                *reinterpret_cast<float4 *>(&s_I[k * CP]) = make_float4(Iv[u][0], Iv[u][1], Iv[u][2], 0.0f);
            } else {
#pragma unroll
                for (int c = 0; c < CM; ++c)
                    if (c < C) {
                        s_G[k * CP + c] = Gv[u][c];
                        s_I[k * CP + c] = Iv[u][c];
                    }
            }
        }
    }
    __syncthreads();
    PHASE_TS(1);
    const int32_t gp = in_frame ? s_gb[kme] : -2;
    {
        const int rt = (t & 63) * 4 + (t >> 6);  // 0..255 spread over the four waves
        // the tile's own records (run heads only; all distinct keys may not fit: the rest read global
        // memory).  The halo's records are not needed: pair coverage comes from the forward's bits.
        (void)rt;
        const int32_t g = s_gb[kme];
        const int key = g >= 0 ? g : -1;
        const int start = run_start(key, lx);
        int slot = slot_insert_wave(T, key, key >= 0 && start == lx);
        if (key >= 0 && start == lx && slot >= 0) atomicAdd(&s_tcnt[slot], 1);  // one run (one tail later)
        slot = __shfl(slot, (t & 48) + start, 64);
        s_slot[kme] = key >= 0 ? slot : -1;
    }
    __syncthreads();
    PHASE_TS(2);
    PHASE_TS(3);
    const int nslots = T.n;
    static_assert(kSlots <= 64, "one slot per lane of wave 0");
    if (t < 64) {
        // wave 0: each slot's range of run-tail partials, in slot-list order (exclusive prefix)
        const int sl = t < nslots ? T.list[t] : 0;
        const int cnt = t < nslots ? s_tcnt[sl] : 0;
        int inc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(inc, d, 64);
            inc += t >= d ? v : 0;
        }
        if (t < nslots) {
            s_toff[sl] = inc - cnt;
            s_lbeg[t] = inc - cnt;
            s_lcnt[t] = cnt;
        }
    }
    {
        // slot fill: the record loads are issued first and land while the pair scalars are computed
        const bool filler = t < nslots;
        int sf = 0;
        EdgePart ep{};
        FaceData fd{};
        float riw0 = 0.f, riw1 = 0.f, riw2 = 0.f;
        if (filler) {
            sf = T.list[t];
            const int32_t ri = T.key[sf] & kGbufIndexMask;
            ep = *reinterpret_cast<const EdgePart *>(&frame_recs[ri]);
            fd = fdata_frame[face_of_record(ri, F)];
            const Rec &r = frame_recs[ri];
            riw0 = r.iw[0]; riw1 = r.iw[1]; riw2 = r.iw[2];
        }
        // pair scalars of the pairs starting at an own pixel (right, up) and at the left column /
        // bottom row of the halo (their one pair into the tile); nothing reads the others
        if constexpr (!kRecompute) {
        const int rt = (t & 63) * 4 + (t >> 6);
        s_sx[kme] = pair_scalar<CP, CM>(s_gb, s_G, s_I, kme, kme + 1, C);
        s_sy[kme] = pair_scalar<CP, CM>(s_gb, s_G, s_I, kme, kme + kHalo, C);
        if (rt < 16) {
            const int k = (rt + 1) * kHalo;  // (0, rt + 1)
            s_sx[k] = pair_scalar<CP, CM>(s_gb, s_G, s_I, k, k + 1, C);
        } else if (rt < 32) {
            const int k = rt - 15;  // (rt - 15, 0)
            s_sy[k] = pair_scalar<CP, CM>(s_gb, s_G, s_I, k, k + kHalo, C);
        }
        }
        if (filler) {
            bool small = true;
            int64_t E0[3];
            edge_values(ep, hi0, hj0, E0);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                T.A[k][sf] = ep.A[k]; T.B[k][sf] = ep.B[k];
                T.v[k][t] = fd.v[k];  // by list position (read only by the flush)
                T.w[k][sf] = fd.w[k];
                small = small && ep.A[k] > -kGradSmallEdge && ep.A[k] < kGradSmallEdge && ep.B[k] > -kGradSmallEdge &&
                        ep.B[k] < kGradSmallEdge;
                T.e[k][sf] = (int32_t)E0[k] + owned_bit(ep.A[k], ep.B[k]);  // meaningful only when small
            }
            T.iw[0][sf] = riw0; T.iw[1][sf] = riw1; T.iw[2][sf] = riw2;
            T.h2d[sf] = 0.5f / (float)(E0[0] + E0[1] + E0[2]);
            T.bx[sf] = (uint32_t)ep.i0 | ((uint32_t)ep.i1 << 16) | (small ? 0u : kSlotLarge);
            T.by[sf] = (uint32_t)ep.j0 | ((uint32_t)ep.j1 << 16);
        }
    }
    __syncthreads();
    PHASE_TS(4);

    // ---- phase B: per-pixel contributions to the face visible at this pixel
    const int32_t rp = gp >= 0 ? (gp & kGbufIndexMask) : gp;
    if (in_frame) {
        float *gbg_f = grad_bg + (int64_t)b * H * W * C;
        const uint32_t o = (uint32_t)((H - 1 - j) * W + i);
        float *gbq = gbg_f + o * (uint32_t)C;  // (RGB: one global_store_dwordx3)
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            const float gv = s_G[kme * CP + c];
            if (c < C) gbq[c] = rp < 0 ? gv : 0.0f;
        }
    }

    float acc[NVM];
#pragma unroll
    for (int v = 0; v < NVM; ++v) acc[v] = 0.0f;
    const int sp = rp >= 0 ? s_slot[kme] : -1;
    if (rp >= 0) {
        // Ownership decisions (coverage tests) are exact int64; the interpolation weights use fast
        // reciprocals (contributions agree with the oracle to ~1e-6 relative, far inside the 1e-4
        // tolerance the atomic summation order already needs).  The own record comes through the
        // vector-memory path (L1-resident: a wave touches a handful of records).
        const int f = face_of_record(rp, F);
        const bool multi = (gp & kGbufMulti) != 0;
        // the own record (large records and the basis of clipped faces): its address is recomputed at
        // each use from rp (the asm hides the common subexpression) instead of living in two registers
        auto rec = [&]() -> const Rec & {
            int r2 = rp;
            asm volatile("" : "+v"(r2));
            return frame_recs[r2];
        };
        const int hx = lx + 1, hy = ly + 1;  // region coordinates of this pixel
        int32_t mA[3], mB[3], eme[3];       // eme: E + owned here (small records only)
        float iw0, iw1, iw2, h2d;
        float fEp[3];
        bool me_small;
        if (sp >= 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) { mA[k] = T.A[k][sp]; mB[k] = T.B[k][sp]; }
            iw0 = T.iw[0][sp]; iw1 = T.iw[1][sp]; iw2 = T.iw[2][sp];
            h2d = T.h2d[sp];
            me_small = !slot_is_large(T, sp);
        } else {
            const Rec &rr = rec();
            const EdgePart me = *reinterpret_cast<const EdgePart *>(&rr);
#pragma unroll
            for (int k = 0; k < 3; ++k) { mA[k] = me.A[k]; mB[k] = me.B[k]; }
            iw0 = rr.iw[0]; iw1 = rr.iw[1]; iw2 = rr.iw[2];
            int64_t E0[3];
            edge_values(me, i, j, E0);
            h2d = 0.5f / (float)(E0[0] + E0[1] + E0[2]);
            me_small = false;
        }
        if (me_small) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                eme[k] = T.e[k][sp] + __mul24(mA[k], hx * 256) + __mul24(mB[k], hy * 256);
                fEp[k] = (float)(eme[k] - owned_bit(mA[k], mB[k]));
            }
        } else {
            const EdgePart me = *reinterpret_cast<const EdgePart *>(&rec());
            int64_t Ep[3];
            edge_values(me, i, j, Ep);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                fEp[k] = fast_i64_to_f32(Ep[k]);
                eme[k] = 0;
            }
        }
        // the four pairs around the pixel: dir 0 right, 1 left (x axis); 2 up, 3 down (y axis, window).
        // Pass 1 decides ownership (exact integer coverage tests) into 2-bit codes (0 skip, 1 half,
        // 2 whole); pass 2 interpolates and accumulates.  Splitting keeps the coverage tests' and the
        // accumulators' registers apart (occupancy).
        PHASE_TS(10 + (fEp[0] == 12345.f));
        if (!(AB & 17) && __builtin_amdgcn_ballot_w64(multi) == 0) {
            // No clipped face in this wave: ownership and accumulation of the four pairs without
            // branches.  A neighbour shows my face iff it shows my record (a non-clipped face has exactly
            // one).  Ownership code: outside the frame 0, background 2, same face 2 for the
            // lower pixel of the pair / 0 for the upper, else 1 + (q's face covers p) - (p's face covers q).
            // The pair weight of vertex k is c_d * m_k with m_k = (2 E_k +- 256 A_k (or B_k)) / w_k =
            // P_k +- Q_k and c_d = code_d * s_d * (W/2 or H/2) / (4D), so the two pairs of an axis fold
            // into (c_0 + c_1) P_k + (c_0 - c_1) Q_k (and the same with the NDC factors for w).
            const uint32_t covme = s_cov[kme];
            float cd[4];
#pragma unroll
            for (int dir = 0; dir < 4; ++dir) {
                const int axis = dir >> 1;
                const bool me_low = (dir & 1) == 0;
                const int di = axis == 0 ? (me_low ? 1 : -1) : 0, dj = axis == 1 ? (me_low ? 1 : -1) : 0;
                const int kq = kme + dj * kHalo + di;
                const int32_t gq = s_gb[kq];
                const uint32_t covq = s_cov[kq];  // read unconditionally: the code below is all selects
                const float s = pair_s(axis, me_low ? kme : kq);
                const int32_t rq = gq & kGbufIndexMask;
                int code = 1 + (int)((covq >> (dir ^ 1)) & 1u) - (int)((covme >> dir) & 1u);
                code = rq == rp ? (me_low ? 2 : 0) : code;
                code = gq < 0 ? 2 : code;
                code = gq == -2 ? 0 : code;
                const float K = (axis == 0 ? ns.half_w : ns.half_h) * h2d * 0.5f;
                cd[dir] = code == 0 ? 0.0f : ((float)code * s) * K;
            }
            const float ndc_r = (float)(i + 1) * inv_hw - 1.0f, ndc_l = (float)i * inv_hw - 1.0f;
            const float ndc_u = (float)(j + 1) * inv_hh - 1.0f, ndc_d = (float)j * inv_hh - 1.0f;
            const float ux = cd[0] + cd[1], vx = cd[0] - cd[1];
            const float uwx = cd[0] * ndc_r + cd[1] * ndc_l, vwx = cd[0] * ndc_r - cd[1] * ndc_l;
            const float uy = cd[2] + cd[3], vy = cd[2] - cd[3];
            const float uwy = cd[2] * ndc_u + cd[3] * ndc_d, vwy = cd[2] * ndc_u - cd[3] * ndc_d;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float iwk = k == 0 ? iw0 : k == 1 ? iw1 : iw2;
                const float P = (2.0f * fEp[k]) * iwk;
                const float Qx = ((float)mA[k] * 256.0f) * iwk, Qy = ((float)mB[k] * 256.0f) * iwk;
                acc[k * 3 + 0] += ux * P + vx * Qx;
                acc[k * 3 + 1] += uy * P + vy * Qy;
                acc[k * 3 + 2] -= (uwx * P + vwx * Qx) + (uwy * P + vwy * Qy);
            }
            PHASE_TS(11 + (acc[0] == 12345.f));
        } else {
        uint32_t codes = 0;
#pragma unroll
        for (int dir = 0; dir < 4; ++dir) {
            if (AB & 1) break;
            const int axis = dir >> 1;
            const bool me_low = (dir & 1) == 0;
            const int di = axis == 0 ? (me_low ? 1 : -1) : 0, dj = axis == 1 ? (me_low ? 1 : -1) : 0;
            const int kq = kme + dj * kHalo + di;
            const int32_t gq = s_gb[kq];
            if (gq == -2) continue;
            const int klo = me_low ? kme : kq;
            const float s = pair_s(axis, klo);
            if (s == 0.0f) continue;
            const int32_t rq = gq >= 0 ? (gq & kGbufIndexMask) : -1;
            const int fq = rq >= 0 ? face_of_record(rq, F) : -1;
            uint32_t code;
            if (fq == f) {
                code = me_low ? 2u : 0u;
            } else if (fq < 0) {
                code = 2u;
            } else if (AB & 16) {
                code = 1u;
            } else {
                // the forward's neighbour_coverage(): my face at q (bit dir of p), q's face at p (bit
                // opposite(dir) of q; opposite flips bit 0 of dir)
                const bool mine_covers_other = (s_cov[kme] >> dir) & 1u;
                const bool other_covers_me = (s_cov[kq] >> (dir ^ 1)) & 1u;
                code = (!mine_covers_other && other_covers_me) ? 2u : (mine_covers_other && !other_covers_me) ? 0u : 1u;
            }
            codes |= code << (2 * dir);
        }
        PHASE_TS(11 + (codes == 12345u));
#pragma unroll
        for (int dir = 0; dir < 4; ++dir) {
            const uint32_t code = (codes >> (2 * dir)) & 3u;
            if (code == 0u) continue;
            const int axis = dir >> 1;
            const bool me_low = (dir & 1) == 0;
            const int di = axis == 0 ? (me_low ? 1 : -1) : 0, dj = axis == 1 ? (me_low ? 1 : -1) : 0;
            const int klo = me_low ? kme : kme + dj * kHalo + di;
            const float s = pair_s(axis, klo);
            const float omega = code == 2u ? 1.0f : 0.5f;
            // midpoint: E(p) + E(q) = 2 E(p) + step, step = one pixel (256 sub-pixels) of the edge
            float m[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float st = (float)(axis == 0 ? mA[k] : mB[k]) * (me_low ? 256.0f : -256.0f);  // = (float)(A * 256)
                m[k] = (2.0f * fEp[k] + st) * (k == 0 ? iw0 : k == 1 ? iw1 : iw2);
            }
            const int ilo = me_low ? i : i + di, jlo = me_low ? j : j + dj;
            const float half = axis == 0 ? ns.half_w : ns.half_h;
            const float mid = axis == 0 ? (float)(ilo + 1) : (float)(jlo + 1);
            const float ndc = mid * (axis == 0 ? inv_hw : inv_hh) - 1.0f;
            float g[3];
            if (!multi) {
                // Non-clipped face (identity basis, iw_k w_k = 1): lambda_k / Wm = a_k / sum_k (a_k w_k)
                // = a_k / (2E_0 + 2E_1 + 2E_2 + st_0 + st_1 + st_2) = a_k / (2D), since the edge
                // functions sum to the constant D and their steps to 0 -- no division per pair
                const float c = omega * s * half * h2d;
#pragma unroll
                for (int k = 0; k < 3; ++k) g[k] = c * m[k];
            } else {
                float lm[3];
                if (!fast_lambda(rec(), multi, m[0], m[1], m[2], lm)) continue;
                // clip w of the parent vertices, read here (clipped faces only) to keep them out of
                // the registers of the common path
                const float w0 = sp >= 0 ? T.w[0][sp] : fdata_frame[f].w[0];
                const float w1 = sp >= 0 ? T.w[1][sp] : fdata_frame[f].w[1];
                const float w2 = sp >= 0 ? T.w[2][sp] : fdata_frame[f].w[2];
                const float Wm = (lm[0] * w0 + lm[1] * w1) + lm[2] * w2;
                if (Wm == 0.0f) continue;
                const float tt = omega * s * half * __builtin_amdgcn_rcpf(Wm);
#pragma unroll
                for (int k = 0; k < 3; ++k) g[k] = tt * lm[k];
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                acc[k * 3 + axis] += g[k];
                acc[k * 3 + 2] -= g[k] * ndc;
            }
        }
        }
        // colour weights last: keeps their registers out of the pair loop's live range
        float lam[3];
        if (!(AB & 2) && fast_lambda(rec(), multi, fEp[0] * iw0, fEp[1] * iw1, fEp[2] * iw2, lam)) {
            float Gm[CM];
#pragma unroll
            for (int c = 0; c < CM; ++c) Gm[c] = c < C ? s_G[kme * CP + c] : 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                for (int c = 0; c < C; ++c) acc[9 + k * C + c] = lam[k] * Gm[c];
        }
    }
    if (AB & 4) {
        float z = 0.0f;
#pragma unroll
        for (int v = 0; v < NVM; ++v) z += acc[v];
        if (z == 1234.5f) grad_verts[t] = z;  // keep the contributions live
        return;
    }

    // ---- phase C: segmented sum over runs of equal key along each 16-lane row (one DPP row); the
    // run tails store their partial sums with plain LDS writes into their slot's contiguous range
    // (sized in phase A by counting run heads; LDS float atomics serialise on shared addresses); tails
    // without a slot (table full) or past the partial buffer add straight to global memory
    const int key = rp >= 0 ? rp : -1;
    const int start = run_start(key, lx);
    // 0/1 multipliers: x += shifted(x) * m is one v_fmac with a DPP operand (exact: m is 0 or 1,
    // contributions are finite)
    const float mk1 = lx - 1 >= start ? 1.0f : 0.0f, mk2 = lx - 2 >= start ? 1.0f : 0.0f;
    const float mk4 = lx - 4 >= start ? 1.0f : 0.0f, mk8 = lx - 8 >= start ? 1.0f : 0.0f;
    if (!(AB & 32)) {
        // step-major order: each v_fmac_f32_dpp reads a register written >= NVM-1 instructions
        // earlier (no DPP read-after-write hazard inside the asm)
        asm volatile("s_nop 1");  // the accumulators may have been written by the last VALU ops
#pragma unroll
        for (int v = 0; v < NVM; ++v) asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:1 bound_ctrl:0" : "+v"(acc[v]) : "v"(mk1));
#pragma unroll
        for (int v = 0; v < NVM; ++v) asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:2 bound_ctrl:0" : "+v"(acc[v]) : "v"(mk2));
#pragma unroll
        for (int v = 0; v < NVM; ++v) asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:4 bound_ctrl:0" : "+v"(acc[v]) : "v"(mk4));
#pragma unroll
        for (int v = 0; v < NVM; ++v) asm volatile("v_fmac_f32_dpp %0, %0, %1 row_shr:8 bound_ctrl:0" : "+v"(acc[v]) : "v"(mk8));
    }
    const int kr = dpp_shl_i<1>(key, -3);
    const bool tail = key >= 0 && ((AB & 32) || lx == 15 || kr != key);
    float *gvb = grad_verts + (int64_t)b * V * 4;
    float *gcb = grad_colors + (int64_t)b * V * C;
    __syncthreads();  // every read of s_G / s_I is done: the union now holds tail partials
    PHASE_TS(5);
    int q = -1;
    if (tail && sp >= 0) {
        q = atomicAdd(&s_toff[sp], 1);  // the next place in the slot's range
        if (q >= kTailCap) q = -1;
    }
    if (tail) {
        if (q >= 0) {
#pragma unroll
            for (int v = 0; v < NVM; ++v)
                if (v < NV) s_part[q * NVM + v] = acc[v];
        } else {
            const FaceData &fd = fdata_frame[face_of_record(rp, F)];
            const int32_t vid[3] = {fd.v[0], fd.v[1], fd.v[2]};  // before the atomics (may alias for the compiler)
#pragma unroll
            for (int v = 0; v < NVM; ++v) {
                if (v >= NV || acc[v] == 0.0f) continue;
                if (v < 9) atomicAdd(gvb + (int64_t)vid[v / 3] * 4 + ((v % 3) == 2 ? 3 : v % 3), acc[v]);
                else atomicAdd(gcb + (int64_t)vid[(v - 9) / C] * C + (v - 9) % C, acc[v]);
            }
        }
    }
    __syncthreads();
    PHASE_TS(6);

    // ---- phase D: flush.  Thread t handles component t % NV of slot t / NV, so every lane of the
    // workgroup sums one slot's tails in parallel; a slot's components go out as one run of lanes
    // (~3 cache lines of global float atomics per (tile, record)).
    const int n = (AB & 8) ? 0 : nslots;
    const int per_round = 256 / NV;
    for (int e0 = 0; e0 < n; e0 += per_round) {
        const int e = e0 + t / NV, comp_id = t - (t / NV) * NV;
        if (t >= per_round * NV || e >= n) continue;
        const int kv = comp_id < 9 ? comp_id / 3 : (comp_id - 9) / C;
        const int vid = T.v[kv][e];
        // the record's tails are contiguous: four reads in flight per step
        const int beg = s_lbeg[e], hi = min(beg + s_lcnt[e], kTailCap);
        float val = 0.0f;
        for (int q0 = beg; q0 < hi; q0 += 4) {
            float a[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int qq = q0 + u;
                const float x = s_part[min(qq, hi - 1) * NVM + comp_id];
                a[u] = qq < hi ? x : 0.0f;
            }
            val += (a[0] + a[1]) + (a[2] + a[3]);
        }
        if (val == 0.0f) continue;
        if (AB & 256) {  // ablation: sums without the global atomics
            if (val == 12345.f) grad_verts[0] = val;
            continue;
        }
        if (comp_id < 9) {
            const int c3 = comp_id % 3;
            atomicAdd(gvb + (int64_t)vid * 4 + (c3 == 2 ? 3 : c3), val);
        } else {
            atomicAdd(gcb + (int64_t)vid * C + (comp_id - 9) % C, val);
        }
    }
    if (AB & 128) {
        __syncthreads();
        PHASE_TS(7);
    }
}

// zero two float arrays in one launch (the backward's atomically accumulated outputs)
__global__ __launch_bounds__(256) void zero2_kernel(float *__restrict__ a, int64_t na, float *__restrict__ b, int64_t nb)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // 16-B stores over a 16-B aligned buffer (torch allocations), scalar stores otherwise; then the tail
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t na4 = (reinterpret_cast<uintptr_t>(a) & 15) == 0 ? na / 4 : 0;
    const int64_t nb4 = (reinterpret_cast<uintptr_t>(b) & 15) == 0 ? nb / 4 : 0;
    for (int64_t k = gid; k < na4; k += stride) reinterpret_cast<float4 *>(a)[k] = z;
    for (int64_t k = na4 * 4 + gid; k < na; k += stride) a[k] = 0.0f;
    for (int64_t k = gid; k < nb4; k += stride) reinterpret_cast<float4 *>(b)[k] = z;
    for (int64_t k = nb4 * 4 + gid; k < nb; k += stride) b[k] = 0.0f;
}

// PMC calibration (tools/pmc_calibrate.py): read `n` elements of W bytes once each, coalesced, with the
// access widths the product kernels use, so FETCH_SIZE can be converted to bytes per width
template <int W>
__global__ __launch_bounds__(256) void read_bytes_kernel(const char *__restrict__ src, int64_t n, float *out)
{
    float acc = 0.0f;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const char *p = src + e * W;
        if (W == 4) acc += *reinterpret_cast<const float *>(p);
        if (W == 12) {
            const float *q = reinterpret_cast<const float *>(p);
            acc += q[0] + q[1] + q[2];
        }
        if (W == 16) {
            const float4 q = *reinterpret_cast<const float4 *>(p);
            acc += q.x + q.y + q.z + q.w;
        }
    }
    if (acc == 1.2345e-30f) out[0] = acc;  // keep the loads
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

int dirt_abi_version(void) { return 6; }

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

}  // extern "C"

// the forward of every op; tcb = channels of `background` (== C except for hill's terrain lookup)
static int rasterise_fwd_impl(const float *background, int tcb, const float *vertices, const float *vertex_colors,
                              const int32_t *faces, const float *camera_pos, int B, int H, int W, int C, int V, int F,
                              int shader_id, float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes,
                              void *scratch, size_t scratch_bytes, int64_t bin_capacity, unsigned flags,
                              float *zero_grad_vertices, float *zero_grad_vertex_colors, void *stream_)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (shader_id < DIRT_SHADER_GOURAUD || shader_id > DIRT_SHADER_HILL)
        return fail(DIRT_EINVAL, "Rasterise: unsupported shader_id");
    if (shader_id != DIRT_SHADER_GOURAUD && !camera_pos)
        return fail(DIRT_EINVAL, "Rasterise: procedural fragment programs need camera_pos");
    if (shader_id == DIRT_SHADER_HILL && tcb != 1 && tcb != 3 && tcb != 4)
        return fail(DIRT_EINVAL, "Hill: the terrain lookup must have 1, 3 or 4 channels");
    if (B == 0) return DIRT_OK;
    const bool need_colors = shader_id == DIRT_SHADER_GOURAUD;
    if (!background || !pixels || !gbuffer || !saved || !scratch || (F > 0 && (!faces || !vertices)) ||
        (V > 0 && (!vertices || (need_colors && !vertex_colors))))
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
    uint8_t *covbits = reinterpret_cast<uint8_t *>(sv + L.saved_cov);
    uint32_t *ccount = reinterpret_cast<uint32_t *>(sc + L.off_count);
    uint32_t *flag = reinterpret_cast<uint32_t *>(sc + L.off_flag);
    uint2 *bins = reinterpret_cast<uint2 *>(sc + L.off_bins);

    // count sets and parity words: one memset, unless the caller vouches that the scratch is clean
    // (DIRT_FWD_SCRATCH_CLEAN: zeroed once and since used only by forwards of the same layout)
    if (!(flags & DIRT_FWD_SCRATCH_CLEAN)) HIP_TRY(hipMemsetAsync(ccount, 0, L.off_bins - L.off_count, stream));
    if (F > 0) {
        ProfScope ps(K_SETUP, stream);
        launch_setup<0>(vertices, faces, B, H, W, V, F, L, recs, fdata, ccount, flag, bins, stream, zero_grad_vertices,
                        (int64_t)B * V * 4, zero_grad_vertex_colors, (int64_t)B * V * C);
        HIP_TRY(hipGetLastError());
        // (the setup grid's filler workgroups zero the accumulators; the raster does it only when F == 0)
        zero_grad_vertices = nullptr;
        zero_grad_vertex_colors = nullptr;
    }
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
    ProfScope ps(K_RASTER, stream);
#define LAUNCH_PROC(CC, SHT)                                                                                     \
    raster_kernel<CC, 0, SHT><<<grid, dim3(256), 0, stream>>>(                                                   \
        background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F,                     \
        tile_grid(L.ntx),                                                                                                     \
        L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                         \
        zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                      \
        zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb)
#define LAUNCH_RASTER(CC)                                                                                        \
    if (shader_id == DIRT_SHADER_OCEANIC_HORIZON)                                                                \
        LAUNCH_PROC(CC, DIRT_SHADER_OCEANIC_HORIZON);                                                            \
    else if (shader_id == DIRT_SHADER_HILL)                                                                      \
        LAUNCH_PROC(CC, DIRT_SHADER_HILL);                                                                       \
    else if (shader_id >= DIRT_SHADER_OCEANIC)                                                                   \
        LAUNCH_PROC(CC, DIRT_SHADER_OCEANIC);                                                                    \
    else                                                                                                         \
    raster_kernel<CC><<<grid, dim3(256), 0, stream>>>(background, vertex_colors, recs, fdata, ccount, flag,       \
                                                      bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx),                     \
                                                      L.cshift,                                                  \
                                                      L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits,          \
                                                      zero_grad_vertices,                                          \
                                                      zero_grad_vertices ? (int64_t)B * V * 4 : 0,                 \
                                                      zero_grad_vertex_colors,                                     \
                                                      zero_grad_vertex_colors ? (int64_t)B * V * C : 0,            \
                                                      vertices, camera_pos, shader_id, tcb)
    if (C == 1) LAUNCH_RASTER(1);
    else if (C == 3) LAUNCH_RASTER(3);
    else if (C == 7) LAUNCH_RASTER(7);
    else LAUNCH_RASTER(0);
#undef LAUNCH_RASTER
#undef LAUNCH_PROC
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

extern "C" {

int dirt_rasterise_fwd(const float *background, const float *vertices, const float *vertex_colors,
                       const int32_t *faces, const float *camera_pos, int B, int H, int W, int C, int V, int F,
                       int shader_id, float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes, void *scratch,
                       size_t scratch_bytes, int64_t bin_capacity, unsigned flags, float *zero_grad_vertices,
                       float *zero_grad_vertex_colors, void *stream_)
{
    return rasterise_fwd_impl(background, C, vertices, vertex_colors, faces, camera_pos, B, H, W, C, V, F, shader_id,
                              pixels, gbuffer, saved, saved_bytes, scratch, scratch_bytes, bin_capacity, flags,
                              zero_grad_vertices, zero_grad_vertex_colors, stream_);
}

int dirt_hill_fwd(const float *terrain, int terrain_channels, const float *vertices, const int32_t *faces,
                  const float *camera_pos, int B, int H, int W, int C, int V, int F, float *pixels, int32_t *gbuffer,
                  void *saved, size_t saved_bytes, void *scratch, size_t scratch_bytes, int64_t bin_capacity,
                  void *stream_)
{
    return rasterise_fwd_impl(terrain, terrain_channels, vertices, nullptr, faces, camera_pos, B, H, W, C, V, F,
                              DIRT_SHADER_HILL, pixels, gbuffer, saved, saved_bytes, scratch, scratch_bytes,
                              bin_capacity, 0u, nullptr, nullptr, stream_);
}

static NdcScale ndc_scale(int W, int H)
{
    return NdcScale{2.0f / (float)W, 2.0f / (float)H, 0.5f * (float)W, 0.5f * (float)H};
}

int dirt_rasterise_bwd(const float *vertices, const float *vertex_colors, const int32_t *faces, const float *pixels,
                       const float *grad_pixels, const int32_t *gbuffer, const void *saved, int B, int H, int W, int C,
                       int V, int F, float *grad_vertices, float *grad_vertex_colors, float *grad_background,
                       unsigned flags, void *stream_)
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
    const uint8_t *covbits = reinterpret_cast<const uint8_t *>(sv + L.saved_cov);
    if (V > 0 && !(flags & DIRT_BWD_ACCUMULATE)) {
        const int64_t na = (int64_t)B * V * 4, nb = (int64_t)B * V * C;
        const int64_t blocks = std::min<int64_t>(2048, (na / 4 + 255) / 256 + 1);
        zero2_kernel<<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(grad_vertices, na, grad_vertex_colors, nb);
        HIP_TRY(hipGetLastError());
    }
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
    ProfScope ps(K_GRAD, stream);
#define LAUNCH_GRAD(CC)                                                                                       \
    grad_kernel<CC><<<grid, dim3(256), 0, stream>>>(pixels, grad_pixels, gbuffer, covbits, recs, fdata, B, H, W, C, \
                                                    V, F,                                                        \
                                                    tile_grid(L.ntx), L.nrec, grad_vertices, grad_vertex_colors,            \
                                                    grad_background, ndc_scale(W, H))
    if (C == 1) LAUNCH_GRAD(1);
    else if (C == 3) LAUNCH_GRAD(3);
    else if (C == 7) LAUNCH_GRAD(7);
    else LAUNCH_GRAD(0);
#undef LAUNCH_GRAD
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

// Ablation entry point (tools/ablate.py): re-runs raster_kernel (C == 3) on the bins a preceding
// dirt_rasterise_fwd left in `scratch`, with parts switched off; returns the kernel time in ms.
int dirt_debug_raster_variant(int variant, const float *background, const float *vertices, const float *vertex_colors,
                              const int32_t *faces, int B, int H, int W, int C, int V, int F, float *pixels,
                              int32_t *gbuffer, void *saved, void *scratch, void *stream_, float *ms)
{
    if (C != 3) return fail(DIRT_EINVAL, "dirt_debug_raster_variant: C must be 3");
    Layout L;
    int rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    char *sv = static_cast<char *>(saved), *sc = static_cast<char *>(scratch);
    Rec *recs = reinterpret_cast<Rec *>(sv + L.saved_recs);
    FaceData *fdata = reinterpret_cast<FaceData *>(sv + L.saved_fdata);
    uint8_t *covbits = reinterpret_cast<uint8_t *>(sv + L.saved_cov);
    uint32_t *ccount = reinterpret_cast<uint32_t *>(sc + L.off_count);
    uint32_t *flag = reinterpret_cast<uint32_t *>(sc + L.off_flag);
    uint2 *bins = reinterpret_cast<uint2 *>(sc + L.off_bins);
    // re-bin from a clean scratch, then time the raster variant alone
    HIP_TRY(hipMemsetAsync(ccount, 0, L.off_bins - L.off_count, stream));
    if (F > 0) launch_setup<0>(vertices, faces, B, H, W, V, F, L, recs, fdata, ccount, flag, bins, stream);
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, stream));
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
#define V_RAST(AB)                                                                                                 \
    case AB:                                                                                                       \
        raster_kernel<3, AB><<<grid, dim3(256), 0, stream>>>(background, vertex_colors, recs, fdata, ccount, flag,    \
                                                             bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), L.cshift,         \
                                                             L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits,     \
                                                             nullptr, 0,                                              \
                                                             nullptr, 0, nullptr, nullptr, 0, C);                    \
        break
    switch (variant) {
        V_RAST(0); V_RAST(1); V_RAST(2); V_RAST(4); V_RAST(8); V_RAST(32); V_RAST(64); V_RAST(96); V_RAST(128);
    default:
        return fail(DIRT_EINVAL, "dirt_debug_raster_variant: unknown variant");
    }
#undef V_RAST
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, stream));
    HIP_TRY(hipEventSynchronize(e1));
    HIP_TRY(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return DIRT_OK;
}

// Instrumented setup (tools/setup_ts.py): clean scratch, one setup_kernel<128> launch, its time in ms;
// per-workgroup phase timestamps land in g_phase_ts (dirt_debug_read_phase_ts).
// variant 0: timestamps, 1: timestamps without the slab reservation atomics, 2 / 3: the same untimestamped
int dirt_debug_setup_ts(int variant, const float *vertices, const int32_t *faces, int B, int H, int W, int V, int F,
                        void *saved, void *scratch, void *stream_, float *ms)
{
    Layout L;
    int rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    char *sv = static_cast<char *>(saved), *sc = static_cast<char *>(scratch);
    Rec *recs = reinterpret_cast<Rec *>(sv + L.saved_recs);
    FaceData *fdata = reinterpret_cast<FaceData *>(sv + L.saved_fdata);
    uint32_t *ccount = reinterpret_cast<uint32_t *>(sc + L.off_count);
    uint32_t *flag = reinterpret_cast<uint32_t *>(sc + L.off_flag);
    uint2 *bins = reinterpret_cast<uint2 *>(sc + L.off_bins);
    HIP_TRY(hipMemsetAsync(ccount, 0, L.off_bins - L.off_count, stream));
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, stream));
    switch (variant) {
#define V_SETUP(K, AB)                                                                                        \
    case K:                                                                                                   \
        launch_setup<AB>(vertices, faces, B, H, W, V, F, L, recs, fdata, ccount, flag, bins, stream);         \
        break
        V_SETUP(0, 128); V_SETUP(1, 129); V_SETUP(2, 0); V_SETUP(3, 1);
#undef V_SETUP
    default:
        return fail(DIRT_EINVAL, "dirt_debug_setup_ts: unknown variant");
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, stream));
    HIP_TRY(hipEventSynchronize(e1));
    HIP_TRY(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return DIRT_OK;
}

// Ablation entry point (tools/ablate.py): the backward with parts of grad_kernel switched off.
// Not part of include/dirt_mi355x.h; C == 3 only.  Returns the kernel time in ms (hipEvents).
int dirt_debug_bwd_variant(int variant, const float *pixels, const float *grad_pixels, const int32_t *gbuffer,
                           const void *saved, int B, int H, int W, int C, int V, int F, float *grad_vertices,
                           float *grad_vertex_colors, float *grad_background, void *stream_, float *ms)
{
    if (C != 3) return fail(DIRT_EINVAL, "dirt_debug_bwd_variant: C must be 3");
    Layout L;
    int rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const char *sv = static_cast<const char *>(saved);
    const Rec *recs = reinterpret_cast<const Rec *>(sv + L.saved_recs);
    const FaceData *fdata = reinterpret_cast<const FaceData *>(sv + L.saved_fdata);
    const uint8_t *covbits = reinterpret_cast<const uint8_t *>(sv + L.saved_cov);
    HIP_TRY(hipMemsetAsync(grad_vertices, 0, (size_t)B * V * 4 * sizeof(float), stream));
    HIP_TRY(hipMemsetAsync(grad_vertex_colors, 0, (size_t)B * V * C * sizeof(float), stream));
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, stream));
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
#define V_GRAD(AB)                                                                                                   \
    case AB:                                                                                                         \
        grad_kernel<3, AB><<<grid, dim3(256), 0, stream>>>(pixels, grad_pixels, gbuffer, covbits, recs, fdata, B, H, W,\
                                                           C, V,                                                     \
                                                           F, tile_grid(L.ntx), L.nrec, grad_vertices, grad_vertex_colors,     \
                                                           grad_background, ndc_scale(W, H));                        \
        break
    switch (variant) {
        V_GRAD(0); V_GRAD(1); V_GRAD(2); V_GRAD(3); V_GRAD(4); V_GRAD(5); V_GRAD(8); V_GRAD(16); V_GRAD(7);
        V_GRAD(32); V_GRAD(64); V_GRAD(72); V_GRAD(128); V_GRAD(256);
    default:
        return fail(DIRT_EINVAL, "dirt_debug_bwd_variant: unknown variant");
    }
#undef V_GRAD
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, stream));
    HIP_TRY(hipEventSynchronize(e1));
    HIP_TRY(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return DIRT_OK;
}

int dirt_debug_read_bytes(int width, const void *src, size_t bytes, float *out, void *stream_)
{
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    if (width != 4 && width != 12 && width != 16) return fail(DIRT_EINVAL, "dirt_debug_read_bytes: width 4, 12 or 16");
    const int64_t n = (int64_t)(bytes / (size_t)width);
    const dim3 grid(2048), block(256);
    if (width == 4) read_bytes_kernel<4><<<grid, block, 0, stream>>>(static_cast<const char *>(src), n, out);
    if (width == 12) read_bytes_kernel<12><<<grid, block, 0, stream>>>(static_cast<const char *>(src), n, out);
    if (width == 16) read_bytes_kernel<16><<<grid, block, 0, stream>>>(static_cast<const char *>(src), n, out);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

// copy the phase timestamps of the last instrumented backward (variant 128): 10 words per workgroup (8 timestamps, HW_ID, XCC_ID)
int dirt_debug_read_phase_ts(uint64_t *host, int nwg)
{
    if (nwg < 0 || nwg > kTsMaxWG) return fail(DIRT_EINVAL, "dirt_debug_read_phase_ts: bad count");
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase_ts), (size_t)nwg * kTsStride * sizeof(uint64_t), 0,
                                hipMemcpyDeviceToHost));
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

int dirt_scratch_clear(int B, int H, int W, int F, int64_t bin_capacity, void *scratch, size_t scratch_bytes,
                       void *stream_)
{
    if (B < 0 || F < 0 || H <= 0 || W <= 0 || H > DIRT_MAX_DIM || W > DIRT_MAX_DIM)
        return fail(DIRT_EINVAL, "dirt_scratch_clear: bad sizes");
    if (B == 0) return DIRT_OK;
    Layout L;
    const int rc = make_layout(B, H, W, F, bin_capacity, L);
    if (rc) return rc;
    if (!scratch || scratch_bytes < L.scratch_total)
        return fail(DIRT_EINVAL, "dirt_scratch_clear: scratch smaller than dirt_workspace_sizes()");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    HIP_TRY(hipMemsetAsync(static_cast<char *>(scratch) + L.off_count, 0, L.off_bins - L.off_count, stream));
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
