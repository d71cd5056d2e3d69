// dirt_raster.hip -- MI355X (gfx950) software rasteriser behind the C ABI of include/dirt_mi355x.h.
//
// CDNA4 has no graphics pipeline, so the reference's GL fixed-function raster
// (csrc/rasterise_egl.cpp:440-487 + the NVIDIA driver) becomes a compute pipeline of three launches:
//
//   K1 setup_kernel    (setup_kernel.h) one thread per (frame, face): fetch 3 clip vertices, project +
//                      snap (R1/R2), edge equations (R3), depth plane (R4), guard-band clipping (R5, rare
//                      slow path); writes 128-B setup records + 32-B FaceData; counts its (coarse tile,
//                      record) pairs in LDS, reserves its range of every touched coarse-tile slab with one
//                      returning device atomic per (workgroup, tile) and writes the 8-B bin entries there.
//                      Filler workgroups past the faces zero the caller's gradient accumulators.
//   K4 raster_kernel   (raster_kernel.h) one 256-thread workgroup per 16x16 tile (a wave per 8x8 block):
//                      reads its coarse slab once, stages the tile's survivors in LDS with tile-relative
//                      32-bit edge values (exact), each lane owns one pixel and keeps the min
//                      (depth24<<32 | face) key over its wave's entry list (long lists depth-culled), then
//                      resolves in-kernel: perspective-correct Gouraud colour (R6) or background, coalesced
//                      [B,H,W,C] writes + the int32 g-buffer + neighbour-coverage bits.  This fuses the
//                      reference's upload_background + raster + second pass + download_pixels
//                      (csrc/rasterise_egl.cu:16-129, rasterise_egl.cpp:370-503) into one HBM pass.
//   K5 grad_kernel     (grad_kernel.h) backward: dL/dbackground, dL/dvertex_colors and the
//                      filter-based dL/dvertices (README.md:146-147) for the gradient contract of
//                      csrc/rasterise_grad_common.h:19-24.
//
// This file holds the shared device helpers, the scratch layout, validation, launches and the C ABI; the
// three kernels live in the headers named above, included into this one translation unit.

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <mutex>
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
#ifndef DIRT_BIN_THREADS
#define DIRT_BIN_THREADS 256
#endif
constexpr int kBinThreads = DIRT_BIN_THREADS;
// entries (4 GiB of the 288 GB HBM) above which the default slab shrinks: B = 64 frames of 1024^2 and 20k faces
// (config 5 on one GPU) keep the full F + F/4 + 64 per slab, so a mesh crowded into a few coarse tiles does
// not send them to the overflow path (dirt_debug_bin_occupancy reports the fullest slab)
constexpr int64_t kDefaultBinBudget = 1ll << 29;
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

#include "setup_kernel.h"
#include "raster_kernel.h"
#include "grad_kernel.h"
#include "lighting_kernels.h"

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

// ---- gradient stash of the single-output op (header words: setup_kernel.h kStash*)
struct StashDims {
    uint32_t d[5];  // B, H, W, V, F
};

// words of a and b equal?  (16-B loads when both are 16-B aligned, the tail and misaligned buffers by words)
__device__ __forceinline__ bool words_differ(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b, int64_t n,
                                             int64_t gid, int64_t gs)
{
    bool diff = false;
    const bool vec = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
    const int64_t n4 = vec ? n / 4 : 0;
    for (int64_t k = gid; k < n4; k += gs) {
        const uint4 x = reinterpret_cast<const uint4 *>(a)[k], y = reinterpret_cast<const uint4 *>(b)[k];
        diff = diff || x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
    }
    for (int64_t k = 4 * n4 + gid; k < n; k += gs) diff = diff || a[k] != b[k];
    return diff;
}

// Does the workspace hold the records of exactly this geometry?  Bitwise comparison of vertices and faces with the
// copies the last forward-stash or recompute left (the records, g-buffer and coverage bits are a deterministic
// function of those bits and the frame size), plus the header's magic and dims.  Any difference sets this call's
// miss flag; the next call's flag is zeroed here (nothing reads it in this call).
__global__ __launch_bounds__(256) void stash_check_kernel(const uint32_t *__restrict__ v, const uint32_t *__restrict__ vt,
                                                          int64_t nv, const uint32_t *__restrict__ f,
                                                          const uint32_t *__restrict__ ft, int64_t nf, uint32_t *hdr,
                                                          StashDims dims)
{
    const uint32_t p = hdr[kStashP] & 1u;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
    bool miss = words_differ(v, vt, nv, gid, gs) || words_differ(f, ft, nf, gid, gs);
    if (gid == 0) {
        hdr[kStashMiss + 16 * (p ^ 1u)] = 0u;
        miss = miss || hdr[kStashMagicW] != kStashMagic;
        for (int k = 0; k < 5; ++k) miss = miss || hdr[kStashDims + k] != dims.d[k];
    }
    if (__ballot(miss) != 0 && (threadIdx.x & 63) == 0) atomicOr(&hdr[kStashMiss + 16 * p], 1u);
}

// zero n bytes (a multiple of 4, 4-B aligned) with a kernel: the scratch / stash clears run inside HIP graphs that
// the public op captures, and a kernel node is ordered like every other kernel of the graph
__global__ __launch_bounds__(256) void zero_words_kernel(uint32_t *__restrict__ p, int64_t n)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) p[k] = 0u;
}

__global__ void stash_flip_kernel(uint32_t *p)
{
    if (threadIdx.x == 0) p[0] ^= 1u;
}

// zero `bytes` (multiple of 4) at p on `stream` with zero_words_kernel
int zero_async(void *p, size_t bytes, hipStream_t stream)
{
    const int64_t n = (int64_t)(bytes / 4);
    if (n == 0) return DIRT_OK;
    const unsigned blocks = (unsigned)std::min<int64_t>(1024, (n + 255) / 256);
    zero_words_kernel<<<dim3(blocks), dim3(256), 0, stream>>>(static_cast<uint32_t *>(p), n);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}


// After a recomputation (this call's miss flag set), or unconditionally for a forward-stash (`force`): record the
// geometry the workspace now holds.
__global__ __launch_bounds__(256) void stash_update_kernel(const uint32_t *__restrict__ v, uint32_t *__restrict__ vt,
                                                           int64_t nv, const uint32_t *__restrict__ f,
                                                           uint32_t *__restrict__ ft, int64_t nf, uint32_t *hdr,
                                                           StashDims dims, int force)
{
    if (!force && stash_hit(hdr)) return;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = gid; k < nv; k += gs) vt[k] = v[k];
    for (int64_t k = gid; k < nf; k += gs) ft[k] = f[k];
    if (gid == 0) {
        hdr[kStashMagicW] = kStashMagic;
        for (int k = 0; k < 5; ++k) hdr[kStashDims + k] = dims.d[k];
    }
}

}  // namespace

// ================================================================================================
// C ABI

extern "C" {

int dirt_abi_version(void) { return 13; }

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

// Automatic deep-scene culling: the Gouraud raster counts its long per-wave entry lists
// (raster_kernel deep_host) into one of two count slots of its scratch's flag area, and the next launch on the same
// scratch reports whether that count made the previous launch deep, by writing the previous launch's generation into
// a host-mapped word per device, then clears that slot.  A forward takes the occluder-culling instantiation (OCC)
// when a launch within the last kDeepRecent generations was deep: a deep scene switches after one launch (plus the
// queue's lag), a scene turning shallow switches back after kDeepRecent.  Both instantiations are exact, so the
// choice changes time only.  DIRT_FWD_DEEP_CULL forces OCC, DIRT_FWD_DEEP_CULL_OFF the plain raster;
// DIRT_DEEP_CULL_AUTO=0 disables the rule.
// Per scratch, the host remembers the generation and count slot of the last launch on it, so
// launches on several scratches interleaved on one device (two layouts, streams or sessions) each report their own
// previous launch; a launch counts into the slot its predecessor on that scratch did not use.  A launch captured
// into a graph neither counts nor reports (its instantiation is fixed at capture; replays would re-count into one
// slot forever), and the word is allocated outside any capture (relaxed capture mode, so another
// thread's global-mode capture is not invalidated by the host allocation).
constexpr uint32_t kDeepRecent = 8;
struct DeepScratch {
    const void *flag = nullptr;  // the scratch's flag area (identifies the scratch)
    uint32_t gen = 0;            // generation of the last launch on it
    uint32_t slot = 0;           // the count slot that launch used
};
constexpr int kDeepScratches = 64;
struct DeepAuto {
    uint32_t *host = nullptr;  // host-mapped word: generation of the last launch reported deep (0 = none)
    uint32_t *dev = nullptr;   // its device address
    uint32_t gen = 0;          // launches issued with the rule on
    DeepScratch scr[kDeepScratches];  // recently used scratches (round-robin replacement)
    int next = 0;
};
static std::mutex g_deep_mu;
static DeepAuto g_deep[64];

static bool deep_auto_enabled()
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("DIRT_DEEP_CULL_AUTO");
        v = (e && *e) ? (atoi(e) != 0) : 1;
    }
    return v != 0;
}

// the device's state with its word allocated (nullptr: rule off or the allocation failed)
static DeepAuto *deep_auto_state()
{
    if (!deep_auto_enabled()) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    DeepAuto &d = g_deep[dev];
    std::lock_guard<std::mutex> lk(g_deep_mu);
    if (d.host) return &d;
    // (relaxed capture mode for this thread: a host allocation is an unsafe call while any stream captures in
    // global mode, torch.cuda.graph's default)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    void *h = nullptr, *dp = nullptr;
    bool ok = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
    if (ok && hipHostGetDevicePointer(&dp, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        ok = false;
    }
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (!ok) return nullptr;
    static_cast<volatile uint32_t *>(h)[0] = 0u;
    d.dev = static_cast<uint32_t *>(dp);
    d.host = static_cast<uint32_t *>(h);
    return &d;
}

// the record of `flag`'s scratch (created on first use: no previous launch, generation 0); g_deep_mu held
static DeepScratch &deep_scratch(DeepAuto &d, const void *flag)
{
    for (DeepScratch &e : d.scr)
        if (e.flag == flag) return e;
    DeepScratch &e = d.scr[d.next];
    d.next = (d.next + 1) % kDeepScratches;
    e = DeepScratch{flag, 0u, 0u};
    return e;
}

// the forward of every op; tcb = channels of `background` (== C except for hill's terrain lookup)
static int rasterise_fwd_impl(const float *background, int tcb, const float *vertices, const float *vertex_colors,
                              const int32_t *faces, const float *camera_pos, int B, int H, int W, int C, int V, int F,
                              int shader_id, float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes,
                              void *scratch, size_t scratch_bytes, int64_t bin_capacity, unsigned flags,
                              float *zero_grad_vertices, float *zero_grad_vertex_colors, void *stream_,
                              GbufOut gbo = GbufOut{}, bool nopix = false, const uint32_t *stash_hdr = nullptr)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    const bool want_gb = gbo.depth || gbo.bary || gbo.face;
    if (want_gb && shader_id != DIRT_SHADER_GOURAUD)
        return fail(DIRT_EINVAL, "Rasterise: depth / barycentric / face outputs are produced by the Gouraud program only");
    if (shader_id < DIRT_SHADER_GOURAUD || shader_id > DIRT_SHADER_HILL)
        return fail(DIRT_EINVAL, "Rasterise: unsupported shader_id");
    if (shader_id != DIRT_SHADER_GOURAUD && !camera_pos)
        return fail(DIRT_EINVAL, "Rasterise: procedural fragment programs need camera_pos");
    if (shader_id == DIRT_SHADER_HILL && tcb != 1 && tcb != 3 && tcb != 4)
        return fail(DIRT_EINVAL, "Hill: the terrain lookup must have 1, 3 or 4 channels");
    if (B == 0) return DIRT_OK;
    if (nopix && (shader_id != DIRT_SHADER_GOURAUD || want_gb))
        return fail(DIRT_EINVAL, "Rasterise: the coverage-only pass is Gouraud without G-buffer outputs");
    // (nopix: the coverage-only pass of dirt_rasterise_bwd_recompute reads no background or colours)
    const bool need_colors = shader_id == DIRT_SHADER_GOURAUD && !nopix;
    if ((!nopix && (!background || !pixels)) || !gbuffer || !saved || !scratch || (F > 0 && (!faces || !vertices)) ||
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
    if (!(flags & DIRT_FWD_SCRATCH_CLEAN)) {
        rc = zero_async(ccount, L.off_bins - L.off_count, stream);
        if (rc) return rc;
    }
    // small scenes (Gouraud, F <= kFusedMaxF, at most kFusedMaxTiles tiles): the raster sets up the faces itself
    // (one launch, no bins)
    const bool fused = shader_id == DIRT_SHADER_GOURAUD && F > 0 && F <= kFusedMaxF &&
                       (int64_t)B * L.ntiles <= kFusedMaxTiles;
    // occluder culling of long per-wave entry lists (deep scenes, raster_kernel.h OCC): forced by DIRT_FWD_DEEP_CULL,
    // else automatic (DeepAuto) for the binned Gouraud forward
    bool deep = (flags & DIRT_FWD_DEEP_CULL) != 0 && shader_id == DIRT_SHADER_GOURAUD && !nopix;
    DeepArgs dga{};
    if (shader_id == DIRT_SHADER_GOURAUD && !nopix && !fused && !want_gb && F > 0 && !(flags & DIRT_FWD_DEEP_CULL_OFF)) {
        if (DeepAuto *da = deep_auto_state()) {
            // (a launch captured into a graph neither counts nor reports, nor does it advance the generation: it
            // does not execute now, and its replays keep the instantiation chosen here)
            hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
            const bool capturing = hipStreamIsCapturing(stream, &cst) == hipSuccess && cst != hipStreamCaptureStatusNone;
            std::lock_guard<std::mutex> lk(g_deep_mu);
            const uint32_t last = static_cast<volatile uint32_t *>(da->host)[0];
            const uint32_t next_gen = da->gen + 1u == 0u ? 1u : da->gen + 1u;  // (0 means "never deep")
            deep = deep || (last != 0u && next_gen - last <= kDeepRecent);
            if (!capturing) {
                da->gen = next_gen;
                DeepScratch &ds = deep_scratch(*da, flag);
                dga.host = da->dev;
                dga.gen = next_gen;
                dga.prev_gen = ds.gen;
                dga.slot = ds.slot ^ 1u;
                ds.gen = next_gen;
                ds.slot = dga.slot;
            }
        }
    }
    if (F > 0 && !fused) {
        ProfScope ps(K_SETUP, stream);
        launch_setup<0>(vertices, faces, B, H, W, V, F, L, recs, fdata, ccount, flag, bins, stream, zero_grad_vertices,
                        (int64_t)B * V * 4, zero_grad_vertex_colors, (int64_t)B * V * C, stash_hdr);
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
    else if (nopix && fused)                                                                                     \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, false, true, true><<<grid, dim3(256), 0, stream>>>(            \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, gbo, faces,    \
            stash_hdr);                                                                                          \
    else if (nopix)                                                                                              \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, false, false, true><<<grid, dim3(256), 0, stream>>>(           \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, gbo, nullptr,  \
            stash_hdr);                                                                                          \
    else if (deep && !fused && !want_gb)                                                                         \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, false, false, false, true><<<grid, dim3(256), 0, stream>>>(     \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, GbufOut{},      \
            nullptr, nullptr, dga);                                                                              \
    else if (fused && want_gb)                                                                                   \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, true, true><<<grid, dim3(256), 0, stream>>>(                   \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, gbo, faces);   \
    else if (fused)                                                                                              \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, false, true><<<grid, dim3(256), 0, stream>>>(                  \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, gbo, faces);   \
    else if (want_gb)                                                                                            \
        raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, true><<<grid, dim3(256), 0, stream>>>(                         \
            background, vertex_colors, recs, fdata, ccount, flag, bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx), \
            L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits, zero_grad_vertices,                     \
            zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                  \
            zero_grad_vertex_colors ? (int64_t)B * V * C : 0, vertices, camera_pos, shader_id, tcb, gbo);          \
    else                                                                                                         \
    raster_kernel<CC><<<grid, dim3(256), 0, stream>>>(background, vertex_colors, recs, fdata, ccount, flag,       \
                                                      bins, L.slab, B, H, W, C, V, F, tile_grid(L.ntx),                     \
                                                      L.cshift,                                                  \
                                                      L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, covbits,          \
                                                      zero_grad_vertices,                                          \
                                                      zero_grad_vertices ? (int64_t)B * V * 4 : 0,                 \
                                                      zero_grad_vertex_colors,                                     \
                                                      zero_grad_vertex_colors ? (int64_t)B * V * C : 0,            \
                                                      vertices, camera_pos, shader_id, tcb, GbufOut{}, nullptr,    \
                                                      nullptr, dga)
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

int dirt_rasterise_fwd_gbuffer(const float *background, const float *vertices, const float *vertex_colors,
                               const int32_t *faces, int B, int H, int W, int C, int V, int F, float *pixels,
                               int32_t *gbuffer, void *saved, size_t saved_bytes, void *scratch, size_t scratch_bytes,
                               int64_t bin_capacity, unsigned flags, float *zero_grad_vertices,
                               float *zero_grad_vertex_colors, float *depth, float *barycentrics, int32_t *face_ids,
                               void *stream_)
{
    return rasterise_fwd_impl(background, C, vertices, vertex_colors, faces, nullptr, B, H, W, C, V, F,
                              DIRT_SHADER_GOURAUD, pixels, gbuffer, saved, saved_bytes, scratch, scratch_bytes,
                              bin_capacity, flags, zero_grad_vertices, zero_grad_vertex_colors, stream_,
                              GbufOut{depth, barycentrics, face_ids});
}

// A render sharing its geometry with the earlier Gouraud forward that filled gbuffer_in / saved (ABI 13): the resolve
// alone, over this render's colours and background (raster_kernel RESOLVE)
int dirt_rasterise_fwd_resolve(const float *background, const float *vertex_colors, int B, int H, int W, int C, int V,
                               int F, const int32_t *gbuffer_in, const void *saved, size_t saved_bytes, float *pixels,
                               int32_t *gbuffer, float *zero_grad_vertices, float *zero_grad_vertex_colors, void *stream_)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (B == 0) return DIRT_OK;
    if (!background || !pixels || !gbuffer || !gbuffer_in || !saved || (V > 0 && !vertex_colors))
        return fail(DIRT_EINVAL, "RasteriseResolve: null tensor pointer");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    if (saved_bytes < L.saved_total) return fail(DIRT_EINVAL, "RasteriseResolve: saved smaller than dirt_workspace_sizes()");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const char *sv = static_cast<const char *>(saved);
    const Rec *recs = reinterpret_cast<const Rec *>(sv + L.saved_recs);
    const FaceData *fdata = reinterpret_cast<const FaceData *>(sv + L.saved_fdata);
    dim3 grid((unsigned)L.ntiles, (unsigned)B);
    ProfScope ps(K_RASTER, stream);
#define LAUNCH_RESOLVE(CC)                                                                                         \
    raster_kernel<CC, 0, DIRT_SHADER_GOURAUD, false, false, false, false, true><<<grid, dim3(256), 0, stream>>>(     \
        background, vertex_colors, recs, fdata, nullptr, nullptr, nullptr, 0u, B, H, W, C, V, F, tile_grid(L.ntx),   \
        L.cshift, L.nctx, L.ncoarse, L.nrec, pixels, gbuffer, nullptr, zero_grad_vertices,                        \
        zero_grad_vertices ? (int64_t)B * V * 4 : 0, zero_grad_vertex_colors,                                     \
        zero_grad_vertex_colors ? (int64_t)B * V * C : 0, nullptr, nullptr, DIRT_SHADER_GOURAUD, C, GbufOut{},      \
        nullptr, nullptr, DeepArgs{}, gbuffer_in)
    if (C == 1) LAUNCH_RESOLVE(1);
    else if (C == 3) LAUNCH_RESOLVE(3);
    else if (C == 7) LAUNCH_RESOLVE(7);
    else LAUNCH_RESOLVE(0);
#undef LAUNCH_RESOLVE
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
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

}  // extern "C"

// the backward of dirt_rasterise_bwd; stash_flip: the recompute workspace's stash parity (flipped by the launch)
static int rasterise_bwd_impl(const float *vertices, const float *vertex_colors, const int32_t *faces,
                              const float *pixels, const float *grad_pixels, const int32_t *gbuffer, const void *saved,
                              int B, int H, int W, int C, int V, int F, float *grad_vertices, float *grad_vertex_colors,
                              float *grad_background, unsigned flags, void *stream_, uint32_t *stash_flip)
{
    // vertices / vertex_colors / faces are part of the contract (rasterise_grad_common.h:19-24); the
    // forward's FaceData in `saved` already holds what the kernel needs from them.
    (void)vertex_colors;
    (void)vertices;
    (void)faces;
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (B == 0) return DIRT_OK;
    if (!pixels || !grad_pixels || !gbuffer || !saved || (V > 0 && !grad_vertices && !grad_vertex_colors))
        return fail(DIRT_EINVAL, "RasteriseGrad: null tensor pointer");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const char *sv = static_cast<const char *>(saved);
    const Rec *recs = reinterpret_cast<const Rec *>(sv + L.saved_recs);
    const FaceData *fdata = reinterpret_cast<const FaceData *>(sv + L.saved_fdata);
    const uint8_t *covbits = reinterpret_cast<const uint8_t *>(sv + L.saved_cov);
    // which gradients to produce: a null grad_vertices / grad_vertex_colors is not computed at all (GM bits)
    const int gm = (grad_vertices ? 1 : 0) | (grad_vertex_colors ? 2 : 0);
    if (V > 0 && !(flags & DIRT_BWD_ACCUMULATE)) {
        const int64_t na = grad_vertices ? (int64_t)B * V * 4 : 0, nb = grad_vertex_colors ? (int64_t)B * V * C : 0;
        const int64_t blocks = std::min<int64_t>(2048, (std::max(na, nb) / 4 + 255) / 256 + 1);
        zero2_kernel<<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(grad_vertices, na, grad_vertex_colors, nb);
        HIP_TRY(hipGetLastError());
    }
    if (gm == 0) {
        // V == 0 (no vertex or colour gradient exists): the launch still writes grad_background; the colour
        // path's instantiation with a null colour pointer has nothing to flush (every pixel is background)
        if (!grad_background) {
            if (stash_flip) {  // (no grad launch to flip the stash parity)
                stash_flip_kernel<<<dim3(1), dim3(64), 0, stream>>>(stash_flip);
                HIP_TRY(hipGetLastError());
            }
            return DIRT_OK;
        }
    }
    // backward tiles: kGradTileW x grad_tile_h(C) (grad_kernel.h)
    const int gntx = (W + kGradTileW - 1) / kGradTileW, gnty = (H + grad_tile_h(C) - 1) / grad_tile_h(C);
    dim3 grid((unsigned)(gntx * gnty), (unsigned)B);
    ProfScope ps(K_GRAD, stream);
#define LAUNCH_GRAD_GM(CC, GMV)                                                                              \
    grad_kernel<CC, 0, kGradTileW, grad_tile_h(CC), GMV><<<grid, dim3(GradGeom<kGradTileW, grad_tile_h(CC)>::NT), 0, \
                                                          stream>>>(                                            \
        pixels, grad_pixels, gbuffer, covbits, recs, fdata, B, H, W, C, V, F, tile_grid(gntx), L.nrec,          \
        grad_vertices, grad_vertex_colors, grad_background, ndc_scale(W, H), stash_flip)
#define LAUNCH_GRAD(CC)                                                                                       \
    do {                                                                                                      \
        if (gm == 1) LAUNCH_GRAD_GM(CC, 1);                                                                   \
        else if (gm == 2) LAUNCH_GRAD_GM(CC, 2);                                                              \
        else LAUNCH_GRAD_GM(CC, 3);                                                                           \
    } while (0)
    if (C == 1) LAUNCH_GRAD(1);
    else if (C == 3) LAUNCH_GRAD(3);
    else if (C == 7) LAUNCH_GRAD(7);
    else LAUNCH_GRAD(0);
#undef LAUNCH_GRAD
#undef LAUNCH_GRAD_GM
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

extern "C" {

int dirt_rasterise_bwd(const float *vertices, const float *vertex_colors, const int32_t *faces, const float *pixels,
                       const float *grad_pixels, const int32_t *gbuffer, const void *saved, int B, int H, int W, int C,
                       int V, int F, float *grad_vertices, float *grad_vertex_colors, float *grad_background,
                       unsigned flags, void *stream_)
{
    return rasterise_bwd_impl(vertices, vertex_colors, faces, pixels, grad_pixels, gbuffer, saved, B, H, W, C, V, F,
                              grad_vertices, grad_vertex_colors, grad_background, flags, stream_, nullptr);
}

// Workspace of the recompute backward: [saved | scratch | g-buffer | stash header | vertex copy | face copy], each
// 256-B aligned.  The stash (ABI v11): the geometry (vertices, faces, bitwise) whose records, g-buffer and coverage
// bits the workspace holds, written by dirt_rasterise_fwd_stash or after a recomputation.
struct RecomputeParts {
    size_t off_scratch, off_gbuf, off_hdr, off_vtag, off_ftag, total;
};
static RecomputeParts recompute_parts(const Layout &L, int B, int H, int W, int V, int F)
{
    RecomputeParts P;
    P.off_scratch = (size_t)align_up((int64_t)L.saved_total, 256);
    P.off_gbuf = P.off_scratch + (size_t)align_up((int64_t)L.scratch_total, 256);
    P.off_hdr = P.off_gbuf + (size_t)align_up((int64_t)B * H * W * 4, 256);
    P.off_vtag = P.off_hdr + 256;
    P.off_ftag = P.off_vtag + (size_t)align_up((int64_t)B * V * 16, 256);
    P.total = P.off_ftag + (size_t)align_up((int64_t)B * F * 12, 256);
    return P;
}

// launch the stash check (check = true) or update of a recompute workspace for this geometry
static int launch_stash(bool check, bool force, const float *vertices, const int32_t *faces, int B, int H, int W,
                        int V, int F, char *ws, const RecomputeParts &P, hipStream_t stream)
{
    const int64_t nv = (int64_t)B * V * 4, nf = (int64_t)B * F * 3;
    const StashDims dims{{(uint32_t)B, (uint32_t)H, (uint32_t)W, (uint32_t)V, (uint32_t)F}};
    uint32_t *hdr = reinterpret_cast<uint32_t *>(ws + P.off_hdr);
    uint32_t *vt = reinterpret_cast<uint32_t *>(ws + P.off_vtag), *ft = reinterpret_cast<uint32_t *>(ws + P.off_ftag);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, (std::max(nv / 4, nf) + 255) / 256));
    if (check)
        stash_check_kernel<<<dim3(blocks), dim3(256), 0, stream>>>(reinterpret_cast<const uint32_t *>(vertices), vt, nv,
                                                                   reinterpret_cast<const uint32_t *>(faces), ft, nf,
                                                                   hdr, dims);
    else
        stash_update_kernel<<<dim3(blocks), dim3(256), 0, stream>>>(reinterpret_cast<const uint32_t *>(vertices), vt,
                                                                    nv, reinterpret_cast<const uint32_t *>(faces), ft,
                                                                    nf, hdr, dims, force ? 1 : 0);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_bwd_recompute_workspace_size(int B, int H, int W, int C, int V, int F, size_t *workspace_bytes)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    if (workspace_bytes) *workspace_bytes = recompute_parts(L, B, H, W, V, F).total;
    return DIRT_OK;
}

// The registered gradient of the single-output op: upstream DIRT's gradient re-derived its G-buffer from the
// op's inputs (csrc/rasterise_grad_common.h:5-24: launch_vertex_upload, then launch_grad_assembly on pixels,
// grad_pixels and vertices).  Here: setup + binning + a coverage-only raster pass (g-buffer and the
// neighbour-coverage bits, bit-identical to the forward's: same integer rules, same inputs) into the
// caller's workspace, then the same backward kernel as dirt_rasterise_bwd.
int dirt_rasterise_bwd_recompute(const float *background, const float *vertices, const float *vertex_colors,
                                 const int32_t *faces, const float *pixels, const float *grad_pixels, int B, int H,
                                 int W, int C, int V, int F, float *grad_vertices, float *grad_vertex_colors,
                                 float *grad_background, void *workspace, size_t workspace_bytes, unsigned flags,
                                 void *stream_)
{
    (void)background;  // part of the op's inputs (the gradient of an uncovered pixel does not depend on it)
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (B == 0) return DIRT_OK;
    if (!pixels || !grad_pixels || !workspace || (F > 0 && (!faces || !vertices)) ||
        (V > 0 && !grad_vertices && !grad_vertex_colors))
        return fail(DIRT_EINVAL, "RasteriseGrad: null tensor pointer");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    const RecomputeParts P = recompute_parts(L, B, H, W, V, F);
    if (workspace_bytes < P.total)
        return fail(DIRT_EINVAL, "RasteriseGrad: workspace smaller than dirt_bwd_recompute_workspace_size()");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    char *ws = static_cast<char *>(workspace);
    int32_t *gbuf = reinterpret_cast<int32_t *>(ws + P.off_gbuf);
    uint32_t *hdr = reinterpret_cast<uint32_t *>(ws + P.off_hdr);
    const bool acc = (flags & DIRT_BWD_ACCUMULATE) != 0;
    const bool clean = (flags & DIRT_BWD_SCRATCH_CLEAN) != 0;
    // (a workspace not vouched clean starts from scratch: bin counters and the stash header zeroed -- a miss)
    if (!clean) {
        rc = zero_async(hdr, 256, stream);
        if (rc) return rc;
    }
    // stash check: does the workspace already hold this geometry's records, g-buffer and coverage bits (left by
    // dirt_rasterise_fwd_stash or by the previous recomputation)?  The recomputation below then exits at once
    // (device-side; the setup's filler workgroups still zero the accumulators).
    rc = launch_stash(true, false, vertices, faces, B, H, W, V, F, ws, P, stream);
    if (rc) return rc;
    // the recomputation zero-fills the gradient accumulators in passing (setup filler workgroups), so the
    // backward below only adds into them
    rc = rasterise_fwd_impl(nullptr, C, vertices, nullptr, faces, nullptr, B, H, W, C, V, F, DIRT_SHADER_GOURAUD,
                            nullptr, gbuf, ws, L.saved_total, ws + P.off_scratch, L.scratch_total, 0,
                            clean ? DIRT_FWD_SCRATCH_CLEAN : 0u, acc ? nullptr : grad_vertices,
                            acc ? nullptr : grad_vertex_colors, stream_, GbufOut{}, /*nopix=*/true, hdr);
    if (rc) return rc;
    // after a recomputation the workspace holds this geometry: record it for the next call
    rc = launch_stash(false, false, vertices, faces, B, H, W, V, F, ws, P, stream);
    if (rc) return rc;
    return rasterise_bwd_impl(vertices, vertex_colors, faces, pixels, grad_pixels, gbuf, ws, B, H, W, C, V, F,
                              grad_vertices, grad_vertex_colors, grad_background, DIRT_BWD_ACCUMULATE, stream_, hdr);
}

// The single-output op's forward with its gradient stash: dirt_rasterise_fwd (Gouraud) whose records, g-buffer and
// coverage bits go into a recompute workspace, which then also records the geometry; a dirt_rasterise_bwd_recompute
// with that workspace and bitwise the same vertices and faces skips its recomputation.
int dirt_rasterise_fwd_stash(const float *background, const float *vertices, const float *vertex_colors,
                             const int32_t *faces, int B, int H, int W, int C, int V, int F, float *pixels,
                             void *workspace, size_t workspace_bytes, unsigned flags, void *stream_)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (B == 0) return DIRT_OK;
    if (!workspace) return fail(DIRT_EINVAL, "Rasterise: null workspace");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    const RecomputeParts P = recompute_parts(L, B, H, W, V, F);
    if (workspace_bytes < P.total)
        return fail(DIRT_EINVAL, "Rasterise: workspace smaller than dirt_bwd_recompute_workspace_size()");
    char *ws = static_cast<char *>(workspace);
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const bool clean = (flags & DIRT_FWD_SCRATCH_CLEAN) != 0;
    if (!clean) {
        rc = zero_async(ws + P.off_hdr, 256, stream);
        if (rc) return rc;
    }
    rc = rasterise_fwd_impl(background, C, vertices, vertex_colors, faces, nullptr, B, H, W, C, V, F,
                            DIRT_SHADER_GOURAUD, pixels, reinterpret_cast<int32_t *>(ws + P.off_gbuf), ws,
                            L.saved_total, ws + P.off_scratch, L.scratch_total, 0, clean ? DIRT_FWD_SCRATCH_CLEAN : 0u,
                            nullptr, nullptr, stream_);
    if (rc) return rc;
    return launch_stash(false, true, vertices, faces, B, H, W, V, F, ws, P, stream);
}

__global__ void bin_occupancy_kernel(const uint32_t *__restrict__ counts, int64_t nslabs, uint32_t slab, uint32_t *out)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nslabs; k += (int64_t)gridDim.x * blockDim.x) {
        // this forward's count set holds the counts, the other set is zero (kParP)
        const uint32_t n = counts[k * kCountStride] + counts[(nslabs + k) * kCountStride];
        atomicMax(&out[0], n);
        if (n > slab) atomicAdd(&out[1], 1u);
    }
}

// Debug (synchronises `stream`): the bin occupancy the last forward left in `scratch` -- the fullest slab's
// entry count, the number of slabs that overflowed (their tiles took the all-records path) and the slab
// capacity.  Not part of include/dirt_mi355x.h.
int dirt_debug_bin_occupancy(int B, int H, int W, int F, int64_t bin_capacity, const void *scratch,
                             size_t scratch_bytes, void *stream_, uint32_t *max_count, uint32_t *overflowed,
                             uint32_t *slab)
{
    Layout L;
    int rc = make_layout(B, H, W, F, bin_capacity, L);
    if (rc) return rc;
    if (!scratch || scratch_bytes < L.scratch_total) return fail(DIRT_EINVAL, "dirt_debug_bin_occupancy: scratch too small");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    uint32_t *d = nullptr;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&d), 8, stream));
    HIP_TRY(hipMemsetAsync(d, 0, 8, stream));
    const int64_t nslabs = (int64_t)B * L.ncoarse;
    bin_occupancy_kernel<<<dim3(256), dim3(256), 0, stream>>>(
        reinterpret_cast<const uint32_t *>(static_cast<const char *>(scratch) + L.off_count), nslabs, L.slab, d);
    HIP_TRY(hipGetLastError());
    uint32_t h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipFreeAsync(d, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if (max_count) *max_count = h[0];
    if (overflowed) *overflowed = h[1];
    if (slab) *slab = L.slab;
    return DIRT_OK;
}

// Debug (synchronises `stream`): the R5 deviation counters of `scratch` (setup_kernel.h kStatCapCulled /
// kStatClamped), summed over every forward since the scratch was last cleared: faces culled by the R5 vertex cap
// and clipped faces whose sub-vertices the R5 clamp moved.  reset != 0 zeroes them afterwards.  Not part of
// include/dirt_mi355x.h.
int dirt_debug_clip_stats(int B, int H, int W, int F, int64_t bin_capacity, void *scratch, size_t scratch_bytes,
                          void *stream_, int reset, uint32_t *cap_culled, uint32_t *clamped)
{
    Layout L;
    int rc = make_layout(B, H, W, F, bin_capacity, L);
    if (rc) return rc;
    if (!scratch || scratch_bytes < L.scratch_total) return fail(DIRT_EINVAL, "dirt_debug_clip_stats: scratch too small");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    uint32_t *flag = reinterpret_cast<uint32_t *>(static_cast<char *>(scratch) + L.off_flag);
    uint32_t h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&h[0], flag + kStatCapCulled, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(&h[1], flag + kStatClamped, 4, hipMemcpyDeviceToHost, stream));
    if (reset) {
        HIP_TRY(hipMemsetAsync(flag + kStatCapCulled, 0, 4, stream));
        HIP_TRY(hipMemsetAsync(flag + kStatClamped, 0, 4, stream));
    }
    HIP_TRY(hipStreamSynchronize(stream));
    if (cap_culled) *cap_culled = h[0];
    if (clamped) *clamped = h[1];
    return DIRT_OK;
}

// Debug: the automatic deep-cull rule of the current device (DeepAuto): launches issued with it, the generation of
// the last launch reported deep (0 = none), and whether the next forward would take the occluder instantiation.
// Not part of include/dirt_mi355x.h.
int dirt_debug_deep_cull_state(uint32_t *gen, uint32_t *last_deep, int *next_deep)
{
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(DIRT_EINVAL, "dirt_debug_deep_cull_state: device index");
    std::lock_guard<std::mutex> lk(g_deep_mu);
    const DeepAuto &d = g_deep[dev];
    const uint32_t last = d.host ? static_cast<volatile uint32_t *>(d.host)[0] : 0u;
    if (gen) *gen = d.gen;
    if (last_deep) *last_deep = last;
    if (next_deep) *next_deep = (last != 0u && d.gen + 1u - last <= kDeepRecent) ? 1 : 0;
    return DIRT_OK;
}

// Debug (synchronises `stream`): whether the last dirt_rasterise_bwd_recompute on `workspace` recomputed (1: the
// stash did not hold its geometry) or reused the stash (0), and the header's magic word.  Not part of
// include/dirt_mi355x.h.
int dirt_debug_stash_state(int B, int H, int W, int C, int V, int F, const void *workspace, size_t workspace_bytes,
                           void *stream_, uint32_t *last_missed, uint32_t *magic)
{
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    const RecomputeParts P = recompute_parts(L, B, H, W, V, F);
    if (!workspace || workspace_bytes < P.total) return fail(DIRT_EINVAL, "dirt_debug_stash_state: workspace too small");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    uint32_t h[64];
    HIP_TRY(hipMemcpyAsync(h, static_cast<const char *>(workspace) + P.off_hdr, 256, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    const uint32_t p = h[kStashP] & 1u;  // (the last call's grad launch flipped it: that call used p ^ 1)
    if (last_missed) *last_missed = h[kStashMiss + 16 * (p ^ 1u)];
    if (magic) *magic = h[kStashMagicW];
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
        V_RAST(0); V_RAST(1); V_RAST(2); V_RAST(4); V_RAST(8); V_RAST(32); V_RAST(64); V_RAST(96); V_RAST(128); V_RAST(512); V_RAST(1024); V_RAST(2048);
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
        V_SETUP(0, 128); V_SETUP(1, 129); V_SETUP(2, 0); V_SETUP(3, 1); V_SETUP(4, 2); V_SETUP(5, 3); V_SETUP(6, 4);
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
// Not part of include/dirt_mi355x.h; C == 3 or 7.  Returns the kernel time in ms (hipEvents).
int dirt_debug_bwd_variant(int variant, const float *pixels, const float *grad_pixels, const int32_t *gbuffer,
                           const void *saved, int B, int H, int W, int C, int V, int F, float *grad_vertices,
                           float *grad_vertex_colors, float *grad_background, void *stream_, float *ms)
{
    if (C != 3 && C != 7) return fail(DIRT_EINVAL, "dirt_debug_bwd_variant: C must be 3 or 7");
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
    const int gntx = (W + kGradTileW - 1) / kGradTileW, gnty = (H + grad_tile_h(C) - 1) / grad_tile_h(C);
    dim3 grid((unsigned)(gntx * gnty), (unsigned)B), blk(C == 3 ? GradGeom<kGradTileW, grad_tile_h(3)>::NT
                                                                : GradGeom<kGradTileW, grad_tile_h(7)>::NT);
#define V_GRAD(AB)                                                                                                   \
    case AB:                                                                                                         \
        if (C == 3)                                                                                                  \
            grad_kernel<3, AB><<<grid, blk, 0, stream>>>(pixels, grad_pixels, gbuffer, covbits, recs, fdata, B,       \
                                                         H, W, C, V, F, tile_grid(gntx), L.nrec, grad_vertices,       \
                                                         grad_vertex_colors, grad_background, ndc_scale(W, H));       \
        else                                                                                                         \
            grad_kernel<7, AB><<<grid, blk, 0, stream>>>(pixels, grad_pixels, gbuffer, covbits, recs, fdata, B,       \
                                                         H, W, C, V, F, tile_grid(gntx), L.nrec, grad_vertices,       \
                                                         grad_vertex_colors, grad_background, ndc_scale(W, H));       \
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

// Debug (synchronises `stream`): the product backward kernel (C == 3, vertex and colour gradients) launched `reps`
// times through hipExtLaunchKernel with start / stop events, which the runtime takes from the dispatch itself: the mean
// kernel duration in ms, as rocprofv3 --kernel-trace reports it (an event pair around an ordinary launch, or a graph of
// back-to-back launches, adds each launch's dependent-launch gap).  Accumulates into the gradient buffers.  bench.py's
// roofline uses it.  Not part of include/dirt_mi355x.h.
int dirt_debug_bwd_dispatch_ms(const float *pixels, const float *grad_pixels, const int32_t *gbuffer, const void *saved,
                               int B, int H, int W, int C, int V, int F, float *grad_vertices, float *grad_vertex_colors,
                               float *grad_background, int reps, void *stream_, float *ms)
{
    if (C != 3 || !grad_vertices || !grad_vertex_colors || reps < 1 || !ms)
        return fail(DIRT_EINVAL, "dirt_debug_bwd_dispatch_ms: C == 3, both gradient buffers, reps >= 1");
    int rc = validate(B, H, W, C, V, F);
    if (rc) return rc;
    if (!pixels || !grad_pixels || !gbuffer || !saved) return fail(DIRT_EINVAL, "dirt_debug_bwd_dispatch_ms: null pointer");
    Layout L;
    rc = make_layout(B, H, W, F, 0, L);
    if (rc) return rc;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const char *sv = static_cast<const char *>(saved);
    const Rec *recs = reinterpret_cast<const Rec *>(sv + L.saved_recs);
    const FaceData *fdata = reinterpret_cast<const FaceData *>(sv + L.saved_fdata);
    const uint8_t *covbits = reinterpret_cast<const uint8_t *>(sv + L.saved_cov);
    const int gntx = (W + kGradTileW - 1) / kGradTileW, gnty = (H + grad_tile_h(3) - 1) / grad_tile_h(3);
    const dim3 grid((unsigned)(gntx * gnty), (unsigned)B), blk(GradGeom<kGradTileW, grad_tile_h(3)>::NT);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t err = hipEventCreate(&e0);
    if (err == hipSuccess) err = hipEventCreate(&e1);
    float total = 0.0f;
    for (int r = 0; r < reps && err == hipSuccess; ++r) {
        hipExtLaunchKernelGGL(grad_kernel<3, 0, kGradTileW, grad_tile_h(3), 3>, grid, blk, 0u, stream, e0, e1, 0u,
                              pixels, grad_pixels, gbuffer, covbits, recs, fdata, B, H, W, C, V, F, tile_grid(gntx),
                              L.nrec, grad_vertices, grad_vertex_colors, grad_background, ndc_scale(W, H),
                              static_cast<uint32_t *>(nullptr));
        err = hipGetLastError();
        if (err == hipSuccess) err = hipEventSynchronize(e1);
        float t = 0.0f;
        if (err == hipSuccess) err = hipEventElapsedTime(&t, e0, e1);
        total += t;
    }
    // (the events are released on every path)
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    HIP_TRY(err);
    *ms = total / (float)reps;
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
    return zero_async(static_cast<char *>(scratch) + L.off_count, L.off_bins - L.off_count, stream);
}

int dirt_stream_capture_id(void *stream_, unsigned long long *capture_id)
{
    if (!capture_id) return fail(DIRT_EINVAL, "dirt_stream_capture_id: null pointer");
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    HIP_TRY(hipStreamGetCaptureInfo(reinterpret_cast<hipStream_t>(stream_), &st, &id));
    *capture_id = st == hipStreamCaptureStatusActive ? id : 0ull;
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


// ---- fused lighting helpers (lighting_kernels.h; dirt/lighting.py)

int dirt_vertex_normals_fwd(const float *vertices, int vertex_stride, const void *faces, int faces_int64, int B, int V,
                            int F, float *summed, float *normals, void *stream_)
{
    if (B < 0 || V < 0 || F < 0 || vertex_stride < 3)
        return fail(DIRT_EINVAL, "vertex_normals: negative size or vertex stride < 3");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const int64_t nv = (int64_t)B * V;
    if (nv == 0) return DIRT_OK;
    if (!vertices || !summed || !normals || (F > 0 && !faces)) return fail(DIRT_EINVAL, "vertex_normals: null pointer");
    int rc_z;
    rc_z = zero_async(summed, (size_t)nv * 3 * sizeof(float), stream);  // (a kernel: graph-captured like the rest)
    if (rc_z) return rc_z;
    if (F > 0 && B > 0) {
        const dim3 grid(light_blocks(F), (unsigned)B);
        if (faces_int64)
            vnormals_face_kernel<int64_t><<<grid, dim3(kLightThreads), 0, stream>>>(
                vertices, vertex_stride, static_cast<const int64_t *>(faces), V, F, summed);
        else
            vnormals_face_kernel<int32_t><<<grid, dim3(kLightThreads), 0, stream>>>(
                vertices, vertex_stride, static_cast<const int32_t *>(faces), V, F, summed);
        HIP_TRY(hipGetLastError());
    }
    vnormals_vertex_kernel<<<dim3(light_blocks(nv)), dim3(kLightThreads), 0, stream>>>(summed, nv, normals);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_vertex_normals_bwd(const float *vertices, int vertex_stride, const void *faces, int faces_int64, int B, int V,
                            int F, const float *summed, const float *grad_normals, float *grad_summed,
                            float *grad_vertices, int grad_stride, void *stream_)
{
    if (B < 0 || V < 0 || F < 0 || vertex_stride < 3 || grad_stride < 3)
        return fail(DIRT_EINVAL, "vertex_normals: negative size or vertex stride < 3");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const int64_t nv = (int64_t)B * V;
    if (nv == 0) return DIRT_OK;
    if (!vertices || !summed || !grad_normals || !grad_summed || !grad_vertices || (F > 0 && !faces))
        return fail(DIRT_EINVAL, "vertex_normals: null pointer");
    const int rc_z = zero_async(grad_vertices, (size_t)nv * grad_stride * sizeof(float), stream);
    if (rc_z) return rc_z;
    if (F == 0) return DIRT_OK;
    vnormals_vertex_bwd_kernel<<<dim3(light_blocks(nv)), dim3(kLightThreads), 0, stream>>>(summed, grad_normals, nv,
                                                                                          grad_summed);
    HIP_TRY(hipGetLastError());
    const dim3 grid(light_blocks(F), (unsigned)B);
    if (faces_int64)
        vnormals_face_bwd_kernel<int64_t><<<grid, dim3(kLightThreads), 0, stream>>>(
            vertices, vertex_stride, static_cast<const int64_t *>(faces), V, F, grad_summed, grad_vertices, grad_stride);
    else
        vnormals_face_bwd_kernel<int32_t><<<grid, dim3(kLightThreads), 0, stream>>>(
            vertices, vertex_stride, static_cast<const int32_t *>(faces), V, F, grad_summed, grad_vertices, grad_stride);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_diffuse_directional_fwd(const float *normals, const float *colors, int64_t N, const float *light_direction,
                                 const float *light_color, int double_sided, float *out, void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "diffuse_directional: negative size");
    if (N == 0) return DIRT_OK;
    if (!normals || !colors || !light_direction || !light_color || !out)
        return fail(DIRT_EINVAL, "diffuse_directional: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    diffuse_fwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(normals, colors, N, light_direction,
                                                                                  light_color, double_sided, out);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_diffuse_directional_bwd(const float *normals, const float *colors, int64_t N, const float *light_direction,
                                 const float *light_color, int double_sided, const float *grad_out,
                                 float *grad_normals, float *grad_colors, void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "diffuse_directional: negative size");
    if (N == 0 || (!grad_normals && !grad_colors)) return DIRT_OK;
    if (!normals || !colors || !light_direction || !light_color || !grad_out)
        return fail(DIRT_EINVAL, "diffuse_directional: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    diffuse_bwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(
        normals, colors, N, light_direction, light_color, double_sided, grad_out, grad_normals, grad_colors);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_diffuse_point_fwd(const float *positions, const float *normals, const float *colors, int64_t N,
                           const float *light_position, const float *light_color, int double_sided, float *out,
                           void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "diffuse_point: negative size");
    if (N == 0) return DIRT_OK;
    if (!positions || !normals || !colors || !light_position || !light_color || !out)
        return fail(DIRT_EINVAL, "diffuse_point: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    diffuse_point_fwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(
        positions, normals, colors, N, light_position, light_color, double_sided, out);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_diffuse_point_bwd(const float *positions, const float *normals, const float *colors, int64_t N,
                           const float *light_position, const float *light_color, int double_sided,
                           const float *grad_out, float *grad_positions, float *grad_normals, float *grad_colors,
                           void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "diffuse_point: negative size");
    if (N == 0 || (!grad_positions && !grad_normals && !grad_colors)) return DIRT_OK;
    if (!positions || !normals || !colors || !light_position || !light_color || !grad_out)
        return fail(DIRT_EINVAL, "diffuse_point: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    diffuse_point_bwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(
        positions, normals, colors, N, light_position, light_color, double_sided, grad_out, grad_positions,
        grad_normals, grad_colors);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_specular_directional_fwd(const float *positions, const float *normals, const float *reflectivities, int64_t N,
                                  const float *light_direction, const float *light_color,
                                  const float *camera_position, float shininess, int double_sided, float *out,
                                  void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "specular_directional: negative size");
    if (N == 0) return DIRT_OK;
    if (!positions || !normals || !reflectivities || !light_direction || !light_color || !camera_position || !out)
        return fail(DIRT_EINVAL, "specular_directional: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    specular_fwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(
        positions, normals, reflectivities, N, light_direction, light_color, camera_position, shininess, double_sided,
        out);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

int dirt_specular_directional_bwd(const float *positions, const float *normals, const float *reflectivities, int64_t N,
                                  const float *light_direction, const float *light_color,
                                  const float *camera_position, float shininess, int double_sided,
                                  const float *grad_out, float *grad_positions, float *grad_normals,
                                  float *grad_reflectivities, void *stream_)
{
    if (N < 0) return fail(DIRT_EINVAL, "specular_directional: negative size");
    if (N == 0 || (!grad_positions && !grad_normals && !grad_reflectivities)) return DIRT_OK;
    if (!positions || !normals || !reflectivities || !light_direction || !light_color || !camera_position || !grad_out)
        return fail(DIRT_EINVAL, "specular_directional: null pointer");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    specular_bwd_kernel<<<dim3(light_blocks(N)), dim3(kLightThreads), 0, stream>>>(
        positions, normals, reflectivities, N, light_direction, light_color, camera_position, shininess, double_sided,
        grad_out, grad_positions, grad_normals, grad_reflectivities);
    HIP_TRY(hipGetLastError());
    return DIRT_OK;
}

}  // extern "C"
