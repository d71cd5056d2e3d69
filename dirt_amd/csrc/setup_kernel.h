// Part of dirt_raster.hip's translation unit: included inside its anonymous namespace after the shared
// definitions (raster_rules.h, oceanic.h, hill.h, the layout and error helpers).  Not a standalone header.

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

// a triangle clipped by 5 planes has at most 8 vertices (6 fan sub-triangles: kExtraPerFace + 1)
constexpr int kMaxClipVerts = 8;
static_assert(kMaxClipVerts - 2 == kExtraPerFace + 1, "sub-triangle slots");

// R5 deviation counters, words of the scratch's flag area (cleared with the bin counters,
// cumulative until then; dirt_debug_clip_stats reads them): faces culled by the R5 vertex cap, and clipped faces
// with at least one sub-vertex moved by the R5 sub-vertex clamp.  A GL driver keeps both kinds of face (it has no
// fixed polygon buffer and clips in higher precision), so these count where this rasteriser's output may differ
// from the reference's for reasons other than driver arithmetic.  Only the clipping slow path touches them.
constexpr int kStatCapCulled = 48, kStatClamped = 52;
// Automatic deep-scene culling (raster_kernel DeepArgs): per launch, the number of sampled workgroups (one in
// kDeepSample) whose wave 0 found more than kDeepMark entries in its first list, in two slots that alternate between
// the launches on one scratch (words kDeepCnt, kDeepCnt + 4).  A launch zeroes its predecessor's slot after reporting
// it; a launch is deep when at least 1 / kDeepFrac of the sampled workgroups marked it.
constexpr int kDeepCnt = 56;
constexpr int kDeepMark = 64;
constexpr uint32_t kDeepSample = 16, kDeepFrac = 8;

// Gradient stash of the single-output op (dirt_rasterise_fwd_stash / dirt_rasterise_bwd_recompute): a 256-B header
// in the recompute workspace.  Words: kStashP parity p; kStashMiss + 16 p the current call's miss flag (set by
// stash_check_kernel when the workspace does not hold this geometry), the other one zeroed by the same check for the
// next call; the backward's grad launch flips p.  Between calls the current flag is 0 (zeroed workspace: p = 0).
constexpr int kStashP = 0, kStashMiss = 16, kStashMagicW = 48, kStashDims = 49;  // dims: B, H, W, V, F
constexpr uint32_t kStashMagic = 0xD1275A5Eu;
__device__ __forceinline__ bool stash_hit(const uint32_t *hdr)
{
    const uint32_t p = hdr[kStashP] & 1u;
    return hdr[kStashMiss + 16 * p] == 0u;
}

// R5 slow path: clip against z>=-w and the guard planes, fan-triangulate, write the sub-records.
// Not inlined so that its stack arrays do not inflate the fast path.  Returns nsub.  `flag`: the scratch's
// flag area (the R5 deviation counters above), may be null.
__device__ __noinline__ int clip_face(Tri tri, int W, int H, int F, int f, Rec *frame_recs, uint32_t *flag)
{
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    float poly[kMaxClipVerts][7], tmp[kMaxClipVerts][7];
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
            // R5 vertex cap: more than 8 vertices (possible only when rounding near w = 0 makes the polygon
            // non-convex) culls the face -- it would need more than the 6 sub-triangle slots
            if ((ina ? 1 : 0) + (ina != inc ? 1 : 0) > kMaxClipVerts - m) {
                if (flag) atomicAdd(&flag[kStatCapCulled], 1u);
                return 0;
            }
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
    if (flag) {
        // the sub-vertex clamp of make_record<true> (the same quotients): does it move any sub-vertex?
        bool moved = false;
        for (int i = 0; i < n; ++i) {
            const float iw = 1.0f / poly[i][3], xn = poly[i][0] * iw, yn = poly[i][1] * iw;
            moved = moved || guard_clamp(xn, 2.0f * gx) != xn || guard_clamp(yn, 2.0f * gy) != yn;
        }
        if (moved) atomicAdd(&flag[kStatClamped], 1u);
    }
    for (int s = 0; s < nsub; ++s) {
        float sv[3][4], sb[3][3];
        const int idx[3] = {0, s + 1, s + 2};
        for (int k = 0; k < 3; ++k) {
            for (int c = 0; c < 4; ++c) sv[k][c] = poly[idx[k]][c];
            for (int i = 0; i < 3; ++i) sb[k][i] = poly[idx[k]][4 + i];
        }
        Rec r;
        make_record<true>(sv, sb, W, H, f, r, 2.0f * gx, 2.0f * gy);
        frame_recs[rec_index(F, f, s)] = r;
    }
    return nsub;
}

// One face's setup (R1..R5, as setup_kernel) into `frame_recs`, which may live in any address space (the
// fused small-scene raster passes LDS): the fast-path record at slot f, or the clipped sub-records.
// Returns the face's FaceData; `oob` = a vertex index outside [0, V) (the face is culled).
__device__ __forceinline__ FaceData setup_face_into(const float *vb, const int32_t *face3, int V, int F, int W, int H,
                                                    int f, Rec *frame_recs, bool &oob, uint32_t *flag)
{
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    const int32_t vidx[3] = {face3[0], face3[1], face3[2]};
    Tri tri;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool in = vidx[k] >= 0 && vidx[k] < V;
        const float4 pv = in ? *reinterpret_cast<const float4 *>(vb + (int64_t)vidx[k] * 4) : make_float4(0.f, 0.f, 0.f, 1.f);
        tri.v[k][0] = pv.x; tri.v[k][1] = pv.y; tri.v[k][2] = pv.z; tri.v[k][3] = pv.w;
        ok = ok && in;
    }
    oob = !ok;
#pragma unroll
    for (int k = 0; k < 3; ++k) ok = ok && finite4(tri.v[k]);
    FaceData fd;
    fd.v[0] = vidx[0]; fd.v[1] = vidx[1]; fd.v[2] = vidx[2];
    fd.q[0] = tri.v[0][3]; fd.q[1] = tri.v[1][3]; fd.q[2] = tri.v[2][3];
    fd.clipped = 0;
    bool fast = ok;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float w = tri.v[k][3];
        fast = fast && (w > 0.0f && fabsf(tri.v[k][0]) <= gx * w && fabsf(tri.v[k][1]) <= gy * w);
    }
    Rec r;
    set_empty(r, f);
    int nsub = 0;
    if (fast) {
        const float id[3][3] = {{1.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, {0.f, 0.f, 1.f}};
        make_record(tri.v, id, W, H, f, r);
        frame_recs[f] = r;
        fd.q[0] = r.iw[0]; fd.q[1] = r.iw[1]; fd.q[2] = r.iw[2];
        nsub = 1;
    } else {
        frame_recs[f] = r;  // empty unless clip_face overwrites it
        if (ok) {
            nsub = clip_face(tri, W, H, F, f, frame_recs, flag);
            fd.clipped = 1;
        }
    }
    fd.nsub = nsub;
    return fd;
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
    const uint2 q = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(&r) + kRecBboxOffset);
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
template <int AB = 0, int NT = kBinThreads>
__global__ __launch_bounds__(NT) void setup_kernel(const float *__restrict__ verts,
                                                            const int32_t *__restrict__ faces, int V, int F, int W,
                                                            int H, int cshift, int nctx, int ncoarse, int64_t nrec,
                                                            Rec *__restrict__ recs, FaceData *__restrict__ fdata,
                                                            uint32_t *__restrict__ counts, uint32_t *__restrict__ flag,
                                                            uint2 *__restrict__ bins, uint32_t slab, int B,
                                                            const ZeroFill zf, const float gx, const float gy,
                                                            const uint32_t *__restrict__ stash_hdr = nullptr)
{
    // workgroups past the faces zero-fill the caller's gradient accumulators (DIRT_FWD zero_grad_*): the
    // setup grid leaves most CUs idle (196 workgroups at config 3), so the fill costs the raster nothing
    if ((int)blockIdx.x >= zf.nfb) {
        zf.run((int64_t)blockIdx.y * (gridDim.x - zf.nfb) + (blockIdx.x - zf.nfb), (int64_t)(gridDim.x - zf.nfb) * gridDim.y);
        return;
    }
    // the recompute backward's setup: nothing to do when the workspace already holds this geometry's records
    // (stash hit, dirt_raster.hip stash_check_kernel)
    if (stash_hdr != nullptr && stash_hit(stash_hdr)) return;
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
        for (int64_t k = g * NT + t; k < ncount; k += ng * NT) other[k * kCountStride] = 0;
    }
    for (int c = t; c < ncoarse; c += NT) hist[c] = 0;
    if (t == 0) Q.n = 0;
    __syncthreads();
    auto count = [&](int32_t, uint32_t, uint32_t, int cx, int cy) { atomicAdd(&hist[cy * nctx + cx], 1u); };
    Rec *frame_recs = recs + (int64_t)b * nrec;
    const float *vb = verts + (int64_t)b * V * 4;
    // (guard band gx = 32768 / W, gy = 32768 / H: IEEE divisions on the host, the same floats -- two
    // correctly rounded division sequences fewer in the one-wave-per-SIMD chain)
    const int f = blockIdx.x * NT + t;  // (one face per thread)
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
        fd.q[0] = tri.v[0][3]; fd.q[1] = tri.v[1][3]; fd.q[2] = tri.v[2][3];  // clip w (clipped faces)
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
            if (AB & 2) {
                // ablation (timing only, wrong records): the pixel bbox of the three vertices without the
                // record arithmetic (divisions, int64 edge setup, depth plane)
                const float hw = 0.5f * (float)W, hh = 0.5f * (float)H;
                float x0 = 1e30f, x1 = -1e30f, y0 = 1e30f, y1 = -1e30f;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const float xw = (tri.v[k][0] + 1.0f) * hw, yw = (tri.v[k][1] + 1.0f) * hh;
                    x0 = fminf(x0, xw); x1 = fmaxf(x1, xw); y0 = fminf(y0, yw); y1 = fmaxf(y1, yw);
                }
                // (clamped exactly as make_record does: an empty box stays empty, no index past the frame)
                const int i0 = (int)fminf(fmaxf(x0, 0.0f), (float)W), i1 = (int)fminf(fmaxf(x1, -1.0f), (float)(W - 1));
                const int j0 = (int)fminf(fmaxf(y0, 0.0f), (float)H), j1 = (int)fminf(fmaxf(y1, -1.0f), (float)(H - 1));
                if (i0 <= i1 && j0 <= j1) {
                    r.i0 = (uint16_t)i0; r.i1 = (uint16_t)i1; r.j0 = (uint16_t)j0; r.j1 = (uint16_t)j1;
                }
            } else {
                make_record(tri.v, id, W, H, f, r);
            }
            nsub = 1;
            // (the record's first 64 B; its 1/w go with the FaceData: one 64-B piece per record instead of
            // two to write back when the kernel ends and for the raster to fetch)
            store_record_fast(&frame_recs[f], r);
            fd.q[0] = r.iw[0]; fd.q[1] = r.iw[1]; fd.q[2] = r.iw[2];
            fbx = (uint32_t)r.i0 | ((uint32_t)r.i1 << 16);
            fby = (uint32_t)r.j0 | ((uint32_t)r.j1 << 16);
            coarse_pairs_add(Q, f, fbx, fby, cshift, count);
        } else {
            frame_recs[f] = r;  // empty unless clip_face overwrites it
#ifndef DIRT_SETUP_NO_CLIP
            if (ok) {
                nsub = clip_face(tri, W, H, F, f, frame_recs, flag);
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
    const int nbig = coarse_pairs_flush<NT>(Q, count);
    PHASE_TS(2);
    // reserve this workgroup's range of every touched slab: one returning device atomic per (workgroup,
    // coarse tile), all in flight together
    uint32_t *cc = ccount + (int64_t)b * ncoarse * kCountStride;
    for (int c = t; c < ncoarse; c += NT) {
        const uint32_t n = hist[c];
        // (AB & 1: ablation, no reservation; AB & 4: probe, workgroups split over two counters per tile --
        // timing only, the raster would not find the second half)
        const int shard = (AB & 4) ? (int)(blockIdx.x & 1) * 32 : 0;
        base[c] = (AB & 1) ? 0u : n ? atomicAdd(&cc[c * kCountStride + shard], n) : 0u;
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
    if (nbig > 0) coarse_pairs_flush<NT>(Q, place);
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

// Setup workgroup size.  256 faces per workgroup keep the slab-reservation atomics few (one per workgroup and
// touched coarse tile); a batch with fewer than kSetupSmallGrid such workgroups (BASELINE config 4: one frame of
// 20k faces, 79 workgroups) leaves most CUs idle, and 128-face workgroups there shorten the setup (c4 setup
// 8.6-10.0 -> 7.6-8.0 us; c3, 196 workgroups, loses 1 us with them: profiles/r03/ab_setup_threads/).
constexpr int64_t kSetupSmallGrid = 128;
#ifndef DIRT_SETUP_SMALL_THREADS
#define DIRT_SETUP_SMALL_THREADS (kBinThreads / 2)
#endif
constexpr int kSetupSmallThreads = DIRT_SETUP_SMALL_THREADS;

// launch the setup (and binning) of B frames x F faces
template <int AB = 0>
void launch_setup(const float *vertices, const int32_t *faces, int B, int H, int W, int V, int F, const Layout &L,
                  Rec *recs, FaceData *fdata, uint32_t *ccount, uint32_t *flag, uint2 *bins, hipStream_t stream,
                  float *zero_a = nullptr, int64_t nzero_a = 0, float *zero_b = nullptr, int64_t nzero_b = 0,
                  const uint32_t *stash_hdr = nullptr)
{
    const bool small = (int64_t)B * ((F + kBinThreads - 1) / kBinThreads) < kSetupSmallGrid;
    const int nt = small ? kSetupSmallThreads : kBinThreads;
    ZeroFill zf{zero_a, zero_b, zero_a ? nzero_a : 0, zero_b ? nzero_b : 0, (F + nt - 1) / nt};
    // filler workgroups per frame row: ~16 float4 stores per thread, at most 64 in all
    // (rounded up: a few accumulator floats in all, fewer than one float4, still need a filler workgroup)
    const int64_t z4 = (zf.na + zf.nb + 3) / 4, want = std::min<int64_t>((z4 + 4095) / 4096, 64);
    const int nzb = z4 > 0 ? (int)std::max<int64_t>(1, (want + B - 1) / B) : 0;
    const dim3 grid((unsigned)(zf.nfb + nzb), (unsigned)B);
    const float gx = 32768.0f / (float)W, gy = 32768.0f / (float)H;
    if (small)
        setup_kernel<AB, kSetupSmallThreads><<<grid, dim3(kSetupSmallThreads), 0, stream>>>(
            vertices, faces, V, F, W, H, L.cshift, L.nctx, L.ncoarse, L.nrec, recs, fdata, ccount, flag, bins, L.slab, B,
            zf, gx, gy, stash_hdr);
    else
        setup_kernel<AB, kBinThreads><<<grid, dim3(kBinThreads), 0, stream>>>(
            vertices, faces, V, F, W, H, L.cshift, L.nctx, L.ncoarse, L.nrec, recs, fdata, ccount, flag, bins, L.slab, B,
            zf, gx, gy, stash_hdr);
}
