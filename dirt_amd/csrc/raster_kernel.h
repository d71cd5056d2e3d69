// Part of dirt_raster.hip's translation unit: included inside its anonymous namespace after the shared
// definitions (raster_rules.h, oceanic.h, hill.h, the layout and error helpers).  Not a standalone header.

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

// Tiles per row with a host-computed reciprocal: tile / ntx = umulhi(2 tile, m), m = ceil(2^31 / ntx).
// m = 2^31/ntx + e/ntx with 0 <= e < ntx, so 2 tile m / 2^32 = tile/ntx + tile e / (ntx 2^31); the error
// tile e / (ntx 2^31) < tile / 2^31 < 2^-13 (tile < 2^18) stays below the 1/ntx gap to the next integer
// for ntx <= 512, so the floor is exact.  The 2^31 scale keeps m of ntx = 1 in 32 bits (2^32 / 1 would
// not fit).  Two scalar instructions instead of a ~25-instruction division in every wave's prologue.
struct TileGrid {
    int ntx;
    uint32_t inv;
    __device__ __forceinline__ void split(int tile, int &tx, int &ty) const
    {
        // floor(tile / ntx) = umulhi(2 tile, ceil(2^31 / ntx)), exact for tile < 2^18, ntx <= 512; the
        // 2^31 scale keeps the reciprocal of ntx = 1 in 32 bits (2^32 / 1 would not fit)
        ty = (int)__umulhi((uint32_t)tile << 1, inv);
        tx = tile - ty * ntx;
    }
};
static_assert((DIRT_MAX_DIM / kTile) <= 512 && (DIRT_MAX_DIM / kTile) * (DIRT_MAX_DIM / kTile) <= (1 << 18),
              "TileGrid reciprocal range");
inline TileGrid tile_grid(int ntx) { return TileGrid{ntx, (uint32_t)(((1ull << 31) + (uint64_t)ntx - 1) / (uint64_t)ntx)}; }

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
// Lists of at least DIRT_RASTER_HZ_DEEP_N entries run only their first DIRT_RASTER_HZ_DEEP before culling.
#ifndef DIRT_RASTER_HZ_DEEP_N
#define DIRT_RASTER_HZ_DEEP_N 1000000
#endif
#ifndef DIRT_RASTER_HZ_DEEP
#define DIRT_RASTER_HZ_DEEP 8
#endif
// Occluder culling before the entry loop (the OCC instantiation, dirt_rasterise_fwd flag DIRT_FWD_DEEP_CULL): a
// wave whose list holds more than DIRT_RASTER_OCC_MIN entries first bounds its block's final depth by the
// nearest entry that covers the whole block (entry_occluder_qmax), then drops every entry whose depth lower
// bound exceeds it -- in deep scenes (large overlapping triangles) most of the list, before any of it runs.
// Results are bit-identical.  Opt-in: the pass runs only for long lists, but its mere presence costs the
// common case (c3) ~0.6 us of raster time (profiles/r04/ab_occluder), while deep scenes gain 15 %.
#ifndef DIRT_RASTER_OCC_MIN
#define DIRT_RASTER_OCC_MIN 32
#endif
constexpr int kWaveList = 256 + 2;  // a staging round's entries + the even pad
constexpr int kFilterBlock = 128;  // coarse-bin entries filtered per wave and chunk (2 loads per lane in flight)
// A staged record is "small" when every |A|, |B| < 2^15: its edge steps inside a strip are one
// v_dot2_i32_i16 of the packed (A, B) with the lane's packed (dx, dy) offsets (<= 15*256, 3*256).
constexpr int kDotEdge = 1 << 15;
constexpr uint32_t kLargeAB = 0x80008000u;  // ab[0] of a large entry (A = B = -2^15 never occurs in a small one)
// the resolve's int32 path: winners with every |A|, |B| < 2^14 (see the resolve)
constexpr int32_t kResolveSmall = 1 << 14;
#ifndef DIRT_RASTER_RESOLVE32
#define DIRT_RASTER_RESOLVE32 1
#endif

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
    const float zw = depth_at(r.za, r.zb, r.z0, fxl - rec_fx0(r.X0), fyl - rec_fx0(r.Y0));
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
        const int64_t e0 = (int64_t)R.A[k] * (int64_t)(px0 - R.X0) + ((int64_t)R.B[k] * (int64_t)(py0 - R.Y0) + (k == 0 ? R.D : 0)) + owned;
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
        const int64_t e64 =
            (int64_t)R.A[k] * (int64_t)(px0 - R.X0) + ((int64_t)R.B[k] * (int64_t)(py0 - R.Y0) + (k == 0 ? R.D : 0)) + owned;
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
    E.za = R.za; E.zb = R.zb; E.z0 = R.z0; E.fx0 = rec_fx0(R.X0); E.fy0 = rec_fx0(R.Y0);
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

// Occluder bound (DIRT_RASTER_OCC): a staged small entry that covers the wave's whole 8x8 block (all four
// corner pixel centres inside -- the block is convex) with its depth inside [0, 1) there writes or beats every
// pixel of the block, so every final key of the block has depth <= this entry's maximum there.  Returns a
// conservative upper bound of that maximum (the plane at the corner its slopes point to, plus twice the
// two-rounding error bound and two quanta), or 0xffffffff when the entry is not such an occluder.
__device__ __forceinline__ uint32_t entry_occluder_qmax(const StripEntry *ent, uint32_t off, int bx, int by, int x0,
                                                        int y0)
{
    lds_int4v *ve = (lds_int4v *)((const char *)ent + off);
    const int cx0 = 256 * bx, cx1 = 256 * (bx + kWaveW - 1), cy0 = 256 * by, cy1 = 256 * (by + kWaveH - 1);
    // two rounds of (volatile, so ordered) LDS reads: the coverage half first, then the depth plane -- fewer
    // registers live at once than one batch of three b128 reads
    bool cover = true;
    {
        const int4v q0 = ve[0], q1 = ve[1];
        const int e[3] = {q0.x, q0.y, q0.z};
        const uint32_t ab[3] = {(uint32_t)q0.w, (uint32_t)q1.x, (uint32_t)q1.y};
        // a large entry keeps its record index in e[0] and the kLargeAB sentinel in ab[0]; its other fields are
        // not edge values of this tile, so it is never taken as an occluder
        cover = ab[0] != kLargeAB;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int A = (int)(short)(ab[k] & 0xffffu), B = (int)(short)(ab[k] >> 16);
            // the edge function is linear: its minimum over the block is at a corner (E + owned > 0 = inside)
            cover = cover && e[k] + min(A * cx0, A * cx1) + min(B * cy0, B * cy1) > 0;
        }
    }
    const int4v q1 = ve[1], q2 = ve[2];
    const float za = __int_as_float(q1.z), zb = __int_as_float(q1.w), z0 = __int_as_float(q2.w);
    const float xa = (float)x0 + 0.5f - __int_as_float(q2.x), xb = (float)(x0 + kWaveW - 1) + 0.5f - __int_as_float(q2.x);
    const float ya = (float)y0 + 0.5f - __int_as_float(q2.y), yb = (float)(y0 + kWaveH - 1) + 0.5f - __int_as_float(q2.y);
    const float zhi = depth_at(za, zb, z0, za > 0.0f ? xb : xa, zb > 0.0f ? yb : ya);
    const float zlo = depth_at(za, zb, z0, za > 0.0f ? xa : xb, zb > 0.0f ? ya : yb);
    const float m = (fabsf(za) * fmaxf(fabsf(xa), fabsf(xb)) + fabsf(zb) * fmaxf(fabsf(ya), fabsf(yb)) + fabsf(z0)) * 0x1p-21f;
    const float hi = zhi + m;
    // (false for NaN planes; the far margin keeps every pixel's quantised depth below the cleared 2^24 - 1)
    const bool in_range = zlo - m >= 0.0f && hi < 0.999f;
    return cover && in_range ? (uint32_t)__builtin_fmaf(hi, 16777215.0f, 2.5f) : 0xffffffffu;
}

// minimum of v over the wave, wave-uniform (as wave_max_u32)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));
    const uint32_t a = __builtin_amdgcn_readlane(v, 15), b = __builtin_amdgcn_readlane(v, 31);
    const uint32_t c = __builtin_amdgcn_readlane(v, 47), d = __builtin_amdgcn_readlane(v, 63);
    return min(min(a, b), min(c, d));
}

// The occluder pass over one wave's entry list (out of line: it runs only for long lists, and inlined its
// registers cost the common path a spill): the block's depth bound from its full-block occluders, then an
// in-place compaction to the entries whose depth lower bound does not exceed it.  Returns the new length.
__device__ __noinline__ int occluder_cull(const StripEntry *ent, uint32_t *wl, int ns, int bxo, int byo, int ti0, int tj0)
{
    const int lane = threadIdx.x & 63;
    uint32_t bound = 0xffffffffu;
    for (int c0 = 0; c0 < ns; c0 += 64) {
        const int kk = c0 + lane;
        if (kk < ns) bound = min(bound, entry_occluder_qmax(ent, wl[kk], bxo, byo, ti0 + bxo, tj0 + byo));
        // no occluder among the first 64 entries (small triangles, however deep): give up early -- the
        // pass is an optional cull, and lists of small faces rarely hold one further on
        if (c0 == 0 && __builtin_amdgcn_ballot_w64(bound != 0xffffffffu) == 0) return ns;
    }
    bound = wave_min_u32(bound);
    if (bound == 0xffffffffu) return ns;
    // (each group's offsets are read by every lane before any is written)
    int n2 = 0;
    for (int c0 = 0; c0 < ns; c0 += 64) {
        const int kk = c0 + lane;
        const bool tst = kk < ns;
        const uint32_t off = tst ? wl[kk] : 0u;
        const bool live = tst && entry_qmin(ent, off, ti0 + bxo, tj0 + byo) <= bound;
        const uint64_t lm = __ballot(live);
        if (live) wl[n2 + lane_rank(lm)] = off;
        n2 += __popcll(lm);
    }
    if (lane == 0) wl[n2] = 256u * sizeof(StripEntry);  // pad / sentinel
    wave_lds_sync();
    return n2;
}

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
__device__ __forceinline__ uint32_t neighbour_coverage(const RasterPart &r, const int64_t E[3], bool multi, int32_t ri,
                                                       const Rec *frame_recs, const FaceData *fdata_frame, int F, int f,
                                                       int i, int j, bool known_small = false)
{
    // int32 when every lane's |E| < 2^30 and |A|, |B| < 2^22 (a one-pixel step stays inside int32);
    // otherwise the out-of-line int64 version (a real branch, not both paths).  `known_small` (wave-uniform):
    // the resolve's int32 path already bounds |E| < 2^30 and |A|, |B| < 2^14
    bool small = true;
    if (!known_small) {
#pragma unroll
        for (int k = 0; k < 3; ++k)
            small = small && (uint64_t)(E[k] + (1ll << 30)) < (2ull << 30) && (uint32_t)(r.A[k] + (1 << 22)) < (2u << 22) &&
                    (uint32_t)(r.B[k] + (1 << 22)) < (2u << 22);
    }
    uint32_t bits = 0;
    if (known_small || __builtin_amdgcn_ballot_w64(!small) == 0) {
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
        // (the global record, not the caller's register copy: a noinline callee would put that in scratch)
        bits = neighbour_bits_i64(*reinterpret_cast<const EdgePart *>(&frame_recs[ri]), E[0], E[1], E[2]);
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
// 32 no neighbour-coverage bits, 64 no colour loads (lambda written), 128 phase timestamps, 512 / 1024 / 2048 one
// extra dependent global round trip before the slab loads / before the colour loads / before the record loads
// extra kernel attributes for experiments, e.g. -DDIRT_RASTER_ATTR='__attribute__((amdgpu_num_sgpr(80)))': 256-thread
// workgroups are admitted per CU up to floor(800 / (ceil(sgpr / 16) * 16 + 16)) -- 7 at 82-96 SGPRs, 8 at <= 80
// (MI355X_MICROARCH.md, residency), whatever the VGPR budget allows
#ifndef DIRT_RASTER_ATTR
#define DIRT_RASTER_ATTR __attribute__((amdgpu_num_sgpr(80)))
#endif
#ifndef DIRT_RASTER_WAVES
#define DIRT_RASTER_WAVES 8  // min waves per SIMD the register allocation must allow (Gouraud, C = 1 or 3;
                             // the procedural programs and the generic-C path keep their natural allocation).
                             // 8 with <= 80 SGPRs (DIRT_RASTER_ATTR): 8 workgroups per CU, round 4
                             // (profiles/r04/ab_raster_occupancy: raster 24.0-24.3 -> 23.6-23.8 us)
#endif
// Optional deferred-shading outputs of the resolve (dirt_rasterise_fwd_gbuffer; instantiated only when
// asked for, GB = true, so the default kernel is unchanged): window depth as the DEPTH24 buffer holds it,
// read back as float (d / (2^24 - 1), 1.0 = cleared), perspective-correct barycentrics of the visible face's
// three vertices, and the face index; every pointer may be null.  Upstream DIRT's G-buffer programs
// (csrc/shaders.cpp:2187-2221) saved barycentrics, 1/gl_FragCoord.w and the face's vertex indices.
struct GbufOut {
    float *depth;         // [B,H,W]
    float *bary;          // [B,H,W,3]
    int32_t *face;        // [B,H,W], -1 background
};

// FUSED (frames of at most kFusedMaxF faces, Gouraud): no setup launch and no bins -- every workgroup sets up
// all faces of its frame itself into LDS (one face per thread, clipping included) and filters them against
// its tile (the overflow path's all-records filter, reading LDS); the workgroup of tile 0 writes the records
// and FaceData of its frame to `saved` for the backward.  One launch instead of two for small scenes.
constexpr int kFusedMaxF = 32;
// ... and of at most kFusedMaxTiles tiles in the batch: every workgroup repeats the frame's setup
// (~1 us of dependent latency at the start of its life), which a large frame's many rounds of workgroups would
// pay again and again -- past a few rounds the separate setup launch (~5 us) and the bins are cheaper
#ifndef DIRT_FUSED_MAX_TILES
#define DIRT_FUSED_MAX_TILES 8192
#endif
constexpr int64_t kFusedMaxTiles = DIRT_FUSED_MAX_TILES;

// Automatic deep-scene culling (dirt_raster.hip DeepAuto): `host` null = off.  Sampled workgroups count long lists
// into count slot `slot` of the scratch's flag area; the first workgroup reports the previous launch on this scratch
// (generation `prev_gen`, 0 = none, which counted into slot ^ 1) to the host-mapped word if it was deep, then
// clears that slot.
struct DeepArgs {
    uint32_t *host;
    uint32_t gen, prev_gen, slot;
};

// NOPIX (Gouraud): coverage-only resolve for dirt_rasterise_bwd_recompute -- the g-buffer and the
// neighbour-coverage bits the backward reads, no pixels (no background or colour loads, no pixel stores).
template <int CC, int AB = 0, int SH = DIRT_SHADER_GOURAUD, bool GB = false, bool FUSED = false, bool NOPIX = false,
          bool OCC = false, bool RESOLVE = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256), amdgpu_waves_per_eu(SH == DIRT_SHADER_GOURAUD && CC > 0 ? DIRT_RASTER_WAVES : 1))) DIRT_RASTER_ATTR void raster_kernel(const float *__restrict__ background, const float *__restrict__ colors,
                                                     const Rec *__restrict__ recs, const FaceData *__restrict__ fdata,
                                                     const uint32_t *__restrict__ counts, uint32_t *__restrict__ flag,
                                                     const uint2 *__restrict__ bins, uint32_t slab,
                                                     int B, int H, int W, int Cdyn, int V, int F, TileGrid tg, int cshift,
                                                     int nctx, int ncoarse, int64_t nrec, float *__restrict__ pixels,
                                                     int32_t *__restrict__ gbuffer, uint8_t *__restrict__ covbits,
                                                     float *__restrict__ zero_a,
                                                     int64_t nzero_a, float *__restrict__ zero_b, int64_t nzero_b,
                                                     const float *__restrict__ verts, const float *__restrict__ cam,
                                                     int sid, int tcb, GbufOut gbo = GbufOut{},
                                                     const int32_t *__restrict__ faces = nullptr,
                                                     const uint32_t *__restrict__ stash_hdr = nullptr,
                                                     const DeepArgs dga = DeepArgs{},
                                                     const int32_t *__restrict__ gb_in = nullptr)
{
    constexpr bool kNoDepth = SH == DIRT_SHADER_HILL;
    static_assert(!(GB && kNoDepth), "hill has no depth buffer");
    static_assert(!FUSED || SH == DIRT_SHADER_GOURAUD, "the fused small-scene forward is Gouraud only");
    static_assert(!NOPIX || (SH == DIRT_SHADER_GOURAUD && !GB), "the coverage-only resolve is Gouraud only");
    // RESOLVE (dirt_rasterise_fwd_resolve): a render sharing its geometry with an earlier forward -- no bins, no
    // visibility pass: the visible record comes from that forward's g-buffer (`gb_in`), the rest is the resolve below,
    // which then writes this render's own copy of the g-buffer word and leaves the coverage bits alone
    static_assert(!RESOLVE || (SH == DIRT_SHADER_GOURAUD && !GB && !FUSED && !NOPIX && !OCC), "resolve-only: plain Gouraud");
    // FUSED: the frame's records and FaceData, set up in LDS by this workgroup
    __shared__ Rec s_recs[FUSED ? (1 + kExtraPerFace) * kFusedMaxF : 1];
    __shared__ FaceData s_fd[FUSED ? kFusedMaxF : 1];
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
#ifndef DIRT_RASTER_REMAT_IJ
#define DIRT_RASTER_REMAT_IJ 1
#endif
    const int pi = tx * kTile + lx, pj = ty * kTile + ly;  // this lane's pixel (the resolve recomputes it: i, j)
    const int dx = lx * 256, dy = ly * 256;  // offset from the tile origin (sub-pixels)
    const float fxl = (float)pi + 0.5f, fyl = (float)pj + 0.5f;
    const Rec *frame_recs = FUSED ? s_recs : recs + (int64_t)b * nrec;
    const FaceData *fdata_frame = FUSED ? s_fd : fdata + (int64_t)b * F;
    if constexpr (FUSED) {
        if (t < F) {
            bool oob;
            // (only the workgroup of tile 0 counts the R5 deviations: every workgroup repeats the frame's setup)
            s_fd[t] = setup_face_into(verts + (int64_t)b * V * 4, faces + ((int64_t)b * F + t) * 3, V, F, W, H, t,
                                      s_recs, oob, blockIdx.x == 0 ? flag : nullptr);
            if (oob) atomicOr(flag, 1u);
        }
        __syncthreads();
        if (blockIdx.x == 0) {
            // publish the frame's records and FaceData for the backward (plain stores; the backward is a
            // later launch)
            Rec *gr = const_cast<Rec *>(recs) + (int64_t)b * nrec;
            for (int k = t; k < (int)nrec; k += 256) {
                const int f = face_of_record(k, F);
                const int s = k < F ? 0 : (k - F) - (f * kExtraPerFace) + 1;
                if (k < F || s < s_fd[f].nsub) gr[k] = s_recs[k];
            }
            if (t < F) const_cast<FaceData *>(fdata)[(int64_t)b * F + t] = s_fd[t];
        }
    }


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
        // (the lane index from an opaque mbcnt: recomputed here instead of kept live across the chunk loop)
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = chunk + wave * kFilterBlock + u * 64 + ln;
            ev[u] = slab_bins[min(idx, slab - 1u)];
        }
    };
    if (AB & 512) {
        // ablation: one extra dependent global round trip before the first slab loads (how exposed is the
        // workgroup's initial load latency?)
        uint32_t dep = flag[kParQ] & 0u;
        asm volatile("" : "+v"(dep));
        slab_bins += dep;
    }
    if (!FUSED && slab > 0 && !(AB & 8)) load_chunk(0);
    // This forward's setup zeroed the other count set, so the count is the sum of both (no dependent
    // parity load); F == 0: setup did not run.  FUSED: no bins (the count sets stay clean), every record
    // of the frame is filtered (the overflow path)
    const uint32_t raw = RESOLVE ? 0u : FUSED ? 0xffffffffu
                               : F > 0 ? counts[cc * kCountStride] + counts[((int64_t)B * ncoarse + cc) * kCountStride] : 0u;
    if (!FUSED && !RESOLVE && blockIdx.x == 0 && blockIdx.y == 0 && t == 0 && !(AB & 16)) flag[kParQ] = (flag[kParP] & 1u) ^ 1u;
    if (dga.host != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && t == 0) {
        // automatic deep culling: report whether the previous launch on this scratch was deep (to the host-mapped
        // word the host reads when it picks the next launch's instantiation), then clear its count slot
        uint32_t *prev = &flag[kDeepCnt + 4 * (dga.slot ^ 1u)];
        const uint32_t sampled = gridDim.y * ((gridDim.x + kDeepSample - 1) / kDeepSample);
        if (dga.prev_gen != 0u && *prev >= max(1u, sampled / kDeepFrac))
            __hip_atomic_store(dga.host, dga.prev_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *prev = 0u;
    }
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
    // the recompute backward's coverage pass: nothing more to do on a stash hit (the workspace already holds this
    // geometry's g-buffer and coverage bits; the Q parity above republished the value it had, setup having skipped)
    if (NOPIX && stash_hdr != nullptr && stash_hit(stash_hdr)) return;
    // an overflowed slab (more pairs than its capacity): filter every record of the frame instead
    const bool overflow = FUSED || raw > slab;
    const uint32_t n_items = overflow ? (uint32_t)nrec : raw;
    // tile rectangle relative to the coarse tile
    const uint32_t rx0 = (uint32_t)(ti0 - (cx << cshift)), rx1 = rx0 + kTile - 1;
    const uint32_t ry0 = (uint32_t)(tj0 - (cy << cshift)), ry1 = ry0 + kTile - 1;

    if (RESOLVE) {
        // (no visibility pass)
    } else if (AB & 8) {
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
            // (wave-uniform: scalar registers, not four VGPRs live through the staging rounds)
            for (int w = 0; w < kStrips; ++w) pre[w + 1] = pre[w] + __builtin_amdgcn_readfirstlane(t_nw[par][w]);
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
                    // automatic deep culling: one workgroup in kDeepSample counts the long lists of its wave 0 (one
                    // non-returning atomic per such staging round: the counter is a single word)
                    if (dga.host != nullptr && wave == 0 && lane == 0 && (blockIdx.x & (kDeepSample - 1)) == 0 &&
                        ns > kDeepMark)
                        atomicAdd(&flag[kDeepCnt + 4 * dga.slot], 1u);
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
#if DIRT_RASTER_HZ
                    if (OCC && !kNoDepth && ns > DIRT_RASTER_OCC_MIN)
                        // (readfirstlane: the call returns in a VGPR, and a divergent-looking ns would turn the
                        // list walks' uniform loop control into exec-masked vector code)
                        ns = __builtin_amdgcn_readfirstlane(
                            occluder_cull(t_ent, t_wl[wave], ns, wave_ox(wave), wave_oy(wave), ti0, tj0));
#endif
                    int base = 0;
                    // (a long list -- large overlapping faces -- runs only DIRT_RASTER_HZ_DEEP entries before its
                    // first cull: they cover the block, and the cull drops most of the rest)
                    int seg = (!kNoDepth && DIRT_RASTER_HZ)
                                  ? min(ns, ns >= DIRT_RASTER_HZ_DEEP_N ? DIRT_RASTER_HZ_DEEP : DIRT_RASTER_HZ_MIN)
                                  : ns;
                    int rp = seg;  // first list position not yet run or culled
                    for (;;) {
                        u32x2 oo = *(lds_u32x2 *)&t_wl[wave][base];
                        for (int k = base; k < base + seg; k += 2) {
                            const EntryRegs qa = load_entry_at(t_ent, oo.x), qb = load_entry_at(t_ent, oo.y);
                            oo = *(lds_u32x2 *)&t_wl[wave][k + 2];
                            raster_entry<kNoDepth, false>(qa, frame_recs, pix, pxy, pi, pj, best);
                            raster_entry<kNoDepth, false>(qb, frame_recs, pix, pxy, pi, pj, best);
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
                                                     pxy, pi, pj, best);
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
                                    raster_entry<kNoDepth, false>(qa, frame_recs, pix, pxy, pi, pj, best);
                                    raster_entry<kNoDepth, false>(qb, frame_recs, pix, pxy, pi, pj, best);
                                } else {
                                    raster_entry<kNoDepth, false>(load_entry(t_ent, e0), frame_recs, pix, pxy, pi, pj, best);
                                }
                            }
                        } else {
                            while (mine) {
                                const int bit = (int)__builtin_ctzll(mine);
                                mine &= mine - 1;
                                const EntryRegs q = load_entry(t_ent, c0 + bit);
                                if ((big >> bit) & 1)
                                    raster_entry<kNoDepth, true>(q, frame_recs, pix, pxy, pi, pj, best);
                                else
                                    raster_entry<kNoDepth, false>(q, frame_recs, pix, pxy, pi, pj, best);
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
            if (!FUSED && !overflow && chunk + kStrips * kFilterBlock < n_items) {
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
#if DIRT_RASTER_REMAT_IJ
    // the lane's pixel again, from an opaque copy of threadIdx.x: the compiler cannot reuse the values computed
    // before the chunk loop, so they need not stay live (in VGPRs) across it
    int i, j;
    {
        int t2 = threadIdx.x;
        asm volatile("" : "+v"(t2));
        const int lane2 = t2 & 63, wave2 = __builtin_amdgcn_readfirstlane(t2 >> 6);
        i = tx * kTile + wave_ox(wave2) + lane2 % kWaveW;
        j = ty * kTile + wave_oy(wave2) + lane2 / kWaveW;
    }
#else
    const int i = pi, j = pj;
#endif
    // (the pixel's offset is computed here, after the chunk loop: live across it, it cost a VGPR spill)
    if (!(i < W && j < H)) return;
    const int64_t o = ((int64_t)b * H + (H - 1 - j)) * W + i;
    float *out = pixels + o * C;
    if (AB & 15) {
        gbuffer[o] = (int32_t)best;
        return;
    }
    int32_t best_rec;
    if constexpr (RESOLVE) {
        const int32_t g = gb_in[o];
        best_rec = g >= 0 ? (g & kGbufIndexMask) : -1;
    } else {
        best_rec = best != kKeyInit<kNoDepth> ? key_rec(key_low<kNoDepth>(best), F) : -1;
    }
    if (best_rec < 0) {
        gbuffer[o] = -1;
        if constexpr (GB) {
            if (gbo.depth) gbo.depth[o] = 1.0f;
            if (gbo.bary) {
                gbo.bary[o * 3] = 0.0f;
                gbo.bary[o * 3 + 1] = 0.0f;
                gbo.bary[o * 3 + 2] = 0.0f;
            }
            if (gbo.face) gbo.face[o] = -1;
        }
        if constexpr (SH == DIRT_SHADER_GOURAUD && !RESOLVE) covbits[o] = 0;
        if constexpr (!NOPIX) {
#pragma unroll
            for (int c2 = 0; c2 < CM; ++c2)
                if (c2 < C) out[c2] = kNoDepth ? 0.0f : background[o * C + c2];  // (hill: no background copy)
        }
        PHASE_TS(4);
        PHASE_TS(5);
        return;
    }
    int32_t best_q = best_rec;
    if (AB & 2048) {
        // ablation: one extra dependent global round trip between the depth resolve and the record loads
        uint32_t z0, z1;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z0) : "v"(best_rec));
        const uint32_t w = flag[kParQ + z0];
        asm volatile("v_mov_b32 %0, 0" : "=v"(z1) : "v"(w));
        best_q += (int32_t)z1;
    }
    const Rec &r = frame_recs[best_q];
    // the record's first 64 B as one batch of loads (four dwordx4 in flight with the FaceData): reading
    // fields on demand lets the compiler split them into dependent rounds behind the range test below
    const RasterPart rp = *reinterpret_cast<const RasterPart *>(&r);
    const FaceData fd = fdata_frame[face_of_record(best_rec, F)];
    gbuffer[o] = best_rec | (fd.clipped ? kGbufMulti : 0);
    int64_t E[3];
    float lam[3] = {0.0f, 0.0f, 0.0f};
    float fE[3];
    // Small winners (every |A|, |B| < 2^14: edges shorter than 64 px) -- the pixel centre lies inside the
    // triangle, so |px - X0|, |py - Y0| <= the bbox extent < 2^14 and |D| < 2^29: E = A dx + B dy (+ D) in
    // int32 with 24-bit multiplies, exact (|E| < 2^30), instead of six 32x32->64 multiply-adds; the same
    // integers, so the same floats.  Otherwise (a wave-uniform branch) the int64 path below.
    bool small_rec = true;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        small_rec = small_rec && (uint32_t)(rp.A[k] + kResolveSmall) < 2u * kResolveSmall &&
                    (uint32_t)(rp.B[k] + kResolveSmall) < 2u * kResolveSmall;
    const bool resolve_small = DIRT_RASTER_RESOLVE32 && __builtin_amdgcn_ballot_w64(!small_rec) == 0;
    if (resolve_small) {
        const int32_t dx = i * 256 + 128 - rp.X0, dy = j * 256 + 128 - rp.Y0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int32_t e = __mul24(rp.A[k], dx) + __mul24(rp.B[k], dy) + (k == 0 ? (int32_t)rp.D : 0);
            E[k] = e;
            fE[k] = (float)e;
        }
    } else {
        edge_values(rp, i, j, E);
        // R6 with the int64 -> float conversions done in int32 when every value of the wave fits (the same
        // integers, so the same floats); non-clipped faces skip the identity basis (m_k >= +0 are exact)
        bool fits = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) fits = fits && E[k] == (int64_t)(int32_t)E[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) fE[k] = (float)(int32_t)E[k];
        if (__builtin_amdgcn_ballot_w64(!fits) != 0) {  // (a real branch: the int64 conversions are not inlined)
            const float3 w = i64x3_to_f32(E[0], E[1], E[2]);
            fE[0] = w.x; fE[1] = w.y; fE[2] = w.z;
        }
    }
    // 1/w: the FaceData's of a non-clipped face (its record's second half is never written), the record's
    // own of a clipped sub-triangle
    float iwv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) iwv[k] = fd.clipped ? r.iw[k] : fd.q[k];
    parent_lambda_f(r, iwv, fE, fd.clipped == 0, lam);
    if constexpr (GB) {
        if (gbo.depth) gbo.depth[o] = (float)(uint32_t)(best >> 32) / 16777215.0f;
        if (gbo.bary) {
            gbo.bary[o * 3] = lam[0];
            gbo.bary[o * 3 + 1] = lam[1];
            gbo.bary[o * 3 + 2] = lam[2];
        }
        if (gbo.face) gbo.face[o] = face_of_record(best_rec, F);
    }
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
        if constexpr (NOPIX) {
            // (coverage only: the caller holds the pixels)
        } else if (AB & 64) {
            for (int k = 0; k < C; ++k) out[k] = lam[k % 3];
        } else {
            const float *cb = colors + (int64_t)b * V * C;
            if (AB & 1024) {
                // ablation: one extra dependent global round trip between the FaceData and the colour loads
                uint32_t z0, z1;
                asm volatile("v_mov_b32 %0, 0" : "=v"(z0) : "v"(fd.v[0]));
                const uint32_t w = flag[kParQ + z0];
                asm volatile("v_mov_b32 %0, 0" : "=v"(z1) : "v"(w));
                cb += z1;
            }
            const float *c0 = cb + (int64_t)fd.v[0] * C, *c1 = cb + (int64_t)fd.v[1] * C, *c2 = cb + (int64_t)fd.v[2] * C;
            for (int k = 0; k < C; ++k) out[k] = (lam[0] * c0[k] + lam[1] * c1[k]) + lam[2] * c2[k];
        }
        if (!RESOLVE)
        covbits[o] = (AB & 32) ? (uint8_t)0
                               : (uint8_t)neighbour_coverage(rp, E, fd.clipped != 0, best_rec, frame_recs,
                                                             fdata_frame, F, face_of_record(best_rec, F), i, j,
                                                             resolve_small);
        PHASE_TS(5);
    }
}
