// Part of dirt_raster.hip's translation unit: included inside its anonymous namespace after the shared
// definitions (raster_rules.h, oceanic.h, hill.h, the layout and error helpers).  Not a standalone header.

// ------------------------------------------------------------------------------------------------
// K5: backward
//
// One workgroup per TWX x TH tile (16 x 16: 256 threads; TWX = 32 or TH = 8 variants), one lane per pixel.  Every contribution of a lane goes to
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
#ifndef DIRT_GRAD_GM1_WAVES
#define DIRT_GRAD_GM1_WAVES 8  // C = 3, vertex gradients only (64 VGPRs without SLP vectorisation, Makefile)
#endif
#ifndef DIRT_GRAD_ATTR
#define DIRT_GRAD_ATTR
#endif

// window-transform constants of the chain rule, computed on the host (IEEE, as the oracle)
struct NdcScale {
    float inv_hw, inv_hh, half_w, half_h;
};

// Backward tile width: 16 (16x16 tiles, 256-thread workgroups) or 32 (32x16, 512 threads: 1.20 instead of
// 1.27 staged pixels per pixel, and records spanning both halves are inserted, loaded and flushed once).
#ifndef DIRT_GRAD_TILE_W
#define DIRT_GRAD_TILE_W 16
#endif
constexpr int kGradTileW = DIRT_GRAD_TILE_W;
// Backward tile height: 16 rows (256 threads at TWX = 16) or 8 (128 threads: twice the workgroups, for frames
// whose tile count alone does not fill the chip twice over).  RGB / one channel and the wide paths separately.
#ifndef DIRT_GRAD_TILE_H
#define DIRT_GRAD_TILE_H 16
#endif
#ifndef DIRT_GRAD_TILE_H_WIDE
#define DIRT_GRAD_TILE_H_WIDE 16
#endif
__host__ __device__ constexpr int grad_tile_h(int C) { return C == 1 || C == 3 ? DIRT_GRAD_TILE_H : DIRT_GRAD_TILE_H_WIDE; }
// staged tile with a one-pixel border: row stride TWX + 2, TH + 2 rows
template <int TWX, int TH>
struct GradGeom {
    static constexpr int NT = TWX * TH;           // threads
    static constexpr int HX = TWX + 2;            // staged row stride
    static constexpr int HY = TH + 2;
    static constexpr int PIX = HX * HY;
};
constexpr int kSlots = 64;         // distinct records of a tile kept in LDS (typ. 10-40)
constexpr int kNoSlot = -3;        // record not in the slot table: read it from global memory
static_assert(kSlots <= 128, "slot ids (0 .. kSlots-1) are stored as int8");

// The records visible in a tile (its own pixels; the halo's are not needed: pair coverage comes from the
// forward's bits): keys for the run-tail ranges of the reduction and vertex ids for the flush.  Each lane reads
// its own pixel's record itself (phase A, right after its g-buffer word), so nothing else is kept here.
struct SlotTable {
    int32_t key[kSlots];     // g-buffer word (record index | clipped flag), -1 = free
    int8_t list[kSlots];     // occupied slots in insertion order
    int32_t v[3][kSlots];    // vertex ids, indexed by list position
    int32_t n;
};

// A record is "small" when every |A|, |B| < 2^14 (edges shorter than 64 px): at a pixel it covers, every
// offset to its vertex 0 is below 2^14 sub-pixels, so E = A dx + B dy (+ D) is exact in int32 with 24-bit
// multiplies (|E| < 2^30), as in the raster's resolve; larger records take the int64 edge values.
constexpr int32_t kGradSmallEdge = 1 << 14;

__device__ __forceinline__ int slot_hash(int32_t key) { return (int)(((uint32_t)key * 2654435761u) >> 25) & (kSlots - 1); }

// Insert `key` for every lane with `want` (called by the whole wave, converged): probes advance in
// lockstep, and the lanes that created a slot append it to the slot list with one atomic per wave.
// Returns the slot, kNoSlot if the table is full, -1 where !want; a lane that created its slot gets the slot's
// list position in *list_pos (others: unchanged).
__device__ __forceinline__ int slot_insert_wave(SlotTable &T, int32_t key, bool want, int *list_pos)
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
        const int p = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (fresh) {
            T.list[p] = (int8_t)result;
            *list_pos = p;
        }
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
    } else if constexpr (CP == 8) {
        // 5..8 channels at a 32-B stride: each operand is two ds_read_b128 instead of C ds_read_b32
        float Gp[8], Gq[8], Ip[8], Iq[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<float4 *>(&Gp[4 * h]) = *reinterpret_cast<const float4 *>(&s_G[k * 8 + 4 * h]);
            *reinterpret_cast<float4 *>(&Gq[4 * h]) = *reinterpret_cast<const float4 *>(&s_G[k2 * 8 + 4 * h]);
            *reinterpret_cast<float4 *>(&Ip[4 * h]) = *reinterpret_cast<const float4 *>(&s_I[k * 8 + 4 * h]);
            *reinterpret_cast<float4 *>(&Iq[4 * h]) = *reinterpret_cast<const float4 *>(&s_I[k2 * 8 + 4 * h]);
        }
#pragma unroll
        for (int c = 0; c < CM; ++c)
            if (c < C) a += (Gp[c] + Gq[c]) * (Iq[c] - Ip[c]);
    } else {
        for (int c = 0; c < C; ++c) a += (s_G[k * CP + c] + s_G[k2 * CP + c]) * (s_I[k2 * CP + c] - s_I[k * CP + c]);
    }
    return (g1 != -2 && g2 != -2) ? -0.5f * a : 0.0f;
}

// pair_scalar with pixel p's operands in registers (its g-buffer word, G and I): s = -0.5 sum_c (G(p)+G(q))
// (I(q)-I(p)), the same operand order as pair_scalar; 0 when either pixel is outside the frame
template <int CP, int CM>
__device__ __forceinline__ float pair_scalar_own(int32_t g1, const float *Gp, const float *Ip, const int32_t *s_gb,
                                                 const float *s_G, const float *s_I, int k2, int C)
{
    const int32_t g2 = s_gb[k2];
    float Gq[CP > CM ? CP : CM], Iq[CP > CM ? CP : CM];
    if constexpr (CP == 8) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<float4 *>(&Gq[4 * h]) = *reinterpret_cast<const float4 *>(&s_G[k2 * 8 + 4 * h]);
            *reinterpret_cast<float4 *>(&Iq[4 * h]) = *reinterpret_cast<const float4 *>(&s_I[k2 * 8 + 4 * h]);
        }
    } else {
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            Gq[c] = c < C ? s_G[k2 * CP + c] : 0.0f;
            Iq[c] = c < C ? s_I[k2 * CP + c] : 0.0f;
        }
    }
    float a = 0.0f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
        if (c < C) a += (Gp[c] + Gq[c]) * (Iq[c] - Ip[c]);
    return (g1 != -2 && g2 != -2) ? -0.5f * a : 0.0f;
}

// Index (0..15) of the first lane of this lane's run of equal `key` in its 16-lane DPP row.
__device__ __forceinline__ int run_start(int key, int lx)  // lx: lane index within its 16-lane DPP row
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
// GM: which gradients the launch produces -- bit 0 the vertices' (the pairs), bit 1 the vertex colours' (the
// colour weights); a launch without one of them neither computes, reduces nor flushes its values.
template <int CC, int AB = 0, int TWX = kGradTileW, int TH = grad_tile_h(CC), int GM = 3>
__global__ __attribute__((amdgpu_flat_work_group_size(1, GradGeom<TWX, TH>::NT),
                          amdgpu_waves_per_eu(CC == 3 ? (GM == 1 ? DIRT_GRAD_GM1_WAVES : DIRT_GRAD_WAVES_C3) : DIRT_GRAD_WAVES))) DIRT_GRAD_ATTR void grad_kernel(const float *__restrict__ pixels, const float *__restrict__ grad_pixels,
                                                   const int32_t *__restrict__ gbuffer, const uint8_t *__restrict__ covbits,
                                                   const Rec *__restrict__ recs,
                                                   const FaceData *__restrict__ fdata, int B, int H, int W, int Cdyn,
                                                   int V, int F, TileGrid tg, int64_t nrec, float *__restrict__ grad_verts,
                                                   float *__restrict__ grad_colors, float *__restrict__ grad_bg,
                                                   const NdcScale ns, uint32_t *__restrict__ stash_flip = nullptr)
{    // recompute backward: flip the gradient stash's parity for the next call (dirt_raster.hip stash_check_kernel)
    if (stash_flip != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) stash_flip[0] ^= 1u;

    constexpr int CM = CC > 0 ? CC : DIRT_MAX_CHANNELS;
    constexpr int NT = GradGeom<TWX, TH>::NT, kHalo = GradGeom<TWX, TH>::HX, kHaloPix = GradGeom<TWX, TH>::PIX;
    // LDS pixel stride: float4 for RGB, two float4 for 5..8 channels (wide LDS reads)
    constexpr int CP = CM == 3 ? 4 : (CM > 4 && CM <= 8) ? 8 : CM;
    static_assert(GM >= 1 && GM <= 3, "at least one of the vertex and colour gradients");
    constexpr int kNVV = (GM & 1) ? 9 : 0;  // vertex values per record (x, y, w of three vertices), then colours
    constexpr int NVM = kNVV + ((GM & 2) ? 3 * CM : 0);
    const int C = CC > 0 ? CC : Cdyn;
    const int NV = kNVV + ((GM & 2) ? 3 * C : 0);
#if defined(DIRT_GRAD_LDS_PAD) && DIRT_GRAD_LDS_PAD > 0
    __shared__ volatile char occupancy_probe[DIRT_GRAD_LDS_PAD];  // experiment: caps workgroups per CU
    if (threadIdx.x == 1023) occupancy_probe[0] = 0;
#endif
    // RGB (kPacked): one 32-B record per staged pixel, {G.xyz, g-buffer word} and {I.xyz, coverage bits}, the two
    // 16-B halves swapped on odd region rows.  A neighbour's operands are then two ds_read_b128 (4 LDS cycles each,
    // conflict-free over every lane group for the own pixel and its four neighbours) instead of two ds_read_b96
    // (8 cycles each, 2-way conflicts at the 18-pixel row stride) plus the g-buffer and coverage reads: the pair
    // phase's LDS cycles per wave 190 -> 40 by the MI355X bank rule (MI355X_MICROARCH.md LDS table), where they
    // were a third bank conflicts (profiles/r06/pmc_ablate_lds_c3.txt).  Other channel counts keep separate arrays.
    constexpr bool kPacked = CM == 3;
    __shared__ int32_t s_gb[kPacked ? 1 : kHaloPix];
    __shared__ uint8_t s_cov[kPacked ? 1 : kHaloPix];  // neighbour_coverage() bits of the pixel's face (forward)
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
    // packed layout: the half holding {G, g-buffer word} of region pixel k on a region row of parity `par` (the
    // other half holds {I, coverage bits})
    auto px_half = [&](int k, int par, int h) -> float4 { return reinterpret_cast<const float4 *>(s_u)[2 * k + (h ^ par)]; };
    auto ld_gb = [&](int k, int par) -> int32_t {
        if constexpr (kPacked) return __float_as_int(s_u[8 * k + 4 * par + 3]);
        else return s_gb[k];
    };
    auto ld_cov = [&](int k, int par) -> uint32_t {
        if constexpr (kPacked) return (uint32_t)__float_as_int(s_u[8 * k + 4 * (par ^ 1) + 3]);
        else return s_cov[k];
    };
    // pair scalar of the pair (klo, klo + x) (axis 0) or (klo, klo + kHalo) (axis 1)
    auto pair_s = [&](int axis, int klo) -> float {
        if constexpr (kPacked) {
            // (the slow path's pairs: the same operands and operation order as pair_scalar)
            const int par = (klo / kHalo) & 1, k2 = klo + (axis == 0 ? 1 : kHalo), par2 = axis == 0 ? par : par ^ 1;
            const float4 Gp = px_half(klo, par, 0), Ip = px_half(klo, par, 1);
            const float4 Gq = px_half(k2, par2, 0), Iq = px_half(k2, par2, 1);
            float a = (Gp.x + Gq.x) * (Iq.x - Ip.x);
            a = a + (Gp.y + Gq.y) * (Iq.y - Ip.y);
            a = a + (Gp.z + Gq.z) * (Iq.z - Ip.z);
            return (__float_as_int(Gp.w) != -2 && __float_as_int(Gq.w) != -2) ? -0.5f * a : 0.0f;
        } else if constexpr (kRecompute)
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
    const int t = threadIdx.x, lx = t % TWX, ly = t / TWX;
    const int lr = lx & 15;  // lane within its 16-lane DPP row (a pixel row, or half of one at TWX = 32)
    const int i = tx * TWX + lx, j = ty * TH + ly;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const FaceData *fdata_frame = fdata + (int64_t)b * F;
    // uniform: readfirstlane (convergent) keeps the divisions at the top instead of in every pair branch
    const float inv_hw = ns.inv_hw, inv_hh = ns.inv_hh;  // 2/W, 2/H from the host (no division in the kernel)
    const int kme = (ly + 1) * kHalo + (lx + 1);
    const bool in_frame = i < W && j < H;

    // ---- phase A: stage g-buffer / G / I of the tile + one-pixel halo, pair scalars, slot table
    PHASE_TS(0);
    for (int k = t; k < kSlots; k += NT) {
        T.key[k] = -1;
        s_tcnt[k] = 0;
    }
    if (t == 0) T.n = 0;
    const int hi0 = tx * TWX - 1, hj0 = ty * TH - 1;
    // the staged pixels' g-buffer words and G / I (for the staged pair scalars below, !kRecompute)
    int32_t gbv[2];
    float Gv[2][CM], Iv[2][CM];
    // The lane's own pixel: its g-buffer word (loaded with the staging loads) and its record's edge part and FaceData,
    // read by the lane itself right after the staging round trip -- in flight across the LDS stores, the first barrier
    // and the slot inserts, instead of a second round trip after them by the slot table's fill (phase B is the first
    // reader; the records of a wave's pixels are a handful, so the loads are mostly L1 hits).
    int32_t g_own = -2;
    EdgePart me{};
    FaceData mfd{};
    {
        // every load of both passes in flight before the first LDS store (kHaloPix <= 2 * NT)
        static_assert(kHaloPix <= 2 * NT, "two staging passes");
        // frame base pointers (64-bit, uniform) + 32-bit per-lane offsets: H * W * C < 2^29
        const int64_t fpix = (int64_t)b * H * W;
        const int32_t *gb_f = gbuffer + fpix;
        const uint8_t *cov_f = covbits + fpix;
        const float *gp_f = grad_pixels + fpix * C, *px_f = pixels + fpix * C;
        uint32_t cvv[2];
        bool ok[2];
        if (in_frame) g_own = gb_f[(uint32_t)((H - 1 - j) * W + i)];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = t + NT * u;
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
            const int k = t + NT * u;
            if (k >= kHaloPix) continue;
            // a background pixel with a non-finite value (G-buffers rendered over -inf,
            // samples/deferred.py:67,81) defines no image difference: staged as "outside the frame", so
            // none of its pairs carries vertex gradient; its grad_background stays G
            if (gbv[u] == -1) {
                bool fin = true;
#pragma unroll
                for (int c = 0; c < CM; ++c)
                    if (c < C) fin = fin && __builtin_isfinite(Iv[u][c]);
                gbv[u] = fin ? -1 : -2;
            }
            if constexpr (kPacked) {
                // (outside the frame: zeros and the -2 word; every reader selects them away)
                const int par = (k / kHalo) & 1;
                float4 *d = reinterpret_cast<float4 *>(s_u) + 2 * k;
                d[par] = ok[u] ? make_float4(Gv[u][0], Gv[u][1], Gv[u][2], __int_as_float(gbv[u]))
                               : make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-2));
                d[par ^ 1] = ok[u] ? make_float4(Iv[u][0], Iv[u][1], Iv[u][2], __int_as_float((int)cvv[u]))
                                   : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                continue;
            } else {
                s_gb[k] = gbv[u];
                s_cov[k] = (uint8_t)cvv[u];
            }
            if (!ok[u]) continue;
            if constexpr (CP == 8) {
                float g8[8], i8[8];
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    g8[c] = c < CM && c < C ? Gv[u][c < CM ? c : 0] : 0.0f;
                    i8[c] = c < CM && c < C ? Iv[u][c < CM ? c : 0] : 0.0f;
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    *reinterpret_cast<float4 *>(&s_G[k * 8 + 4 * h]) = *reinterpret_cast<const float4 *>(&g8[4 * h]);
                    *reinterpret_cast<float4 *>(&s_I[k * 8 + 4 * h]) = *reinterpret_cast<const float4 *>(&i8[4 * h]);
                }
            } else {
#pragma unroll
                for (int c = 0; c < CM; ++c)
                    if (c < C) {
                        s_G[k * CP + c] = Gv[u][c];
                        s_I[k * CP + c] = Iv[u][c];
                    }
            }
        }
        // (after the stores: issued before them, the loads would make the stores' wait cover them too)
        if (g_own >= 0) {
            const int32_t ri = g_own & kGbufIndexMask;
            me = *reinterpret_cast<const EdgePart *>(&frame_recs[ri]);
            mfd = fdata_frame[face_of_record(ri, F)];
        }
    }
    __syncthreads();
    PHASE_TS(1);
    const int prow = (ly + 1) & 1;  // parity of this pixel's region row (packed layout)
    const int32_t gp = in_frame ? ld_gb(kme, prow) : -2;
    int sp, fpos = -1;  // the own pixel's slot; the list position of a slot this lane created
    {
        // the tile's records (run heads only; all distinct keys may not fit: the rest go to global memory)
        const int32_t g = ld_gb(kme, prow);
        const int key = g >= 0 ? g : -1;
        const int start = run_start(key, lr);
        int slot = slot_insert_wave(T, key, key >= 0 && start == lr, &fpos);
        if (key >= 0 && start == lr && slot >= 0) atomicAdd(&s_tcnt[slot], 1);  // one run (one tail later)
        slot = __shfl(slot, (t & 48) + start, 64);
        sp = key >= 0 ? slot : -1;
    }
    if constexpr (!kRecompute) {
        // staged pair scalars: the lane that staged region pixel k computes the pairs starting there that phase B
        // reads -- (k, k+x) for hx in 0..TWX, hy in 1..16 and (k, k+y) for hx in 1..TWX, hy in 0..16 -- with k's own
        // G / I still in its registers (only the neighbour's come from LDS)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = t + NT * u;
            if (k >= kHaloPix) continue;
            const int hx = k % kHalo, hy = k / kHalo;
            const bool need_x = hx <= TWX && hy >= 1 && hy <= TH;
            const bool need_y = hx >= 1 && hx <= TWX && hy <= TH;
            if (need_x) s_sx[k] = pair_scalar_own<CP, CM>(gbv[u], Gv[u], Iv[u], s_gb, s_G, s_I, k + 1, C);
            if (need_y) s_sy[k] = pair_scalar_own<CP, CM>(gbv[u], Gv[u], Iv[u], s_gb, s_G, s_I, k + kHalo, C);
        }
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
        // inclusive scan over the wave with DPP (no LDS round trips on wave 0's way into phase B): within each
        // 16-lane row by row_shr 1, 2, 4, 8, then across rows by row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3)
        int inc = cnt;
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xF, 0xF, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xF, 0xF, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xF, 0xF, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xF, 0xF, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x142, 0xA, 0xF, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x143, 0xC, 0xF, false);
        if (t < nslots) {
            s_toff[sl] = inc - cnt;
            s_lbeg[t] = inc - cnt;
            s_lcnt[t] = cnt;
        }
    }
    // a slot's creator (a run head showing its record) holds the record's FaceData: its vertex ids for the flush
    // (read after the barriers of phase C)
    if (fpos >= 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) T.v[k][fpos] = mfd.v[k];
    }
    PHASE_TS(4);

    // ---- phase B: per-pixel contributions to the face visible at this pixel
    const int32_t rp = gp >= 0 ? (gp & kGbufIndexMask) : gp;
    if (in_frame && grad_bg != nullptr) {  // (null: the caller needs no background gradient)
        float *gbg_f = grad_bg + (int64_t)b * H * W * C;
        const uint32_t o = (uint32_t)((H - 1 - j) * W + i);
        float *gbq = gbg_f + o * (uint32_t)C;  // (RGB: one global_store_dwordx3)
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            const float gv = kPacked ? s_u[8 * kme + 4 * prow + c] : s_G[kme * CP + c];
            // (non-temporal: nothing in this pipeline reads grad_background back, so its lines need not
            // stay dirty in L2 for the write-back that ends the launch)
            if (c < C) __builtin_nontemporal_store(rp < 0 ? gv : 0.0f, &gbq[c]);
        }
    }

    float acc[NVM];
#pragma unroll
    for (int v = 0; v < NVM; ++v) acc[v] = 0.0f;
    if (rp >= 0) {
        // Ownership decisions (coverage tests) are exact int64; the interpolation weights use fast
        // reciprocals (contributions agree with the oracle to ~1e-6 relative, far inside the 1e-4
        // tolerance the atomic summation order already needs).  The own record's edge part and FaceData
        // were read in phase A (me, mfd).
        const int f = face_of_record(rp, F);
        const bool multi = (gp & kGbufMulti) != 0;
        // the whole own record (the 1/w and basis of clipped faces): its address is recomputed at each use
        // from rp (the asm hides the common subexpression) instead of living in two registers
        auto rec = [&]() -> const Rec & {
            int r2 = rp;
            asm volatile("" : "+v"(r2));
            return frame_recs[r2];
        };
        int32_t mA[3], mB[3];
        float iw0 = mfd.q[0], iw1 = mfd.q[1], iw2 = mfd.q[2];  // 1/w of a non-clipped face
        float fEp[3];
        bool small = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mA[k] = me.A[k];
            mB[k] = me.B[k];
            small = small && mA[k] > -kGradSmallEdge && mA[k] < kGradSmallEdge && mB[k] > -kGradSmallEdge &&
                    mB[k] < kGradSmallEdge;
        }
        if (__builtin_amdgcn_ballot_w64(multi) != 0 && multi) {
            const Rec &rr = rec();
            iw0 = rr.iw[0]; iw1 = rr.iw[1]; iw2 = rr.iw[2];
        }
        const float h2d = 0.5f / (float)me.D;  // 1 / (2 D), D = E0 + E1 + E2 (constant over the plane)
        if (small) {
            // E at this pixel (which the record covers): exact in int32, as the raster's resolve
            const int32_t dx = i * 256 + 128 - me.X0, dy = j * 256 + 128 - me.Y0;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                fEp[k] = (float)(__mul24(mA[k], dx) + __mul24(mB[k], dy) + (k == 0 ? (int32_t)me.D : 0));
        } else {
            int64_t Ep[3];
            edge_values(me, i, j, Ep);
#pragma unroll
            for (int k = 0; k < 3; ++k) fEp[k] = fast_i64_to_f32(Ep[k]);
        }
        // the four pairs around the pixel: dir 0 right, 1 left (x axis); 2 up, 3 down (y axis, window).
        // Pass 1 decides ownership (exact integer coverage tests) into 2-bit codes (0 skip, 1 half,
        // 2 whole); pass 2 interpolates and accumulates.  Splitting keeps the coverage tests' and the
        // accumulators' registers apart (occupancy).
        if constexpr ((GM & 1) != 0) {
        PHASE_TS(10 + (fEp[0] == 12345.f));
        if (!(AB & 17) && __builtin_amdgcn_ballot_w64(multi) == 0) {
            // No clipped face in this wave: ownership and accumulation of the four pairs without
            // branches.  A neighbour shows my face iff it shows my record (a non-clipped face has exactly
            // one).  Ownership code: outside the frame 0, background 2, same face 2 for the
            // lower pixel of the pair / 0 for the upper, else 1 + (q's face covers p) - (p's face covers q).
            // The pair weight of vertex k is c_d * m_k with m_k = (2 E_k +- 256 A_k (or B_k)) / w_k =
            // P_k +- Q_k and c_d = code_d * s_d * (W/2 or H/2) / (4D), so the two pairs of an axis fold
            // into (c_0 + c_1) P_k + (c_0 - c_1) Q_k (and the same with the NDC factors for w).
            // packed layout: the own pixel's two halves once, each neighbour's two halves (G, I, its g-buffer word and
            // coverage bits) as two ds_read_b128
            float4 Gme, Ime;
            if constexpr (kPacked) {
                Gme = px_half(kme, prow, 0);
                Ime = px_half(kme, prow, 1);
            }
            const uint32_t covme = kPacked ? (uint32_t)__float_as_int(Ime.w) : ld_cov(kme, prow);
            float cd[4];
#pragma unroll
            for (int dir = 0; dir < 4; ++dir) {
                const int axis = dir >> 1;
                const bool me_low = (dir & 1) == 0;
                const int di = axis == 0 ? (me_low ? 1 : -1) : 0, dj = axis == 1 ? (me_low ? 1 : -1) : 0;
                const int kq = kme + dj * kHalo + di;
                int32_t gq;
                uint32_t covq;  // read unconditionally: the code below is all selects
                float s;
                if constexpr (kPacked) {
                    const int pq = axis == 0 ? prow : prow ^ 1;
                    const float4 Gq = px_half(kq, pq, 0), Iq = px_half(kq, pq, 1);
                    gq = __float_as_int(Gq.w);
                    covq = (uint32_t)__float_as_int(Iq.w);
                    // pair_scalar(klo, khi)'s operands and order: (G(lo) + G(hi)) (I(hi) - I(lo)) per channel
                    const float4 Il = me_low ? Ime : Iq, Ih = me_low ? Iq : Ime;
                    float a = (Gme.x + Gq.x) * (Ih.x - Il.x);
                    a = a + (Gme.y + Gq.y) * (Ih.y - Il.y);
                    a = a + (Gme.z + Gq.z) * (Ih.z - Il.z);
                    s = (gp != -2 && gq != -2) ? -0.5f * a : 0.0f;
                } else {
                    gq = ld_gb(kq, 0);
                    covq = ld_cov(kq, 0);
                    s = pair_s(axis, me_low ? kme : kq);
                }
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
            const int32_t gq = ld_gb(kq, axis == 0 ? prow : prow ^ 1);
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
                const bool mine_covers_other = (ld_cov(kme, prow) >> dir) & 1u;
                const bool other_covers_me = (ld_cov(kq, axis == 0 ? prow : prow ^ 1) >> (dir ^ 1)) & 1u;
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
            // lambda_k / Wm = a_k / sum_k (a_k w_k) = a_k / (2E_0 + 2E_1 + 2E_2 + st_0 + st_1 + st_2) = a_k / (2D)
            // (iw_k w_k = 1, the edge functions sum to the constant D and their steps to 0): no division per
            // pair and nothing to cancel.  For a clipped face these are the weights of its sub-triangle's
            // vertices; they are mapped to the parent's below, once per pixel.
            const float c = omega * s * half * h2d;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float g = c * m[k];
                acc[k * 3 + axis] += g;
                acc[k * 3 + 2] -= g * ndc;
            }
        }
        if (multi) {
            // A clipped face's sub-triangle has vertices that are convex combinations of the parent's (the
            // clip basis rows; w_sub = basis . w), so the parent's lambda_i / Wm = sum_k basis_ki a_k / (2D)
            // (the normalised form lambda = a / sum a, Wm = sum lambda w cancelled on slivers).
            // Linear in the weights: the pixel's accumulated sub-vertex sums are mapped once, all pairs of
            // a lane being owned by its own record.
            const Rec &rr = rec();
            float sub[9];
#pragma unroll
            for (int v = 0; v < 9; ++v) sub[v] = acc[v];
#pragma unroll
            for (int i2 = 0; i2 < 3; ++i2)
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    acc[i2 * 3 + a] = (rr.basis[i2] * sub[a] + rr.basis[3 + i2] * sub[3 + a]) + rr.basis[6 + i2] * sub[6 + a];
        }
        }
        }
        // colour weights last: keeps their registers out of the pair loop's live range
        float lam[3];
        if ((GM & 2) && !(AB & 2) && fast_lambda(rec(), multi, fEp[0] * iw0, fEp[1] * iw1, fEp[2] * iw2, lam)) {
            float Gm[CM];
#pragma unroll
            for (int c = 0; c < CM; ++c) Gm[c] = c < C ? (kPacked ? s_u[8 * kme + 4 * prow + c] : s_G[kme * CP + c]) : 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                for (int c = 0; c < C; ++c) acc[(kNVV + k * C + c) < NVM ? kNVV + k * C + c : 0] = lam[k] * Gm[c];
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
    const int start = run_start(key, lr);
    // 0/1 multipliers: x += shifted(x) * m is one v_fmac with a DPP operand (exact: m is 0 or 1,
    // contributions are finite)
    const float mk1 = lr - 1 >= start ? 1.0f : 0.0f, mk2 = lr - 2 >= start ? 1.0f : 0.0f;
    const float mk4 = lr - 4 >= start ? 1.0f : 0.0f, mk8 = lr - 8 >= start ? 1.0f : 0.0f;
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
    const bool tail = key >= 0 && ((AB & 32) || lr == 15 || kr != key);
    float *gvb = (GM & 1) ? grad_verts + (int64_t)b * V * 4 : nullptr;
    float *gcb = (GM & 2) ? grad_colors + (int64_t)b * V * C : nullptr;
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
            const int32_t vid[3] = {mfd.v[0], mfd.v[1], mfd.v[2]};  // (the lane's own record's face, phase A)
#pragma unroll
            for (int v = 0; v < NVM; ++v) {
                if (v >= NV || acc[v] == 0.0f) continue;
                if (v < kNVV) atomicAdd(gvb + (int64_t)vid[v / 3] * 4 + ((v % 3) == 2 ? 3 : v % 3), acc[v]);
                else atomicAdd(gcb + (int64_t)vid[(v - kNVV) / C] * C + (v - kNVV) % C, acc[v]);
            }
        }
    }
    __syncthreads();
    PHASE_TS(6);

    // ---- phase D: flush.  Thread t handles component t % NV of slot t / NV, so every lane of the
    // workgroup sums one slot's tails in parallel; a slot's components go out as one run of lanes
    // (~3 cache lines of global float atomics per (tile, record)).
    const int n = (AB & 8) ? 0 : nslots;
    // whole records per wave: no record's components straddle two waves, so each record's atomics leave
    // in one wave instruction (the cache lines one atomic instruction touches are what it costs)
    const int rpw = 64 / NV, per_round = (NT / 64) * rpw;
    const int wl = t & 63;
    for (int e0 = 0; e0 < n; e0 += per_round) {
        const int e = e0 + (t >> 6) * rpw + wl / NV, comp_id = wl - (wl / NV) * NV;
        if (wl >= rpw * NV || e >= n) continue;
        const int kv = comp_id < kNVV ? comp_id / 3 : (comp_id - kNVV) / C;
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
        if (comp_id < kNVV) {
            const int c3 = comp_id % 3;
            atomicAdd(gvb + (int64_t)vid * 4 + (c3 == 2 ? 3 : c3), val);
        } else {
            atomicAdd(gcb + (int64_t)vid * C + (comp_id - kNVV) % C, val);
        }
    }
    if (AB & 128) {
        __syncthreads();
        PHASE_TS(7);
    }
}
