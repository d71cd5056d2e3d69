// Part of dirt_raster.hip's translation unit, after grad_kernel.h (its helpers and LDS types).  Not a standalone
// header.
//
// K5p: the backward as a persistent grid (design (b)) -- the same per-tile algorithm as
// grad_kernel (identical arithmetic, so the same gradients up to float-atomic order), with the
// tiles of the batch dealt to a fixed number of workgroups instead of one workgroup per tile.  Experiment behind
// DIRT_GRAD_PERSIST (workgroups per CU); grad_kernel stays the product path until an A/B says otherwise.
#ifndef DIRT_GRAD_PERSIST_WAVES
#define DIRT_GRAD_PERSIST_WAVES 5  // register budget: 96 VGPRs (89 used: 5 waves / SIMD, 5 workgroups per CU; at 80 it spills the
                                   // prefetched staging values right after loading them)
#endif

// PERSIST: a persistent grid (gridDim.x workgroups, gridDim.y = 1) over all B x ntiles tiles -- each XCD's
// workgroups (blockIdx.x % 8, the round-robin dispatch) walk a contiguous band of the batch's tiles, workgroup k of
// the band taking tiles k, k + R, k + 2R, ... (R workgroups per band), and each issues the staging loads of its next
// tile before the current tile's reduction and flush, so those loads overlap the tail of the current tile instead
// of every workgroup of a round loading at once.  ntiles_frame: tiles per frame (PERSIST only).
template <int CC, int AB = 0, int TWX = kGradTileW, int TH = grad_tile_h(CC), int GM = 3, bool PERSIST = true>
__global__ __attribute__((amdgpu_flat_work_group_size(1, GradGeom<TWX, TH>::NT),
                          amdgpu_waves_per_eu(DIRT_GRAD_PERSIST_WAVES))) DIRT_GRAD_ATTR void grad_kernel_persist(const float *__restrict__ pixels, const float *__restrict__ grad_pixels,
                                                   const int32_t *__restrict__ gbuffer, const uint8_t *__restrict__ covbits,
                                                   const Rec *__restrict__ recs,
                                                   const FaceData *__restrict__ fdata, int B, int H, int W, int Cdyn,
                                                   int V, int F, TileGrid tg, int64_t nrec, float *__restrict__ grad_verts,
                                                   float *__restrict__ grad_colors, float *__restrict__ grad_bg,
                                                   const NdcScale ns, int ntiles_frame = 0,
                                                   uint32_t *__restrict__ stash_flip = nullptr)
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

    static_assert(kHaloPix <= 2 * NT, "two staging passes");
    // PERSIST schedule (see above): this workgroup's first tile (linear over the batch), its stride and count
    int lin0 = 0, lstride = 0, nit = 1;
    if constexpr (PERSIST) {
        const int T_all = B * ntiles_frame, P = gridDim.x, g = blockIdx.x & 7, k = blockIdx.x >> 3;
        const int q = T_all >> 3, r = T_all & 7;
        const int band0 = g * q + min(g, r), band_len = q + (g < r ? 1 : 0);
        lstride = (P - g + 7) >> 3;  // workgroups of this band
        lin0 = band0 + k;
        nit = k < band_len ? (band_len - k + lstride - 1) / lstride : 0;
    }
    // tile of iteration `it`: (frame, tile x, tile y)
    auto tile_of = [&](int it, int &b_, int &tx_, int &ty_) {
        int tile_;
        if constexpr (PERSIST) {
            const int lin = __builtin_amdgcn_readfirstlane(lin0 + it * lstride);
            b_ = __builtin_amdgcn_readfirstlane(lin / ntiles_frame);
            tile_ = lin - b_ * ntiles_frame;
        } else {
            tile_ = xcd_tile(blockIdx.x, gridDim.x);
            b_ = blockIdx.y;
        }
        tg.split(tile_, tx_, ty_);
    };
    // the staged pixels' g-buffer words, coverage bits and G / I (for the staged pair scalars, !kRecompute): loaded
    // by stage_loads for the current tile (PERSIST: for the next one, while the current one is reduced)
    int32_t gbv[2];
    uint32_t cvv[2];
    bool ok[2];
    float Gv[2][CM], Iv[2][CM];
    auto stage_loads = [&](int b_, int tx_, int ty_) {
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        // every load of both passes in flight before the first LDS store (kHaloPix <= 2 * NT)
        // frame base pointers (64-bit, uniform) + 32-bit per-lane offsets: H * W * C < 2^29
        const int64_t fpix = (int64_t)b_ * H * W;
        const int32_t *gb_f = gbuffer + fpix;
        const uint8_t *cov_f = covbits + fpix;
        const float *gp_f = grad_pixels + fpix * C, *px_f = pixels + fpix * C;
        const int hi0_ = tx_ * TWX - 1, hj0_ = ty_ * TH - 1;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = t + NT * u;
            const int hi = hi0_ + k % kHalo, hj = hj0_ + k / kHalo;
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
    };
    for (int it = 0; it < nit; ++it) {
    // the lane's coordinates from an opaque copy of threadIdx.x, per tile: values derived from them are then not
    // hoisted out of the tile loop (live across every phase, they would spill)
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    const int lx = t % TWX, ly = t / TWX;
    const int lr = lx & 15;  // lane within its 16-lane DPP row (a pixel row, or half of one at TWX = 32)
    const float inv_hw = ns.inv_hw, inv_hh = ns.inv_hh;  // 2/W, 2/H from the host (no division in the kernel)
    const int kme = (ly + 1) * kHalo + (lx + 1);
    int b, tx, ty;
    tile_of(it, b, tx, ty);
    const int i = tx * TWX + lx, j = ty * TH + ly;
    const Rec *frame_recs = recs + (int64_t)b * nrec;
    const FaceData *fdata_frame = fdata + (int64_t)b * F;
    const bool in_frame = i < W && j < H;
    // (PERSIST: the previous tile's flush still reads the slot table and the tail partials)
    if (PERSIST && it > 0) __syncthreads();

    // ---- phase A: stage g-buffer / G / I of the tile + one-pixel halo, pair scalars, slot table
    PHASE_TS(0);
    for (int k = t; k < kSlots; k += NT) {
        T.key[k] = -1;
        s_tcnt[k] = 0;
    }
    if (t == 0) T.n = 0;
    const int hi0 = tx * TWX - 1, hj0 = ty * TH - 1;
    if (!PERSIST || it == 0) stage_loads(b, tx, ty);
    {
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
            s_gb[k] = gbv[u];
            s_cov[k] = (uint8_t)cvv[u];
            if (!ok[u]) continue;
            if constexpr (CM == 3) {
                *reinterpret_cast<float4 *>(&s_G[k * CP]) = make_float4(Gv[u][0], Gv[u][1], Gv[u][2], 0.0f);
                *reinterpret_cast<float4 *>(&s_I[k * CP]) = make_float4(Iv[u][0], Iv[u][1], Iv[u][2], 0.0f);
            } else if constexpr (CP == 8) {
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
    }
    __syncthreads();
    PHASE_TS(1);
    const int32_t gp = in_frame ? s_gb[kme] : -2;
    {
        // the tile's own records (run heads only; all distinct keys may not fit: the rest read global
        // memory).  The halo's records are not needed: pair coverage comes from the forward's bits.
        const int32_t g = s_gb[kme];
        const int key = g >= 0 ? g : -1;
        const int start = run_start(key, lr);
        int slot = slot_insert_wave(T, key, key >= 0 && start == lr);
        if (key >= 0 && start == lr && slot >= 0) atomicAdd(&s_tcnt[slot], 1);  // one run (one tail later)
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
            // 1/w of a non-clipped face: its FaceData's q (a clipped record's own 1/w, in the record's second
            // half, are read in phase B by the lanes that show it)
            riw0 = fd.q[0]; riw1 = fd.q[1]; riw2 = fd.q[2];
        }
        // pair scalars of the pairs starting at an own pixel (right, up) and at the left column /
        // bottom row of the halo (their one pair into the tile); nothing reads the others
        if constexpr (!kRecompute) {
            // staged pair scalars: the lane that staged region pixel k computes the pairs starting there that
            // phase B reads -- (k, k+x) for hx in 0..TWX, hy in 1..16 and (k, k+y) for hx in 1..TWX, hy in 0..16
            // -- with k's own G / I still in its registers (only the neighbour's come from LDS)
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
        if (filler) {
            bool small = true;
            int64_t E0[3];
            edge_values(ep, hi0, hj0, E0);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                T.A[k][sf] = ep.A[k]; T.B[k][sf] = ep.B[k];
                T.v[k][t] = fd.v[k];  // by list position (read only by the flush)
                small = small && ep.A[k] > -kGradSmallEdge && ep.A[k] < kGradSmallEdge && ep.B[k] > -kGradSmallEdge &&
                        ep.B[k] < kGradSmallEdge;
                T.e[k][sf] = (int32_t)E0[k] + owned_bit(ep.A[k], ep.B[k]);  // meaningful only when small
            }
            T.q[0][sf] = riw0; T.q[1][sf] = riw1; T.q[2][sf] = riw2;
            T.h2d[sf] = 0.5f / (float)ep.D;  // (E_0 + E_1 + E_2 = D at every pixel)
            T.bx[sf] = (uint32_t)ep.i0 | ((uint32_t)ep.i1 << 16) | (small ? 0u : kSlotLarge);
            T.by[sf] = (uint32_t)ep.j0 | ((uint32_t)ep.j1 << 16);
        }
    }
    __syncthreads();
    PHASE_TS(4);

    // ---- phase B: per-pixel contributions to the face visible at this pixel
    const int32_t rp = gp >= 0 ? (gp & kGbufIndexMask) : gp;
    if (in_frame && grad_bg != nullptr) {  // (null: the caller needs no background gradient)
        float *gbg_f = grad_bg + (int64_t)b * H * W * C;
        const uint32_t o = (uint32_t)((H - 1 - j) * W + i);
        float *gbq = gbg_f + o * (uint32_t)C;  // (RGB: one global_store_dwordx3)
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            const float gv = s_G[kme * CP + c];
            // (non-temporal: nothing in this pipeline reads grad_background back, so its lines need not
            // stay dirty in L2 for the write-back that ends the launch)
            if (c < C) __builtin_nontemporal_store(rp < 0 ? gv : 0.0f, &gbq[c]);
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
            iw0 = T.q[0][sp]; iw1 = T.q[1][sp]; iw2 = T.q[2][sp];  // (1/w unless clipped)
            h2d = T.h2d[sp];
            me_small = !slot_is_large(T, sp);
            if (__builtin_amdgcn_ballot_w64(multi) != 0 && multi) {
                const Rec &rr = rec();
                iw0 = rr.iw[0]; iw1 = rr.iw[1]; iw2 = rr.iw[2];
            }
        } else {
            const Rec &rr = rec();
            const EdgePart me = *reinterpret_cast<const EdgePart *>(&rr);
#pragma unroll
            for (int k = 0; k < 3; ++k) { mA[k] = me.A[k]; mB[k] = me.B[k]; }
            if (multi) {
                iw0 = rr.iw[0]; iw1 = rr.iw[1]; iw2 = rr.iw[2];
            } else {
                const FaceData &fq = fdata_frame[f];
                iw0 = fq.q[0]; iw1 = fq.q[1]; iw2 = fq.q[2];
            }
            h2d = 0.5f / (float)me.D;
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
            for (int c = 0; c < CM; ++c) Gm[c] = c < C ? s_G[kme * CP + c] : 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                for (int c = 0; c < C; ++c) acc[(kNVV + k * C + c) < NVM ? kNVV + k * C + c : 0] = lam[k] * Gm[c];
        }
    }
    if constexpr (PERSIST) {
        // the next tile's staging loads, in flight through this tile's reduction and flush (no load of those
        // phases waits for them: the barriers wait for LDS only, the flush's atomics return nothing)
        if (it + 1 < nit) {
            int b2, tx2, ty2;
            tile_of(it + 1, b2, tx2, ty2);
            stage_loads(b2, tx2, ty2);
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
            const FaceData &fd = fdata_frame[face_of_record(rp, F)];
            const int32_t vid[3] = {fd.v[0], fd.v[1], fd.v[2]};  // before the atomics (may alias for the compiler)
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
    }  // tiles of this workgroup
}
