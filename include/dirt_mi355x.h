/*
 * dirt_mi355x.h -- C ABI of the MI355X-native dirt rasteriser (libdirt_mi355x.so).
 *
 * Drop-in boundary for the reference's TensorFlow custom ops in librasterise.so
 * (loaded by tf.load_op_library at dirt/rasterise_ops.py:7):
 *
 *   dirt_rasterise_fwd  replaces  REGISTER_OP("Rasterise")           csrc/rasterise_egl.cpp:33-53
 *                                 RasteriseOpGpu::Compute            csrc/rasterise_egl.cpp:284-514
 *                                 upload_background/download_pixels  csrc/rasterise_egl.cu:16-129
 *   dirt_rasterise_bwd  replaces  launch_grad_assembly (declared,    csrc/rasterise_grad_common.h:19-24
 *                                 never defined in the fork) -- the gradient DIRT registers upstream
 *                                 for "Rasterise"; the fork's REGISTER_OP("RasteriseGrad")
 *                                 (csrc/rasterise_grad_egl.cpp:33-53) is a forward render
 *   dirt_rasterise_bwd_recompute  the same gradient from the op's inputs + output + grad_pixels only, for
 *                                 a single-output `Rasterise` with tf.RegisterGradient (upstream DIRT's
 *                                 shape: rasterise_grad_common.h:5-24 re-derives its G-buffer)
 *   dirt_hill_fwd       replaces  REGISTER_OP("Hill") + HillOpGpu     csrc/hill.cpp:33-53, 282-498
 *                                 (the other procedural ops are shader ids of dirt_rasterise_fwd:
 *                                 RasteriseGrad, OceanicStillCloud, OceanicNoCloud, OceanicOptFlow,
 *                                 OceanicSimpleProxy -- csrc/rasterise_grad_egl.cpp, csrc/oceanic_*.cpp)
 *   dirt_last_error     replaces  OP_REQUIRES(..., errors::InvalidArgument(...)) messages,
 *                                 csrc/rasterise_egl.cpp:310-336 (the reference aborts on everything
 *                                 else via LOG(FATAL)/CHECK; this ABI never aborts)
 *
 * Conventions
 *   - every tensor pointer is a DEVICE pointer to a dense row-major array (HBM of the current HIP device);
 *   - float32 data, int32 faces; shapes use the reference's batch-leading layout
 *       background    [B,H,W,C]   top row first (rasterise_egl.cu:29)
 *       vertices      [B,V,4]     OpenGL clip space x,y,z,w (README.md:131)
 *       vertex_colors [B,V,C]
 *       faces         [B,F,3]     indices into the same frame's vertices (base vertex b*V, rasterise_egl.cpp:457)
 *       pixels        [B,H,W,C]   output
 *   - outputs are caller-owned; work is enqueued asynchronously on `stream` (a hipStream_t, 0 = null stream);
 *   - `saved` is the state the backward needs (per-face setup records); `scratch` is forward-only
 *     (tile bins).  Query their sizes with dirt_workspace_sizes; the caller owns both.
 *   - channels C may be 1..DIRT_MAX_CHANNELS (the reference accepts 1 or 3, csrc/hwc.h:27).
 *
 * Return codes: DIRT_OK, DIRT_EINVAL (bad shape/argument; message in dirt_last_error()),
 * DIRT_EHIP (a HIP runtime error).  Out-of-range face indices cull the face (the reference reads
 * out of bounds); dirt_check_faces() reports them on request.
 */
#ifndef DIRT_MI355X_H
#define DIRT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DIRT_OK 0
#define DIRT_EINVAL 1
#define DIRT_EFACE 2
#define DIRT_EHIP 3

#define DIRT_MAX_CHANNELS 8
#define DIRT_MAX_DIM 8192

/* fragment programs (shader_id); 0 = Gouraud (README.md:134-137) */
#define DIRT_SHADER_GOURAUD 0
#define DIRT_SHADER_OCEANIC_HORIZON 1 /* csrc/shaders.cpp:1668-1919 (the fork's `Rasterise` program) */
#define DIRT_SHADER_OCEANIC 2             /* csrc/shaders.cpp:556-864 (`RasteriseGrad`, rasterise_grad_egl.cpp:399) */
#define DIRT_SHADER_OCEANIC_STILL_CLOUD 3 /* csrc/shaders.cpp:866-1176 (`OceanicStillCloud`; camera_pos[8] = cloud_t) */
#define DIRT_SHADER_OCEANIC_NO_CLOUD 4    /* csrc/shaders.cpp:1402-1666 (`OceanicNoCloud`) */
#define DIRT_SHADER_OCEANIC_SIMPLE_PROXY 5 /* csrc/shaders.cpp:1921-2185 (`OceanicSimpleProxy`) */
#define DIRT_SHADER_OCEANIC_OPT_FLOW 6 /* csrc/shaders.cpp:1178-1398 (`OceanicOptFlow`; camera_pos: 16 floats,
                                          oceanic_opt_flow.cpp:399-414); pixels = previous-frame coordinates */
#define DIRT_SHADER_HILL 7 /* csrc/shaders.cpp:123-554 (`Hill`, csrc/hill.cpp; camera_pos: 12 floats); no depth
                              test (last face wins), background = terrain lookup, uncovered pixels 0 */

/* ABI version, bumped on any signature or workspace-layout change (4: + dirt_hill_fwd, shader ids 6 and 7;
 * 5: setup bins directly into fixed-capacity per-coarse-tile slabs, 3 profiled kernels; 6: bin counters on
 * separate 256-B lines of the scratch; 7: + dirt_rasterise_fwd_gbuffer; 8: + dirt_rasterise_bwd_recompute,
 * dirt_bwd_recompute_workspace_size; 9: + the fused lighting helpers dirt_vertex_normals_*,
 * dirt_diffuse_directional_*, dirt_specular_directional_*, dirt_diffuse_point_*; 10: + dirt_stream_capture_id;
 * 11: + dirt_rasterise_fwd_stash, the recompute workspace grows by the gradient stash; 12: the Gouraud forward
 * picks the occluder culling by itself (DIRT_FWD_DEEP_CULL forces it, + DIRT_FWD_DEEP_CULL_OFF); 13: +
 * dirt_rasterise_fwd_resolve) */
int dirt_abi_version(void);

/* Byte sizes of the caller-provided buffers for one call.
 * bin_capacity = number of (coarse tile, triangle) bin entries the scratch can hold, split evenly into
 * one slab per (frame, coarse tile); <=0: default policy (F + F/4 + 64 entries per slab, so no slab of
 * a frame overflows unless many faces are clipped into one tile, up to 2^29 entries (4 GiB) in all).  A slab
 * that overflows is still rendered exactly, by a slow path that filters every record of the frame. */
int dirt_workspace_sizes(int B, int H, int W, int C, int V, int F, int64_t bin_capacity,
                         size_t *saved_bytes, size_t *scratch_bytes);

/* Forward: pixels = Rasterise(background, vertices, vertex_colors, faces).
 * gbuffer [B,H,W] int32 receives the per-pixel visible setup-record index (-1 = background),
 * which together with `saved` is what dirt_rasterise_bwd consumes.
 * camera_pos: device pointer to >= 8 floats (9 for DIRT_SHADER_OCEANIC_STILL_CLOUD, 16 for
 * DIRT_SHADER_OCEANIC_OPT_FLOW, 12 for DIRT_SHADER_HILL), used only by the procedural programs
 * (shader_id != 0; may be NULL for Gouraud).  DIRT_SHADER_HILL here reads `background` as a C-channel
 * terrain lookup; dirt_hill_fwd takes one with its own channel count. */
int dirt_rasterise_fwd(const float *background, const float *vertices, const float *vertex_colors,
                       const int32_t *faces, const float *camera_pos,
                       int B, int H, int W, int C, int V, int F, int shader_id,
                       float *pixels, int32_t *gbuffer,
                       void *saved, size_t saved_bytes, void *scratch, size_t scratch_bytes,
                       int64_t bin_capacity, unsigned flags,
                       float *zero_grad_vertices, float *zero_grad_vertex_colors, void *stream);
/* Forward with the deferred-shading G-buffer (Gouraud program): dirt_rasterise_fwd plus, per pixel,
 *   depth        [B,H,W]   window depth as the reference's DEPTH24 buffer holds it (rasterise_egl.cpp:248),
 *                          read back as float: d / (2^24 - 1); 1.0 (the clear value, :449) where uncovered
 *   barycentrics [B,H,W,3] perspective-correct barycentrics of the visible face's vertices
 *                          faces[b, face_ids, 0..2] (the `smooth` interpolation, shaders.cpp:16-34); 0 uncovered
 *   face_ids     [B,H,W]   index of the visible face, -1 uncovered
 * (rows top first, like pixels).  Each may be NULL.  Replaces upstream DIRT's G-buffer programs
 * backward_vertex / backward_fragment (csrc/shaders.cpp:2187-2221: barycentrics, 1/gl_FragCoord.w and the
 * face's vertex indices) and the Vertex layout of csrc/rasterise_grad_common.h:5-11. */
int dirt_rasterise_fwd_gbuffer(const float *background, const float *vertices, const float *vertex_colors,
                               const int32_t *faces, int B, int H, int W, int C, int V, int F,
                               float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes,
                               void *scratch, size_t scratch_bytes, int64_t bin_capacity, unsigned flags,
                               float *zero_grad_vertices, float *zero_grad_vertex_colors,
                               float *depth, float *barycentrics, int32_t *face_ids, void *stream);
/* Forward of a render that shares its geometry with an earlier one (ABI 13): the same vertices, faces, B, H, W and
 * default bin capacity as the Gouraud dirt_rasterise_fwd that wrote `gbuffer_in` and `saved`, other vertex colours
 * [B,V,C] and background [B,H,W,C] (C may differ from that forward's).  Only the resolve runs -- per pixel the visible
 * record from gbuffer_in, its perspective-correct barycentrics from saved, the Gouraud colour of these vertex colours
 * or this background -- so the pixels are bit-identical to a dirt_rasterise_fwd of the same inputs, whose coverage
 * and depth depend on the geometry only.  `gbuffer` [B,H,W] receives this render's copy of the g-buffer (the same
 * words); gbuffer_in and saved are only read, and the later dirt_rasterise_bwd of this render takes `gbuffer` and the
 * same `saved`.  zero_grad_*: as dirt_rasterise_fwd (zero-filled in passing).  samples/deferred.py:63-83 renders
 * one geometry three times (positions, albedo, normals). */
int dirt_rasterise_fwd_resolve(const float *background, const float *vertex_colors, int B, int H, int W, int C, int V,
                               int F, const int32_t *gbuffer_in, const void *saved, size_t saved_bytes, float *pixels,
                               int32_t *gbuffer, float *zero_grad_vertices, float *zero_grad_vertex_colors,
                               void *stream);
/* Forward of the Hill op (csrc/hill.cpp:282-498, REGISTER_OP("Hill") :33-53): DIRT_SHADER_HILL with a
 * terrain lookup `terrain` [B,H,W,terrain_channels] (1, 3 or 4 channels, uploaded like a background,
 * rasterise_egl.cu:33-47) in place of the background; vertex colours are not read.  pixels [B,H,W,C];
 * gbuffer / saved / scratch as dirt_rasterise_fwd (same dirt_workspace_sizes). */
int dirt_hill_fwd(const float *terrain, int terrain_channels, const float *vertices, const int32_t *faces,
                  const float *camera_pos, int B, int H, int W, int C, int V, int F,
                  float *pixels, int32_t *gbuffer, void *saved, size_t saved_bytes, void *scratch,
                  size_t scratch_bytes, int64_t bin_capacity, void *stream);
/* flags of dirt_rasterise_fwd.  Every forward leaves the scratch ready for the next one (the bin counts
 * alternate between two sets, each zeroed by the forward that does not use it), so a scratch buffer that
 * was zero-filled once (or passed to dirt_scratch_clear) and since used only by forwards with the same
 * B, H, W, F and bin_capacity is "clean". */
#define DIRT_FWD_SCRATCH_CLEAN 1u /* the scratch is clean: skip the forward's own clearing memset */
#define DIRT_FWD_DEEP_CULL 2u     /* Gouraud: occluder culling of long per-tile triangle lists before they are
                                     rasterised -- for deep scenes (large overlapping triangles: depth complexity
                                     ~45 at r = 64 px, raster -15 %); results are identical either way, and
                                     scenes of small triangles run slightly faster without it.  Since ABI 12 the
                                     binned Gouraud forward chooses it by itself: each launch counts its long
                                     per-wave lists, and a device takes the culling raster while one of its last
                                     8 forwards was deep (env DIRT_DEEP_CULL_AUTO=0 turns the rule off); this
                                     flag forces it */
#define DIRT_FWD_DEEP_CULL_OFF 8u /* Gouraud: never the occluder culling (the plain raster, as before ABI 12) */
/* zero_grad_vertices [B,V,4] / zero_grad_vertex_colors [B,V,C] (each may be NULL): accumulators the
 * forward zero-fills in passing (filler workgroups of its setup launch, idle CUs), for a later dirt_rasterise_bwd with
 * DIRT_BWD_ACCUMULATE -- a fixed-shape training loop then pays no separate clearing launch.
 * Alignment: no pointer argument of this ABI needs more than its element's natural alignment (4 B);
 * 16-B aligned buffers (every torch / hipMalloc allocation) take the vectorised zero-fill path, others
 * (views at an offset) a scalar one. */

/* Backward: given grad_pixels = dL/dpixels, writes dL/dvertices [B,V,4] (z component is 0),
 * dL/dvertex_colors [B,V,C] and dL/dbackground [B,H,W,C].  All three outputs are fully
 * overwritten (see DIRT_BWD_ACCUMULATE).  grad_background may be NULL when the caller needs no background
 * gradient (a constant background: 4 C bytes per pixel not written); so may one of grad_vertices and
 * grad_vertex_colors (that gradient is then not computed at all: ~30 % less backward time at config 4).  Filter-based (DIRT/OpenDR) derivative,
 * DESIGN.md section 4. */
int dirt_rasterise_bwd(const float *vertices, const float *vertex_colors, const int32_t *faces,
                       const float *pixels, const float *grad_pixels, const int32_t *gbuffer,
                       const void *saved,
                       int B, int H, int W, int C, int V, int F,
                       float *grad_vertices, float *grad_vertex_colors, float *grad_background,
                       unsigned flags, void *stream);
/* flags of dirt_rasterise_bwd */
#define DIRT_BWD_ACCUMULATE 1u /* add into grad_vertices / grad_vertex_colors instead of overwriting them
                                  (e.g. zeroed by the caller on a side stream, off the critical path);
                                  grad_background is always overwritten */
/* Backward of the single-output op: the registered gradient of `Rasterise` computed from the op's own inputs,
 * its output and grad_pixels only -- nothing kept from the forward, so the TensorFlow op stays
 * single-output (csrc/rasterise_egl.cpp:33-53; dirt/rasterise_ops.py:50-54 indexes `[0]`).  Replaces upstream
 * DIRT's gradient path, which re-derived its G-buffer from the op's inputs: launch_vertex_upload +
 * launch_grad_assembly(grad_vertices, grad_vertex_colors, grad_background, ..., pixels, grad_pixels,
 * vertices, ...) (csrc/rasterise_grad_common.h:5-24, declared only in the fork).  Recomputes setup, binning
 * and a coverage-only raster pass (g-buffer + neighbour-coverage bits, bit-identical to the forward's) into
 * `workspace`, then runs the backward kernel of dirt_rasterise_bwd: the same gradients (up to float-atomic
 * summation order), at the cost of the forward's setup and a raster pass without pixel traffic.
 * `pixels` must be the op's output for these inputs.  background / vertex_colors are part of the gradient's
 * inputs and are not read.  Outputs as dirt_rasterise_bwd (fully overwritten unless DIRT_BWD_ACCUMULATE).
 * workspace: caller-owned device memory of dirt_bwd_recompute_workspace_size() bytes; no state survives the
 * call unless DIRT_BWD_SCRATCH_CLEAN is used. */
int dirt_bwd_recompute_workspace_size(int B, int H, int W, int C, int V, int F, size_t *workspace_bytes);
int dirt_rasterise_bwd_recompute(const float *background, const float *vertices, const float *vertex_colors,
                                 const int32_t *faces, const float *pixels, const float *grad_pixels,
                                 int B, int H, int W, int C, int V, int F,
                                 float *grad_vertices, float *grad_vertex_colors, float *grad_background,
                                 void *workspace, size_t workspace_bytes, unsigned flags, void *stream);
/* flags of dirt_rasterise_bwd_recompute: DIRT_BWD_ACCUMULATE, and */
#define DIRT_BWD_SCRATCH_CLEAN 2u /* the workspace was zero-filled once and since used only by recompute
                                     backwards and forward-stashes of the same B, H, W, V, F: skip the bin-counter
                                     memset, and keep the gradient stash */
/* Gradient stash (v11).  The workspace also records the geometry (vertices and faces, bitwise) whose setup records,
 * g-buffer and coverage bits it holds.  dirt_rasterise_bwd_recompute first compares its vertices and faces with that
 * record on the device: when they are identical it skips the recomputation (device-side: the setup and coverage
 * launches exit at once) and runs the backward kernel on what the workspace holds -- the same gradients, since those
 * intermediates are a deterministic function of the geometry and the frame size.  Otherwise it recomputes, and
 * records the new geometry.  dirt_rasterise_fwd_stash is the single-output op's forward that fills the stash as it
 * renders (pixels only as output; background / vertex colours do not enter the stash), so the gradient of that
 * forward costs only the comparison: a TensorFlow kernel pair would share the workspace through a per-device
 * resource keyed by the layout.  A different geometry in between (another render of the same layout) costs one
 * recomputation, never a wrong gradient.  workspace: dirt_bwd_recompute_workspace_size() bytes; flags:
 * DIRT_FWD_SCRATCH_CLEAN when the workspace is clean as DIRT_BWD_SCRATCH_CLEAN describes. */
int dirt_rasterise_fwd_stash(const float *background, const float *vertices, const float *vertex_colors,
                             const int32_t *faces, int B, int H, int W, int C, int V, int F, float *pixels,
                             void *workspace, size_t workspace_bytes, unsigned flags, void *stream);

/* Zero the bin counters of `scratch` for the next forward with the same B, H, W, F, bin_capacity
 * (an async memset of a few KB; lets a caller clear them on another stream, see DIRT_FWD_SCRATCH_CLEAN). */
int dirt_scratch_clear(int B, int H, int W, int F, int64_t bin_capacity, void *scratch, size_t scratch_bytes,
                       void *stream);

/* The id of the HIP graph capture `stream` is recording (hipStreamGetCaptureInfo), 0 when it records none.
 * A scratch created and cleared inside one capture is clean only for that graph's own replays (its clearing
 * memset runs when the graph replays), so callers that cache scratch per stream key it by this id too. */
int dirt_stream_capture_id(void *stream, unsigned long long *capture_id);

/* Debug check (synchronises `stream`): returns DIRT_EFACE if any face index is outside [0,V).  Uses the
 * first 4 bytes of `scratch` as its flag: pass a scratch that no forward is using, or clear it after. */
int dirt_check_faces(const int32_t *faces, int B, int V, int F, void *scratch, size_t scratch_bytes, void *stream);

/* Optional per-kernel timing with HIP events around every launch (used by bench.py for the roofline).
 * dirt_profile_enable(1) clears and starts recording, (0) clears and stops.  dirt_profile_read
 * synchronises the recorded events of kernel `kernel_id` (0..DIRT_NUM_KERNELS-1) and returns its name,
 * launch count and summed duration.  Not thread-safe; do not enable during hipGraph capture. */
#define DIRT_NUM_KERNELS 3
int dirt_profile_enable(int enable);
int dirt_profile_read(int kernel_id, const char **name, int *launches, double *total_ms);

/* Fused lighting helpers: dirt/lighting.py's vertex_normals (:34-98), diffuse_directional (:182-225),
 * specular_directional (:228-288) and diffuse_point (:291-344) -- TensorFlow compositions in the reference (no op of librasterise.so), one
 * kernel per forward / backward here (the deferred-shading chain of samples/deferred.py:62-118 runs them per
 * pixel).  Formulas: dirt_amd/lighting.py.  Light parameters are DEVICE pointers to 3 floats; gradients with
 * respect to them are not computed (the Python layer uses its framework-op statement when they are needed).
 * Backward rules at the kinks as the framework's: d|x| = sign(x) (0 at 0), max(x, 0) passes where x >= 0.
 *
 * vertex_normals: vertices [B,V,vertex_stride] (x, y, z first; stride >= 3), faces [F,3] shared by the B
 * frames (int32, or int64 when faces_int64), out-of-range faces skipped.  summed [B,V,3] (zeroed by the call)
 * is the unnormalised sum the backward needs; normals [B,V,3].  The sums use float atomics: the result may
 * differ in the last bit between calls (as the framework's index_add on a GPU).
 * The backward zero-fills grad_vertices [B,V,grad_stride] and accumulates into its first 3 components;
 * grad_summed [B,V,3] is scratch. */
int dirt_vertex_normals_fwd(const float *vertices, int vertex_stride, const void *faces, int faces_int64, int B, int V,
                            int F, float *summed, float *normals, void *stream);
int dirt_vertex_normals_bwd(const float *vertices, int vertex_stride, const void *faces, int faces_int64, int B, int V,
                            int F, const float *summed, const float *grad_normals, float *grad_summed,
                            float *grad_vertices, int grad_stride, void *stream);
/* diffuse_directional: normals, colors, out [N,3]; out = light_color * colors * clamp(normals . -light_direction).
 * Backward: grad_normals / grad_colors [N,3] overwritten (either may be NULL). */
int dirt_diffuse_directional_fwd(const float *normals, const float *colors, int64_t N, const float *light_direction,
                                 const float *light_color, int double_sided, float *out, void *stream);
int dirt_diffuse_directional_bwd(const float *normals, const float *colors, int64_t N, const float *light_direction,
                                 const float *light_color, int double_sided, const float *grad_out,
                                 float *grad_normals, float *grad_colors, void *stream);
/* diffuse_point: positions, normals, colors, out [N,3]; out = light_color * colors * clamp(normals . unit(positions -
 * light_position)).  Backward: grad_positions / grad_normals / grad_colors [N,3] overwritten (each may be NULL). */
int dirt_diffuse_point_fwd(const float *positions, const float *normals, const float *colors, int64_t N,
                           const float *light_position, const float *light_color, int double_sided, float *out,
                           void *stream);
int dirt_diffuse_point_bwd(const float *positions, const float *normals, const float *colors, int64_t N,
                           const float *light_position, const float *light_color, int double_sided,
                           const float *grad_out, float *grad_positions, float *grad_normals, float *grad_colors,
                           void *stream);
/* specular_directional: positions, normals, reflectivities, out [N,3]; Phong lobe around the reflected light
 * direction, out = light_color * reflectivities * clamp(cos)^shininess.  Backward: the three input gradients
 * [N,3] overwritten (each may be NULL). */
int dirt_specular_directional_fwd(const float *positions, const float *normals, const float *reflectivities, int64_t N,
                                  const float *light_direction, const float *light_color,
                                  const float *camera_position, float shininess, int double_sided, float *out,
                                  void *stream);
int dirt_specular_directional_bwd(const float *positions, const float *normals, const float *reflectivities, int64_t N,
                                  const float *light_direction, const float *light_color,
                                  const float *camera_position, float shininess, int double_sided,
                                  const float *grad_out, float *grad_positions, float *grad_normals,
                                  float *grad_reflectivities, void *stream);

/* Thread-local message for the last non-OK return on this thread. */
const char *dirt_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* DIRT_MI355X_H */
