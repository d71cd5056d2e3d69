// Part of dirt_raster.hip's translation unit: included inside its anonymous namespace after the shared
// definitions (HIP_TRY, fail).  Not a standalone header.
//
// Fused lighting helpers of the reference's dirt/lighting.py (vertex_normals :34-98, diffuse_directional
// :182-225, specular_directional :228-288, diffuse_point :291-344): one kernel per forward and per backward
// instead of the dozen elementwise launches each costs as a composition of framework ops (BASELINE config 4, the deferred-shading
// chain of samples/deferred.py:62-118, shades 512 x 512 pixels through them every step).  Formulas and operand
// order follow dirt_amd/lighting.py's torch statement, which is the tests' fp32 reference for these kernels.
// All of it is elementwise or a gather / scatter over faces: HBM- or latency-bound, no MFMA shape.
//
// Light parameters (direction, colour, camera position) are device pointers to 3 floats: nothing is copied
// from the host per call, so the calls can be captured into a HIP graph.

constexpr int kLightThreads = 256;

__device__ __forceinline__ float3 ld3(const float *p) { return make_float3(p[0], p[1], p[2]); }
__device__ __forceinline__ void st3(float *p, float3 v)
{
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}
__device__ __forceinline__ float dot3(float3 a, float3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float3 cross3(float3 a, float3 b)
{
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float3 sub3(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 add3(float3 a, float3 b) { return make_float3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ float3 mul3(float3 a, float s) { return make_float3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float norm3(float3 a) { return sqrtf(dot3(a, a)); }
__device__ __forceinline__ void atomic_add3(float *p, float3 v)
{
    atomicAdd(p, v.x);
    atomicAdd(p + 1, v.y);
    atomicAdd(p + 2, v.z);
}

// face f's three vertex indices (int32 or int64 faces), false if any is outside [0, V)
template <typename I>
__device__ __forceinline__ bool face_vertices(const I *faces, int64_t f, int V, int v[3])
{
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t x = (int64_t)faces[f * 3 + k];
        ok = ok && x >= 0 && x < V;
        v[k] = ok ? (int)x : 0;
    }
    return ok;
}

// ---- vertex_normals (dirt/lighting.py:34-98): face normal n = (v1 - v0) x (v2 - v0), normalised as
// n / (|n| + 1e-12), summed into the face's three vertices, each sum normalised the same way.  vertices:
// [B, V, vstride] (x, y, z first), faces [F, 3] shared by the B frames.

template <typename I>
__global__ __launch_bounds__(kLightThreads) void vnormals_face_kernel(const float *__restrict__ verts, int vstride,
                                                                      const I *__restrict__ faces, int V, int64_t F,
                                                                      float *__restrict__ summed)
{
    const int64_t f = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (f >= F) return;
    const int b = blockIdx.y;
    int v[3];
    if (!face_vertices(faces, f, V, v)) return;
    const float *vb = verts + (int64_t)b * V * vstride;
    const float3 p0 = ld3(vb + (int64_t)v[0] * vstride), p1 = ld3(vb + (int64_t)v[1] * vstride),
                 p2 = ld3(vb + (int64_t)v[2] * vstride);
    const float3 n = cross3(sub3(p1, p0), sub3(p2, p0));
    const float3 nn = mul3(n, 1.0f / (norm3(n) + 1.e-12f));
    float *sb = summed + (int64_t)b * V * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) atomic_add3(sb + (int64_t)v[k] * 3, nn);
}

__global__ __launch_bounds__(kLightThreads) void vnormals_vertex_kernel(const float *__restrict__ summed, int64_t n,
                                                                        float *__restrict__ normals)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 s = ld3(summed + e * 3);
    st3(normals + e * 3, mul3(s, 1.0f / (norm3(s) + 1.e-12f)));
}

// backward, per vertex: d summed = g / (|s| + eps) - s (s . g) / (|s| (|s| + eps)^2)
__global__ __launch_bounds__(kLightThreads) void vnormals_vertex_bwd_kernel(const float *__restrict__ summed,
                                                                            const float *__restrict__ grad, int64_t n,
                                                                            float *__restrict__ grad_summed)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 s = ld3(summed + e * 3), g = ld3(grad + e * 3);
    const float m = norm3(s), d = m + 1.e-12f;
    float3 r = mul3(g, 1.0f / d);
    if (m > 0.0f) r = sub3(r, mul3(s, dot3(s, g) / (m * d * d)));
    st3(grad_summed + e * 3, r);
}

// backward, per face: the three vertices' d summed -> d n (normalisation) -> d(v1 - v0) = (v2 - v0) x dn,
// d(v2 - v0) = dn x (v1 - v0) -> scattered into the vertices
template <typename I>
__global__ __launch_bounds__(kLightThreads) void vnormals_face_bwd_kernel(const float *__restrict__ verts, int vstride,
                                                                          const I *__restrict__ faces, int V,
                                                                          int64_t F, const float *__restrict__ grad_summed,
                                                                          float *__restrict__ grad_verts, int gstride)
{
    const int64_t f = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (f >= F) return;
    const int b = blockIdx.y;
    int v[3];
    if (!face_vertices(faces, f, V, v)) return;
    const float *vb = verts + (int64_t)b * V * vstride;
    const float *gs = grad_summed + (int64_t)b * V * 3;
    const float3 p0 = ld3(vb + (int64_t)v[0] * vstride), p1 = ld3(vb + (int64_t)v[1] * vstride),
                 p2 = ld3(vb + (int64_t)v[2] * vstride);
    const float3 dnn = add3(add3(ld3(gs + (int64_t)v[0] * 3), ld3(gs + (int64_t)v[1] * 3)), ld3(gs + (int64_t)v[2] * 3));
    const float3 a = sub3(p1, p0), c = sub3(p2, p0);
    const float3 n = cross3(a, c);
    const float m = norm3(n), d = m + 1.e-12f;
    float3 dn = mul3(dnn, 1.0f / d);
    if (m > 0.0f) dn = sub3(dn, mul3(n, dot3(n, dnn) / (m * d * d)));
    const float3 da = cross3(c, dn), dc = cross3(dn, a);
    float *gb = grad_verts + (int64_t)b * V * gstride;
    atomic_add3(gb + (int64_t)v[1] * gstride, da);
    atomic_add3(gb + (int64_t)v[2] * gstride, dc);
    atomic_add3(gb + (int64_t)v[0] * gstride, mul3(add3(da, dc), -1.0f));
}

// ---- diffuse_directional (dirt/lighting.py:182-225): cos = n . (-l), |cos| (double-sided) or max(cos, 0),
// out = light_color * colour * cos.  Backward: the framework's rules at the kinks (d|x| = sign(x), 0 at 0;
// max(x, 0) passes the gradient where x >= 0).
__device__ __forceinline__ float shade_clamp(float c, bool two) { return two ? fabsf(c) : fmaxf(c, 0.0f); }
__device__ __forceinline__ float shade_clamp_grad(float c, float g, bool two)
{
    return two ? (c > 0.0f ? g : c < 0.0f ? -g : 0.0f) : (c >= 0.0f ? g : 0.0f);
}

__global__ __launch_bounds__(kLightThreads) void diffuse_fwd_kernel(const float *__restrict__ normals,
                                                                    const float *__restrict__ colors, int64_t n,
                                                                    const float *__restrict__ ldir,
                                                                    const float *__restrict__ lcol, int two,
                                                                    float *__restrict__ out)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 nl = mul3(ld3(ldir), -1.0f), lc = ld3(lcol);
    const float3 nv = ld3(normals + e * 3), col = ld3(colors + e * 3);
    const float cs = shade_clamp(dot3(nv, nl), two);
    st3(out + e * 3, make_float3(lc.x * col.x * cs, lc.y * col.y * cs, lc.z * col.z * cs));
}

__global__ __launch_bounds__(kLightThreads) void diffuse_bwd_kernel(const float *__restrict__ normals,
                                                                    const float *__restrict__ colors, int64_t n,
                                                                    const float *__restrict__ ldir,
                                                                    const float *__restrict__ lcol, int two,
                                                                    const float *__restrict__ grad,
                                                                    float *__restrict__ grad_normals,
                                                                    float *__restrict__ grad_colors)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 nl = mul3(ld3(ldir), -1.0f), lc = ld3(lcol);
    const float3 nv = ld3(normals + e * 3), col = ld3(colors + e * 3), g = ld3(grad + e * 3);
    const float c = dot3(nv, nl), cs = shade_clamp(c, two);
    const float3 glc = make_float3(g.x * lc.x, g.y * lc.y, g.z * lc.z);
    if (grad_colors) st3(grad_colors + e * 3, mul3(glc, cs));
    if (grad_normals) st3(grad_normals + e * 3, mul3(nl, shade_clamp_grad(c, dot3(glc, col), two)));
}

// ---- specular_directional (dirt/lighting.py:228-288), in dirt_amd/lighting.py's operand order:
//   r = l + 2 (n . (-l)) n,  t = cam - p,  u = t / |t| + 1e-12,  cos = u . r,  |cos| or max(cos, 0),
//   out = light_color * reflectivity * cos^shininess
struct SpecTerms {
    float3 r, t, u;
    float tn, c, cs, p;
};
__device__ __forceinline__ SpecTerms spec_terms(float3 pos, float3 nv, float3 l, float3 cam, float shin, bool two)
{
    SpecTerms s;
    const float3 tl = mul3(l, -1.0f);
    s.r = add3(l, mul3(nv, 2.0f * dot3(nv, tl)));
    s.t = sub3(cam, pos);
    s.tn = norm3(s.t);
    const float it = 1.0f / s.tn;
    s.u = make_float3(s.t.x * it + 1.e-12f, s.t.y * it + 1.e-12f, s.t.z * it + 1.e-12f);
    s.c = dot3(s.u, s.r);
    s.cs = shade_clamp(s.c, two);
    s.p = powf(s.cs, shin);
    return s;
}

__global__ __launch_bounds__(kLightThreads) void specular_fwd_kernel(const float *__restrict__ positions,
                                                                     const float *__restrict__ normals,
                                                                     const float *__restrict__ refl, int64_t n,
                                                                     const float *__restrict__ ldir,
                                                                     const float *__restrict__ lcol,
                                                                     const float *__restrict__ campos, float shin,
                                                                     int two, float *__restrict__ out)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 lc = ld3(lcol);
    const SpecTerms s = spec_terms(ld3(positions + e * 3), ld3(normals + e * 3), ld3(ldir), ld3(campos), shin, two);
    const float3 rf = ld3(refl + e * 3);
    st3(out + e * 3, make_float3(lc.x * rf.x * s.p, lc.y * rf.y * s.p, lc.z * rf.z * s.p));
}

__global__ __launch_bounds__(kLightThreads) void specular_bwd_kernel(
    const float *__restrict__ positions, const float *__restrict__ normals, const float *__restrict__ refl, int64_t n,
    const float *__restrict__ ldir, const float *__restrict__ lcol, const float *__restrict__ campos, float shin,
    int two, const float *__restrict__ grad, float *__restrict__ grad_positions, float *__restrict__ grad_normals,
    float *__restrict__ grad_refl)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 l = ld3(ldir), lc = ld3(lcol);
    const float3 nv = ld3(normals + e * 3);
    const SpecTerms s = spec_terms(ld3(positions + e * 3), nv, l, ld3(campos), shin, two);
    const float3 rf = ld3(refl + e * 3), g = ld3(grad + e * 3);
    const float3 glc = make_float3(g.x * lc.x, g.y * lc.y, g.z * lc.z);
    if (grad_refl) st3(grad_refl + e * 3, mul3(glc, s.p));
    // d cos^k = k cos^(k-1) (0 for k = 0), through the clamp
    const float dpow = shin == 0.0f ? 0.0f : shin * powf(s.cs, shin - 1.0f);
    const float dc = shade_clamp_grad(s.c, dot3(glc, rf) * dpow, two);
    const float3 du = mul3(s.r, dc), dr = mul3(s.u, dc);
    if (grad_positions) {
        // u = t / |t| (+ eps): dt = du / |t| - t (t . du) / |t|^3; d pos = -dt
        const float it = 1.0f / s.tn;
        const float3 dt = sub3(mul3(du, it), mul3(s.t, dot3(s.t, du) * it * it * it));
        st3(grad_positions + e * 3, mul3(dt, -1.0f));
    }
    if (grad_normals) {
        // r = l + 2 (n . tl) n, tl = -l: dn = 2 tl (dr . n) + 2 (n . tl) dr
        const float3 tl = mul3(l, -1.0f);
        st3(grad_normals + e * 3, add3(mul3(tl, 2.0f * dot3(dr, nv)), mul3(dr, 2.0f * dot3(nv, tl))));
    }
}

// ---- diffuse_point (dirt/lighting.py:291-344), in dirt_amd/lighting.py's operand order:
//   d = p - light_position,  u = d / (|d| + 1e-12),  cos = n . u,  |cos| or max(cos, 0),  out = light_color * colour * cos
__global__ __launch_bounds__(kLightThreads) void diffuse_point_fwd_kernel(const float *__restrict__ positions,
                                                                          const float *__restrict__ normals,
                                                                          const float *__restrict__ colors, int64_t n,
                                                                          const float *__restrict__ lpos,
                                                                          const float *__restrict__ lcol, int two,
                                                                          float *__restrict__ out)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 d = sub3(ld3(positions + e * 3), ld3(lpos)), lc = ld3(lcol), col = ld3(colors + e * 3);
    const float3 u = mul3(d, 1.0f / (norm3(d) + 1.e-12f));
    const float cs = shade_clamp(dot3(ld3(normals + e * 3), u), two);
    st3(out + e * 3, make_float3(lc.x * col.x * cs, lc.y * col.y * cs, lc.z * col.z * cs));
}

__global__ __launch_bounds__(kLightThreads) void diffuse_point_bwd_kernel(
    const float *__restrict__ positions, const float *__restrict__ normals, const float *__restrict__ colors, int64_t n,
    const float *__restrict__ lpos, const float *__restrict__ lcol, int two, const float *__restrict__ grad,
    float *__restrict__ grad_positions, float *__restrict__ grad_normals, float *__restrict__ grad_colors)
{
    const int64_t e = (int64_t)blockIdx.x * kLightThreads + threadIdx.x;
    if (e >= n) return;
    const float3 d = sub3(ld3(positions + e * 3), ld3(lpos)), lc = ld3(lcol), col = ld3(colors + e * 3);
    const float3 nv = ld3(normals + e * 3), g = ld3(grad + e * 3);
    const float m = norm3(d), dm = m + 1.e-12f;
    const float3 u = mul3(d, 1.0f / dm);
    const float c = dot3(nv, u), cs = shade_clamp(c, two);
    const float3 glc = make_float3(g.x * lc.x, g.y * lc.y, g.z * lc.z);
    if (grad_colors) st3(grad_colors + e * 3, mul3(glc, cs));
    const float dc = shade_clamp_grad(c, dot3(glc, col), two);
    if (grad_normals) st3(grad_normals + e * 3, mul3(u, dc));
    if (grad_positions) {
        // u = d / (|d| + eps): dd = du / (|d| + eps) - d (d . du) / (|d| (|d| + eps)^2), du = dc n
        const float3 du = mul3(nv, dc);
        float3 dd = mul3(du, 1.0f / dm);
        if (m > 0.0f) dd = sub3(dd, mul3(d, dot3(d, du) / (m * dm * dm)));
        st3(grad_positions + e * 3, dd);
    }
}

inline unsigned light_blocks(int64_t n) { return (unsigned)((n + kLightThreads - 1) / kLightThreads); }
