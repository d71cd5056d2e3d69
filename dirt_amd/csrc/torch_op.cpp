// torch_op.cpp -- the public rasterise op's autograd function in C++ (PyTorch extension `_dirt_torch`).
//
// Same semantics as dirt_amd.rasterise_ops._RasteriseFunction (the Python torch.autograd.Function kept as
// the fallback): forward = dirt_rasterise_fwd / dirt_rasterise_fwd_gbuffer, registered gradient =
// dirt_rasterise_bwd, through the C ABI of include/dirt_mi355x.h.  The reference registers its op in C++
// too (REGISTER_OP("Rasterise"), csrc/rasterise_egl.cpp:33-53, RasteriseOpGpu::Compute :284-514); doing the
// per-call bookkeeping here (allocation, workspace cache, stream lookup, the backward run by the autograd
// engine without a trip through Python) keeps the eager op close to the kernels' time.
//
// The library is not linked: init(path) dlopens the same libdirt_mi355x.so the ctypes binding loaded
// (dirt_amd/_lib.py, DIRT_MI355X_LIB honoured) and resolves the entry points by name.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <dlfcn.h>

#include <atomic>

#include <list>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

#include "../../include/dirt_mi355x.h"

namespace {

struct Api {
    decltype(&dirt_workspace_sizes) workspace_sizes = nullptr;
    decltype(&dirt_rasterise_fwd) fwd = nullptr;
    decltype(&dirt_rasterise_fwd_gbuffer) fwd_gbuffer = nullptr;
    decltype(&dirt_rasterise_fwd_resolve) fwd_resolve = nullptr;
    decltype(&dirt_rasterise_bwd) bwd = nullptr;
    decltype(&dirt_scratch_clear) scratch_clear = nullptr;
    decltype(&dirt_check_faces) check_faces = nullptr;
    decltype(&dirt_stream_capture_id) capture_id = nullptr;
    decltype(&dirt_last_error) last_error = nullptr;
    decltype(&dirt_vertex_normals_fwd) vn_fwd = nullptr;
    decltype(&dirt_vertex_normals_bwd) vn_bwd = nullptr;
    decltype(&dirt_diffuse_directional_fwd) diffuse_fwd = nullptr;
    decltype(&dirt_diffuse_directional_bwd) diffuse_bwd = nullptr;
    decltype(&dirt_diffuse_point_fwd) point_fwd = nullptr;
    decltype(&dirt_diffuse_point_bwd) point_bwd = nullptr;
    decltype(&dirt_specular_directional_fwd) specular_fwd = nullptr;
    decltype(&dirt_specular_directional_bwd) specular_bwd = nullptr;
} g_api;

void check(int rc)
{
    if (rc == DIRT_OK) return;
    const std::string msg = g_api.last_error ? g_api.last_error() : "dirt: error";
    if (rc == DIRT_EINVAL) throw std::invalid_argument(msg);   // ValueError, like OP_REQUIRES InvalidArgument
    if (rc == DIRT_EFACE) throw std::out_of_range(msg);        // IndexError
    throw std::runtime_error(msg);
}

void init(const std::string &path)
{
    void *h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (!h) throw std::runtime_error(std::string("_dirt_torch: cannot load ") + path + ": " + dlerror());
    auto sym = [&](const char *name) {
        void *p = dlsym(h, name);
        if (!p) throw std::runtime_error(std::string("_dirt_torch: ") + path + " lacks " + name);
        return p;
    };
    g_api.workspace_sizes = reinterpret_cast<decltype(g_api.workspace_sizes)>(sym("dirt_workspace_sizes"));
    g_api.fwd = reinterpret_cast<decltype(g_api.fwd)>(sym("dirt_rasterise_fwd"));
    g_api.fwd_gbuffer = reinterpret_cast<decltype(g_api.fwd_gbuffer)>(sym("dirt_rasterise_fwd_gbuffer"));
    g_api.fwd_resolve = reinterpret_cast<decltype(g_api.fwd_resolve)>(sym("dirt_rasterise_fwd_resolve"));
    g_api.bwd = reinterpret_cast<decltype(g_api.bwd)>(sym("dirt_rasterise_bwd"));
    g_api.scratch_clear = reinterpret_cast<decltype(g_api.scratch_clear)>(sym("dirt_scratch_clear"));
    g_api.check_faces = reinterpret_cast<decltype(g_api.check_faces)>(sym("dirt_check_faces"));
    g_api.capture_id = reinterpret_cast<decltype(g_api.capture_id)>(sym("dirt_stream_capture_id"));
    g_api.last_error = reinterpret_cast<decltype(g_api.last_error)>(sym("dirt_last_error"));
    g_api.vn_fwd = reinterpret_cast<decltype(g_api.vn_fwd)>(sym("dirt_vertex_normals_fwd"));
    g_api.vn_bwd = reinterpret_cast<decltype(g_api.vn_bwd)>(sym("dirt_vertex_normals_bwd"));
    g_api.diffuse_fwd = reinterpret_cast<decltype(g_api.diffuse_fwd)>(sym("dirt_diffuse_directional_fwd"));
    g_api.diffuse_bwd = reinterpret_cast<decltype(g_api.diffuse_bwd)>(sym("dirt_diffuse_directional_bwd"));
    g_api.point_fwd = reinterpret_cast<decltype(g_api.point_fwd)>(sym("dirt_diffuse_point_fwd"));
    g_api.point_bwd = reinterpret_cast<decltype(g_api.point_bwd)>(sym("dirt_diffuse_point_bwd"));
    g_api.specular_fwd = reinterpret_cast<decltype(g_api.specular_fwd)>(sym("dirt_specular_directional_fwd"));
    g_api.specular_bwd = reinterpret_cast<decltype(g_api.specular_bwd)>(sym("dirt_specular_directional_bwd"));
}

// Forward-only scratch (bins, bin counters) per (device, stream, layout), cleared once: every forward
// leaves it clean for the next one of the same layout (DIRT_FWD_SCRATCH_CLEAN).  LRU of a few layouts.
// Graph capture: a scratch created while the stream captures a HIP graph comes from that graph's
// memory pool and is cleared by a kernel captured into the graph, i.e. it is clean only for that graph's replays.
// Those entries are keyed by the capture id too (dirt_stream_capture_id): forwards of one capture share one, no
// other capture or eager call sees it, and they stay PINNED until clear(force = true) -- the graph writes them at
// every replay, and a block released to a pool that a later capture shares (torch.cuda.graph(pool=...),
// make_graphed_callables) could otherwise be handed to that capture too.  An entry whose forward failed is
// discarded (its alternating count sets may be dirty).  The Python twin is dirt_amd.rasterise_ops._CaptureKeyedCache.
struct ScratchCache {
    typedef std::tuple<int, uintptr_t, int64_t, int64_t, int64_t, int64_t, int64_t> Key;
    struct Entry {
        Key key;
        at::Tensor t;
    };
    std::mutex mu;
    std::list<Entry> lru;                                  // eager entries
    std::map<unsigned long long, std::list<Entry>> caps;  // capture id -> its entries (pinned)
    static unsigned long long capture_id(hipStream_t stream)
    {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusActive) return 0;
        unsigned long long id = 0;
        check(g_api.capture_id(stream, &id));
        return id;
    }
    static at::Tensor *find(std::list<Entry> &l, const Key &k, bool to_front)
    {
        for (auto it = l.begin(); it != l.end(); ++it)
            if (it->key == k) {
                if (to_front) l.splice(l.begin(), l, it);
                return to_front ? &l.front().t : &it->t;
            }
        return nullptr;
    }
    static bool debug()
    {
        static int v = -1;
        if (v < 0) v = getenv("DIRT_DEBUG_SCRATCH") != nullptr;
        return v != 0;
    }
    at::Tensor get(const Key &k, size_t bytes, const at::Device &dev, hipStream_t stream)
    {
        const unsigned long long cid = capture_id(stream);
        {
            std::lock_guard<std::mutex> g(mu);
            if (at::Tensor *t = find(cid ? caps[cid] : lru, k, !cid)) {
                if (debug()) fprintf(stderr, "[dirt scratch] hit stream %p capture %llu ptr %p\n", (void *)stream, cid, t->data_ptr());
                return *t;
            }
        }
        at::Tensor t = at::empty({(int64_t)std::max<size_t>(bytes, 1)}, at::TensorOptions().dtype(at::kByte).device(dev));
        if (debug()) fprintf(stderr, "[dirt scratch] new stream %p capture %llu ptr %p\n", (void *)stream, cid, t.data_ptr());
        check(g_api.scratch_clear((int)std::get<2>(k), (int)std::get<3>(k), (int)std::get<4>(k), (int)std::get<5>(k),
                                  std::get<6>(k), t.data_ptr(), bytes, stream));
        std::lock_guard<std::mutex> g(mu);
        if (cid) {
            caps[cid].push_front(Entry{k, t});
        } else {
            lru.push_front(Entry{k, t});
            while (lru.size() > 4) lru.pop_back();
        }
        return t;
    }
    void discard(const Key &k)
    {
        std::lock_guard<std::mutex> g(mu);
        lru.remove_if([&](const Entry &e) { return e.key == k; });
        for (auto &c : caps) c.second.remove_if([&](const Entry &e) { return e.key == k; });
    }
    // eager entries; `force`: the captures' pinned entries too (once their graphs are destroyed)
    void clear(bool force)
    {
        std::lock_guard<std::mutex> g(mu);
        lru.clear();
        if (force) caps.clear();
    }
    size_t size()
    {
        std::lock_guard<std::mutex> g(mu);
        size_t n = lru.size();
        for (auto &c : caps) n += c.second.size();
        return n;
    }
} g_scratch;

// Renders that share their geometry (samples/deferred.py:63-83 renders one mesh three times, as
// positions, albedo and normals): the last plain Gouraud forward per (device, stream, capture) remembers its geometry
// -- the vertices' and faces' storage, offset, sizes, strides and version counters (detached aliases, so no autograd
// graph is kept) -- with its g-buffer and saved records.  A forward whose vertices and faces are the same tensors
// (or views of the same storage, same elements), unmodified since (version counters unchanged: every in-place op on
// them or a view bumps it), at the same B, H, W, F, takes dirt_rasterise_fwd_resolve: no setup, bins or visibility
// pass, pixels bit-identical.  Its backward reads the shared saved records (read-only) and its own g-buffer copy.
// Writes that bypass the version counter (`.data`, raw pointers) are not seen -- the same limitation as autograd's
// own saved-tensor checks; DIRT_SHARE_GEOMETRY=0 turns the cache off.  A capture's entries are its own (its g-buffer
// is recomputed by its replays), and eager entries are never used inside a capture or the other way round.
struct GeomCache {
    struct Entry {
        int dev = -1;
        uintptr_t stream = 0;
        unsigned long long cid = 0;
        at::Tensor v, f, gbuffer, saved;
        int64_t vver = 0, fver = 0, H = 0, W = 0;
    };
    std::mutex mu;
    std::list<Entry> entries;  // one per (device, stream, capture id), a few at most
    // on unless DIRT_SHARE_GEOMETRY=0; set_geometry_sharing() switches it at run time (both implementations)
    static std::atomic<int> &flag()
    {
        static std::atomic<int> v{[] {
            const char *e = getenv("DIRT_SHARE_GEOMETRY");
            return (e && *e) ? (atoi(e) != 0 ? 1 : 0) : 1;
        }()};
        return v;
    }
    static bool enabled() { return flag().load(std::memory_order_relaxed) != 0; }
    // the same elements of the same storage (strides of size-1 dimensions do not matter)
    static bool same(const at::Tensor &a, const at::Tensor &b)
    {
        if (!a.defined() || !b.defined() || a.unsafeGetTensorImpl()->storage().unsafeGetStorageImpl() !=
                                                b.unsafeGetTensorImpl()->storage().unsafeGetStorageImpl() ||
            a.storage_offset() != b.storage_offset() || a.sizes() != b.sizes() || a.scalar_type() != b.scalar_type())
            return false;
        for (int64_t d = 0; d < a.dim(); ++d)
            if (a.size(d) > 1 && a.stride(d) != b.stride(d)) return false;
        return true;
    }
    // the shared (gbuffer, saved) of an unchanged geometry, or undefined tensors
    std::pair<at::Tensor, at::Tensor> find(int dev, hipStream_t stream, unsigned long long cid, const at::Tensor &v,
                                           const at::Tensor &f, int64_t H, int64_t W)
    {
        std::lock_guard<std::mutex> g(mu);
        for (const Entry &e : entries)
            if (e.dev == dev && e.stream == reinterpret_cast<uintptr_t>(stream) && e.cid == cid && e.H == H && e.W == W &&
                same(e.v, v) && same(e.f, f) && e.vver == (int64_t)v._version() && e.fver == (int64_t)f._version())
                return {e.gbuffer, e.saved};
        return {at::Tensor(), at::Tensor()};
    }
    void store(int dev, hipStream_t stream, unsigned long long cid, const at::Tensor &v, const at::Tensor &f, int64_t H,
               int64_t W, const at::Tensor &gbuffer, const at::Tensor &saved)
    {
        std::lock_guard<std::mutex> g(mu);
        entries.remove_if([&](const Entry &e) {
            return e.dev == dev && e.stream == reinterpret_cast<uintptr_t>(stream) && e.cid == cid;
        });
        Entry e;
        e.dev = dev;
        e.stream = reinterpret_cast<uintptr_t>(stream);
        e.cid = cid;
        e.v = v.detach();
        e.f = f.detach();
        e.vver = (int64_t)v._version();
        e.fver = (int64_t)f._version();
        e.H = H;
        e.W = W;
        e.gbuffer = gbuffer;
        e.saved = saved;
        entries.push_front(e);
        while (entries.size() > 8) entries.pop_back();
    }
    void clear()
    {
        std::lock_guard<std::mutex> g(mu);
        entries.clear();
    }
} g_geom;

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct RasteriseFn : public torch::autograd::Function<RasteriseFn> {
    static variable_list forward(AutogradContext *ctx, at::Tensor background, at::Tensor vertices,
                                 at::Tensor vertex_colors, at::Tensor faces, c10::optional<at::Tensor> camera_pos,
                                 int64_t H, int64_t W, int64_t C, int64_t shader_id, int64_t bin_capacity,
                                 bool want_gbuf, bool check_faces, bool grad_possible, int64_t fwd_flags)
    {
        const int64_t B = vertices.size(0), V = vertices.size(1), F = faces.size(1);
        const at::Device dev = vertices.device();
        c10::hip::HIPGuard guard(dev.index());
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev.index()).stream();
        size_t saved_bytes = 0, scratch_bytes = 0;
        check(g_api.workspace_sizes((int)B, (int)H, (int)W, (int)C, (int)V, (int)F, bin_capacity, &saved_bytes,
                                    &scratch_bytes));
        const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
        const auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
        at::Tensor pixels = at::empty({B, H, W, C}, f32);
        at::Tensor gbuffer = at::empty({B, H, W}, i32);
        // (needs_input_grad is only defined when the node records a graph: grad_possible, decided outside
        // forward where GradMode is visible)
        const bool need_grad = grad_possible && shader_id == DIRT_SHADER_GOURAUD && V > 0 &&
                               (ctx->needs_input_grad(0) || ctx->needs_input_grad(1) || ctx->needs_input_grad(2));
        // which accumulators the backward fills: the vertices' and / or the colours' -- the backward computes
        // only those (a background-only gradient still runs the kernel, with both)
        bool want_v = need_grad && ctx->needs_input_grad(1), want_c = need_grad && ctx->needs_input_grad(2);
        if (need_grad && !want_v && !want_c) want_v = want_c = true;
        at::Tensor gv, gc;
        if (want_v) gv = at::empty({B, V, 4}, f32);  // zero-filled by the forward in passing; the backward accumulates
        if (want_c) gc = at::empty({B, V, C}, f32);
        if (check_faces) {
            at::Tensor flag = at::empty({256}, at::TensorOptions().dtype(at::kByte).device(dev));
            check(g_api.check_faces(faces.data_ptr<int32_t>(), (int)B, (int)V, (int)F, flag.data_ptr(), 256, stream));
        }
        // a render of the same geometry as the last plain Gouraud forward on this stream: the resolve alone
        const bool shareable = GeomCache::enabled() && shader_id == DIRT_SHADER_GOURAUD && !want_gbuf && F > 0 &&
                               !(fwd_flags & (DIRT_FWD_DEEP_CULL | DIRT_FWD_DEEP_CULL_OFF));
        const unsigned long long cid = shareable ? ScratchCache::capture_id(stream) : 0ull;
        if (shareable) {
            std::pair<at::Tensor, at::Tensor> hit = g_geom.find(dev.index(), stream, cid, vertices, faces, H, W);
            if (hit.first.defined()) {
                check(g_api.fwd_resolve(background.data_ptr<float>(), vertex_colors.data_ptr<float>(), (int)B, (int)H,
                                        (int)W, (int)C, (int)V, (int)F, hit.first.data_ptr<int32_t>(),
                                        hit.second.data_ptr(), (size_t)hit.second.numel(), pixels.data_ptr<float>(),
                                        gbuffer.data_ptr<int32_t>(), want_v ? gv.data_ptr<float>() : nullptr,
                                        want_c ? gc.data_ptr<float>() : nullptr, stream));
                finish_forward(ctx, vertices, vertex_colors, faces, pixels, gbuffer, hit.second, B, H, W, C, V, F,
                               shader_id, need_grad, want_v, want_c, gv, gc);
                ctx->mark_non_differentiable({gbuffer});
                return {pixels, gbuffer};
            }
        }
        at::Tensor saved = at::empty({(int64_t)std::max<size_t>(saved_bytes, 1)}, at::TensorOptions().dtype(at::kByte).device(dev));
        const ScratchCache::Key skey{dev.index(), reinterpret_cast<uintptr_t>(stream), B, H, W, F, bin_capacity};
        at::Tensor scratch = g_scratch.get(skey, scratch_bytes, dev, stream);
        float *zgv = want_v ? gv.data_ptr<float>() : nullptr;
        float *zgc = want_c ? gc.data_ptr<float>() : nullptr;
        variable_list out{pixels, gbuffer};
        // a failed forward may leave the cached scratch's count sets dirty: drop it
        struct DropOnThrow {
            const ScratchCache::Key &k;
            bool armed = true;
            ~DropOnThrow()
            {
                if (armed) g_scratch.discard(k);
            }
        } drop{skey};
        if (want_gbuf) {
            at::Tensor depth = at::empty({B, H, W}, f32), bary = at::empty({B, H, W, 3}, f32), face = at::empty({B, H, W}, i32);
            check(g_api.fwd_gbuffer(background.data_ptr<float>(), vertices.data_ptr<float>(),
                                    vertex_colors.data_ptr<float>(), faces.data_ptr<int32_t>(), (int)B, (int)H, (int)W,
                                    (int)C, (int)V, (int)F, pixels.data_ptr<float>(), gbuffer.data_ptr<int32_t>(),
                                    saved.data_ptr(), saved_bytes, scratch.data_ptr(), scratch_bytes, bin_capacity,
                                    (unsigned)fwd_flags | DIRT_FWD_SCRATCH_CLEAN, zgv, zgc, depth.data_ptr<float>(), bary.data_ptr<float>(),
                                    face.data_ptr<int32_t>(), stream));
            out.push_back(depth);
            out.push_back(bary);
            out.push_back(face);
        } else {
            const float *cam = camera_pos.has_value() ? camera_pos->data_ptr<float>() : nullptr;
            check(g_api.fwd(background.data_ptr<float>(), vertices.data_ptr<float>(), vertex_colors.data_ptr<float>(),
                            faces.data_ptr<int32_t>(), cam, (int)B, (int)H, (int)W, (int)C, (int)V, (int)F,
                            (int)shader_id, pixels.data_ptr<float>(), gbuffer.data_ptr<int32_t>(), saved.data_ptr(),
                            saved_bytes, scratch.data_ptr(), scratch_bytes, bin_capacity,
                            (unsigned)fwd_flags | DIRT_FWD_SCRATCH_CLEAN, zgv, zgc, stream));
        }
        drop.armed = false;
        if (shareable) g_geom.store(dev.index(), stream, cid, vertices, faces, H, W, gbuffer, saved);
        finish_forward(ctx, vertices, vertex_colors, faces, pixels, gbuffer, saved, B, H, W, C, V, F, shader_id,
                       need_grad, want_v, want_c, gv, gc);
        variable_list nd(out.begin() + 1, out.end());
        ctx->mark_non_differentiable(nd);
        return out;
    }

    static void finish_forward(AutogradContext *ctx, const at::Tensor &vertices, const at::Tensor &vertex_colors,
                               const at::Tensor &faces, const at::Tensor &pixels, const at::Tensor &gbuffer,
                               const at::Tensor &saved, int64_t B, int64_t H, int64_t W, int64_t C, int64_t V, int64_t F,
                               int64_t shader_id, bool need_grad, bool want_v, bool want_c, const at::Tensor &gv,
                               const at::Tensor &gc)
    {
        // the backward takes the pixels' gradient only: without this, autograd would fill a zero gradient for
        // each non-differentiable output (the int32 g-buffer: a 4 MB fill kernel per backward at config 3)
        ctx->set_materialize_grads(false);
        ctx->save_for_backward({vertices, vertex_colors, faces, pixels, gbuffer, saved});
        ctx->saved_data["dims"] = std::vector<int64_t>{B, H, W, C, V, F, shader_id};
        ctx->saved_data["prezeroed"] = need_grad;
        ctx->saved_data["want"] = (int64_t)((want_v ? 1 : 0) | (want_c ? 2 : 0));
        if (need_grad) {
            ctx->saved_data["gv"] = gv;
            ctx->saved_data["gc"] = gc;
        }
    }

    static variable_list backward(AutogradContext *ctx, variable_list grads)
    {
        const std::vector<int64_t> d = ctx->saved_data["dims"].toIntVector();
        const int64_t B = d[0], H = d[1], W = d[2], C = d[3], V = d[4], F = d[5], shader_id = d[6];
        if (shader_id != DIRT_SHADER_GOURAUD)
            throw std::runtime_error("only the Gouraud fragment program has a gradient (the reference registers none)");
        auto sv = ctx->get_saved_variables();
        const at::Tensor &vertices = sv[0], &vertex_colors = sv[1], &faces = sv[2], &pixels = sv[3], &gbuffer = sv[4],
                         &saved = sv[5];
        const at::Device dev = vertices.device();
        c10::hip::HIPGuard guard(dev.index());
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev.index()).stream();
        const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
        at::Tensor gp = grads[0].defined() ? grads[0].to(at::kFloat).contiguous() : at::zeros({B, H, W, C}, f32);
        // the forward's zero-filled buffers serve one backward (autograd may keep the returned tensors as
        // .grad); a second backward of the same graph (retain_graph) starts from fresh ones
        unsigned flags = 0;
        at::Tensor gv, gc;
        const int64_t want = ctx->saved_data["want"].toInt();
        if (ctx->saved_data["prezeroed"].toBool()) {
            gv = ctx->saved_data["gv"].toTensor();
            gc = ctx->saved_data["gc"].toTensor();
            ctx->saved_data["prezeroed"] = false;
            ctx->saved_data.erase("gv");
            ctx->saved_data.erase("gc");
            flags = DIRT_BWD_ACCUMULATE;
        } else {
            if ((want & 1) || want == 0) gv = at::empty({B, V, 4}, f32);
            if ((want & 2) || want == 0) gc = at::empty({B, V, C}, f32);
        }
        // (a background that needs no gradient -- a constant one -- is not written at all)
        at::Tensor gbg = ctx->needs_input_grad(0) ? at::empty({B, H, W, C}, f32) : at::Tensor();
        check(g_api.bwd(vertices.data_ptr<float>(), vertex_colors.data_ptr<float>(), faces.data_ptr<int32_t>(),
                        pixels.data_ptr<float>(), gp.data_ptr<float>(), gbuffer.data_ptr<int32_t>(), saved.data_ptr(),
                        (int)B, (int)H, (int)W, (int)C, (int)V, (int)F, gv.defined() ? gv.data_ptr<float>() : nullptr,
                        gc.defined() ? gc.data_ptr<float>() : nullptr, gbg.defined() ? gbg.data_ptr<float>() : nullptr,
                        flags, stream));
        return {gbg, gv, gc, at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(),
                at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor()};
    }
};

// dtype / device / layout of an op input as the kernels take it (recorded by autograd, outside the op's node)
at::Tensor prep(const at::Tensor &x, at::ScalarType t, const at::Device &dev)
{
    at::Tensor y = (x.device() != dev || x.scalar_type() != t) ? x.to(dev, t) : x;
    return y.is_contiguous() ? y : y.contiguous();
}

// The reference op's shape checks (csrc/rasterise_egl.cpp:310-336, messages as dirt_amd.rasterise_ops._check_shapes)
void check_shapes(const at::Tensor &bg, const at::Tensor &v, const at::Tensor &vc, const at::Tensor &f, int64_t H,
                  int64_t W, int64_t C)
{
    if (bg.dim() != 4 || bg.size(1) != H || bg.size(2) != W || bg.size(3) != C)
        throw std::invalid_argument("Rasterise expects background_tensor to be 4D, and bgcolor.shape == [None, height, width, channels]");
    if (v.dim() != 3 || v.size(2) != 4)
        throw std::invalid_argument("Rasterise expects vertices to be 3D, and vertices.shape[2] == 4");
    if (vc.dim() != 3 || vc.size(1) != v.size(1) || vc.size(2) != C)
        throw std::invalid_argument("Rasterise expects vertex_colors to be 3D, and vertex_colors.shape == [None, vertices.shape[1], channels]");
    if (f.dim() != 3 || f.size(2) != 3)
        throw std::invalid_argument("Rasterise expects faces to be 3D, and faces.shape[2] == 3");
    if (bg.size(0) != v.size(0) || vc.size(0) != v.size(0) || f.size(0) != v.size(0))
        throw std::invalid_argument("Rasterise expects all arguments to have same leading (batch) dimension");
    if (C < 1 || C > DIRT_MAX_CHANNELS) throw std::invalid_argument("Rasterise expects 1 <= channels <= 8");
}

// The public op's fast path (dirt_amd.rasterise_ops._rasterise_batched with tensor inputs): the Python
// wrapper's conversions and checks done here, in one call.
variable_list rasterise_checked(at::Tensor background, at::Tensor vertices, at::Tensor vertex_colors, at::Tensor faces,
                                int64_t H, int64_t W, int64_t C, int64_t bin_capacity, bool want_gbuf,
                                bool check_faces, int64_t fwd_flags);

variable_list rasterise(at::Tensor background, at::Tensor vertices, at::Tensor vertex_colors, at::Tensor faces,
                        c10::optional<at::Tensor> camera_pos, int64_t H, int64_t W, int64_t C, int64_t shader_id,
                        int64_t bin_capacity, bool want_gbuf, bool check_faces, int64_t fwd_flags)
{
    if (!g_api.fwd) throw std::runtime_error("_dirt_torch.init(path) was not called");
    const bool grad_possible = at::GradMode::is_enabled() &&
                               (background.requires_grad() || vertices.requires_grad() || vertex_colors.requires_grad());
    return RasteriseFn::apply(background, vertices, vertex_colors, faces, camera_pos, H, W, C, shader_id, bin_capacity,
                              want_gbuf, check_faces, grad_possible, fwd_flags);
}

variable_list rasterise_checked(at::Tensor background, at::Tensor vertices, at::Tensor vertex_colors, at::Tensor faces,
                                int64_t H, int64_t W, int64_t C, int64_t bin_capacity, bool want_gbuf,
                                bool check_faces, int64_t fwd_flags)
{
    // the tensors' device: the first one on the GPU, else the current HIP device (the Python wrapper's _device_of)
    const at::Tensor *on_gpu = nullptr;
    for (const at::Tensor *x : {&background, &vertices, &vertex_colors, &faces})
        if (x->is_cuda()) {
            on_gpu = x;
            break;
        }
    if (!on_gpu && c10::hip::device_count() == 0)
        throw std::runtime_error("dirt_amd.rasterise requires a ROCm/HIP GPU: there is no CPU implementation");
    const at::Device dev = on_gpu ? on_gpu->device() : at::Device(at::kCUDA, c10::hip::current_device());
    background = prep(background, at::kFloat, dev);
    vertices = prep(vertices, at::kFloat, dev);
    vertex_colors = prep(vertex_colors, at::kFloat, dev);
    faces = prep(faces, at::kInt, dev);
    check_shapes(background, vertices, vertex_colors, faces, H, W, C);
    return rasterise(background, vertices, vertex_colors, faces, c10::nullopt, H, W, C, DIRT_SHADER_GOURAUD,
                     bin_capacity, want_gbuf, check_faces, fwd_flags);
}

// ---- fused lighting helpers (dirt/lighting.py; dirt_amd/lighting.py decides when they apply: CUDA float32
// tensors, [..., 3] operands of one shape, light parameters of shape [3] that need no gradient)

hipStream_t stream_of(const at::Tensor &x)
{
    return c10::hip::getCurrentHIPStream(x.device().index()).stream();
}

at::Tensor grad_or_zeros(const at::Tensor &g, const at::Tensor &like)
{
    return g.defined() ? g.to(at::kFloat).contiguous() : at::zeros_like(like);
}

// The fused helpers' backwards are raw kernels: their results carry no graph, so a second-order gradient
// (create_graph=True, e.g. a gradient penalty) through them would be silently missing.  Refuse it instead
// (ADVICE r4); DIRT_FUSED_LIGHTING=0 routes dirt_amd.lighting to its framework-op statement, which supports it.
void no_double_backward(const char *fn)
{
    if (at::GradMode::is_enabled())
        throw std::runtime_error(std::string(fn) +
                                 ": the fused HIP backward does not support create_graph=True (double backward); "
                                 "set DIRT_FUSED_LIGHTING=0 to use the framework-op statement");
}

struct VertexNormalsFn : public torch::autograd::Function<VertexNormalsFn> {
    // vertices [*, V, D >= 3] contiguous (only x, y, z read), faces [F, 3] int32 / int64
    static at::Tensor forward(AutogradContext *ctx, at::Tensor vertices, at::Tensor faces)
    {
        c10::hip::HIPGuard guard(vertices.device().index());
        const int64_t V = vertices.size(-2), F = faces.size(0), B = vertices.numel() / std::max<int64_t>(V * vertices.size(-1), 1);
        std::vector<int64_t> shape = vertices.sizes().vec();
        shape.back() = 3;
        at::Tensor summed = at::empty(shape, vertices.options()), normals = at::empty(shape, vertices.options());
        check(g_api.vn_fwd(vertices.data_ptr<float>(), (int)vertices.size(-1), faces.data_ptr(),
                           faces.scalar_type() == at::kLong, (int)B, (int)V, (int)F, summed.data_ptr<float>(),
                           normals.data_ptr<float>(), stream_of(vertices)));
        ctx->save_for_backward({vertices, faces, summed});
        return normals;
    }
    static variable_list backward(AutogradContext *ctx, variable_list grads)
    {
        no_double_backward("vertex_normals");
        auto sv = ctx->get_saved_variables();
        const at::Tensor &vertices = sv[0], &faces = sv[1], &summed = sv[2];
        c10::hip::HIPGuard guard(vertices.device().index());
        const int64_t V = vertices.size(-2), F = faces.size(0), D = vertices.size(-1);
        const int64_t B = vertices.numel() / std::max<int64_t>(V * D, 1);
        at::Tensor g = grad_or_zeros(grads[0], summed);
        at::Tensor gsum = at::empty_like(summed), gv = at::empty(vertices.sizes(), vertices.options());
        check(g_api.vn_bwd(vertices.data_ptr<float>(), (int)D, faces.data_ptr(), faces.scalar_type() == at::kLong,
                           (int)B, (int)V, (int)F, summed.data_ptr<float>(), g.data_ptr<float>(),
                           gsum.data_ptr<float>(), gv.data_ptr<float>(), (int)D, stream_of(vertices)));
        return {gv, at::Tensor()};
    }
};

struct DiffuseFn : public torch::autograd::Function<DiffuseFn> {
    static at::Tensor forward(AutogradContext *ctx, at::Tensor normals, at::Tensor colors, at::Tensor light_direction,
                              at::Tensor light_color, bool double_sided)
    {
        c10::hip::HIPGuard guard(normals.device().index());
        at::Tensor out = at::empty_like(normals);
        check(g_api.diffuse_fwd(normals.data_ptr<float>(), colors.data_ptr<float>(), normals.numel() / 3,
                                light_direction.data_ptr<float>(), light_color.data_ptr<float>(), double_sided,
                                out.data_ptr<float>(), stream_of(normals)));
        ctx->save_for_backward({normals, colors, light_direction, light_color});
        ctx->saved_data["two"] = double_sided;
        return out;
    }
    static variable_list backward(AutogradContext *ctx, variable_list grads)
    {
        no_double_backward("diffuse_directional");
        auto sv = ctx->get_saved_variables();
        const at::Tensor &normals = sv[0], &colors = sv[1];
        c10::hip::HIPGuard guard(normals.device().index());
        at::Tensor g = grad_or_zeros(grads[0], normals);
        const bool wn = ctx->needs_input_grad(0), wc = ctx->needs_input_grad(1);
        at::Tensor gn = wn ? at::empty_like(normals) : at::Tensor(), gc = wc ? at::empty_like(colors) : at::Tensor();
        check(g_api.diffuse_bwd(normals.data_ptr<float>(), colors.data_ptr<float>(), normals.numel() / 3,
                                sv[2].data_ptr<float>(), sv[3].data_ptr<float>(), ctx->saved_data["two"].toBool(),
                                g.data_ptr<float>(), wn ? gn.data_ptr<float>() : nullptr,
                                wc ? gc.data_ptr<float>() : nullptr, stream_of(normals)));
        return {gn, gc, at::Tensor(), at::Tensor(), at::Tensor()};
    }
};

struct DiffusePointFn : public torch::autograd::Function<DiffusePointFn> {
    static at::Tensor forward(AutogradContext *ctx, at::Tensor positions, at::Tensor normals, at::Tensor colors,
                              at::Tensor light_position, at::Tensor light_color, bool double_sided)
    {
        c10::hip::HIPGuard guard(positions.device().index());
        at::Tensor out = at::empty_like(positions);
        check(g_api.point_fwd(positions.data_ptr<float>(), normals.data_ptr<float>(), colors.data_ptr<float>(),
                              positions.numel() / 3, light_position.data_ptr<float>(), light_color.data_ptr<float>(),
                              double_sided, out.data_ptr<float>(), stream_of(positions)));
        ctx->save_for_backward({positions, normals, colors, light_position, light_color});
        ctx->saved_data["two"] = double_sided;
        return out;
    }
    static variable_list backward(AutogradContext *ctx, variable_list grads)
    {
        no_double_backward("diffuse_point");
        auto sv = ctx->get_saved_variables();
        const at::Tensor &positions = sv[0], &normals = sv[1], &colors = sv[2];
        c10::hip::HIPGuard guard(positions.device().index());
        at::Tensor g = grad_or_zeros(grads[0], positions);
        const bool wp = ctx->needs_input_grad(0), wn = ctx->needs_input_grad(1), wc = ctx->needs_input_grad(2);
        at::Tensor gp = wp ? at::empty_like(positions) : at::Tensor(), gn = wn ? at::empty_like(normals) : at::Tensor(),
                   gc = wc ? at::empty_like(colors) : at::Tensor();
        check(g_api.point_bwd(positions.data_ptr<float>(), normals.data_ptr<float>(), colors.data_ptr<float>(),
                              positions.numel() / 3, sv[3].data_ptr<float>(), sv[4].data_ptr<float>(),
                              ctx->saved_data["two"].toBool(), g.data_ptr<float>(), wp ? gp.data_ptr<float>() : nullptr,
                              wn ? gn.data_ptr<float>() : nullptr, wc ? gc.data_ptr<float>() : nullptr,
                              stream_of(positions)));
        return {gp, gn, gc, at::Tensor(), at::Tensor(), at::Tensor()};
    }
};

struct SpecularFn : public torch::autograd::Function<SpecularFn> {
    static at::Tensor forward(AutogradContext *ctx, at::Tensor positions, at::Tensor normals, at::Tensor reflectivities,
                              at::Tensor light_direction, at::Tensor light_color, at::Tensor camera_position,
                              double shininess, bool double_sided)
    {
        c10::hip::HIPGuard guard(positions.device().index());
        at::Tensor out = at::empty_like(positions);
        check(g_api.specular_fwd(positions.data_ptr<float>(), normals.data_ptr<float>(), reflectivities.data_ptr<float>(),
                                 positions.numel() / 3, light_direction.data_ptr<float>(), light_color.data_ptr<float>(),
                                 camera_position.data_ptr<float>(), (float)shininess, double_sided,
                                 out.data_ptr<float>(), stream_of(positions)));
        ctx->save_for_backward({positions, normals, reflectivities, light_direction, light_color, camera_position});
        ctx->saved_data["two"] = double_sided;
        ctx->saved_data["shininess"] = shininess;
        return out;
    }
    static variable_list backward(AutogradContext *ctx, variable_list grads)
    {
        no_double_backward("specular_directional");
        auto sv = ctx->get_saved_variables();
        const at::Tensor &positions = sv[0], &normals = sv[1], &refl = sv[2];
        c10::hip::HIPGuard guard(positions.device().index());
        at::Tensor g = grad_or_zeros(grads[0], positions);
        const bool wp = ctx->needs_input_grad(0), wn = ctx->needs_input_grad(1), wr = ctx->needs_input_grad(2);
        at::Tensor gp = wp ? at::empty_like(positions) : at::Tensor(), gn = wn ? at::empty_like(normals) : at::Tensor(),
                   gr = wr ? at::empty_like(refl) : at::Tensor();
        check(g_api.specular_bwd(positions.data_ptr<float>(), normals.data_ptr<float>(), refl.data_ptr<float>(),
                                 positions.numel() / 3, sv[3].data_ptr<float>(), sv[4].data_ptr<float>(),
                                 sv[5].data_ptr<float>(), (float)ctx->saved_data["shininess"].toDouble(),
                                 ctx->saved_data["two"].toBool(), g.data_ptr<float>(),
                                 wp ? gp.data_ptr<float>() : nullptr, wn ? gn.data_ptr<float>() : nullptr,
                                 wr ? gr.data_ptr<float>() : nullptr, stream_of(positions)));
        return {gp, gn, gr, at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor()};
    }
};

void need_api()
{
    if (!g_api.vn_fwd) throw std::runtime_error("_dirt_torch.init(path) was not called");
}

// the fused helpers take raw device pointers: every operand on the first one's GPU, float32 (or int faces),
// contiguous, with the element counts the kernels index by (dirt_amd/lighting.py checks this before calling)
void check_operands(const char *fn, std::initializer_list<const at::Tensor *> xs, std::initializer_list<const at::Tensor *> params)
{
    const at::Tensor &x0 = **xs.begin();
    auto bad = [&](const char *what) { throw std::invalid_argument(std::string(fn) + ": " + what); };
    if (!x0.is_cuda()) bad("operands must be GPU tensors");
    for (const at::Tensor *x : xs) {
        if (x->device() != x0.device() || x->scalar_type() != at::kFloat || !x->is_contiguous())
            bad("operands must be contiguous float32 tensors on one GPU");
        if (x->sizes() != x0.sizes() || x->dim() < 1 || x->size(-1) != 3) bad("operands must share one [..., 3] shape");
    }
    for (const at::Tensor *p : params)
        if (p->device() != x0.device() || p->scalar_type() != at::kFloat || !p->is_contiguous() || p->numel() != 3)
            bad("light parameters must be contiguous float32 [3] tensors on the operands' GPU");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m)
{
    m.doc() = "dirt_amd rasterise op: C++ autograd function over the C ABI of libdirt_mi355x.so";
    m.def("init", &init, "dlopen libdirt_mi355x.so and resolve the C ABI");
    m.def("rasterise", &rasterise, "rasterise forward (+ registered backward)", py::arg("background"),
          py::arg("vertices"), py::arg("vertex_colors"), py::arg("faces"), py::arg("camera_pos"), py::arg("height"),
          py::arg("width"), py::arg("channels"), py::arg("shader_id"), py::arg("bin_capacity"), py::arg("want_gbuf"),
          py::arg("check_faces"), py::arg("fwd_flags") = (int64_t)DIRT_FWD_SCRATCH_CLEAN);
    m.def("rasterise_checked", &rasterise_checked,
          "Gouraud rasterise of tensor inputs with the wrapper's dtype / device / shape handling",
          py::arg("background"), py::arg("vertices"), py::arg("vertex_colors"), py::arg("faces"), py::arg("height"),
          py::arg("width"), py::arg("channels"), py::arg("bin_capacity"), py::arg("want_gbuf"), py::arg("check_faces"),
          py::arg("fwd_flags") = (int64_t)DIRT_FWD_SCRATCH_CLEAN);
    m.def("scratch_cache_clear", [](bool force) {
        g_scratch.clear(force);
        g_geom.clear();
    }, py::arg("force") = false);
    m.def("scratch_cache_size", []() { return g_scratch.size(); });
    m.def("set_geometry_sharing", [](bool on) {
        const bool prev = GeomCache::flag().exchange(on ? 1 : 0) != 0;
        if (!on) g_geom.clear();
        return prev;
    }, py::arg("enabled"));
    // fused lighting helpers: operands already CUDA float32 and contiguous (dirt_amd/lighting.py checks)
    m.def("vertex_normals", [](at::Tensor vertices, at::Tensor faces) {
        need_api();
        if (!vertices.is_cuda() || vertices.scalar_type() != at::kFloat || !vertices.is_contiguous() ||
            vertices.dim() < 2 || vertices.size(-1) < 3)
            throw std::invalid_argument("vertex_normals: vertices must be a contiguous float32 [..., V, >=3] GPU tensor");
        if (faces.device() != vertices.device() || !faces.is_contiguous() || faces.dim() != 2 || faces.size(1) != 3 ||
            (faces.scalar_type() != at::kInt && faces.scalar_type() != at::kLong))
            throw std::invalid_argument("vertex_normals: faces must be a contiguous int32 / int64 [F, 3] tensor on the vertices' GPU");
        return VertexNormalsFn::apply(vertices, faces);
    });
    m.def("diffuse_directional", [](at::Tensor n, at::Tensor c, at::Tensor ld, at::Tensor lc, bool two) {
        need_api();
        check_operands("diffuse_directional", {&n, &c}, {&ld, &lc});
        return DiffuseFn::apply(n, c, ld, lc, two);
    });
    m.def("diffuse_point", [](at::Tensor p, at::Tensor n, at::Tensor c, at::Tensor lp, at::Tensor lc, bool two) {
        need_api();
        check_operands("diffuse_point", {&p, &n, &c}, {&lp, &lc});
        return DiffusePointFn::apply(p, n, c, lp, lc, two);
    });
    m.def("specular_directional", [](at::Tensor p, at::Tensor n, at::Tensor r, at::Tensor ld, at::Tensor lc,
                                     at::Tensor cam, double shininess, bool two) {
        need_api();
        check_operands("specular_directional", {&p, &n, &r}, {&ld, &lc, &cam});
        return SpecularFn::apply(p, n, r, ld, lc, cam, shininess, two);
    });
}
