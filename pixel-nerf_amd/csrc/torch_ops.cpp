// torch.ops.pnr.* — the renderer's plug point as PyTorch operators, registered
// from libpnr_torch.so over the C ABI of libpnr.so (include/pnr_abi.h).  The operators take
// and return tensors, allocate outputs and scratch through the caching allocator on the
// tensors' device, and run on the current HIP stream; a non-zero pnr_status becomes a
// TORCH_CHECK error carrying pnr_last_error().  Meta kernels give the output shapes so the
// operators trace under torch.compile / FakeTensor.
//
//   pnr::render_rays   NeRFRenderer.forward with a PixelNeRFNet (nerf.py:251-303; the reference
//                      plug point is the model call at nerf.py:212-216); `events`: none, or 7
//                      hipEvent_t handles recorded around the launches (pnr_render_forward_events)
//   pnr::point_query   PixelNeRFNet.forward (models.py:146-266)
//   pnr::composite     NeRFRenderer.composite's volume integral (nerf.py:176-249)
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "../../include/pnr_abi.h"

namespace {

void check(int rc, const char *what) {
    TORCH_CHECK(rc == PNR_OK, what, " failed (status ", rc, "): ", pnr_last_error());
}

void *stream_of(const at::Tensor &t) {
    return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

const float *fptr(const at::Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, " must be on the HIP device");
    TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    return t.data_ptr<float>();
}

const float *opt_fptr(const c10::optional<at::Tensor> &t, const char *name) {
    if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
    return fptr(*t, name);
}

// every tensor of one call lives on the call's device (the library dereferences raw pointers:
// a host or other-device buffer would fault inside a kernel instead of failing here)
void same_device(const at::Tensor &t, const at::Device &dev, const char *name) {
    TORCH_CHECK(t.device() == dev, name, " is on ", t.device(), ", the call runs on ", dev);
}

const void *packed_ptr(const at::Tensor &t, const at::Device &dev, const char *name) {
    TORCH_CHECK(t.defined() && t.numel() > 0, name, " is empty");
    same_device(t, dev, name);
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    return t.data_ptr();
}

void same_device_opt(const c10::optional<at::Tensor> &t, const at::Device &dev, const char *name) {
    if (t.has_value() && t->defined() && t->numel() > 0) same_device(*t, dev, name);
}

pnr_scene make_scene(const at::Tensor &latent_cl, const at::Tensor &cams, int64_t n_obj, int64_t n_views,
                     double image_w, double image_h) {
    TORCH_CHECK(latent_cl.dim() == 4, "latent_cl must be (n_obj * n_views, H_l, W_l, C)");
    pnr_scene s{};
    s.latent = fptr(latent_cl, "latent_cl");
    s.cams = fptr(cams, "cams");
    s.n_obj = (int32_t)n_obj;
    s.n_views = (int32_t)n_views;
    s.latent_h = (int32_t)latent_cl.size(1);
    s.latent_w = (int32_t)latent_cl.size(2);
    s.latent_c = (int32_t)latent_cl.size(3);
    s.image_w = (float)image_w;
    s.image_h = (float)image_h;
    return s;
}

pnr_mlp_desc make_desc(at::IntArrayRef d) {
    TORCH_CHECK(d.size() == 8, "desc = [d_in, d_latent, d_hidden, d_out, n_blocks, combine_layer, pe_n, precision]");
    pnr_mlp_desc m{};
    m.d_in = (int32_t)d[0];
    m.d_latent = (int32_t)d[1];
    m.d_hidden = (int32_t)d[2];
    m.d_out = (int32_t)d[3];
    m.n_blocks = (int32_t)d[4];
    m.combine_layer = (int32_t)d[5];
    m.pe_n = (int32_t)d[6];
    m.precision = (int32_t)d[7];
    return m;
}

at::TensorOptions f32_like(const at::Tensor &t) { return t.options().dtype(at::kFloat); }

// outputs: [coarse_rgb (B,3), coarse_depth (B), coarse_weights (B,Kc) | empty, fine_rgb, fine_depth,
//           fine_weights (B,Kc+Kf) | empty, z_coarse | empty, z_fine | empty]; fine entries empty
//           when n_fine == 0
std::vector<at::Tensor> render_rays(const at::Tensor &latent_cl, const at::Tensor &cams, int64_t n_obj,
                                    int64_t n_views, double image_w, double image_h, at::IntArrayRef desc,
                                    const at::Tensor &coarse_packed, const at::Tensor &fine_packed,
                                    const c10::optional<at::Tensor> &coarse_proj,
                                    const c10::optional<at::Tensor> &fine_proj, const at::Tensor &rays,
                                    int64_t rays_per_obj, int64_t n_coarse, int64_t n_fine, int64_t n_fine_depth,
                                    double depth_std, bool white_bkgd, bool lindisp,
                                    const c10::optional<at::Tensor> &u_coarse, const c10::optional<at::Tensor> &u_fine,
                                    const c10::optional<at::Tensor> &u_fine_jit,
                                    const c10::optional<at::Tensor> &n_depth, int64_t seed, int64_t offset,
                                    bool want_weights, bool want_z, at::IntArrayRef events, int64_t march_mode,
                                    const c10::optional<at::Tensor> &ray_order) {
    TORCH_CHECK(rays.dim() == 2 && rays.size(1) == 8, "rays must be (B, 8)");
    TORCH_CHECK(events.empty() || events.size() == 7, "events: none or 7 hipEvent_t handles");
    const at::Device dev = rays.device();
    c10::OptionalDeviceGuard guard(dev);
    same_device(latent_cl, dev, "latent_cl");
    same_device(cams, dev, "cams");
    const void *cpk = packed_ptr(coarse_packed, dev, "coarse_packed");
    const void *fpk = n_fine > 0 ? packed_ptr(fine_packed, dev, "fine_packed") : nullptr;
    same_device_opt(coarse_proj, dev, "coarse_proj");
    same_device_opt(fine_proj, dev, "fine_proj");
    same_device_opt(u_coarse, dev, "u_coarse");
    same_device_opt(u_fine, dev, "u_fine");
    same_device_opt(u_fine_jit, dev, "u_fine_jit");
    same_device_opt(n_depth, dev, "n_depth");
    const pnr_scene sc = make_scene(latent_cl, cams, n_obj, n_views, image_w, image_h);
    const pnr_mlp_desc d = make_desc(desc);
    const int64_t B = rays.size(0);
    const auto o = f32_like(rays);
    const bool fine = n_fine > 0;
    at::Tensor c_rgb = at::empty({B, 3}, o), c_depth = at::empty({B}, o);
    at::Tensor c_w = (want_weights || fine) ? at::empty({B, n_coarse}, o) : at::empty({0}, o);
    at::Tensor f_rgb = fine ? at::empty({B, 3}, o) : at::empty({0}, o);
    at::Tensor f_depth = fine ? at::empty({B}, o) : at::empty({0}, o);
    at::Tensor f_w = (fine && want_weights) ? at::empty({B, n_coarse + n_fine}, o) : at::empty({0}, o);
    at::Tensor z_c = want_z ? at::empty({B, n_coarse}, o) : at::empty({0}, o);
    at::Tensor z_f = (want_z && fine) ? at::empty({B, n_coarse + n_fine}, o) : at::empty({0}, o);
    pnr_render_out out{};
    out.coarse_rgb = c_rgb.data_ptr<float>();
    out.coarse_depth = c_depth.data_ptr<float>();
    out.coarse_weights = c_w.numel() ? c_w.data_ptr<float>() : nullptr;
    out.fine_rgb = fine ? f_rgb.data_ptr<float>() : nullptr;
    out.fine_depth = fine ? f_depth.data_ptr<float>() : nullptr;
    out.fine_weights = f_w.numel() ? f_w.data_ptr<float>() : nullptr;
    out.z_coarse = z_c.numel() ? z_c.data_ptr<float>() : nullptr;
    out.z_fine = z_f.numel() ? z_f.data_ptr<float>() : nullptr;
    pnr_rays r{fptr(rays, "rays"), B, rays_per_obj};
    pnr_rng rng{};
    rng.u_coarse = opt_fptr(u_coarse, "u_coarse");
    rng.u_fine = opt_fptr(u_fine, "u_fine");
    rng.u_fine_jit = opt_fptr(u_fine_jit, "u_fine_jit");
    rng.n_depth = opt_fptr(n_depth, "n_depth");
    rng.seed = (uint64_t)seed;
    rng.offset = (uint64_t)offset;
    pnr_render_cfg cfg{(int32_t)n_coarse, (int32_t)n_fine, (int32_t)n_fine_depth, (float)depth_std,
                       (int32_t)white_bkgd, (int32_t)lindisp, (int32_t)march_mode, nullptr};
    if (ray_order.has_value() && ray_order->defined()) {   // ABI 8: the march's processing order
        const at::Tensor &ro = *ray_order;
        same_device(ro, dev, "ray_order");
        TORCH_CHECK(ro.scalar_type() == at::kInt && ro.dim() == 1 && ro.size(0) == B && ro.is_contiguous(),
                    "ray_order must be a contiguous int32 (B,) tensor");
        cfg.ray_order = ro.data_ptr<int32_t>();
    }
    const size_t ws_bytes = pnr_render_workspace_bytes(&sc, &cfg, B);
    at::Tensor ws = at::empty({(int64_t)(ws_bytes ? ws_bytes : 1)}, rays.options().dtype(at::kByte));
    void *ev[7] = {};
    for (size_t i = 0; i < events.size(); ++i) ev[i] = reinterpret_cast<void *>((intptr_t)events[i]);
    check(pnr_render_forward_proj(&sc, &d, cpk, fpk, opt_fptr(coarse_proj, "coarse_proj"),
                                  fine ? opt_fptr(fine_proj, "fine_proj") : nullptr, &r, &rng, &cfg, &out,
                                  ws.data_ptr(), ws_bytes, stream_of(rays),
                                  events.empty() ? nullptr : reinterpret_cast<void *const *>(ev)),
          "pnr::render_rays");
    return {c_rgb, c_depth, want_weights ? c_w : at::empty({0}, o), f_rgb, f_depth, f_w, z_c, z_f};
}

std::vector<at::Tensor> render_rays_meta(const at::Tensor &latent_cl, const at::Tensor &cams, int64_t n_obj,
                                         int64_t n_views, double image_w, double image_h, at::IntArrayRef desc,
                                         const at::Tensor &coarse_packed, const at::Tensor &fine_packed,
                                         const c10::optional<at::Tensor> &coarse_proj,
                                         const c10::optional<at::Tensor> &fine_proj, const at::Tensor &rays,
                                         int64_t rays_per_obj, int64_t n_coarse, int64_t n_fine,
                                         int64_t n_fine_depth, double depth_std, bool white_bkgd, bool lindisp,
                                         const c10::optional<at::Tensor> &u_coarse,
                                         const c10::optional<at::Tensor> &u_fine,
                                         const c10::optional<at::Tensor> &u_fine_jit,
                                         const c10::optional<at::Tensor> &n_depth, int64_t seed, int64_t offset,
                                         bool want_weights, bool want_z, at::IntArrayRef events,
                                         int64_t march_mode, const c10::optional<at::Tensor> &ray_order) {
    const int64_t B = rays.size(0);
    const auto o = f32_like(rays);
    const bool fine = n_fine > 0;
    auto e = [&](std::vector<int64_t> s, bool keep) { return keep ? at::empty(s, o) : at::empty({0}, o); };
    return {e({B, 3}, true), e({B}, true), e({B, n_coarse}, want_weights), e({B, 3}, fine), e({B}, fine),
            e({B, n_coarse + n_fine}, fine && want_weights), e({B, n_coarse}, want_z),
            e({B, n_coarse + n_fine}, want_z && fine)};
}

at::Tensor point_query(const at::Tensor &latent_cl, const at::Tensor &cams, int64_t n_obj, int64_t n_views,
                       double image_w, double image_h, at::IntArrayRef desc, const at::Tensor &packed,
                       const c10::optional<at::Tensor> &proj, const at::Tensor &xyz,
                       const c10::optional<at::Tensor> &viewdirs) {
    TORCH_CHECK(xyz.dim() == 3 && xyz.size(2) == 3, "xyz must be (SB, B, 3)");
    TORCH_CHECK(xyz.size(0) == n_obj, "xyz has ", xyz.size(0), " objects, the scene ", n_obj);
    const at::Device dev = xyz.device();
    c10::OptionalDeviceGuard guard(dev);
    same_device(latent_cl, dev, "latent_cl");
    same_device(cams, dev, "cams");
    const void *pk = packed_ptr(packed, dev, "packed");
    same_device_opt(proj, dev, "proj");
    same_device_opt(viewdirs, dev, "viewdirs");
    const pnr_scene sc = make_scene(latent_cl, cams, n_obj, n_views, image_w, image_h);
    const pnr_mlp_desc d = make_desc(desc);
    const int64_t P = xyz.size(0) * xyz.size(1);
    at::Tensor out = at::empty({xyz.size(0), xyz.size(1), 4}, f32_like(xyz));
    const size_t ws_bytes = pnr_point_query_workspace_bytes(&sc, P);
    at::Tensor ws = at::empty({(int64_t)(ws_bytes ? ws_bytes : 1)}, xyz.options().dtype(at::kByte));
    check(pnr_point_query_proj(&sc, &d, pk, opt_fptr(proj, "proj"), fptr(xyz, "xyz"),
                               opt_fptr(viewdirs, "viewdirs"), xyz.size(1), out.data_ptr<float>(), ws.data_ptr(),
                               ws_bytes, stream_of(xyz)),
          "pnr::point_query");
    return out;
}

at::Tensor point_query_meta(const at::Tensor &latent_cl, const at::Tensor &cams, int64_t n_obj, int64_t n_views,
                            double image_w, double image_h, at::IntArrayRef desc, const at::Tensor &packed,
                            const c10::optional<at::Tensor> &proj, const at::Tensor &xyz,
                            const c10::optional<at::Tensor> &viewdirs) {
    return at::empty({xyz.size(0), xyz.size(1), 4}, f32_like(xyz));
}

std::vector<at::Tensor> composite(const at::Tensor &z, const at::Tensor &raw, const at::Tensor &rays,
                                  bool white_bkgd, bool want_weights) {
    TORCH_CHECK(z.dim() == 2 && raw.dim() == 3 && raw.size(2) == 4 && raw.size(0) == z.size(0) &&
                    raw.size(1) == z.size(1),
                "composite: z (B, K), raw (B, K, 4)");
    const int64_t B = z.size(0), K = z.size(1);
    const at::Device dev = z.device();
    c10::OptionalDeviceGuard guard(dev);
    same_device(raw, dev, "raw");
    same_device(rays, dev, "rays");
    const auto o = f32_like(z);
    at::Tensor w = want_weights ? at::empty({B, K}, o) : at::empty({0}, o);
    at::Tensor rgb = at::empty({B, 3}, o), depth = at::empty({B}, o);
    check(pnr_composite(fptr(z, "z"), fptr(raw, "raw"), fptr(rays, "rays"), B, (int32_t)K, (int32_t)white_bkgd,
                        want_weights ? w.data_ptr<float>() : nullptr, rgb.data_ptr<float>(), depth.data_ptr<float>(),
                        stream_of(z)),
          "pnr::composite");
    return {w, rgb, depth};
}

std::vector<at::Tensor> composite_meta(const at::Tensor &z, const at::Tensor &raw, const at::Tensor &rays,
                                       bool white_bkgd, bool want_weights) {
    const auto o = f32_like(z);
    return {want_weights ? at::empty({z.size(0), z.size(1)}, o) : at::empty({0}, o), at::empty({z.size(0), 3}, o),
            at::empty({z.size(0)}, o)};
}

}  // namespace

TORCH_LIBRARY(pnr, m) {
    m.def("render_rays(Tensor latent_cl, Tensor cams, int n_obj, int n_views, float image_w, float image_h, "
          "int[] desc, Tensor coarse_packed, Tensor fine_packed, Tensor? coarse_proj, Tensor? fine_proj, "
          "Tensor rays, int rays_per_obj, int n_coarse, int n_fine, int n_fine_depth, float depth_std, "
          "bool white_bkgd, bool lindisp, Tensor? u_coarse, Tensor? u_fine, Tensor? u_fine_jit, Tensor? n_depth, "
          "int seed, int offset, bool want_weights, bool want_z, int[] events=[], int march_mode=-1, "
          "Tensor? ray_order=None) -> Tensor[]");
    m.def("point_query(Tensor latent_cl, Tensor cams, int n_obj, int n_views, float image_w, float image_h, "
          "int[] desc, Tensor packed, Tensor? proj, Tensor xyz, Tensor? viewdirs) -> Tensor");
    m.def("composite(Tensor z, Tensor raw, Tensor rays, bool white_bkgd, bool want_weights) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(pnr, CUDA, m) {
    m.impl("render_rays", &render_rays);
    m.impl("point_query", &point_query);
    m.impl("composite", &composite);
}

TORCH_LIBRARY_IMPL(pnr, Meta, m) {
    m.impl("render_rays", &render_rays_meta);
    m.impl("point_query", &point_query_meta);
    m.impl("composite", &composite_meta);
}
