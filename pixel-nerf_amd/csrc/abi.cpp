// extern "C" entry points of libpnr.so (declared in include/pnr_abi.h):
// argument validation, workspace carving and the stream-ordered launch
// sequence of the coarse + fine ray march.  No allocation, no host sync.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "march_dev.h"

namespace pnr {

// launchers (march.hip, mlp.hip)
int launch_sample_coarse(const float *, int64_t, int, const RngSrc &, int, float *, hipStream_t);
int launch_sample_fine(const float *, int64_t, int, const float *, const float *, const float *,
                       int, int, float, const RngSrc &, const RngSrc &, const RngSrc &, int, float *,
                       hipStream_t, int *origin = nullptr, float *z_new = nullptr);
int launch_rng_fill(const RngSrc &, int64_t, int, float *, hipStream_t);
int launch_merge_raw(const int *, const float *, const float *, int64_t, int, int, float *, hipStream_t);
int launch_gen_rays(const float *, int64_t, int, int, int, float, float, float, float, float, float,
                    float *, hipStream_t);
int launch_composite(const float *, const float *, const float *, int64_t, int, int, float *,
                     float *, float *, hipStream_t);
size_t mlp_packed_bytes(const pnr_mlp_desc &);
int mlp_check_desc(const pnr_mlp_desc &);
int mlp_pack(const pnr_mlp_weights &, void *, size_t, hipStream_t);
size_t mlp_xsum_bytes(int ns);
int64_t mlp_save_floats(const pnr_mlp_desc &d, int64_t n_points);
size_t mlp_packed_t_bytes(const pnr_mlp_desc &);
int mlp_pack_t(const pnr_mlp_weights &, const void *, void *, size_t, hipStream_t);
int launch_mlp_bwd(const pnr_mlp_desc &, const void *, const void *, const float *, const float *, const float *,
                   int64_t, float *, float *, hipStream_t, float *, void *, size_t, int n_views);
size_t mlp_bwd_workspace_bytes(const pnr_mlp_desc &, int64_t);
size_t wgrad_workspace_bytes(int, int64_t);
int launch_wgrad(const float *const *, const float *const *, float *const *, int, int64_t, void *, size_t,
                 hipStream_t, int arith);
int launch_fold_bn(const pnr_bn_fold *, int, int64_t, hipStream_t);
int launch_latent_cl_bwd(const float *, float *const *, const int32_t *, const int32_t *, const int32_t *, int, int, int,
                         int, hipStream_t);
int launch_latent_cl(const float *const *, const int32_t *, const int32_t *, const int32_t *, int, int, float *,
                     int, int, bool, hipStream_t);
int launch_composite_bwd(const float *, const float *, const float *, int64_t, int, int, const float *,
                         const float *, const float *, float *, float *, hipStream_t);
int launch_points_in_bwd(const float *, const float *, int, int64_t, int64_t, int, const float *, const float *,
                         int, int, float, float, const float *, int, const float *, const float *, float *,
                         float *, const uint8_t *, hipStream_t);
int launch_point_mlp(const pnr_scene &, const pnr_mlp_desc &, const void *, const float *,
                     const float *, int, int64_t, const float *, const float *, int64_t, int64_t,
                     float *, float *, hipStream_t, float *save = nullptr, const float *proj = nullptr,
                     const MarchCfg *march = nullptr);
int sort_width(int n);
int64_t latent_proj_floats(const pnr_scene &, const pnr_mlp_desc &);
int launch_latent_proj(const pnr_scene &, const pnr_mlp_weights &, float *, size_t, hipStream_t);

static thread_local char g_err[1024];
// pnr_render_set_fused: the DEFAULT march mode of calls whose pnr_render_cfg.march_mode is -1:
// the fused ray march (2: draws + composite in the MLP passes, the fine draws in their own
// kernel; 1: those too in the coarse epilogue) or the separate sample / composite kernels (0).
// Set once at start-up by callers that want another default; a call naming its own mode never
// reads it.
static std::atomic<int> g_fused_default{2};

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int fail(int status, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return status;
}

int device_cu_count() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

static int check_scene(const pnr_scene *sc) {
    if (!sc) return fail(PNR_ERR_INVALID, "scene is NULL");
    if (!sc->latent || !sc->cams) return fail(PNR_ERR_INVALID, "scene latent/cams NULL");
    if (sc->n_obj < 1 || sc->n_views < 1) return fail(PNR_ERR_INVALID, "n_obj/n_views < 1");
    if (sc->latent_h < 2 || sc->latent_w < 2)
        return fail(PNR_ERR_INVALID, "latent must be at least 2x2 (align_corners scaling)");
    if (sc->latent_c != 512) return fail(PNR_ERR_UNSUPPORTED, "latent_c must be 512 (got %d)", sc->latent_c);
    if (!(sc->image_w > 0.f) || !(sc->image_h > 0.f)) return fail(PNR_ERR_INVALID, "image size <= 0");
    if ((reinterpret_cast<uintptr_t>(sc->latent) & 15) != 0)
        return fail(PNR_ERR_INVALID, "latent must be 16-byte aligned");
    if ((int64_t)sc->n_obj * sc->n_views * sc->latent_h * sc->latent_w * sc->latent_c >= (1ll << 32))
        return fail(PNR_ERR_UNSUPPORTED, "latent larger than 2^32 floats (32-bit gather offsets)");
    return PNR_OK;
}

static int check_desc_for_scene(const pnr_mlp_desc *d, const pnr_scene *sc) {
    if (!d) return fail(PNR_ERR_INVALID, "mlp desc is NULL");
    int rc = mlp_check_desc(*d);
    if (rc) return rc;
    if (sc->n_views > 1 && d->combine_layer >= d->n_blocks)
        return fail(PNR_ERR_UNSUPPORTED, "n_views > 1 needs combine_layer < n_blocks");
    return PNR_OK;
}

}  // namespace pnr

using namespace pnr;

extern "C" {

int pnr_abi_version(void) { return PNR_ABI_VERSION; }

const char *pnr_last_error(void) { return g_err; }

size_t pnr_mlp_packed_bytes(const pnr_mlp_desc *desc) {
    if (!desc || mlp_check_desc(*desc) != PNR_OK) return 0;
    return mlp_packed_bytes(*desc);
}

int pnr_mlp_pack(const pnr_mlp_weights *w, void *packed, size_t packed_bytes, pnr_stream_t stream) {
    if (!w || !packed) return fail(PNR_ERR_INVALID, "pnr_mlp_pack: NULL argument");
    return mlp_pack(*w, packed, packed_bytes, (hipStream_t)stream);
}

size_t pnr_point_query_workspace_bytes(const pnr_scene *scene, int64_t n_points) {
    (void)n_points;
    return scene ? align_up(mlp_xsum_bytes(scene->n_views)) : 0;
}

int pnr_point_query(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                    const float *xyz, const float *viewdirs, int64_t points_per_obj, float *out,
                    void *workspace, size_t workspace_bytes, pnr_stream_t stream) {
    return pnr_point_query_proj(scene, desc, packed, nullptr, xyz, viewdirs, points_per_obj, out, workspace,
                                workspace_bytes, stream);
}

size_t pnr_latent_project_bytes(const pnr_scene *scene, const pnr_mlp_desc *desc) {
    if (!scene || !desc || check_scene(scene) != PNR_OK || mlp_check_desc(*desc) != PNR_OK) return 0;
    return sizeof(float) * (size_t)latent_proj_floats(*scene, *desc);
}

int pnr_latent_project(const pnr_scene *scene, const pnr_mlp_weights *w, float *proj, size_t proj_bytes,
                       pnr_stream_t stream) {
    int rc = check_scene(scene);
    if (rc) return rc;
    if (!w || !proj) return fail(PNR_ERR_INVALID, "pnr_latent_project: NULL argument");
    if ((rc = check_desc_for_scene(&w->desc, scene))) return rc;
    if ((reinterpret_cast<uintptr_t>(proj) & 15) != 0)
        return fail(PNR_ERR_INVALID, "pnr_latent_project: proj must be 16-byte aligned");
    return launch_latent_proj(*scene, *w, proj, proj_bytes, (hipStream_t)stream);
}

int pnr_point_query_proj(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                         const float *proj, const float *xyz, const float *viewdirs, int64_t points_per_obj,
                         float *out, void *workspace, size_t workspace_bytes, pnr_stream_t stream) {
    int rc = check_scene(scene);
    if (rc) return rc;
    if ((rc = check_desc_for_scene(desc, scene))) return rc;
    if (!packed || !xyz || !out) return fail(PNR_ERR_INVALID, "pnr_point_query: NULL pointer");
    if (points_per_obj < 0) return fail(PNR_ERR_INVALID, "points_per_obj < 0");
    const int64_t n_points = points_per_obj * scene->n_obj;
    if (n_points == 0) return PNR_OK;
    const size_t need = pnr_point_query_workspace_bytes(scene, n_points);
    if (need && (!workspace || workspace_bytes < need))
        return fail(PNR_ERR_WORKSPACE, "pnr_point_query: workspace %zu < %zu", workspace_bytes, need);
    if (proj && (reinterpret_cast<uintptr_t>(proj) & 15) != 0)
        return fail(PNR_ERR_INVALID, "pnr_point_query_proj: proj must be 16-byte aligned");
    return launch_point_mlp(*scene, *desc, packed, nullptr, nullptr, 0, 1, xyz, viewdirs,
                            points_per_obj, n_points, out, static_cast<float *>(workspace),
                            (hipStream_t)stream, nullptr, proj);
}

size_t pnr_point_save_floats(const pnr_mlp_desc *desc, int64_t n_points) {
    if (!desc || n_points < 0 || mlp_check_desc(*desc) != PNR_OK) return 0;
    return (size_t)mlp_save_floats(*desc, n_points);
}

static int check_rays_z(const pnr_scene *scene, const pnr_rays *rays, const float *z, int32_t k) {
    if (!rays || (rays->n_rays > 0 && (!rays->rays || !z))) return fail(PNR_ERR_INVALID, "rays / z NULL");
    if (rays->n_rays < 0 || k < 1) return fail(PNR_ERR_INVALID, "bad n_rays / k");
    if (rays->rays_per_obj < 1 || rays->n_rays != rays->rays_per_obj * scene->n_obj)
        return fail(PNR_ERR_INVALID, "n_rays must equal rays_per_obj * n_obj");
    return PNR_OK;
}

int pnr_render_points(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                      const pnr_rays *rays, const float *z, int32_t k, float *out, float *save,
                      void *workspace, size_t workspace_bytes, pnr_stream_t stream) {
    int rc = check_scene(scene);
    if (rc) return rc;
    if ((rc = check_desc_for_scene(desc, scene))) return rc;
    if ((rc = check_rays_z(scene, rays, z, k))) return rc;
    if (!packed || !out) return fail(PNR_ERR_INVALID, "pnr_render_points: NULL pointer");
    const int64_t n_points = rays->n_rays * k;
    if (n_points == 0) return PNR_OK;
    const size_t need = pnr_point_query_workspace_bytes(scene, n_points);
    if (need && (!workspace || workspace_bytes < need))
        return fail(PNR_ERR_WORKSPACE, "pnr_render_points: workspace %zu < %zu", workspace_bytes, need);
    return launch_point_mlp(*scene, *desc, packed, rays->rays, z, k, rays->rays_per_obj, nullptr, nullptr, 1,
                            n_points, out, static_cast<float *>(workspace), (hipStream_t)stream, save);
}

int pnr_composite_backward(const float *z, const float *raw, const float *rays, int64_t n_rays, int32_t k,
                           int32_t white_bkgd, const float *d_rgb, const float *d_depth,
                           const float *d_weights, float *d_raw, float *d_z, pnr_stream_t stream) {
    if (n_rays < 0 || k < 1) return fail(PNR_ERR_INVALID, "pnr_composite_backward: bad sizes");
    if (k > 256) return fail(PNR_ERR_UNSUPPORTED, "pnr_composite_backward: k <= 256");
    if (n_rays == 0) return PNR_OK;
    if (!z || !raw || !rays || !d_rgb || !d_raw) return fail(PNR_ERR_INVALID, "pnr_composite_backward: NULL");
    if (((reinterpret_cast<uintptr_t>(raw) | reinterpret_cast<uintptr_t>(d_raw)) & 15) != 0)
        return fail(PNR_ERR_INVALID, "raw / d_raw must be 16-byte aligned");
    return launch_composite_bwd(z, raw, rays, n_rays, k, white_bkgd, d_rgb, d_depth, d_weights, d_raw, d_z,
                                (hipStream_t)stream);
}

int pnr_points_input_backward_masked(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                                     const pnr_rays *rays, const float *z, int32_t k, const float *d_feat,
                                     const float *d_zlat, float *d_latent, float *d_z, const uint8_t *z_mask,
                                     pnr_stream_t stream) {
    int rc = check_scene(scene);
    if (rc) return rc;
    if ((rc = check_desc_for_scene(desc, scene))) return rc;
    if ((rc = check_rays_z(scene, rays, z, k))) return rc;
    if (scene->latent_c != 512) return fail(PNR_ERR_UNSUPPORTED, "input backward: latent_c == 512");
    if (!packed || !d_feat || !d_zlat) return fail(PNR_ERR_INVALID, "pnr_points_input_backward: NULL");
    return launch_points_in_bwd(rays->rays, z, k, rays->rays_per_obj, rays->n_rays * k, scene->n_views, scene->cams,
                                scene->latent, scene->latent_h, scene->latent_w, scene->image_w,
                                scene->image_h, static_cast<const float *>(packed), desc->pe_n, d_feat,
                                d_zlat, d_latent, d_z, z_mask, (hipStream_t)stream);
}

int pnr_points_input_backward(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                              const pnr_rays *rays, const float *z, int32_t k, const float *d_feat,
                              const float *d_zlat, float *d_latent, float *d_z, pnr_stream_t stream) {
    return pnr_points_input_backward_masked(scene, desc, packed, rays, z, k, d_feat, d_zlat, d_latent, d_z, nullptr,
                                            stream);
}

size_t pnr_mlp_packed_t_bytes(const pnr_mlp_desc *desc) {
    if (!desc) return 0;
    return mlp_packed_t_bytes(*desc);
}

int pnr_mlp_pack_t(const pnr_mlp_weights *w, const void *packed, void *packed_t, size_t packed_t_bytes,
                   pnr_stream_t stream) {
    if (!w || !packed || !packed_t) return fail(PNR_ERR_INVALID, "pnr_mlp_pack_t: NULL argument");
    return mlp_pack_t(*w, packed, packed_t, packed_t_bytes, (hipStream_t)stream);
}

int pnr_mlp_backward(const pnr_mlp_desc *desc, const void *packed, const void *packed_t, const float *lin_out_w,
                     const float *save, const float *d_o, int64_t n_points, float *dy, float *d_zlat,
                     pnr_stream_t stream) {
    return pnr_mlp_backward_bias(desc, packed, packed_t, lin_out_w, save, d_o, n_points, dy, d_zlat, nullptr,
                                 nullptr, 0, stream);
}

size_t pnr_mlp_backward_workspace_bytes(const pnr_mlp_desc *desc, int64_t n_points) {
    return desc ? mlp_bwd_workspace_bytes(*desc, n_points) : 0;
}

int pnr_mlp_backward_bias(const pnr_mlp_desc *desc, const void *packed, const void *packed_t,
                          const float *lin_out_w, const float *save, const float *d_o, int64_t n_points, float *dy,
                          float *d_zlat, float *d_bias, void *workspace, size_t workspace_bytes,
                          pnr_stream_t stream) {
    return pnr_mlp_backward_views(desc, packed, packed_t, lin_out_w, save, d_o, n_points, 1, dy, d_zlat, d_bias,
                                  workspace, workspace_bytes, stream);
}

int pnr_mlp_backward_views(const pnr_mlp_desc *desc, const void *packed, const void *packed_t,
                           const float *lin_out_w, const float *save, const float *d_o, int64_t n_points,
                           int32_t n_views, float *dy, float *d_zlat, float *d_bias, void *workspace,
                           size_t workspace_bytes, pnr_stream_t stream) {
    if (!desc || n_points < 0 || n_views < 1) return fail(PNR_ERR_INVALID, "pnr_mlp_backward: bad arguments");
    if (n_points > 0 && (!packed || !packed_t || !lin_out_w || !save || !d_o || !dy))
        return fail(PNR_ERR_INVALID, "pnr_mlp_backward: NULL argument");
    if (((reinterpret_cast<uintptr_t>(lin_out_w) | reinterpret_cast<uintptr_t>(save) |
          reinterpret_cast<uintptr_t>(d_o) | reinterpret_cast<uintptr_t>(dy) |
          reinterpret_cast<uintptr_t>(d_zlat)) & 15) != 0)
        return fail(PNR_ERR_INVALID, "pnr_mlp_backward: buffers must be 16-byte aligned");
    return launch_mlp_bwd(*desc, packed, packed_t, lin_out_w, save, d_o, n_points, dy, d_zlat, (hipStream_t)stream,
                          d_bias, workspace, workspace_bytes, n_views);
}

size_t pnr_weight_grad_workspace_bytes(int32_t n_layers, int64_t n_points) {
    return wgrad_workspace_bytes(n_layers, n_points);
}

int pnr_weight_grad(const float *const *dy, const float *const *x, float *const *d_weight, int32_t n_layers,
                    int64_t n_points, void *workspace, size_t workspace_bytes, pnr_stream_t stream) {
    if (!dy || !x || !d_weight) return fail(PNR_ERR_INVALID, "pnr_weight_grad: NULL argument");
    return launch_wgrad(dy, x, d_weight, n_layers, n_points, workspace, workspace_bytes, (hipStream_t)stream,
                        PNR_WGRAD_F16X3);
}

int pnr_weight_grad_arith(const float *const *dy, const float *const *x, float *const *d_weight, int32_t n_layers,
                          int64_t n_points, int32_t arith, void *workspace, size_t workspace_bytes,
                          pnr_stream_t stream) {
    if (!dy || !x || !d_weight) return fail(PNR_ERR_INVALID, "pnr_weight_grad_arith: NULL argument");
    return launch_wgrad(dy, x, d_weight, n_layers, n_points, workspace, workspace_bytes, (hipStream_t)stream, arith);
}

// workspace layout of pnr_render_forward
struct RenderWs {
    size_t z_c, raw_c, w_c, z_f, raw_f, xsum, origin, z_new, raw_new, total;
};

static RenderWs render_ws(const pnr_scene *sc, const pnr_render_cfg *cfg, int64_t n) {
    RenderWs w;
    const size_t kc = (size_t)cfg->n_coarse, kall = (size_t)(cfg->n_coarse + cfg->n_fine);
    size_t o = 0;
    w.z_c = o; o += align_up(sizeof(float) * n * kc);
    w.raw_c = o; o += align_up(sizeof(float) * n * kc * 4);
    w.w_c = o; o += align_up(sizeof(float) * n * kc);
    w.z_f = o; o += cfg->n_fine > 0 ? align_up(sizeof(float) * n * kall) : 0;
    w.raw_f = o; o += cfg->n_fine > 0 ? align_up(sizeof(float) * n * kall * 4) : 0;
    w.xsum = o; o += align_up(mlp_xsum_bytes(sc->n_views));
    // coarse-output reuse when the fine pass runs the coarse MLP (see pnr_render_forward_proj)
    const size_t kf = (size_t)cfg->n_fine;
    w.origin = o; o += kf > 0 ? align_up(sizeof(int) * n * kall) : 0;
    w.z_new = o; o += kf > 0 ? align_up(sizeof(float) * n * kf) : 0;
    w.raw_new = o; o += kf > 0 ? align_up(sizeof(float) * n * kf * 4) : 0;
    w.total = o;
    return w;
}

size_t pnr_render_workspace_bytes(const pnr_scene *scene, const pnr_render_cfg *cfg, int64_t n_rays) {
    if (!scene || !cfg || n_rays < 0) return 0;
    return render_ws(scene, cfg, n_rays).total;
}

int pnr_render_forward(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *coarse_packed,
                       const void *fine_packed, const pnr_rays *rays, const pnr_rng *rng,
                       const pnr_render_cfg *cfg, const pnr_render_out *out, void *workspace,
                       size_t workspace_bytes, pnr_stream_t stream) {
    return pnr_render_forward_events(scene, desc, coarse_packed, fine_packed, rays, rng, cfg, out,
                                     workspace, workspace_bytes, stream, nullptr);
}

int pnr_render_forward_events(const pnr_scene *scene, const pnr_mlp_desc *desc,
                              const void *coarse_packed, const void *fine_packed,
                              const pnr_rays *rays, const pnr_rng *rng, const pnr_render_cfg *cfg,
                              const pnr_render_out *out, void *workspace, size_t workspace_bytes,
                              pnr_stream_t stream, void *const *events) {
    return pnr_render_forward_proj(scene, desc, coarse_packed, fine_packed, nullptr, nullptr, rays, rng, cfg,
                                   out, workspace, workspace_bytes, stream, events);
}

int pnr_render_forward_proj(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *coarse_packed,
                            const void *fine_packed, const float *coarse_proj, const float *fine_proj,
                            const pnr_rays *rays, const pnr_rng *rng, const pnr_render_cfg *cfg,
                            const pnr_render_out *out, void *workspace, size_t workspace_bytes,
                            pnr_stream_t stream, void *const *events) {
    int rc = check_scene(scene);
    if (rc) return rc;
    if ((rc = check_desc_for_scene(desc, scene))) return rc;
    if (!rays || !rng || !cfg || !out) return fail(PNR_ERR_INVALID, "pnr_render_forward: NULL struct");
    if (!coarse_packed) return fail(PNR_ERR_INVALID, "coarse_packed is NULL");
    const int kc = cfg->n_coarse, kf = cfg->n_fine, kfd = cfg->n_fine_depth;
    if (kc < 1) return fail(PNR_ERR_INVALID, "n_coarse < 1");
    if (cfg->march_mode < -1 || cfg->march_mode > 3)
        return fail(PNR_ERR_INVALID, "march_mode must be -1 (default), 0, 1, 2 or 3 (got %d)", cfg->march_mode);
    const int mode = cfg->march_mode >= 0 ? cfg->march_mode : g_fused_default.load(std::memory_order_relaxed);
    if (kf < 0 || kfd < 0 || kfd > kf) return fail(PNR_ERR_INVALID, "need 0 <= n_fine_depth <= n_fine");
    if (kc + kf > 1024) return fail(PNR_ERR_UNSUPPORTED, "n_coarse + n_fine must be <= 1024");
    if (kf > 0 && !fine_packed) return fail(PNR_ERR_INVALID, "fine_packed is NULL");
    if (((reinterpret_cast<uintptr_t>(coarse_proj) | reinterpret_cast<uintptr_t>(fine_proj)) & 15) != 0)
        return fail(PNR_ERR_INVALID, "latent projections must be 16-byte aligned");
    const int64_t n = rays->n_rays;
    if (n < 0 || !rays->rays) return fail(PNR_ERR_INVALID, "bad rays");
    if (n == 0) return PNR_OK;
    if (rays->rays_per_obj <= 0 || n % rays->rays_per_obj != 0 || n / rays->rays_per_obj != scene->n_obj)
        return fail(PNR_ERR_INVALID, "n_rays (%lld) must be n_obj (%d) x rays_per_obj (%lld)",
                    (long long)n, scene->n_obj, (long long)rays->rays_per_obj);
    // injected streams, or counter mode when every stream pointer is NULL (pnr_abi.h)
    const bool counter = !rng->u_coarse && !rng->u_fine && !rng->u_fine_jit && !rng->n_depth;
    if (!counter) {
        if (!rng->u_coarse) return fail(PNR_ERR_INVALID, "u_coarse stream is NULL");
        if (kf - kfd > 0 && (!rng->u_fine || !rng->u_fine_jit)) return fail(PNR_ERR_INVALID, "fine streams NULL");
        if (kfd > 0 && !rng->n_depth) return fail(PNR_ERR_INVALID, "n_depth stream NULL");
    }
    const RngSrc r_uc{rng->u_coarse, rng->seed, rng->offset, PNR_RNG_U_COARSE};
    const RngSrc r_uf{rng->u_fine, rng->seed, rng->offset, PNR_RNG_U_FINE};
    const RngSrc r_uj{rng->u_fine_jit, rng->seed, rng->offset, PNR_RNG_U_FINE_JIT};
    const RngSrc r_nd{rng->n_depth, rng->seed, rng->offset, PNR_RNG_N_DEPTH};
    if (!out->coarse_rgb || !out->coarse_depth) return fail(PNR_ERR_INVALID, "coarse outputs NULL");
    if (kf > 0 && (!out->fine_rgb || !out->fine_depth)) return fail(PNR_ERR_INVALID, "fine outputs NULL");
    const RenderWs w = render_ws(scene, cfg, n);
    if (!workspace || workspace_bytes < w.total)
        return fail(PNR_ERR_WORKSPACE, "pnr_render_forward: workspace %zu < %zu", workspace_bytes, w.total);
    char *ws = static_cast<char *>(workspace);
    hipStream_t st = (hipStream_t)stream;
    float *zc = out->z_coarse ? out->z_coarse : reinterpret_cast<float *>(ws + w.z_c);
    float *rawc = reinterpret_cast<float *>(ws + w.raw_c);
    float *wc = out->coarse_weights ? out->coarse_weights : reinterpret_cast<float *>(ws + w.w_c);
    float *xsum = reinterpret_cast<float *>(ws + w.xsum);
    auto mark = [&](int i) -> int {
        if (!events || !events[i]) return PNR_OK;
        hipError_t e = hipEventRecord((hipEvent_t)events[i], st);
        return e == hipSuccess ? PNR_OK : fail(PNR_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(e));
    };

    // Fused ray march (default): each pass is ONE k_point_mlp launch whose prologue draws the
    // coarse depths and whose epilogue composites the ray from LDS (raw never reaches HBM); the
    // coarse epilogue also draws the fine samples.  Needs rays that are whole 64-point tiles
    // (K = 64 or 128); other shapes, and the coarse-output reuse below, take the separate
    // sample / composite kernels, which run the same device code (march_dev.h).
    const int kall = kc + kf;
    // mlp_fine is None (the coarse pack passed twice, models.py:242-255; eval_approx.py --coarse):
    // the kc coarse samples re-enter the fine pass with the MLP that already evaluated them, so
    // only the kf new samples run through it and the coarse outputs are merged in.
    const bool reuse = kf > 0 && fine_packed == coarse_packed && fine_proj == coarse_proj;
    const bool fused = mode != 0;
    const bool fuse_c = fused && kc % 64 == 0 && kc <= 128;
    const bool fuse_s = fuse_c && mode == 1 && kf > 0 && !reuse &&
                        kc <= 64 && sort_width(kall) <= 128;
    const bool fuse_f = fused && kf > 0 && !reuse && kall % 64 == 0 && kall <= 128;
    float *zf = kf > 0 ? (out->z_fine ? out->z_fine : reinterpret_cast<float *>(ws + w.z_f)) : nullptr;
    // mode 3: both passes in ONE launch (a ray's coarse tile, then its fine tiles; the fine depths
    // stay in LDS), for kc = 64 and kc + kf = 128 with both projections; other shapes run mode 2
    const bool single = mode == 3 && fuse_c && kf > 0 && !reuse && kc == 64 && kall == 128 &&
                        sort_width(kall) <= 128 && coarse_proj && fine_proj;
    if (single) {
        MarchCfg m = {};
        m.order = cfg->ray_order;
        m.kpt = 1;
        m.sample_coarse = 1;
        m.lindisp = cfg->lindisp;
        m.white_bkgd = cfg->white_bkgd;
        m.u_coarse = r_uc;
        m.z_out = out->z_coarse;
        m.weights = out->coarse_weights;
        m.rgb = out->coarse_rgb;
        m.depth = out->coarse_depth;
        m.kf = kf;
        m.kfd = kfd;
        m.n_sort = sort_width(kall);
        m.depth_std = cfg->depth_std;
        m.u_fine = r_uf;
        m.u_jit = r_uj;
        m.n_depth = r_nd;
        m.z_fine = out->z_fine;   // NULL unless the caller wants the fine depths
        m.single = 1;
        m.kpt_f = kall / 64;
        m.packed_f = static_cast<const float *>(fine_packed);
        m.proj_f = fine_proj;
        m.weights_f = out->fine_weights;
        m.rgb_f = out->fine_rgb;
        m.depth_f = out->fine_depth;
        if ((rc = mark(0)) || (rc = mark(1))) return rc;
        if ((rc = launch_point_mlp(*scene, *desc, coarse_packed, rays->rays, zc, kc, rays->rays_per_obj, nullptr,
                                   nullptr, 1, n * (kc + kall), nullptr, xsum, st, nullptr, coarse_proj, &m)))
            return rc;
        for (int i = 2; i <= 6; ++i)
            if ((rc = mark(i))) return rc;
        return PNR_OK;
    }

    // coarse pass (nerf.py:273-276)
    if ((rc = mark(0))) return rc;
    if (fuse_c) {
        MarchCfg m = {};
        m.order = cfg->ray_order;
        m.kpt = kc / 64;
        m.sample_coarse = 1;
        m.lindisp = cfg->lindisp;
        m.white_bkgd = cfg->white_bkgd;
        m.u_coarse = r_uc;
        m.z_out = fuse_s ? out->z_coarse : zc;
        m.weights = fuse_s ? out->coarse_weights : wc;
        m.rgb = out->coarse_rgb;
        m.depth = out->coarse_depth;
        if (fuse_s) {
            m.kf = kf;
            m.kfd = kfd;
            m.n_sort = sort_width(kall);
            m.depth_std = cfg->depth_std;
            m.u_fine = r_uf;
            m.u_jit = r_uj;
            m.n_depth = r_nd;
            m.z_fine = zf;
        }
        if ((rc = mark(1))) return rc;
        if ((rc = launch_point_mlp(*scene, *desc, coarse_packed, rays->rays, zc, kc, rays->rays_per_obj, nullptr,
                                   nullptr, 1, n * kc, reuse ? rawc : nullptr, xsum, st, nullptr, coarse_proj, &m)))
            return rc;
        if ((rc = mark(2))) return rc;
    } else {
        if ((rc = launch_sample_coarse(rays->rays, n, kc, r_uc, cfg->lindisp, zc, st))) return rc;
        if ((rc = mark(1))) return rc;
        if ((rc = launch_point_mlp(*scene, *desc, coarse_packed, rays->rays, zc, kc, rays->rays_per_obj,
                                   nullptr, nullptr, 1, n * kc, rawc, xsum, st, nullptr, coarse_proj)))
            return rc;
        if ((rc = mark(2))) return rc;
        if ((rc = launch_composite(zc, rawc, rays->rays, n, kc, cfg->white_bkgd, wc, out->coarse_rgb,
                                   out->coarse_depth, st)))
            return rc;
    }
    if ((rc = mark(3))) return rc;
    if (kf == 0) return PNR_OK;
    // fine pass (nerf.py:284-301)
    float *rawf = reinterpret_cast<float *>(ws + w.raw_f);
    int *origin = reuse ? reinterpret_cast<int *>(ws + w.origin) : nullptr;
    float *z_new = reuse ? reinterpret_cast<float *>(ws + w.z_new) : nullptr;
    if (!fuse_s && (rc = launch_sample_fine(rays->rays, n, kc, zc, wc, out->coarse_depth, kf, kfd, cfg->depth_std,
                                            r_uf, r_uj, r_nd, cfg->lindisp, zf, st, origin, z_new)))
        return rc;
    if ((rc = mark(4))) return rc;
    if (fuse_f) {
        MarchCfg m = {};
        m.order = cfg->ray_order;
        m.kpt = kall / 64;
        m.white_bkgd = cfg->white_bkgd;
        m.weights = out->fine_weights;
        m.rgb = out->fine_rgb;
        m.depth = out->fine_depth;
        if ((rc = launch_point_mlp(*scene, *desc, fine_packed, rays->rays, zf, kall, rays->rays_per_obj, nullptr,
                                   nullptr, 1, n * kall, nullptr, xsum, st, nullptr, fine_proj, &m)))
            return rc;
        if ((rc = mark(5))) return rc;
        return mark(6);
    }
    if (reuse) {
        float *raw_new = reinterpret_cast<float *>(ws + w.raw_new);
        if ((rc = launch_point_mlp(*scene, *desc, fine_packed, rays->rays, z_new, kf, rays->rays_per_obj,
                                   nullptr, nullptr, 1, n * kf, raw_new, xsum, st, nullptr, fine_proj)))
            return rc;
        if ((rc = launch_merge_raw(origin, rawc, raw_new, n, kc, kf, rawf, st))) return rc;
    } else if ((rc = launch_point_mlp(*scene, *desc, fine_packed, rays->rays, zf, kall, rays->rays_per_obj,
                                      nullptr, nullptr, 1, n * kall, rawf, xsum, st, nullptr, fine_proj))) {
        return rc;
    }
    if ((rc = mark(5))) return rc;
    if ((rc = launch_composite(zf, rawf, rays->rays, n, kall, cfg->white_bkgd, out->fine_weights,
                               out->fine_rgb, out->fine_depth, st)))
        return rc;
    return mark(6);
}

int32_t pnr_render_set_fused(int32_t on) { return g_fused_default.exchange(on < 0 || on > 3 ? 2 : on); }

int pnr_sample_coarse(const float *rays, int64_t n_rays, int32_t n_coarse, const float *u_coarse,
                      int32_t lindisp, float *z, pnr_stream_t stream) {
    if (n_rays < 0 || n_coarse < 1) return fail(PNR_ERR_INVALID, "pnr_sample_coarse: bad sizes");
    if (n_rays > 0 && (!rays || !u_coarse || !z)) return fail(PNR_ERR_INVALID, "pnr_sample_coarse: NULL");
    return launch_sample_coarse(rays, n_rays, n_coarse, RngSrc{u_coarse, 0, 0, PNR_RNG_U_COARSE}, lindisp, z,
                                (hipStream_t)stream);
}

int pnr_sample_fine(const float *rays, int64_t n_rays, int32_t n_coarse, const float *z_coarse,
                    const float *coarse_weights, const float *coarse_depth, int32_t n_fine,
                    int32_t n_fine_depth, float depth_std, const float *u_fine,
                    const float *u_fine_jit, const float *n_depth, int32_t lindisp, float *z_fine,
                    pnr_stream_t stream) {
    if (n_rays < 0 || n_coarse < 1 || n_fine < 1 || n_fine_depth < 0 || n_fine_depth > n_fine)
        return fail(PNR_ERR_INVALID, "pnr_sample_fine: bad sizes");
    if (n_coarse + n_fine > 1024) return fail(PNR_ERR_UNSUPPORTED, "n_coarse + n_fine must be <= 1024");
    if (n_rays == 0) return PNR_OK;
    if (!rays || !z_coarse || !coarse_weights || !z_fine) return fail(PNR_ERR_INVALID, "pnr_sample_fine: NULL");
    if (n_fine - n_fine_depth > 0 && (!u_fine || !u_fine_jit)) return fail(PNR_ERR_INVALID, "fine streams NULL");
    if (n_fine_depth > 0 && (!n_depth || !coarse_depth)) return fail(PNR_ERR_INVALID, "depth inputs NULL");
    return launch_sample_fine(rays, n_rays, n_coarse, z_coarse, coarse_weights, coarse_depth, n_fine,
                              n_fine_depth, depth_std, RngSrc{u_fine, 0, 0, PNR_RNG_U_FINE},
                              RngSrc{u_fine_jit, 0, 0, PNR_RNG_U_FINE_JIT}, RngSrc{n_depth, 0, 0, PNR_RNG_N_DEPTH},
                              lindisp, z_fine, (hipStream_t)stream);
}

int pnr_rng_fill(uint64_t seed, uint64_t offset, int32_t stream, int64_t n_rays, int32_t width, float *out,
                 pnr_stream_t stream_h) {
    if (stream < PNR_RNG_U_COARSE || stream > PNR_RNG_N_DEPTH) return fail(PNR_ERR_INVALID, "pnr_rng_fill: bad stream");
    if (n_rays < 0 || width < 0) return fail(PNR_ERR_INVALID, "pnr_rng_fill: bad sizes");
    if (n_rays * (int64_t)width == 0) return PNR_OK;
    if (!out) return fail(PNR_ERR_INVALID, "pnr_rng_fill: NULL");
    return launch_rng_fill(RngSrc{nullptr, seed, offset, stream}, n_rays, width, out, (hipStream_t)stream_h);
}

int pnr_composite(const float *z, const float *raw, const float *rays, int64_t n_rays, int32_t k,
                  int32_t white_bkgd, float *weights, float *rgb, float *depth, pnr_stream_t stream) {
    if (n_rays < 0 || k < 1) return fail(PNR_ERR_INVALID, "pnr_composite: bad sizes");
    if (n_rays == 0) return PNR_OK;
    if (!z || !raw || !rays || !rgb || !depth) return fail(PNR_ERR_INVALID, "pnr_composite: NULL");
    if ((reinterpret_cast<uintptr_t>(raw) & 15) != 0) return fail(PNR_ERR_INVALID, "raw must be 16-byte aligned");
    return launch_composite(z, raw, rays, n_rays, k, white_bkgd, weights, rgb, depth, (hipStream_t)stream);
}

int pnr_latent_channels_last(const float *const *maps, const int32_t *channels, const int32_t *heights,
                             const int32_t *widths, int32_t n_maps, int32_t n_images, float *latent_cl,
                             int32_t out_h, int32_t out_w, pnr_stream_t stream) {
    if (!maps || !channels || !heights || !widths || !latent_cl)
        return fail(PNR_ERR_INVALID, "pnr_latent_channels_last: NULL");
    if (n_images < 0 || out_h < 1 || out_w < 1) return fail(PNR_ERR_INVALID, "pnr_latent_channels_last: bad sizes");
    return launch_latent_cl(maps, channels, heights, widths, n_maps, n_images, latent_cl, out_h, out_w, false,
                            (hipStream_t)stream);
}

int pnr_latent_channels_last_nhwc(const float *const *maps, const int32_t *channels, const int32_t *heights,
                                  const int32_t *widths, int32_t n_maps, int32_t n_images, float *latent_cl,
                                  int32_t out_h, int32_t out_w, pnr_stream_t stream) {
    if (!maps || !channels || !heights || !widths || !latent_cl)
        return fail(PNR_ERR_INVALID, "pnr_latent_channels_last_nhwc: NULL");
    if (n_images < 0 || out_h < 1 || out_w < 1)
        return fail(PNR_ERR_INVALID, "pnr_latent_channels_last_nhwc: bad sizes");
    return launch_latent_cl(maps, channels, heights, widths, n_maps, n_images, latent_cl, out_h, out_w, true,
                            (hipStream_t)stream);
}

int pnr_latent_channels_last_backward(const float *g, float *const *d_maps, const int32_t *channels,
                                      const int32_t *heights, const int32_t *widths, int32_t n_maps,
                                      int32_t n_images, int32_t out_h, int32_t out_w, pnr_stream_t stream) {
    if (!d_maps || !channels || !heights || !widths)
        return fail(PNR_ERR_INVALID, "pnr_latent_channels_last_backward: NULL");
    return launch_latent_cl_bwd(g, d_maps, channels, heights, widths, n_maps, n_images, out_h, out_w,
                                (hipStream_t)stream);
}

int pnr_fold_batchnorm(const pnr_bn_fold *folds, int32_t n_folds, int64_t max_elems, pnr_stream_t stream) {
    if (n_folds < 0 || n_folds > 65535 || max_elems < 0) return fail(PNR_ERR_INVALID, "pnr_fold_batchnorm: bad sizes");
    if (n_folds > 0 && !folds) return fail(PNR_ERR_INVALID, "pnr_fold_batchnorm: NULL");
    return launch_fold_bn(folds, n_folds, max_elems, (hipStream_t)stream);
}

int pnr_gen_rays(const float *poses, int64_t n_images, int32_t pose_rows, int32_t width, int32_t height,
                 float fx, float fy, float cx, float cy, float z_near, float z_far, float *rays,
                 pnr_stream_t stream) {
    if (n_images < 0 || width < 0 || height < 0) return fail(PNR_ERR_INVALID, "pnr_gen_rays: bad sizes");
    if (pose_rows != 3 && pose_rows != 4) return fail(PNR_ERR_INVALID, "pnr_gen_rays: pose_rows must be 3 or 4");
    if (n_images == 0 || width == 0 || height == 0) return PNR_OK;
    if (!poses || !rays) return fail(PNR_ERR_INVALID, "pnr_gen_rays: NULL");
    if ((reinterpret_cast<uintptr_t>(rays) & 15) != 0) return fail(PNR_ERR_INVALID, "rays must be 16-byte aligned");
    return launch_gen_rays(poses, n_images, pose_rows, width, height, fx, fy, cx, cy, z_near, z_far, rays,
                           (hipStream_t)stream);
}

}  // extern "C"
