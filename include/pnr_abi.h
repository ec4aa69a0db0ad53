/*
 * pnr_abi.h — C ABI of the MI355X (gfx950) pixelNeRF ray-march library (libpnr.so).
 *
 * The library replaces the per-ray hot path of the reference (etiiiR/pixel-nerf):
 *   src/render/nerf.py      NeRFRenderer.forward / sample_* / composite  (nerf.py:98-303)
 *   src/model/models.py     PixelNeRFNet.forward                         (models.py:146-266)
 *   src/model/resnetfc.py   ResnetFC / ResnetBlockFC                     (resnetfc.py:10-184)
 *   src/model/code.py       PositionalEncoding                           (code.py:30-42)
 *   src/model/encoder.py    SpatialEncoder.index (grid_sample)           (encoder.py:80-109)
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer owned by the caller, except the struct
 *     arguments themselves (host memory, read during the call only).
 *   - All tensors are fp32, C-contiguous, row-major, in the shapes given below.
 *   - Calls are asynchronous and stream-ordered on `stream` (a hipStream_t; NULL
 *     = the default stream).  The library never allocates device memory: scratch
 *     comes from a caller-provided workspace sized by the *_workspace_bytes query.
 *   - Functions return PNR_OK (0) or a negative pnr_status; pnr_last_error()
 *     returns a thread-local message for the last failing call on that thread.
 *     No C++ exception crosses this boundary.
 *   - Re-entrant: no mutable global state; callers may use one thread per GPU.
 */
#ifndef PNR_ABI_H
#define PNR_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNR_ABI_VERSION 8   /* 4: pnr_weight_grad_arith (per-call weight-gradient arithmetic);
                               5: pnr_latent_channels_last_nhwc;
                               6: pnr_fold_batchnorm;
                               7: pnr_latent_channels_last_backward,
                                  pnr_points_input_backward_masked;
                               8: pnr_render_cfg.ray_order */

typedef enum pnr_status {
    PNR_OK = 0,
    PNR_ERR_INVALID = -1,     /* bad argument / shape / null pointer               */
    PNR_ERR_UNSUPPORTED = -2, /* configuration the kernels do not implement        */
    PNR_ERR_HIP = -3,         /* HIP runtime error (launch or device query)        */
    PNR_ERR_WORKSPACE = -4    /* workspace missing or too small                    */
} pnr_status;

typedef void *pnr_stream_t; /* hipStream_t */

/* Encoded source views: what PixelNeRFNet.encode() leaves in the model
 * (models.py:111-141) plus the encoder feature map (encoder.py:160-163). */
typedef struct pnr_scene {
    const float *latent; /* (n_obj*n_views, latent_h, latent_w, latent_c), channels-LAST  */
    const float *cams;   /* (n_obj*n_views, 16): R_wc[3][3] row-major, t_wc[3],
                            fx, fy (already negated as models.py:130 does), cx, cy         */
    int32_t n_obj;       /* SB: objects in the super-batch                                 */
    int32_t n_views;     /* NS: source views per object                                    */
    int32_t latent_h, latent_w, latent_c;
    float image_w, image_h; /* PixelNeRFNet.image_shape = [W, H] (models.py:116-117)       */
} pnr_scene;

/* Shape of a ResnetFC (resnetfc.py:65-130) + positional encoding (code.py). */
typedef struct pnr_mlp_desc {
    int32_t d_in;          /* 42 for the shipped conf (xyz PE 39 + viewdir 3)             */
    int32_t d_latent;      /* 512                                                          */
    int32_t d_hidden;      /* 512                                                          */
    int32_t d_out;         /* 4                                                            */
    int32_t n_blocks;      /* 5                                                            */
    int32_t combine_layer; /* 3 (>= n_blocks means never combine; requires n_views == 1)  */
    int32_t pe_n;          /* entries of code._freqs / code._phases (2*num_freqs = 12)    */
    int32_t precision;     /* PNR_PREC_*: arithmetic of the 512-wide layers (see below)  */
} pnr_mlp_desc;

/* Arithmetic of the ResnetFC GEMMs (fp32 in, fp32 out, fp32 accumulation in all modes):
 *   PNR_PREC_F32    v_mfma_f32_16x16x4_f32 — fp32 products, fp32 accumulation.
 *   PNR_PREC_BF16X9 both operands split EXACTLY into three bf16 parts (x = x0+x1+x2),
 *                   all 9 part-products on v_mfma_f32_16x16x32_bf16: every product exact,
 *                   only the fp32 accumulation rounds (numerically an fp32 GEMM).
 *   PNR_PREC_BF16X6 the 6 largest of those products (drops x1*y2, x2*y1, x2*y2, each
 *                   < 2^-24 |x y|): error at the fp32 unit roundoff.
 *   PNR_PREC_F16X3  W (per layer) and every activation column scaled by a power of two
 *                   (max <= 2^14), each split into two fp16 parts x = x0 + x1 (|x - x0 - x1|
 *                   <= 2^-22 |x|); 3 exact products x0 y0 + x0 y1 + x1 y0 on
 *                   v_mfma_f32_16x16x32_f16, fp32 accumulation, scales undone exactly.
 *                   Error at the fp32 level (tools/precision_study.py). */
#define PNR_PREC_F32 0
#define PNR_PREC_F16X3 3
#define PNR_PREC_BF16X6 6
#define PNR_PREC_BF16X9 9

/* Unpacked weights in torch nn.Linear layout: weight (out, in), bias (out). */
typedef struct pnr_mlp_weights {
    pnr_mlp_desc desc;
    const float *lin_in_w, *lin_in_b;
    const float *lin_z_w[8], *lin_z_b[8];  /* min(combine_layer, n_blocks) entries  */
    const float *fc0_w[8], *fc0_b[8];      /* blocks[i].fc_0, n_blocks entries       */
    const float *fc1_w[8], *fc1_b[8];      /* blocks[i].fc_1                         */
    const float *lin_out_w, *lin_out_b;
    const float *pe_freqs, *pe_phases;     /* code._freqs, code._phases (pe_n each)  */
} pnr_mlp_weights;

/* Rays, (n_rays, 8) = [ox, oy, oz, dx, dy, dz, near, far] (nerf.py:101).  Rays are
 * object-major: ray b belongs to object b / rays_per_obj (nerf.py:191-196). */
typedef struct pnr_rays {
    const float *rays;
    int64_t n_rays;
    int64_t rays_per_obj;
} pnr_rays;

/* Random draws of the march (nerf.py:111, 135, 141, 158), in one of two modes:
 *   injected  the four streams below, drawn by the caller in the reference's order (tests
 *             and fixtures: the reference's own torch.rand draws replayed exactly);
 *   counter   every stream pointer NULL: the kernels draw on device from {seed, offset}
 *             with Philox4x32-10.  Draw k of ray b of stream s uses the counter
 *             (lo32 e, hi32 e, s, 0), e = (offset + b) * width_s + k, key (lo32 seed,
 *             hi32 seed); U[0,1) = (word0 >> 8) * 2^-24; N(0,1) = Box-Muller on
 *             u1 = ((word0 >> 8) + 1) * 2^-24, u2 = (word1 >> 8) * 2^-24.  A ray's draws
 *             depend on its global index (offset + b) only, so chunking a batch with
 *             offset = the chunk's first ray gives the same samples as one call.
 *             No HBM streams are written or read.  pnr_rng_fill materialises a stream. */
#define PNR_RNG_U_COARSE 0   /* width n_coarse                      */
#define PNR_RNG_U_FINE 1     /* width n_fine - n_fine_depth         */
#define PNR_RNG_U_FINE_JIT 2 /* width n_fine - n_fine_depth         */
#define PNR_RNG_N_DEPTH 3    /* width n_fine_depth, normal          */
typedef struct pnr_rng {
    const float *u_coarse;   /* (n_rays, n_coarse)          U[0,1)  */
    const float *u_fine;     /* (n_rays, n_fine - n_fine_depth)     */
    const float *u_fine_jit; /* (n_rays, n_fine - n_fine_depth)     */
    const float *n_depth;    /* (n_rays, n_fine_depth)      N(0,1)  */
    uint64_t seed;           /* counter mode (all four pointers NULL) */
    uint64_t offset;         /* global index of ray 0 of this call    */
} pnr_rng;

typedef struct pnr_render_cfg {
    int32_t n_coarse;     /* Kc                          (nerf.py:75)       */
    int32_t n_fine;       /* Kf incl. depth samples       (nerf.py:76)       */
    int32_t n_fine_depth; /* Kfd                          (nerf.py:77)       */
    float depth_std;      /*                              (nerf.py:80)       */
    int32_t white_bkgd;   /*                              (nerf.py:83)       */
    int32_t lindisp;      /*                              (nerf.py:84)       */
    /* ABI 3: ray-march schedule of THIS call (no process state is read or written):
     *   3  coarse and fine pass in ONE launch (n_coarse = 64, n_coarse + n_fine = 128,
     *      projected latents; other shapes run mode 2),
     *   2  fused passes + fine-draw kernel, 1  fine draws in the coarse epilogue too,
     *   0  separate sample / MLP / composite kernels (see pnr_render_set_fused);
     *  -1  the process default set by pnr_render_set_fused (initially 2).
     * All modes give bit-identical results. */
    int32_t march_mode;
    /* ABI 8: the order in which the fused march (modes 1-3) takes the rays, or NULL (input
     * order).  ray_order[i] is the index of the i-th ray to process; it should be a permutation
     * of 0 .. n_rays - 1 (an entry out of range processes ray i instead).  Every draw and every
     * output stays at the ray's own index, so the results are bit-identical to NULL's; only the
     * schedule -- which rays share an XCD's L2 at a time -- changes (NeRFRenderer.ray_order:
     * pixel blocks of 16 x 16 rays). */
    const int32_t *ray_order;
} pnr_render_cfg;

/* Outputs; any pointer may be NULL except the rgb/depth of each pass that runs. */
typedef struct pnr_render_out {
    float *coarse_rgb;     /* (n_rays, 3)                              */
    float *coarse_depth;   /* (n_rays)                                 */
    float *coarse_weights; /* (n_rays, n_coarse)                       */
    float *fine_rgb;       /* (n_rays, 3)           if n_fine > 0      */
    float *fine_depth;     /* (n_rays)                                 */
    float *fine_weights;   /* (n_rays, n_coarse + n_fine)              */
    float *z_coarse;       /* (n_rays, n_coarse)    sample depths      */
    float *z_fine;         /* (n_rays, n_coarse + n_fine), sorted      */
} pnr_render_out;

/* ---- library ---------------------------------------------------------------- */
int pnr_abi_version(void);
const char *pnr_last_error(void);

/* ---- MLP weight packing (ResnetFC -> MFMA fragment order) ------------------- */
/* Replaces: the nn.Linear parameters of ResnetFC (resnetfc.py:88-112) as the hot
 * path consumes them.  Pack once per weight version; the packed buffer is what
 * pnr_point_query / pnr_render_forward read. */
size_t pnr_mlp_packed_bytes(const pnr_mlp_desc *desc);
int pnr_mlp_pack(const pnr_mlp_weights *w, void *packed, size_t packed_bytes,
                 pnr_stream_t stream);

/* ---- per-point model query ---------------------------------------------------- */
/* Replaces: PixelNeRFNet.forward(xyz, coarse, viewdirs) (models.py:146-266):
 * world->camera transform, PE, projection + bilinear latent gather, ResnetFC with
 * the multi-view mean, sigmoid/relu head.  xyz/viewdirs (n_obj*points_per_obj, 3);
 * viewdirs may be NULL (zeros).  out (n_obj*points_per_obj, 4). */
size_t pnr_point_query_workspace_bytes(const pnr_scene *scene, int64_t n_points);
int pnr_point_query(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                    const float *xyz, const float *viewdirs, int64_t points_per_obj,
                    float *out, void *workspace, size_t workspace_bytes,
                    pnr_stream_t stream);

/* ---- full coarse + fine render ------------------------------------------------ */
/* Replaces: NeRFRenderer.forward(model, rays, want_weights) (nerf.py:251-303)
 * with model = PixelNeRFNet (mlp_coarse / mlp_fine; pass the coarse pack twice when
 * mlp_fine is None, models.py:242). */
size_t pnr_render_workspace_bytes(const pnr_scene *scene, const pnr_render_cfg *cfg,
                                  int64_t n_rays);
int pnr_render_forward(const pnr_scene *scene, const pnr_mlp_desc *desc,
                       const void *coarse_packed, const void *fine_packed,
                       const pnr_rays *rays, const pnr_rng *rng,
                       const pnr_render_cfg *cfg, const pnr_render_out *out,
                       void *workspace, size_t workspace_bytes, pnr_stream_t stream);

/* Same as pnr_render_forward, plus hipEventRecord of caller-created events on
 * `stream` around every launch: events[0] before sample_coarse, [1] after it
 * (= before the coarse point MLP), [2] after the coarse MLP, [3] after the coarse
 * composite, [4] after sample_fine, [5] after the fine MLP, [6] after the fine
 * composite (entries 4-6 unused when n_fine == 0).  `events` holds 7 hipEvent_t;
 * no host synchronization is added.  Used by bench.py for per-kernel timing.
 * With the fused ray march (pnr_render_set_fused) a pass is one launch: [1]-[2] and
 * [4]-[5] then time the whole coarse / fine pass (sampling and composite included),
 * and the other intervals are empty; with march_mode 3 the single launch is [1]-[2]. */
int pnr_render_forward_events(const pnr_scene *scene, const pnr_mlp_desc *desc,
                              const void *coarse_packed, const void *fine_packed,
                              const pnr_rays *rays, const pnr_rng *rng,
                              const pnr_render_cfg *cfg, const pnr_render_out *out,
                              void *workspace, size_t workspace_bytes, pnr_stream_t stream,
                              void *const *events);

/* ---- projected latent (lin_z folded into the latent, inference) --------------- */
/* Floats-as-bytes of one model's projected latent for `scene`: n_linz x (n_obj * n_views)
 * x latent_h x latent_w x 512 fp32, n_linz = min(combine_layer, n_blocks); 0 if invalid. */
size_t pnr_latent_project_bytes(const pnr_scene *scene, const pnr_mlp_desc *desc);

/* Replaces: the per-point lin_z GEMMs of ResnetFC (resnetfc.py:160-163) on the bilinearly
 * sampled latent (encoder.py:102-108).  grid_sample's output is a blend of four latent
 * pixels and lin_z is linear, so lin_z[b](z) = blend of the rows of
 *   proj[b][image][y][x][:] = lin_z[b].weight . latent[image][y][x][:]      (no bias)
 * computed here once per (scene, weight version) with fp32 products and accumulation.
 * The *_proj entry points below blend four rows per point instead of the lin_z GEMM
 * (same results up to fp32 reassociation).  Forward (inference) only. */
int pnr_latent_project(const pnr_scene *scene, const pnr_mlp_weights *w, float *proj, size_t proj_bytes,
                       pnr_stream_t stream);

/* pnr_point_query / pnr_render_forward_events with the projected latent of the model(s):
 * `proj` (point query), `coarse_proj` / `fine_proj` (render; pass the coarse projection
 * twice when mlp_fine is None) from pnr_latent_project on the same scene and weights.
 * NULL projections select the latent gather + lin_z GEMM path.  `events` may be NULL.
 * When fine_packed == coarse_packed and fine_proj == coarse_proj (mlp_fine is None), the fine
 * pass evaluates only the n_fine new samples and reuses the coarse pass's outputs for the
 * n_coarse coarse samples (bit-identical: a point's output does not depend on the others). */
int pnr_point_query_proj(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                         const float *proj, const float *xyz, const float *viewdirs,
                         int64_t points_per_obj, float *out, void *workspace,
                         size_t workspace_bytes, pnr_stream_t stream);
int pnr_render_forward_proj(const pnr_scene *scene, const pnr_mlp_desc *desc,
                            const void *coarse_packed, const void *fine_packed,
                            const float *coarse_proj, const float *fine_proj,
                            const pnr_rays *rays, const pnr_rng *rng,
                            const pnr_render_cfg *cfg, const pnr_render_out *out,
                            void *workspace, size_t workspace_bytes, pnr_stream_t stream,
                            void *const *events);

/* Fused ray march.  3: the whole march is ONE k_point_mlp launch -- a workgroup takes a ray's
 * coarse tile, composites it and draws its fine samples in the epilogue into LDS, then runs the
 * ray's two fine tiles with the fine MLP and composites them (nerf.py:273-301 per ray; the fine
 * depths never reach HBM unless pnr_render_out.z_fine asks for them).  It applies to
 * n_coarse = 64, n_coarse + n_fine = 128 with both projected latents (the headline shape) and
 * falls back to mode 2 otherwise.  2 (the default): each pass of pnr_render_forward* is one
 * k_point_mlp launch
 * that draws the coarse depths in its prologue and composites each ray from LDS in its
 * epilogue (the per-point rgb/sigma never reach HBM); the fine draws (inverse CDF + sort) run
 * in their own small kernel between the passes.  1: the coarse epilogue draws the fine samples
 * too (one launch per pass; measured 0.3-0.5 % slower on MI355X, since one wave runs them while
 * the workgroup's other seven wait).  0: the separate sample / MLP / composite kernels.  The
 * fusion applies when a pass's samples per ray are 64 or 128 (and kc + kf <= 128 for the fine
 * draws) and mlp_fine is not None; other shapes take the separate kernels.  All modes run the
 * same device code and give bit-identical results.  This only sets the DEFAULT that calls with
 * pnr_render_cfg.march_mode = -1 use (ABI 3); a call that names its mode reads no process state,
 * so host threads (DataParallel replicas, nerf.py:370) may render with different modes at once.
 * Returns the previous default. */
int32_t pnr_render_set_fused(int32_t on);

/* ---- building blocks (also the generic model-callback path) ------------------ */
/* Replaces: NeRFRenderer.sample_coarse (nerf.py:98-118).  z (n_rays, n_coarse). */
int pnr_sample_coarse(const float *rays, int64_t n_rays, int32_t n_coarse,
                      const float *u_coarse, int32_t lindisp, float *z,
                      pnr_stream_t stream);

/* Replaces: sample_fine + sample_fine_depth + cat + sort (nerf.py:120-161, 284-295).
 * weights/depth of the coarse pass; z_fine (n_rays, n_coarse + n_fine) sorted. */
int pnr_sample_fine(const float *rays, int64_t n_rays, int32_t n_coarse,
                    const float *z_coarse, const float *coarse_weights,
                    const float *coarse_depth, int32_t n_fine, int32_t n_fine_depth,
                    float depth_std, const float *u_fine, const float *u_fine_jit,
                    const float *n_depth, int32_t lindisp, float *z_fine,
                    pnr_stream_t stream);

/* Replaces: NeRFRenderer.composite's alpha compositing (nerf.py:176-249).
 * z (n_rays, K), raw (n_rays, K, 4) = model output [r, g, b, sigma];
 * weights (n_rays, K) may be NULL; rgb (n_rays, 3); depth (n_rays).
 * raw must be 16-byte aligned (PNR_ERR_INVALID otherwise); z and weights need only float
 * alignment. */
int pnr_composite(const float *z, const float *raw, const float *rays, int64_t n_rays,
                  int32_t k, int32_t white_bkgd, float *weights, float *rgb, float *depth,
                  pnr_stream_t stream);

/* ---- counter-mode draws --------------------------------------------------------- */
/* Replaces: the torch.rand / torch.randn draws of the march (nerf.py:111, 135, 141, 158) in
 * counter mode: writes out (n_rays, width) = the draws of `stream` (PNR_RNG_*) for rays
 * offset .. offset + n_rays - 1 exactly as the render kernels draw them (uniform for
 * streams 0-2, normal for 3). */
int pnr_rng_fill(uint64_t seed, uint64_t offset, int32_t stream, int64_t n_rays, int32_t width, float *out,
                 pnr_stream_t stream_h);

/* ---- ray generation ------------------------------------------------------------ */
/* Replaces: util.gen_rays (util.py:238-276) with unproj_map (util.py:113-143), ndc=False.
 * poses (n_images, pose_rows, 4) row-major camera-to-world (pose_rows 3 or 4); focal
 * (fx, fy) and principal point (cx, cy) in pixels, as the reference's float(f[0]) etc.;
 * rays (n_images, height, width, 8) = [o, d (unit), near, far]. */
int pnr_gen_rays(const float *poses, int64_t n_images, int32_t pose_rows, int32_t width,
                 int32_t height, float fx, float fy, float cx, float cy, float z_near,
                 float z_far, float *rays, pnr_stream_t stream);

/* ---- encoder latent, channels-last --------------------------- */
/* Replaces: the upsample + concat tail of SpatialEncoder.forward (encoder.py:150-160):
 * n_maps (<= 8) trunk feature maps, maps[k] (n_images, channels[k], heights[k], widths[k])
 * NCHW fp32 device pointers (the pointer arrays themselves are host memory), bilinearly
 * upsampled with align_corners = True to (out_h, out_w) and concatenated along channels,
 * written channels-LAST: latent_cl (n_images, out_h, out_w, sum channels). */
int pnr_latent_channels_last(const float *const *maps, const int32_t *channels,
                             const int32_t *heights, const int32_t *widths, int32_t n_maps,
                             int32_t n_images, float *latent_cl, int32_t out_h, int32_t out_w,
                             pnr_stream_t stream);

/* pnr_latent_channels_last with every maps[k] channels-last, (n_images, heights[k], widths[k],
 * channels[k]) (the trunk's maps when its convolutions run in channels-last memory format):
 * the same arithmetic and output (ABI 5). */
int pnr_latent_channels_last_nhwc(const float *const *maps, const int32_t *channels,
                                  const int32_t *heights, const int32_t *widths, int32_t n_maps,
                                  int32_t n_images, float *latent_cl, int32_t out_h, int32_t out_w,
                                  pnr_stream_t stream);

/* Backward of pnr_latent_channels_last_nhwc: d_maps[k] (n_images, heights[k], widths[k], channels[k],
 * channels-last) = the adjoint of map k's bilinear upsample (align_corners = True) applied to its
 * channel slice of g (n_images, out_h, out_w, sum channels) -- what autograd of encoder.py:150-160's
 * F.interpolate + torch.cat computes (upsample_bilinear2d_backward).  Gathered per source element in
 * a fixed order (deterministic; torch scatters with atomics); one launch for all maps (ABI 7). */
int pnr_latent_channels_last_backward(const float *g, float *const *d_maps, const int32_t *channels,
                                      const int32_t *heights, const int32_t *widths, int32_t n_maps,
                                      int32_t n_images, int32_t out_h, int32_t out_w, pnr_stream_t stream);

/* One (convolution, BatchNorm) pair of the eval-mode encoder trunk (encoder.py:135-149 with the
 * BatchNorms on their running statistics).  conv_w / w_out: n_out blocks of per_out contiguous
 * floats (OIHW or channels-last OHWI weights: the output channel is outermost in both); gamma /
 * beta NULL for a BatchNorm without affine parameters. */
typedef struct pnr_bn_fold {
    const float *conv_w;
    const float *gamma, *beta, *mean, *var;
    float *w_out, *b_out;
    int64_t n_out, per_out;
    float eps;
    int32_t pad_;
} pnr_bn_fold;

/* Fold every pair: w_out[o, :] = conv_w[o, :] s[o], b_out[o] = beta[o] - mean[o] s[o] with
 * s = gamma[o] / sqrt(var[o] + eps) (correctly rounded sqrt and divide).  `folds` is a DEVICE
 * array of n_folds records (the kernel reads it; a HIP graph that captured this call keeps
 * reading the same array); max_elems = max n_out * per_out.  Replaces the per-encode BatchNorm
 * arithmetic of SpatialEncoder.forward in eval mode (encoder.py:135-149); ABI 6. */
int pnr_fold_batchnorm(const pnr_bn_fold *folds, int32_t n_folds, int64_t max_elems, pnr_stream_t stream);

/* ---- training (autograd over the ray march) ------------ */
/* Floats of the activation save of pnr_render_points for n_points rows; call it with
 * n_points = n_rays * k * n_views.  Regions, each [row][width] with R = n_rays * k *
 * n_views rows: features (64) | z (512) | relu(x) into fc_0 of each block (512 each) |
 * relu(h) of each block (512 each) | relu(x) into lin_out (512), then the relu sign masks
 * of the 2 n_blocks + 1 relu regions (same order), each [row][64 bytes], [activation n > 0]
 * of n = 64 w + 16 r + 4 g + e (w, r, g, e = 0..7, 0..3, 0..3, 0..3) at bit 4 (r & 1) + e
 * of byte 8 w + 2 g + (r >> 1).  Row v * (n_rays * k) + p holds (source view v, point p)
 * for the per-view stages (features, z, the blocks before combine_layer); the blocks from
 * combine_layer on and lin_out use rows p < n_rays * k (the view mean). */
size_t pnr_point_save_floats(const pnr_mlp_desc *desc, int64_t n_points);

/* Replaces: the model call of NeRFRenderer.composite (nerf.py:182-216) under autograd:
 * PixelNeRFNet.forward at the points o + z d of every ray (z (n_rays, k)), writing
 * out (n_rays * k, 4) and, when `save` is not NULL, the activations the backward needs
 * (pnr_point_save_floats(desc, n_rays * k * n_views) floats).  Workspace as pnr_point_query. */
int pnr_render_points(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                      const pnr_rays *rays, const float *z, int32_t k, float *out, float *save,
                      void *workspace, size_t workspace_bytes, pnr_stream_t stream);

/* Replaces: autograd of NeRFRenderer.composite (nerf.py:225-247).  Given d_rgb (n_rays, 3),
 * d_depth (n_rays, may be NULL) and d_weights (n_rays, k, may be NULL): d_raw (n_rays, k, 4)
 * = d [rgb, sigma] and d_z (n_rays, k, may be NULL).  k <= 256. */
int pnr_composite_backward(const float *z, const float *raw, const float *rays, int64_t n_rays,
                           int32_t k, int32_t white_bkgd, const float *d_rgb, const float *d_depth,
                           const float *d_weights, float *d_raw, float *d_z, pnr_stream_t stream);

/* Replaces: autograd of the input stage of PixelNeRFNet.forward (models.py:156-221,
 * code.py:30-42, encoder.py:80-109).  d_feat (n_views * n_rays * k, 64): gradient of the
 * lin_in input; d_zlat (n_views * n_rays * k, 512): gradient of the sampled latent feature,
 * rows as the activation save (view-major).  Accumulates d_latent (channels-last, like
 * scene->latent; may be NULL) and writes d_z (n_rays * k, may be NULL) = dL / d z_sample,
 * summed over the views in view order.  `packed` supplies the PE buffers. */
int pnr_points_input_backward(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                              const pnr_rays *rays, const float *z, int32_t k, const float *d_feat,
                              const float *d_zlat, float *d_latent, float *d_z, pnr_stream_t stream);

/* pnr_points_input_backward with z_mask (n_rays * k bytes, may be NULL = every point): d_z is
 * computed only where z_mask is nonzero and written 0 elsewhere.  The fine pass's depths are the
 * sort of [importance samples (no gradient), depth samples (gradient to the coarse depth)]
 * (nerf.py:150-161, 292), so only the depth samples' dL/dz reaches the graph; the mask skips the
 * latent-corner reads of the others (ABI 7). */
int pnr_points_input_backward_masked(const pnr_scene *scene, const pnr_mlp_desc *desc, const void *packed,
                                     const pnr_rays *rays, const float *z, int32_t k, const float *d_feat,
                                     const float *d_zlat, float *d_latent, float *d_z, const uint8_t *z_mask,
                                     pnr_stream_t stream);

/* Bytes of the transposed (backward) weight pack of an f16x3 model (precision
 * PNR_PREC_F16X3); 0 for an invalid desc or another precision. */
size_t pnr_mlp_packed_t_bytes(const pnr_mlp_desc *desc);

/* Pack W^T of every 512-wide ResnetFC layer for pnr_mlp_backward.  `packed` is the model's
 * pnr_mlp_pack output (same weights, same stream order): its header holds the scales. */
int pnr_mlp_pack_t(const pnr_mlp_weights *w, const void *packed, void *packed_t, size_t packed_t_bytes,
                   pnr_stream_t stream);

/* Replaces: autograd of ResnetFC.forward (resnetfc.py:132-184, n_views == 1) up to the
 * weight GEMMs, for an f16x3 model.  Given the forward's activation save (pnr_render_points)
 * and d_o (n_points, 4) = dL / d lin_out output, writes the gradient of every layer's output:
 *   dy ((2 n_blocks + 1), n_points, 512): [b] fc_0 of block b, [n_blocks] lin_in,
 *       [n_blocks + 1 + b] fc_1 of block b; the lin_z of block b takes dy[n_blocks + b];
 *   d_zlat (n_points, 512): dL / d (sampled latent), summed over the lin_z layers
 *       (required when the model has lin_z layers).
 * Weight and bias gradients are then dy^T . (saved layer input) and column sums of dy. */
int pnr_mlp_backward(const pnr_mlp_desc *desc, const void *packed, const void *packed_t,
                     const float *lin_out_w, const float *save, const float *d_o, int64_t n_points,
                     float *dy, float *d_zlat, pnr_stream_t stream);

/* Workspace bytes of pnr_mlp_backward_bias for n_points points (0 if n_points <= 0). */
size_t pnr_mlp_backward_workspace_bytes(const pnr_mlp_desc *desc, int64_t n_points);

/* pnr_mlp_backward plus the ResnetFC bias gradients (resnetfc.py:132-184: the column sums of
 * the dy slots over the points) in the same pass: d_bias ((2 n_blocks + 1), 512) in dy's slot
 * order, summed per workgroup over its tiles and then over the workgroups, both in a fixed
 * order (deterministic).  d_bias NULL = pnr_mlp_backward; otherwise `workspace` holds
 * pnr_mlp_backward_workspace_bytes. */
int pnr_mlp_backward_bias(const pnr_mlp_desc *desc, const void *packed, const void *packed_t,
                          const float *lin_out_w, const float *save, const float *d_o, int64_t n_points,
                          float *dy, float *d_zlat, float *d_bias, void *workspace, size_t workspace_bytes,
                          pnr_stream_t stream);

/* pnr_mlp_backward_bias for n_views >= 1 source views per point (resnetfc.py:151-172 with
 * util.combine_interleaved's mean): `save` from pnr_render_points with n_views views (its
 * regions have n_views * n_points rows, row v * n_points + p for the blocks before
 * combine_layer); dy is (2 n_blocks + 1) x (n_views * n_points) x 512, the slots of the blocks
 * from combine_layer on (and lin_out's input) using their first n_points rows, the others the
 * view rows; d_zlat is (n_views * n_points, 512); d_bias sums every slot over all its rows.
 * The blocks after the mean run once per point; dL/d(mean) / n_views then enters the chain of
 * the blocks before it once per view.  n_views == 1 is pnr_mlp_backward_bias. */
int pnr_mlp_backward_views(const pnr_mlp_desc *desc, const void *packed, const void *packed_t,
                           const float *lin_out_w, const float *save, const float *d_o, int64_t n_points,
                           int32_t n_views, float *dy, float *d_zlat, float *d_bias, void *workspace,
                           size_t workspace_bytes, pnr_stream_t stream);

/* Workspace bytes of pnr_weight_grad (n_layers in 1..16); 0 if the sizes are invalid. */
size_t pnr_weight_grad_workspace_bytes(int32_t n_layers, int64_t n_points);

/* Arithmetic of pnr_weight_grad_arith (ABI 4).  fp32 in, fp32 out, fp32 accumulation in both.
 *   PNR_WGRAD_F16X3  (the default of pnr_weight_grad) every operand scaled by a power of two per
 *       (point chunk, channel) that follows the data, split into two fp16 parts, 3 products on
 *       v_mfma_f32_16x16x32_f16.  Error bound PER VALUE, relative to M = the running maximum of
 *       its channel in its chunk (not to the value itself): 22 significand bits down to 2^-8 M,
 *       an absolute error below ~2^-30 M beneath that (subnormal fp16 parts), zero below
 *       ~2^-31 M.  So an output element G_ij is fp32-accurate relative to
 *       sum_p |dy_pi| M_j + M_i |x_pj| (the scale of its channel pair), and an element built
 *       ONLY from values far below their channels' maxima (x_j nonzero only where dy_i is
 *       2^-20 M_i) can carry a large RELATIVE error.  Measured on training-step data at the
 *       fp32 GEMM error scale (DESIGN.md §3 training path).
 *   PNR_WGRAD_BF16X6 three exact bf16 parts per operand (fp32's exponent range, no scales), the
 *       6 largest products on v_mfma_f32_16x16x32_bf16 (dropped terms < 2^-24 |x y|): fp32-level
 *       error PER ELEMENT relative to sum_p |dy_pi x_pj|, whatever the dynamic range.
 *       ~1.4x the kernel time of F16X3. */
#define PNR_WGRAD_F16X3 0
#define PNR_WGRAD_BF16X6 1

/* Replaces: the weight-gradient GEMMs autograd runs for the 512 x 512 nn.Linear layers of
 * ResnetFC (resnetfc.py:132-184): for each layer j,
 *   d_weight[j] (512 x 512, [out][in]) = dy[j]^T x[j],
 * dy[j] (n_points x 512) the layer's output gradient (pnr_mlp_backward's slots), x[j]
 * (n_points x 512) its input (the activation save).  dy, x, d_weight are host arrays of
 * n_layers device pointers (16-byte aligned).  PNR_WGRAD_F16X3 arithmetic (bound above);
 * deterministic (fixed reduction order). */
int pnr_weight_grad(const float *const *dy, const float *const *x, float *const *d_weight, int32_t n_layers,
                    int64_t n_points, void *workspace, size_t workspace_bytes, pnr_stream_t stream);

/* pnr_weight_grad with the arithmetic named per call (PNR_WGRAD_*; another value is
 * PNR_ERR_INVALID); the same workspace. */
int pnr_weight_grad_arith(const float *const *dy, const float *const *x, float *const *d_weight,
                          int32_t n_layers, int64_t n_points, int32_t arith, void *workspace,
                          size_t workspace_bytes, pnr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PNR_ABI_H */
