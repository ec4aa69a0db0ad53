// Backward kernels of the ray march (training).
//
// The reference trains through torch autograd over NeRFRenderer.forward (nerf.py:163-303)
// and PixelNeRFNet.forward (models.py:146-266).  These kernels are the backward of the
// fused forward kernels, so the HIP path reproduces that autograd graph:
//   k_composite_bwd   composite (nerf.py:225-247): d(rgb, depth, weights) -> d raw, d z
//   k_points_in_bwd   the per-point input stage of PixelNeRFNet.forward: d(features),
//                     d(latent feature z) -> d latent (bilinear scatter, grid_sample
//                     backward, encoder.py:102-108) and d z_sample (through the PE,
//                     code.py:38, and the projection, models.py:206-212)
// The ResnetFC backward runs as plain per-layer GEMMs on the saved activations
// (pnr/train.py).
#include "pnr_common.h"

namespace pnr {

// ---------------------------------------------------------------------------
// composite backward (K <= 64 S; lane l owns samples S l .. S l + S - 1, like the forward)
//   w_i = a_i T_i,  T_i = prod_{j<i} s_j,  s_j = 1 - a_j + 1e-10,  a = 1 - exp(-delta relu(sigma))
//   g_i = dL/dw_i = d_rgb . c_i + d_depth z_i (- sum d_rgb if white_bkgd) + d_weights_i
//   da_i = g_i T_i - (sum_{k>i} g_k w_k) / s_i
//   dsigma_i = da_i exp(-delta_i relu(sigma_i)) delta_i [sigma_i > 0]
//   ddelta_i = da_i exp(-delta_i relu(sigma_i)) relu(sigma_i)
//   dz_i = ddelta_{i-1} - ddelta_i + d_depth w_i     (delta_{K-1} = far - z_{K-1})
// ---------------------------------------------------------------------------
template <int S>
__global__ __launch_bounds__(256) void k_composite_bwd(
    const float *__restrict__ z, const float *__restrict__ raw, const float *__restrict__ rays,
    int64_t n_rays, int K, int white_bkgd, const float *__restrict__ d_rgb,
    const float *__restrict__ d_depth, const float *__restrict__ d_weights, float *__restrict__ d_raw,
    float *__restrict__ d_z) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= n_rays) return;
    const float far = rays[b * 8 + 7];
    const float *zr = z + b * K;
    const f4 *rr = reinterpret_cast<const f4 *>(raw) + b * K;
    const int k0 = S * lane;
    float zk[S];
    f4 v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const int kc = k0 + i < K ? k0 + i : K - 1;
        zk[i] = zr[kc];
        v[i] = rr[kc];
    }
    const float z_next_lane = dpp_f<0x130>(far, zk[0]);
    const float gr = d_rgb[b * 3 + 0], gg = d_rgb[b * 3 + 1], gb = d_rgb[b * 3 + 2];
    const float gd = d_depth ? d_depth[b] : 0.f;
    const float gwhite = white_bkgd ? -((gr + gg) + gb) : 0.f;
    float alpha[S], ex[S], delta[S], sg[S];
    double lp[S + 1];
    lp[0] = 1.0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const int k = k0 + i;
        const bool valid = k < K;
        const float zn = k + 1 >= K ? far : (i + 1 < S ? zk[i + 1] : z_next_lane);
        delta[i] = sub_rn(zn, zk[i]);
        sg[i] = max_nc(v[i].w, 0.0f);
        ex[i] = expf(mul_rn(-delta[i], sg[i]));
        alpha[i] = valid ? sub_rn(1.0f, ex[i]) : 0.0f;
        const float shifted = valid ? add_rn(sub_rn(1.0f, alpha[i]), 1e-10f) : 1.0f;
        lp[i + 1] = lp[i] * (double)shifted;
    }
    const double excl = wave_shr1(wave_scan_mul(lp[S]), 1.0);
    float T[S], w[S], g[S], gw_local = 0.f;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const bool valid = k0 + i < K;
        T[i] = (float)(excl * lp[i]);
        w[i] = valid ? mul_rn(alpha[i], T[i]) : 0.f;
        float gi = gr * v[i].x + gg * v[i].y + gb * v[i].z + gd * zk[i] + gwhite;
        if (d_weights && valid) gi += d_weights[b * K + k0 + i];
        g[i] = valid ? gi : 0.f;
        gw_local += g[i] * w[i];
    }
    // suffix sums of g w: total - inclusive prefix (over lanes, then inside the lane)
    float incl = gw_local;
    incl += dpp_f<0x111>(0.f, incl);
    incl += dpp_f<0x112>(0.f, incl);
    incl += dpp_f<0x114>(0.f, incl);
    incl += dpp_f<0x118>(0.f, incl);
    incl += dpp_f<0x142, 0xa>(0.f, incl);
    incl += dpp_f<0x143, 0xc>(0.f, incl);
    const float total = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
    float after = total - incl;   // sum over the lanes after this one
    float ddel[S];
#pragma unroll
    for (int i = S - 1; i >= 0; --i) {
        const int k = k0 + i;
        const bool valid = k < K;
        const float s_i = add_rn(sub_rn(1.0f, alpha[i]), 1e-10f);
        const float da = g[i] * T[i] - after / s_i;
        after += g[i] * w[i];
        const float dsig = v[i].w > 0.f ? da * ex[i] * delta[i] : 0.f;
        ddel[i] = valid ? da * ex[i] * sg[i] : 0.f;
        if (valid) {
            f4 o = {gr * w[i], gg * w[i], gb * w[i], dsig};
            reinterpret_cast<f4 *>(d_raw)[b * K + k] = o;
        }
    }
    if (d_z) {
        const float prev_lane = dpp_f<0x138>(0.f, ddel[S - 1]);   // wave_shr:1
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const int k = k0 + i;
            if (k < K) {
                const float dprev = i > 0 ? ddel[i - 1] : prev_lane;
                d_z[b * K + k] = (k > 0 ? dprev : 0.f) - ddel[i] + gd * w[i];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// per-point input backward (NS == 1).  One wave per run of RUN consecutive points
// (o + z d of ray b, in sample order):
//   d latent[corner][c] += w_corner d_zlat[c]        (channels-last; see below)
//   d z_sample = d . R^T (d x_rot)   with d x_rot from
//     features: d f[0:3] (x_rot) + sum_q d f[3 + 3q + j] cos(phase_q + x_rot_j freq_q) freq_q
//     projection: d x_cam through u = -x/z fx + cx, v = -y/z fy + cy and the bilinear
//       weights (out-of-range corners count as 0; clipped coordinates pass no gradient,
//       as torch's grid_sampler_2d_backward with border padding)
// Consecutive samples of a ray often fall in the same latent cell, so the wave keeps the
// four corner gradients of the current cell in registers (lane = 8 channels per corner,
// lane-contiguous so each atomic instruction touches 2 cache lines)
// and flushes them with atomics only when the cell changes: one atomic per channel and
// corner per run of equal cells instead of per point.  The dL/dz chains of the run's
// points are computed afterwards by lanes 0 .. RUN-1 in parallel.
// ---------------------------------------------------------------------------
constexpr int RUN = 8;   // 4 and 16 measured slower on the cfg5 step (profiles/r5r)

struct PointGeo {
    float xr[3], xc[3];
    float ix, iy, ixu, iyu;
    int64_t o00, o01, o10, o11;
    bool inx1, iny1;
};

__device__ __forceinline__ PointGeo point_geo(const float *__restrict__ rays, const float *__restrict__ zs, int K,
                                              int64_t rays_per_obj, const float *__restrict__ cams, int hl, int wl,
                                              float img_w, float img_h, int64_t p, int ns, int v) {
    PointGeo G;
    const int64_t b = p / K;
    const float *ray = rays + b * 8;
    const float zz = zs[p];
    const float px = add_rn(ray[0], mul_rn(zz, ray[3]));
    const float py = add_rn(ray[1], mul_rn(zz, ray[4]));
    const float pz = add_rn(ray[2], mul_rn(zz, ray[5]));
    const int64_t cv = (b / rays_per_obj) * ns + v;   // camera / latent of (object, view v)
    const float *cam = cams + cv * 16;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        G.xr[i] = add_rn(add_rn(mul_rn(cam[3 * i], px), mul_rn(cam[3 * i + 1], py)), mul_rn(cam[3 * i + 2], pz));
        G.xc[i] = add_rn(G.xr[i], cam[9 + i]);
    }
    const float fx = cam[12], fy = cam[13], cx = cam[14], cy = cam[15];
    // forward projection, as k_point_mlp
    const float u0 = __fdiv_rn(-G.xc[0], G.xc[2]), v0 = __fdiv_rn(-G.xc[1], G.xc[2]);
    const float u = add_rn(mul_rn(u0, fx), cx), w = add_rn(mul_rn(v0, fy), cy);
    const float wlf = (float)wl, hlf = (float)hl;
    const float lsx = mul_rn(__fdiv_rn(wlf, sub_rn(wlf, 1.f)), 2.f);
    const float lsy = mul_rn(__fdiv_rn(hlf, sub_rn(hlf, 1.f)), 2.f);
    const float gx = sub_rn(mul_rn(u, __fdiv_rn(lsx, img_w)), 1.f);
    const float gy = sub_rn(mul_rn(w, __fdiv_rn(lsy, img_h)), 1.f);
    G.ixu = mul_rn(add_rn(gx, 1.f), mul_rn(sub_rn(wlf, 1.f), 0.5f));
    G.iyu = mul_rn(add_rn(gy, 1.f), mul_rn(sub_rn(hlf, 1.f), 0.5f));
    G.ix = fminf(fmaxf(G.ixu, 0.f), wlf - 1.f);
    G.iy = fminf(fmaxf(G.iyu, 0.f), hlf - 1.f);
    const int x0 = (int)floorf(G.ix), y0 = (int)floorf(G.iy);
    G.inx1 = x0 + 1 < wl;
    G.iny1 = y0 + 1 < hl;
    const int64_t base = cv * (int64_t)hl * wl * 512;
    const int x1 = G.inx1 ? x0 + 1 : x0, y1 = G.iny1 ? y0 + 1 : y0;
    G.o00 = base + ((int64_t)y0 * wl + x0) * 512;
    G.o01 = base + ((int64_t)y0 * wl + x1) * 512;
    G.o10 = base + ((int64_t)y1 * wl + x0) * 512;
    G.o11 = base + ((int64_t)y1 * wl + x1) * 512;
    return G;
}

__global__ __launch_bounds__(256) void k_points_in_bwd(
    const float *__restrict__ rays, const float *__restrict__ zs, int K, int64_t rays_per_obj,
    int64_t n_points, int ns, const float *__restrict__ cams, const float *__restrict__ latent, int hl, int wl,
    float img_w, float img_h, const float *__restrict__ pe, int pe_n, const float *__restrict__ d_feat,
    const float *__restrict__ d_zlat, float *__restrict__ d_latent, float *__restrict__ d_z,
    const uint8_t *__restrict__ z_mask) {
    const int lane = threadIdx.x & 63;
    const int64_t p0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RUN;
    if (p0 >= n_points) return;
    const int n_run = n_points - p0 < RUN ? (int)(n_points - p0) : RUN;
    // d_feat / d_zlat rows v n_points + p: (view v, point p); d_z sums the views in order
    float dz_sum = 0.f;   // lane j: point p0 + j
    for (int v = 0; v < ns; ++v) {
        // current cell's corner gradients: [corner][half] x 4 channels (lane * 4 + 256 half)
        f4 acc[4][2];
        int64_t cur = -1;
        bool cur_x1 = false, cur_y1 = false;
        int64_t c01 = 0, c10 = 0, c11 = 0;
        auto flush = [&]() {
            if (cur < 0 || !d_latent) return;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    // lane-contiguous channels: one atomic instruction covers 256 B (2 lines)
                    const int ch = half * 256 + q * 64 + lane;
                    atomicAdd(d_latent + cur + ch, acc[0][half][q]);
                    if (cur_x1) atomicAdd(d_latent + c01 + ch, acc[1][half][q]);
                    if (cur_y1) atomicAdd(d_latent + c10 + ch, acc[2][half][q]);
                    if (cur_x1 && cur_y1) atomicAdd(d_latent + c11 + ch, acc[3][half][q]);
                }
            }
        };
        float dix_run = 0.f, diy_run = 0.f;   // lane j: point j's d ix / d iy (wave sums)
        for (int j = 0; j < n_run; ++j) {
            const int64_t p = p0 + j;
            // the depth chain only where a caller needs dL / dz (z_mask: the fine pass's depth samples)
            const bool need_z = d_z && (!z_mask || z_mask[p]);   // wave-uniform
            const PointGeo G = point_geo(rays, zs, K, rays_per_obj, cams, hl, wl, img_w, img_h, p, ns, v);
            const float we = sub_rn(G.ix, floorf(G.ix)), wn = sub_rn(G.iy, floorf(G.iy));
            const float wnw = mul_rn(sub_rn(1.f, wn), sub_rn(1.f, we)), wne = mul_rn(sub_rn(1.f, wn), we);
            const float wsw = mul_rn(wn, sub_rn(1.f, we)), wse = mul_rn(wn, we);
            if (G.o00 != cur) {   // wave-uniform
                flush();
                cur = G.o00;
                c01 = G.o01; c10 = G.o10; c11 = G.o11;
                cur_x1 = G.inx1; cur_y1 = G.iny1;
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[c][0] = acc[c][1] = f4{0.f, 0.f, 0.f, 0.f};
            }
            float dwe = 0.f, dwn = 0.f;
            const float *gz = d_zlat + (v * n_points + p) * 512;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                // channel half * 256 + q * 64 + lane (q = vector element): coalesced 256-B rows
                // per load, and the same lane-contiguous layout for the flush atomics
                const int ch = half * 256 + lane;
                f4 gv;
#pragma unroll
                for (int q = 0; q < 4; ++q) gv[q] = gz[ch + q * 64];
                if (need_z) {   // the latent corners only feed d ix / d iy (the depth chain)
                    f4 l00, l01, l10, l11;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        l00[q] = latent[G.o00 + ch + q * 64];
                        l01[q] = latent[G.o01 + ch + q * 64];
                        l10[q] = latent[G.o10 + ch + q * 64];
                        l11[q] = latent[G.o11 + ch + q * 64];
                    }
                    if (!G.inx1) { l01 = f4{0.f, 0.f, 0.f, 0.f}; l11 = l01; }
                    if (!G.iny1) { l10 = f4{0.f, 0.f, 0.f, 0.f}; l11 = l10; }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        dwe += gv[q] * ((1.f - wn) * (l01[q] - l00[q]) + wn * (l11[q] - l10[q]));
                        dwn += gv[q] * ((1.f - we) * (l10[q] - l00[q]) + we * (l11[q] - l01[q]));
                    }
                }
                acc[0][half] += wnw * gv;
                acc[1][half] += wne * gv;
                acc[2][half] += wsw * gv;
                acc[3][half] += wse * gv;
            }
            if (need_z) {
                dwe = wave_sum_dpp(dwe);
                dwn = wave_sum_dpp(dwn);
                if (lane == j) { dix_run = dwe; diy_run = dwn; }
            }
        }
        flush();
        if (!d_z || lane >= n_run) continue;
        // lane j: the dL/dz chain of point p0 + j through view v
        const int64_t p = p0 + lane;
        if (z_mask && !z_mask[p]) continue;   // d_z written 0 below
        const PointGeo G = point_geo(rays, zs, K, rays_per_obj, cams, hl, wl, img_w, img_h, p, ns, v);
        const float *ray = rays + (p / K) * 8;
        const float *cam = cams + (((p / K) / rays_per_obj) * ns + v) * 16;
        const float fx = cam[12], fy = cam[13];
        const float wlf = (float)wl, hlf = (float)hl;
        const float sx = __fdiv_rn(mul_rn(__fdiv_rn(wlf, sub_rn(wlf, 1.f)), 2.f), img_w);
        const float sy = __fdiv_rn(mul_rn(__fdiv_rn(hlf, sub_rn(hlf, 1.f)), 2.f), img_h);
        const float hx = mul_rn(sub_rn(wlf, 1.f), 0.5f), hy = mul_rn(sub_rn(hlf, 1.f), 0.5f);
        // torch clip_coordinates_set_grad: borders count as out of bounds (NaN -> 0)
        const float gclip_x = (G.ixu > 0.f && G.ixu < wlf - 1.f) ? 1.f : 0.f;
        const float gclip_y = (G.iyu > 0.f && G.iyu < hlf - 1.f) ? 1.f : 0.f;
        // projection chain: ix = (gx + 1) hx, gx = u sx - 1, u = -(xc0 / xc2) fx + cx
        const float du = dix_run * gclip_x * hx * sx, dv = diy_run * gclip_y * hy * sy;
        const float inv = 1.f / G.xc[2];
        float dxc[3];
        dxc[0] = -du * fx * inv;
        dxc[1] = -dv * fy * inv;
        dxc[2] = (du * fx * G.xc[0] + dv * fy * G.xc[1]) * inv * inv;
        // features: x_rot (3) then PE sin(phase_q + x_rot_j freq_q) at 3 + 3q + j
        const float *df = d_feat + (v * n_points + p) * 64;
        float dxr[3] = {df[0] + dxc[0], df[1] + dxc[1], df[2] + dxc[2]};
        for (int q = 0; q < pe_n; ++q) {
            const float f = pe[q], ph = pe[16 + q];
#pragma unroll
            for (int jj = 0; jj < 3; ++jj)
                dxr[jj] += df[3 + 3 * q + jj] * cosf(add_rn(ph, mul_rn(G.xr[jj], f))) * f;
        }
        // x_rot = R x, x = o + z d
        float dzs = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float dxw = cam[i] * dxr[0] + cam[3 + i] * dxr[1] + cam[6 + i] * dxr[2];
            dzs += dxw * ray[3 + i];
        }
        dz_sum = v == 0 ? dzs : dz_sum + dzs;
    }
    if (d_z && lane < n_run) d_z[p0 + lane] = (z_mask && !z_mask[p0 + lane]) ? 0.f : dz_sum;
}

// ---------------------------------------------------------------------------
int launch_composite_bwd(const float *z, const float *raw, const float *rays, int64_t n_rays, int K,
                         int white_bkgd, const float *d_rgb, const float *d_depth, const float *d_weights,
                         float *d_raw, float *d_z, hipStream_t st) {
    if (n_rays == 0) return PNR_OK;
    const int nch = (K + 63) / 64;
    if (nch > 4) return fail(PNR_ERR_UNSUPPORTED, "composite backward: K <= 256");
    auto kern = nch == 1 ? k_composite_bwd<1> : nch == 2 ? k_composite_bwd<2>
              : nch == 3 ? k_composite_bwd<3> : k_composite_bwd<4>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((n_rays + 3) / 4)), dim3(256), 0, st, z, raw, rays, n_rays, K,
                       white_bkgd, d_rgb, d_depth, d_weights, d_raw, d_z);
    return launch_ok("composite_bwd") ? PNR_OK : PNR_ERR_HIP;
}

int launch_points_in_bwd(const float *rays, const float *zs, int K, int64_t rays_per_obj, int64_t n_points,
                         int ns, const float *cams, const float *latent, int hl, int wl, float img_w, float img_h,
                         const float *pe, int pe_n, const float *d_feat, const float *d_zlat,
                         float *d_latent, float *d_z, const uint8_t *z_mask, hipStream_t st) {
    if (n_points == 0) return PNR_OK;
    const int64_t waves = (n_points + RUN - 1) / RUN;
    hipLaunchKernelGGL(k_points_in_bwd, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, rays, zs, K,
                       rays_per_obj, n_points, ns, cams, latent, hl, wl, img_w, img_h, pe, pe_n, d_feat, d_zlat,
                       d_latent, d_z, z_mask);
    return launch_ok("points_in_bwd") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
