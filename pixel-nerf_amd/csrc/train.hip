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
        sg[i] = fmaxf(v[i].w, 0.0f);
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
// per-point input backward (NS == 1).  One wave per point (o + z d of ray b):
//   d latent[corner][c] += w_corner d_zlat[c]                  (atomic, channels-last)
//   d z_sample = d . R^T (d x_rot)   with d x_rot from
//     features: d f[0:3] (x_rot) + sum_q d f[3 + 3q + j] cos(phase_q + x_rot_j freq_q) freq_q
//     projection: d x_cam through u = -x/z fx + cx, v = -y/z fy + cy and the bilinear
//       weights (out-of-range corners count as 0; clipped coordinates pass no gradient,
//       as torch's grid_sampler_2d_backward with border padding)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_points_in_bwd(
    const float *__restrict__ rays, const float *__restrict__ zs, int K, int64_t rays_per_obj,
    int64_t n_points, const float *__restrict__ cams, const float *__restrict__ latent, int hl, int wl,
    float img_w, float img_h, const float *__restrict__ pe, int pe_n, const float *__restrict__ d_feat,
    const float *__restrict__ d_zlat, float *__restrict__ d_latent, float *__restrict__ d_z) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= n_points) return;
    const int64_t b = p / K;
    const float *ray = rays + b * 8;
    const float zz = zs[p];
    const float dx = ray[3], dy = ray[4], dz = ray[5];
    const float px = add_rn(ray[0], mul_rn(zz, dx));
    const float py = add_rn(ray[1], mul_rn(zz, dy));
    const float pz = add_rn(ray[2], mul_rn(zz, dz));
    const int64_t obj = b / rays_per_obj;
    const float *cam = cams + obj * 16;
    float xr[3], xc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        xr[i] = add_rn(add_rn(mul_rn(cam[3 * i], px), mul_rn(cam[3 * i + 1], py)), mul_rn(cam[3 * i + 2], pz));
        xc[i] = add_rn(xr[i], cam[9 + i]);
    }
    const float fx = cam[12], fy = cam[13], cx = cam[14], cy = cam[15];
    // forward projection, as k_point_mlp
    const float u0 = __fdiv_rn(-xc[0], xc[2]), v0 = __fdiv_rn(-xc[1], xc[2]);
    const float u = add_rn(mul_rn(u0, fx), cx), w = add_rn(mul_rn(v0, fy), cy);
    const float wlf = (float)wl, hlf = (float)hl;
    const float lsx = mul_rn(__fdiv_rn(wlf, sub_rn(wlf, 1.f)), 2.f);
    const float lsy = mul_rn(__fdiv_rn(hlf, sub_rn(hlf, 1.f)), 2.f);
    const float sx = __fdiv_rn(lsx, img_w), sy = __fdiv_rn(lsy, img_h);
    const float gx = sub_rn(mul_rn(u, sx), 1.f), gy = sub_rn(mul_rn(w, sy), 1.f);
    const float hx = mul_rn(sub_rn(wlf, 1.f), 0.5f), hy = mul_rn(sub_rn(hlf, 1.f), 0.5f);
    const float ixu = mul_rn(add_rn(gx, 1.f), hx), iyu = mul_rn(add_rn(gy, 1.f), hy);
    const float ix = fminf(fmaxf(ixu, 0.f), wlf - 1.f), iy = fminf(fmaxf(iyu, 0.f), hlf - 1.f);
    // torch clip_coordinates_set_grad: borders count as out of bounds (NaN -> 0)
    const float gclip_x = (ixu > 0.f && ixu < wlf - 1.f) ? 1.f : 0.f;
    const float gclip_y = (iyu > 0.f && iyu < hlf - 1.f) ? 1.f : 0.f;
    const float x0f = floorf(ix), y0f = floorf(iy);
    const float we = sub_rn(ix, x0f), wn = sub_rn(iy, y0f);
    const int x0 = (int)x0f, y0 = (int)y0f;
    const bool inx1 = x0 + 1 < wl, iny1 = y0 + 1 < hl;
    const float wnw = mul_rn(sub_rn(1.f, wn), sub_rn(1.f, we)), wne = mul_rn(sub_rn(1.f, wn), we);
    const float wsw = mul_rn(wn, sub_rn(1.f, we)), wse = mul_rn(wn, we);
    const int64_t base = obj * (int64_t)hl * wl * 512;
    const int64_t o00 = base + ((int64_t)y0 * wl + x0) * 512;
    const int64_t o01 = base + ((int64_t)y0 * wl + (inx1 ? x0 + 1 : x0)) * 512;
    const int64_t o10 = base + ((int64_t)(iny1 ? y0 + 1 : y0) * wl + x0) * 512;
    const int64_t o11 = base + ((int64_t)(iny1 ? y0 + 1 : y0) * wl + (inx1 ? x0 + 1 : x0)) * 512;
    float dwe = 0.f, dwn = 0.f;
    const float *gz = d_zlat + p * 512;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int ch = half * 256 + lane * 4;
        const f4 gv = *reinterpret_cast<const f4 *>(gz + ch);
        const f4 l00 = *reinterpret_cast<const f4 *>(latent + o00 + ch);
        f4 l01 = *reinterpret_cast<const f4 *>(latent + o01 + ch);
        f4 l10 = *reinterpret_cast<const f4 *>(latent + o10 + ch);
        f4 l11 = *reinterpret_cast<const f4 *>(latent + o11 + ch);
        if (!inx1) { l01 = f4{0.f, 0.f, 0.f, 0.f}; l11 = l01; }
        if (!iny1) { l10 = f4{0.f, 0.f, 0.f, 0.f}; l11 = l10; }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            dwe += gv[q] * ((1.f - wn) * (l01[q] - l00[q]) + wn * (l11[q] - l10[q]));
            dwn += gv[q] * ((1.f - we) * (l10[q] - l00[q]) + we * (l11[q] - l01[q]));
            if (d_latent) {
                atomicAdd(d_latent + o00 + ch + q, wnw * gv[q]);
                if (inx1) atomicAdd(d_latent + o01 + ch + q, wne * gv[q]);
                if (iny1) atomicAdd(d_latent + o10 + ch + q, wsw * gv[q]);
                if (inx1 && iny1) atomicAdd(d_latent + o11 + ch + q, wse * gv[q]);
            }
        }
    }
    if (!d_z) return;
    dwe = wave_sum_dpp(dwe);
    dwn = wave_sum_dpp(dwn);
    if (lane != 0) return;
    // projection chain: ix = (gx + 1) hx, gx = u sx - 1, u = -(xc0 / xc2) fx + cx
    const float dix = dwe * gclip_x, diy = dwn * gclip_y;
    const float du = dix * hx * sx, dv = diy * hy * sy;
    const float inv = 1.f / xc[2];
    float dxc[3];
    dxc[0] = -du * fx * inv;
    dxc[1] = -dv * fy * inv;
    dxc[2] = (du * fx * xc[0] + dv * fy * xc[1]) * inv * inv;
    // features: x_rot (3) then PE sin(phase_q + x_rot_j freq_q) at 3 + 3q + j
    const float *df = d_feat + p * 64;
    float dxr[3] = {df[0] + dxc[0], df[1] + dxc[1], df[2] + dxc[2]};
    for (int q = 0; q < pe_n; ++q) {
        const float f = pe[q], ph = pe[16 + q];
#pragma unroll
        for (int j = 0; j < 3; ++j)
            dxr[j] += df[3 + 3 * q + j] * cosf(add_rn(ph, mul_rn(xr[j], f))) * f;
    }
    // x_rot = R x, x = o + z d
    float dzs = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float dxw = cam[i] * dxr[0] + cam[3 + i] * dxr[1] + cam[6 + i] * dxr[2];
        dzs += dxw * (i == 0 ? dx : (i == 1 ? dy : dz));
    }
    d_z[p] = dzs;
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
                         const float *cams, const float *latent, int hl, int wl, float img_w, float img_h,
                         const float *pe, int pe_n, const float *d_feat, const float *d_zlat,
                         float *d_latent, float *d_z, hipStream_t st) {
    if (n_points == 0) return PNR_OK;
    hipLaunchKernelGGL(k_points_in_bwd, dim3((unsigned)((n_points + 3) / 4)), dim3(256), 0, st, rays, zs, K,
                       rays_per_obj, n_points, cams, latent, hl, wl, img_w, img_h, pe, pe_n, d_feat, d_zlat,
                       d_latent, d_z);
    return launch_ok("points_in_bwd") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
