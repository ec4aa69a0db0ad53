// Along-ray kernels of the ray march: stratified coarse sampling, inverse-CDF
// fine sampling + depth samples + merge sort, and the alpha composite.
//
// One wavefront owns one ray (rays are independent; the only along-ray
// dependencies are the transmittance cumprod, the cdf cumsum and the sort),
// so every cross-sample step is a wave64 shuffle scan or an LDS sort private
// to that wave.  Loads of the (B, K) / (B, K, 4) tensors are coalesced:
// lane k of chunk c reads sample c*64+k.
#include "march_dev.h"

namespace pnr {

// ---------------------------------------------------------------------------
// sample_coarse — nerf.py:98-118 (coarse_z, march_dev.h)
// ---------------------------------------------------------------------------
__global__ void k_sample_coarse(const float *__restrict__ rays, int64_t n_rays, int kc,
                                const RngSrc u, int lindisp, float *__restrict__ z) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_rays * kc) return;
    const int64_t b = idx / kc;
    const int k = (int)(idx - b * kc);
    z[idx] = coarse_z(u, b, kc, k, rays[b * 8 + 6], rays[b * 8 + 7], lindisp != 0);
}

// ---------------------------------------------------------------------------
// sample_fine + sample_fine_depth + sort — nerf.py:120-161, 284-295 (sample_fine_wave)
// One 64-lane block per ray.  LDS: cdf[Kc+1] then the sort buffer[N].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_sample_fine(
    const float *__restrict__ rays, int kc, const float *__restrict__ z_coarse,
    const float *__restrict__ weights, const float *__restrict__ depth, int kf, int kfd,
    float depth_std, const RngSrc u_fine, const RngSrc u_jit, const RngSrc n_depth, int lindisp,
    int n_sort, float *__restrict__ z_fine,
    int *__restrict__ origin, float *__restrict__ z_new) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *cdf = smem;            // kc + 1
    float *s = smem + kc + 1;     // n_sort (power of two >= kc + kf)
    int *si = reinterpret_cast<int *>(s + n_sort);   // origin of each sorted value (origin != NULL)
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    sample_fine_wave(lane, b, rays[b * 8 + 6], rays[b * 8 + 7], kc, weights + b * kc, z_coarse + b * kc,
                     kfd > 0 ? depth[b] : 0.f, kf, kfd, depth_std, u_fine, u_jit, n_depth, lindisp != 0, n_sort,
                     cdf, s, si, z_fine, origin, z_new);
}

// raw_f[b][k] = raw of sorted fine sample k: the coarse pass's output for a coarse sample
// (origin < kc), the new-sample evaluation otherwise.  Used when the fine pass runs the
// coarse MLP (mlp_fine is None, models.py:242-255): its kc coarse points were already
// evaluated, bit-identically (a point's output does not depend on its tile neighbours).
__global__ __launch_bounds__(256) void k_merge_raw(const int *__restrict__ origin, const f4 *__restrict__ raw_c,
                                                   const f4 *__restrict__ raw_new, int64_t n, int kc, int kf,
                                                   f4 *__restrict__ raw_f) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k_all = kc + kf;
    const int64_t b = i / k_all;
    const int o = origin[i];
    raw_f[i] = o < kc ? raw_c[b * kc + o] : raw_new[b * kf + (o - kc)];
}

// ---------------------------------------------------------------------------
// composite — nerf.py:176-249 (composite_wave, march_dev.h)
//   delta_i = z_{i+1} - z_i, delta_last = far - z_last
//   alpha = 1 - exp(-delta * relu(sigma));  T = excl. cumprod(1 - alpha + 1e-10)
//   w = alpha * T;  rgb = sum w c;  depth = sum w z;  white: rgb += 1 - sum w
// One wave per ray, 4 rays per 256-thread block; the cumprod accumulates in double
// (torch's CPU cumprod accumulates in double and rounds each prefix).
// ---------------------------------------------------------------------------
// K <= 256: one wave per two rays, lane l loads samples 64 i + l of both (1 KB of raw per load
// instruction), all loads issued before the first wait (clamped addresses), then composite_wave
// (march_dev.h) per ray.  Two rays per wave: +6-8 % over one (0.78-0.79 against 0.72-0.73 of HBM
// peak, same box, profiles/r6e/ab_rpw2.txt): twice the bytes in flight per wave.
template <int S>
__global__ __launch_bounds__(256) void k_composite_c(
    const float *__restrict__ z, const float *__restrict__ raw, const float *__restrict__ rays,
    int64_t n_rays, int K, int white_bkgd, float *__restrict__ weights,
    float *__restrict__ rgb_out, float *__restrict__ depth_out) {
    constexpr int RPW = 2;   // rays per wave
    const int lane = threadIdx.x & 63;
    const int64_t b0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    if (b0 >= n_rays) return;
    float zk[RPW][S], wk[S], far[RPW];
    f4 v[RPW][S];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int64_t b = b0 + j < n_rays ? b0 + j : n_rays - 1;
        far[j] = rays[b * 8 + 7];
        const float *zr = z + b * K;
        const f4 *rr = reinterpret_cast<const f4 *>(raw) + b * K;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const int k = 64 * i + lane;
            const int kc = k < K ? k : K - 1;
            zk[j][i] = __builtin_nontemporal_load(zr + kc);
            v[j][i] = __builtin_nontemporal_load(rr + kc);
        }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        if (b0 + j >= n_rays) break;
        composite_wave<S>(lane, b0 + j, K, far[j], zk[j], v[j], white_bkgd, weights, rgb_out, depth_out, wk);
    }
}

// any K: 64-sample chunks, one wave scan per chunk with a running carry
__global__ __launch_bounds__(256) void k_composite(
    const float *__restrict__ z, const float *__restrict__ raw, const float *__restrict__ rays,
    int64_t n_rays, int K, int white_bkgd, float *__restrict__ weights,
    float *__restrict__ rgb_out, float *__restrict__ depth_out) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= n_rays) return;
    const float far = rays[b * 8 + 7];
    const float *zr = z + b * K;
    const f4 *rr = reinterpret_cast<const f4 *>(raw) + b * K;
    double carry = 1.0;
    float sr = 0.f, sg = 0.f, sb = 0.f, sd = 0.f, sw = 0.f;
    for (int c0 = 0; c0 < K; c0 += 64) {
        const int k = c0 + lane;
        const bool valid = k < K;
        float zk = 0.f, zn = 0.f;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (valid) {
            zk = zr[k];
            zn = (k + 1 < K) ? zr[k + 1] : far;
            v = rr[k];
        }
        const float delta = sub_rn(zn, zk);
        const float alpha = valid ? sub_rn(1.0f, expf(mul_rn(-delta, max_nc(v.w, 0.0f)))) : 0.0f;
        const float shifted = valid ? add_rn(sub_rn(1.0f, alpha), 1e-10f) : 1.0f;
        double p = shifted;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const double q = __shfl_up(p, off, 64);
            if (lane >= off) p *= q;
        }
        double excl = __shfl_up(p, 1, 64);
        if (lane == 0) excl = 1.0;
        const float wk = mul_rn(alpha, (float)(carry * excl));
        carry *= __shfl(p, 63, 64);
        if (valid) {
            if (weights) weights[b * K + k] = wk;
            sr += mul_rn(wk, v.x);
            sg += mul_rn(wk, v.y);
            sb += mul_rn(wk, v.z);
            sd += mul_rn(wk, zk);
            sw += wk;
        }
    }
    sr = wave_sum(sr);
    sg = wave_sum(sg);
    sb = wave_sum(sb);
    sd = wave_sum(sd);
    sw = wave_sum(sw);
    if (lane == 0) {
        if (white_bkgd) {
            sr = sub_rn(add_rn(sr, 1.0f), sw);
            sg = sub_rn(add_rn(sg, 1.0f), sw);
            sb = sub_rn(add_rn(sb, 1.0f), sw);
        }
        rgb_out[b * 3 + 0] = sr;
        rgb_out[b * 3 + 1] = sg;
        rgb_out[b * 3 + 2] = sb;
        depth_out[b] = sd;
    }
}

// ---------------------------------------------------------------------------
// gen_rays — util.py:113-143 (unproj_map) + 238-276.  One thread per pixel:
//   X = (x - cx) / fx, Y = (y - cy) / fy, u = (X, -Y, -1) / |(X, -Y, -1)|,
//   ray = [t_wc, R_wc u, near, far]   (pose row-major, rows 3 or 4 per image)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gen_rays(const float *__restrict__ poses, int pose_rows,
                                                  int64_t n_pix, int width, int height, float fx,
                                                  float fy, float cx, float cy, float near,
                                                  float far, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pix) return;
    const int64_t hw = (int64_t)width * height;
    const int64_t img = i / hw;
    const int pix = (int)(i - img * hw);
    const int y = pix / width, x = pix - y * width;
    const float X = __fdiv_rn(sub_rn((float)x, cx), fx);
    const float Y = __fdiv_rn(sub_rn((float)y, cy), fy);
    const float nrm = __fsqrt_rn(add_rn(add_rn(mul_rn(X, X), mul_rn(Y, Y)), 1.0f));
    const float u0 = __fdiv_rn(X, nrm), u1 = __fdiv_rn(-Y, nrm), u2 = __fdiv_rn(-1.0f, nrm);
    const float *P = poses + img * pose_rows * 4;
    f4 a, b;
    float d[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        d[r] = add_rn(add_rn(mul_rn(P[4 * r], u0), mul_rn(P[4 * r + 1], u1)), mul_rn(P[4 * r + 2], u2));
    a = f4{P[3], P[7], P[11], d[0]};
    b = f4{d[1], d[2], near, far};
    f4 *o = reinterpret_cast<f4 *>(out + i * 8);
    o[0] = a;
    o[1] = b;
}

// ---------------------------------------------------------------------------
// host launchers (validated by the extern "C" layer in abi.cpp)
// ---------------------------------------------------------------------------
int launch_sample_coarse(const float *rays, int64_t n_rays, int kc, const RngSrc &u, int lindisp,
                         float *z, hipStream_t st) {
    const int64_t n = n_rays * kc;
    if (n == 0) return PNR_OK;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_sample_coarse, dim3((unsigned)blocks), dim3(256), 0, st, rays, n_rays,
                       kc, u, lindisp, z);
    return launch_ok("sample_coarse") ? PNR_OK : PNR_ERR_HIP;
}

int sort_width(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

int launch_sample_fine(const float *rays, int64_t n_rays, int kc, const float *z_coarse,
                       const float *weights, const float *depth, int kf, int kfd,
                       float depth_std, const RngSrc &u_fine, const RngSrc &u_jit,
                       const RngSrc &n_depth, int lindisp, float *z_fine, hipStream_t st,
                       int *origin, float *z_new) {
    if (n_rays == 0) return PNR_OK;
    const int n_sort = sort_width(kc + kf);
    const size_t lds = sizeof(float) * (size_t)(kc + 1 + (origin ? 2 : 1) * n_sort);
    hipLaunchKernelGGL(k_sample_fine, dim3((unsigned)n_rays), dim3(64), lds, st, rays, kc,
                       z_coarse, weights, depth, kf, kfd, depth_std, u_fine, u_jit, n_depth,
                       lindisp, n_sort, z_fine, origin, z_new);
    return launch_ok("sample_fine") ? PNR_OK : PNR_ERR_HIP;
}

int launch_merge_raw(const int *origin, const float *raw_c, const float *raw_new, int64_t n_rays, int kc, int kf,
                     float *raw_f, hipStream_t st) {
    const int64_t n = n_rays * (kc + kf);
    if (n == 0) return PNR_OK;
    hipLaunchKernelGGL(k_merge_raw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, origin,
                       reinterpret_cast<const f4 *>(raw_c), reinterpret_cast<const f4 *>(raw_new), n, kc, kf,
                       reinterpret_cast<f4 *>(raw_f));
    return launch_ok("merge_raw") ? PNR_OK : PNR_ERR_HIP;
}

int launch_composite(const float *z, const float *raw, const float *rays, int64_t n_rays, int K,
                     int white_bkgd, float *weights, float *rgb, float *depth, hipStream_t st) {
    if (n_rays == 0) return PNR_OK;
    const int nch = (K + 63) / 64;
    const int64_t grid = (n_rays + 7) / 8;   // one wave per two rays
    auto kern = nch == 1 ? k_composite_c<1> : nch == 2 ? k_composite_c<2> : nch == 3 ? k_composite_c<3>
              : nch == 4 ? k_composite_c<4> : k_composite;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, st, z, raw, rays,
                       n_rays, K, white_bkgd, weights, rgb, depth);
    return launch_ok("composite") ? PNR_OK : PNR_ERR_HIP;
}

int launch_gen_rays(const float *poses, int64_t n_images, int pose_rows, int width, int height,
                    float fx, float fy, float cx, float cy, float near, float far, float *rays,
                    hipStream_t st) {
    const int64_t n = n_images * width * height;
    if (n == 0) return PNR_OK;
    hipLaunchKernelGGL(k_gen_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, poses, pose_rows,
                       n, width, height, fx, fy, cx, cy, near, far, rays);
    return launch_ok("gen_rays") ? PNR_OK : PNR_ERR_HIP;
}

// ---------------------------------------------------------------------------
// counter-mode draws materialised (pnr_rng_fill): the same rng_uniform / rng_normal the
// samplers call, one thread per draw
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rng_fill(const RngSrc r, int64_t n_rays, int width, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_rays * width) return;
    const int64_t b = i / width;
    const int k = (int)(i - b * width);
    out[i] = r.stream == PNR_RNG_N_DEPTH ? rng_normal(r, b, width, k) : rng_uniform(r, b, width, k);
}

int launch_rng_fill(const RngSrc &r, int64_t n_rays, int width, float *out, hipStream_t st) {
    const int64_t n = n_rays * width;
    if (n == 0) return PNR_OK;
    hipLaunchKernelGGL(k_rng_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, r, n_rays, width, out);
    return launch_ok("rng_fill") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
