// Along-ray kernels of the ray march: stratified coarse sampling, inverse-CDF
// fine sampling + depth samples + merge sort, and the alpha composite.
//
// One wavefront owns one ray (rays are independent; the only along-ray
// dependencies are the transmittance cumprod, the cdf cumsum and the sort),
// so every cross-sample step is a wave64 shuffle scan or an LDS sort private
// to that wave.  Loads of the (B, K) / (B, K, 4) tensors are coalesced:
// lane k of chunk c reads sample c*64+k.
#include "pnr_common.h"

namespace pnr {

// ---------------------------------------------------------------------------
// sample_coarse — nerf.py:98-118
//   t_k = linspace(0, 1 - 1/Kc, Kc)[k] + u_k / Kc ;  z = near (1 - t) + far t
// torch.linspace evaluates the first half as start + step*i and the second half
// as end - step*(steps-1-i) (ATen RangeFactoriesKernel); we follow that form.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float linspace_at(int i, int n, float end, float step) {
    if (n == 1) return 0.0f;
    return (i < n / 2) ? mul_rn(step, (float)i) : sub_rn(end, mul_rn(step, (float)(n - 1 - i)));
}

__global__ void k_sample_coarse(const float *__restrict__ rays, int64_t n_rays, int kc,
                                const float *__restrict__ u, int lindisp,
                                float *__restrict__ z) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_rays * kc) return;
    const int64_t b = idx / kc;
    const int k = (int)(idx - b * kc);
    const float near = rays[b * 8 + 6], far = rays[b * 8 + 7];
    const float end = (float)(1.0 - 1.0 / (double)kc);
    const float lstep = (kc > 1) ? __fdiv_rn(end, (float)(kc - 1)) : 0.0f;
    const float step = (float)(1.0 / (double)kc);
    float t = add_rn(linspace_at(k, kc, end, lstep), mul_rn(u[idx], step));
    z[idx] = t_to_z(t, near, far, lindisp != 0);
}

// ---------------------------------------------------------------------------
// sample_fine + sample_fine_depth + sort — nerf.py:120-161, 284-295
// One 64-lane block per ray.  LDS: cdf[Kc+1] then the sort buffer[N].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_sample_fine(
    const float *__restrict__ rays, int kc, const float *__restrict__ z_coarse,
    const float *__restrict__ weights, const float *__restrict__ depth, int kf, int kfd,
    float depth_std, const float *__restrict__ u_fine, const float *__restrict__ u_jit,
    const float *__restrict__ n_depth, int lindisp, int n_sort, float *__restrict__ z_fine) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *cdf = smem;            // kc + 1
    float *s = smem + kc + 1;     // n_sort (power of two >= kc + kf)
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const float near = rays[b * 8 + 6], far = rays[b * 8 + 7];
    const float *w = weights + b * kc;

    // pdf = (w + 1e-5) / sum(w + 1e-5)   (nerf.py:130-131)
    float part = 0.0f;
    for (int k = lane; k < kc; k += 64) part += add_rn(w[k], 1e-5f);
    const float total = wave_sum(part);
    // cdf = [0, cumsum(pdf)]; torch's CPU cumsum accumulates in double (acc_type),
    // rounding every prefix to fp32 — a double wave scan reproduces those values.
    double carry = 0.0;
    if (lane == 0) cdf[0] = 0.0f;
    for (int c0 = 0; c0 < kc; c0 += 64) {
        const int k = c0 + lane;
        double p = (k < kc) ? (double)__fdiv_rn(add_rn(w[k], 1e-5f), total) : 0.0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            double q = __shfl_up(p, off, 64);
            if (lane >= off) p += q;
        }
        if (k < kc) cdf[k + 1] = (float)(carry + p);
        carry += __shfl(p, 63, 64);
    }
    __syncthreads();

    const int nf = kf - kfd;
    const float inv_steps = (float)kc;
    // importance samples (nerf.py:135-148)
    for (int j = lane; j < nf; j += 64) {
        const float u = u_fine[b * nf + j];
        // searchsorted(cdf, u, right=True): number of cdf entries <= u
        int lo = 0, hi = kc + 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
        }
        float ind = fmaxf(sub_rn((float)lo, 1.0f), 0.0f);
        float t = __fdiv_rn(add_rn(ind, u_jit[b * nf + j]), inv_steps);
        s[kc + j] = t_to_z(t, near, far, lindisp != 0);
    }
    // depth samples (nerf.py:157-160): clamp(depth + N(0,1) * std, near, far)
    for (int j = lane; j < kfd; j += 64) {
        float zz = add_rn(depth[b], mul_rn(n_depth[b * kfd + j], depth_std));
        s[kc + nf + j] = fmaxf(fminf(zz, far), near);
    }
    for (int k = lane; k < kc; k += 64) s[k] = z_coarse[b * kc + k];
    for (int k = kc + kf + lane; k < n_sort; k += 64) s[k] = __builtin_inff();
    __syncthreads();
    // bitonic sort of n_sort values, ascending (torch.sort, nerf.py:295)
    for (int size = 2; size <= n_sort; size <<= 1) {
        for (int j = size >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < (n_sort >> 1); t += 64) {
                const int lo = 2 * j * (t / j) + (t % j);
                const int hi = lo + j;
                const bool asc = (lo & size) == 0;
                float a = s[lo], c = s[hi];
                if ((a > c) == asc) { s[lo] = c; s[hi] = a; }
            }
            __syncthreads();
        }
    }
    const int k_all = kc + kf;
    for (int k = lane; k < k_all; k += 64) z_fine[b * k_all + k] = s[k];
}

// ---------------------------------------------------------------------------
// composite — nerf.py:176-249
//   delta_i = z_{i+1} - z_i, delta_last = far - z_last
//   alpha = 1 - exp(-delta * relu(sigma));  T = excl. cumprod(1 - alpha + 1e-10)
//   w = alpha * T;  rgb = sum w c;  depth = sum w z;  white: rgb += 1 - sum w
// One wave per ray, 4 rays per 256-thread block; the cumprod is a double-precision
// wave scan (torch's CPU cumprod accumulates in double and rounds each prefix).
// ---------------------------------------------------------------------------
// NCH > 0: K <= 64 NCH, every chunk's loads are issued before the first scan (more
// bytes in flight per wave: the kernel is HBM-bound); NCH == 0: any K, chunk loop.
template <int NCH>
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
    constexpr int NR = NCH > 0 ? NCH : 1;
    float zk[NR], zn[NR];
    f4 v[NR];
    auto load = [&](int i, int k) {
        zk[i] = 0.f;
        zn[i] = 0.f;
        v[i] = f4{0.f, 0.f, 0.f, 0.f};
        if (k < K) {
            zk[i] = __builtin_nontemporal_load(zr + k);
            zn[i] = (k + 1 < K) ? zr[k + 1] : far;
            const float *rp = reinterpret_cast<const float *>(rr + k);
            v[i] = f4{__builtin_nontemporal_load(rp), __builtin_nontemporal_load(rp + 1),
                      __builtin_nontemporal_load(rp + 2), __builtin_nontemporal_load(rp + 3)};
        }
    };
    if constexpr (NCH > 0) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) load(i, 64 * i + lane);
    }
    double carry = 1.0;
    float sr = 0.f, sg = 0.f, sb = 0.f, sd = 0.f, sw = 0.f;
    auto step = [&](int c, int i) {
        const int k = 64 * c + lane;
        const bool valid = k < K;
        const float delta = sub_rn(zn[i], zk[i]);
        const float alpha = valid ? sub_rn(1.0f, expf(mul_rn(-delta, fmaxf(v[i].w, 0.0f)))) : 0.0f;
        const float shifted = valid ? add_rn(sub_rn(1.0f, alpha), 1e-10f) : 1.0f;
        double p = shifted;  // inclusive product scan
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            double q = __shfl_up(p, off, 64);
            if (lane >= off) p *= q;
        }
        double excl = __shfl_up(p, 1, 64);
        if (lane == 0) excl = 1.0;
        const float T = (float)(carry * excl);
        const float wk = mul_rn(alpha, T);
        carry *= __shfl(p, 63, 64);
        if (valid) {
            if (weights) __builtin_nontemporal_store(wk, weights + b * K + k);
            sr += mul_rn(wk, v[i].x);
            sg += mul_rn(wk, v[i].y);
            sb += mul_rn(wk, v[i].z);
            sd += mul_rn(wk, zk[i]);
            sw += wk;
        }
    };
    if constexpr (NCH > 0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) step(c, c);
    } else {
        for (int c = 0; c < (K + 63) / 64; ++c) {
            load(0, 64 * c + lane);
            step(c, 0);
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
// host launchers (validated by the extern "C" layer in abi.cpp)
// ---------------------------------------------------------------------------
int launch_sample_coarse(const float *rays, int64_t n_rays, int kc, const float *u, int lindisp,
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
                       float depth_std, const float *u_fine, const float *u_jit,
                       const float *n_depth, int lindisp, float *z_fine, hipStream_t st) {
    if (n_rays == 0) return PNR_OK;
    const int n_sort = sort_width(kc + kf);
    const size_t lds = sizeof(float) * (size_t)(kc + 1 + n_sort);
    hipLaunchKernelGGL(k_sample_fine, dim3((unsigned)n_rays), dim3(64), lds, st, rays, kc,
                       z_coarse, weights, depth, kf, kfd, depth_std, u_fine, u_jit, n_depth,
                       lindisp, n_sort, z_fine);
    return launch_ok("sample_fine") ? PNR_OK : PNR_ERR_HIP;
}

int launch_composite(const float *z, const float *raw, const float *rays, int64_t n_rays, int K,
                     int white_bkgd, float *weights, float *rgb, float *depth, hipStream_t st) {
    if (n_rays == 0) return PNR_OK;
    const int64_t blocks = (n_rays + 3) / 4;
    const int nch = (K + 63) / 64;
    auto kern = nch == 1 ? k_composite<1> : nch == 2 ? k_composite<2> : nch == 3 ? k_composite<3>
              : nch == 4 ? k_composite<4> : k_composite<0>;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, z, raw, rays,
                       n_rays, K, white_bkgd, weights, rgb, depth);
    return launch_ok("composite") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
