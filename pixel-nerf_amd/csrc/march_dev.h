// Along-ray device functions shared by the standalone march kernels (march.hip) and the
// fused ray march in k_point_mlp's epilogue (mlp.hip): one wavefront owns one ray.
// The standalone kernels and the fused epilogue run the SAME code, so their results are
// bit-identical (tests/test_gpu_parity.py::test_fused_march_matches_unfused).
#pragma once
#include "pnr_common.h"

namespace pnr {

// Diagnostic stamps of the fused epilogue (pnr_diag.h, included by mlp.hip); no-ops elsewhere.
#ifndef EPI_T
#define EPI_DECL
#define EPI_T(i) ((void)0)
#endif

// LDS ops of one wave complete in order; this only orders them for the compiler and drains
// the wave's own outstanding LDS operations (no s_barrier: callers are single waves).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- sample_coarse — nerf.py:98-118 ------------------------------------------------------
//   t_k = linspace(0, 1 - 1/Kc, Kc)[k] + u_k / Kc ;  z = near (1 - t) + far t
// torch.linspace evaluates the first half as start + step*i and the second half as
// end - step*(steps-1-i) (ATen RangeFactoriesKernel); this follows that form.
__device__ __forceinline__ float linspace_at(int i, int n, float end, float step) {
    if (n == 1) return 0.0f;
    return (i < n / 2) ? mul_rn(step, (float)i) : sub_rn(end, mul_rn(step, (float)(n - 1 - i)));
}

__device__ __forceinline__ float coarse_z(const RngSrc &u, int64_t b, int kc, int k, float near, float far,
                                          bool lindisp) {
    const float end = (float)(1.0 - 1.0 / (double)kc);
    const float lstep = (kc > 1) ? __fdiv_rn(end, (float)(kc - 1)) : 0.0f;
    const float step = (float)(1.0 / (double)kc);
    const float t = add_rn(linspace_at(k, kc, end, lstep), mul_rn(rng_uniform(u, b, kc, k), step));
    return t_to_z(t, near, far, lindisp);
}

// ---- composite — nerf.py:176-249 ------------------------------------------------------------
//   delta_i = z_{i+1} - z_i, delta_last = far - z_last
//   alpha = 1 - exp(-delta * relu(sigma));  T = excl. cumprod(1 - alpha + 1e-10)
//   w = alpha * T;  rgb = sum w c;  depth = sum w z;  white: rgb += 1 - sum w
// K <= 64 S (S = ceil(K / 64) chunks): lane l holds samples 64 i + l of chunk i (zk, v; lanes past
// K hold clamped copies), so a ray's loads are lane-contiguous (1 KB of raw per instruction from
// HBM, conflict-free from LDS).  One exclusive double product scan per chunk (torch's CPU cumprod
// accumulates in double and rounds each prefix) with a running carry; the next sample's z comes
// from the neighbour lane by DPP (lane 63: lane 0 of the next chunk).  Writes the weights (if
// non-NULL), rgb and depth of ray b; returns the weights in wk and the depth (every lane).  The
// standalone composite and the fused march's epilogue both run this, so the unfused march is
// bit-identical to the fused one.  (Round 4's layout -- lane l owning the S consecutive samples
// S l .. -- measured 12-16 % slower standalone: tools/patches/composite_variants.diff, profiles/r6b.)
template <int S>
__device__ __forceinline__ float composite_wave(int lane, int64_t b, int K, float far, const float (&zk)[S],
                                                const f4 (&v)[S], int white_bkgd, float *weights,
                                                float *rgb_out, float *depth_out, float (&wk)[S]) {
    double carry = 1.0;
    float sr = 0.f, sg = 0.f, sb = 0.f, sd = 0.f, sw = 0.f;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const int k = 64 * i + lane;
        const bool valid = k < K;
        // the next sample's depth: lane + 1 of this chunk, or lane 0 of the next one for lane 63
        const float nxt0 = i + 1 < S ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zk[i + 1 < S ? i + 1 : i]), 0))
                                     : far;
        // wave_shl:1, evaluated by every lane: inside the select below the compiler issues it
        // under a branch, and the lane before the last valid sample then reads a disabled lane
        const float zl = dpp_f<0x130>(nxt0, zk[i]);
        const float zn = k + 1 >= K ? far : zl;
        const float delta = sub_rn(zn, zk[i]);
        const float alpha = valid ? sub_rn(1.0f, expf(mul_rn(-delta, max_nc(v[i].w, 0.0f)))) : 0.0f;
        const float shifted = valid ? add_rn(sub_rn(1.0f, alpha), 1e-10f) : 1.0f;
        const double incl = wave_scan_mul((double)shifted);
        const double excl = wave_shr1(incl, 1.0);
        wk[i] = valid ? mul_rn(alpha, (float)(carry * excl)) : 0.f;
        const long long il = __double_as_longlong(incl);
        carry *= __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(il >> 32), 63) << 32) |
                                      (unsigned)__builtin_amdgcn_readlane((int)il, 63));
        if (weights && valid) __builtin_nontemporal_store(wk[i], weights + b * K + k);
        sr += mul_rn(wk[i], v[i].x);
        sg += mul_rn(wk[i], v[i].y);
        sb += mul_rn(wk[i], v[i].z);
        sd += mul_rn(wk[i], zk[i]);
        sw += wk[i];
    }
    sr = wave_sum_dpp(sr);
    sg = wave_sum_dpp(sg);
    sb = wave_sum_dpp(sb);
    sd = wave_sum_dpp(sd);
    sw = wave_sum_dpp(sw);
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
    return sd;
}

// ---- cross-lane helpers of the sort / scans (VALU only: DPP and gfx950 permlane swaps) -------
__device__ __forceinline__ double wave_scan_add(double x) {   // inclusive sum scan over 64 lanes
    x += dpp_d<0x111>(0.0, x);          // row_shr:1
    x += dpp_d<0x112>(0.0, x);          // row_shr:2
    x += dpp_d<0x114>(0.0, x);          // row_shr:4
    x += dpp_d<0x118>(0.0, x);          // row_shr:8
    x += dpp_d<0x142, 0xa>(0.0, x);     // row_bcast:15 -> rows 1, 3
    x += dpp_d<0x143, 0xc>(0.0, x);     // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)v, l), hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// value of lane ^ J.  ds_bpermute (__shfl_xor): a DPP / v_permlane{16,32}_swap version of this
// exchange measured wrong results once the epilogue was inlined inside k_point_mlp's GEMM
// region (deterministically; bit-exact elsewhere), so the sort keeps the LDS-crossbar permute.
template <int J>
__device__ __forceinline__ float lane_xor(float v, int lane) {
    (void)lane;
    return __shfl_xor(v, J, 64);
}
// one compare-exchange stage of a bitonic sort (element e of the sequence, merge size k)
template <int J>
__device__ __forceinline__ float bitonic_step(float v, int e, int k, int lane) {
    const float p = lane_xor<J>(v, lane);
    return ((e & J) == 0) == ((e & k) == 0) ? fminf(v, p) : fmaxf(v, p);
}
__device__ __forceinline__ float bitonic_step_j(float v, int e, int k, int j, int lane) {
    switch (j) {
    case 1: return bitonic_step<1>(v, e, k, lane);
    case 2: return bitonic_step<2>(v, e, k, lane);
    case 4: return bitonic_step<4>(v, e, k, lane);
    case 8: return bitonic_step<8>(v, e, k, lane);
    case 16: return bitonic_step<16>(v, e, k, lane);
    default: return bitonic_step<32>(v, e, k, lane);
    }
}
// ascending bitonic sort of the 64 N values held as v[h] = element 64 h + lane, in registers
template <int N>
__device__ __forceinline__ void sort_lanes(float (&v)[N], int lane) {
#pragma unroll
    for (int k = 2; k <= 64 * N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j == 64) {   // N == 2, k == 128: in-lane pair, ascending
                const float lo = fminf(v[0], v[N - 1]), hi = fmaxf(v[0], v[N - 1]);
                v[0] = lo;
                v[N - 1] = hi;
            } else {
#pragma unroll
                for (int h = 0; h < N; ++h) v[h] = bitonic_step_j(v[h], 64 * h + lane, k, j, lane);
            }
        }
    }
}

// ---- sample_fine + sample_fine_depth + sort — nerf.py:120-161, 284-295 ----------------------
// One wave per ray.  w / zc: the ray's kc coarse weights / depths (global or LDS);
// cdf (kc + 1) and s (n_sort, a power of two >= kc + kf) are LDS scratch private to the wave,
// si (n_sort ints) too when origin != NULL.  Writes the sorted kc + kf depths to z_fine (row
// of ray b), and with origin each value's index in cat(coarse, new) plus the new samples in
// draw order (z_new).  pre (kf <= 64): this lane's draws u_fine[j], u_jit[j], n_depth[j] for
// j = lane, made by the caller (fine_draws) ahead of its other work so their latency overlaps.
struct FineDraws {
    float u, uj, nd;
};
__device__ __forceinline__ FineDraws fine_draws(int lane, int64_t b, int kf, int kfd, const RngSrc &u_fine,
                                                const RngSrc &u_jit, const RngSrc &n_depth) {
    const int nf = kf - kfd;
    FineDraws d = {0.f, 0.f, 0.f};
    if (lane < nf) {
        d.u = rng_uniform(u_fine, b, nf, lane);
        d.uj = rng_uniform(u_jit, b, nf, lane);
    }
    if (lane < kfd) d.nd = rng_normal(n_depth, b, kfd, lane);
    return d;
}
__device__ __forceinline__ void sample_fine_wave(int lane, int64_t b, float near, float far, int kc,
                                                 const float *w, const float *zc, float depth_b, int kf, int kfd,
                                                 float depth_std, const RngSrc &u_fine, const RngSrc &u_jit,
                                                 const RngSrc &n_depth, bool lindisp, int n_sort, float *cdf,
                                                 float *s, int *si, float *z_fine, int *origin, float *z_new,
                                                 bool use_pre = false, FineDraws pre = {0.f, 0.f, 0.f},
                                                 float *z_lds = nullptr) {
    EPI_DECL
    // pdf = (w + 1e-5) / sum(w + 1e-5)   (nerf.py:130-131)
    float part = 0.0f;
    for (int k = lane; k < kc; k += 64) part += add_rn(w[k], 1e-5f);
    const float total = wave_sum_dpp(part);
    // cdf = [0, cumsum(pdf)]; torch's CPU cumsum accumulates in double (acc_type),
    // rounding every prefix to fp32 — a double wave scan reproduces those values.
    double carry = 0.0;
    if (lane == 0) cdf[0] = 0.0f;
    for (int c0 = 0; c0 < kc; c0 += 64) {
        const int k = c0 + lane;
        const double p = wave_scan_add((k < kc) ? (double)__fdiv_rn(add_rn(w[k], 1e-5f), total) : 0.0);
        if (k < kc) cdf[k + 1] = (float)(carry + p);
        carry += readlane_d(p, 63);
    }
    wave_lds_sync();
    EPI_T(1);

    const int nf = kf - kfd;
    const float inv_steps = (float)kc;
    // importance samples (nerf.py:135-148)
    for (int j = lane; j < nf; j += 64) {
        const float u = use_pre ? pre.u : rng_uniform(u_fine, b, nf, j);
        // searchsorted(cdf, u, right=True): number of cdf entries <= u
        int lo = 0, hi = kc + 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
        }
        float ind = fmaxf(sub_rn((float)lo, 1.0f), 0.0f);
        float t = __fdiv_rn(add_rn(ind, use_pre ? pre.uj : rng_uniform(u_jit, b, nf, j)), inv_steps);
        s[kc + j] = t_to_z(t, near, far, lindisp);
    }
    // depth samples (nerf.py:157-160): clamp(depth + N(0,1) * std, near, far)
    for (int j = lane; j < kfd; j += 64) {
        float zz = add_rn(depth_b, mul_rn(use_pre ? pre.nd : rng_normal(n_depth, b, kfd, j), depth_std));
        s[kc + nf + j] = fmaxf(fminf(zz, far), near);
    }
    for (int k = lane; k < kc; k += 64) s[k] = zc[k];
    for (int k = kc + kf + lane; k < n_sort; k += 64) s[k] = __builtin_inff();
    wave_lds_sync();
    EPI_T(2);
    if (origin) {   // the new samples in draw order, and every value's index in cat(coarse, new)
        for (int j = lane; j < kf; j += 64) z_new[b * kf + j] = s[kc + j];
        for (int k = lane; k < n_sort; k += 64) si[k] = k;
        wave_lds_sync();
    }
    const int k_all = kc + kf;
    // ascending sort (torch.sort, nerf.py:295): of <= 128 values in registers (no index to
    // carry), else a bitonic sort of n_sort values in LDS
    if (!origin && n_sort <= 128) {
        if (n_sort <= 64) {
            float v[1] = {s[lane < n_sort ? lane : 0]};
            if (lane >= n_sort) v[0] = __builtin_inff();
            sort_lanes<1>(v, lane);
            if (lane < k_all) {
                if (z_fine) z_fine[b * k_all + lane] = v[0];
                if (z_lds) z_lds[lane] = v[0];
            }
        } else {
            float v[2] = {s[lane], s[64 + lane]};
            sort_lanes<2>(v, lane);
            if (z_fine) {
                z_fine[b * k_all + lane] = v[0];
                if (64 + lane < k_all) z_fine[b * k_all + 64 + lane] = v[1];
            }
            if (z_lds) {
                z_lds[lane] = v[0];
                if (64 + lane < k_all) z_lds[64 + lane] = v[1];
            }
        }
        EPI_T(3);
        return;
    }
    for (int size = 2; size <= n_sort; size <<= 1) {
        for (int j = size >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < (n_sort >> 1); t += 64) {
                const int lo = 2 * j * (t / j) + (t % j);
                const int hi = lo + j;
                const bool asc = (lo & size) == 0;
                float a = s[lo], c = s[hi];
                if ((a > c) == asc) {
                    s[lo] = c; s[hi] = a;
                    if (origin) { const int t0 = si[lo]; si[lo] = si[hi]; si[hi] = t0; }
                }
            }
            wave_lds_sync();
        }
    }
    for (int k = lane; k < k_all; k += 64) {
        if (z_fine) z_fine[b * k_all + k] = s[k];
        if (z_lds) z_lds[k] = s[k];
    }
    if (origin)
        for (int k = lane; k < k_all; k += 64) origin[b * k_all + k] = si[k];
}

// Fused ray march (k_point_mlp render mode, pnr_render_forward_proj): what the epilogue of a
// ray's last tile does, and the prologue's coarse draws.  K = 64 kpt samples per ray, so a
// ray is kpt consecutive 64-point tiles.
struct MarchCfg {
    int kpt;                     // 1 or 2 tiles per ray
    int sample_coarse;           // draw z in the prologue (coarse_z) instead of reading zs
    int lindisp, white_bkgd;
    RngSrc u_coarse;
    float *z_out;                // sample_coarse: the drawn depths (n_rays, K)
    float *weights, *rgb, *depth;   // composite outputs (weights may be NULL)
    // fine sampling in the coarse epilogue (kf > 0; kc + kf <= 128, kc <= 64)
    int kf, kfd, n_sort;
    float depth_std;
    RngSrc u_fine, u_jit, n_depth;
    float *z_fine;               // (n_rays, kc + kf), sorted (may be NULL with `single`)
    // single-launch march (pnr march_mode 3): the ray's fine pass follows its coarse pass in the
    // same launch -- a scheduling unit is the ray's kpt coarse tiles, then its kpt_f fine tiles;
    // the coarse epilogue leaves the sorted fine depths in LDS for them
    int single, kpt_f;
    const float *packed_f, *proj_f;          // the fine MLP's pack and projected latent
    float *weights_f, *rgb_f, *depth_f;      // fine composite outputs (weights_f may be NULL)
    // processing order (pnr_render_cfg.ray_order): scheduling unit i marches ray order[i]; NULL =
    // unit i is ray i.  Draws and outputs use the ray's own index, so results do not depend on it.
    const int *order;
};
// LDS floats of the fused march region (k_point_mlp): the ray's z (128) | raw (128 x 4), the
// epilogue scratch w (128) | cdf (128) | sort (128), near / far (4), and with the single-launch
// march the fine pack's positional-encoding table (32: freqs | phases; the coarse pack's is the
// kernel's own table)
constexpr int MARCH_BUF_FLOATS = 640;
constexpr int MARCH_LDS_FLOATS = MARCH_BUF_FLOATS + 384 + 4 + 32;

}  // namespace pnr
