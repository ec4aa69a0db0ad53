// Projected latent: the lin_z layers of ResnetFC applied to every latent PIXEL once per
// (scene, weight version) instead of to every sampled POINT.
//
// The reference computes, per point and per block b < combine_layer (resnetfc.py:160-163),
//     x += lin_z[b](z),   z = grid_sample(latent, uv)   (bilinear, encoder.py:102-108)
// grid_sample's output is a fixed blend of four latent pixels, z = sum_c w_c L_c, and lin_z
// is linear, so  lin_z[b](z) = sum_c w_c (W_b L_c) + bias_b.  k_latent_proj computes
// P_b = L W_b^T for all H_l x W_l pixels of every source view; k_point_mlp<PREC, true> then
// blends four rows of P_b per point (gather_proj) instead of running the 512 x 512 lin_z
// GEMM per point.  For SRN (64 x 64 latent) that is 3 x 4096 pixel rows per scene against
// 3 x 786,432 point rows per 4096-ray chunk (192 points per ray).
//
// The GEMM: P[layer][pixel][o] = sum_k L[pixel][k] W_layer[o][k] on v_mfma_f32_16x16x4_f32
// (fp32 products, fp32 accumulation).  Workgroup = 4 waves = a 64-pixel x 64-output tile;
// k in chunks of 32 through padded LDS tiles (pitch 33: conflict-free column reads), the
// next chunk's global loads in flight while the current one is multiplied.
#include "pnr_common.h"

namespace pnr {
namespace projk {

constexpr int C = 512;                 // latent channels = hidden width
constexpr int TM = 64, TN = 64, TK = 32, TP = TK + 1;

struct ProjW {
    const float *w[8];                 // lin_z[b].weight (512 out x 512 in), torch layout
};

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void k_latent_proj(const float *__restrict__ lat, int64_t n_pix, ProjW pw,
                                                     float *__restrict__ out, int64_t layer_stride) {
    __shared__ float As[TM * TP], Bs[TN * TP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float *__restrict__ W = pw.w[blockIdx.z];
    const int64_t m0 = (int64_t)blockIdx.x * TM;
    const int n0 = blockIdx.y * TN;
    // loader: thread -> row tid / 4, 8 consecutive k at 8 (tid % 4)
    const int lr = tid >> 2, lk = (tid & 3) * 8;
    const int64_t am = m0 + lr < n_pix ? m0 + lr : n_pix - 1;   // clamped rows are never stored
    const float *ap = lat + am * C + lk;
    const float *bp = W + (int64_t)(n0 + lr) * C + lk;
    f4 a0 = *reinterpret_cast<const f4 *>(ap), a1 = *reinterpret_cast<const f4 *>(ap + 4);
    f4 b0 = *reinterpret_cast<const f4 *>(bp), b1 = *reinterpret_cast<const f4 *>(bp + 4);
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    const int li = lane & 15, lkk = lane >> 4;
    f4 acc[2][2] = {};
    for (int kc = 0; kc < C; kc += TK) {
        __syncthreads();   // previous chunk consumed
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            As[lr * TP + lk + q] = a0[q];
            As[lr * TP + lk + 4 + q] = a1[q];
            Bs[lr * TP + lk + q] = b0[q];
            Bs[lr * TP + lk + 4 + q] = b1[q];
        }
        __syncthreads();
        if (kc + TK < C) {
            a0 = *reinterpret_cast<const f4 *>(ap + kc + TK);
            a1 = *reinterpret_cast<const f4 *>(ap + kc + TK + 4);
            b0 = *reinterpret_cast<const f4 *>(bp + kc + TK);
            b1 = *reinterpret_cast<const f4 *>(bp + kc + TK + 4);
        }
#pragma unroll
        for (int kk = 0; kk < TK; kk += 4) {
            float av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                av[i] = As[(wm + 16 * i + li) * TP + kk + lkk];
                bv[i] = Bs[(wn + 16 * i + li) * TP + kk + lkk];
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma(av[i], bv[j], acc[i][j]);
        }
    }
    // lane: output column n = wn + 16 j + (lane & 15), rows m = wm + 16 i + 4 (lane >> 4) + e
    float *o = out + (int64_t)blockIdx.z * layer_stride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t m = m0 + wm + 16 * i + 4 * lkk + e;
            if (m >= n_pix) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j) o[m * C + n0 + wn + 16 * j + li] = acc[i][j][e];
        }
}

}  // namespace projk

int64_t latent_proj_floats(const pnr_scene &sc, const pnr_mlp_desc &d) {
    const int64_t n_linz = d.combine_layer < d.n_blocks ? d.combine_layer : d.n_blocks;
    return n_linz * (int64_t)sc.n_obj * sc.n_views * sc.latent_h * sc.latent_w * sc.latent_c;
}

int launch_latent_proj(const pnr_scene &sc, const pnr_mlp_weights &w, float *proj, size_t bytes, hipStream_t st) {
    const pnr_mlp_desc &d = w.desc;
    const int n_linz = d.combine_layer < d.n_blocks ? d.combine_layer : d.n_blocks;
    if (sc.latent_c != projk::C || d.d_latent != projk::C || d.d_hidden != projk::C)
        return fail(PNR_ERR_UNSUPPORTED, "latent projection implements latent_c = d_latent = d_hidden = 512");
    if (n_linz > 8) return fail(PNR_ERR_UNSUPPORTED, "latent projection: at most 8 lin_z layers");
    const int64_t need = latent_proj_floats(sc, d);
    if (bytes < sizeof(float) * (size_t)need) return fail(PNR_ERR_WORKSPACE, "latent projection buffer too small");
    if (n_linz == 0) return PNR_OK;
    projk::ProjW pw = {};
    for (int b = 0; b < n_linz; ++b) {
        if (!w.lin_z_w[b]) return fail(PNR_ERR_INVALID, "lin_z_w[%d] is NULL", b);
        if ((reinterpret_cast<uintptr_t>(w.lin_z_w[b]) & 15) != 0)
            return fail(PNR_ERR_INVALID, "lin_z_w[%d] must be 16-byte aligned", b);
        pw.w[b] = w.lin_z_w[b];
    }
    const int64_t n_pix = (int64_t)sc.n_obj * sc.n_views * sc.latent_h * sc.latent_w;
    const int64_t layer_stride = n_pix * projk::C;
    const dim3 grid((unsigned)((n_pix + projk::TM - 1) / projk::TM), projk::C / projk::TN, (unsigned)n_linz);
    hipLaunchKernelGGL(projk::k_latent_proj, grid, dim3(256), 0, st, sc.latent, n_pix, pw, proj, layer_stride);
    return launch_ok("latent_proj") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
