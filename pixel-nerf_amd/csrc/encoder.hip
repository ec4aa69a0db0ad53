// Encoder latent producer, channels-last.
//
// Replaces the tail of SpatialEncoder.forward (encoder.py:150-160): every trunk
// feature map (conv1, layer1..layer3, NCHW) is bilinearly upsampled to the first map's
// size (align_corners = True) and concatenated along channels.  The ray march consumes
// the latent channels-LAST, so this kernel writes (N, H_l, W_l, sum C) directly: no
// NCHW concat and no transpose copy.  The maps may also be channels-last (NHWC) themselves,
// the trunk's layout when its convolutions run in channels-last memory format: consecutive
// threads then read consecutive channels of one source pixel.  Arithmetic as torch's CPU upsample_bilinear2d:
//   scale = (in - 1) / (out - 1) (float), src = scale * dst, i0 = (int) src,
//   l1 = src - i0, l0 = 1 - l1, i1 = i0 + (i0 < in - 1),
//   out = l0h (l0w v00 + l1w v01) + l1h (l0w v10 + l1w v11)
#include "pnr_common.h"

namespace pnr {

constexpr int MAX_MAPS = 8;

struct LatentMaps {
    const float *ptr[MAX_MAPS];
    int c0[MAX_MAPS + 1];   // channel offset of each map in the output (c0[n_maps] = total)
    int h[MAX_MAPS], w[MAX_MAPS];
    int n_maps;
};

__device__ __forceinline__ void src_index(int in, int out, int dst, int &i0, int &i1, float &l0, float &l1) {
    const float scale = out > 1 ? __fdiv_rn((float)(in - 1), (float)(out - 1)) : 0.f;
    const float real = mul_rn(scale, (float)dst);
    i0 = (int)real;
    i1 = i0 + (i0 < in - 1 ? 1 : 0);
    l1 = sub_rn(real, (float)i0);
    l0 = sub_rn(1.f, l1);
}

template <bool NHWC>
__global__ __launch_bounds__(256) void k_latent_cl(LatentMaps m, int64_t n_out, int out_h, int out_w,
                                                   float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_out) return;
    const int C = m.c0[m.n_maps];
    const int c = (int)(i % C);
    const int64_t pix = i / C;
    const int x = (int)(pix % out_w);
    const int64_t t = pix / out_w;
    const int y = (int)(t % out_h);
    const int64_t n = t / out_h;
    int k = 0;
#pragma unroll
    for (int j = 1; j < MAX_MAPS; ++j)
        if (j < m.n_maps && c >= m.c0[j]) k = j;
    const int cc = c - m.c0[k], hm = m.h[k], wm = m.w[k];
    const int cm = m.c0[k + 1] - m.c0[k];
    // element (y, x) of this channel: NCHW plane pitch 1, NHWC pixel pitch cm
    const float *src = NHWC ? m.ptr[k] + n * (int64_t)hm * wm * cm + cc : m.ptr[k] + ((n * cm + cc) * (int64_t)hm) * wm;
    const int64_t px = NHWC ? cm : 1;
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    src_index(hm, out_h, y, y0, y1, ly0, ly1);
    src_index(wm, out_w, x, x0, x1, lx0, lx1);
    const float v00 = src[((int64_t)y0 * wm + x0) * px], v01 = src[((int64_t)y0 * wm + x1) * px];
    const float v10 = src[((int64_t)y1 * wm + x0) * px], v11 = src[((int64_t)y1 * wm + x1) * px];
    const float top = add_rn(mul_rn(lx0, v00), mul_rn(lx1, v01));
    const float bot = add_rn(mul_rn(lx0, v10), mul_rn(lx1, v11));
    out[i] = add_rn(mul_rn(ly0, top), mul_rn(ly1, bot));
}

int launch_latent_cl(const float *const *maps, const int32_t *channels, const int32_t *heights,
                     const int32_t *widths, int n_maps, int n_images, float *latent_cl, int out_h, int out_w,
                     bool nhwc, hipStream_t st) {
    if (n_maps < 1 || n_maps > MAX_MAPS) return fail(PNR_ERR_UNSUPPORTED, "latent: 1..8 feature maps");
    LatentMaps m = {};
    m.n_maps = n_maps;
    m.c0[0] = 0;
    for (int k = 0; k < n_maps; ++k) {
        if (!maps[k] || channels[k] < 1 || heights[k] < 1 || widths[k] < 1)
            return fail(PNR_ERR_INVALID, "latent: bad feature map %d", k);
        m.ptr[k] = maps[k];
        m.h[k] = heights[k];
        m.w[k] = widths[k];
        m.c0[k + 1] = m.c0[k] + channels[k];
    }
    const int64_t n_out = (int64_t)n_images * out_h * out_w * m.c0[n_maps];
    if (n_out == 0) return PNR_OK;
    const dim3 grid((unsigned)((n_out + 255) / 256));
    if (nhwc) hipLaunchKernelGGL(k_latent_cl<true>, grid, dim3(256), 0, st, m, n_out, out_h, out_w, latent_cl);
    else hipLaunchKernelGGL(k_latent_cl<false>, grid, dim3(256), 0, st, m, n_out, out_h, out_w, latent_cl);
    return launch_ok("latent_cl") ? PNR_OK : PNR_ERR_HIP;
}

// Adjoint of k_latent_cl for channels-last maps (the training encode's backward, LatentChannelsLast):
// d map_k (n, ys, xs, c) = sum over the output pixels (y, x) whose bilinear taps include (ys, xs) of
// tap weight (y) x tap weight (x) x g(n, y, x, c0_k + c), gathered per source element -- no atomics,
// a fixed summation order (rows then columns ascending), so the result is deterministic; torch's
// upsample_bilinear2d_backward scatters with atomics.  One thread per source element, consecutive
// threads on consecutive channels (coalesced rows of g); a map at the output size is a slice copy.
__device__ __forceinline__ void tap_range(int in, int out, int s, int &lo, int &hi) {
    if (out <= 1 || in <= 1) {   // scale 0: every output pixel reads source 0
        lo = 0;
        hi = s == 0 ? out - 1 : -1;
        return;
    }
    const float scale = __fdiv_rn((float)(in - 1), (float)(out - 1));
    lo = (int)floorf((float)(s - 1) / scale) - 1;
    hi = (int)ceilf((float)(s + 1) / scale) + 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > out - 1 ? out - 1 : hi;
}

struct LatentGrads {
    float *ptr[MAX_MAPS];
    int64_t off[MAX_MAPS + 1];   // first thread of each map (off[n_maps] = all source elements)
    int c0[MAX_MAPS + 1];
    int h[MAX_MAPS], w[MAX_MAPS];
    int n_maps;
};

__global__ __launch_bounds__(256) void k_latent_cl_bwd(LatentGrads m, int out_h, int out_w,
                                                       const float *__restrict__ g) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= m.off[m.n_maps]) return;
    int k = 0;
#pragma unroll
    for (int j = 1; j < MAX_MAPS; ++j)
        if (j < m.n_maps && tid >= m.off[j]) k = j;
    const int64_t i = tid - m.off[k];
    const int C = m.c0[m.n_maps], cm = m.c0[k + 1] - m.c0[k], hm = m.h[k], wm = m.w[k];
    const int c = (int)(i % cm);
    const int64_t pix = i / cm;
    const int xs = (int)(pix % wm);
    const int64_t t = pix / wm;
    const int ys = (int)(t % hm);
    const int64_t n = t / hm;
    const float *gn = g + n * (int64_t)out_h * out_w * C + m.c0[k] + c;
    float *d = m.ptr[k];
    if (hm == out_h && wm == out_w) {   // scale 1: the identity taps
        d[i] = gn[((int64_t)ys * out_w + xs) * C];
        return;
    }
    int ylo, yhi, xlo, xhi;
    tap_range(hm, out_h, ys, ylo, yhi);
    tap_range(wm, out_w, xs, xlo, xhi);
    float acc = 0.f;
    for (int y = ylo; y <= yhi; ++y) {
        int y0, y1;
        float ly0, ly1;
        src_index(hm, out_h, y, y0, y1, ly0, ly1);
        if (y0 != ys && y1 != ys) continue;
        const float wy = (y0 == ys ? ly0 : 0.f) + (y1 == ys ? ly1 : 0.f);
        float row = 0.f;
        for (int x = xlo; x <= xhi; ++x) {
            int x0, x1;
            float lx0, lx1;
            src_index(wm, out_w, x, x0, x1, lx0, lx1);
            if (x0 != xs && x1 != xs) continue;
            const float wx = (x0 == xs ? lx0 : 0.f) + (x1 == xs ? lx1 : 0.f);
            row += wx * gn[((int64_t)y * out_w + x) * C];
        }
        acc += wy * row;
    }
    d[i] = acc;
}

int launch_latent_cl_bwd(const float *g, float *const *d_maps, const int32_t *channels, const int32_t *heights,
                         const int32_t *widths, int n_maps, int n_images, int out_h, int out_w, hipStream_t st) {
    if (n_maps < 1 || n_maps > MAX_MAPS) return fail(PNR_ERR_UNSUPPORTED, "latent backward: 1..8 feature maps");
    if (!g || out_h < 1 || out_w < 1 || n_images < 0) return fail(PNR_ERR_INVALID, "latent backward: bad output");
    LatentGrads m = {};
    m.n_maps = n_maps;
    for (int k = 0; k < n_maps; ++k) {
        if (!d_maps[k] || channels[k] < 1 || heights[k] < 1 || widths[k] < 1 || heights[k] > out_h ||
            widths[k] > out_w)
            return fail(PNR_ERR_INVALID, "latent backward: bad feature map %d", k);
        m.ptr[k] = d_maps[k];
        m.h[k] = heights[k];
        m.w[k] = widths[k];
        m.c0[k + 1] = m.c0[k] + channels[k];
        m.off[k + 1] = m.off[k] + (int64_t)n_images * heights[k] * widths[k] * channels[k];
    }
    if (m.off[n_maps] == 0) return PNR_OK;
    hipLaunchKernelGGL(k_latent_cl_bwd, dim3((unsigned)((m.off[n_maps] + 255) / 256)), dim3(256), 0, st, m, out_h,
                       out_w, g);
    return launch_ok("latent_cl_bwd") ? PNR_OK : PNR_ERR_HIP;
}

// BatchNorm folded into the convolution before it, for the eval-mode trunk (pnr.encoder.InferenceTrunk):
// W'[o, :] = W[o, :] s[o], b'[o] = beta[o] - mean[o] s[o], s = gamma / sqrt(var + eps) (gamma 1 and
// beta 0 when the BatchNorm has no affine parameters).  One launch folds every (conv, bn) pair of
// the trunk from their live storage (blockIdx.y = pair), so the HIP graph that replays the trunk
// refolds on every replay and in-place edits of any weight or statistic are always seen.
__global__ __launch_bounds__(256) void k_fold_bn(const pnr_bn_fold *__restrict__ folds) {
    const pnr_bn_fold f = folds[blockIdx.y];
    const int64_t n = f.n_out * f.per_out;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = e / f.per_out;
        const float inv = __fdiv_rn(1.f, __fsqrt_rn(add_rn(f.var[o], f.eps)));
        const float s = f.gamma ? mul_rn(f.gamma[o], inv) : inv;
        f.w_out[e] = mul_rn(f.conv_w[e], s);
        if (e - o * f.per_out == 0) {
            const float beta = f.beta ? f.beta[o] : 0.f;
            f.b_out[o] = sub_rn(beta, mul_rn(f.mean[o], s));
        }
    }
}

int launch_fold_bn(const pnr_bn_fold *folds, int n_folds, int64_t max_elems, hipStream_t st) {
    if (n_folds == 0 || max_elems == 0) return PNR_OK;
    const int64_t blocks = (max_elems + 255) / 256;
    const dim3 grid((unsigned)(blocks < 256 ? blocks : 256), (unsigned)n_folds);
    hipLaunchKernelGGL(k_fold_bn, grid, dim3(256), 0, st, folds);
    return launch_ok("fold_bn") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
