// Train-mode BatchNorm of the encoder trunk, fused with its ReLU and residual add (SURVEY §8(f)
// rank 3: the latent producer on the training step; BASELINE cfg5).
//
// The reference trains the ResNet34 trunk with nn.BatchNorm2d on batch statistics
// (encoder.py:135-149, torchvision BasicBlock: relu(bn1(conv1 x)), relu(bn2(conv2 h) + idt), the
// downsample's bn without relu).  MIOpen runs each as three kernels (mean/variance partials, their
// final reduction, the normalisation) plus torch's relu, residual add and num_batches_tracked
// increment -- ~7 launches of 2-5 us on 4 x 64 x 64 .. 4 x 8 x 8 maps, forward and backward alike.
// Here one BatchNorm(+add)(+relu) is two launches each way, on channels-last (NHWC) fp32 maps viewed
// as (M = N H W) x C:
//   k_bn_stats      per row block: sum y and sum y^2 per channel (double) into its partial slot; the
//                   last block to finish (a device-scope arrival counter, write-through partials,
//                   no fences) reduces the partials in
//                   block order -- mean, biased variance, invstd = 1 / sqrt(var + eps), the running
//                   statistics (momentum, unbiased variance) and num_batches_tracked, as torch --
//                   and re-arms the counter;
//   k_bn_apply      out = [relu](((y - mean) invstd) gamma + beta [+ idt]);
//   k_bnb_stats     per row block: sum dz and sum dz x_hat, dz = dout [out > 0], x_hat = (y - mean)
//                   invstd; the last block: d gamma, d beta and the dy coefficients;
//   k_bnb_apply     dy = gamma invstd (dz - d_beta / M - x_hat d_gamma / M); d idt = dz.
// Every reduction runs in double in a fixed order (deterministic; torch's BatchNorm reduces in fp32):
// the result agrees with torch to fp32 rounding (tests/test_gpu_batchnorm.py).
// Workspace: 256 B of arrival counters (zero before the first call, left zero by every call), the
// double partials of ceil(M / 128) row blocks, 3 C floats of backward coefficients.
#include "pnr_common.h"

namespace pnr {
namespace bnk {

constexpr int NTHR = 256;
constexpr int ROWS = 128;   // rows of one partial block

constexpr size_t COUNTER_BYTES = 256;

// The cross-block hand-off of the column sums without fences (MI355X_MICROARCH.md, the valid
// forms of an in-launch hand-off): every partial is stored write-through (an agent-scope relaxed
// 8-B store: global_store sc1), every storing wave drains its stores (vmcnt 0) before the block's
// barrier, ONE lane then adds to the arrival counter (agent scope), the block whose add returns
// nb - 1 is last, and it reads the partials with agent-scope relaxed loads (global_load sc1).  An
// agent-scope __threadfence costs ~3.5 us per block; two of them made these launches slower than
// MIOpen's (profiles/r5j).
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void st_wt(double *p, double v) {
    __hip_atomic_store((gu64 *)(p), (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double *p) {
    return __longlong_as_double((long long)__hip_atomic_load((gu64 *)(const_cast<double *>(p)),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Column sums of a (M x C) block of rows: thread t owns channel group g = t % G (4 channels) and
// row slot r = t / G of R = NTHR / G; the slots combine in slot order (deterministic).  Writes the
// block's [sum a | sum b] (2 C doubles) to its partial slot, write-through.
__device__ __forceinline__ void store_block_partial(const double (&s)[4], const double (&q)[4], int C,
                                                    double *red, double *p) {
    const int G = C >> 2, R = NTHR / G, t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[t * 8 + e] = s[e];
        red[t * 8 + 4 + e] = q[e];
    }
    __syncthreads();
    if (t < G) {
        for (int rr = 1; rr < R; ++rr)
#pragma unroll
            for (int e = 0; e < 8; ++e) red[t * 8 + e] += red[(rr * G + t) * 8 + e];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            st_wt(p + 4 * t + e, red[t * 8 + e]);
            st_wt(p + C + 4 * t + e, red[t * 8 + 4 + e]);
        }
    }
}

// Arrival: true in the block that finishes last (it then reads every block's partial slot with ld_wt).
__device__ __forceinline__ bool last_block(unsigned *counter, int nb) {
    __shared__ int is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through partial stores done
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add((gu32 *)(counter), 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == (unsigned)(nb - 1);
        if (is_last) __hip_atomic_store((gu32 *)(counter), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return is_last != 0;
}

// Channel totals over the nb partial slots, in slot order within J = NTHR / C interleaved slices
// (C <= 256) combined in slice order; channels beyond NTHR loop.  Calls fin(c, sum_a, sum_b).
template <class Fin>
__device__ __forceinline__ void reduce_partials(const double *part, int nb, int C, double *red, Fin fin) {
    const int t = threadIdx.x;
    if (C <= NTHR) {
        const int J = NTHR / C, c = t % C, j = t / C;
        double s = 0.0, q = 0.0;
        for (int b = j; b < nb; b += J) {
            s += ld_wt(part + (int64_t)b * 2 * C + c);
            q += ld_wt(part + (int64_t)b * 2 * C + C + c);
        }
        __syncthreads();   // red reused
        red[2 * t] = s;
        red[2 * t + 1] = q;
        __syncthreads();
        if (t < C) {
            for (int jj = 1; jj < J; ++jj) {
                s += red[2 * (jj * C + t)];
                q += red[2 * (jj * C + t) + 1];
            }
            fin(t, s, q);
        }
    } else {
        for (int c = t; c < C; c += NTHR) {
            double s = 0.0, q = 0.0;
            for (int b = 0; b < nb; ++b) {
                s += ld_wt(part + (int64_t)b * 2 * C + c);
                q += ld_wt(part + (int64_t)b * 2 * C + C + c);
            }
            fin(c, s, q);
        }
    }
}

__global__ __launch_bounds__(NTHR) void k_bn_stats(const float *__restrict__ y, int64_t M, int C, float momentum,
                                                   float eps, float *__restrict__ running_mean,
                                                   float *__restrict__ running_var, int64_t *__restrict__ num_batches,
                                                   float *__restrict__ stats, unsigned *counter,
                                                   double *__restrict__ part) {
    __shared__ double red[NTHR * 8];
    const int G = C >> 2, R = NTHR / G;
    const int t = threadIdx.x, g = t % G, r = t / G;
    const int64_t m0 = (int64_t)blockIdx.x * ROWS;
    const int nb = gridDim.x;
    double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
    for (int64_t m = m0 + r; m < m0 + ROWS && m < M; m += R) {
        const f4 v = *reinterpret_cast<const f4 *>(y + m * C + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            s[e] += (double)v[e];
            q[e] += (double)v[e] * (double)v[e];
        }
    }
    store_block_partial(s, q, C, red, part + (int64_t)blockIdx.x * 2 * C);
    if (!last_block(counter, nb)) return;
    if (t == 0 && num_batches) num_batches[0] += 1;
    reduce_partials(part, nb, C, red, [&](int c, double sum, double sq) {
        const double mean = sum / (double)M;
        double var = sq / (double)M - mean * mean;
        if (var < 0.0) var = 0.0;
        const float meanf = (float)mean;
        stats[c] = meanf;
        stats[C + c] = (float)(1.0 / sqrt(var + (double)eps));
        if (running_mean) {
            const float unbiased = (float)(M > 1 ? var * (double)M / (double)(M - 1) : var);
            running_mean[c] = add_rn(mul_rn(1.f - momentum, running_mean[c]), mul_rn(momentum, meanf));
            running_var[c] = add_rn(mul_rn(1.f - momentum, running_var[c]), mul_rn(momentum, unbiased));
        }
    });
}

template <bool RELU, bool ADD>
__global__ __launch_bounds__(NTHR) void k_bn_apply(const float *__restrict__ y, const float *__restrict__ idt,
                                                   const float *__restrict__ gamma, const float *__restrict__ beta,
                                                   const float *__restrict__ stats, int64_t n4, int C,
                                                   float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * NTHR + threadIdx.x;
    if (i >= n4) return;
    const int c0 = (int)((i * 4) % C);
    const f4 v = reinterpret_cast<const f4 *>(y)[i];
    f4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int c = c0 + e;
        const float xh = mul_rn(sub_rn(v[e], stats[c]), stats[C + c]);
        o[e] = add_rn(mul_rn(xh, gamma[c]), beta[c]);
    }
    if (ADD) o += reinterpret_cast<const f4 *>(idt)[i];
    if (RELU) o = relu4(o);
    reinterpret_cast<f4 *>(out)[i] = o;
}

// coef [3][C]: gamma invstd, d_beta / M, d_gamma / M
template <bool RELU>
__global__ __launch_bounds__(NTHR) void k_bnb_stats(const float *__restrict__ y, const float *__restrict__ out,
                                                    const float *__restrict__ dout, const float *__restrict__ gamma,
                                                    const float *__restrict__ stats, int64_t M, int C,
                                                    float *__restrict__ dgamma, float *__restrict__ dbeta,
                                                    float *__restrict__ coef, unsigned *counter,
                                                    double *__restrict__ part) {
    __shared__ double red[NTHR * 8];
    const int G = C >> 2, R = NTHR / G;
    const int t = threadIdx.x, g = t % G, r = t / G;
    const int64_t m0 = (int64_t)blockIdx.x * ROWS;
    const int nb = gridDim.x;
    double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
    f4 mu, is;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        mu[e] = stats[4 * g + e];
        is[e] = stats[C + 4 * g + e];
    }
    for (int64_t m = m0 + r; m < m0 + ROWS && m < M; m += R) {
        const f4 yv = *reinterpret_cast<const f4 *>(y + m * C + 4 * g);
        f4 dz = *reinterpret_cast<const f4 *>(dout + m * C + 4 * g);
        if (RELU) {
            const f4 ov = *reinterpret_cast<const f4 *>(out + m * C + 4 * g);
#pragma unroll
            for (int e = 0; e < 4; ++e) dz[e] = ov[e] > 0.f ? dz[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float xh = mul_rn(sub_rn(yv[e], mu[e]), is[e]);
            s[e] += (double)dz[e];
            q[e] += (double)dz[e] * (double)xh;
        }
    }
    store_block_partial(s, q, C, red, part + (int64_t)blockIdx.x * 2 * C);
    if (!last_block(counter, nb)) return;
    reduce_partials(part, nb, C, red, [&](int c, double sum, double sxh) {
        if (dbeta) dbeta[c] = (float)sum;
        if (dgamma) dgamma[c] = (float)sxh;
        coef[c] = mul_rn(gamma[c], stats[C + c]);
        coef[C + c] = (float)(sum / (double)M);
        coef[2 * C + c] = (float)(sxh / (double)M);
    });
}

template <bool RELU, bool DIDT>
__global__ __launch_bounds__(NTHR) void k_bnb_apply(const float *__restrict__ y, const float *__restrict__ out,
                                                    const float *__restrict__ dout,
                                                    const float *__restrict__ stats,
                                                    const float *__restrict__ coef, int64_t n4, int C,
                                                    float *__restrict__ dy, float *__restrict__ didt) {
    const int64_t i = (int64_t)blockIdx.x * NTHR + threadIdx.x;
    if (i >= n4) return;
    const int c0 = (int)((i * 4) % C);
    const f4 yv = reinterpret_cast<const f4 *>(y)[i];
    f4 dz = reinterpret_cast<const f4 *>(dout)[i];
    if (RELU) {
        const f4 ov = reinterpret_cast<const f4 *>(out)[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) dz[e] = ov[e] > 0.f ? dz[e] : 0.f;
    }
    f4 g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int c = c0 + e;
        const float xh = mul_rn(sub_rn(yv[e], stats[c]), stats[C + c]);
        g[e] = mul_rn(coef[c], sub_rn(sub_rn(dz[e], coef[C + c]), mul_rn(xh, coef[2 * C + c])));
    }
    reinterpret_cast<f4 *>(dy)[i] = g;
    if (DIDT) reinterpret_cast<f4 *>(didt)[i] = dz;
}

}  // namespace bnk

size_t bn_workspace_bytes(int64_t M, int C) {
    const int64_t nb = (M + bnk::ROWS - 1) / bnk::ROWS;
    return bnk::COUNTER_BYTES + sizeof(double) * (size_t)(nb * 2 * C) + sizeof(float) * (size_t)(3 * C);
}

static int bn_check(int64_t M, int C, const void *ws, size_t ws_bytes) {
    if (M < 1 || C < 4 || C > 1024 || (C & 3) != 0 || (bnk::NTHR % (C >> 2)) != 0)
        return fail(PNR_ERR_UNSUPPORTED, "batchnorm: C must be a multiple of 4 dividing 1024 (got %d), M >= 1", C);
    if ((M + bnk::ROWS - 1) / bnk::ROWS > (1 << 30))
        return fail(PNR_ERR_UNSUPPORTED, "batchnorm: M = %lld rows too large", (long long)M);
    if (!ws || ws_bytes < bn_workspace_bytes(M, C))
        return fail(PNR_ERR_WORKSPACE, "batchnorm: workspace %zu < %zu", ws_bytes, bn_workspace_bytes(M, C));
    if ((reinterpret_cast<uintptr_t>(ws) & 255) != 0)
        return fail(PNR_ERR_INVALID, "batchnorm: workspace must be 256-byte aligned");
    return PNR_OK;
}

int launch_bn_forward(const float *y, const float *idt, const float *gamma, const float *beta, float *running_mean,
                      float *running_var, int64_t *num_batches, int64_t M, int C, float momentum, float eps, int relu,
                      float *out, float *stats, void *ws, size_t ws_bytes, hipStream_t st) {
    const int rc = bn_check(M, C, ws, ws_bytes);
    if (rc != PNR_OK) return rc;
    const int nb = (int)((M + bnk::ROWS - 1) / bnk::ROWS);
    unsigned *counter = static_cast<unsigned *>(ws);
    double *part = reinterpret_cast<double *>(static_cast<char *>(ws) + bnk::COUNTER_BYTES);
    hipLaunchKernelGGL(bnk::k_bn_stats, dim3(nb), dim3(bnk::NTHR), 0, st, y, M, C, momentum, eps, running_mean,
                       running_var, num_batches, stats, counter, part);
    const int64_t n4 = M * C / 4;
    const dim3 grid((unsigned)((n4 + bnk::NTHR - 1) / bnk::NTHR));
    if (relu && idt) hipLaunchKernelGGL((bnk::k_bn_apply<true, true>), grid, dim3(bnk::NTHR), 0, st, y, idt, gamma, beta, stats, n4, C, out);
    else if (relu) hipLaunchKernelGGL((bnk::k_bn_apply<true, false>), grid, dim3(bnk::NTHR), 0, st, y, idt, gamma, beta, stats, n4, C, out);
    else if (idt) hipLaunchKernelGGL((bnk::k_bn_apply<false, true>), grid, dim3(bnk::NTHR), 0, st, y, idt, gamma, beta, stats, n4, C, out);
    else hipLaunchKernelGGL((bnk::k_bn_apply<false, false>), grid, dim3(bnk::NTHR), 0, st, y, idt, gamma, beta, stats, n4, C, out);
    return launch_ok("bn_forward") ? PNR_OK : PNR_ERR_HIP;
}

int launch_bn_backward(const float *y, const float *out, const float *dout, const float *gamma, const float *stats,
                       int64_t M, int C, int relu, float *dy, float *didt, float *dgamma, float *dbeta, void *ws,
                       size_t ws_bytes, hipStream_t st) {
    const int rc = bn_check(M, C, ws, ws_bytes);
    if (rc != PNR_OK) return rc;
    const int nb = (int)((M + bnk::ROWS - 1) / bnk::ROWS);
    unsigned *counter = static_cast<unsigned *>(ws) + 1;
    double *part = reinterpret_cast<double *>(static_cast<char *>(ws) + bnk::COUNTER_BYTES);
    float *coef = reinterpret_cast<float *>(part + (size_t)nb * 2 * C);
    if (relu) hipLaunchKernelGGL(bnk::k_bnb_stats<true>, dim3(nb), dim3(bnk::NTHR), 0, st, y, out, dout, gamma, stats, M, C, dgamma, dbeta, coef, counter, part);
    else hipLaunchKernelGGL(bnk::k_bnb_stats<false>, dim3(nb), dim3(bnk::NTHR), 0, st, y, out, dout, gamma, stats, M, C, dgamma, dbeta, coef, counter, part);
    const int64_t n4 = M * C / 4;
    const dim3 grid((unsigned)((n4 + bnk::NTHR - 1) / bnk::NTHR));
    if (relu && didt) hipLaunchKernelGGL((bnk::k_bnb_apply<true, true>), grid, dim3(bnk::NTHR), 0, st, y, out, dout, stats, coef, n4, C, dy, didt);
    else if (relu) hipLaunchKernelGGL((bnk::k_bnb_apply<true, false>), grid, dim3(bnk::NTHR), 0, st, y, out, dout, stats, coef, n4, C, dy, didt);
    else if (didt) hipLaunchKernelGGL((bnk::k_bnb_apply<false, true>), grid, dim3(bnk::NTHR), 0, st, y, out, dout, stats, coef, n4, C, dy, didt);
    else hipLaunchKernelGGL((bnk::k_bnb_apply<false, false>), grid, dim3(bnk::NTHR), 0, st, y, out, dout, stats, coef, n4, C, dy, didt);
    return launch_ok("bn_backward") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
