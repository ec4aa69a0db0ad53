// Adam parameter update of the training step (BASELINE cfg5: the reference's
// train.py steps torch.optim.Adam after every backward).
//
// torch's fused Adam runs as one multi-tensor kernel per ~100 tensors plus a step-counter kernel
// (5 launches and 0.24 ms per cfg5 step, profiles/r5final/train_step_breakdown.txt) over ~15 M
// parameters = 0.42 GB of parameter, gradient and moment traffic.  Here: ONE launch over a device
// table of chunks (a chunk = up to ADAM_CHUNK consecutive elements of one tensor), one workgroup
// per chunk, 16-B accesses where the chunk is 16-B aligned.  Per element, in fp32, in torch's
// order (FusedAdamKernel / _single_tensor_adam):
//   g += wd p (weight_decay != 0);  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;
//   p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps),  bc_i = 1 - b_i^step (host, per step).
// Against torch.optim.Adam within fp32 rounding (tests/test_gpu_train.py::test_adam_step_matches_torch).
#include <cmath>

#include "pnr_common.h"

namespace pnr {

struct AdamChunk {   // include/pnr_abi.h pnr_adam_chunk
    float *p;
    const float *g;
    float *m, *v;
    int64_t n;
};

struct AdamHyper {
    float b1, b2, omb1, omb2, step_size, sqrt_bc2, eps, wd;
};

__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, const AdamHyper &h) {
    if (h.wd != 0.f) g = g + h.wd * p;
    m = h.b1 * m + h.omb1 * g;
    v = h.b2 * v + h.omb2 * g * g;
    const float denom = sqrtf(v) / h.sqrt_bc2 + h.eps;
    p = p - h.step_size * m / denom;   // torch's fused Adam: param -= step_size * exp_avg / denom
}

__global__ __launch_bounds__(256) void k_adam(const AdamChunk *__restrict__ chunks, AdamHyper h) {
    const AdamChunk c = chunks[blockIdx.x];
    const bool vec = ((reinterpret_cast<uintptr_t>(c.p) | reinterpret_cast<uintptr_t>(c.g) |
                       reinterpret_cast<uintptr_t>(c.m) | reinterpret_cast<uintptr_t>(c.v)) & 15) == 0;
    int64_t done = 0;
    if (vec) {
        const int64_t n4 = c.n >> 2;
        for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
            f4 p = reinterpret_cast<const f4 *>(c.p)[i], m = reinterpret_cast<const f4 *>(c.m)[i];
            f4 v = reinterpret_cast<const f4 *>(c.v)[i];
            const f4 g = reinterpret_cast<const f4 *>(c.g)[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p[e], me = m[e], ve = v[e];
                adam_one(pe, g[e], me, ve, h);
                p[e] = pe;
                m[e] = me;
                v[e] = ve;
            }
            reinterpret_cast<f4 *>(c.p)[i] = p;
            reinterpret_cast<f4 *>(c.m)[i] = m;
            reinterpret_cast<f4 *>(c.v)[i] = v;
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < c.n; i += blockDim.x) {
        float p = c.p[i], m = c.m[i], v = c.v[i];
        adam_one(p, c.g[i], m, v, h);
        c.p[i] = p;
        c.m[i] = m;
        c.v[i] = v;
    }
}

int launch_adam(const void *chunks, int n_chunks, float lr, float beta1, float beta2, float eps, float wd,
                int64_t step, hipStream_t st) {
    if (n_chunks < 0 || step < 1) return fail(PNR_ERR_INVALID, "pnr_adam_step: n_chunks >= 0, step >= 1");
    if (n_chunks == 0) return PNR_OK;
    if (!chunks) return fail(PNR_ERR_INVALID, "pnr_adam_step: NULL chunk table");
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    AdamHyper h;
    h.b1 = beta1;
    h.b2 = beta2;
    h.omb1 = 1.f - beta1;
    h.omb2 = 1.f - beta2;
    h.step_size = (float)(lr / bc1);
    h.sqrt_bc2 = (float)std::sqrt(bc2);
    h.eps = eps;
    h.wd = wd;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)n_chunks), dim3(256), 0, st, static_cast<const AdamChunk *>(chunks), h);
    return launch_ok("adam") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
