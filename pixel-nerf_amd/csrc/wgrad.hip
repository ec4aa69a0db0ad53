// Weight gradients of the ResnetFC 512 x 512 layers (training backward).
//
// Replaces the weight-gradient GEMMs autograd runs for every nn.Linear of ResnetFC
// (resnetfc.py:132-184): G_j = dY_j^T X_j (512 x 512), a sum over the P points of the
// outer products of the layer's output gradient dY_j and its input X_j, both P x 512
// fp32 row-major (the dy slots of pnr_mlp_backward and the activation save).
//
// Arithmetic: split-bf16 products on v_mfma_f32_16x16x32_bf16.  Every operand is split
// exactly into three bf16 parts (x = x0 + x1 + x2, RNE at each step) and the six largest
// products are summed (dropped terms < 2^-24 |x y|), so the result carries fp32 GEMM error
// over bf16's full exponent range: no scaling along the point reduction is needed.
//
// Work decomposition:
//   * a workgroup (4 waves) owns a 128 x 128 output block of one layer over a chunk of
//     points; wave w owns the 64 x 64 quarter (n half w & 1, k half w >> 1), 4 x 4 tiles;
//   * points advance in steps of 32 (one MFMA k-step): each thread loads 16 consecutive
//     floats of one point row of dY and of X (8 threads per 512-B row segment), splits
//     them and stores the parts row-major ([point][column], 256-B rows, the XOR layout
//     of the CDNA guide's dual-use image (b));  MFMA operands (8 consecutive points of one
//     column per lane) come back with ds_read_b64_tr_b16, the hardware transpose read;
//   * the register prefetch of step s + 1 is in flight while step s's MFMAs issue;
//   * split-K over point chunks with deterministic per-chunk partials and a fixed-order
//     reduction (k_wgrad_reduce); the 16 blocks of one (layer, chunk) run on one XCD so
//     the 4x reuse of each dY / X column block is served from that XCD's L2.
#include "pnr_common.h"

namespace pnr {
namespace wg {

constexpr int H = 512;
constexpr int BM = 128;                  // output block edge
constexpr int PS = 32;                   // points per step (MFMA k)
constexpr int NTHR = 256;
constexpr int IMG_BYTES = PS * BM * 2;   // one bf16 part image: 32 rows x 256 B = 8 KB
constexpr int LDS_BYTES = 6 * IMG_BYTES; // dY and X, 3 parts each = 48 KB
constexpr int MAX_JOBS = 16;

struct Args {
    const float *dy[MAX_JOBS];
    const float *x[MAX_JOBS];
    float *partial;          // [job][chunk][512][512]
    int n_jobs, chunks, n_units;
    int64_t n_points, chunk_points;
};

typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

// byte offset of 16-byte chunk ch (0..15) of row r in a [32][256 B] image (guide T10 (b))
__device__ __forceinline__ int img_off(int r, int ch) {
    return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

__device__ __forceinline__ f4 mfma_bf(bf8 a, bf8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// MFMA operand of the 16 columns starting at column c0 (multiple of 16) of an image:
// lane l receives column c0 + (l & 15), points 8 (l >> 4) .. + 7
__device__ __forceinline__ bf8 tr_frag(const char *img, int c0, int lane) {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int ch = (c0 >> 3) + (pp >> 1);
    const char *a0 = img + img_off(8 * g + q, ch) + 8 * (pp & 1);
    const char *a1 = img + img_off(8 * g + 4 + q, ch) + 8 * (pp & 1);
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(a0));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(a1));
    typedef short s8 __attribute__((ext_vector_type(8)));
    const s8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf8, v);
}

__global__ __launch_bounds__(NTHR, 2) void k_wgrad(Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    // blockIdx -> (unit = (job, chunk), block of 16); the 16 blocks of a unit share an XCD
    const int bid = blockIdx.x;
    const int xcd = bid & 7, local = bid >> 3;
    const int b16 = local & 15;
    const int u = 8 * (local >> 4) + xcd;
    if (u >= a.n_units) return;   // whole workgroup: uniform
    const int job = u / a.chunks, chunk = u % a.chunks;
    const int nb = b16 & 3, kb = b16 >> 2;
    const int64_t p0 = (int64_t)chunk * a.chunk_points;
    const int64_t p1 = p0 + a.chunk_points < a.n_points ? p0 + a.chunk_points : a.n_points;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // staging role: row r of the step, columns 16 (t & 7) .. + 15 of the block
    const int r = tid >> 3, c16 = 16 * (tid & 7);
    const float *dsrc = a.dy[job] + nb * BM + c16;
    const float *xsrc = a.x[job] + kb * BM + c16;
    f4 sd[4], sx[4];
    auto load = [&](int64_t pbase) {
        const int64_t p = pbase + r;
        const bool ok = p < p1;
        const int64_t pc = ok ? p : 0;   // in-bounds address (row 0); zeroed below
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sd[i] = *reinterpret_cast<const f4 *>(dsrc + pc * H + 4 * i);
            sx[i] = *reinterpret_cast<const f4 *>(xsrc + pc * H + 4 * i);
            if (!ok) sd[i] = sx[i] = f4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // 16 floats -> 3 parts x 2 chunks of 8 bf16, stored at (row r, chunks c16/8, c16/8 + 1)
    auto put = [&](char *img0, const f4 (&v)[4]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            u4 q0, q1, q2;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f4 &w = v[2 * h + (j >> 1)];
                const float x0 = (j & 1) ? w.z : w.x, x1 = (j & 1) ? w.w : w.y;
                unsigned e0, e1, e2;
                split_pair(x0, x1, e0, e1, e2);
                q0[j] = e0; q1[j] = e1; q2[j] = e2;
            }
            const int off = img_off(r, (c16 >> 3) + h);
            *reinterpret_cast<u4 *>(img0 + off) = q0;
            *reinterpret_cast<u4 *>(img0 + IMG_BYTES + off) = q1;
            *reinterpret_cast<u4 *>(img0 + 2 * IMG_BYTES + off) = q2;
        }
    };
    char *imd = lds, *imx = lds + 3 * IMG_BYTES;

    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int n0 = 64 * (wave & 1), k0 = 64 * (wave >> 1);

    load(p0);
#pragma unroll 1
    for (int64_t pb = p0; pb < p1; pb += PS) {
        __syncthreads();   // the previous step's fragment reads are done
        put(imd, sd);
        put(imx, sx);
        __syncthreads();
        if (pb + PS < p1) load(pb + PS);   // in flight during this step's MFMAs
        bf8 xb[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) xb[j][q] = tr_frag(imx + q * IMG_BYTES, k0 + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf8 da[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) da[q] = tr_frag(imd + q * IMG_BYTES, n0 + 16 * i, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f4 v = acc[i][j];
                v = mfma_bf(da[2], xb[j][0], v);
                v = mfma_bf(da[1], xb[j][1], v);
                v = mfma_bf(da[0], xb[j][2], v);
                v = mfma_bf(da[1], xb[j][0], v);
                v = mfma_bf(da[0], xb[j][1], v);
                v = mfma_bf(da[0], xb[j][0], v);
                acc[i][j] = v;
            }
        }
    }
    // partial block: C rows (n) 4 (l >> 4) + e, column (k) l & 15 of each 16 x 16 tile
    float *out = a.partial + (int64_t)u * H * H + (int64_t)(nb * BM + n0) * H + kb * BM + k0;
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) out[(int64_t)(16 * i + 4 * g + e) * H + 16 * j + li] = acc[i][j][e];
}

// G_j = sum over chunks (in chunk order) of the partials; one thread per 4 outputs
struct Outs {
    float *g[MAX_JOBS];
};
__global__ void k_wgrad_reduce(Outs o, const float *__restrict__ partial, int n_jobs, int chunks) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)n_jobs * (H * H / 4)) return;
    const int job = (int)(t / (H * H / 4));
    const int64_t e = 4 * (t % (H * H / 4));
    const float *src = partial + (int64_t)job * chunks * H * H + e;
    f4 s = *reinterpret_cast<const f4 *>(src);
    for (int c = 1; c < chunks; ++c) s += *reinterpret_cast<const f4 *>(src + (int64_t)c * H * H);
    *reinterpret_cast<f4 *>(o.g[job] + e) = s;
}

// chunk count: about 5 rounds of 2 workgroups per CU over all jobs, >= 8 steps per chunk
inline int wgrad_chunks(int n_jobs, int64_t n_points) {
    const int target = (int)(9.75 * device_cu_count());
    int c = (target + 8 * n_jobs) / (16 * n_jobs);
    const int64_t max_c = (n_points + 8 * PS - 1) / (8 * PS);
    if (c > max_c) c = (int)max_c;
    return c < 1 ? 1 : c;
}

}  // namespace wg

size_t wgrad_workspace_bytes(int n_jobs, int64_t n_points) {
    if (n_jobs < 1 || n_jobs > wg::MAX_JOBS || n_points < 1) return 0;
    return sizeof(float) * (size_t)n_jobs * wg::wgrad_chunks(n_jobs, n_points) * wg::H * wg::H;
}

int launch_wgrad(const float *const *dy, const float *const *x, float *const *g, int n_jobs, int64_t n_points,
                 void *ws, size_t ws_bytes, hipStream_t st) {
    if (n_jobs < 1 || n_jobs > wg::MAX_JOBS) return fail(PNR_ERR_UNSUPPORTED, "weight grad: 1..16 layers");
    if (n_points < 0) return fail(PNR_ERR_INVALID, "weight grad: n_points < 0");
    if (n_points == 0) {
        for (int j = 0; j < n_jobs; ++j)
            if (hipMemsetAsync(g[j], 0, sizeof(float) * wg::H * wg::H, st) != hipSuccess)
                return fail(PNR_ERR_HIP, "weight grad: hipMemsetAsync failed");
        return PNR_OK;
    }
    const size_t need = wgrad_workspace_bytes(n_jobs, n_points);
    if (!ws || ws_bytes < need) return fail(PNR_ERR_WORKSPACE, "weight grad: workspace %zu < %zu", ws_bytes, need);
    wg::Args a = {};
    wg::Outs o = {};
    for (int j = 0; j < n_jobs; ++j) {
        if (!dy[j] || !x[j] || !g[j]) return fail(PNR_ERR_INVALID, "weight grad: NULL matrix (layer %d)", j);
        if (((reinterpret_cast<uintptr_t>(dy[j]) | reinterpret_cast<uintptr_t>(x[j]) |
              reinterpret_cast<uintptr_t>(g[j])) & 15) != 0)
            return fail(PNR_ERR_INVALID, "weight grad: matrices must be 16-byte aligned");
        a.dy[j] = dy[j];
        a.x[j] = x[j];
        o.g[j] = g[j];
    }
    a.n_jobs = n_jobs;
    a.chunks = wg::wgrad_chunks(n_jobs, n_points);
    a.n_units = n_jobs * a.chunks;
    a.n_points = n_points;
    a.chunk_points = ((n_points + a.chunks - 1) / a.chunks + wg::PS - 1) / wg::PS * wg::PS;
    a.partial = static_cast<float *>(ws);
    const int unit_groups = (a.n_units + 7) / 8;   // units padded to a multiple of 8 (one per XCD)
    hipLaunchKernelGGL(wg::k_wgrad, dim3((unsigned)(unit_groups * 8 * 16)), dim3(wg::NTHR), wg::LDS_BYTES, st, a);
    if (!launch_ok("wgrad")) return PNR_ERR_HIP;
    const int64_t nt = (int64_t)n_jobs * (wg::H * wg::H / 4);
    hipLaunchKernelGGL(wg::k_wgrad_reduce, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, o, a.partial,
                       n_jobs, a.chunks);
    return launch_ok("wgrad_reduce") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
