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
//   * a workgroup (8 waves, one per CU) owns a 256 x 256 output block of one layer over a
//     chunk of points; wave w owns 128 x 64 of it (n half w & 1, k quarter w >> 1):
//     8 x 4 tiles of 16 x 16, 128 accumulator VGPRs.  Each staged element feeds 2 (dY) or
//     4 (X) waves' MFMAs, so the split VALU per MFMA is 0.75 instruction;
//   * points advance in steps of 32 (one MFMA k-step): each thread loads 16 floats of one
//     point row of dY and of X (16 threads per 1 KB row), splits them and stores the parts
//     row-major ([point][column], 544-B rows: 512 B + 32 B pad);  MFMA operands (8
//     consecutive points of one column per lane) come back with ds_read_b64_tr_b16, the
//     hardware transpose read.  Point p of a step is stored at row pi(p) (bits 2 and 3
//     swapped): the 8 rows one 32-lane half of a transpose read touches then sit 8 banks
//     apart under the 136-dword pitch (conflict-free), every 8-lane group of a
//     ds_write_b128 stores 128 consecutive bytes (conflict-free), and a tile's operand is
//     a constant byte offset from the lane's base (immediate offsets, no address VALU);
//   * the register prefetch of step s + 1 is in flight during step s;
//   * split-K over point chunks with deterministic per-chunk partials and a fixed-order
//     reduction (k_wgrad_reduce); the 4 blocks of one (layer, chunk) run on one XCD so
//     each dY / X column block's 2x reuse is served from that XCD's L2.
#include "pnr_common.h"

namespace pnr {
namespace wg {

constexpr int H = 512;
constexpr int BM = 256;                  // output block edge
constexpr int PS = 32;                   // points per step (MFMA k)
constexpr int NTHR = 512;
constexpr int PITCH = 2 * BM + 32;       // bytes per image row (bank offset 8 per row)
constexpr int IMG_BYTES = PS * PITCH;    // one bf16 part image: 17,408 B
constexpr int LDS_BYTES = 6 * IMG_BYTES; // dY and X, 3 parts each = 104,448 B
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

// image row of point p (0..31) of a step: bits 2 and 3 swapped
__device__ __forceinline__ int prow(int p) { return (p & ~12) | ((p & 4) << 1) | ((p & 8) >> 1); }

__device__ __forceinline__ f4 mfma_bf(bf8 a, bf8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// MFMA operand of 16 columns: lane l receives column c0 + (l & 15), points 8 (l >> 4) ..
// + 7.  `base` = image + 2 c0 bytes; lo / hi = the lane's byte offsets of its points
// 8g + q and 8g + 4 + q (q = (l & 15) >> 2) plus 8 ((l & 3)) within the 16 columns.
__device__ __forceinline__ bf8 tr_frag(const char *base, int lo, int hi) {
    const s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + lo));
    const s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + hi));
    typedef short s8 __attribute__((ext_vector_type(8)));
    const s8 v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return __builtin_bit_cast(bf8, v);
}

__global__ __launch_bounds__(NTHR, 1) void k_wgrad(Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    // blockIdx -> (unit = (job, chunk), block of 4); the 4 blocks of a unit share an XCD
    const int bid = blockIdx.x;
    const int xcd = bid & 7, local = bid >> 3;
    const int b4 = local & 3;
    const int u = 8 * (local >> 2) + xcd;
    if (u >= a.n_units) return;   // whole workgroup: uniform
    const int job = u / a.chunks, chunk = u % a.chunks;
    const int nb = b4 & 1, kb = b4 >> 1;
    const int64_t p0 = (int64_t)chunk * a.chunk_points;
    const int64_t p1 = p0 + a.chunk_points < a.n_points ? p0 + a.chunk_points : a.n_points;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // staging role: point r of the step, columns 8j .. 8j+7 and 128+8j .. 128+8j+7 (j = t & 15)
    const int r = tid >> 4, jc = tid & 15;
    const float *dsrc = a.dy[job] + nb * BM + 8 * jc;
    const float *xsrc = a.x[job] + kb * BM + 8 * jc;
    const int woff = PITCH * prow(r) + 16 * jc;   // + 256 for the second 8 columns
    f4 sd[4], sx[4];
    auto load = [&](int64_t pbase) {
        const int64_t p = pbase + r;
        const bool ok = p < p1;
        const int64_t pc = ok ? p : 0;   // in-bounds address (row 0); zeroed below
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = 128 * (i >> 1) + 4 * (i & 1);
            sd[i] = *reinterpret_cast<const f4 *>(dsrc + pc * H + col);
            sx[i] = *reinterpret_cast<const f4 *>(xsrc + pc * H + col);
            if (!ok) sd[i] = sx[i] = f4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // 16 floats -> 3 parts x 2 chunks of 8 bf16 at (row pi(r), bytes 16 jc and 256 + 16 jc)
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
            char *d = img0 + woff + 256 * h;
            *reinterpret_cast<u4 *>(d) = q0;
            *reinterpret_cast<u4 *>(d + IMG_BYTES) = q1;
            *reinterpret_cast<u4 *>(d + 2 * IMG_BYTES) = q2;
        }
    };
    char *imd = lds, *imx = lds + 3 * IMG_BYTES;

    f4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int n0 = 128 * (wave & 1), k0 = 64 * (wave >> 1);
    // this lane's transpose-read offsets (points 8g + q and 8g + 4 + q, column pair pp)
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int t_lo = PITCH * prow(8 * g + q) + 8 * pp, t_hi = PITCH * prow(8 * g + 4 + q) + 8 * pp;
    const char *ad = imd + 2 * n0, *ax = imx + 2 * k0;

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
            for (int pt = 0; pt < 3; ++pt) xb[j][pt] = tr_frag(ax + pt * IMG_BYTES + 32 * j, t_lo, t_hi);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            bf8 da[3];
#pragma unroll
            for (int pt = 0; pt < 3; ++pt) da[pt] = tr_frag(ad + pt * IMG_BYTES + 32 * i, t_lo, t_hi);
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
#pragma unroll
    for (int i = 0; i < 8; ++i)
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

// chunk count: about 5 rounds of one workgroup per CU over all jobs (4 blocks per
// (layer, chunk)), >= 8 steps per chunk
inline int wgrad_chunks(int n_jobs, int64_t n_points) {
    const int target = (int)(4.875 * device_cu_count());
    int c = (target + 2 * n_jobs) / (4 * n_jobs);
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
    hipLaunchKernelGGL(wg::k_wgrad, dim3((unsigned)(unit_groups * 8 * 4)), dim3(wg::NTHR), wg::LDS_BYTES, st, a);
    if (!launch_ok("wgrad")) return PNR_ERR_HIP;
    const int64_t nt = (int64_t)n_jobs * (wg::H * wg::H / 4);
    hipLaunchKernelGGL(wg::k_wgrad_reduce, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, o, a.partial,
                       n_jobs, a.chunks);
    return launch_ok("wgrad_reduce") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
