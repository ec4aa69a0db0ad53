// Weight gradients of the ResnetFC 512 x 512 layers (training backward).
//
// Replaces the weight-gradient GEMMs autograd runs for every nn.Linear of ResnetFC
// (resnetfc.py:132-184): G_j = dY_j^T X_j (512 x 512), a sum over the P points of the
// outer products of the layer's output gradient dY_j and its input X_j, both P x 512
// fp32 row-major (the dy slots of pnr_mlp_backward and the activation save).
//
// Work decomposition (both kernels):
//   * a workgroup (8 waves, one per CU) owns a 256 x 256 output block of one layer over a
//     chunk of points; wave w owns 128 x 64 of it (n half w & 1, k quarter w >> 1):
//     8 x 4 tiles of 16 x 16, 128 accumulator VGPRs;
//   * points advance in steps of 32 (one MFMA k-step): each thread loads 16 floats of one
//     point row of dY and of X (16 threads per 1 KB row), splits them and stores the parts
//     row-major ([point][column], 544-B rows: 512 B + 32 B pad);  MFMA operands (8
//     consecutive points of one column per lane) come back with ds_read_b64_tr_b16, the
//     hardware transpose read.  Point p of a step is stored at row pi(p) (bits 2 and 3
//     swapped): the 8 rows one 32-lane half of a transpose read touches then sit 8 banks
//     apart under the 136-dword pitch (conflict-free), every 8-lane group of a
//     ds_write_b128 stores 128 consecutive bytes (conflict-free), and a tile's operand is
//     a constant byte offset from the lane's base (immediate offsets, no address VALU);
//   * split-K over point chunks with deterministic per-chunk partials and a fixed-order
//     reduction (k_wgrad_reduce); the 4 blocks of one (layer, chunk) run on one XCD so
//     each dY / X column block's 2x reuse is served from that XCD's L2.
//
// k_wgrad_h (default): f16x3 products on v_mfma_f32_16x16x32_f16 -- every operand scaled by
// a power of two per (chunk, channel) and split into two fp16 parts (22 significand bits),
// hi*hi + hi*lo + lo*hi: half the MFMAs of the split-bf16 kernel.  The two-part images take
// 68 KB, so they are double-buffered: step s + 1's split runs in four pieces between step s's
// MFMAs (the scheduler interleaves the VALU and the LDS stores with them), one barrier per step.
// Scales: a running per-channel exponent E_c (the operand is v 2^-E_c).  A split value that
// reaches 2^15 raises a flag; after the step's barrier the workgroup then re-reads that step,
// takes the channel maxima (LDS atomics), moves E_c of the overflowing channels so that the
// maximum lands in [2^5, 2^6), multiplies the accumulator rows / columns by 2^(E_old - E_new)
// (exact) and splits the step again.  The chunk's first 4 steps set the first scales; a channel
// still all zero then takes its tensor's maximum (on a training step's data, channels turning
// on later were 98 % of the scale moves).  Measured: 0.34 % of a training step's 32-point steps
// retune.  Every value keeps 22 bits down to 2^-8 of its channel's running maximum, and an
// absolute error below 2^-30 of that maximum beneath it; the result is acc 2^(E_row + E_col).
//
// Bound of k_wgrad_h, per output element: an element whose terms all come from values far
// below their channel's running maximum M in the chunk (e.g. X_j nonzero only where dY_i is
// 2^-20 of M_i) keeps only the absolute error ~2^-30 M of those values, not fp32 relative error:
// values below 2^-8 M lose low bits (the second fp16 part goes subnormal), values below ~2^-19 M
// lose the first part's bits too, and below ~2^-30 M they flush to zero.
// (tests/test_gpu_train.py::test_weight_grad_wide_dynamic_range measures both kernels.)
//
// k_wgrad (PNR_WGRAD_BF16X6, ABI 4, per call; the round-2 kernel): split-bf16 products on
// v_mfma_f32_16x16x32_bf16, three exact bf16 parts per operand and the six largest products
// (dropped terms < 2^-24 |x y|), no scaling (bf16 has fp32's exponent range); one image set,
// split and MFMAs separated by two barriers per step.
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
    bool ok = true;   // the staged row is a point of the chunk (else it is staged as zeros)
    // The zeroing of a row past the chunk happens in put(), not here: a select right after
    // the loads made the compiler wait for them (s_waitcnt vmcnt(0)) before the step's MFMAs,
    // exposing a full L2 / HBM latency per 32-point step on every wave.
    auto load = [&](int64_t pbase) {
        const int64_t p = pbase + r;
        ok = p < p1;
        const int64_t pc = ok ? p : 0;   // in-bounds address (row 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = 128 * (i >> 1) + 4 * (i & 1);
            sd[i] = *reinterpret_cast<const f4 *>(dsrc + pc * H + col);
            sx[i] = *reinterpret_cast<const f4 *>(xsrc + pc * H + col);
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
                float x0 = (j & 1) ? w.z : w.x, x1 = (j & 1) ? w.w : w.y;
                if (!ok) x0 = x1 = 0.f;
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
#ifndef PNR_WG_NOPUT   // diagnostic ablation (stale images)
        put(imd, sd);
        put(imx, sx);
#endif
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
#ifndef PNR_WG_MFMA3   // diagnostic ablation: 3 of the 6 products
                v = mfma_bf(da[2], xb[j][0], v);
                v = mfma_bf(da[1], xb[j][1], v);
                v = mfma_bf(da[0], xb[j][2], v);
#endif
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

// ---- f16x3, double-buffered (k_wgrad_h) --------------------------------------------------
constexpr int SET_BYTES = 4 * IMG_BYTES;            // dY hi | dY lo | X hi | X lo: 69,632 B
constexpr int HS_SC = 2 * SET_BYTES;                // sc[512]: 2^-E per channel (dY 0..255, X 256..511)
constexpr int HS_E = HS_SC + 512 * 4;               // E[512] (int)
constexpr int HS_RS = HS_E + 512 * 4;               // rs[512]: 2^(E_old - E_new) of the last retune
constexpr int HS_MAX = HS_RS + 512 * 4;             // chmax[512] (|v| bits, LDS atomic max)
constexpr int HS_FLAG = HS_MAX + 512 * 4;           // flag[2]: step index of an overflow, by parity; tmax[2]
constexpr int LDS_BYTES_H = HS_FLAG + 16;           // 147,472 B
constexpr int E_UNSET = -100;                       // no nonzero value seen: scale 2^100
constexpr float OVF = 32768.f;                      // |v 2^-E| >= 2^15: the channel's scale moves
#ifndef PNR_WGH_HEAD
#define PNR_WGH_HEAD 5
#endif
#ifndef PNR_WGH_INIT
#define PNR_WGH_INIT 4
#endif
constexpr int E_HEAD = PNR_WGH_HEAD;                // a moved channel's maximum lands in [2^H, 2^(H+1))
constexpr int INIT_STEPS = PNR_WGH_INIT;            // steps whose maxima set the chunk's first scales

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 mfma_h(h8 a, h8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// packed fp16 residuals f16(x - f32(h.lo)), f16(y - f32(h.hi)): one rounding of the exact
// difference (v_fma_mix{lo,hi}_f16, as mlp.hip's split)
__device__ __forceinline__ unsigned resid_pk(unsigned h, float x, float y) {
    unsigned d;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h), "v"(x));
    asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(d) : "v"(h), "v"(y));
    return d;
}
__device__ __forceinline__ h8 tr_frag_h(const char *base, int lo, int hi) {
    const s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + lo));
    const s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + hi));
    typedef short s8 __attribute__((ext_vector_type(8)));
    const s8 v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return __builtin_bit_cast(h8, v);
}

#ifdef PNR_WGH_STATS   // diagnostic: [0] retunes after step 0, [1] steps, [2] workgroups, channel scale moves
                       // after step 0: [3] from unset (no nonzero value yet), [4] by growth (tools/wgrad_stats.py)
__device__ unsigned long long g_wgh_stats[5];
#endif

__global__ __launch_bounds__(NTHR, 1) void k_wgrad_h(Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    float *sc = reinterpret_cast<float *>(lds + HS_SC);
    int *Ee = reinterpret_cast<int *>(lds + HS_E);
    float *rs = reinterpret_cast<float *>(lds + HS_RS);
    unsigned *chmax = reinterpret_cast<unsigned *>(lds + HS_MAX);
    int *flag = reinterpret_cast<int *>(lds + HS_FLAG);
    unsigned *tmax = reinterpret_cast<unsigned *>(lds + HS_FLAG + 8);   // dY, X maxima of a retune
    const int bid = blockIdx.x;
    const int xcd = bid & 7, local = bid >> 3;
    const int b4 = local & 3;
    const int u = 8 * (local >> 2) + xcd;
    if (u >= a.n_units) return;   // whole workgroup: uniform
    const int job = u / a.chunks, chunk = u % a.chunks;
    const int nb = b4 & 1, kb = b4 >> 1;
    const int64_t p0 = (int64_t)chunk * a.chunk_points;
    const int64_t p1 = p0 + a.chunk_points < a.n_points ? p0 + a.chunk_points : a.n_points;
    const int nsteps = p1 > p0 ? (int)((p1 - p0 + PS - 1) / PS) : 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // staging role: point r of the step, columns 8j .. 8j+7 and 128+8j .. 128+8j+7 (j = t & 15)
    const int r = tid >> 4, jc = tid & 15;
    const float *dsrc = a.dy[job] + nb * BM + 8 * jc;
    const float *xsrc = a.x[job] + kb * BM + 8 * jc;
    const int woff = PITCH * prow(r) + 16 * jc;   // + 256 for the second 8 columns
    // (slow path) one step's row of this thread: 4 f4 of dY, 4 of X (columns 8 jc + 0..7,
    // 128 + 8 jc + 0..7); ok = the row is a point of the chunk
    auto load = [&](int step, f4 (&d)[4], f4 (&x)[4], bool &ok) {
#ifdef PNR_WG_L2ROWS   // diagnostic ablation: every step re-reads the chunk's first rows (L2 hits)
        const int64_t p = p0 + r + 0 * step;
#else
        const int64_t p = p0 + (int64_t)step * PS + r;
#endif
        ok = p < p1;
        const int64_t pc = ok ? p : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = 128 * (i >> 1) + 4 * (i & 1);
            d[i] = *reinterpret_cast<const f4 *>(dsrc + pc * H + col);
            x[i] = *reinterpret_cast<const f4 *>(xsrc + pc * H + col);
        }
    };
    // (slow path) v 2^-E -> two fp16 parts of 8 channels x 2 at (row pi(r), bytes 16 jc and
    // 256 + 16 jc) of the image pair at img (hi) / img + IMG_BYTES (lo); a row past the chunk
    // (!ok) is staged as zeros
    auto put = [&](char *img, const float *scb, const f4 (&v)[4], bool ok) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f4 s0 = *reinterpret_cast<const f4 *>(scb + 128 * h + 8 * jc);
            const f4 s1 = *reinterpret_cast<const f4 *>(scb + 128 * h + 8 * jc + 4);
            const f4 z = {0.f, 0.f, 0.f, 0.f};
            const f4 y0 = (ok ? v[2 * h] : z) * s0, y1 = (ok ? v[2 * h + 1] : z) * s1;
            u4 hi, lo;
            const f2 q[4] = {f2{y0.x, y0.y}, f2{y0.z, y0.w}, f2{y1.x, y1.y}, f2{y1.z, y1.w}};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                hi[k] = __builtin_bit_cast(unsigned, __builtin_convertvector(q[k], h2));
                lo[k] = resid_pk(hi[k], q[k].x, q[k].y);
            }
            char *d = img + woff + 256 * h;
            *reinterpret_cast<u4 *>(d) = hi;
            *reinterpret_cast<u4 *>(d + IMG_BYTES) = lo;
        }
    };

    f4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int n0 = 128 * (wave & 1), k0 = 64 * (wave >> 1);
    // this lane's transpose-read offsets (points 8g + q and 8g + 4 + q, column pair pp)
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int t_lo = PITCH * prow(8 * g + q) + 8 * pp, t_hi = PITCH * prow(8 * g + 4 + q) + 8 * pp;

    // the slow path: re-read step `step`, move the scales of its overflowing channels, rescale the
    // accumulators and split the step again into image set `set`
    auto retune = [&](int step, char *set, int scan) {
        f4 td[4], tx[4];
        bool tok;
        // channel maxima (and each tensor's maximum over its 256 channels) of the staged rows
        auto note = [&]() {
            if (!tok) return;
            float md = 0.f, mx = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 128 * (i >> 1) + 8 * jc + 4 * (i & 1);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    atomicMax(chmax + c + e, __float_as_uint(fabsf(td[i][e])));
                    atomicMax(chmax + 256 + c + e, __float_as_uint(fabsf(tx[i][e])));
                    md = fmaxf(md, fabsf(td[i][e]));
                    mx = fmaxf(mx, fabsf(tx[i][e]));
                }
            }
            atomicMax(tmax, __float_as_uint(md));
            atomicMax(tmax + 1, __float_as_uint(mx));
        };
        // the maxima of steps step + 1 .. step + scan - 1 too (the chunk's first scales)
        for (int q = 1; q < scan; ++q) {
            load(step + q, td, tx, tok);
            note();
        }
        load(step, td, tx, tok);
        note();
        __syncthreads();
        {   // channel tid
            const int eo = Ee[tid];
            // a channel without a nonzero value so far takes its tensor's maximum: its scale is
            // then set before its first nonzero step (98 % of the scale moves of a training step
            // were such channels turning on, each one a retune)
            const unsigned mb = chmax[tid] == 0u && eo == E_UNSET ? tmax[tid >> 8] : chmax[tid];
            chmax[tid] = 0u;
            const float m = __uint_as_float(mb);
            float ratio = 1.f;
            if (!(m * sc[tid] < OVF)) {
                int en = (int)((mb >> 23) & 255u) - 127 - E_HEAD;   // m in [2^k, 2^(k+1)): k - E_HEAD
                en = en < E_UNSET ? E_UNSET : (en > 127 ? 127 : en);
                if (en > eo) {
#ifdef PNR_WGH_STATS
                    if (step > 0) atomicAdd(&g_wgh_stats[eo == E_UNSET ? 3 : 4], 1ull);
#endif
                    ratio = __builtin_ldexpf(1.f, eo - en);
                    Ee[tid] = en;
                    sc[tid] = __builtin_ldexpf(1.f, -en);
                }
            }
            rs[tid] = ratio;
        }
        __syncthreads();
        if (tid < 2) tmax[tid] = 0u;   // read by every channel before the barrier
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float cs = rs[256 + k0 + 16 * j + li];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const f4 rw = *reinterpret_cast<const f4 *>(rs + n0 + 16 * i + 4 * g);
                acc[i][j] *= rw * cs;
            }
        }
        put(set, sc, td, tok);
        put(set + 2 * IMG_BYTES, sc + 256, tx, tok);
        __syncthreads();
    };

    if (tid < 512) {
        sc[tid] = 0x1p100f;
        Ee[tid] = E_UNSET;
        chmax[tid] = 0u;
    }
    if (tid < 2) {
        flag[tid] = -1;
        tmax[tid] = 0u;
    }
    __syncthreads();
    if (nsteps > 0) retune(0, lds, nsteps < INIT_STEPS ? nsteps : INIT_STEPS);
    // Step s + 1's split runs inside step s's MFMA loop, in four pieces (piece k = tensor k >> 1,
    // column half k & 1: 8 values of the thread's row) after row tiles 1, 3, 5, 7, so the
    // scheduler interleaves its VALU and LDS stores with the MFMAs.  Each piece's registers are
    // reloaded with step s + 2's values right after its split: a full step of load latency.
    f4 stg[4][2];
    auto load_piece = [&](int step, int k) {
        const int64_t p = p0 + (int64_t)step * PS + r;
        const int64_t pc = p < p1 ? p : 0;   // rows past the chunk: a valid row, zeroed by okf
        const float *src = ((k >> 1) ? xsrc : dsrc) + pc * H + 128 * (k & 1);
        stg[k][0] = *reinterpret_cast<const f4 *>(src);
        stg[k][1] = *reinterpret_cast<const f4 *>(src + 4);
    };
    if (nsteps > 1)
#pragma unroll
        for (int k = 0; k < 4; ++k) load_piece(1, k);
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
        char *cur = lds + (s & 1) * SET_BYTES, *nxt = lds + ((s + 1) & 1) * SET_BYTES;
        const float okf = p0 + (int64_t)(s + 1) * PS + r < p1 ? 1.f : 0.f;   // step s + 1's row
        float m = 0.f;   // max |split value| of step s + 1 (a last step's split is never read)
        auto put_piece = [&](int k) {
            const float *scb = sc + 256 * (k >> 1) + 128 * (k & 1) + 8 * jc;
            const f4 y0 = stg[k][0] * (*reinterpret_cast<const f4 *>(scb) * okf);
            const f4 y1 = stg[k][1] * (*reinterpret_cast<const f4 *>(scb + 4) * okf);
            u4 hi, lo;
            const f2 q[4] = {f2{y0.x, y0.y}, f2{y0.z, y0.w}, f2{y1.x, y1.y}, f2{y1.z, y1.w}};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                hi[e] = __builtin_bit_cast(unsigned, __builtin_convertvector(q[e], h2));
                lo[e] = resid_pk(hi[e], q[e].x, q[e].y);
                m = fmaxf(m, fmaxf(fabsf(q[e].x), fabsf(q[e].y)));
            }
            char *d = nxt + 2 * IMG_BYTES * (k >> 1) + woff + 256 * (k & 1);
            *reinterpret_cast<u4 *>(d) = hi;
            *reinterpret_cast<u4 *>(d + IMG_BYTES) = lo;
            load_piece(s + 2, k);
        };
        const char *ad = cur + 2 * n0, *ax = cur + 2 * IMG_BYTES + 2 * k0;
        h8 xb[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) xb[j][pt] = tr_frag_h(ax + pt * IMG_BYTES + 32 * j, t_lo, t_hi);
        // dY fragments one row tile ahead: tile i + 1's reads are in flight during tile i's MFMAs
        h8 dh = tr_frag_h(ad, t_lo, t_hi), dl = tr_frag_h(ad + IMG_BYTES, t_lo, t_hi);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            h8 nh = dh, nl = dl;
            if (i < 7) {
                nh = tr_frag_h(ad + 32 * (i + 1), t_lo, t_hi);
                nl = tr_frag_h(ad + IMG_BYTES + 32 * (i + 1), t_lo, t_hi);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f4 v = acc[i][j];
                v = mfma_h(dl, xb[j][0], v);
                v = mfma_h(dh, xb[j][1], v);
                v = mfma_h(dh, xb[j][0], v);
                acc[i][j] = v;
            }
#ifndef PNR_WG_NOPUT   // diagnostic ablation (stale images)
            if (i & 1) put_piece(i >> 1);
#endif
            dh = nh;
            dl = nl;
        }
        if (!(m < OVF)) flag[(s + 1) & 1] = s + 1;   // NaN-safe: a NaN maximum retunes too
        __syncthreads();   // step s + 1's images are complete; step s's reads are done
        if (s + 1 < nsteps && flag[(s + 1) & 1] == s + 1) {
            retune(s + 1, nxt, 1);
#ifdef PNR_WGH_STATS
            if (tid == 0) atomicAdd(&g_wgh_stats[0], 1ull);
#endif
        }
    }
#ifdef PNR_WGH_STATS
    if (tid == 0) {
        atomicAdd(&g_wgh_stats[1], (unsigned long long)nsteps);
        atomicAdd(&g_wgh_stats[2], 1ull);
    }
#endif
    // partial block G = acc 2^(E_row + E_col): C rows (n) 4 (l >> 4) + e, column (k) l & 15
    float *out = a.partial + (int64_t)u * H * H + (int64_t)(nb * BM + n0) * H + kb * BM + k0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ec = Ee[256 + k0 + 16 * j + li];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                out[(int64_t)(16 * i + 4 * g + e) * H + 16 * j + li] =
                    __builtin_ldexpf(acc[i][j][e], Ee[n0 + 16 * i + 4 * g + e] + ec);
    }
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

#ifdef PNR_WGH_STATS
extern "C" int pnr_wgrad_stats(unsigned long long *out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(wg::g_wgh_stats), sizeof(wg::g_wgh_stats)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[5] = {0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(wg::g_wgh_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

size_t wgrad_workspace_bytes(int n_jobs, int64_t n_points) {
    if (n_jobs < 1 || n_jobs > wg::MAX_JOBS || n_points < 1) return 0;
    return sizeof(float) * (size_t)n_jobs * wg::wgrad_chunks(n_jobs, n_points) * wg::H * wg::H;
}

int launch_wgrad(const float *const *dy, const float *const *x, float *const *g, int n_jobs, int64_t n_points,
                 void *ws, size_t ws_bytes, hipStream_t st, int arith) {
    if (arith != PNR_WGRAD_F16X3 && arith != PNR_WGRAD_BF16X6)
        return fail(PNR_ERR_INVALID, "weight grad: arithmetic %d is not PNR_WGRAD_F16X3 / PNR_WGRAD_BF16X6", arith);
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
    if (arith == PNR_WGRAD_BF16X6)
        hipLaunchKernelGGL(wg::k_wgrad, dim3((unsigned)(unit_groups * 8 * 4)), dim3(wg::NTHR), wg::LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL(wg::k_wgrad_h, dim3((unsigned)(unit_groups * 8 * 4)), dim3(wg::NTHR), wg::LDS_BYTES_H, st,
                           a);
    if (!launch_ok("wgrad")) return PNR_ERR_HIP;
    const int64_t nt = (int64_t)n_jobs * (wg::H * wg::H / 4);
    hipLaunchKernelGGL(wg::k_wgrad_reduce, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, o, a.partial,
                       n_jobs, a.chunks);
    return launch_ok("wgrad_reduce") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
