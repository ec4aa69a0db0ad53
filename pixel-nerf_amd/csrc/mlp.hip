// Fused per-point pixelNeRF model and ray march on gfx950 MFMA.
//
// Replaces PixelNeRFNet.forward (models.py:146-266) for the shipped conf:
//   world->camera transform (162-165), positional encoding (code.py:30-42),
//   view directions (184-196), pinhole projection + bilinear border gather of
//   the encoder latent (206-221, encoder.py:80-109), ResnetFC (resnetfc.py:132-184)
//   with the multi-view mean at combine_layer (util.py:461-471), and the
//   sigmoid/relu head (258-265); with the fused march (Args::march) also the coarse
//   draws, the composite and the fine draws of NeRFRenderer.forward (nerf.py:251-303).
//
// Work decomposition:
//   * a workgroup = 8 waves (two per SIMD) = a tile of 64 points ("columns"); persistent
//     workgroups, one per CU, take tiles (or a ray's tiles) from per-XCD counters.
//   * every layer is OUT^T (512 x 64) = W (512 x K) * IN^T (K x 64).  Wave w owns output
//     rows [64w, 64w + 64) for all 64 columns: 4 row tiles x 4 column tiles = 16
//     accumulators; x (the residual stream) and h stay in registers for the whole network.
//   * f16x3 (PREC 3, the default): IN^T lives in LDS already scaled per column and split
//     into two fp16 planes P0 / P1 by its producer (features, latent stage, relu publish);
//     W is pre-packed (k_pack_f16) in A-fragment order with a per-layer scale and streamed
//     from L2 through a register ring H_DIST row tiles ahead of v_mfma_f32_16x16x32_f16.
//     fp32 (PREC 0) and split-bf16 (PREC 6 / 9) keep an fp32 image and their own GEMMs.
// Diagnostic build knobs: pnr_diag.h.
#include "pnr_diag.h"
#include <cstddef>

#include "march_dev.h"

namespace pnr {
namespace mlpk {

constexpr int H = 512;             // d_hidden == d_latent (only width implemented)
constexpr int NRT = H / 16;        // 32 row tiles per layer
constexpr int NKB = H / 16;        // 32 k-blocks (16 k each) for K = 512
constexpr int NKB_IN = 4;          // lin_in k-blocks (d_in <= 64, zero padded)
constexpr int WAVES = 8;           // two waves per SIMD
constexpr int NTHR = 64 * WAVES;
constexpr int RTW = NRT / WAVES;   // row tiles per wave (4 at 8 waves)
constexpr int CT = 4;              // column tiles (16 columns each)
constexpr int COLS = 16 * CT;      // 64 points per tile
constexpr int LDS_LD = H + 4;      // floats per column in the LDS activation buffer
constexpr int KB_FLOATS = NRT * 256;          // one k-block of a packed layer (32 KB)
constexpr int LAYER_FLOATS = NKB * KB_FLOATS; // one packed 512x512 layer (1 MB)
constexpr int HDR = 64;            // header floats: pe freqs [0,16), phases [16,32)
// split-bf16 modes (PREC 6 / 9): v_mfma_f32_16x16x32_bf16, k-steps of 32
constexpr int KS32 = H / 32;       // 16 k-steps for K = 512
constexpr int KS32_IN = 2;         // lin_in (d_in <= 64)
constexpr int SRT_FLOATS = 768;    // one (k-step, row tile): 3 parts x 64 lanes x 8 bf16
constexpr int SKS_FLOATS = NRT * SRT_FLOATS;  // one k-step of a packed layer (96 KB)
// scaled-fp16 mode (PREC 3): 2 parts x 64 lanes x 8 f16 per (k-step, row tile)
constexpr int SRT16_FLOATS = 512;
constexpr int SKS16_FLOATS = NRT * SRT16_FLOATS;  // 64 KB
constexpr int HDR_ESCALE = 32;     // header floats [32, 64): per-layer weight scale exponents
                                   // (PREC 3): [32] lin_in, [33 + j] packed 512-wide layer j
__host__ __device__ constexpr int sks_floats(int prec) { return prec == 3 ? SKS16_FLOATS : SKS_FLOATS; }

struct Layout {
    int prec;                      // 0 = f32 MFMA, 6 / 9 = split-bf16 products, 3 = scaled f16
    int n_linz, n_l512, n_blocks, ncomb, d_in, d_out, pe_n;
    int64_t layer_floats;
    int64_t off_lin_in, off_l512, off_lin_out, off_bias, nbias, off_out32, total;
};

inline Layout make_layout(const pnr_mlp_desc &d) {
    Layout L;
    L.n_blocks = d.n_blocks;
    L.n_linz = d.combine_layer < d.n_blocks ? d.combine_layer : d.n_blocks;
    L.ncomb = L.n_linz;
    L.n_l512 = L.n_linz + 2 * d.n_blocks;
    L.d_in = d.d_in;
    L.d_out = d.d_out;
    L.pe_n = d.pe_n;
    L.prec = d.precision;
    L.layer_floats = L.prec ? (int64_t)KS32 * sks_floats(L.prec) : (int64_t)LAYER_FLOATS;
    L.off_lin_in = HDR;
    L.off_l512 = L.off_lin_in + (L.prec ? (int64_t)KS32_IN * sks_floats(L.prec) : (int64_t)NKB_IN * KB_FLOATS);
    L.off_lin_out = L.off_l512 + (int64_t)L.n_l512 * L.layer_floats;
    L.off_bias = L.off_lin_out + (int64_t)NKB * 256;
    L.nbias = (int64_t)(1 + L.n_l512) * H + 16;
    // PREC 3: lin_out's weights in fp32 as [input channel][4 outputs] (the VALU head, k_point_mlp)
    L.off_out32 = ((L.off_bias + L.nbias + 63) / 64) * 64;
    L.total = L.off_out32 + (L.prec == 3 ? 4 * H : 0);
    return L;
}

// packed L512 layer index of block `blk`, kind 0 = lin_z, 1 = fc_0, 2 = fc_1
__host__ __device__ inline int layer_index(int blk, int kind, int n_linz) {
    return blk < n_linz ? 3 * blk + kind : 3 * n_linz + 2 * (blk - n_linz) + (kind - 1);
}

struct PackSrc {
    const float *lin_in_w, *lin_in_b, *lin_out_w, *lin_out_b, *pe_f, *pe_p;
    const float *w[24], *b[24];
};

// One thread per packed float.  Fragment element (kb, rt, lane, s) holds
// W[16 rt + (lane & 15)][16 kb + 4 (lane >> 4) + s]: the A operand of k-step
// (kb, s) for row tile rt (v_mfma_f32_16x16x4_f32: lane l holds A[l&15][l>>4]).
__global__ void k_pack(PackSrc s, Layout L, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.total) return;
    float v = 0.0f;
    if (i < HDR) {
        if (i >= HDR_ESCALE && i < HDR_ESCALE + 1 + L.n_l512 && L.prec == 3) return;   // k_layer_escale's
        if (i < 16 && i < L.pe_n) v = s.pe_f[i];
        else if (i >= 16 && i < 32 && (i - 16) < L.pe_n) v = s.pe_p[i - 16];
    } else if (i < L.off_lin_out && L.prec) {
        return;   // written by k_pack_split / k_pack_f16
    } else if (i < L.off_l512) {
        const int e = (int)(i - L.off_lin_in);
        const int kb = e / KB_FLOATS, rt = (e / 256) % NRT, lane = (e >> 2) & 63, j = e & 3;
        const int row = 16 * rt + (lane & 15), col = 16 * kb + 4 * (lane >> 4) + j;
        if (col < L.d_in) v = s.lin_in_w[(int64_t)row * L.d_in + col];
    } else if (i < L.off_lin_out) {
        const int64_t r = i - L.off_l512;
        const int layer = (int)(r / LAYER_FLOATS);
        const int e = (int)(r % LAYER_FLOATS);
        const int kb = e / KB_FLOATS, rt = (e / 256) % NRT, lane = (e >> 2) & 63, j = e & 3;
        const int row = 16 * rt + (lane & 15), col = 16 * kb + 4 * (lane >> 4) + j;
        v = s.w[layer][(int64_t)row * H + col];
    } else if (i < L.off_bias) {
        const int e = (int)(i - L.off_lin_out);
        const int kb = e >> 8, lane = (e >> 2) & 63, j = e & 3;
        const int row = lane & 15, col = 16 * kb + 4 * (lane >> 4) + j;
        if (row < L.d_out) v = s.lin_out_w[(int64_t)row * H + col];
    } else if (i >= L.off_out32) {
        const int e = (int)(i - L.off_out32);   // [input channel][output]
        const int ch = e >> 2, j = e & 3;
        if (j < L.d_out) v = s.lin_out_w[(int64_t)j * H + ch];
    } else {
        const int64_t r = i - L.off_bias;
        const int64_t nb = (int64_t)(1 + L.n_l512) * H;
        if (r < H) v = s.lin_in_b[r];
        else if (r < nb) v = s.b[r / H - 1][r % H];
        else if (r - nb < L.d_out) v = s.lin_out_b[r - nb];
    }
    out[i] = v;
}

// Split packer: one thread per (layer, k-step, row tile, lane) -> 8 weights
// W[16 rt + (lane & 15)][32 ks + 8 (lane >> 4) + j], each split exactly into three
// bf16 parts w = w0 + w1 + w2 (RNE), stored part-major: [ks][rt][part][lane][8].
__device__ __forceinline__ unsigned short bf16_rne(float x) {
    unsigned u = __float_as_uint(x);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf16_to_f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

__global__ void k_pack_split(PackSrc s, Layout L, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_in = (int64_t)KS32_IN * NRT * 64;
    const int64_t n_l = (int64_t)KS32 * NRT * 64;
    if (t >= n_in + L.n_l512 * n_l) return;
    int layer, ks, rt, lane;
    float *dst;
    if (t < n_in) {
        layer = -1;
        ks = (int)(t / (NRT * 64)); rt = (int)((t / 64) % NRT); lane = (int)(t % 64);
        dst = out + L.off_lin_in + (int64_t)ks * SKS_FLOATS + rt * SRT_FLOATS + lane * 4;
    } else {
        const int64_t r = t - n_in;
        layer = (int)(r / n_l);
        const int64_t e = r % n_l;
        ks = (int)(e / (NRT * 64)); rt = (int)((e / 64) % NRT); lane = (int)(e % 64);
        dst = out + L.off_l512 + layer * L.layer_floats + (int64_t)ks * SKS_FLOATS + rt * SRT_FLOATS + lane * 4;
    }
    const int row = 16 * rt + (lane & 15);
    unsigned short p[3][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = 32 * ks + 8 * (lane >> 4) + j;
        float w = 0.f;
        if (layer < 0) { if (col < L.d_in) w = s.lin_in_w[(int64_t)row * L.d_in + col]; }
        else w = s.w[layer][(int64_t)row * H + col];
        const unsigned short h0 = bf16_rne(w);
        const float r1 = w - bf16_to_f(h0);
        const unsigned short h1 = bf16_rne(r1);
        const float r2 = r1 - bf16_to_f(h1);
        p[0][j] = h0; p[1][j] = h1; p[2][j] = bf16_rne(r2);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        uint4 v;
        v.x = p[q][0] | ((unsigned)p[q][1] << 16); v.y = p[q][2] | ((unsigned)p[q][3] << 16);
        v.z = p[q][4] | ((unsigned)p[q][5] << 16); v.w = p[q][6] | ((unsigned)p[q][7] << 16);
        *reinterpret_cast<uint4 *>(dst + q * 256) = v;
    }
}

// Scaled-fp16 mode: per packed layer, the power-of-two exponent eW with
// max|W| * 2^eW <= 2^14 (fp16 max 65504), clamped to [-64, 40].  One block per layer
// (block 0 = lin_in, 1 + j = packed 512-wide layer j, 1 + n_l512 = lin_out), written
// to the pack header slot HDR_ESCALE + block as a float.
__device__ __forceinline__ int scale_exp(float m) {
    if (!(m > 0.f) || !(m < 3.0e38f)) return 0;       // zero / inf / nan: unscaled
    int e = 14 - __builtin_amdgcn_frexp_expf(m);      // m < 2^frexp_exp
    return e < -64 ? -64 : (e > 40 ? 40 : e);
}
// pass 1: max |w| per layer (blockIdx.y = layer block as above), grid-strided over
// blockIdx.x, combined with an integer atomicMax on the float bits (|w| >= 0) in the
// header slot (zeroed by the host first)
__global__ void k_layer_absmax(PackSrc s, Layout L, float *__restrict__ out) {
    const int layer = (int)blockIdx.y - 1;
    const float *w = layer < 0 ? s.lin_in_w : s.w[layer];
    const int64_t n = layer < 0 ? (int64_t)H * L.d_in : (int64_t)H * H;
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(w[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0)
        atomicMax(reinterpret_cast<unsigned *>(out + HDR_ESCALE + blockIdx.y), __float_as_uint(m));
}
// pass 2: max -> scale exponent (as a float) in place
__global__ void k_layer_escale(int n_slots, float *__restrict__ out) {
    const int i = threadIdx.x;
    if (i < n_slots) out[HDR_ESCALE + i] = (float)scale_exp(out[HDR_ESCALE + i]);
}

// One thread per (layer, k-step, row tile, lane): 8 weights w * 2^eW, each split
// into two fp16 parts w0 = f16(w), w1 = f16(w - w0) (RNE), [ks][rt][part][lane][8].
// (lin_out is not split: the head reads it in fp32 from off_out32.)
__global__ void k_pack_f16(PackSrc s, Layout L, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_in = (int64_t)KS32_IN * NRT * 64;
    const int64_t n_l = (int64_t)KS32 * NRT * 64;
    const int64_t n_all = n_in + L.n_l512 * n_l;
    if (t >= n_all) return;
    int layer, ks, rt, lane;
    float *dst;
    if (t < n_in) {
        layer = -1;
        ks = (int)(t / (NRT * 64)); rt = (int)((t / 64) % NRT); lane = (int)(t % 64);
        dst = out + L.off_lin_in + (int64_t)ks * SKS16_FLOATS + rt * SRT16_FLOATS + lane * 4;
    } else {
        const int64_t r = t - n_in;
        layer = (int)(r / n_l);
        const int64_t e = r % n_l;
        ks = (int)(e / (NRT * 64)); rt = (int)((e / 64) % NRT); lane = (int)(e % 64);
        dst = out + L.off_l512 + layer * L.layer_floats + (int64_t)ks * SKS16_FLOATS + rt * SRT16_FLOATS + lane * 4;
    }
    const int ew = (int)out[HDR_ESCALE + 1 + layer];
    const int row = 16 * rt + (lane & 15);
    _Float16 p[2][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = 32 * ks + 8 * (lane >> 4) + j;
        float w = 0.f;
        if (layer < 0) { if (col < L.d_in) w = s.lin_in_w[(int64_t)row * L.d_in + col]; }
        else w = s.w[layer][(int64_t)row * H + col];
        const float ws = __builtin_ldexpf(w, ew);
        const _Float16 h0 = (_Float16)ws;
        p[0][j] = h0;
        p[1][j] = (_Float16)(ws - (float)h0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        typedef _Float16 h8t __attribute__((ext_vector_type(8)));
        h8t v = {p[q][0], p[q][1], p[q][2], p[q][3], p[q][4], p[q][5], p[q][6], p[q][7]};
        *reinterpret_cast<h8t *>(dst + q * 256) = v;
    }
}

// Backward (training) pack: W^T of every packed 512-wide layer in the k_pack_f16 fragment
// layout, so that IN-gradient = W^T OUT-gradient runs on the forward's GEMM.  One thread
// per (layer, k-step, row tile, lane): A[16 rt + (lane & 15)][32 ks + 8 (lane >> 4) + j] =
// W[32 ks + 8 (lane >> 4) + j][16 rt + (lane & 15)] * 2^eW, eW from the forward pack's
// header (max |W^T| = max |W|).  Output: n_l512 layers of layer_floats, no header.
__global__ void k_pack_f16_t(PackSrc s, Layout L, const float *__restrict__ hdr, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_l = (int64_t)KS32 * NRT * 64;
    if (t >= L.n_l512 * n_l) return;
    const int layer = (int)(t / n_l);
    const int64_t e = t % n_l;
    const int ks = (int)(e / (NRT * 64)), rt = (int)((e / 64) % NRT), lane = (int)(e % 64);
    float *dst = out + layer * L.layer_floats + (int64_t)ks * SKS16_FLOATS + rt * SRT16_FLOATS + lane * 4;
    const int ew = (int)hdr[HDR_ESCALE + 1 + layer];
    const int col = 16 * rt + (lane & 15);
    typedef _Float16 h8t __attribute__((ext_vector_type(8)));
    h8t p0, p1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int row = 32 * ks + 8 * (lane >> 4) + j;
        const float ws = __builtin_ldexpf(s.w[layer][(int64_t)row * H + col], ew);
        const _Float16 h0 = (_Float16)ws;
        p0[j] = h0;
        p1[j] = (_Float16)(ws - (float)h0);
    }
    *reinterpret_cast<h8t *>(dst) = p0;
    *reinterpret_cast<h8t *>(dst + 256) = p1;
}

// ------------------------------------------------------------------------------
struct Args {
    const float *packed;
    Layout L;
    // points: render mode (rays + z) or query mode (xyz + dirs)
    int render_mode;
    const float *rays, *zs;
    int K;
    int64_t rays_per_obj;
    const float *xyz, *dirs;
    int64_t points_per_obj;
    int64_t n_points;
    // scene
    const float *latent, *cams;
    int ns, hl, wl;
    float img_w, img_h;
    float *out;
    float *xsum;       // scratch: gridDim.x x 2 x (COLS * H) floats (x park, multi-view sum)
    int64_t n_tiles;
    // training forward (NS == 1): activations for the backward, fp32 row-major [point][width]:
    //   features (64) | z (512) | relu(x) into fc_0 of block b (512 each) |
    //   relu(h) of block b (512 each) | relu(x) into lin_out (512)          (save_floats())
    float *save;
    // projected latent (k_latent_proj, PZ kernels): lin_z block b reads proj + b * proj_stride,
    // (n_obj * n_views, H_l, W_l, 512) like the latent
    const float *proj;
    int64_t proj_stride;
    // dynamic tile scheduling: 8 per-XCD tile counters, 64 B apart (zeroed per launch)
    int *tile_ctr;
    // fused ray march (render mode, K = 64 m.kpt): a workgroup takes a ray's kpt tiles in a
    // row, keeps their z and head outputs in LDS and composites the ray in the epilogue of
    // its last tile (march_epilogue); `out` may then be NULL (raw never reaches HBM)
    int march;
    MarchCfg m;
};

// floats of the activation save per point (Args::save): the fp32 regions, then the relu
// sign masks of the 2 nb + 1 relu slots, [slot][point][64 bytes] (save_mask's bit order)
// for the backward's masks
__host__ __device__ constexpr int64_t save_floats_per_point(int n_blocks) {
    return 64 + (int64_t)H * (2 + 2 * n_blocks) + 16 * (2 * n_blocks + 1);
}
__host__ __device__ constexpr int64_t save_mask_offset(int n_blocks, int64_t n_points) {
    return (64 + (int64_t)H * (2 + 2 * n_blocks)) * n_points;
}


__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef f4 Acc[RTW][CT];

// The lane index through an empty asm: per-lane LDS / global addresses derived from it are
// recomputed at each inlined use instead of hoisted out of the tile loop, where the 256
// registers of a wave at 2 waves per SIMD turned them into scratch spills whose reloads
// each cost a memory latency.
__device__ __forceinline__ int opaque_lane(int lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}

// relu(acc) of this wave's rows -> save slot [point][512] (points of this tile < n_points)
__device__ __forceinline__ void save_relu(const Acc &acc, float *slot, int64_t tile, int64_t n_points,
                                          int wave, int lane) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int64_t p = tile * COLS + 16 * c + cl;
        if (p >= n_points) continue;
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            const f4 v = acc[r][c];
#ifndef PNR_ABLATE_SAVEF   // diagnostic (training results invalid): no fp32 save-slot stores
            *reinterpret_cast<f4 *>(slot + p * H + 16 * (RTW * wave + r) + 4 * g) = relu4(v);
#endif
        }
    }
}

// [acc > 0] of this wave's rows -> mask slot [point][64 bytes].  Byte 8 wave + 2g + w of a
// point holds rows 16 (RTW wave + r) + 4g + e, r = 2w + h, at bit 4h + e: a lane's 16 bits
// are one contiguous 2-byte store per point, and a wave's 64 rows are one 8-byte word pair.
__device__ __forceinline__ void save_mask(const Acc &acc, uint32_t *mslot, int64_t tile, int64_t n_points,
                                          int wave, int lane) {
    static_assert(RTW == 4, "mask bytes assume 4 row tiles per wave");
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
    auto nib = [](const f4 &v) {
        return (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) | (v.w > 0.f ? 8u : 0u);
    };
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int64_t p = tile * COLS + 16 * c + cl;
        const uint32_t bits = nib(acc[0][c]) | (nib(acc[1][c]) << 4) | (nib(acc[2][c]) << 8) | (nib(acc[3][c]) << 12);
#ifndef PNR_ABLATE_SAVEM   // diagnostic (training results invalid): no relu-mask stores
        if (p < n_points)
            *reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(mslot) + p * 64 + 8 * wave + 2 * g) =
                (uint16_t)bits;
#else
        (void)bits;
#endif
    }
}

// acc[r][c] (+)= W(rows of this wave) * IN^T over nkb k-blocks.
//   wp  : this layer's packed weights, already offset to this wave's first row
//         tile and this lane (stride KB_FLOATS per k-block, 256 per row tile)
//   inb : LDS activation buffer, already offset to this lane's (column, k) slot
// Software pipeline: k-block kb+1's A (8 x f4) and B (4 x f4) are loaded while
// kb's 128 MFMAs issue.
template <int NK>
__device__ __forceinline__ void gemm(Acc &acc, const float *__restrict__ wp, const float *inb) {
    f4 A[RTW], B[CT];
#pragma unroll
    for (int r = 0; r < RTW; ++r) A[r] = *reinterpret_cast<const f4 *>(wp + r * 256);
#pragma unroll
    for (int c = 0; c < CT; ++c) B[c] = *reinterpret_cast<const f4 *>(inb + c * 16 * LDS_LD);
#pragma unroll 2
    for (int kb = 0; kb < NK; ++kb) {
        f4 An[RTW], Bn[CT];
        const int kn = kb + 1 < NK ? kb + 1 : kb;
#pragma unroll
        for (int r = 0; r < RTW; ++r)
            An[r] = *reinterpret_cast<const f4 *>(wp + (int64_t)kn * KB_FLOATS + r * 256);
#pragma unroll
        for (int c = 0; c < CT; ++c)
            Bn[c] = *reinterpret_cast<const f4 *>(inb + c * 16 * LDS_LD + kn * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int r = 0; r < RTW; ++r) acc[r][c] = mfma(A[r][j], B[c][j], acc[r][c]);
#pragma unroll
        for (int r = 0; r < RTW; ++r) A[r] = An[r];
#pragma unroll
        for (int c = 0; c < CT; ++c) B[c] = Bn[c];
    }
}

typedef float f8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f4 mfma_bf(bf8 a, bf8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split3(const f4 &lo, const f4 &hi, bf8 &x0, bf8 &x1, bf8 &x2) {
    const float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#ifdef PNR_ABLATE_SPLIT
    {   // diagnostic: hi part only (wrong numerics), no split VALU
        u4 p;
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = cvt_pk(x[2 * q], x[2 * q + 1]);
        x0 = x1 = x2 = __builtin_bit_cast(bf8, p);
        return;
    }
#endif
    u4 p0, p1, p2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned a, b, c;
        split_pair(x[2 * q], x[2 * q + 1], a, b, c);
        p0[q] = a;
        p1[q] = b;
        p2[q] = c;
    }
    x0 = __builtin_bit_cast(bf8, p0);
    x1 = __builtin_bit_cast(bf8, p1);
    x2 = __builtin_bit_cast(bf8, p2);
}

// workgroup barrier that waits only for LDS traffic: a __syncthreads() would also
// emit s_waitcnt vmcnt(0) and drain the weight prefetch that spans k-steps.  k_point_mlp
// uses it for every barrier: no wave there reads global memory another wave of the
// workgroup wrote (outputs, activation saves and per-wave scratch are written once per
// address), so global loads in flight (projected rows, biases) cross its barriers.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

constexpr int STG_FLOATS = CT * 3 * 256;   // one staging buffer: [ct][part][lane][8 bf16]
constexpr int A_DIST = 3;                          // weight prefetch distance (row tiles)
constexpr int A_RING = A_DIST < 4 ? 4 : 8;         // register ring (divides RTW = 8)

// Split-bf16 GEMM: acc[r][c] += sum over the NTERM largest products of the exact
// 3-way splits of W and IN (6 terms: error ~ fp32 unit roundoff; 9 terms: every
// product exact, only fp32 accumulation rounds) on v_mfma_f32_16x16x32_bf16.
//   wp   : packed layer + this wave's first row tile + lane*4 (floats)
//   inbw : LDS activations at (column 16*wave + cl, k 8g): the tile this wave splits
//   stg  : LDS staging ring, 2 x [ct][part][lane][8 bf16] (24 KB)
// Each wave splits ONE column tile of the next k-step into the staging ring (a
// quarter of the split VALU) and all waves read every tile's parts from it; A
// fragments stream from L2 three row tiles ahead into a 4-deep register ring.
template <int NKS, int NTERM>
__device__ __forceinline__ void gemm_split(Acc &acc, const float *__restrict__ wp, const float *inbw,
                                           float *stg, int wave, int lane) {
    bf8 ra[A_RING][3];
    auto loadA = [&](bf8 (&dst)[3], int ks, int r) {
#ifdef PNR_ABLATE_WSTREAM
        ks = 0;  // diagnostic: every k-step re-reads k-step 0 (L1/L2-hot), no weight stream
#endif
        const float *src = wp + (int64_t)ks * SKS_FLOATS + r * SRT_FLOATS;
#pragma unroll
        for (int q = 0; q < 3; ++q) dst[q] = *reinterpret_cast<const bf8 *>(src + q * 256);
    };
    // wave w splits the k-half w / 4 (4 values per lane) of column tile w % 4
    auto split_own = [&](int ks, int buf) {
        const float *bp = inbw + 32 * ks;
        const f4 v = *reinterpret_cast<const f4 *>(bp);
        unsigned a0, a1, a2, b0, b1, b2;
        split_pair(v.x, v.y, a0, a1, a2);
        split_pair(v.z, v.w, b0, b1, b2);
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        float *d = stg + buf * STG_FLOATS + (wave % CT) * 768 + lane * 4 + 2 * (wave / CT);
        *reinterpret_cast<u2 *>(d) = u2{a0, b0};
        *reinterpret_cast<u2 *>(d + 256) = u2{a1, b1};
        *reinterpret_cast<u2 *>(d + 512) = u2{a2, b2};
    };
    split_own(0, 0);
#pragma unroll
    for (int r = 0; r < A_DIST; ++r) loadA(ra[r], 0, r);
    lds_barrier();
#pragma unroll 1
    for (int ks = 0; ks < NKS; ++ks) {
        const int kn = ks + 1 < NKS ? ks + 1 : ks;   // branch-free tail: redundant re-split
        bf8 b0[CT], b1[CT], b2[CT];
        const float *sp = stg + (ks & 1) * STG_FLOATS + lane * 4;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
#ifdef PNR_ABLATE_STGREAD
            b0[c] = ra[0][c % 3]; b1[c] = ra[1][c % 3]; b2[c] = ra[2][c % 3];  // diagnostic
#else
            b0[c] = *reinterpret_cast<const bf8 *>(sp + c * 768);
            b1[c] = *reinterpret_cast<const bf8 *>(sp + c * 768 + 256);
            b2[c] = *reinterpret_cast<const bf8 *>(sp + c * 768 + 512);
#endif
        }
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            // split after the first row tile so its LDS reads don't gate the k-step start
            if (r == 1) split_own(kn, (ks + 1) & 1);
            const int rn = r + A_DIST;
            if (rn < RTW) loadA(ra[rn % A_RING], ks, rn);
            else loadA(ra[rn % A_RING], kn, rn - RTW);
            // keep the prefetch where it is: without the barrier the scheduler sinks
            // the loads next to their use to save registers and serializes the ring
            __builtin_amdgcn_sched_barrier(0);
            const bf8 *a = ra[r % A_RING];
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                f4 v = acc[r][c];
                if (NTERM >= 9) {
                    v = mfma_bf(a[2], b2[c], v);
                    v = mfma_bf(a[1], b2[c], v);
                    v = mfma_bf(a[2], b1[c], v);
                }
                v = mfma_bf(a[2], b0[c], v);
                v = mfma_bf(a[1], b1[c], v);
                v = mfma_bf(a[0], b2[c], v);
                v = mfma_bf(a[1], b0[c], v);
                v = mfma_bf(a[0], b1[c], v);
                v = mfma_bf(a[0], b0[c], v);
                acc[r][c] = v;
            }
        }
#ifndef PNR_ABLATE_KBARRIER
        lds_barrier();
#endif
    }
}

// ---- scaled-fp16 mode (PREC 3) -----------------------------------------------------
// W * 2^eW and every IN column * 2^e_col are split exactly enough into two fp16 parts
// (x = x0 + x1 + O(2^-22 x)); three products x0 y0 + x0 y1 + x1 y0 are exact in the
// f32 accumulate of v_mfma_f32_16x16x32_f16 (dropped x1 y1 < 2^-22 |x y|).  The
// power-of-two scales keep both operands in fp16's normal range (max <= 2^14) and are
// undone exactly on the fp32 accumulators.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 mfma_h(h8 a, h8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// fp16 residuals of a pair: f16(x - f32(h.lo)), f16(y - f32(h.hi)) by v_fma_mix{lo,hi}_f16
// (the fp16 operand widened in the instruction, one rounding of the exact difference: the
// same bits as subtracting in fp32 and converting, in 2 instructions instead of 5)
__device__ __forceinline__ unsigned resid_pk(unsigned h, float x, float y) {
    unsigned d;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h), "v"(x));
    asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(d) : "v"(h), "v"(y));
    return d;
}
// 4 values * s -> packed fp16 parts (2 dwords each): v_cvt_pk_f16_f32 (RNE), residuals
__device__ __forceinline__ void split_f16x4(const f4 &v, float s, u2 &p0, u2 &p1) {
    const f2 a = {v.x * s, v.y * s}, b = {v.z * s, v.w * s};
    const unsigned a0 = __builtin_bit_cast(unsigned, __builtin_convertvector(a, h2));
    const unsigned b0 = __builtin_bit_cast(unsigned, __builtin_convertvector(b, h2));
    p0 = u2{a0, b0};
    p1 = u2{resid_pk(a0, a.x, a.y), resid_pk(b0, b.x, b.y)};
}

// LDS image of the GEMM input in PREC 3: each activation column c scaled by 2^e_c and
// split ONCE by its producer into two fp16 parts, P0 / P1 = [column][ROWH halves]
// (4 B per element, the same as fp32).  The row pitch (1056 B = 66 x 16 B) makes the
// B-fragment ds_read_b128 of every lane group hit 16 distinct 16-B bank quads.
constexpr int ROWH = H + 16;                    // halves per column row
constexpr int PART_HALVES = COLS * ROWH;        // one part (67,584 B)
// Swizzle: the 16-B chunk index of element k (k >> 3) is XORed with (column >> 2) & 3.
// With the 1056-B pitch the B reads stay conflict-free and the producers' 8-B stores
// (16 columns x one chunk) drop from 4-way to 2-way bank conflicts.  k % 4 == 0.
__device__ __forceinline__ int swz(int col, int k) {
    return 8 * ((k >> 3) ^ ((col >> 2) & 3)) + (k & 7);
}

// acc[r][c] += (W 2^eW)(IN 2^e) over NKS k-steps of 32 from the pre-split LDS image:
// no staging, no split, no barrier inside the layer (waves run free).  A fragments
// stream from L2 A_DIST row tiles ahead; the last k-step is peeled so no load is in
// flight when the accumulators are handed back.
//   pb0 / pb1: P0 / P1 at (column cl, k 8g) of column tile 0
constexpr int H_DIST = 4;          // f16 weight prefetch distance (row tiles), every kernel: 4 measured
                                   // 1.7 % faster than 3 on the forward (5, 6 slower), and the training
                                   // step 1.2 % faster (17.29 -> 17.10 ms) although k_mlp_bwd spills
// The weight register ring of gemm_f16: row tile t = RTW * ks + r of the layer's stream lives
// in slot t % slots.  hring_prime issues the first DIST row tiles; gemm_f16_primed runs the
// layer on a primed ring.  Priming the next layer's ring before the publish that precedes it
// (k_point_mlp) lets those loads' L2 latency pass under the publish and its LDS-only barriers.
template <int DIST>
struct HRing {
    static constexpr int slots = DIST < RTW ? RTW : 2 * RTW;
    h8 ra[slots][2];
};

template <int DIST>
__device__ __forceinline__ void hring_load(HRing<DIST> &R, const float *__restrict__ wp, int slot, int ks, int r) {
#ifdef PNR_ABLATE_WSTREAM
    ks = 0;  // diagnostic: no weight stream
#endif
    const float *src = wp + (int64_t)ks * SKS16_FLOATS + r * SRT16_FLOATS;
    R.ra[slot][0] = *reinterpret_cast<const h8 *>(src);
    R.ra[slot][1] = *reinterpret_cast<const h8 *>(src + 256);
}

template <int DIST, int NKS = KS32>
__device__ __forceinline__ void hring_prime(HRing<DIST> &R, const float *__restrict__ wp) {
#pragma unroll
    for (int t = 0; t < DIST; ++t) hring_load(R, wp, t, (t / RTW) & (NKS - 1), t % RTW);
}

// Fair pipe sharing between the two waves of a SIMD (waves w and w ^ 4): each GEMM iteration a
// wave publishes its running iteration count in LDS and takes issue priority 1 while it is behind
// its SIMD-mate (the count read one iteration earlier), 0 otherwise.  At equal priority the older
// wave wins every MFMA slot, so without this the younger wave finished each layer alone, with a
// one-k-step weight prefetch that a solo wave's MFMA rate does not cover.
struct Fair {
    int *prog;   // LDS: iteration count per wave (8 ints)
    int wave, it, mate;
};
template <int NKS, int DIST = H_DIST>
__device__ __forceinline__ void gemm_f16_primed(Acc &acc, HRing<DIST> &R, const float *__restrict__ wp,
                                                const _Float16 *pb0, const _Float16 *pb1, Fair *F = nullptr) {
    constexpr int H_RING = HRing<DIST>::slots;   // register ring slots
    static_assert(DIST < H_RING && H_RING % RTW == 0, "ring");
    constexpr int U = H_RING / RTW;   // k-steps per loop iteration (static ring slots)
    static_assert(NKS % U == 0, "k-steps");
    static_assert((NKS & (NKS - 1)) == 0, "rotation mask");
    // one k-step; ph = ks % U (static), tail = this is one of the last U k-steps
    auto kstep = [&](int ks, auto ph_tag, auto tail_tag) {
        constexpr int ph = decltype(ph_tag)::value;
        constexpr bool tail = decltype(tail_tag)::value;
        h8 b0[CT], b1[CT];
        const int kr = ks & (NKS - 1);
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            b0[c] = *reinterpret_cast<const h8 *>(pb0 + c * 16 * ROWH + 32 * kr);
            b1[c] = *reinterpret_cast<const h8 *>(pb1 + c * 16 * ROWH + 32 * kr);
        }
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            const int tn = ph * RTW + r + DIST;            // prefetch target, relative to the iteration
            if (!tail || tn < U * RTW)
                hring_load(R, wp, tn % H_RING, (ks - ph + tn / RTW) & (NKS - 1), tn % RTW);
            __builtin_amdgcn_sched_barrier(0);
            const h8 *a = R.ra[(ph * RTW + r) % H_RING];
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                f4 v = acc[r][c];
                v = mfma_h(a[1], b0[c], v);
                v = mfma_h(a[0], b1[c], v);
                v = mfma_h(a[0], b0[c], v);
                acc[r][c] = v;
            }
        }
    };
    auto iter = [&](int ks0, auto tail_tag) {
        if (F) {
            const int it = ++F->it;
            // the mate's count loaded one iteration ago (its LDS latency passed under the MFMAs)
            if (it > __builtin_amdgcn_readfirstlane(F->mate)) __builtin_amdgcn_s_setprio(0);
            else __builtin_amdgcn_s_setprio(1);
            F->prog[F->wave] = it;
            F->mate = F->prog[F->wave ^ 4];
        }
        kstep(ks0, std::integral_constant<int, 0>{}, tail_tag);
        if constexpr (U > 1) kstep(ks0 + 1, std::integral_constant<int, 1>{}, tail_tag);
    };
#pragma unroll 1
    for (int ks = 0; ks + U < NKS; ks += U) iter(ks, std::false_type{});
    iter(NKS - U, std::true_type{});
    if (F) __builtin_amdgcn_s_setprio(0);
}

template <int NKS, int DIST = H_DIST>
__device__ __forceinline__ void gemm_f16(Acc &acc, const float *__restrict__ wp, const _Float16 *pb0,
                                         const _Float16 *pb1, Fair *F = nullptr) {
    HRing<DIST> R;
    hring_prime<DIST, NKS>(R, wp);
    gemm_f16_primed<NKS, DIST>(acc, R, wp, pb0, pb1, F);
}

// 4 (or 8) fp32 values -> scaled fp16 parts written to P0 / P1 at half offset `off`
__device__ __forceinline__ void put_split4(_Float16 *P0, _Float16 *P1, int off, const f4 &v, float s) {
    u2 p0, p1;
    split_f16x4(v, s, p0, p1);
    *reinterpret_cast<u2 *>(P0 + off) = p0;
    *reinterpret_cast<u2 *>(P1 + off) = p1;
}

// relu(acc) (RELU) or |acc| of this wave's rows -> per-column partial maxima cmax[column][wave slot]
template <bool RELU = true>
__device__ __forceinline__ void relu_colmax(const Acc &acc, float *cmax, int wave, int lane) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        float m = 0.f;   // max(0, ...) = the max of the relu'd values
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            f4 v = acc[r][c];
            if constexpr (!RELU) v = f4{fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
            m = max3_nc(max3_nc(m, v.x, v.y), v.z, v.w);
        }
        m = rows_max(m);
        if (g == 0) cmax[(16 * c + cl) * 8 + wave] = m;
    }
}

// after relu_colmax + barrier: relu(acc) (RELU) or acc, * 2^e_col split into P0 / P1 (this
// wave's rows), e_col -> ecol[column] (LDS, wave 0) and -> e_col (this lane's columns 16 c + cl:
// every wave computes the same exponents, so the next GEMM takes them from registers)
// A relu-publish store: lanes g and g ^ 1 (16 apart) hold rows 4g .. 4g + 3 of one column in
// both parts; one v_permlane16_swap per dword leaves the column's 8-row P0 chunk (16 B, k order)
// in the even lane and its P1 chunk in the odd one, stored with ONE ds_write_b128 at the lane's
// plane (Pl: P0 for even g, P1 for odd g).  Eight consecutive lanes then write eight distinct
// bank quads (the B-read swizzle), where two ds_write_b64 per lane were 2-way bank conflicted:
// the same bytes at the same addresses, half the LDS-array cycles.
__device__ __forceinline__ void put_split4_pair(_Float16 *Pl, int off, const f4 &v, float s) {
    u2 p0, p1;
#ifdef PNR_ABLATE_PUBSPLIT   // diagnostic (results invalid): the value bits stored, no split VALU
    p0 = u2{__float_as_uint(v.x), __float_as_uint(v.y)};
    p1 = u2{__float_as_uint(v.z), __float_as_uint(v.w)};
#else
    split_f16x4(v, s, p0, p1);
#endif
    const auto w0 = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
    const auto w1 = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
#ifdef PNR_ABLATE_PUBSTORE   // diagnostic (results invalid): the publish's image stores removed
    if ((w0[0] ^ w1[0] ^ w0[1] ^ w1[1]) == 0x12345u) *reinterpret_cast<u4 *>(Pl + off) = u4{w0[0], w1[0], w0[1], w1[1]};
#else
    *reinterpret_cast<u4 *>(Pl + off) = u4{w0[0], w1[0], w0[1], w1[1]};
#endif
}
template <bool RELU = true>
__device__ __forceinline__ void relu_store_split(const Acc &acc, _Float16 *P0, _Float16 *P1,
                                                 const float *cmax, int *ecol, int wave, int lane,
                                                 int (&e_col)[CT]) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
    // store bases of row tiles r = 0 and 1 (r + 2: +32 halves, the swizzle only XORs the low two
    // chunk bits; column tile c: +16 ROWH, the swizzle depends on column bits 2-3 only), so the
    // 16 stores take constant ds_write offsets
    _Float16 *Pl = (g & 1) ? P1 : P0;
    const int kb = 16 * RTW * wave + 4 * (g & ~1);
    _Float16 *q0 = Pl + cl * ROWH + swz(cl, kb), *q1 = Pl + cl * ROWH + swz(cl, kb + 16);
    // every column exponent first: a wave's LDS operations complete in order, so a cmax read
    // issued after stores waits for them (s_waitcnt lgkmcnt), which serialized the four column
    // tiles' reads behind the previous tiles' stores
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int col = 16 * c + cl;
#ifdef PNR_ABLATE_CMAXREAD   // diagnostic (results invalid): no column-maximum reads
        e_col[c] = 2 + (cl & 1);
#else
        const f4 m0 = *reinterpret_cast<const f4 *>(cmax + col * 8);
        const f4 m1 = *reinterpret_cast<const f4 *>(cmax + col * 8 + 4);
        e_col[c] = scale_exp(max3_nc(max3_nc(m0.x, m0.y, m0.z), max3_nc(m0.w, m1.x, m1.y), max_nc(m1.z, m1.w)));
#endif
    }
    if (wave == 0 && g == 0) {
#pragma unroll
        for (int c = 0; c < CT; ++c) ecol[16 * c + cl] = e_col[c];
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int col = 16 * c + cl;
        const float sc = __builtin_ldexpf(1.f, e_col[c]);
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            const f4 v = acc[r][c];
#ifdef PNR_ABLATE_PUBSPLIT
            const f4 o = v;
#else
            const f4 o = RELU ? relu4(v) : v;
#endif
            put_split4_pair((r & 1) ? q1 : q0, c * 16 * ROWH + (r >> 1) * 32, o, sc);
        }
    }
}

// this wave's rows of a bias vector (loaded ahead of use: the loads cross LDS-only barriers)
__device__ __forceinline__ void load_bias(f4 (&b)[RTW], const float *__restrict__ bias, int wave, int lane) {
    const int g = opaque_lane(lane) >> 4;
#pragma unroll
    for (int r = 0; r < RTW; ++r) b[r] = *reinterpret_cast<const f4 *>(bias + 16 * (RTW * wave + r) + 4 * g);
}
__device__ __forceinline__ void set_bias(Acc &acc, const f4 (&b)[RTW], bool accumulate) {
#pragma unroll
    for (int r = 0; r < RTW; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[r][c] = accumulate ? acc[r][c] + b[r] : b[r];
}

// acc = bias (per output row) [+ acc]
__device__ __forceinline__ void add_bias(Acc &acc, const float *__restrict__ bias, int wave, int lane,
                                         bool accumulate) {
    const int g = opaque_lane(lane) >> 4;
#pragma unroll
    for (int r = 0; r < RTW; ++r) {
#ifdef PNR_ABLATE_BIAS
        const f4 b = f4{0.01f, 0.02f, 0.03f, 0.04f} * (float)(r + 1);   // diagnostic: no bias loads
#else
        const f4 b = *reinterpret_cast<const f4 *>(bias + 16 * (RTW * wave + r) + 4 * g);
#endif
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[r][c] = accumulate ? acc[r][c] + b : b;
    }
}

// IN^T[column][row] = relu(acc) for this wave's rows (4 consecutive rows per lane)
__device__ __forceinline__ void store_relu(const Acc &acc, float *inbuf, int wave, int lane) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int r = 0; r < RTW; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const f4 v = acc[r][c];
            const f4 o = relu4(v);
            *reinterpret_cast<f4 *>(inbuf + (16 * c + cl) * LDS_LD + 16 * (RTW * wave + r) + 4 * g) = o;
        }
}

#ifdef PNR_PHASE_TIMING   // pnr_diag.h
constexpr int PT_SLOTS = 20;
__device__ unsigned long long g_phase[PT_SLOTS];
#endif

struct GemmCtx {
    int64_t wl_off, ws_off;   // f32 / split fragment offsets of this wave + lane
    const float *inb4;        // f32 B: column 16c + cl, k 16kb + 4g
    const float *inbw;        // split: own column tile 16*wave + cl, k 8g
    float *stg;               // split staging ring
    const float *hdr;         // pack header (PREC 3 weight scale exponents)
    const _Float16 *pb0, *pb1;  // PREC 3: P0 / P1 at (column cl, k 8g)
    const int *ecol;          // PREC 3: scale exponent of each IN column
    int ecl[CT];              // PREC 3: this lane's columns' exponents from the wave's last publish
    Fair fair;                // PREC 3 forward: pipe sharing with the SIMD-mate (fair.prog NULL: off)
    int wave, lane;
#ifdef PNR_PHASE_TIMING
    uint64_t pt[PT_SLOTS], pt_last;
#endif
};

// lin_z(z) - bias of the bilinear latent sample z of every column of the tile, staged in
// LDS as fp32 stage[column][LDS_LD]: resnetfc.py:160-163 on grid_sample's blend
// (encoder.py:102-108), evaluated by linearity as the blend of four rows of the projected
// latent P = latent W_z^T (proj.hip), torch's nw, ne, sw, se summation order.  Wave w blends
// the COLS / WAVES columns [8w, 8w + 8); each load instruction reads one contiguous 1 KB half
// of a corner's 2 KB row.  The stage aliases the GEMM input image, so the first loads are
// issued BEFORE the barrier that frees it and land while the wave waits for its SIMD-mate's
// GEMM; blends and LDS writes come after.
// The stage is run-deduplicated.  A wave's 8 columns are consecutive
// samples of one ray, and consecutive samples mostly project into the same latent cell
// (cfg3: 2.1 runs of equal cell per 8 columns, cfg2: 4.9): the 4 corner rows of a run are
// loaded ONCE and blended with each of its columns' weights (the blend arithmetic per column
// is unchanged).  Three register slots (96 VGPRs, the two-batch stage holds 128) rotate over
// the runs: runs 0-2 are issued before the barrier that frees the stage, run k + 3 as soon
// as run k's columns are blended.  The run pattern is wave-uniform (SGPR bit mask), so every
// branch below is a scalar branch.
struct CellRows {
    f4 c[2][4];   // [channel half][corner nw, ne, sw, se]
};
__device__ __forceinline__ void cell_load(CellRows &C, const float *__restrict__ pz, const float *gtab, int cj,
                                          int lane) {
    const f4 to = *reinterpret_cast<const f4 *>(gtab + cj * 8);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const uint32_t ch = half * 256 + opaque_lane(lane) * 4;
#ifdef PNR_ABLATE_GATHER   // diagnostic (results invalid): no projected-row loads
        C.c[half][0] = C.c[half][1] = C.c[half][2] = C.c[half][3] = to;
#else
        C.c[half][0] = *reinterpret_cast<const f4 *>(pz + __float_as_uint(to.x) + ch);
        C.c[half][1] = *reinterpret_cast<const f4 *>(pz + __float_as_uint(to.y) + ch);
        C.c[half][2] = *reinterpret_cast<const f4 *>(pz + __float_as_uint(to.z) + ch);
        C.c[half][3] = *reinterpret_cast<const f4 *>(pz + __float_as_uint(to.w) + ch);
#endif
    }
}
__device__ __forceinline__ void cell_blend_store(const CellRows &C, const float *gtab, float *stage, int cj,
                                                 int lane) {
    const f4 tw = *reinterpret_cast<const f4 *>(gtab + cj * 8 + 4);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const uint32_t ch = half * 256 + opaque_lane(lane) * 4;
        const f4 *c = C.c[half];
        f4 zz;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            zz[q] = add_rn(add_rn(add_rn(mul_rn(c[0][q], tw.x), mul_rn(c[1][q], tw.y)), mul_rn(c[2][q], tw.z)),
                           mul_rn(c[3][q], tw.w));
        *reinterpret_cast<f4 *>(stage + cj * LDS_LD + ch) = zz;
    }
}
// bit j set: column c0 + j starts a run (its nw corner offset, which fixes all four corners,
// differs from column c0 + j - 1's); bit 0 always set
__device__ __forceinline__ uint32_t cell_run_starts(const float *gtab, int c0) {
    uint32_t starts = 1u;
    uint32_t prev = __builtin_amdgcn_readfirstlane(__float_as_uint(gtab[c0 * 8]));
#pragma unroll
    for (int j = 1; j < COLS / WAVES; ++j) {
        const uint32_t k = __builtin_amdgcn_readfirstlane(__float_as_uint(gtab[(c0 + j) * 8]));
        if (k != prev) starts |= 1u << j;
        prev = k;
    }
    return starts;
}
// the whole stage of one wave, including the barrier that frees the image it aliases
__device__ __forceinline__ void stage_proj_runs(const float *__restrict__ pz, const float *gtab, float *stage,
                                                int wave, int lane) {
    constexpr int NC = COLS / WAVES;
    const int c0 = NC * wave;
    const uint32_t starts = cell_run_starts(gtab, c0);
    // first run start after column j (NC = none)
    auto next = [&](int j) -> int {
        const uint32_t m = starts & ~((2u << j) - 1u);
        return m ? __builtin_ctz(m) : NC;
    };
    CellRows A, B, C;
    int a = 0, b = next(0), c = b < NC ? next(b) : NC;
    cell_load(A, pz, gtab, c0 + a, lane);
    if (b < NC) cell_load(B, pz, gtab, c0 + b, lane);
    if (c < NC) cell_load(C, pz, gtab, c0 + c, lane);
    lds_barrier();   // the previous GEMM's image reads are done: the stage may overwrite it
    int j = 0;
    for (;;) {
        // A holds the run [a, b), B [b, c), C [c, d)
        const int d = c < NC ? next(c) : NC;
        for (; j < b; ++j) cell_blend_store(A, gtab, stage, c0 + j, lane);
        if (j >= NC) break;
        if (d < NC) cell_load(A, pz, gtab, c0 + d, lane);
        const int e = d < NC ? next(d) : NC;
        for (; j < c; ++j) cell_blend_store(B, gtab, stage, c0 + j, lane);
        if (j >= NC) break;
        if (e < NC) cell_load(B, pz, gtab, c0 + e, lane);
        const int f = e < NC ? next(e) : NC;
        for (; j < d; ++j) cell_blend_store(C, gtab, stage, c0 + j, lane);
        if (j >= NC) break;
        if (f < NC) cell_load(C, pz, gtab, c0 + f, lane);
        a = d;
        b = e;
        c = f;
    }
}
static_assert(sizeof(float) * COLS * LDS_LD <= 2 * sizeof(_Float16) * PART_HALVES,
              "the fp32 stage fits in the split image it aliases");
// x[r][c] += stage rows of this wave (column 16c + cl, rows 16 (RTW wave + r) + 4g ..)
__device__ __forceinline__ void add_stage(Acc &x, const float *stage, int wave, int lane) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int r = 0; r < RTW; ++r)
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const f4 v = *reinterpret_cast<const f4 *>(stage + (16 * c + cl) * LDS_LD + 16 * (RTW * wave + r) + 4 * g);
            f4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = add_rn(x[r][c][q], v[q]);
            x[r][c] = o;
        }
}

// hidx: header slot of the layer's weight scale (0 lin_in, 1 + packed 512-wide index).
// R: a ring primed (hring_prime) on this layer's weights, or nullptr (PREC 3 only).
// OWN (PREC 3, the input image written by the wave's last publish): the column exponents come from
// that publish's registers (g.ecl) instead of LDS, so the accumulator scaling does not wait on a read.
template <int PREC, int NK, int DIST = H_DIST, bool OWN = false>
__device__ __forceinline__ void layer_gemm(Acc &acc, const float *layer_base, GemmCtx &g, int hidx,
                                           HRing<DIST> *R = nullptr) {
    PT(g, 3);
    PT_COUNT(g, 5);
    if constexpr (PREC == 0) {
        gemm<NK>(acc, layer_base + g.wl_off, g.inb4);
    } else if constexpr (PREC == 3) {
        // the accumulators run in the products' scale 2^(eW + e_col): exact for powers of
        // two, so the fp32 rounding sequence is that of the unscaled sum
        const int cl = opaque_lane(g.lane) & 15;
        const int ew = (int)g.hdr[HDR_ESCALE + hidx];
        float sa[CT], ia[CT];
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const int e = (OWN ? g.ecl[c] : g.ecol[16 * c + cl]) + ew;
            sa[c] = __builtin_ldexpf(1.f, e);
            ia[c] = __builtin_ldexpf(1.f, -e);
        }
#pragma unroll
        for (int r = 0; r < RTW; ++r)
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                acc[r][c] *= sa[c];
            }
        Fair *F = g.fair.prog ? &g.fair : nullptr;
        if (R) gemm_f16_primed<NK / 2, DIST>(acc, *R, layer_base + opaque_lane((int)g.ws_off), g.pb0, g.pb1, F);
        else gemm_f16<NK / 2, DIST>(acc, layer_base + opaque_lane((int)g.ws_off), g.pb0, g.pb1, F);
#pragma unroll
        for (int r = 0; r < RTW; ++r)
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                acc[r][c] *= ia[c];
            }
    } else {
        gemm_split<NK / 2, PREC>(acc, layer_base + g.ws_off, g.inbw, g.stg, g.wave, g.lane);
    }
    PT(g, 2);
}

// One lane's global atomic add of 1 to *p; the old value is returned to every lane.  The lane mask
// is narrowed and restored inside the asm, so the caller is straight-line code with no divergent
// region.  (The tile claim was `if (tid == 0) *s_next = grab();`: ROCm 7.2's register allocator
// placed a spill of the thread id in that branch's join block BEFORE its EXEC restore, so only
// lane 0 stored it and every other lane reloaded stale scratch -- the round-5 illegal-address
// faults.  isa_lint.py now rejects any build with a spill in that position.)  Called by a whole
// wave with every lane active, so lane 0 is the lane that adds.
__device__ __forceinline__ int claim_one(int *p) {
    int old;
    unsigned long long saved;
    asm volatile(
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "s_nop 4\n\t"
        "global_atomic_add %0, %2, %3, off sc0\n\t"
        "s_mov_b64 exec, %1\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_nop 4"
        : "=&v"(old), "=&s"(saved)
        : "v"(p), "v"(1)
        : "memory");
    return __builtin_amdgcn_readfirstlane(old);
}

// The march config read where it is used (kernarg s_loads through a pointer the compiler cannot
// see through): hoisted out of the tile loop, its ~30 loop-invariant dwords held SGPRs across
// the GEMMs and spilled them (256 SGPR spills, 40 B/lane of VGPR scratch against 16).
typedef const __attribute__((address_space(4))) MarchCfg *CfgPtr;
// (k_point_mlp's only parameter is Args, so Args::m sits at offsetof(Args, m) in the kernarg
// segment; taking &a instead would copy the whole by-value Args to the stack)
__device__ __forceinline__ CfgPtr march_cfg(const Args &) {
    uint64_t v = (uint64_t)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() +
                            offsetof(Args, m));
    asm volatile("" : "+s"(v));
    return (CfgPtr)v;
}
__device__ __forceinline__ RngSrc ld_rng(const __attribute__((address_space(4))) RngSrc &r) {
    RngSrc o;
    o.p = r.p;
    o.seed = r.seed;
    o.offset = r.offset;
    o.stream = r.stream;
    return o;
}
// Fused ray march, one wave: composite ray b from the z / head outputs its kpt tiles left in
// LDS (buf: z [128] | raw [128][4]; nf: near, far) with the standalone composite's code
// (composite_wave), then, in a coarse pass that feeds a fine pass, draw the ray's fine
// samples (sample_fine_wave) from the weights it just computed (scr: w | cdf | sort).  The
// Philox draws come first: they depend only on the ray, so their latency overlaps the
// composite's.
template <int S>
__device__ __forceinline__ void march_ray(const Args &a, int64_t b, const float *buf, const float *nf, float *scr,
                                          int lane, bool fine_pass) {
    const CfgPtr c = march_cfg(a);
    EPI_DECL
    const int kf = fine_pass ? 0 : c->kf;   // the single-launch fine pass draws nothing
    FineDraws d = {0.f, 0.f, 0.f};
    if (kf > 0) d = fine_draws(lane, b, kf, c->kfd, ld_rng(c->u_fine), ld_rng(c->u_jit), ld_rng(c->n_depth));
    const float near = nf[0], far = nf[1];
    float zk[S], wk[S];
    f4 v[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {   // composite_wave's lane ownership: sample 64 i + lane
        zk[i] = buf[64 * i + lane];
        v[i] = *reinterpret_cast<const f4 *>(buf + 128 + 4 * (64 * i + lane));
    }
    const float depth = fine_pass
        ? composite_wave<S>(lane, b, COLS * S, far, zk, v, c->white_bkgd, c->weights_f, c->rgb_f, c->depth_f, wk)
        : composite_wave<S>(lane, b, COLS * S, far, zk, v, c->white_bkgd, c->weights, c->rgb, c->depth, wk);
    EPI_T(0);
#ifdef PNR_EPI_TIMING
    if (lane == 0) atomicAdd(&g_epi[7], 1ull);
#endif
    if (kf > 0) {
        float *w = scr;
#pragma unroll
        for (int i = 0; i < S; ++i) w[64 * i + lane] = wk[i];
        wave_lds_sync();
        // single launch: the sorted fine depths also go to buf's z region (whose coarse depths
        // composite_wave and the sort's inputs have consumed) for the ray's fine tiles
        sample_fine_wave(lane, b, near, far, COLS * S, w, buf, depth, kf, c->kfd, c->depth_std, RngSrc{}, RngSrc{},
                         RngSrc{}, c->lindisp != 0, c->n_sort, scr + 128, scr + 256, nullptr, c->z_fine, nullptr,
                         nullptr, true, d, c->single ? const_cast<float *>(buf) : nullptr);
    }
}
__device__ __forceinline__ void march_epilogue(const Args &a, int64_t b, const float *buf, const float *nf,
                                               float *scr, int lane, bool fine_pass) {
    if ((fine_pass ? march_cfg(a)->kpt_f : march_cfg(a)->kpt) == 1) march_ray<1>(a, b, buf, nf, scr, lane, fine_pass);
    else march_ray<2>(a, b, buf, nf, scr, lane, fine_pass);
}

// PZ: lin_z from the projected latent (gather_proj) instead of the latent gather + GEMM;
// MARCH: the fused ray march (a.m), a separate instantiation so that the plain point model
// keeps its own register allocation
template <int PREC, bool PZ, bool MARCH>
__global__ __launch_bounds__(NTHR) void k_point_mlp(Args a) {
    constexpr int KD = H_DIST;   // weight ring distance
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *inbuf = smem;                   // COLS x LDS_LD
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int cl = lane & 15;
    const Layout &L = a.L;

    // per-lane fragment bases
    const int64_t wl_off = (int64_t)(RTW * wave) * 256 + lane * 4;         // f32 fragments
    const int64_t ws_off = (int64_t)(RTW * wave) * (PREC == 3 ? SRT16_FLOATS : SRT_FLOATS) + lane * 4;
    const float *inb = inbuf + cl * LDS_LD + 4 * g;     // B (f32): column 16c + cl, k 16kb + 4g
    GemmCtx gc;
    gc.wl_off = wl_off;
    gc.ws_off = ws_off;
    gc.inb4 = inb;
    gc.inbw = inbuf + (16 * (wave % CT) + cl) * LDS_LD + 8 * g + 4 * (wave / CT);
    gc.stg = inbuf + COLS * LDS_LD;
    // PREC 3 LDS: P0 | P1 | gtab | cmax | ecol; else: inbuf (fp32) | staging | gtab
    _Float16 *P0 = reinterpret_cast<_Float16 *>(smem);
    _Float16 *P1 = P0 + PART_HALVES;
    float *gtab = PREC == 3 ? reinterpret_cast<float *>(P1 + PART_HALVES) : gc.stg + 2 * STG_FLOATS;
    float *cmax = gtab + COLS * 8;           // PREC 3: per-column partial maxima (64 x 8)
    int *ecol = reinterpret_cast<int *>(cmax + COLS * 8);
    // PE freqs [0, 16) / phases [16, 32) of the pack header, in LDS: the feature loop indexes
    // them per lane, and vector global loads there put a memory latency in every iteration
    float *petab = PREC == 3 ? reinterpret_cast<float *>(ecol + COLS) : gtab + COLS * 8;
    // (the one-time LDS fills below are whole-wave writes -- lanes 32 apart store the same value --
    // rather than `if (tid < 32)` branches: no divergent region for a misplaced spill, claim_one)
    if (wave == 0) petab[lane & 31] = a.packed[lane & 31];   // visible after the first barrier of a tile
    gc.hdr = a.packed;
    // B fragment (column 16c + cl, k 32 ks + 8g): swz keeps it linear in ks and c
    gc.pb0 = P0 + cl * ROWH + swz(cl, 8 * g);
    gc.pb1 = P1 + cl * ROWH + swz(cl, 8 * g);
    gc.ecol = ecol;
    gc.fair.prog = nullptr;
    gc.fair.wave = wave;
    gc.fair.it = 0;
    gc.fair.mate = 0;
    if constexpr (PREC == 3) {
        gc.fair.prog = reinterpret_cast<int *>(petab + 40);   // petab + 32 / 33: s_next, + 64: hpart
        if (wave == 0) gc.fair.prog[lane & (WAVES - 1)] = 0;   // visible after the first barrier
    }
    gc.wave = wave;
    gc.lane = lane;
#ifdef PNR_PHASE_TIMING
    for (int i = 0; i < PT_SLOTS; ++i) gc.pt[i] = 0;
    gc.pt_last = __builtin_amdgcn_s_memtime();
#endif
    // feature role: thread -> (column col, part qt of WAVES); FPT features each
    constexpr int FPT = 64 / WAVES;

    // relu(acc) -> the next GEMM's input image (callers barrier before and after)
    // activation save slots (training forward)
    // Every region has PS = n_points * n_views rows: row v P + p holds (view v, point p) of
    // the per-view stages (features, z, the blocks before the combine layer), row p the
    // per-point stages after it (their other rows are unused).
    const int64_t P = a.n_points, PS = P * a.ns;
    float *sv_f = a.save, *sv_z = a.save ? a.save + PS * 64 : nullptr;
    auto sv_slot = [&](int i) { return sv_z + PS * H * (1 + i); };   // i: block b -> x_in, nb + b -> h, 2nb -> x_f
    uint32_t *sv_mask = a.save ? reinterpret_cast<uint32_t *>(a.save + save_mask_offset(L.n_blocks, PS)) : nullptr;
    // Barrier between a GEMM that reads the input image and the publish that rewrites it.
    // PREC 3's publish writes only its column maxima before its own internal barrier, and
    // the image after it, so there the barrier is redundant and waves that finish their GEMM
    // early start the publish VALU under their SIMD-mate's MFMAs.
    auto pre_publish_sync = [&]() {
#ifndef PNR_GEMM_ONLY
        if constexpr (PREC != 3)
#endif
            lds_barrier();
    };
    auto publish_relu = [&](const Acc &acc, int64_t tile, int save_idx, int64_t row0) {
        if (a.save) {
            save_relu(acc, sv_slot(save_idx) + row0 * H, tile, P, wave, lane);
            save_mask(acc, sv_mask + PS * 16 * save_idx + row0 * 16, tile, P, wave, lane);
        }
#ifdef PNR_GEMM_ONLY
        {   // diagnostic: GEMM chain only (garbage results); a checksum keeps acc live
            float t = 0.f;
#pragma unroll
            for (int r = 0; r < RTW; ++r)
#pragma unroll
                for (int c = 0; c < CT; ++c) t += acc[r][c].x + acc[r][c].y + acc[r][c].z + acc[r][c].w;
            cmax[tid & 511] = t;
            for (int c = 0; c < CT; ++c) gc.ecl[c] = -8;
            return;
        }
#endif
        if constexpr (PREC == 3) {
            // (phase-timing slots 17, 13-15, 16: glue split into the ring prime / bias loads
            // before the publish, colmax VALU, its barrier, the split, the closing barrier)
            PT(gc, 17);
            relu_colmax(acc, cmax, wave, lane);
            PT(gc, 13);
            lds_barrier();
            PT(gc, 14);
            relu_store_split(acc, P0, P1, cmax, ecol, wave, lane, gc.ecl);
            PT(gc, 15);
        } else {
            store_relu(acc, inbuf, wave, lane);
        }
    };

#ifdef PNR_GEMM_ONLY
    if (tid < COLS) ecol[tid] = -8;
    for (int i = tid; i < 2 * PART_HALVES; i += NTHR)   // nonzero operands (power / clock)
        P0[i] = (_Float16)(0.25f + 0.001f * (float)(i % 977));
    lds_barrier();
#endif
    Acc x, h;
    // Dynamic, XCD-aware tile order.  Workgroups are placed round-robin on the 8 XCDs
    // (blockIdx.x % 8); XCD x owns the contiguous tile range [x T / 8, (x + 1) T / 8)
    // (neighbouring tiles are neighbouring rays, which sample neighbouring latent pixels, so
    // each XCD's L2 holds its own band of the projected latent).  Its workgroups take tiles
    // from that range through an atomic counter and, once it is empty, from the other XCDs'
    // ranges: a slower CU or XCD no longer leaves the rest of the chip idle at the end of
    // the launch.  The next tile is fetched before the head, so the atomic's latency hides.
    int *s_next = reinterpret_cast<int *>(petab + 32);
    float *hpart = petab + 64;   // PREC 3 head: per-wave partials [wave][column][4] (8 KB)
    // fused march (MARCH): the ray's z [128] | head outputs [128][4], the epilogue scratch,
    // near / far.  (Deferring a ray's epilogue into the next tile, under the SIMD-mate's MFMAs,
    // was measured: the double buffers and the call inside the GEMM region cost more in spills
    // than it hid.)
    float *mreg = PREC == 3 ? hpart + 2048 : petab + 36;
    float *mscr = mreg + MARCH_BUF_FLOATS;
    float *mnf = mscr + 384;
    const int kpt = MARCH ? march_cfg(a)->kpt : 1;   // tiles per ray and pass when marching
    // tiles per scheduling unit (a ray when marching): its kpt tiles, and with the single-launch
    // march (m.single) its kpt_f fine tiles after them
    const bool single = MARCH && march_cfg(a)->single;
    const int upt = single ? kpt + march_cfg(a)->kpt_f : kpt;
    // single launch: the fine tiles' PE table from the fine pack's header (the packs
    // of two MLPs may carry different tables); visible after the first barrier
    float *petab_f = mnf + 4;
    if (single && wave == 1) petab_f[lane & 31] = march_cfg(a)->packed_f[lane & 31];
    // the next unit's first tile, claimed by wave 0 (wave-uniform: every value here is scalar)
    auto grab = [&]() -> int {
        const int64_t T = a.n_tiles / upt;
        const int x0 = blockIdx.x & 7;
        for (int k = 0; k < 8; ++k) {
            const int x = (x0 + k) & 7;
            const int64_t lo = x * T / 8, hi = (x + 1) * T / 8;
            if (lo >= hi) continue;
            const int64_t i = lo + claim_one(a.tile_ctr + 16 * x);
            if (i < hi) return (int)(i * upt);
        }
        return (int)a.n_tiles;
    };
    if (wave == 0) *s_next = grab();
    lds_barrier();
    for (int64_t tile = *s_next; tile < a.n_tiles; tile = *s_next) {
        // this tile within its unit: pass_f = a fine tile of the single-launch march; sub = the
        // tile within its pass (the ray's kpt_t tiles of K_t = 64 kpt_t samples)
        const int64_t unit = tile / upt;
        const int s_in = (int)(tile - unit * upt);
        const bool pass_f = single && s_in >= kpt;
        const int sub = pass_f ? s_in - kpt : s_in;
        const int kpt_t = pass_f ? march_cfg(a)->kpt_f : kpt;
        // MARCH: the unit's ray (pnr_render_cfg.ray_order; read at use, an L2-hit scalar load);
        // an entry out of range marches the unit's own index instead of faulting
        auto ray_of = [&]() -> int64_t {
            const int *o = MARCH ? march_cfg(a)->order : nullptr;
            if (!o) return unit;
            const int64_t r = o[unit];
            return r >= 0 && r < a.n_tiles / upt ? r : unit;
        };
        // the pass's pack and projected latent (read at use: no per-tile SGPR state)
        auto PK = [&]() -> const float * { return pass_f ? march_cfg(a)->packed_f : a.packed; };
        auto PJ_ = [&]() -> const float * { return pass_f ? march_cfg(a)->proj_f : a.proj; };
        const float *bias = PK() + L.off_bias;
        gc.hdr = PK();
        // per-workgroup scratch (L2-resident): [0] x parked during fc_0, [1] multi-view sum
        // (addresses formed at use: nothing per tile stays live across the GEMMs)
        auto xp_ptr = [&]() { return a.xsum + (int64_t)blockIdx.x * (2 * COLS * H) + wave * (RTW * CT * 256) + opaque_lane(lane) * 4; };
        auto xs_ptr = [&]() { return xp_ptr() + COLS * H; };

        for (int v = 0; v < a.ns; ++v) {
            // per view: keeps the feature addresses out of scratch across the GEMMs
            const int tid_t = opaque_lane(tid);
            const int col = tid_t / WAVES, qt = tid_t % WAVES;
            const int64_t p_raw = tile * COLS + col;
            const int64_t p = p_raw < a.n_points ? p_raw : a.n_points - 1;
            // the point (re-read per view from L2 rather than held in registers across the
            // per-view blocks' GEMMs)
            float px, py, pz, dx, dy, dz, zz = 0.f;
            int64_t obj;
            if (a.render_mode) {
                // ray b, sample kk of its pass (MARCH: the unit's ray, K = 64 kpt_t)
                const int64_t b = MARCH ? ray_of() : p / a.K;
                const int kk = MARCH ? sub * COLS + col : (int)(p - b * a.K);
                const int kt = MARCH ? COLS * kpt_t : a.K;
                const float *ray = a.rays + b * 8;
                if (MARCH && pass_f) {
                    // single launch: the coarse epilogue left the ray's sorted fine depths in
                    // mreg (its wave joins this barrier after writing them)
                    lds_barrier();
                    zz = mreg[kk];
                } else if (MARCH && march_cfg(a)->sample_coarse) {
                    // the coarse draw in the prologue (nerf.py:98-118), or the given depth
                    const CfgPtr m = march_cfg(a);
                    zz = coarse_z(ld_rng(m->u_coarse), b, kt, kk, ray[6], ray[7], m->lindisp != 0);
                    float *zo = m->z_out;
                    if (zo && qt == 0 && v == 0) zo[b * kt + kk] = zz;
                } else {
                    zz = a.zs[b * kt + kk];
                }
                dx = ray[3]; dy = ray[4]; dz = ray[5];
                // points = o + z * d  (nerf.py:185)
                px = add_rn(ray[0], mul_rn(zz, dx));
                py = add_rn(ray[1], mul_rn(zz, dy));
                pz = add_rn(ray[2], mul_rn(zz, dz));
                obj = b / a.rays_per_obj;
            } else {
                px = a.xyz[p * 3 + 0]; py = a.xyz[p * 3 + 1]; pz = a.xyz[p * 3 + 2];
                if (a.dirs) { dx = a.dirs[p * 3 + 0]; dy = a.dirs[p * 3 + 1]; dz = a.dirs[p * 3 + 2]; }
                else { dx = dy = dz = 0.f; }
                obj = p / a.points_per_obj;
            }
            PT_WAIT();
            PT(gc, 8);
            // ---- per (point, view) geometry (this thread's column) ----------------
            const float *cam = a.cams + (obj * a.ns + v) * 16;
            float xr[3], vd[3], xc[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float r0 = cam[3 * i], r1 = cam[3 * i + 1], r2 = cam[3 * i + 2];
                xr[i] = add_rn(add_rn(mul_rn(r0, px), mul_rn(r1, py)), mul_rn(r2, pz));
                vd[i] = add_rn(add_rn(mul_rn(r0, dx), mul_rn(r1, dy)), mul_rn(r2, dz));
                xc[i] = add_rn(xr[i], cam[9 + i]);
            }
            const float fx = cam[12], fy = cam[13], cx = cam[14], cy = cam[15];
            PT_WAIT();
            PT(gc, 9);
            // features f = FPT qt .. FPT qt + FPT - 1 of [xyz_rot | PE | viewdir_cam | 0]
            lds_barrier();   // previous users of inbuf are done
            PT(gc, 10);
            if (MARCH && qt == 0 && v == 0) {   // for the epilogue
                if (!pass_f) mreg[sub * COLS + col] = zz;
                if (col == 0 && sub == 0) {
                    const float *rr = a.rays + ray_of() * 8;
                    mnf[0] = rr[6];
                    mnf[1] = rr[7];
                }
            }
            {
                const int npe = 3 * L.pe_n;
                const float *pet = MARCH && pass_f ? petab_f : petab;   // this pass's PE table
                float fv[FPT];
#pragma unroll
                for (int i = 0; i < FPT; ++i) {
                    const int f = FPT * qt + i;
                    float val = 0.f;
                    if (f < 3) val = xr[f];
                    else if (f < 3 + npe) {
                        const int m = f - 3, q = m / 3, d = m - 3 * q;
                        const float xd = d == 0 ? xr[0] : (d == 1 ? xr[1] : xr[2]);
                        val = sinf(add_rn(pet[16 + q], mul_rn(xd, pet[q])));   // code._phases, _freqs
                    } else if (f < 6 + npe) {
                        const int d = f - 3 - npe;
                        val = d == 0 ? vd[0] : (d == 1 ? vd[1] : vd[2]);
                    }
                    fv[i] = val;
                }
                if (a.save && p_raw < a.n_points) {
#pragma unroll
                    for (int i = 0; i < FPT / 4; ++i)
                        *reinterpret_cast<f4 *>(sv_f + (v * P + p_raw) * 64 + FPT * qt + 4 * i) =
                            f4{fv[4 * i], fv[4 * i + 1], fv[4 * i + 2], fv[4 * i + 3]};
                }
                if constexpr (PREC == 3) {
                    // column max over its WAVES feature threads (adjacent lanes), scale, split
                    float m = 0.f;
#pragma unroll
                    for (int i = 0; i < FPT; ++i) m = fmaxf(m, fabsf(fv[i]));
#pragma unroll
                    for (int o = 1; o < WAVES; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
                    const int e = scale_exp(m);
                    const float sc = __builtin_ldexpf(1.f, e);
#pragma unroll
                    for (int i = 0; i < FPT / 4; ++i)
                        put_split4(P0, P1, col * ROWH + swz(col, FPT * qt + 4 * i),
                                   f4{fv[4 * i], fv[4 * i + 1], fv[4 * i + 2], fv[4 * i + 3]}, sc);
                    if (qt == 0) ecol[col] = e;
                } else {
#pragma unroll
                    for (int i = 0; i < FPT / 4; ++i)
                        *reinterpret_cast<f4 *>(inbuf + col * LDS_LD + FPT * qt + 4 * i) =
                            f4{fv[4 * i], fv[4 * i + 1], fv[4 * i + 2], fv[4 * i + 3]};
                }
            }
            PT(gc, 11);
            // projection (models.py:206-212) -> grid_sample coords (encoder.py:95-108)
            float u = mul_rn(__fdiv_rn(-xc[0], xc[2]), fx);
            float w = mul_rn(__fdiv_rn(-xc[1], xc[2]), fy);
            u = add_rn(u, cx);
            w = add_rn(w, cy);
            const float wlf = (float)a.wl, hlf = (float)a.hl;
            const float lsx = mul_rn(__fdiv_rn(wlf, sub_rn(wlf, 1.f)), 2.f);
            const float lsy = mul_rn(__fdiv_rn(hlf, sub_rn(hlf, 1.f)), 2.f);
            const float gx = sub_rn(mul_rn(u, __fdiv_rn(lsx, a.img_w)), 1.f);
            const float gy = sub_rn(mul_rn(w, __fdiv_rn(lsy, a.img_h)), 1.f);
            float ix = mul_rn(add_rn(gx, 1.f), mul_rn(sub_rn(wlf, 1.f), 0.5f));
            float iy = mul_rn(add_rn(gy, 1.f), mul_rn(sub_rn(hlf, 1.f), 0.5f));
            ix = fminf(fmaxf(ix, 0.f), wlf - 1.f);   // border padding; NaN -> 0
            iy = fminf(fmaxf(iy, 0.f), hlf - 1.f);
            const float x0f = floorf(ix), y0f = floorf(iy);
            const float we = sub_rn(ix, x0f), wn = sub_rn(iy, y0f);
            const float ee = sub_rn(1.f, we), ss = sub_rn(1.f, wn);
            float wnw = mul_rn(ss, ee), wne = mul_rn(ss, we), wsw = mul_rn(wn, ee), wse = mul_rn(wn, we);
            const int x0 = (int)x0f, y0 = (int)y0f;
            const int x1 = x0 + 1 < a.wl ? x0 + 1 : x0, y1 = y0 + 1 < a.hl ? y0 + 1 : y0;
            if (x0 + 1 >= a.wl) { wne = 0.f; wse = 0.f; }
            if (y0 + 1 >= a.hl) { wsw = 0.f; wse = 0.f; }
            if (qt == 0) {
                // per-column gather record: 4 corner offsets (floats from a.latent) + weights
                const uint32_t base = (uint32_t)((obj * a.ns + v) * (int64_t)a.hl * a.wl * H);
                const uint32_t o00 = base + (uint32_t)(y0 * a.wl + x0) * H, o01 = base + (uint32_t)(y0 * a.wl + x1) * H;
                const uint32_t o10 = base + (uint32_t)(y1 * a.wl + x0) * H, o11 = base + (uint32_t)(y1 * a.wl + x1) * H;
                float *t = gtab + col * 8;
                *reinterpret_cast<f4 *>(t) = f4{__uint_as_float(o00), __uint_as_float(o01),
                                                __uint_as_float(o10), __uint_as_float(o11)};
                *reinterpret_cast<f4 *>(t + 4) = f4{wnw, wne, wsw, wse};
            }
            PT(gc, 12);
            lds_barrier();   // features visible
            PT(gc, 0);
            // ---- lin_in ---------------------------------------------------------------
            add_bias(x, bias, wave, lane, false);
            layer_gemm<PREC, NKB_IN, KD>(x, PK() + L.off_lin_in, gc, 0);
            // ---- blocks before the combine layer: x += lin_z(z); x = block(x) ------
            for (int blk = 0; blk < L.ncomb; ++blk) {
                const int lz = layer_index(blk, 0, L.ncomb);
                if constexpr (PZ) {
                    // the stage aliases the image the previous GEMM read; publish_relu's
                    // internal barrier orders the add_stage reads before the image writes
                    const float *pz = PJ_() + blk * a.proj_stride;
                    stage_proj_runs(pz, gtab, inbuf, wave, lane);
                    PT(gc, 3);
                    lds_barrier();
                    PT(gc, 1);
                    add_bias(x, bias + (1 + lz) * H, wave, lane, true);
                    add_stage(x, inbuf, wave, lane);
                } else {
                lds_barrier();
                PT(gc, 3);
                // z = bilinear latent gather (torch's nw, ne, sw, se summation order).
                // Wave w walks its COLS / WAVES columns; each load instruction reads one
                // contiguous 1 KB half of a corner's 2 KB channel row (lane = 4 channels).
#ifdef PNR_GEMM_ONLY
                if (0)
#endif
#pragma unroll 4
                for (int j = 0; j < COLS / WAVES; ++j) {
                    const int cj = (COLS / WAVES) * wave + j;
                    const f4 to = *reinterpret_cast<const f4 *>(gtab + cj * 8);
                    const f4 tw = *reinterpret_cast<const f4 *>(gtab + cj * 8 + 4);
                    f4 zh[2];
#pragma unroll
                    for (int half = 0; half < 2; ++half) {
                        const uint32_t ch = half * 256 + opaque_lane(lane) * 4;
#ifdef PNR_ABLATE_GATHER
                        const f4 c0 = tw, c1 = to, c2 = tw, c3 = to;  // diagnostic
#else
                        const f4 c0 = *reinterpret_cast<const f4 *>(a.latent + __float_as_uint(to.x) + ch);
                        const f4 c1 = *reinterpret_cast<const f4 *>(a.latent + __float_as_uint(to.y) + ch);
                        const f4 c2 = *reinterpret_cast<const f4 *>(a.latent + __float_as_uint(to.z) + ch);
                        const f4 c3 = *reinterpret_cast<const f4 *>(a.latent + __float_as_uint(to.w) + ch);
#endif
                        f4 zz;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            zz[q] = add_rn(add_rn(add_rn(mul_rn(c0[q], tw.x), mul_rn(c1[q], tw.y)),
                                                  mul_rn(c2[q], tw.z)), mul_rn(c3[q], tw.w));
                        if constexpr (PREC == 3) zh[half] = zz;
                        else *reinterpret_cast<f4 *>(inbuf + cj * LDS_LD + ch) = zz;
                        if (a.save && blk == 0 && tile * COLS + cj < P)
                            *reinterpret_cast<f4 *>(sv_z + (v * P + tile * COLS + cj) * H + ch) = zz;
                    }
                    if constexpr (PREC == 3) {
                        // column max over the wave (all 512 channels), scale, split
                        float m = 0.f;
#pragma unroll
                        for (int hf = 0; hf < 2; ++hf)
                            m = fmaxf(m, fmaxf(fmaxf(fabsf(zh[hf][0]), fabsf(zh[hf][1])),
                                               fmaxf(fabsf(zh[hf][2]), fabsf(zh[hf][3]))));
                        m = wave_max(m);
                        const int e = scale_exp(m);
                        const float sc = __builtin_ldexpf(1.f, e);
                        put_split4(P0, P1, cj * ROWH + swz(cj, lane * 4), zh[0], sc);
                        put_split4(P0, P1, cj * ROWH + swz(cj, 256 + lane * 4), zh[1], sc);
                        if (lane == 0) ecol[cj] = e;
                    }
                }
                lds_barrier();
                PT(gc, 1);
                add_bias(x, bias + (1 + lz) * H, wave, lane, true);
                layer_gemm<PREC, NKB, KD>(x, PK() + L.off_l512 + (int64_t)lz * L.layer_floats, gc, 1 + lz);
                pre_publish_sync();
                }
                HRing<KD> R0;   // fc_0's ring, primed before or during the publish (PREC 3)
                const float *w0p = PK() + L.off_l512 + (int64_t)(lz + 1) * L.layer_floats;
                if constexpr (PREC == 3) hring_prime(R0, w0p + opaque_lane((int)gc.ws_off));
                f4 nb0[RTW];   // fc_0's bias rows, loaded before the publish too
                load_bias(nb0, bias + (2 + lz) * H, wave, lane);
                publish_relu(x, tile, blk, v * P);
                lds_barrier();
                PT(gc, 16);
                set_bias(h, nb0, false);
                layer_gemm<PREC, NKB, KD, PREC == 3>(h, PK() + L.off_l512 + (int64_t)(lz + 1) * L.layer_floats, gc, 2 + lz,
                                          PREC == 3 ? &R0 : nullptr);
                pre_publish_sync();
                HRing<KD> R1;   // fc_1's
                const float *w1p = PK() + L.off_l512 + (int64_t)(lz + 2) * L.layer_floats;
                if constexpr (PREC == 3) hring_prime(R1, w1p + opaque_lane((int)gc.ws_off));
                f4 nb1[RTW];
                load_bias(nb1, bias + (3 + lz) * H, wave, lane);
                publish_relu(h, tile, L.n_blocks + blk, v * P);
                lds_barrier();
                PT(gc, 16);
                set_bias(x, nb1, true);
                layer_gemm<PREC, NKB, KD, PREC == 3>(x, PK() + L.off_l512 + (int64_t)(lz + 2) * L.layer_floats, gc, 3 + lz,
                                          PREC == 3 ? &R1 : nullptr);
            }
            // ---- multi-view mean (combine_interleaved: sum over views, then / NS) --
            if (a.ns > 1) {
                float *xs = xs_ptr();
                if (v == 0) {
#pragma unroll
                    for (int r = 0; r < RTW; ++r)
#pragma unroll
                        for (int c = 0; c < CT; ++c)
                            *reinterpret_cast<f4 *>(xs + (r * CT + c) * 256) = x[r][c];
                } else if (v < a.ns - 1) {
#pragma unroll
                    for (int r = 0; r < RTW; ++r)
#pragma unroll
                        for (int c = 0; c < CT; ++c) {
                            f4 *ptr = reinterpret_cast<f4 *>(xs + (r * CT + c) * 256);
                            *ptr = *ptr + x[r][c];
                        }
                } else {
                    const float nsf = (float)a.ns;
#pragma unroll
                    for (int r = 0; r < RTW; ++r)
#pragma unroll
                        for (int c = 0; c < CT; ++c) {
                            const f4 sum = *reinterpret_cast<const f4 *>(xs + (r * CT + c) * 256) + x[r][c];
                            x[r][c] = sum / nsf;
                        }
                }
            }
        }
        // ---- blocks after the combine layer ------------------------------------------
        for (int blk = L.ncomb; blk < L.n_blocks; ++blk) {
            const int l0 = layer_index(blk, 1, L.ncomb);
            pre_publish_sync();
            HRing<KD> R0;
            const float *w0p = PK() + L.off_l512 + (int64_t)l0 * L.layer_floats;
            if constexpr (PREC == 3) hring_prime(R0, w0p + opaque_lane((int)gc.ws_off));
            f4 nb0[RTW];
            load_bias(nb0, bias + (1 + l0) * H, wave, lane);
            publish_relu(x, tile, blk, 0);
            lds_barrier();
            PT(gc, 16);
            set_bias(h, nb0, false);
            layer_gemm<PREC, NKB, KD, PREC == 3>(h, PK() + L.off_l512 + (int64_t)l0 * L.layer_floats, gc, 1 + l0,
                                      PREC == 3 ? &R0 : nullptr);
            pre_publish_sync();
            HRing<KD> R1;
            const float *w1p = PK() + L.off_l512 + (int64_t)(l0 + 1) * L.layer_floats;
            if constexpr (PREC == 3) hring_prime(R1, w1p + opaque_lane((int)gc.ws_off));
            f4 nb1[RTW];
            load_bias(nb1, bias + (2 + l0) * H, wave, lane);
            publish_relu(h, tile, L.n_blocks + blk, 0);
            lds_barrier();
            PT(gc, 16);
            set_bias(x, nb1, true);
            layer_gemm<PREC, NKB, KD, PREC == 3>(x, PK() + L.off_l512 + (int64_t)(l0 + 1) * L.layer_floats, gc, 2 + l0,
                                      PREC == 3 ? &R1 : nullptr);
        }
        // ---- lin_out(relu(x)) + head [sigmoid(rgb), relu(sigma)]: wave w < CT -> columns 16w..
        if (wave == 0) *s_next = s_in + 1 < upt ? (int)tile + 1 : grab();   // read after the closing barrier
        pre_publish_sync();
        if constexpr (PREC == 3) {
            // no publish: the head reads relu(x) from the accumulators (below); only the
            // activation save of lin_out's input remains
            if (a.save) {
                save_relu(x, sv_slot(2 * L.n_blocks), tile, P, wave, lane);
                save_mask(x, sv_mask + PS * 16 * (2 * L.n_blocks), tile, P, wave, lane);
            }
        } else {
            publish_relu(x, tile, 2 * L.n_blocks, 0);
            lds_barrier();
        }
        PT(gc, 16);
        PT(gc, 3);
#ifdef PNR_GEMM_ONLY
        if (0)
#endif
        if (PREC == 3) {
            // fp32 head straight from the accumulators (resnetfc.py:184 lin_out on relu(x)):
            // lane (g, cl) holds rows 16 (RTW wave + r) + 4 g + i of column 16 c + cl; it sums
            // W_out^T (fp32, [channel][output] at off_out32) times relu(x) over its 16 rows, then
            // over the wave's four lane rows (rows_sum), and lane row g stores column tile g's
            // partial at hpart[wave][column][output]; after the closing barrier waves 0-3 add the
            // 8 waves' partials in wave order.  Replaces the last layer's colmax / split publish
            // and the split-fp16 head GEMM (the k_point_mlp round-4 head change).
            const int ln = opaque_lane(lane), g4 = ln >> 4, c16 = ln & 15;
            const float *w32 = PK() + L.off_out32;
            f4 o[CT];
#pragma unroll
            for (int c = 0; c < CT; ++c) o[c] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < RTW; ++r) {
                const f4 *wr = reinterpret_cast<const f4 *>(w32 + 4 * (16 * (RTW * wave + r) + 4 * g4));
                const f4 w[4] = {wr[0], wr[1], wr[2], wr[3]};
#pragma unroll
                for (int c = 0; c < CT; ++c) {
                    const f4 v = relu4(x[r][c]);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) o[c][j] = fmaf(v[i], w[i][j], o[c][j]);
                }
            }
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j) o[c][j] = rows_sum(o[c][j]);
            const f4 mine = g4 == 0 ? o[0] : g4 == 1 ? o[1] : g4 == 2 ? o[2] : o[3];
            *reinterpret_cast<f4 *>(hpart + (wave * COLS + 16 * g4 + c16) * 4) = mine;
        } else if (PREC != 3 && wave < CT) {   // wave-uniform: the first CT waves own one column tile each
            const float *wo = PK() + L.off_lin_out + lane * 4;
            const float *bi = inbuf + (16 * wave + cl) * LDS_LD + 4 * g;
            f4 o0 = *reinterpret_cast<const f4 *>(bias + (1 + L.n_l512) * H + 4 * g);
            f4 o1 = {0.f, 0.f, 0.f, 0.f}, o2 = o1, o3 = o1;
#pragma unroll 4
            for (int kb = 0; kb < NKB; ++kb) {
                const f4 wv = *reinterpret_cast<const f4 *>(wo + kb * 256);
                const f4 bv = *reinterpret_cast<const f4 *>(bi + kb * 16);
                o0 = mfma(wv.x, bv.x, o0);
                o1 = mfma(wv.y, bv.y, o1);
                o2 = mfma(wv.z, bv.z, o2);
                o3 = mfma(wv.w, bv.w, o3);
            }
            const f4 o = (o0 + o1) + (o2 + o3);
            const int64_t po = tile * COLS + 16 * wave + cl;
            if (g == 0 && po < a.n_points) {
                f4 r;
                r.x = __fdiv_rn(1.f, add_rn(1.f, expf(-o.x)));
                r.y = __fdiv_rn(1.f, add_rn(1.f, expf(-o.y)));
                r.z = __fdiv_rn(1.f, add_rn(1.f, expf(-o.z)));
                r.w = max_nc(o.w, 0.f);   // torch.relu: NaN stays NaN
                if (!MARCH || a.out)   // MARCH: the ray's own points (ray_order)
                    *reinterpret_cast<f4 *>(a.out + (MARCH ? ray_of() * (COLS * kpt_t) + sub * COLS + 16 * wave + cl
                                                           : po) * 4) = r;
                if (MARCH) *reinterpret_cast<f4 *>(mreg + 128 + 4 * (sub * COLS + 16 * wave + cl)) = r;
            }
        }
        PT(gc, 4);
        PT_COUNT(gc, 6);
        lds_barrier();   // s_next and the head partials written
        if (PREC == 3 && wave < CT) {   // [sigmoid(rgb), relu(sigma)] of column tile `wave`
            const int ln = opaque_lane(lane), gg = ln >> 4, cc = ln & 15;
            const int col = 16 * wave + cc;
            f4 o = *reinterpret_cast<const f4 *>(hpart + col * 4);
#pragma unroll
            for (int w = 1; w < WAVES; ++w) o = o + *reinterpret_cast<const f4 *>(hpart + (w * COLS + col) * 4);
            const f4 b = *reinterpret_cast<const f4 *>(bias + (1 + L.n_l512) * H + 4 * gg);
            o = o + b;
            const int64_t po = tile * COLS + col;
            if (gg == 0 && po < a.n_points) {
                f4 r;
                r.x = __fdiv_rn(1.f, add_rn(1.f, expf(-o.x)));
                r.y = __fdiv_rn(1.f, add_rn(1.f, expf(-o.y)));
                r.z = __fdiv_rn(1.f, add_rn(1.f, expf(-o.z)));
                r.w = max_nc(o.w, 0.f);   // torch.relu: NaN stays NaN
                if (!MARCH || a.out)   // MARCH: the ray's own points (ray_order)
                    *reinterpret_cast<f4 *>(a.out + (MARCH ? ray_of() * (COLS * kpt_t) + sub * COLS + col : po) * 4) = r;
                if (MARCH) *reinterpret_cast<f4 *>(mreg + 128 + 4 * (sub * COLS + 16 * wave + cc)) = r;
            }
        }
        // ---- fused march: the ray's last tile composites it (and draws its fine samples) --
        if (MARCH && sub == kpt_t - 1) {   // the ray's last tile of this pass
            lds_barrier();   // the ray's head outputs visible
            if (wave == WAVES - 1) march_epilogue(a, ray_of(), mreg, mnf, mscr, opaque_lane(lane), pass_f);
        }
    }
#ifdef PNR_PHASE_TIMING
    if (threadIdx.x == 64 * PNR_PT_WAVE)   // the recorded wave
        for (int i = 0; i < PT_SLOTS; ++i) atomicAdd(&g_phase[i], (unsigned long long)gc.pt[i]);
#endif
}

// ---- training backward of ResnetFC (resnetfc.py:132-184, n_views == 1), PREC 3 -------------
// Per 64-point tile, the input-gradient chain in reverse block order on the forward's GEMM
// (W^T packed by k_pack_f16_t, the LDS image holding the signed gradient), with the relu
// masks read from the forward's activation save:
//   dx = (d_o W_out) . [x_f > 0]       (masks: the forward's sign bits, save_mask)
//   for b = nb-1 .. 0:  dY(fc_1 b) = dx
//                       dh = (W_1^T dx) . [h_b > 0]              dY(fc_0 b) = dh
//                       dx = dx + (W_0^T dh) . [x_b > 0]
//                       b < n_linz:  dY(lin_z b) = dx,  dzlat += W_z^T dx
//   dY(lin_in) = dx
// With NS > 1 source views (resnetfc.py:151-172, util.combine_interleaved) the blocks from
// combine_layer on run once per point; dL/d(view mean) / NS then enters the chain of the blocks
// before it once per view, on the forward save's view rows v P + p (masks, dY, dzlat).  View 0
// stores that value as its first dY slot (dY(fc_1, ncomb - 1)); views 1.. reload it from there.
// The output gradients dY of every layer go to global memory for the weight gradients
// (dW = dY^T IN over the points) and the bias gradients (column sums).  Slot order, chosen
// so that those are strided batched GEMMs over the save's slots:
//   dy[b] = dY(fc_0 b),  dy[nb] = dY(lin_in),  dy[nb + 1 + b] = dY(fc_1 b);
//   dY(lin_z b) = dy[nb + b] (the same values).
struct BwdArgs {
    const float *hdr;        // forward pack (header: weight scale exponents)
    const float *packed_t;   // k_pack_f16_t output
    const float *w_out;      // lin_out weight (4 x 512, fp32)
    const float *save;       // forward activation save (Args::save)
    const float *d_o;        // (P, 4) gradient of the pre-head output
    float *dy;               // (2 nb + 1) x (NS P) x 512; the slots of the blocks from combine_layer
                             // on use their first P rows
    float *dzlat;            // (NS P, 512) gradient of the sampled latent (n_linz > 0)
    float *bsum;             // NULL, or [workgroup][2 nb + 1][512] column sums of each dy slot
                             // over the workgroup's tiles (its tiles in order: deterministic)
    Layout L;
    int64_t n_points, n_tiles;
    int ns;                  // source views per point (the save's view rows)
};

// sum over the 16 lanes of a DPP row (every lane gets it; lane 0's order is the fixed tree
// ((a + a8) + (a4 + a12)) + ...)
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0x128>(0.f, v);   // row_ror:8
    v += dpp_f<0x124>(0.f, v);   // row_ror:4
    v += dpp_f<0x122>(0.f, v);   // row_ror:2
    v += dpp_f<0x121>(0.f, v);   // row_ror:1
    return v;
}

// this wave's rows of acc -> slot [point][512] (points < n_points)
__device__ __forceinline__ void store_rows(const Acc &acc, float *slot, int64_t tile, int64_t n_points,
                                           int wave, int lane, float *bs = nullptr, bool first = false) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int64_t p = tile * COLS + 16 * c + cl;
        if (p >= n_points) continue;
#pragma unroll
        for (int r = 0; r < RTW; ++r)
            *reinterpret_cast<f4 *>(slot + p * H + 16 * (RTW * wave + r) + 4 * g) = acc[r][c];
    }
    if (bs) {   // bias gradient: this tile's column sums of the wave's rows, added to bs
        f4 sr[RTW];
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            f4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < CT; ++c)
                if (tile * COLS + 16 * c + cl < n_points) t += acc[r][c];
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = row16_sum(t[e]);
            sr[r] = t;
        }
        if (cl == 0) {
#pragma unroll
            for (int r = 0; r < RTW; ++r) {
                f4 *q = reinterpret_cast<f4 *>(bs + 16 * (RTW * wave + r) + 4 * g);
                *q = first ? sr[r] : *q + sr[r];
            }
        }
    }
}
// relu backward masks from the forward's sign bits (save_mask): this lane's two words of
// each of its CT points, loaded before the GEMM whose output they mask
typedef unsigned u2m __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void load_mask(u2m (&mk)[CT], const uint32_t *mslot, int64_t tile, int64_t n_points,
                                          int wave, int lane) {
    const int cl = opaque_lane(lane) & 15;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const int64_t p = tile * COLS + 16 * c + cl;
        const int64_t pc = p < n_points ? p : n_points - 1;
        mk[c] = *reinterpret_cast<const u2m *>(mslot + pc * 16 + 2 * wave);
    }
}
// acc *= [activation > 0] (torch's relu backward); 0 past n_points
__device__ __forceinline__ void relu_mask(Acc &acc, const u2m (&mk)[CT], int64_t tile, int64_t n_points,
                                          int lane) {
    lane = opaque_lane(lane);
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        const bool valid = tile * COLS + 16 * c + cl < n_points;
#pragma unroll
        for (int r = 0; r < RTW; ++r) {
            // byte 2g + (r >> 1) of the wave's 8 bytes, bit 4 (r & 1) + e
            const int byte = 2 * g + (r >> 1);
            const uint32_t nib = valid ? (byte >= 4 ? mk[c].y : mk[c].x) >> (8 * (byte & 3) + 4 * (r & 1)) : 0u;
            const f4 v = acc[r][c];
            acc[r][c] = f4{(nib & 1u) ? v.x : 0.f, (nib & 2u) ? v.y : 0.f, (nib & 4u) ? v.z : 0.f,
                           (nib & 8u) ? v.w : 0.f};
        }
    }
}

__global__ __launch_bounds__(NTHR) void k_mlp_bwd(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, cl = lane & 15;
    const Layout &L = a.L;
    const int nb = L.n_blocks;
    const int64_t P = a.n_points, PS = P * a.ns;
    // blocks [nc, nb) run per point, [0, nc) per view (all per point when NS == 1)
    const int nc = a.ns > 1 ? L.ncomb : 0;
    // LDS: P0 | P1 | cmax | ecol (as the forward's PREC 3 layout, no gather records)
    _Float16 *P0 = reinterpret_cast<_Float16 *>(smem);
    _Float16 *P1 = P0 + PART_HALVES;
    float *cmax = reinterpret_cast<float *>(P1 + PART_HALVES);
    int *ecol = reinterpret_cast<int *>(cmax + COLS * 8);
    GemmCtx gc = {};
    gc.ws_off = (int64_t)(RTW * wave) * SRT16_FLOATS + lane * 4;
    gc.hdr = a.hdr;
    gc.pb0 = P0 + cl * ROWH + swz(cl, 8 * g);
    gc.pb1 = P1 + cl * ROWH + swz(cl, 8 * g);
    gc.ecol = ecol;
    gc.fair.prog = nullptr;
    gc.fair.wave = wave;
    gc.fair.it = 0;
    gc.fair.mate = 0;
    {
        gc.fair.prog = ecol + COLS;   // 8 ints after ecol (the launch's LDS size counts them)
        if (threadIdx.x < WAVES) gc.fair.prog[threadIdx.x] = 0;
    }
    gc.wave = wave;
    gc.lane = lane;
    // relu sign masks of the forward: slot b: relu(x_b), nb + b: relu(h_b), 2 nb: x_f; every
    // region has PS rows (view rows v P + p before combine_layer)
    const uint32_t *msk = reinterpret_cast<const uint32_t *>(a.save + save_mask_offset(nb, PS));
    auto mask_slot = [&](int i, int64_t row0) { return msk + PS * 16 * i + row0 * 16; };
    u2m mk[CT];
    auto dy_slot = [&](int i, int64_t row0) { return a.dy + PS * H * i + row0 * H; };
    auto bs_slot = [&](int i) -> float * {
        return a.bsum ? a.bsum + ((int64_t)blockIdx.x * (2 * nb + 1) + i) * H : nullptr;
    };
    auto publish = [&](const Acc &acc) {
        // no barrier first: the column maxima are written before the internal barrier and the
        // image after it, when every wave has left the GEMM that read the previous image
        relu_colmax<false>(acc, cmax, wave, lane);
        __syncthreads();
        relu_store_split<false>(acc, P0, P1, cmax, ecol, wave, lane, gc.ecl);
        __syncthreads();
    };
    auto zero = [](Acc &acc) {
#pragma unroll
        for (int r = 0; r < RTW; ++r)
#pragma unroll
            for (int c = 0; c < CT; ++c) acc[r][c] = f4{0.f, 0.f, 0.f, 0.f};
    };
    auto layer = [&](int li) { return a.packed_t + (int64_t)li * L.layer_floats; };

    Acc x, h;
    // segments of the chain: NS == 1: blocks nb-1 .. 0; else blocks nb-1 .. nc per point, then
    // nc-1 .. 0 once per view on its rows v P + p
    const int n_seg = a.ns == 1 ? 1 : 1 + a.ns;
    for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const bool first_tile = tile == blockIdx.x;
        {   // dx = (d_o W_out) . [x_f > 0]
            load_mask(mk, mask_slot(2 * nb, 0), tile, P, wave, lane);
            f4 wo[4][RTW];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < RTW; ++r)
                    wo[j][r] = *reinterpret_cast<const f4 *>(a.w_out + j * H + 16 * (RTW * wave + r) + 4 * g);
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                const int64_t p = tile * COLS + 16 * c + cl;
                const f4 d = p < P ? *reinterpret_cast<const f4 *>(a.d_o + p * 4) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < RTW; ++r)
                    x[r][c] = ((d.x * wo[0][r] + d.y * wo[1][r]) + d.z * wo[2][r]) + d.w * wo[3][r];
            }
            relu_mask(x, mk, tile, P, lane);
        }
        for (int sgi = 0; sgi < n_seg; ++sgi) {
            const int v = sgi - 1;   // the view of a per-view segment
            const int b_hi = sgi == 0 ? nb : nc, b_lo = sgi == 0 ? nc : 0;
            const int64_t row0 = v > 0 ? (int64_t)v * P : 0;
            // the first store of the workgroup to the bias partials of these slots
            const bool first = first_tile && v <= 0;
            if (v == 0) {   // torch.mean's backward: dL/d(mean) / NS to every view
                const float inv = (float)a.ns;
#pragma unroll
                for (int r = 0; r < RTW; ++r)
#pragma unroll
                    for (int c = 0; c < CT; ++c) x[r][c] = x[r][c] / inv;
            } else if (v > 0 && nc > 0) {   // the same, as view 0 stored it (this lane's own rows)
                const float *src = dy_slot(nb + nc, 0);
                const int ln = opaque_lane(lane), gz = ln >> 4;
#pragma unroll
                for (int c = 0; c < CT; ++c) {
                    const int64_t p = tile * COLS + 16 * c + (ln & 15);
                    const int64_t pc = p < P ? p : P - 1;
#pragma unroll
                    for (int r = 0; r < RTW; ++r)
                        x[r][c] = *reinterpret_cast<const f4 *>(src + pc * H + 16 * (RTW * wave + r) + 4 * gz);
                }
            }
            bool published = false;
            for (int b = b_hi - 1; b >= b_lo; --b) {
                if (!published) publish(x);
                store_rows(x, dy_slot(nb + 1 + b, row0), tile, P, wave, lane, bs_slot(nb + 1 + b), first);
                const int l1 = layer_index(b, 2, L.n_linz), l0 = layer_index(b, 1, L.n_linz);
                zero(h);
                load_mask(mk, mask_slot(nb + b, row0), tile, P, wave, lane);   // lands during the GEMM
                layer_gemm<3, NKB, H_DIST, true>(h, layer(l1), gc, 1 + l1);
                relu_mask(h, mk, tile, P, lane);
                store_rows(h, dy_slot(b, row0), tile, P, wave, lane, bs_slot(b), first);
                publish(h);
                zero(h);
                load_mask(mk, mask_slot(b, row0), tile, P, wave, lane);
                layer_gemm<3, NKB, H_DIST, true>(h, layer(l0), gc, 1 + l0);
                relu_mask(h, mk, tile, P, lane);
#pragma unroll
                for (int r = 0; r < RTW; ++r)
#pragma unroll
                    for (int c = 0; c < CT; ++c) x[r][c] += h[r][c];
                published = false;
                if (b < L.n_linz) {
                    publish(x);
                    published = true;
                    const int lz = layer_index(b, 0, L.n_linz);
                    zero(h);
                    layer_gemm<3, NKB, H_DIST, true>(h, layer(lz), gc, 1 + lz);
                    const bool zfirst = b == L.n_linz - 1;
#pragma unroll
                    for (int c = 0; c < CT; ++c) {
                        const int ln = opaque_lane(lane), gz = ln >> 4;
                        const int64_t p = tile * COLS + 16 * c + (ln & 15);
                        if (p >= P) continue;
#pragma unroll
                        for (int r = 0; r < RTW; ++r) {
                            f4 *q = reinterpret_cast<f4 *>(a.dzlat + (row0 + p) * H + 16 * (RTW * wave + r) + 4 * gz);
                            *q = zfirst ? h[r][c] : *q + h[r][c];
                        }
                    }
                }
            }
            if (b_lo == 0) store_rows(x, dy_slot(nb, row0), tile, P, wave, lane, bs_slot(nb), first);
        }
    }
}

// d_bias[i] = sum over the workgroups of their column-sum partials.  One workgroup per 64
// columns (coalesced 256-B rows), BIAS_SLICES waves each summing a strided slice of the
// workgroup partials, then the slices added in slice order through LDS: a fixed order, so
// the result is deterministic.  The one-thread-per-column loop it replaces was a chain of
// n_wg dependent loads on 22 workgroups (≈0.1 ms per launch, 58 GB/s).
constexpr int BIAS_SLICES = 16;
__global__ void __launch_bounds__(64 * BIAS_SLICES)
k_bias_reduce(const float *__restrict__ part, int n_wg, int n, float *__restrict__ out) {
    __shared__ float acc[BIAS_SLICES][64];
    const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + c;
    float s0 = 0.f, s1 = 0.f;
    if (t < n) {
        int w = sl;
        for (; w + BIAS_SLICES < n_wg; w += 2 * BIAS_SLICES) {
            s0 += part[(int64_t)w * n + t];
            s1 += part[(int64_t)(w + BIAS_SLICES) * n + t];
        }
        if (w < n_wg) s0 += part[(int64_t)w * n + t];
    }
    acc[sl][c] = s0 + s1;
    __syncthreads();
    if (sl == 0 && t < n) {
        float s = acc[0][c];
#pragma unroll
        for (int k = 1; k < BIAS_SLICES; ++k) s += acc[k][c];
        out[t] = s;
    }
}

}  // namespace mlpk

// ------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------
#ifdef PNR_EPI_TIMING
extern "C" int pnr_debug_epi(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(::g_epi), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    static const unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(::g_epi), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef PNR_PHASE_TIMING
// diagnostic: copy (and optionally clear) the phase counters; not part of the ABI
extern "C" int pnr_debug_phase(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mlpk::g_phase), sizeof(unsigned long long) * mlpk::PT_SLOTS) != hipSuccess)
        return -1;
    if (reset) {
        static const unsigned long long zero[mlpk::PT_SLOTS] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mlpk::g_phase), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
size_t mlp_packed_bytes(const pnr_mlp_desc &d) {
    return sizeof(float) * (size_t)mlpk::make_layout(d).total;
}

int mlp_check_desc(const pnr_mlp_desc &d) {
    if (d.d_hidden != mlpk::H || d.d_latent != mlpk::H)
        return fail(PNR_ERR_UNSUPPORTED, "fused MLP implements d_hidden = d_latent = 512 (got %d, %d)",
                    d.d_hidden, d.d_latent);
    if (d.d_out != 4) return fail(PNR_ERR_UNSUPPORTED, "d_out must be 4 (got %d)", d.d_out);
    if (d.n_blocks < 1 || d.n_blocks > 8) return fail(PNR_ERR_UNSUPPORTED, "n_blocks in [1, 8] (got %d)", d.n_blocks);
    if (d.combine_layer < 0) return fail(PNR_ERR_INVALID, "combine_layer < 0");
    if (d.pe_n < 0 || d.pe_n > 16) return fail(PNR_ERR_UNSUPPORTED, "pe_n in [0, 16] (got %d)", d.pe_n);
    if (d.d_in != 3 + 3 * d.pe_n + 3)
        return fail(PNR_ERR_UNSUPPORTED, "d_in must be 3 + 3*pe_n + 3 (xyz PE + raw viewdirs); got %d", d.d_in);
    if (d.d_in > 16 * mlpk::NKB_IN) return fail(PNR_ERR_UNSUPPORTED, "d_in <= 64");
    if (d.precision != PNR_PREC_F32 && d.precision != PNR_PREC_F16X3 && d.precision != PNR_PREC_BF16X6 &&
        d.precision != PNR_PREC_BF16X9)
        return fail(PNR_ERR_UNSUPPORTED, "precision must be 0 (f32), 3 (scaled f16) or 6 / 9 (split bf16); got %d",
                    d.precision);
    return PNR_OK;
}

static int pack_src(const pnr_mlp_weights &w, const mlpk::Layout &L, mlpk::PackSrc &s) {
    const pnr_mlp_desc &d = w.desc;
    s = {};
    s.lin_in_w = w.lin_in_w; s.lin_in_b = w.lin_in_b;
    s.lin_out_w = w.lin_out_w; s.lin_out_b = w.lin_out_b;
    s.pe_f = w.pe_freqs; s.pe_p = w.pe_phases;
    if (!s.lin_in_w || !s.lin_in_b || !s.lin_out_w || !s.lin_out_b || (d.pe_n && (!s.pe_f || !s.pe_p)))
        return fail(PNR_ERR_INVALID, "null weight pointer");
    for (int blk = 0; blk < d.n_blocks; ++blk) {
        for (int kind = 0; kind < 3; ++kind) {
            if (kind == 0 && blk >= L.n_linz) continue;
            const int li = mlpk::layer_index(blk, kind, L.n_linz);
            const float *wp = kind == 0 ? w.lin_z_w[blk] : kind == 1 ? w.fc0_w[blk] : w.fc1_w[blk];
            const float *bp = kind == 0 ? w.lin_z_b[blk] : kind == 1 ? w.fc0_b[blk] : w.fc1_b[blk];
            if (!wp || !bp) return fail(PNR_ERR_INVALID, "null weight pointer (block %d kind %d)", blk, kind);
            s.w[li] = wp;
            s.b[li] = bp;
        }
    }
    return PNR_OK;
}

int mlp_pack(const pnr_mlp_weights &w, void *packed, size_t bytes, hipStream_t st) {
    const pnr_mlp_desc &d = w.desc;
    int rc = mlp_check_desc(d);
    if (rc) return rc;
    mlpk::Layout L = mlpk::make_layout(d);
    if (bytes < sizeof(float) * (size_t)L.total) return fail(PNR_ERR_WORKSPACE, "packed buffer too small");
    mlpk::PackSrc s;
    if ((rc = pack_src(w, L, s))) return rc;
    const int64_t blocks = (L.total + 255) / 256;
    hipLaunchKernelGGL(mlpk::k_pack, dim3((unsigned)blocks), dim3(256), 0, st, s, L,
                       static_cast<float *>(packed));
    if (!launch_ok("mlp_pack")) return PNR_ERR_HIP;
    const int64_t n = (int64_t)(mlpk::KS32_IN + L.n_l512 * mlpk::KS32) * mlpk::NRT * 64;
    if (L.prec == PNR_PREC_F16X3) {
        float *hdr = static_cast<float *>(packed);
        if (hipMemsetAsync(hdr + mlpk::HDR_ESCALE, 0, sizeof(float) * (1 + L.n_l512), st) != hipSuccess)
            return fail(PNR_ERR_HIP, "mlp_pack: hipMemsetAsync failed");
        hipLaunchKernelGGL(mlpk::k_layer_absmax, dim3(32, (unsigned)(1 + L.n_l512)), dim3(256), 0, st, s, L, hdr);
        if (!launch_ok("mlp_layer_absmax")) return PNR_ERR_HIP;
        hipLaunchKernelGGL(mlpk::k_layer_escale, dim3(1), dim3(64), 0, st, 1 + L.n_l512, hdr);
        if (!launch_ok("mlp_layer_escale")) return PNR_ERR_HIP;
        hipLaunchKernelGGL(mlpk::k_pack_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           s, L, static_cast<float *>(packed));
        if (!launch_ok("mlp_pack_f16")) return PNR_ERR_HIP;
    } else if (L.prec) {
        hipLaunchKernelGGL(mlpk::k_pack_split, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           s, L, static_cast<float *>(packed));
        if (!launch_ok("mlp_pack_split")) return PNR_ERR_HIP;
    }
    return PNR_OK;
}

// ---- training backward (PREC 3) ----------------------------------------------------------
size_t mlp_packed_t_bytes(const pnr_mlp_desc &d) {
    if (mlp_check_desc(d) || d.precision != PNR_PREC_F16X3) return 0;
    const mlpk::Layout L = mlpk::make_layout(d);
    return sizeof(float) * (size_t)(L.n_l512 * L.layer_floats);
}

int mlp_pack_t(const pnr_mlp_weights &w, const void *packed, void *packed_t, size_t bytes, hipStream_t st) {
    const pnr_mlp_desc &d = w.desc;
    int rc = mlp_check_desc(d);
    if (rc) return rc;
    if (d.precision != PNR_PREC_F16X3)
        return fail(PNR_ERR_UNSUPPORTED, "the fused MLP backward implements precision 3 (f16x3); got %d", d.precision);
    const mlpk::Layout L = mlpk::make_layout(d);
    if (bytes < mlp_packed_t_bytes(d)) return fail(PNR_ERR_WORKSPACE, "transposed pack buffer too small");
    mlpk::PackSrc s;
    if ((rc = pack_src(w, L, s))) return rc;
    const int64_t n = (int64_t)L.n_l512 * mlpk::KS32 * mlpk::NRT * 64;
    hipLaunchKernelGGL(mlpk::k_pack_f16_t, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, L,
                       static_cast<const float *>(packed), static_cast<float *>(packed_t));
    return launch_ok("mlp_pack_t") ? PNR_OK : PNR_ERR_HIP;
}

static int64_t mlp_bwd_grid(int64_t n_points) {
    const int64_t tiles = (n_points + mlpk::COLS - 1) / mlpk::COLS;
    const int cus = device_cu_count();
    return tiles < cus ? tiles : cus;
}

size_t mlp_bwd_workspace_bytes(const pnr_mlp_desc &d, int64_t n_points) {
    if (n_points <= 0) return 0;
    return sizeof(float) * (size_t)mlp_bwd_grid(n_points) * (2 * d.n_blocks + 1) * mlpk::H;
}

int launch_mlp_bwd(const pnr_mlp_desc &d, const void *packed, const void *packed_t, const float *w_out,
                   const float *save, const float *d_o, int64_t n_points, float *dy, float *dzlat, hipStream_t st,
                   float *d_bias, void *ws, size_t ws_bytes, int n_views) {
    int rc = mlp_check_desc(d);
    if (rc) return rc;
    if (d.precision != PNR_PREC_F16X3)
        return fail(PNR_ERR_UNSUPPORTED, "the fused MLP backward implements precision 3 (f16x3); got %d", d.precision);
    mlpk::BwdArgs a = {};
    a.L = mlpk::make_layout(d);
    if (a.L.n_linz > 0 && !dzlat) return fail(PNR_ERR_INVALID, "mlp backward: d_zlat is required (n_linz > 0)");
    if (n_points == 0) return PNR_OK;
    a.hdr = static_cast<const float *>(packed);
    a.packed_t = static_cast<const float *>(packed_t);
    a.w_out = w_out;
    a.save = save;
    a.d_o = d_o;
    a.dy = dy;
    a.dzlat = dzlat;
    a.n_points = n_points;
    a.n_tiles = (n_points + mlpk::COLS - 1) / mlpk::COLS;
    if (n_views < 1) return fail(PNR_ERR_INVALID, "mlp backward: n_views < 1");
    a.ns = n_views;
    const int64_t grid = mlp_bwd_grid(n_points);
    if (d_bias) {
        const size_t need = mlp_bwd_workspace_bytes(d, n_points);
        if (!ws || ws_bytes < need) return fail(PNR_ERR_WORKSPACE, "mlp backward: workspace %zu < %zu", ws_bytes, need);
        a.bsum = static_cast<float *>(ws);
    }
    // split image P0 + P1, column maxima, exponents = 137,472 B
    const size_t lds = 2 * sizeof(_Float16) * mlpk::PART_HALVES + sizeof(float) * (mlpk::COLS * 8 + mlpk::COLS + 8);
    hipLaunchKernelGGL(mlpk::k_mlp_bwd, dim3((unsigned)grid), dim3(mlpk::NTHR), lds, st, a);
    if (!launch_ok("mlp_bwd")) return PNR_ERR_HIP;
    if (d_bias) {
        const int n = (2 * d.n_blocks + 1) * mlpk::H;
        hipLaunchKernelGGL(mlpk::k_bias_reduce, dim3((unsigned)((n + 63) / 64)), dim3(64 * mlpk::BIAS_SLICES), 0,
                           st, a.bsum, (int)grid, n, d_bias);
        if (!launch_ok("bias_reduce")) return PNR_ERR_HIP;
    }
    return PNR_OK;
}

int64_t mlp_save_floats(const pnr_mlp_desc &d, int64_t n_points) {
    return mlpk::save_floats_per_point(d.n_blocks) * n_points;
}

size_t mlp_xsum_bytes(int ns) {
    (void)ns;  // x park + multi-view sum, one pair of 128 KB regions per resident workgroup,
               // then the 8 per-XCD tile counters (512 B)
    return sizeof(float) * (size_t)device_cu_count() * 2 * mlpk::COLS * mlpk::H + 512;
}

// Launch the fused model over n_points points (render mode if rays != nullptr).
int launch_point_mlp(const pnr_scene &sc, const pnr_mlp_desc &d, const void *packed,
                     const float *rays, const float *zs, int K, int64_t rays_per_obj,
                     const float *xyz, const float *dirs, int64_t points_per_obj,
                     int64_t n_points, float *out, float *xsum_ws, hipStream_t st, float *save,
                     const float *proj, const MarchCfg *march) {
    if (n_points == 0) return PNR_OK;
    if (proj && save) return fail(PNR_ERR_UNSUPPORTED, "the activation save (training) needs the latent gather path");
    if (march && (!rays || save || (march->kpt != 1 && march->kpt != 2) || K != mlpk::COLS * march->kpt ||
                  n_points % K != 0 || (march->kf > 0 && (K > 64 || march->n_sort > 128 || K + march->kf > march->n_sort))))
        return fail(PNR_ERR_INVALID, "point_mlp: fused march needs K = 64 kpt (kpt 1 or 2) and kc + kf <= 128");
    if (march && march->single &&
        (!proj || !march->packed_f || !march->proj_f || march->kf <= 0 || march->kpt != 1 ||
         march->kpt_f * mlpk::COLS != K + march->kf || (march->kpt_f != 1 && march->kpt_f != 2) ||
         !march->rgb_f || !march->depth_f || n_points % (K + march->kpt_f * mlpk::COLS) != 0))
        return fail(PNR_ERR_INVALID, "point_mlp: the single-launch march needs kc = 64, kc + kf = 64 kpt_f, both "
                    "packs and projections, fine outputs, and n_points = n_rays (kc + kc + kf)");
    mlpk::Args a = {};
    a.packed = static_cast<const float *>(packed);
    a.L = mlpk::make_layout(d);
    a.render_mode = rays != nullptr;
    a.rays = rays; a.zs = zs; a.K = K; a.rays_per_obj = rays_per_obj;
    a.xyz = xyz; a.dirs = dirs; a.points_per_obj = points_per_obj;
    a.n_points = n_points;
    a.latent = sc.latent; a.cams = sc.cams;
    a.ns = sc.n_views; a.hl = sc.latent_h; a.wl = sc.latent_w;
    a.img_w = sc.image_w; a.img_h = sc.image_h;
    a.out = out;
    a.xsum = xsum_ws;
    a.march = march != nullptr;
    if (march) a.m = *march;
    a.n_tiles = (n_points + mlpk::COLS - 1) / mlpk::COLS;
    a.save = save;
    a.proj = proj;
    a.proj_stride = (int64_t)sc.n_obj * sc.n_views * sc.latent_h * sc.latent_w * mlpk::H;
    const int cus = device_cu_count();
    if (a.n_tiles >= (1ll << 31)) return fail(PNR_ERR_UNSUPPORTED, "more than 2^31 point tiles in one launch");
    a.tile_ctr = reinterpret_cast<int *>(xsum_ws + (size_t)cus * 2 * mlpk::COLS * mlpk::H);
    if (hipMemsetAsync(a.tile_ctr, 0, 512, st) != hipSuccess) return fail(PNR_ERR_HIP, "point_mlp: hipMemsetAsync failed");
    const int64_t grid = a.n_tiles < cus ? a.n_tiles : cus;
    // PREC 3: split image P0 + P1, gather records, column maxima, exponents, PE table, next tile
    //         = 143,760 B; else: fp32 activations + staging ring + gather records + PE table +
    //         next tile = 158,864 B
    const size_t lds = (d.precision == PNR_PREC_F16X3
        ? 2 * sizeof(_Float16) * mlpk::PART_HALVES + sizeof(float) * (2 * mlpk::COLS * 8 + mlpk::COLS + 64 + 2048)
        : sizeof(float) * ((size_t)mlpk::COLS * mlpk::LDS_LD + 2 * mlpk::STG_FLOATS + mlpk::COLS * 8 + 32 + 4)
        ) + (march ? sizeof(float) * MARCH_LDS_FLOATS : 0);   // + the fused march region
#define PNR_LAUNCH_MLP(P)                                                                              \
    do {                                                                                               \
        if (proj && march) hipLaunchKernelGGL((mlpk::k_point_mlp<P, true, true>), dim3((unsigned)grid), dim3(mlpk::NTHR), lds, st, a); \
        else if (proj) hipLaunchKernelGGL((mlpk::k_point_mlp<P, true, false>), dim3((unsigned)grid), dim3(mlpk::NTHR), lds, st, a); \
        else if (march) hipLaunchKernelGGL((mlpk::k_point_mlp<P, false, true>), dim3((unsigned)grid), dim3(mlpk::NTHR), lds, st, a); \
        else hipLaunchKernelGGL((mlpk::k_point_mlp<P, false, false>), dim3((unsigned)grid), dim3(mlpk::NTHR), lds, st, a);     \
    } while (0)
    switch (d.precision) {
    case PNR_PREC_F16X3: PNR_LAUNCH_MLP(3); break;
    case PNR_PREC_BF16X6: PNR_LAUNCH_MLP(6); break;
    case PNR_PREC_BF16X9: PNR_LAUNCH_MLP(9); break;
    default: PNR_LAUNCH_MLP(0);
    }
#undef PNR_LAUNCH_MLP
    return launch_ok("point_mlp") ? PNR_OK : PNR_ERR_HIP;
}

}  // namespace pnr
