// Shared helpers for the pixelNeRF gfx950 kernels (internal header).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pnr_abi.h"

namespace pnr {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---- error reporting (thread-local; no exceptions cross the ABI) ------------
void set_error(const char *fmt, ...);
int fail(int status, const char *fmt, ...);

// multiprocessor count of the current device (cached per device id)
int device_cu_count();

inline bool launch_ok(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return false;
    }
    return true;
}

// ---- device helpers ------------------------------------------------------------
// Round-to-nearest fp32 arithmetic without contraction: the reference evaluates
// these expressions as separate torch ops (one rounding each), so the sampling
// and projection code keeps the same roundings instead of fusing into FMAs.
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float sub_rn(float a, float b) { return __fsub_rn(a, b); }

// z = near * (1 - t) + far * t  (nerf.py:113 / 145), or the lindisp form (115 / 147)
__device__ __forceinline__ float t_to_z(float t, float near, float far, bool lindisp) {
    if (!lindisp) return add_rn(mul_rn(near, sub_rn(1.0f, t)), mul_rn(far, t));
    float inv = add_rn(mul_rn(__fdiv_rn(1.0f, near), sub_rn(1.0f, t)),
                       mul_rn(__fdiv_rn(1.0f, far), t));
    return __fdiv_rn(1.0f, inv);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---- DPP wave64 scans / reductions (GFX9 row_shr, row_bcast:15/31, wave_shr:1; no LDS) ----
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float old, float src) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL,
                                                      ROW_MASK, 0xf, false));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double old, double src) {
    const long long o = __double_as_longlong(old), v = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)v, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(v >> 32), CTRL, ROW_MASK, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// inclusive product scan over the 64 lanes (lanes out of range contribute 1)
__device__ __forceinline__ double wave_scan_mul(double x) {
    x *= dpp_d<0x111>(1.0, x);          // row_shr:1
    x *= dpp_d<0x112>(1.0, x);          // row_shr:2
    x *= dpp_d<0x114>(1.0, x);          // row_shr:4
    x *= dpp_d<0x118>(1.0, x);          // row_shr:8
    x *= dpp_d<0x142, 0xa>(1.0, x);     // row_bcast:15 -> rows 1, 3
    x *= dpp_d<0x143, 0xc>(1.0, x);     // row_bcast:31 -> rows 2, 3
    return x;
}
// value of lane - 1 (lane 0: `first`)
__device__ __forceinline__ double wave_shr1(double x, double first) { return dpp_d<0x138>(first, x); }
// sum over the 64 lanes, returned wave-uniform
__device__ __forceinline__ float wave_sum_dpp(float x) {
    x += dpp_f<0x111>(0.f, x);
    x += dpp_f<0x112>(0.f, x);
    x += dpp_f<0x114>(0.f, x);
    x += dpp_f<0x118>(0.f, x);
    x += dpp_f<0x142, 0xa>(0.f, x);
    x += dpp_f<0x143, 0xc>(0.f, x);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

// IEEE-754-2019 maximum (v_maximum3_f32 on gfx950: NaN-propagating like torch.relu / torch.max,
// so no operand canonicalization; fmaxf's quieting doubled the max count of every publish)
__device__ __forceinline__ float max_nc(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float max3_nc(float a, float b, float c) { return max_nc(max_nc(a, b), c); }
__device__ __forceinline__ f4 relu4(const f4 &v) { return __builtin_elementwise_maximum(v, f4{0.f, 0.f, 0.f, 0.f}); }
// max over the four 16-lane rows of the wave, every lane: v_permlane16_swap / v_permlane32_swap
// of a value with itself puts the row partner's value in one of the two results (max is symmetric,
// so which one does not matter); VALU only, no LDS crossbar round trip
__device__ __forceinline__ float rows_max(float m) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    m = max_nc(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
    const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return max_nc(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

// sum over the four 16-lane rows of a wave (v_permlane16/32_swap; every lane gets the same
// ((r0 + r1) + (r2 + r3)) in some operand order: IEEE addition is commutative, so the lanes agree)
__device__ __forceinline__ float rows_sum(float m) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    m = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// ---- counter-based random streams (pnr_rng {seed, offset}, include/pnr_abi.h) ----------
// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3",
// SC'11; the Random123 constants).  Draw e of stream s keyed by `seed` uses the counter
// (lo32 e, hi32 e, s, 0); e = (offset + ray) * width + k, so a ray's draws depend only on
// its global index and not on how the batch is chunked.  oracle/philox.py restates it.
struct RngSrc {
    const float *p;          // injected stream (n_rays, width); NULL = Philox
    uint64_t seed, offset;
    int stream;              // PNR_RNG_U_COARSE .. PNR_RNG_N_DEPTH
};

__device__ __forceinline__ void philox4x32_10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
}

__device__ __forceinline__ void rng_bits(const RngSrc &r, int64_t ray, int width, int k, uint32_t &x0,
                                         uint32_t &x1) {
    const uint64_t e = (r.offset + (uint64_t)ray) * (uint64_t)width + (uint64_t)k;
    uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(e >> 32), c2 = (uint32_t)r.stream, c3 = 0u;
    philox4x32_10(c0, c1, c2, c3, (uint32_t)r.seed, (uint32_t)(r.seed >> 32));
    x0 = c0;
    x1 = c1;
}

// U[0, 1): the top 24 bits of the first Philox word times 2^-24 (exact in fp32)
__device__ __forceinline__ float rng_uniform(const RngSrc &r, int64_t ray, int width, int k) {
    if (r.p) return r.p[ray * width + k];
    uint32_t x0, x1;
    rng_bits(r, ray, width, k, x0, x1);
    return (float)(x0 >> 8) * 0x1p-24f;
}

// N(0, 1) by Box-Muller on the first two words: u1 in (0, 1], u2 in [0, 1)
__device__ __forceinline__ float rng_normal(const RngSrc &r, int64_t ray, int width, int k) {
    if (r.p) return r.p[ray * width + k];
    uint32_t x0, x1;
    rng_bits(r, ray, width, k, x0, x1);
    const float u1 = (float)((x0 >> 8) + 1u) * 0x1p-24f;
    const float u2 = (float)(x1 >> 8) * 0x1p-24f;
    return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647f * u2);
}

// ---- exact 3-way bf16 split (split-bf16 products: mlp.hip PREC 6 / 9, wgrad.hip) ------
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// x = x0 + x1 + x2 of fp32 values into bf16 (RNE at each step).  Per pair:
// v_cvt_pk_bf16_f32, then the two halves back to fp32 by a shift / mask (11 VALU per pair,
// no second conversion).
__device__ __forceinline__ unsigned cvt_pk(float a, float b) {
    bf2 v = __builtin_convertvector((float __attribute__((ext_vector_type(2)))){a, b}, bf2);
    return __builtin_bit_cast(unsigned, v);
}
// one pair (a, b) -> the packed bf16 pairs of its three parts (the pair's subtractions as
// one packed fp32 op, v_pk_add_f32: same per-element RNE rounding)
__device__ __forceinline__ void split_pair(float a, float b, unsigned &p0, unsigned &p1, unsigned &p2) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    const unsigned h = cvt_pk(a, b);
    const f2v r = f2v{a, b} - f2v{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};
    const unsigned m = cvt_pk(r.x, r.y);
    const f2v t = r - f2v{__uint_as_float(m << 16), __uint_as_float(m & 0xffff0000u)};
    p0 = h;
    p1 = m;
    p2 = cvt_pk(t.x, t.y);
}

}  // namespace pnr
