// Diagnostic kernels for tests/test_gpu_lane_exchange.py, built into
// pnr/libpnr_selftest.so, not into libpnr.so: the cross-lane exchanges the render path's
// epilogue and publish rely on (DPP row shifts / broadcasts, v_permlane16/32_swap, ds_bpermute),
// exercised in the placements a fused kernel puts them in:
//   placement 0  wave-uniform control flow, nothing else live;
//   placement 1  inside a lane-divergent branch (EXEC = lanes with (lane * 7) % 5 != 0);
//   placement 2  right after a long MFMA chain whose 16 accumulators stay live across the
//                exchange (register pressure and MFMA -> VALU / DPP hazards, as in the GEMM region).
// Each kernel writes what every lane ends with; the test compares the variants with each other
// and with the semantics on the host.
#include "march_dev.h"

namespace pnr {
namespace selftest {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// lane ^ J by ds_bpermute (__shfl_xor): what march_dev.h's lane_xor uses
template <int J>
__device__ __forceinline__ float xor_bperm(float v) { return __shfl_xor(v, J, 64); }

// lane ^ J without LDS: J = 1, 2 quad_perm DPP; J = 4, 8 two row shifts with complementary bank
// masks (DPP banks are groups of 4 lanes of a 16-lane row); J = 16, 32 v_permlane16/32_swap
template <int J>
__device__ __forceinline__ float xor_dpp(float v) {
    const int x = __float_as_int(v);
    if constexpr (J == 1) return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, false));
    if constexpr (J == 2) return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, false));
    if constexpr (J == 4) {
        int y = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xf, 0x5, false);   // row_shl:4, banks 0, 2
        return __int_as_float(__builtin_amdgcn_update_dpp(y, x, 0x114, 0xf, 0xa, false));   // row_shr:4, banks 1, 3
    }
    if constexpr (J == 8) {
        int y = __builtin_amdgcn_update_dpp(x, x, 0x108, 0xf, 0x3, false);   // row_shl:8, banks 0, 1
        return __int_as_float(__builtin_amdgcn_update_dpp(y, x, 0x118, 0xf, 0xc, false));   // row_shr:8, banks 2, 3
    }
    if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return __int_as_float((threadIdx.x & 16) ? r[0] : r[1]);   // {vdst, vsrc} after the swap
    }
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return __int_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

template <int J, int VAR>
__device__ __forceinline__ float lx(float v) { return VAR ? xor_dpp<J>(v) : xor_bperm<J>(v); }

// march_dev.h's register bitonic sort of 64 values (one per lane), with the exchange variant
template <int VAR>
__device__ __forceinline__ float sort64(float v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            float p;
            switch (j) {
            case 1: p = lx<1, VAR>(v); break;
            case 2: p = lx<2, VAR>(v); break;
            case 4: p = lx<4, VAR>(v); break;
            case 8: p = lx<8, VAR>(v); break;
            case 16: p = lx<16, VAR>(v); break;
            default: p = lx<32, VAR>(v); break;
            }
            v = ((lane & j) == 0) == ((lane & k) == 0) ? fminf(v, p) : fmaxf(v, p);
        }
    }
    return v;
}

// out[8 w + t][lane] for wave w: t = 0..5 the exchanges J = 1..32 of in, t = 6 the sorted
// wave, t = 7 wave_scan_add + wave_sum_dpp + rows_max folded (the epilogue / publish helpers)
template <int VAR, int PLACE>
__global__ __launch_bounds__(64) void k_lane_exchange(const float *__restrict__ in, float *__restrict__ out,
                                                      const float *__restrict__ wts) {
    const int lane = threadIdx.x;
    const float v = in[blockIdx.x * 64 + lane];
    float *o = out + (size_t)blockIdx.x * 8 * 64;
    f4 acc[4][4];
    if constexpr (PLACE == 2) {
        // a GEMM-region stand-in: 16 accumulators through a chain of f16 MFMAs, live across
        // the exchanges below (folded into the output afterwards)
        const h8 *wa = reinterpret_cast<const h8 *>(wts);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = f4{0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < 16; ++ks) {
            const h8 a = wa[(ks * 64 + lane) % 256], b = wa[(ks * 64 + lane + 77) % 256];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[r][c], 0, 0, 0);
        }
    }
    auto body = [&]() {
        o[0 * 64 + lane] = lx<1, VAR>(v);
        o[1 * 64 + lane] = lx<2, VAR>(v);
        o[2 * 64 + lane] = lx<4, VAR>(v);
        o[3 * 64 + lane] = lx<8, VAR>(v);
        o[4 * 64 + lane] = lx<16, VAR>(v);
        o[5 * 64 + lane] = lx<32, VAR>(v);
        o[6 * 64 + lane] = sort64<VAR>(v, lane);
        const double sc = wave_scan_add((double)v);
        o[7 * 64 + lane] = (float)sc + wave_sum_dpp(v) + rows_max(v);
    };
    if constexpr (PLACE == 1) {
        if ((lane * 7) % 5 != 0) body();   // lane-divergent: some source lanes are inactive
    } else {
        body();
    }
    if constexpr (PLACE == 2) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) t += acc[r][c].x - acc[r][c].y + acc[r][c].z - acc[r][c].w;
        // keeps the MFMA chain live; written where the test ignores it (never an output slot)
        out[(size_t)gridDim.x * 8 * 64 + blockIdx.x * 64 + lane] = t;
    }
}

}  // namespace selftest
}  // namespace pnr

// variant 0 ds_bpermute, 1 DPP / permlane; placement 0-2 (above).  in: n_waves x 64 floats;
// out: n_waves x 8 x 64 floats (+ n_waves x 64 scratch for placement 2); wts: 256 x 8 f16.
extern "C" int pnr_selftest_lane_exchange(int variant, int placement, const float *in, float *out, const void *wts,
                                          int n_waves, hipStream_t st) {
    using namespace pnr::selftest;
    const float *w = static_cast<const float *>(wts);
#define PNR_LX(V, P) hipLaunchKernelGGL((k_lane_exchange<V, P>), dim3(n_waves), dim3(64), 0, st, in, out, w)
    if (variant == 0) {
        if (placement == 0) PNR_LX(0, 0); else if (placement == 1) PNR_LX(0, 1); else PNR_LX(0, 2);
    } else {
        if (placement == 0) PNR_LX(1, 0); else if (placement == 1) PNR_LX(1, 1); else PNR_LX(1, 2);
    }
#undef PNR_LX
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
