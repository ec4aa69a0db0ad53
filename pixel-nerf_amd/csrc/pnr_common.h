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

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

}  // namespace pnr
