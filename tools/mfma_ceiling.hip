// Practical MFMA ceiling of this MI355X under load (diagnostic, not part of libpnr.so).
// Every wave issues back-to-back v_mfma_f32_16x16x32_f16 on register operands loaded
// once from random data (the chip clocks down with operand toggling, so zeros would
// overstate the rate), with the kernel's layout: 8 waves per workgroup, one workgroup per
// CU, 16 independent accumulators per wave.  Prints TFLOP/s (dense, f16 products).
// Build: hipcc --offload-arch=gfx950 -O3 mfma_ceiling.hip -o mfma_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_mfma(const h8 *in, float *out, int iters) {
    const int t = threadIdx.x + blockIdx.x * blockDim.x;
    h8 a0 = in[(t * 4 + 0) & 4095], a1 = in[(t * 4 + 1) & 4095];
    h8 b0 = in[(t * 4 + 2) & 4095], b1 = in[(t * 4 + 3) & 4095];
    f4 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, acc[i], 0, 0, 0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
    out[t] = s;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<_Float16> host(4096 * 8);
    srand(1);
    for (auto &v : host) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    h8 *in;
    float *out;
    hipMalloc(&in, host.size() * sizeof(_Float16));
    hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
    hipMemcpy(in, host.data(), host.size() * sizeof(_Float16), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(cus), dim3(512), 0, 0, in, out, 100);   // warm-up
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(cus), dim3(512), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)cus * 8 * iters * 48 * (16.0 * 16 * 32 * 2);
    printf("{\"mfma\": \"v_mfma_f32_16x16x32_f16\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", cus, ms,
           flop / (ms * 1e-3) / 1e12);
    return 0;
}
