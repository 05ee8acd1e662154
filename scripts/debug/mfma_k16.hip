// micro-benchmark: cycles per v_mfma_f32_16x16x16_f16 vs v_mfma_f32_16x16x32_f16 on gfx950 (one wave per SIMD,
// 4 independent accumulators, back-to-back)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ void bench(float* out, long long* cyc, int iters) {
    f4 acc[4] = {};
    h8 a8, b8;
    h4 a4, b4;
    for (int j = 0; j < 8; ++j) { a8[j] = (_Float16)(threadIdx.x * 0.001f + j); b8[j] = (_Float16)(0.5f + j); }
    for (int j = 0; j < 4; ++j) { a4[j] = a8[j]; b4[j] = b8[j]; }
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (K == 16)
                acc[r] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc[r], 0, 0, 0);
            else
                acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc[r], 0, 0, 0);
        }
    }
    long long t1 = clock64();
    float s = 0;
    for (int r = 0; r < 4; ++r) s += acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out; long long* cyc;
    hipMalloc(&out, 1024 * 64 * 4); hipMalloc(&cyc, 1024 * 8);
    const int iters = 20000;
    for (int k = 0; k < 2; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            if (k == 0) hipLaunchKernelGGL(bench<16>, dim3(1024), dim3(64), 0, 0, out, cyc, iters);
            else hipLaunchKernelGGL(bench<32>, dim3(1024), dim3(64), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
        }
        long long h[1024];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double m = 0; for (int i = 0; i < 1024; ++i) m += h[i];
        m /= 1024;
        printf("16x16x%d_f16: %.2f clock64 ticks per MFMA (4 chains)\n", k == 0 ? 16 : 32, m / (iters * 4.0));
    }
    return 0;
}
