// mfma_shape_valu.hip -- does the MFMA shape change what the int8 epilogue costs?  Per loop iteration a wave
// issues the MFMA work of 16 keys per lane (K = 64) and 24 epilogue VOP3 (16 v_lshl_add + 8 v_min3):
//   A: 4 x v_mfma_i32_16x16x64_i8 (4 independent accumulators, one per 16-frame block)
//   B: 2 x v_mfma_i32_32x32x32_i8 (one 32x32 block, K split in two)
// Same matrix-pipe cycles (64 per iteration), same VALU; B issues half the MFMAs.  Cycles per iteration
// per SIMD (s_memtime, median over waves) at 1..4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma_shape_valu scripts/debug/mfma_shape_valu.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define ITER 1000
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ void run(unsigned long long* out, int seed) {
    const i32x4 x = {seed, seed + 1, seed + 2, seed + 3};
    int best[8];
    for (int i = 0; i < 8; ++i)
        best[i] = seed * 7 + i;
    int pr[4] = {seed * 3, seed * 5, seed * 9, seed * 11};
    asm volatile("" : "+v"(pr[0]), "+v"(pr[1]), "+v"(pr[2]), "+v"(pr[3]));
    unsigned sh = (seed & 7) + 1;
    asm volatile("" : "+s"(sh));
    i32x4 xv = x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
        int k[16];
        asm volatile("" : "+v"(xv));  // new operands every iteration: the MFMAs stay in the loop
        if constexpr (SHAPE == 0) {
            i32x4 a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xv, x, i32x4{0, 0, 0, 0}, 0, 0, 0);
            i32x4 a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, x + 1, i32x4{0, 0, 0, 0}, 0, 0, 0);
            i32x4 a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, x + 2, i32x4{0, 0, 0, 0}, 0, 0, 0);
            i32x4 a3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, x + 3, i32x4{0, 0, 0, 0}, 0, 0, 0);
            for (int r = 0; r < 4; ++r) {
                k[r] = a0[r];
                k[4 + r] = a1[r];
                k[8 + r] = a2[r];
                k[12 + r] = a3[r];
            }
        }
        else {
            i32x16 a = __builtin_amdgcn_mfma_i32_32x32x32_i8(xv, x, i32x16{}, 0, 0, 0);
            a        = __builtin_amdgcn_mfma_i32_32x32x32_i8(x + 1, x, a, 0, 0, 0);
            for (int r = 0; r < 16; ++r)
                k[r] = a[r];
        }
        for (int r = 0; r < 16; ++r)
            k[r] = static_cast<int>((static_cast<unsigned>(k[r]) << sh) + static_cast<unsigned>(pr[r & 3]));
        for (int s = 0; s < 8; ++s)
            best[s] = min(best[s], min(k[s], k[s + 8]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int acc = 0;
    for (int i = 0; i < 8; ++i)
        acc ^= best[i];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0)
        out[wave] = (t1 - t0) + (acc == 0x12345678 ? 1 : 0);
}

template <int SHAPE>
void measure(const char* name) {
    for (int w = 1; w <= 4; ++w) {
        const int threads = 256 * w, blocks = 256, nw = blocks * threads / 64;
        unsigned long long* d;
        (void)hipMalloc(&d, nw * sizeof(unsigned long long));
        hipLaunchKernelGGL(run<SHAPE>, dim3(blocks), dim3(threads), 0, 0, d, 1);
        hipLaunchKernelGGL(run<SHAPE>, dim3(blocks), dim3(threads), 0, 0, d, 1);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> h(nw);
        (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double per = static_cast<double>(h[nw / 2]) / ITER;
        std::printf("%-22s waves/SIMD %d: %.1f cycles per iteration per wave, %.1f per SIMD (matrix pipe 64)\n", name, w,
                    per, per / w);
        (void)hipFree(d);
    }
}

int main() {
    measure<0>("4 x 16x16x64 + 24 VOP3");
    measure<1>("2 x 32x32x32 + 24 VOP3");
    return 0;
}
