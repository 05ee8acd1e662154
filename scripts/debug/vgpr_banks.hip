// vgpr_banks.hip -- do VGPR bank conflicts (register index mod 4) slow the int8 epilogue's VOP3 ops on gfx950?
// 16 independent instructions per iteration with hard-coded registers: every source of an instruction in the
// destination's bank ("same") or in the other banks ("spread").  Cycles per instruction per SIMD, 1..4 waves.
//   hipcc --offload-arch=gfx950 -O3 -o build/vgpr_banks scripts/debug/vgpr_banks.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define ITER 2000
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15", \
             "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31", \
             "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47"

// dst d in v0..v15 (16 instructions); sources: "same" picks d+16, d+32 (same bank as d), "spread" d+17, d+34
#define I3(op, d, a, b) op " v" #d ", v" #d ", v" #a ", v" #b "\n"
#define I2S(op, d, a) op " v" #d ", v" #d ", s4, v" #a "\n"

template <int OP>
__global__ void run(unsigned long long* out) {
    asm volatile("v_mov_b32 v0, 1\n v_mov_b32 v1, 2\n v_mov_b32 v2, 3\n v_mov_b32 v3, 4\n" ::: CLOB);
    asm volatile("s_mov_b32 s4, 3" ::: "s4");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
        if constexpr (OP == 0)  // min3, all sources in the destination's bank
            asm volatile(I3("v_min3_u32", 0, 16, 32) I3("v_min3_u32", 1, 17, 33) I3("v_min3_u32", 2, 18, 34)
                         I3("v_min3_u32", 3, 19, 35) I3("v_min3_u32", 4, 20, 36) I3("v_min3_u32", 5, 21, 37)
                         I3("v_min3_u32", 6, 22, 38) I3("v_min3_u32", 7, 23, 39) I3("v_min3_u32", 8, 24, 40)
                         I3("v_min3_u32", 9, 25, 41) I3("v_min3_u32", 10, 26, 42) I3("v_min3_u32", 11, 27, 43)
                         I3("v_min3_u32", 12, 28, 44) I3("v_min3_u32", 13, 29, 45) I3("v_min3_u32", 14, 30, 46)
                         I3("v_min3_u32", 15, 31, 47) ::: CLOB);
        if constexpr (OP == 1)  // min3, sources in three different banks
            asm volatile(I3("v_min3_u32", 0, 17, 34) I3("v_min3_u32", 1, 18, 35) I3("v_min3_u32", 2, 19, 32)
                         I3("v_min3_u32", 3, 16, 33) I3("v_min3_u32", 4, 21, 38) I3("v_min3_u32", 5, 22, 39)
                         I3("v_min3_u32", 6, 23, 36) I3("v_min3_u32", 7, 20, 37) I3("v_min3_u32", 8, 25, 42)
                         I3("v_min3_u32", 9, 26, 43) I3("v_min3_u32", 10, 27, 40) I3("v_min3_u32", 11, 24, 41)
                         I3("v_min3_u32", 12, 29, 46) I3("v_min3_u32", 13, 30, 47) I3("v_min3_u32", 14, 31, 44)
                         I3("v_min3_u32", 15, 28, 45) ::: CLOB);
        if constexpr (OP == 2)  // lshl_add, the two VGPR sources in one bank
            asm volatile(I2S("v_lshl_add_u32", 0, 16) I2S("v_lshl_add_u32", 1, 17) I2S("v_lshl_add_u32", 2, 18)
                         I2S("v_lshl_add_u32", 3, 19) I2S("v_lshl_add_u32", 4, 20) I2S("v_lshl_add_u32", 5, 21)
                         I2S("v_lshl_add_u32", 6, 22) I2S("v_lshl_add_u32", 7, 23) I2S("v_lshl_add_u32", 8, 24)
                         I2S("v_lshl_add_u32", 9, 25) I2S("v_lshl_add_u32", 10, 26) I2S("v_lshl_add_u32", 11, 27)
                         I2S("v_lshl_add_u32", 12, 28) I2S("v_lshl_add_u32", 13, 29) I2S("v_lshl_add_u32", 14, 30)
                         I2S("v_lshl_add_u32", 15, 31) ::: CLOB);
        if constexpr (OP == 3)  // lshl_add, the two VGPR sources in different banks
            asm volatile(I2S("v_lshl_add_u32", 0, 17) I2S("v_lshl_add_u32", 1, 18) I2S("v_lshl_add_u32", 2, 19)
                         I2S("v_lshl_add_u32", 3, 16) I2S("v_lshl_add_u32", 4, 21) I2S("v_lshl_add_u32", 5, 22)
                         I2S("v_lshl_add_u32", 6, 23) I2S("v_lshl_add_u32", 7, 20) I2S("v_lshl_add_u32", 8, 25)
                         I2S("v_lshl_add_u32", 9, 26) I2S("v_lshl_add_u32", 10, 27) I2S("v_lshl_add_u32", 11, 24)
                         I2S("v_lshl_add_u32", 12, 29) I2S("v_lshl_add_u32", 13, 30) I2S("v_lshl_add_u32", 14, 31)
                         I2S("v_lshl_add_u32", 15, 28) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0)
        out[wave] = t1 - t0;
}

template <int OP>
void measure(const char* name) {
    for (int w = 1; w <= 4; w *= 2) {
        const int threads = 256 * w, blocks = 256, nw = blocks * threads / 64;
        unsigned long long* d;
        (void)hipMalloc(&d, nw * sizeof(unsigned long long));
        hipLaunchKernelGGL(run<OP>, dim3(blocks), dim3(threads), 0, 0, d);
        hipLaunchKernelGGL(run<OP>, dim3(blocks), dim3(threads), 0, 0, d);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> h(nw);
        (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double per = static_cast<double>(h[nw / 2]) / (ITER * 16.0);
        std::printf("%-28s waves/SIMD %d: %.2f cycles per instruction per wave, %.2f per SIMD\n", name, w, per, per / w);
        (void)hipFree(d);
    }
}

int main() {
    measure<0>("v_min3_u32 same bank");
    measure<1>("v_min3_u32 spread banks");
    measure<2>("v_lshl_add_u32 same bank");
    measure<3>("v_lshl_add_u32 spread banks");
    return 0;
}
