// valu_rate.hip -- issue rate of the epilogue instruction kinds on gfx950, per SIMD, with 1..4 waves per SIMD.
// Each wave runs ITER iterations of 16 independent instructions of one kind (inline asm, so the compiler
// neither folds nor reorders them) and records s_memtime (shader clock) around the loop; lane 0 stores the
// cycle count with a vector store.  Output: cycles per instruction per wave and per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_rate scripts/debug/valu_rate.hip && build/valu_rate
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define ITER 2000

#define OP16(ins)                                                                                         \
    asm volatile(ins " %0, %0, %16, %17\n" ins " %1, %1, %16, %17\n" ins " %2, %2, %16, %17\n"             \
                 ins " %3, %3, %16, %17\n" ins " %4, %4, %16, %17\n" ins " %5, %5, %16, %17\n"             \
                 ins " %6, %6, %16, %17\n" ins " %7, %7, %16, %17\n" ins " %8, %8, %16, %17\n"             \
                 ins " %9, %9, %16, %17\n" ins " %10, %10, %16, %17\n" ins " %11, %11, %16, %17\n"         \
                 ins " %12, %12, %16, %17\n" ins " %13, %13, %16, %17\n" ins " %14, %14, %16, %17\n"       \
                 ins " %15, %15, %16, %17\n"                                                               \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),      \
                   "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]),  \
                   "+v"(r[14]), "+v"(r[15])                                                                 \
                 : "v"(a), "v"(b))

#define OP16_2(ins)                                                                                       \
    asm volatile(ins " %0, %0, %16\n" ins " %1, %1, %16\n" ins " %2, %2, %16\n" ins " %3, %3, %16\n"      \
                 ins " %4, %4, %16\n" ins " %5, %5, %16\n" ins " %6, %6, %16\n" ins " %7, %7, %16\n"      \
                 ins " %8, %8, %16\n" ins " %9, %9, %16\n" ins " %10, %10, %16\n" ins " %11, %11, %16\n"  \
                 ins " %12, %12, %16\n" ins " %13, %13, %16\n" ins " %14, %14, %16\n" ins " %15, %15, %16\n" \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),      \
                   "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]),  \
                   "+v"(r[14]), "+v"(r[15])                                                                 \
                 : "v"(a))

template <int OP>
__global__ void rate(unsigned long long* out, float seed) {
    float r[16];
    for (int i = 0; i < 16; ++i)
        r[i] = seed + i;
    const float a = seed * 0.5f, b = seed * 0.25f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
        if constexpr (OP == 0) OP16("v_min3_u32");
        if constexpr (OP == 1) OP16("v_min3_f32");
        if constexpr (OP == 2) OP16("v_and_or_b32");
        if constexpr (OP == 3) OP16("v_lshl_add_u32");
        if constexpr (OP == 4) OP16("v_fma_f32");
        if constexpr (OP == 5) OP16_2("v_add_f32");
        if constexpr (OP == 6) OP16_2("v_min_u32");
        if constexpr (OP == 7) OP16_2("v_min_f32");
        if constexpr (OP == 8) OP16_2("v_add_u32");
        if constexpr (OP == 9) OP16("v_or3_b32");
        if constexpr (OP == 10 || OP == 11) {
            // one v_mfma_i32_16x16x64_i8 per 4 epilogue instructions (8 per iteration pair of 16)
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            i32x4 acc = {0, 0, 0, 0};
            const i32x4 x = {__float_as_int(a), 1, 2, 3};
            for (int j = 0; j < 4; ++j) {
                acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, x, acc, 0, 0, 0);
                if constexpr (OP == 10)
                    asm volatile("v_min3_u32 %0, %0, %4, %5\nv_min3_u32 %1, %1, %4, %5\nv_min3_u32 %2, %2, %4, %5\n"
                                 "v_min3_u32 %3, %3, %4, %5\n"
                                 : "+v"(r[4 * j]), "+v"(r[4 * j + 1]), "+v"(r[4 * j + 2]), "+v"(r[4 * j + 3])
                                 : "v"(a), "v"(b));
                else
                    asm volatile("v_min3_f32 %0, %0, %4, %5\nv_min3_f32 %1, %1, %4, %5\nv_min3_f32 %2, %2, %4, %5\n"
                                 "v_min3_f32 %3, %3, %4, %5\n"
                                 : "+v"(r[4 * j]), "+v"(r[4 * j + 1]), "+v"(r[4 * j + 2]), "+v"(r[4 * j + 3])
                                 : "v"(a), "v"(b));
            }
            r[0] += static_cast<float>(acc[0] & 1);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 16; ++i)
        s += r[i];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0)
        out[wave] = (t1 - t0) + (s == 12345.0f ? 1 : 0);
}

template <int OP>
void run(const char* name) {
    for (int wavesPerSimd = 1; wavesPerSimd <= 4; wavesPerSimd *= 2) {
        const int threads = 256 * wavesPerSimd;  // one workgroup per CU: 4 SIMDs x wavesPerSimd waves
        const int blocks  = 256;
        const int nw      = blocks * threads / 64;
        unsigned long long* d;
        (void)hipMalloc(&d, nw * sizeof(unsigned long long));
        hipLaunchKernelGGL(rate<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0f);
        hipLaunchKernelGGL(rate<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0f);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> h(nw);
        (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::vector<unsigned long long> s(h);
        std::sort(s.begin(), s.end());
        const double med = static_cast<double>(s[nw / 2]);
        const double perInstWave = med / (ITER * 16.0);
        std::printf("%-16s waves/SIMD %d: %.2f cycles per instruction per wave, %.2f per SIMD\n", name, wavesPerSimd,
                    perInstWave, perInstWave / wavesPerSimd);
        (void)hipFree(d);
    }
}


template <int OP>
__global__ void rate64(unsigned long long* out, float seed) {
    unsigned long long r[8];
    for (int i = 0; i < 8; ++i)
        r[i] = __float_as_uint(seed) + i;
    const unsigned long long a = __float_as_uint(seed) * 3ull;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
#define R8 "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
        if constexpr (OP == 0)
            asm volatile("v_lshl_add_u64 %0, %0, 9, %8\nv_lshl_add_u64 %1, %1, 9, %8\nv_lshl_add_u64 %2, %2, 9, %8\n"
                         "v_lshl_add_u64 %3, %3, 9, %8\nv_lshl_add_u64 %4, %4, 9, %8\nv_lshl_add_u64 %5, %5, 9, %8\n"
                         "v_lshl_add_u64 %6, %6, 9, %8\nv_lshl_add_u64 %7, %7, 9, %8\n" : R8 : "v"(a));
        if constexpr (OP == 1)
            asm volatile("v_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\n"
                         "v_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\n"
                         "v_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8\n" : R8 : "v"(a));
        if constexpr (OP == 2)
            asm volatile("v_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\n"
                         "v_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\n"
                         "v_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\n" : R8 : "v"(a));
        if constexpr (OP == 3)
            asm volatile("v_lshl_add_u64 %0, %0, 0, %8\nv_lshl_add_u64 %1, %1, 0, %8\nv_lshl_add_u64 %2, %2, 0, %8\n"
                         "v_lshl_add_u64 %3, %3, 0, %8\nv_lshl_add_u64 %4, %4, 0, %8\nv_lshl_add_u64 %5, %5, 0, %8\n"
                         "v_lshl_add_u64 %6, %6, 0, %8\nv_lshl_add_u64 %7, %7, 0, %8\n" : R8 : "v"(a));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long s = 0;
    for (int i = 0; i < 8; ++i)
        s += r[i];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0)
        out[wave] = (t1 - t0) + (s == 12345ull ? 1 : 0);
}

template <int OP>
void run64(const char* name) {
    for (int wavesPerSimd = 1; wavesPerSimd <= 4; wavesPerSimd *= 2) {
        const int threads = 256 * wavesPerSimd, blocks = 256, nw = blocks * threads / 64;
        unsigned long long* d;
        (void)hipMalloc(&d, nw * sizeof(unsigned long long));
        hipLaunchKernelGGL(rate64<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0f);
        hipLaunchKernelGGL(rate64<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0f);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> h(nw);
        (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double per = static_cast<double>(h[nw / 2]) / (ITER * 8.0);
        std::printf("%-16s waves/SIMD %d: %.2f cycles per instruction per wave, %.2f per SIMD\n", name, wavesPerSimd, per,
                    per / wavesPerSimd);
        (void)hipFree(d);
    }
}

int main() {
    run64<0>("v_lshl_add_u64 9");
    run64<3>("v_lshl_add_u64 0");
    run64<1>("v_pk_add_f32");
    run64<2>("v_pk_fma_f32");
    return 0;
}
