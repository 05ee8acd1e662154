// lshl_add_u64_check.hip -- semantics and issue rate of v_lshl_add_u64 on gfx950 for shift amounts 0..15:
// is D = (S0 << S1) + S2 exact for shifts above 4 (the compiler only selects it for 0..4)?
//   hipcc --offload-arch=gfx950 -O3 -o build/lshl_add_u64_check scripts/debug/lshl_add_u64_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void check(const uint64_t* a, const uint64_t* c, uint64_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t s = static_cast<uint32_t>(i % 16);
    uint64_t       d;
    asm volatile("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(d) : "v"(a[i]), "v"(s), "v"(c[i]));
    out[i] = d;
}

#define ITER 2000
__global__ void rate(unsigned long long* cycles, uint32_t sh, uint64_t seed) {
    uint64_t r[8];
    for (int i = 0; i < 8; ++i)
        r[i] = seed + i;
    const uint64_t add = seed * 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
            asm volatile("v_lshl_add_u64 %0, %0, %8, %9\n v_lshl_add_u64 %1, %1, %8, %9\n"
                         "v_lshl_add_u64 %2, %2, %8, %9\n v_lshl_add_u64 %3, %3, %8, %9\n"
                         "v_lshl_add_u64 %4, %4, %8, %9\n v_lshl_add_u64 %5, %5, %8, %9\n"
                         "v_lshl_add_u64 %6, %6, %8, %9\n v_lshl_add_u64 %7, %7, %8, %9\n"
                         : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),
                           "+v"(r[7])
                         : "v"(sh), "v"(add));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t x = 0;
    for (int i = 0; i < 8; ++i)
        x ^= r[i];
    if ((threadIdx.x & 63) == 0)
        cycles[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = (t1 - t0) + (x == 12345 ? 1 : 0);
}

int main() {
    const int             n = 1 << 16;
    std::vector<uint64_t> a(n), c(n), o(n);
    uint64_t              z = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < n; ++i) {
        z ^= z << 13, z ^= z >> 7, z ^= z << 17;
        a[i] = z;
        z ^= z << 13, z ^= z >> 7, z ^= z << 17;
        c[i] = z;
    }
    uint64_t *da, *dc, *dout;
    hipMalloc(&da, n * 8), hipMalloc(&dc, n * 8), hipMalloc(&dout, n * 8);
    hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dc, c.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check, dim3(n / 256), dim3(256), 0, 0, da, dc, dout, n);
    hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
    int bad[16] = {};
    for (int i = 0; i < n; ++i) {
        const uint32_t s = i % 16;
        if (o[i] != (a[i] << s) + c[i])
            ++bad[s];
    }
    for (int s = 0; s < 16; ++s)
        printf("shift %2d: %d / %d wrong\n", s, bad[s], n / 16);
    unsigned long long* dcy;
    const int           blocks = 256 * 4, threads = 256;  // 4 waves per SIMD
    hipMalloc(&dcy, blocks * 4 * 8);
    for (uint32_t sh : {2u, 9u}) {
        hipLaunchKernelGGL(rate, dim3(blocks), dim3(threads), 0, 0, dcy, sh, 7ull);
        hipDeviceSynchronize();
        std::vector<unsigned long long> cy(blocks * 4);
        hipMemcpy(cy.data(), dcy, cy.size() * 8, hipMemcpyDeviceToHost);
        double mean = 0;
        for (auto v : cy)
            mean += v;
        mean /= cy.size();
        // s_memtime counts at a fixed 100 MHz; report per-wave instruction time, 4 waves share a SIMD
        printf("shift %u: %.3f memtime ticks per instruction per wave\n", sh, mean / (ITER * 16.0));
    }
    return 0;
}
