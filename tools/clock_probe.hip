// Shader clock under a one-wave load (what a single-lane Process.Run launch sees) and under a full
// grid: s_memtime (shader clock cycles) against s_memrealtime (100 MHz) around a dependent ALU loop.
//   hipcc --offload-arch=gfx950 -O3 -o tools/clock_probe tools/clock_probe.hip && tools/clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void spin(uint64_t *out, uint32_t iters, uint32_t seed) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x + seed;
    for (uint32_t k = 0; k < iters; k++) x = x * 1664525u + 1013904223u;
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
        out[2] = x;
    }
}

int main() {
    uint64_t *d = nullptr, h[3];
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    const struct { const char *name; uint32_t blocks, threads, iters; } runs[] = {
        {"one wave, 20k iters", 1, 64, 20000}, {"one wave, 200k iters", 1, 64, 200000},
        {"one wave again", 1, 64, 200000}, {"4096 blocks x 256", 4096, 256, 20000}, {"one wave after load", 1, 64, 200000}};
    for (auto &r : runs) {
        hipLaunchKernelGGL(spin, dim3(r.blocks), dim3(r.threads), 0, 0, d, r.iters, 1u);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
        const double us = h[1] / 100.0;
        printf("{\"run\": \"%s\", \"cycles\": %llu, \"us\": %.2f, \"mhz\": %.0f, \"cycles_per_iter\": %.2f}\n", r.name,
               (unsigned long long)h[0], us, h[0] / us, (double)h[0] / r.iters);
    }
    hipFree(d);
    return 0;
}
