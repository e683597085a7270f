// Shader clock under light and heavy load: each wave runs a dependent VALU
// chain and records s_memtime (shader clock) and s_memrealtime (100 MHz
// constant clock) around it; the ratio of the deltas is the clock in MHz.
// usage: clock_probe  (prints one line per grid size)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(64) chain(uint64_t* out, uint32_t iters) {
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        x = x * 1664525u + 1013904223u;
        x ^= x >> 13;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 3 + 0] = t1 - t0;
        out[blockIdx.x * 3 + 1] = r1 - r0;
        out[blockIdx.x * 3 + 2] = x;
    }
}

int main() {
    const int grids[] = {1, 64, 256, 1024, 4096};
    uint64_t* d = nullptr;
    hipMalloc(&d, 3 * 8 * 4096);
    for (int g : grids) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(chain, dim3(g), dim3(64), 0, 0, d, 2000000u);
            hipDeviceSynchronize();
        }
        std::vector<uint64_t> h(3 * g);
        hipMemcpy(h.data(), d, 24 * g, hipMemcpyDeviceToHost);
        double mhz = 0;
        for (int i = 0; i < g; ++i) mhz += (double)h[3 * i] / (double)h[3 * i + 1] * 100.0;
        printf("{\"waves\": %d, \"shader_mhz\": %.1f, \"ms\": %.2f}\n", g, mhz / g, h[1] / 1e5);
    }
    hipFree(d);
    return 0;
}
