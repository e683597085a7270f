// PMC calibration for tools/pmc_summary.py: how FETCH_SIZE / WRITE_SIZE
// (rocprofv3, KiB per dispatch) relate to the bytes a kernel actually moves on
// gfx950, for the access shapes the engine uses (16 B per lane, coalesced
// across the wave; the thread records are quad-major, so a wave's quad access is
// one contiguous 1 KiB).
//
// Three kernels over a 2 GiB buffer (far past the 256 MB Infinity Cache):
//   read_stream   every lane loads 16 B per iteration (sums them into one word)
//   write_stream  every lane stores 16 B per iteration
//   copy_stream   a read of one half and a write of the other
// Each prints its algorithmic bytes; run it under separate --pmc passes:
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT/f -o run -- ./pmc_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -d OUT/w -o run -- ./pmc_calib
// and tools/pmc_calib.py turns the CSVs into profiles/pmc_calibration.json.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void __launch_bounds__(256) read_stream(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads; practically never stores
}

__global__ void __launch_bounds__(256) write_stream(uint4* __restrict__ p, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i ^ seed, seed, (uint32_t)(i >> 32), 1u);
}

__global__ void __launch_bounds__(256) copy_stream(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

int main() {
    const size_t bytes = 2ull << 30;
    const size_t n = bytes / 16;
    uint4* buf = nullptr;
    uint32_t* out = nullptr;
    CHK(hipMalloc((void**)&buf, bytes));
    CHK(hipMalloc((void**)&out, 4));
    const dim3 grid(256 * 32), block(256);
    hipLaunchKernelGGL(write_stream, grid, block, 0, 0, buf, n, 7u);  // first touch
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(read_stream, grid, block, 0, 0, buf, n, out);
    CHK(hipDeviceSynchronize());
    printf("read_stream bytes_read=%zu bytes_written=0\n", bytes);
    hipLaunchKernelGGL(write_stream, grid, block, 0, 0, buf, n, 11u);
    CHK(hipDeviceSynchronize());
    printf("write_stream bytes_read=0 bytes_written=%zu\n", bytes);
    hipLaunchKernelGGL(copy_stream, grid, block, 0, 0, buf, buf + n / 2, n / 2);
    CHK(hipDeviceSynchronize());
    printf("copy_stream bytes_read=%zu bytes_written=%zu\n", bytes / 2, bytes / 2);
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
