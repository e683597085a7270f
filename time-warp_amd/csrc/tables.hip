// Link tables drawn on the GPU (tw_draw_link_table, include/timewarp.h).
//
// random-1.1's StdGen (an un-vendored dependency of the reference, lts-7.9;
// its published algorithm; restated on the host in
// timewarp/stdgen.py):
//   mkStdGen s : s' = s .&. 0x7fffffff (s taken as Int32); (q, s1) = s' divMod
//                2147483562; s2 = q mod 2147483398; StdGen (s1+1) (s2+1)
//   next       : L'Ecuyer's combined MLCG (Schrage steps), z in [1, 2147483562]
//   randomR    : for ranges k <= 2147483, one `next`: lo + (z - 1) mod k
// Every intermediate fits in 32 bits: 40014 * (s1 mod 53668) <= 2,147,431,938
// and 40692 * (s2 mod 52774) <= 2,147,438,916, both below 2^31.
//
// One thread per replica walks its own generator through the drawn links in
// the host's order; lanes are consecutive replicas, so each draw's stores
// (table[l][k][r], replica-minor) coalesce into whole lines.  The walk is a
// dependent chain of ~20 ALU ops per draw: C3's 65,536 replicas x 8,192 draws
// take milliseconds against the host's ~13 s of numpy vector steps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/timewarp.h"

namespace {

struct Gen {
    int32_t s1, s2;
};

__device__ __forceinline__ Gen mk_stdgen(int64_t seed) {
    const int32_t s = (int32_t)(uint32_t)(uint64_t)seed & 0x7FFFFFFF;
    return Gen{s % 2147483562 + 1, (s / 2147483562) % 2147483398 + 1};
}

__device__ __forceinline__ uint32_t next(Gen& g) {
    const int32_t k = g.s1 / 53668;
    int32_t s1 = 40014 * (g.s1 - k * 53668) - k * 12211;
    s1 += s1 < 0 ? 2147483563 : 0;
    const int32_t k2 = g.s2 / 52774;
    int32_t s2 = 40692 * (g.s2 - k2 * 52774) - k2 * 3791;
    s2 += s2 < 0 ? 2147483399 : 0;
    g.s1 = s1;
    g.s2 = s2;
    const int32_t z = s1 - s2;
    return (uint32_t)(z < 1 ? z + 2147483562 : z);
}

// a drawn link: lo and the range size k (hi - lo + 1), in walk order
struct DrawLink {
    uint32_t link;
    uint32_t k;
    int64_t lo;
};

__global__ void __launch_bounds__(256) tw_draw_kernel(const DrawLink* __restrict__ links, uint32_t n_drawn,
                                                      uint32_t D, uint32_t R, uint32_t drop_k, int64_t seed_base,
                                                      uint32_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    Gen g = mk_stdgen(seed_base + (int64_t)r);
    for (uint32_t i = 0; i < n_drawn; ++i) {
        const DrawLink dl = links[i];  // uniform across the wave: a scalar load
        uint32_t* row = out + (size_t)dl.link * D * R + r;
        for (uint32_t k = 0; k < D; ++k) {
            uint32_t e = (uint32_t)(dl.lo + (int64_t)((next(g) - 1u) % dl.k));
            if (drop_k) e |= ((next(g) - 1u) % drop_k) == 0 ? TW_LINK_DROP : 0u;
            row[(size_t)k * R] = e;
        }
    }
}

// the constant links' entries: row l (D x R words) = cval[l] unless the link is drawn
__global__ void __launch_bounds__(256) tw_fill_kernel(const uint32_t* __restrict__ cval, const uint8_t* __restrict__ drawn,
                                                      uint32_t L, size_t row, uint32_t* __restrict__ out) {
    for (uint32_t l = blockIdx.y; l < L; l += gridDim.y) {
        if (drawn[l]) continue;
        const uint32_t v = cval[l];
        uint32_t* o = out + (size_t)l * row;
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < row; i += (size_t)gridDim.x * blockDim.x)
            o[i] = v;
    }
}

}  // namespace

extern "C" int tw_draw_link_table(int device, const tw_table_draw* s, uint32_t* out) {
    if (!s || !out || !s->drawn || !s->lo || (!s->hi && s->n_links) || s->n_links == 0 || s->link_depth == 0 ||
        s->n_replicas == 0 || s->drop_log2 < 0 || s->drop_log2 > 21)
        return TW_ERR_INVALID;
    const uint32_t L = s->n_links, D = s->link_depth, R = s->n_replicas;
    std::vector<DrawLink> dl;
    std::vector<uint32_t> cval(L, 0);  // constant links' entry
    std::vector<uint8_t> drawn(L, 0);
    for (uint32_t l = 0; l < L; ++l) {
        if (s->drawn[l]) {
            int64_t lo = s->lo[l], hi = s->hi[l];
            if (lo > hi) std::swap(lo, hi);  // randomR swaps a reversed range
            const int64_t k = hi - lo + 1;
            if (lo < 0 || hi > 0x7FFFFFFF || k * 1000 > 2147483562) return TW_ERR_INVALID;
            dl.push_back(DrawLink{l, (uint32_t)k, lo});
            drawn[l] = 1;
        } else {
            if (s->lo[l] < 0 || s->lo[l] > 0x7FFFFFFF) return TW_ERR_INVALID;
            cval[l] = (uint32_t)s->lo[l];
        }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return TW_ERR_NO_DEVICE;
    // the calling thread's current device is restored on every return below
    // (a torch or multi-GPU host process keeps its own device selection)
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (hipSetDevice(device) != hipSuccess) return TW_ERR_NO_DEVICE;
    const size_t n = (size_t)L * D * R;
    uint32_t* d_out = nullptr;
    DrawLink* d_links = nullptr;
    uint32_t* d_cval = nullptr;
    uint8_t* d_drawn = nullptr;
    hipStream_t st = nullptr;
    int rc = TW_OK;
    auto chk = [&](hipError_t e) {
        if (e != hipSuccess && rc == TW_OK) rc = e == hipErrorOutOfMemory ? TW_ERR_OOM : TW_ERR_HIP;
        return rc == TW_OK;
    };
    if (chk(hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) && chk(hipMalloc(&d_out, 4 * n)) &&
        chk(hipMalloc(&d_links, sizeof(DrawLink) * (dl.size() + 1))) && chk(hipMalloc(&d_cval, 4ull * L)) &&
        chk(hipMalloc(&d_drawn, L)) &&
        chk(hipMemcpyAsync(d_links, dl.data(), sizeof(DrawLink) * dl.size(), hipMemcpyHostToDevice, st)) &&
        chk(hipMemcpyAsync(d_cval, cval.data(), 4ull * L, hipMemcpyHostToDevice, st)) &&
        chk(hipMemcpyAsync(d_drawn, drawn.data(), L, hipMemcpyHostToDevice, st))) {
        if (dl.size() < L) {
            const size_t row = (size_t)D * R;
            const uint32_t gx = (uint32_t)std::min<size_t>((row + 255) / 256, 64);
            hipLaunchKernelGGL(tw_fill_kernel, dim3(gx, std::min<uint32_t>(L, 4096)), dim3(256), 0, st, d_cval,
                               d_drawn, L, row, d_out);
        }
        if (!dl.empty())
            hipLaunchKernelGGL(tw_draw_kernel, dim3((R + 255) / 256), dim3(256), 0, st, d_links,
                               (uint32_t)dl.size(), D, R, s->drop_log2 ? (1u << s->drop_log2) : 0u, s->seed_base,
                               d_out);
        if (chk(hipGetLastError()) && chk(hipMemcpyAsync(out, d_out, 4 * n, hipMemcpyDeviceToHost, st)))
            chk(hipStreamSynchronize(st));
    }
    if (d_drawn) (void)hipFree(d_drawn);
    if (d_cval) (void)hipFree(d_cval);
    if (d_links) (void)hipFree(d_links);
    if (d_out) (void)hipFree(d_out);
    if (st) (void)hipStreamDestroy(st);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return rc;
}
