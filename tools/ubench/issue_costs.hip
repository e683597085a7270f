// Micro-benchmark: per-instruction costs at ONE wave per SIMD (1024 waves on
// 256 CUs), the occupancy of the event engine.  Each test runs a loop of
// N iterations; cycles per iteration come from s_memtime around the loop.
// Build: hipcc -O3 --offload-arch=gfx950 -o issue_costs issue_costs.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define N 4096

template <int T>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned long long* cyc, unsigned seed) {
    __shared__ unsigned lds[256 * 16];
    unsigned tid = threadIdx.x;
    for (int i = 0; i < 16; ++i) lds[i * 256 + tid] = (tid + i * 7 + 1) & 15;
    __syncthreads();
    unsigned v = tid ^ seed, w = tid * 3, x = tid + 7, y = seed;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        if (T == 0) {  // 8 dependent VALU
            asm volatile("v_add_u32 %0, %0, 1\n v_xor_b32 %0, %0, 5\n v_add_u32 %0, %0, 3\n v_xor_b32 %0, %0, 9\n"
                         "v_add_u32 %0, %0, 1\n v_xor_b32 %0, %0, 5\n v_add_u32 %0, %0, 3\n v_xor_b32 %0, %0, 9" : "+v"(v));
        } else if (T == 1) {  // 8 independent VALU (4 chains)
            asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
                         "v_xor_b32 %0, %0, 5\n v_xor_b32 %1, %1, 5\n v_xor_b32 %2, %2, 5\n v_xor_b32 %3, %3, 5"
                         : "+v"(v), "+v"(w), "+v"(x), "+v"(y));
        } else if (T == 2) {  // 8 taken scalar branches
            asm volatile("s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_1\n s_nop 0\n L%=_1:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_2\n s_nop 0\n L%=_2:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_3\n s_nop 0\n L%=_3:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_4\n s_nop 0\n L%=_4:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_5\n s_nop 0\n L%=_5:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_6\n s_nop 0\n L%=_6:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_7\n s_nop 0\n L%=_7:\n"
                         "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 L%=_8\n s_nop 0\n L%=_8:\n" :: "s"(seed) : "scc");
        } else if (T == 3) {  // 8 NOT-taken scalar branches
            asm volatile("s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_1\n L%=_1:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_2\n L%=_2:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_3\n L%=_3:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_4\n L%=_4:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_5\n L%=_5:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_6\n L%=_6:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_7\n L%=_7:\n"
                         "s_cmp_eq_u32 %0, 12345\n s_cbranch_scc1 L%=_8\n L%=_8:\n" :: "s"(seed) : "scc");
        } else if (T == 4) {  // 2 dependent LDS reads
            v = lds[(v & 15) * 256 + tid];
            v = lds[(v & 15) * 256 + tid];
        } else if (T == 5) {  // 8 dependent SALU
            asm volatile("s_add_u32 %0, %0, 1\n s_xor_b32 %0, %0, 5\n s_add_u32 %0, %0, 3\n s_xor_b32 %0, %0, 9\n"
                         "s_add_u32 %0, %0, 1\n s_xor_b32 %0, %0, 5\n s_add_u32 %0, %0, 3\n s_xor_b32 %0, %0, 9" : "+s"(y) : : "scc");
        } else if (T == 6) {  // 4x (v_cmp -> s_and_saveexec -> s_or exec) divergent-if skeleton, all lanes true
            asm volatile("v_cmp_ne_u32 vcc, %1, -1\n s_and_saveexec_b64 s[40:41], vcc\n s_cbranch_execz L%=_1\n v_add_u32 %0, %0, 1\n L%=_1:\n s_or_b64 exec, exec, s[40:41]\n"
                         "v_cmp_ne_u32 vcc, %1, -1\n s_and_saveexec_b64 s[40:41], vcc\n s_cbranch_execz L%=_2\n v_add_u32 %0, %0, 1\n L%=_2:\n s_or_b64 exec, exec, s[40:41]\n"
                         "v_cmp_ne_u32 vcc, %1, -1\n s_and_saveexec_b64 s[40:41], vcc\n s_cbranch_execz L%=_3\n v_add_u32 %0, %0, 1\n L%=_3:\n s_or_b64 exec, exec, s[40:41]\n"
                         "v_cmp_ne_u32 vcc, %1, -1\n s_and_saveexec_b64 s[40:41], vcc\n s_cbranch_execz L%=_4\n v_add_u32 %0, %0, 1\n L%=_4:\n s_or_b64 exec, exec, s[40:41]\n"
                         : "+v"(v) : "v"(w) : "vcc", "s40", "s41", "scc", "exec");
        } else if (T == 7) {  // 4x readfirstlane -> s_cmp -> branch (waterfall head)
            unsigned s;
            asm volatile("v_readfirstlane_b32 %1, %0\n s_cmp_eq_u32 %1, 12345\n s_cbranch_scc1 L%=_1\n L%=_1:\n"
                         "v_readfirstlane_b32 %1, %0\n s_cmp_eq_u32 %1, 12345\n s_cbranch_scc1 L%=_2\n L%=_2:\n"
                         "v_readfirstlane_b32 %1, %0\n s_cmp_eq_u32 %1, 12345\n s_cbranch_scc1 L%=_3\n L%=_3:\n"
                         "v_readfirstlane_b32 %1, %0\n s_cmp_eq_u32 %1, 12345\n s_cbranch_scc1 L%=_4\n L%=_4:\n"
                         : "+v"(v), "=s"(s) : : "scc");
        } else if (T == 8) {  // 1 global load (L2-resident, per-lane) + use
            v = out[(v & 1023) * 64 + (tid & 63)] + 1;
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + tid + 65536] = v + w + x + y;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int T>
double run(unsigned* d_out, unsigned long long* d_cyc) {
    hipLaunchKernelGGL(k<T>, dim3(256), dim3(256), 0, 0, d_out, d_cyc, 1u);
    hipLaunchKernelGGL(k<T>, dim3(256), dim3(256), 0, 0, d_out, d_cyc, 1u);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(256);
    hipMemcpy(c.data(), d_cyc, 256 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto x : c) s += x;
    return s / 256 / N;
}

int main(int argc, char** argv) {
    unsigned* d_out;
    unsigned long long* d_cyc;
    hipMalloc(&d_out, (65536 * 2 + 1024 * 64) * 4);
    hipMemset(d_out, 0, (65536 * 2 + 1024 * 64) * 4);
    hipMalloc(&d_cyc, 256 * 8);
    const char* names[] = {"8 dep VALU", "8 indep VALU", "8 taken s_cbranch", "8 untaken s_cbranch", "2 dep LDS reads",
                           "8 dep SALU", "4 divergent-if skeletons", "4 readfirstlane+cmp+branch", "1 global load L2"};
    int t = argc > 1 ? atoi(argv[1]) : 0;
    double r = 0;
    switch (t) {
    case 0: r = run<0>(d_out, d_cyc); break;
    case 1: r = run<1>(d_out, d_cyc); break;
    case 2: r = run<2>(d_out, d_cyc); break;
    case 3: r = run<3>(d_out, d_cyc); break;
    case 4: r = run<4>(d_out, d_cyc); break;
    case 5: r = run<5>(d_out, d_cyc); break;
    case 6: r = run<6>(d_out, d_cyc); break;
    case 7: r = run<7>(d_out, d_cyc); break;
    case 8: r = run<8>(d_out, d_cyc); break;
    }
    printf("%-28s %8.1f cycles/iter\n", names[t], r);
    return 0;
}
