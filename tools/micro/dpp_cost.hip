// Micro-benchmark (diagnostic): issue cost and dependent latency of DPP adds vs plain VALU adds, one wave per SIMD.
// 1024 blocks of 64 threads (one wave per SIMD on 256 CUs); per-thread s_memtime around an unrolled loop.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(64) k(float* out, unsigned long long* cyc, int iters) {
    float a = threadIdx.x * 1e-3f, b = a + 1, c = a + 2, d = a + 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if constexpr (MODE == 0) {   // dependent plain adds
                a = a + __int_as_float(__float_as_int(a) ^ 0) * 0.5f;
            } else if constexpr (MODE == 1) {   // dependent DPP adds (row_ror:1)
                a = a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x121, 0xF, 0xF, true));
            } else if constexpr (MODE == 2) {   // 4 independent DPP add chains
                a = a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x121, 0xF, 0xF, true));
                b = b + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b), 0x122, 0xF, 0xF, true));
                c = c + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c), 0x124, 0xF, 0xF, true));
                d = d + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x128, 0xF, 0xF, true));
            } else if constexpr (MODE == 3) {   // 4 independent plain fma chains
                a = fmaf(a, 0.999f, 1e-3f); b = fmaf(b, 0.999f, 1e-3f); c = fmaf(c, 0.999f, 1e-3f); d = fmaf(d, 0.999f, 1e-3f);
            } else {   // 4 independent row_newbcast movs feeding adds
                a = a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x150, 0xF, 0xF, false));
                b = b + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b), 0x151, 0xF, 0xF, false));
                c = c + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(c), 0x152, 0xF, 0xF, false));
                d = d + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x153, 0xF, 0xF, false));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
double run(float* out, unsigned long long* cyc, unsigned long long* h, int iters) {
    hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(64), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(64), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 1024 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 1024; i++) s += h[i];
    return s / 1024 / iters / 16;   // cycles per inner step
}

int main() {
    float* out; unsigned long long* cyc; static unsigned long long h[1024];
    hipMalloc(&out, 1024 * 64 * 4); hipMalloc(&cyc, 1024 * 8);
    const int it = 2000;
    printf("dependent plain add (+xor) : %.2f cyc/step\n", run<0>(out, cyc, h, it));
    printf("dependent DPP add ror1     : %.2f cyc/step\n", run<1>(out, cyc, h, it));
    printf("4 indep DPP add chains     : %.2f cyc/step (4 instr)\n", run<2>(out, cyc, h, it));
    printf("4 indep fma chains         : %.2f cyc/step (4 instr)\n", run<3>(out, cyc, h, it));
    printf("4 indep newbcast+add       : %.2f cyc/step (4 instr)\n", run<4>(out, cyc, h, it));
    return 0;
}
