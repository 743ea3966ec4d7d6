// Micro-benchmark (diagnostic): what SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU count on gfx950 when
// only M of a wave's 64 lanes are active (exec mask), for tools/lane_util.py's per-phase lane utilisation.
// 1024 blocks of one wave; each active lane runs 4 independent fp32 fma chains, ITER x 16 fmas each.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 256;

template <int M>
__global__ void __launch_bounds__(64) lanes_active(float* out) {
    float a = threadIdx.x * 1e-3f, b = a + 1, c = a + 2, d = a + 3;
    if ((int)(threadIdx.x & 63) < M) {
        for (int i = 0; i < ITER; i++) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                a = fmaf(a, 0.999f, 1e-3f); b = fmaf(b, 0.999f, 1e-3f);
                c = fmaf(c, 0.999f, 1e-3f); d = fmaf(d, 0.999f, 1e-3f);
            }
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a + b + c + d;
}

template <int M>
void run(float* out) {
    hipLaunchKernelGGL(lanes_active<M>, dim3(1024), dim3(64), 0, 0, out);
}

int main() {
    float* out;
    if (hipMalloc(&out, 1024 * 64 * sizeof(float)) != hipSuccess) return 1;
    run<64>(out); run<32>(out); run<16>(out); run<4>(out); run<1>(out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("lane_util: 5 kernels x 1024 waves x %d fmas per active lane\n", ITER * 64);
    (void)hipFree(out);
    return 0;
}
