// Micro-benchmark (diagnostic): calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// step kernel uses (MI355X_MICROARCH.md: only 16 B/lane streaming reads and stores are calibrated).  Each kernel
// moves a known byte count (64 MiB, past every L2); compare the counter per dispatch with the printed bytes.
//   rd4   4 B/lane coalesced loads (SoA f32 / i32 state and bookkeeping)
//   rd8   8 B/lane coalesced loads (SoA f64 bookkeeping)
//   rd16  16 B/lane loads (the guide's calibrated case)
//   wr4 / wr8 / wr16 the same widths as stores; wr1 1 B/lane stores (done flags)
//   wrrow 4 lanes per wave store one dword each at a 280-B row stride, 70 dwords per row (the obs row store of
//         the cooperative kernel: lane 0 of each 16-lane env group)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 64ull << 20;

__global__ void rd4(const float* __restrict__ p, float* out, size_t n) {
    float s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
    if (s == 1234.5f) out[0] = s;
}
__global__ void rd8(const double* __restrict__ p, float* out, size_t n) {
    double s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
    if (s == 1234.5) out[0] = (float)s;
}
__global__ void rd16(const float4* __restrict__ p, float* out, size_t n) {
    float s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void wr1(unsigned char* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (unsigned char)i;
}
__global__ void wr4(float* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (float)i;
}
__global__ void wr8(double* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (double)i;
}
__global__ void wr16(float4* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
// rows of 70 floats; one 64-lane wave = 4 rows, lane 16 g stores row g
__global__ void wrrow(float* p, size_t rows) {
    const size_t r = (blockIdx.x * 256ull + threadIdx.x) / 16;
    if ((threadIdx.x & 15) != 0 || r >= rows) return;
#pragma unroll
    for (int k = 0; k < 70; k++) p[r * 70 + k] = (float)k;
}

int main() {
    void* buf;
    float* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 0, BYTES) != hipSuccess) return 1;
    const int G = 2048;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(rd4, dim3(G), dim3(256), 0, 0, (const float*)buf, out, BYTES / 4);
        hipLaunchKernelGGL(rd8, dim3(G), dim3(256), 0, 0, (const double*)buf, out, BYTES / 8);
        hipLaunchKernelGGL(rd16, dim3(G), dim3(256), 0, 0, (const float4*)buf, out, BYTES / 16);
        hipLaunchKernelGGL(wr1, dim3(G), dim3(256), 0, 0, (unsigned char*)buf, BYTES);
        hipLaunchKernelGGL(wr4, dim3(G), dim3(256), 0, 0, (float*)buf, BYTES / 4);
        hipLaunchKernelGGL(wr8, dim3(G), dim3(256), 0, 0, (double*)buf, BYTES / 8);
        hipLaunchKernelGGL(wr16, dim3(G), dim3(256), 0, 0, (float4*)buf, BYTES / 16);
        const size_t rows = BYTES / 280;
        hipLaunchKernelGGL(wrrow, dim3((unsigned)((rows * 16 + 255) / 256)), dim3(256), 0, 0, (float*)buf, rows);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("bytes per dispatch: %zu (wrrow: %zu)\n", BYTES, (BYTES / 280) * 280);
    return 0;
}
