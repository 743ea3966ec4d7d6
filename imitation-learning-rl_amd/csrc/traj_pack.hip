// traj_pack.hip - the learner feed's packing launch (include/humanoid_env.h hum_pack_rows): k x n rows of each field
// from time-major step outputs into lane-major per-lane records, one launch for every field.
//
// MI355X mapping: a block per (16 lanes, step, field); its 256 threads walk the 16 rows' bytes as 4-byte words, so
// consecutive threads read consecutive words of a source row (rows of consecutive lanes are adjacent in a time-major
// [k, n, w] output) and write consecutive words of a record row: both sides coalesced within a row.  u8 fields of one
// byte per row (done) go a byte per thread.  HBM-bound: bytes moved = 2 x the fragment.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/humanoid_env.h"

void hum_internal_set_error(const char* msg);

namespace {

struct PackArgs {
    hum_pack_field f[HUM_PACK_MAX_FIELDS];
    int nfields, k, n, t0;
};

constexpr int LANES_PER_BLOCK = 16;

__global__ void __launch_bounds__(256) pack_rows_kernel(PackArgs a) {
    const int t = blockIdx.y, fi = blockIdx.z, i0 = blockIdx.x * LANES_PER_BLOCK;
    const hum_pack_field& f = a.f[fi];
    const char* src = (const char*)f.src + (long)t * f.src_step;
    char* dst = (char*)f.dst + (long)(a.t0 + t) * f.dst_step;
    if (f.row_bytes % 4 == 0) {
        const int w = f.row_bytes / 4, total = LANES_PER_BLOCK * w;
        for (int e = threadIdx.x; e < total; e += blockDim.x) {
            const int r = e / w, c = e - r * w, i = i0 + r;
            if (i < a.n)
                *(int*)(dst + (long)i * f.dst_lane + 4 * c) = *(const int*)(src + (long)i * f.src_lane + 4 * c);
        }
    } else {   // one byte per row
        const int i = i0 + threadIdx.x;
        if (threadIdx.x < LANES_PER_BLOCK && i < a.n) dst[(long)i * f.dst_lane] = src[(long)i * f.src_lane];
    }
}

}  // namespace

extern "C" int hum_pack_rows(const hum_pack_field* fields, int32_t nfields, int32_t k, int32_t n, int32_t t0,
                             void* stream) {
    if (!fields || nfields < 1 || nfields > HUM_PACK_MAX_FIELDS || k < 1 || n < 1 || t0 < 0) {
        hum_internal_set_error("hum_pack_rows: bad argument");
        return HUM_ERR_ARG;
    }
    PackArgs a;
    a.nfields = nfields;
    a.k = k;
    a.n = n;
    a.t0 = t0;
    for (int j = 0; j < nfields; j++) {
        const hum_pack_field& f = fields[j];
        const bool words = f.row_bytes > 0 && f.row_bytes % 4 == 0 && f.src_lane % 4 == 0 && f.dst_lane % 4 == 0 &&
                           f.src_step % 4 == 0 && f.dst_step % 4 == 0 && ((uintptr_t)f.src | (uintptr_t)f.dst) % 4 == 0;
        if (!f.src || !f.dst || !(words || f.row_bytes == 1)) {
            hum_internal_set_error("hum_pack_rows: a field needs row_bytes 1 or a multiple of 4 with 4-byte aligned "
                                   "pointers and strides");
            return HUM_ERR_ARG;
        }
        a.f[j] = f;
    }
    hipLaunchKernelGGL(pack_rows_kernel, dim3((n + LANES_PER_BLOCK - 1) / LANES_PER_BLOCK, k, nfields), dim3(256), 0,
                       (hipStream_t)stream, a);
    const hipError_t st = hipGetLastError();
    if (st != hipSuccess) {
        hum_internal_set_error((std::string("hum_pack_rows: ") + hipGetErrorString(st)).c_str());
        return HUM_ERR_HIP;
    }
    return HUM_OK;
}
