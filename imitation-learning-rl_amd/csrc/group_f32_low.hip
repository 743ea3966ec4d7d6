// group_f32_low.hip - the benchmarked kernel: cooperative, fp32, 4 envs per wavefront, the low-level env only
// (POLICY 3: the hierarchical branches compiled out - bitwise equal to the shared kernel, +0.7 % same box,
// profiles/r05_low_twin_ab.txt).  A translation unit of its own, like the other hot twins: kernels instantiated
// together share inlining / register-allocation decisions (group_f32_policy.hip)
#include "kernels.h"

namespace hkk {
hipError_t launch_group_f32_4_low(const KArgs& a, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL((step_group_kernel<float, 4, false, 3>), dim3(nblocks), dim3(4 * GL), 0, s, a);
    return hipGetLastError();
}
}  // namespace hkk
