// group_f32_hier_policy.hip - the cooperative kernel with both networks of the hierarchical env inside the step
// loop (hum_hier_rollout_fused: per transition the high-level 44 -> 2 network for the envs expecting the high agent,
// the low-level 70 -> 17 network for the others, then the hierarchical step), in a translation unit of its own for
// the same reason as group_f32_policy.hip (no shared inlining / register-allocation decisions with the others)
#include "kernels.h"

namespace hkk {
hipError_t launch_group_f32_4_hier_policy(const KArgs& a, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL((step_group_kernel<float, 4, false, 2>), dim3(nblocks), dim3(4 * GL), 0, s, a);
    return hipGetLastError();
}
}  // namespace hkk
