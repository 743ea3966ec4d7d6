// group_f32_policy.hip - the benchmarked kernel's fused-policy twin (hum_rollout_fused: the policy network inside
// the step loop), in a translation unit of its own: instantiated next to the benchmarked kernel it cost that kernel
// 4.3 % (31.4 -> 30.1 M env-steps/s, shared inlining / register-allocation decisions; profiles/r03_pgs_sched_ab.txt)
#include "kernels.h"

namespace hkk {
hipError_t launch_group_f32_4_policy(const KArgs& a, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL((step_group_kernel<float, 4, false, true>), dim3(nblocks), dim3(4 * GL), 0, s, a);
    return hipGetLastError();
}
}  // namespace hkk
