// group_f32.hip - the hierarchical env's cooperative fp32 kernel, 4 envs per wavefront (POLICY 4: the low-level-only
// branches compiled out; the low-level env runs group_f32_low.hip's twin), compiled on its own (see kernels.h for why
// it is a separate translation unit).
#include "kernels.h"

namespace hkk {
hipError_t launch_group_f32_4(const KArgs& a, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL((step_group_kernel<float, 4, false, 4>), dim3(nblocks), dim3(4 * GL), 0, s, a);
    return hipGetLastError();
}
}  // namespace hkk
