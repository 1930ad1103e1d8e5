// group_two_link.hip -- the built-in 2-link arm's 16-lane group kernels (sqp_group.h; the cfg#2 headline path) in a
// translation unit of their own, compiled with LLVM's default (greedy) register allocators.  Every other kernel of the
// library is built with -mllvm -sgpr-regalloc=basic (Makefile REGALLOC): ROCm 7.2's greedy SGPR allocator
// miscompiled kernels at the 512-register limit -- five lane-kernel builds and, in round 4, the exo
// group kernel with the exact Hessian (an illegal memory access after the exo polynomials changed form).  The 2-link
// group kernels do not spill VGPRs and run ~1 % faster with the greedy allocator.
#include <hip/hip_runtime.h>

#include "../../include/mmpc.h"
#include "group_launch.h"
#include "models.h"
#include "sqp_group.h"

namespace mmpc {
namespace {
template <bool BOUNDED, bool XB = false, bool EXACT = false>
hipError_t launch(dim3 grid, dim3 block, size_t lds, hipStream_t stream, const SolveParams& p, GroupWork gwk) {
    auto* k = sqp_group_kernel<TwoLinkArm, BOUNDED, XB, EXACT>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return e;
    }
    k<<<grid, block, lds, stream>>>(p, gwk);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_group_two_link(bool bounded, bool xb, bool exact, dim3 grid, dim3 block, size_t lds,
                                 hipStream_t stream, const SolveParams& p, const GroupWork& gwk) {
    if (exact) return bounded ? launch<true, false, true>(grid, block, lds, stream, p, gwk)
                              : launch<false, false, true>(grid, block, lds, stream, p, gwk);
    if (xb) return launch<false, true>(grid, block, lds, stream, p, gwk);
    return bounded ? launch<true>(grid, block, lds, stream, p, gwk) : launch<false>(grid, block, lds, stream, p, gwk);
}

// this translation unit's copy of the phase-timing table (as lane_kernels.hip)
hipError_t group_two_link_phase_cycles(unsigned long long* out16, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_mmpc_phase_cycles), 16 * sizeof(unsigned long long));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_mmpc_phase_cycles), z, sizeof(z));
    }
    return e;
}
}  // namespace mmpc
