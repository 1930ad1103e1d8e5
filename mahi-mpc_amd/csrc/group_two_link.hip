// group_two_link.hip -- the built-in 2-link arm's 16-lane group kernels (sqp_group.h; the cfg#2 headline path) in
// translation units of their own.  This file is compiled twice (Makefile):
//   * build/group_two_link.o: the UNBOUNDED kernels (Gauss-Newton and exact Hessian, the cfg#2 path) with LLVM's
//     default (greedy) register allocators -- they allocate without VGPR spills or scratch (tests/test_build_flags.py
//     checks the built code object's metadata), and run ~1 % faster than with the basic SGPR allocator;
//   * build/group_two_link_bounded.o (-DMMPC_GROUP_BOUNDED_UNIT): the control-bounded and state-bounded kernels with
//     -mllvm -sgpr-regalloc=basic like every other unit: they reach the 512-register limit with VGPR spills to
//     scratch, the profile of the greedy-allocator miscompiles of DESIGN.md 4b.
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
// this translation unit's copy of the phase-timing table (as lane_kernels.hip)
hipError_t unit_phase_cycles(unsigned long long* out16, int n, bool reset) { return phase_table_read(out16, n, reset); }
}  // namespace

#ifndef MMPC_GROUP_BOUNDED_UNIT
hipError_t launch_group_two_link(bool exact, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                                 const SolveParams& p, const GroupWork& gwk) {
    return exact ? launch<false, false, true>(grid, block, lds, stream, p, gwk)
                 : launch<false>(grid, block, lds, stream, p, gwk);
}
hipError_t group_two_link_phase_cycles(unsigned long long* out16, int n, bool reset) {
    return unit_phase_cycles(out16, n, reset);
}
#else
hipError_t launch_group_two_link_bounded(bool xb, bool exact, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                                         const SolveParams& p, const GroupWork& gwk) {
    if (xb) return exact ? launch<false, true, true>(grid, block, lds, stream, p, gwk)   // the interior point
                         : launch<false, true>(grid, block, lds, stream, p, gwk);
    return exact ? launch<true, false, true>(grid, block, lds, stream, p, gwk)
                 : launch<true>(grid, block, lds, stream, p, gwk);
}
hipError_t group_two_link_bounded_phase_cycles(unsigned long long* out16, int n, bool reset) {
    return unit_phase_cycles(out16, n, reset);
}
#endif
}  // namespace mmpc
