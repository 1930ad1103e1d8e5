// group_launch.h -- the built-in 2-link arm's group kernels live in group_two_link.hip, the one translation unit
// compiled with the greedy register allocators (why: that file's header); mmpc.hip launches them through this entry.
#pragma once
#include <hip/hip_runtime.h>

#include "sqp_wave.h"

namespace mmpc {
struct GroupWork;
hipError_t launch_group_two_link(bool bounded, bool xb, bool exact, dim3 grid, dim3 block, size_t lds,
                                 hipStream_t stream, const SolveParams& p, const GroupWork& gwk);
// the phase-timing table of those kernels (diagnostic build; mmpc_debug_phase_cycles adds it to its own)
hipError_t group_two_link_phase_cycles(unsigned long long* out16, bool reset);
}  // namespace mmpc
