// group_launch.h -- the built-in 2-link arm's group kernels live in group_two_link.hip, compiled as two units: the
// unbounded kernels (cfg#2) with the greedy register allocators, the bounded ones with the basic SGPR allocator (why:
// that file's header); mmpc.hip launches them through these entries.
#pragma once
#include <hip/hip_runtime.h>

#include "sqp_wave.h"

namespace mmpc {
struct GroupWork;
// unbounded solves (build/group_two_link.o)
hipError_t launch_group_two_link(bool exact, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                                 const SolveParams& p, const GroupWork& gwk);
// control-bounded (BOUNDED) and state-bounded (xb, interior point) solves (build/group_two_link_bounded.o)
hipError_t launch_group_two_link_bounded(bool xb, bool exact, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                                         const SolveParams& p, const GroupWork& gwk);
// the phase-timing tables of those units (diagnostic build; mmpc_debug_phase_cycles adds them to its own)
// (the first n <= kPhaseSlots slots of the unit's table)
hipError_t group_two_link_phase_cycles(unsigned long long* out16, int n, bool reset);
hipError_t group_two_link_bounded_phase_cycles(unsigned long long* out16, int n, bool reset);
}  // namespace mmpc
