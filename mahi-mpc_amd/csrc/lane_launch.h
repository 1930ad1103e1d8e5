// lane_launch.h -- the lane-per-instance Riccati kernels (sqp_lane.h) are compiled in their own translation unit,
// lane_kernels.hip, with the basic instead of the greedy SGPR register allocator (-mllvm -sgpr-regalloc=basic):
// five exo lane-kernel builds at the 512-register limit computed wrong steps with the greedy allocator of ROCm 7.2's
// LLVM and right ones with either basic allocator, from the same IR ("wrong-result builds").
// mmpc.hip launches them only through this entry point, so no lane kernel is instantiated in its translation unit.
#pragma once
#include <hip/hip_runtime.h>

#include "sqp_wave.h"

namespace mmpc {
struct LaneWork;
// 0, or -1 when model_id is not compiled into this library
int launch_lane_kernels(int model_id, bool fp32, bool bounded, bool xb, bool exact, dim3 grid, dim3 block,
                        hipStream_t stream, const SolveParams& p, const LaneWork& lw);
// the phase-timing table of the lane kernels (diagnostic build; mmpc_debug_phase_cycles adds it to its own)
hipError_t lane_phase_cycles(unsigned long long* out16, int n, bool reset);
}  // namespace mmpc
