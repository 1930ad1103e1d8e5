// lane_kernels.hip -- translation unit of the lane-per-instance Riccati kernels (sqp_lane.h), built with
// -mllvm -sgpr-regalloc=basic (Makefile LANEFLAGS; why: lane_launch.h).  A library generated for SX-defined dynamics
// (ModelGenerator::compile_model) compiles this file with the same -DMMPC_USER_MODEL_HEADER as mmpc.hip.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mmpc.h"
#include "lane_launch.h"
#include "models.h"
#include "sqp_lane.h"
#ifdef MMPC_USER_MODEL_HEADER
#include MMPC_USER_MODEL_HEADER
#define MMPC_LANE_BUILTIN_MODELS 0
#else
#define MMPC_LANE_BUILTIN_MODELS 1
#endif

namespace mmpc {
namespace {
template <class Model, class FT>
void launch_lane(bool bounded, bool xb, bool exact, dim3 grid, dim3 block, hipStream_t stream, const SolveParams& p,
                 LaneWork lw) {
    if constexpr (HasHess<Model>::value && std::is_same<FT, double>::value) {
        if (exact) {
            if (xb) sqp_lane_kernel<Model, double, false, true, true><<<grid, block, 0, stream>>>(p, lw);
            else if (bounded) sqp_lane_kernel<Model, double, true, false, true><<<grid, block, 0, stream>>>(p, lw);
            else sqp_lane_kernel<Model, double, false, false, true><<<grid, block, 0, stream>>>(p, lw);
            return;
        }
    }
    if (xb) sqp_lane_kernel<Model, FT, false, true><<<grid, block, 0, stream>>>(p, lw);
    else if (bounded) sqp_lane_kernel<Model, FT, true><<<grid, block, 0, stream>>>(p, lw);
    else sqp_lane_kernel<Model, FT, false><<<grid, block, 0, stream>>>(p, lw);
}
template <class Model>
void launch_model(bool fp32, bool bounded, bool xb, bool exact, dim3 grid, dim3 block, hipStream_t stream,
                  const SolveParams& p, LaneWork lw) {
    if (fp32) launch_lane<Model, float>(bounded, xb, false, grid, block, stream, p, lw);
    else launch_lane<Model, double>(bounded, xb, exact, grid, block, stream, p, lw);
}
}  // namespace

int launch_lane_kernels(int model_id, bool fp32, bool bounded, bool xb, bool exact, dim3 grid, dim3 block,
                        hipStream_t stream, const SolveParams& p, const LaneWork& lw) {
#if MMPC_LANE_BUILTIN_MODELS
    if (model_id == MMPC_MODEL_TWO_LINK_ARM) {
        launch_model<TwoLinkArm>(fp32, bounded, xb, exact, grid, block, stream, p, lw);
        return 0;
    }
    if (model_id == MMPC_MODEL_EXO_ARM) {
        launch_model<ExoArm>(fp32, bounded, xb, exact, grid, block, stream, p, lw);
        return 0;
    }
#else
    if (model_id == MMPC_MODEL_USER) {
        launch_model<UserModel>(fp32, bounded, xb, exact, grid, block, stream, p, lw);
        return 0;
    }
#endif
    return -1;
}

// this translation unit's copy of the phase-timing table (device variables are per code object without -fgpu-rdc)
hipError_t lane_phase_cycles(unsigned long long* out16, int n, bool reset) { return phase_table_read(out16, n, reset); }
}  // namespace mmpc
