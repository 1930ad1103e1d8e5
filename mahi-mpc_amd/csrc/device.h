// device.h -- the qualifier of the device model and solver helpers (inlined into the kernels).
#pragma once
#include <hip/hip_runtime.h>

#define MMPC_HD __device__ __forceinline__
