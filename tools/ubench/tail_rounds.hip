// Microbenchmark (diagnostic, not product): does a wave's work slow down once most waves of the kernel have left?
// Mimics the 16-lane group kernel's W pass + Riccati sweep memory pattern (sqp_group.h): 1024 one-wave blocks, each
// runs ROUNDS rounds of
//   (a) every lane stores 48 doubles of its own 192-byte rows of a per-wave workspace slice (strided partial lines),
//   (b) optionally a workgroup release/acquire fence,
//   (c) a serial chain of 30 steps that each load 6 doubles written by another lane (one step ahead) and do ~200
//       dependent FP64 FMAs,
// and blocks with blockIdx % 5 == 0 run one round more (20 % of the waves: the cfg#2 tol-1e-5 tail).  Per wave the
// s_memrealtime duration of every round is recorded; printed: the mean round time of the common rounds and of the
// tail round, for variants {stores+fence, stores only, no stores}.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kWaves = 1024, kRounds = 3, kStages = 30, kRow = 24;   // 4 instances x 30 stages x 24 doubles per wave

__global__ __launch_bounds__(64) void kern(double* ws, long long* out, int mode) {
  const int b = blockIdx.x, t = threadIdx.x, gi = t >> 4, gl = t & 15;
  double* w = ws + (size_t)b * 4 * kStages * kRow + (size_t)gi * kStages * kRow;
  const int rounds = kRounds + (b % 5 == 0 ? 1 : 0);
  double acc = t * 1e-3;
  for (int r = 0; r < rounds; ++r) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    if (mode != 2) {   // (a) W pass: stages gl, gl + 16 of this lane's instance
      for (int k = gl; k < kStages; k += 16)
        for (int j = 0; j < kRow; ++j) w[k * kRow + j] = acc + j + r;
    }
    if (mode == 0) {   // (b)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    // (c) serial sweep: 6 loads of stage k - 1 (prefetched one stage ahead), ~200 dependent FMAs
    double nb[6];
    for (int j = 0; j < 6; ++j) nb[j] = w[(kStages - 1) * kRow + (gl % 4) * 6 + j];
    for (int k = kStages - 1; k >= 0; --k) {
      double cur[6];
      for (int j = 0; j < 6; ++j) cur[j] = nb[j];
      if (k > 0)
        for (int j = 0; j < 6; ++j) nb[j] = w[(k - 1) * kRow + (gl % 4) * 6 + j];
      for (int i = 0; i < 33; ++i)
        for (int j = 0; j < 6; ++j) acc = fma(acc, 0.999, cur[j] * 1e-9);
    }
    const long long t1 = __builtin_amdgcn_s_memrealtime();
    if (t == 0) out[b * (kRounds + 1) + r] = t1 - t0;
  }
  ws[(size_t)kWaves * 4 * kStages * kRow + b * 64 + t] = acc;
}

int main() {
  double* ws;
  long long* out;
  const size_t n = (size_t)kWaves * 4 * kStages * kRow + kWaves * 64;
  hipMalloc(&ws, n * sizeof(double));
  hipMemset(ws, 0, n * sizeof(double));
  hipMalloc(&out, kWaves * (kRounds + 1) * sizeof(long long));
  const char* names[] = {"stores+fence", "stores      ", "no stores   "};
  for (int mode = 0; mode < 3; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      kern<<<kWaves, 64>>>(ws, out, mode);
      hipDeviceSynchronize();
      std::vector<long long> o(kWaves * (kRounds + 1));
      hipMemcpy(o.data(), out, o.size() * sizeof(long long), hipMemcpyDeviceToHost);
      double common = 0, tail = 0;
      int nc = 0, nt = 0;
      for (int b = 0; b < kWaves; ++b) {
        for (int r = 0; r < kRounds; ++r) { common += o[b * (kRounds + 1) + r]; ++nc; }
        if (b % 5 == 0) { tail += o[b * (kRounds + 1) + kRounds]; ++nt; }
      }
      printf("%s rep %d: common round %.2f us, tail round (20 %% of the waves alone) %.2f us\n", names[mode], rep,
             common / nc / 100.0, tail / nt / 100.0);
    }
  return 0;
}
