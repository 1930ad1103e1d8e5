// Microbenchmark (diagnostic, not product): VALU issue throughput per SIMD at 1, 2 and 4 waves per SIMD.
// Each wave runs R steps of 8 independent chains of one operation; the shader-clock cycles per step (s_memtime,
// per wave) and the wall time give cycles per wave-instruction for one wave alone and for co-resident waves:
//   f64 fma | f64 mul | f32 fma | v_mov_b64_dpp row_newbcast | dpp + f64 fma pair | u32 add
// Decides whether a second wave per SIMD adds FP64 issue bandwidth (SIMD-32: a wave64 instruction is 2 passes).
// Round 4: R = 32768 steps (262,144 instructions per wave, ~1 ms) so the ~6 us launch overhead no longer inflates the
// wall-clock "SIMD throughput" column (round 3 ran R = 512: 4,096 instructions, 13-44 us kernels); the effective
// shader clock (s_memtime cycles / wall time) is printed so both columns are in the same cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
#ifndef R_STEPS
#define R_STEPS 32768
#endif
constexpr int R = R_STEPS;
template <int L> __device__ __forceinline__ double bc(double v) { return __builtin_amdgcn_update_dpp(v, v, 0x150 + L, 0xf, 0xf, true); }

template <int OP>
__global__ __launch_bounds__(64) void kern(double* out, long long* cyc, double a, double b) {
  const int t = threadIdx.x;
  double y[8];
  float z[8];
  unsigned u[8];
  for (int j = 0; j < 8; ++j) { y[j] = out[t] + j; z[j] = (float)y[j]; u[j] = t + j; }
  const long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == 0) y[j] = fma(y[j], a, b);
      if constexpr (OP == 1) y[j] = y[j] * a;
      if constexpr (OP == 2) z[j] = fmaf(z[j], (float)a, (float)b);
      if constexpr (OP == 3) y[j] = bc<5>(y[j]);
      if constexpr (OP == 4) y[j] = fma(bc<5>(y[j]), a, b);
      if constexpr (OP == 5) u[j] = u[j] + 0x9e3779b9u;
    }
    asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
    asm volatile("" : "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(z[4]), "+v"(z[5]), "+v"(z[6]), "+v"(z[7]));
    asm volatile("" : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]));
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
  for (int j = 0; j < 8; ++j) s += y[j] + z[j] + u[j];
  out[blockIdx.x * 64 + t] = s;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int OP>
void run(const char* name, double* d, long long* c) {
  for (int grid : {1024, 2048, 4096}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<OP><<<grid, 64>>>(d, c, 0.999, 1e-3);
    hipEventRecord(e0);
    kern<OP><<<grid, 64>>>(d, c, 0.999, 1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    static long long h[4096];
    hipMemcpy(h, c, grid * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < grid; ++i) mean += h[i];
    mean /= grid;
    const double per_wave = mean / (R * 8.0);                       // wave's own cycles per instruction
    const double clk = mean / (ms * 1e-3);                          // s_memtime cycles per second of wall time
    const double wall_simd = ms * 1e-3 * clk * 1024 / (grid * R * 8.0);  // SIMD cycles per wave-instr, same clock
    printf("%-28s waves/SIMD %d: per-wave %6.2f cyc/instr, per-wave / waves %6.2f, SIMD throughput (wall) %6.2f "
           "cyc/instr, clock %.2f GHz (wall %.3f ms)\n", name, grid / 1024, per_wave, per_wave / (grid / 1024), wall_simd,
           clk * 1e-9, ms);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
}

int main() {
  double* d;
  long long* c;
  hipMalloc(&d, 64 * 8 * 4096);
  hipMalloc(&c, 8 * 4096);
  hipMemset(d, 0, 64 * 8 * 4096);
  run<0>("fma f64", d, c);
  run<1>("mul f64", d, c);
  run<2>("fma f32", d, c);
  run<3>("v_mov_b64_dpp newbcast", d, c);
  run<4>("dpp + fma f64 (per pair)", d, c);
  run<5>("add u32", d, c);
  return 0;
}
