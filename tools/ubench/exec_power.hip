// Microbenchmark (diagnostic, not product): does masking lanes off (EXEC) raise the shader clock of an FP64-bound
// wave?  One wave per SIMD (grid 1024) or one per two SIMDs (grid 512), 8 independent v_fma_f64 chains per wave,
// with ACT of every 16 lanes active (16 = all; 6 = one instance row of the 2-link group kernel's lane-distributed
// sweeps, 4 = its x rows).  Prints the wave's own cycles per instruction (s_memtime), the wall time and the clock
// they imply.  The 16-lane group kernel's serial sweeps run on all 64 lanes although only NS of every 16 carry rows.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int R = 32768;

template <int ACT>
__global__ __launch_bounds__(64) void kern(double* out, long long* cyc, double a, double b) {
  const int t = threadIdx.x;
  double y[8];
  for (int j = 0; j < 8; ++j) y[j] = out[t] + j;
  const long long c0 = __builtin_amdgcn_s_memtime();
  if ((t & 15) < ACT) {
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = fma(y[j], a, b);
      asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
    }
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
  for (int j = 0; j < 8; ++j) s += y[j];
  out[blockIdx.x * 64 + t] = s;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int ACT>
void run(double* d, long long* c) {
  for (int grid : {1024, 512, 256}) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<ACT><<<grid, 64>>>(d, c, 0.999, 1e-3);
    hipEventRecord(e0);
    kern<ACT><<<grid, 64>>>(d, c, 0.999, 1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    static long long h[4096];
    hipMemcpy(h, c, grid * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < grid; ++i) mean += h[i];
    mean /= grid;
    printf("active %2d/16 lanes, %4d waves: per-wave %6.2f cyc/instr, wall %.3f ms, clock %.2f GHz\n", ACT, grid,
           mean / (R * 8.0), ms, mean / (ms * 1e-3) * 1e-9);
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
  run<16>(d, c);
  run<6>(d, c);
  run<4>(d, c);
  run<16>(d, c);
  return 0;
}
