// Microbenchmark (diagnostic, not product): one wave, shader-clock cycles per dependent step of
//   fma f64 chain | 8 independent fma chains (issue) | fma through v_mov_b64_dpp row_newbcast |
//   fma through __shfl (ds_bpermute) | fma through an LDS write+read round trip | rcp f64 chain
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int R = 256;
template <int L> __device__ __forceinline__ double bc(double v) { return __builtin_amdgcn_update_dpp(v, v, 0x150 + L, 0xf, 0xf, true); }
__global__ void kern(double* out, long long* cyc, double a, double b) {
  __shared__ double s[64];
  const int t = threadIdx.x;
  double x = out[t];
  long long c0, c1;
  // 0: dependent fma chain
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { x = fma(x, a, b); asm volatile("" : "+v"(x)); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[0] = c1 - c0;
  // 1: 8 independent chains
  double y[8];
  for (int j = 0; j < 8; ++j) y[j] = x + j;
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = fma(y[j], a, b);
    asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
  }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[1] = c1 - c0;
  for (int j = 0; j < 8; ++j) x += y[j];
  // 2: dpp newbcast dependent
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { x = fma(bc<3>(x), a, b); asm volatile("" : "+v"(x)); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[2] = c1 - c0;
  // 3: shfl dependent
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { x = fma(__shfl(x, (t & ~15) + 3), a, b); asm volatile("" : "+v"(x)); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[3] = c1 - c0;
  // 4: lds round trip dependent
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { s[t] = x; __builtin_amdgcn_wave_barrier(); x = fma(s[(t & ~15) + 3], a, b); __builtin_amdgcn_wave_barrier(); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[4] = c1 - c0;
  // 5: dependent mul (v_mul_f64)
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { x = x * a; asm volatile("" : "+v"(x)); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[5] = c1 - c0;
  // 6: dependent rcp f64
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) { x = __builtin_amdgcn_rcp(x) + b; asm volatile("" : "+v"(x)); }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[6] = c1 - c0;
  // 7: 8 independent dpp movs + fma (issue of broadcast-operand fma)
  for (int j = 0; j < 8; ++j) y[j] = x + j;
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = fma(bc<5>(y[j]), a, b);
    asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
  }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[7] = c1 - c0;
  for (int j = 0; j < 8; ++j) x += y[j];
  // 8: 8 independent f32 fma chains (reference point)
  float z[8];
  for (int j = 0; j < 8; ++j) z[j] = (float)x + j;
  c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = fmaf(z[j], (float)a, (float)b);
    asm volatile("" : "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(z[4]), "+v"(z[5]), "+v"(z[6]), "+v"(z[7]));
  }
  c1 = __builtin_amdgcn_s_memtime(); if (t == 0) cyc[8] = c1 - c0;
  for (int j = 0; j < 8; ++j) x += z[j];
  out[t] = x;
}
int main() {
  double* d; long long* c; hipMalloc(&d, 64 * 8 * 1024); hipMalloc(&c, 64 * 8);
  hipMemset(d, 0, 64 * 8 * 1024);
  long long h[16];
  const char* names[] = {"dep fma f64", "8 indep fma f64 (per instr)", "dep fma via dpp newbcast", "dep fma via shfl",
                         "dep fma via lds roundtrip", "dep mul f64", "dep rcp f64 + add", "8 indep dpp+fma (per pair)",
                         "8 indep fma f32 (per instr)"};
  for (int grid : {1, 1024}) {
    for (int rep = 0; rep < 2; ++rep) kern<<<grid, 64>>>(d, c, 0.999, 1e-3);
    hipDeviceSynchronize();
    hipMemcpy(h, c, 9 * 8, hipMemcpyDeviceToHost);
    printf("grid %d (memtime counts; divide by steps):\n", grid);
    for (int i = 0; i < 9; ++i) {
      double per = (double)h[i] / R / ((i == 1 || i == 7 || i == 8) ? 8 : 1);
      printf("  %-32s %8.2f\n", names[i], per);
    }
  }
  return 0;
}
