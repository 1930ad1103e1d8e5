// Microbenchmark (diagnostic, not product): execution rate of a wave once the other waves of its kernel have left.
// 1024 one-wave blocks (one per SIMD, 40 KB of LDS each like the 16-lane group kernel's workgroups, so four per CU);
// blocks b % 5 == 0 ("late" waves, 20 %) time a workload after every other block has left (tail) or while the others
// still run the same workload (busy).  Workloads: a dependent FP64 FMA chain; an LDS write/read chain; a DPP row
// broadcast + FMA chain; global stores of 192-byte rows.  Prints the late waves' mean time per workload.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 20000;

template <int W>
__global__ __launch_bounds__(64) void kern(double* out, long long* t, int tail, double* ws) {
  __shared__ double lds[5120];   // 40 KB
  const int b = blockIdx.x, l = threadIdx.x;
  const bool late = b % 5 == 0;
  double y = out[b * 64 + l] + 1.0;
  for (int i = l; i < 5120; i += 64) lds[i] = i;
  __syncthreads();
  // the other waves: the workload for 2x the late waves' time (busy) or a short warm-up (tail)
  const int pre = late ? (tail ? 4 * kIters : 0) : (tail ? kIters / 4 : 4 * kIters);
  for (int i = 0; i < pre; ++i) {
    y = fma(y, 0.999, 1e-3);
    asm volatile("" : "+v"(y));
  }
  if (late) {
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    if (W == 0) {
      for (int i = 0; i < kIters; ++i) {
        y = fma(y, 0.999, 1e-3);
        asm volatile("" : "+v"(y));
      }
    } else if (W == 1) {
      int idx = l;
      for (int i = 0; i < kIters / 4; ++i) {
        lds[idx] = y;
        y = lds[(idx + 64) % 5120] * 0.5 + 1.0;
        idx = (idx + 128) % 5120;
      }
    } else if (W == 2) {
      for (int i = 0; i < kIters / 2; ++i) {
        const double v = __builtin_amdgcn_update_dpp(y, y, 0x153, 0xf, 0xf, true);
        y = fma(v, 0.999, 1e-3);
      }
    } else {
      double* w = ws + (size_t)b * 64 * 24;
      for (int i = 0; i < kIters / 40; ++i)
        for (int j = 0; j < 24; ++j) w[l * 24 + j] = y + i + j;
    }
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if (l == 0) t[b] = r1 - r0;
  }
  out[b * 64 + l] = y;
}

template <int W>
void run(const char* name, double* out, long long* t, double* ws) {
  for (int tail = 0; tail < 2; ++tail)
    for (int rep = 0; rep < 2; ++rep) {
      kern<W><<<1024, 64>>>(out, t, tail, ws);
      hipDeviceSynchronize();
      long long h[1024];
      hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      int n = 0;
      for (int b = 0; b < 1024; b += 5) { s += h[b]; ++n; }
      printf("%-14s %s rep %d: late waves %.2f us\n", name, tail ? "tail" : "busy", rep, s / n / 100.0);
    }
}

int main() {
  double *out, *ws;
  long long* t;
  hipMalloc(&out, 1024 * 64 * sizeof(double));
  hipMemset(out, 0, 1024 * 64 * sizeof(double));
  hipMalloc(&ws, (size_t)1024 * 64 * 24 * sizeof(double));
  hipMalloc(&t, 1024 * sizeof(long long));
  run<0>("fp64 fma chain", out, t, ws);
  run<1>("lds chain", out, t, ws);
  run<2>("dpp+fma chain", out, t, ws);
  run<3>("row stores", out, t, ws);
  return 0;
}
