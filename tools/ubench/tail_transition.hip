// Microbenchmark (diagnostic, not product): does a wave stall when the other workgroups of its CU terminate?
// 1024 one-wave blocks with 40 KB of LDS each (four per CU, as the 16-lane group kernel at cfg#2).  "Late" blocks
// (b % 4 == 0: one per CU if the dispatcher places four consecutive blocks on one CU, else spread) run 256 chunks of
// 512 dependent FP64 FMAs and stamp s_memrealtime after each; the other blocks run the same chain for 1/2 of that
// (transition: they terminate in the middle of the late blocks' series) or 2x (busy: they outlive it).  Prints, over
// the late blocks, the median chunk time and the largest chunk time (a stall at the others' termination would show
// as one long chunk), and the same with the others' LDS footprint 0 (lds=0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kChunks = 256, kPer = 512;

template <int LDS>
__global__ __launch_bounds__(64) void kern(double* out, long long* ts, int others_chunks) {
  __shared__ double lds[LDS ? 5120 : 1];
  const int b = blockIdx.x, l = threadIdx.x;
  const bool late = (b & 3) == 0;
  double y = out[b * 64 + l] + 1.0;
  if (LDS) {
    for (int i = l; i < 5120; i += 64) lds[i] = i;
    __syncthreads();
    y += lds[(l * 7) % 5120];
  }
  const int chunks = late ? kChunks : others_chunks;
  for (int c = 0; c < chunks; ++c) {
    for (int i = 0; i < kPer; ++i) {
      y = fma(y, 0.999, 1e-3);
      asm volatile("" : "+v"(y));
    }
    if (late && l == 0) ts[(size_t)(b >> 2) * kChunks + c] = __builtin_amdgcn_s_memrealtime();
  }
  out[b * 64 + l] = y;
}

template <int LDS>
void run(double* out, long long* ts) {
  for (int mode = 0; mode < 2; ++mode) {
    const int oc = mode ? kChunks / 2 : 2 * kChunks;
    kern<LDS><<<1024, 64>>>(out, ts, oc);
    hipDeviceSynchronize();
    std::vector<long long> h(256 * kChunks);
    hipMemcpy(h.data(), ts, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    std::vector<double> d;
    double worst = 0;
    int worst_c = -1;
    for (int w = 0; w < 256; ++w)
      for (int c = 1; c < kChunks; ++c) {
        const double v = (h[w * kChunks + c] - h[w * kChunks + c - 1]) / 100.0;
        d.push_back(v);
        if (v > worst) { worst = v; worst_c = c; }
      }
    std::sort(d.begin(), d.end());
    printf("lds=%d %-10s: chunk median %.2f us, p99 %.2f us, max %.2f us (at chunk %d of %d)\n", LDS,
           mode ? "transition" : "busy", d[d.size() / 2], d[d.size() * 99 / 100], worst, worst_c, kChunks);
  }
}

int main() {
  double* out;
  long long* ts;
  hipMalloc(&out, 1024 * 64 * sizeof(double));
  hipMemset(out, 0, 1024 * 64 * sizeof(double));
  hipMalloc(&ts, 256 * kChunks * sizeof(long long));
  for (int rep = 0; rep < 2; ++rep) {
    run<1>(out, ts);
    run<0>(out, ts);
  }
  return 0;
}
