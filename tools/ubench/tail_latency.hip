// Microbenchmark (diagnostic, not product): latency of a dependent global load for a wave that runs while the rest
// of the chip computes, against the same wave once the other waves have left (the tail of a kernel, where the 16-lane
// group kernel's last iterations ran 6x slower at tol 1e-5: DESIGN.md 4c, profiles/r06/s3).  1024 one-wave blocks
// (one per SIMD); blocks 0..7 chase pointers through their own 1 MB (one 64-byte line per step, random cyclic order:
// L2 hits after a warm pass) while
//   busy : every other block spins FP64 FMAs for 4x the chasers' spin, i.e. throughout the chase;
//   tail : every other block spins 1/4 of the chasers' spin and leaves before the chase;
//   lone : a grid of the 8 chasers alone.
// Prints ns per dependent load (s_memrealtime, 100 MHz) and the chasers' shader clock over the chase.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

constexpr int kLines = 16384;       // 1 MB per chaser in 64-byte lines
constexpr long long kBigLines = 1 << 20;   // hbm mode: 64 MB per chaser (8 chasers: 512 MB, beyond L2 and MALL)
constexpr int kSteps = 4096;        // timed dependent loads

__global__ __launch_bounds__(64) void kern(const int* chain, double* sink, long long* out, int spin_chaser,
                                           int spin_other, int cold, int* scratch, int with_store, const int* big,
                                           int hbm, int start) {
  const int b = blockIdx.x, t = threadIdx.x;
  const bool chaser = b < 8;
  double y = sink[b * 64 + t] + 1.0;
  const int spin = chaser ? spin_chaser : spin_other;
  if (!chaser && spin < 0) {   // memory-busy then leave: -spin rounds of 16 KB stores per wave (the solver's traffic)
    double* st = sink + 1024 * 64 + (size_t)b * 2048;
    for (int r = 0; r < -spin; ++r)
      for (int i = 0; i < 32; ++i) st[i * 64 + t] = y + r;
  } else {
    for (int i = 0; i < spin; ++i) {
      y = fma(y, 0.999, 1e-3);
      asm volatile("" : "+v"(y));
    }
  }
  if (chaser && t == 0) {
    const int* c = chain + (size_t)b * kLines * 16;
    int idx = 0;
    if (!cold)
      for (int i = 0; i < kLines; ++i) idx = c[idx * 16];   // warm: every line into L2
    const long long r0 = __builtin_amdgcn_s_memrealtime(), m0 = __builtin_amdgcn_s_memtime();
    int* sc = scratch + (size_t)b * kSteps * 16;
    if (hbm) {   // dependent loads at random lines of 64 MB: L2 / MALL misses
      const int* g = big + (size_t)b * kBigLines * 16;
      long long j = start;   // a segment of the cycle no earlier launch walked (cold lines)
      for (int i = 0; i < kSteps; ++i) j = g[j * 16];
      idx = (int)j;
    } else if (with_store) {   // a store before every dependent load (gfx9: stores and loads share vmcnt)
      for (int i = 0; i < kSteps; ++i) {
        sc[i * 16] = idx;
        idx = c[idx * 16];
      }
    } else {
      for (int i = 0; i < kSteps; ++i) idx = c[idx * 16];
    }
    const long long r1 = __builtin_amdgcn_s_memrealtime(), m1 = __builtin_amdgcn_s_memtime();
    out[b * 3 + 0] = r1 - r0;
    out[b * 3 + 1] = m1 - m0;
    out[b * 3 + 2] = idx;
  }
  sink[b * 64 + t] = y;
}

int main() {
  std::vector<int> h((size_t)8 * kLines * 16, 0);
  std::mt19937 rng(7);
  for (int w = 0; w < 8; ++w) {   // random cyclic permutation of the lines
    std::vector<int> p(kLines);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin() + 1, p.end(), rng);
    for (int i = 0; i < kLines; ++i) h[(size_t)w * kLines * 16 + (size_t)p[i] * 16] = p[(i + 1) % kLines];
  }
  int* d;
  double* sink;
  long long* out;
  hipMalloc(&d, h.size() * sizeof(int));
  hipMalloc(&sink, (1024 * 64 + 1024 * 2048) * sizeof(double));
  hipMemset(sink, 0, (1024 * 64 + 1024 * 2048) * sizeof(double));
  hipMalloc(&out, 8 * 3 * sizeof(long long));
  // hbm mode: a random cyclic permutation of 2^20 lines per chaser (8 x 64 MB)
  std::vector<int> hb((size_t)8 * kBigLines * 16, 0);
  for (int w = 0; w < 8; ++w) {
    std::vector<int> p(kBigLines);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin() + 1, p.end(), rng);
    for (long long i = 0; i < kBigLines; ++i) hb[(size_t)w * kBigLines * 16 + (size_t)p[i] * 16] = p[(i + 1) % kBigLines];
  }
  int* big;
  hipMalloc(&big, hb.size() * sizeof(int));
  hipMemcpy(big, hb.data(), hb.size() * sizeof(int), hipMemcpyHostToDevice);
  int* scratch;
  hipMalloc(&scratch, (size_t)8 * kSteps * 16 * sizeof(int));
  hipMemcpy(d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice);
  hipMemset(sink, 0, 1024 * 64 * sizeof(double));
  const int S = 200000;   // ~0.4 ms of FMAs at 1 wave / SIMD
  struct Mode { const char* name; int grid, spin_chaser, spin_other; };
  const Mode modes[] = {{"busy", 1024, S, 4 * S}, {"tail", 1024, S, S / 4}, {"lone", 8, S, 0},
                        {"tailmem", 1024, S, -400}, {"busymem", 1024, S, -8000}};
  for (int ws = 0; ws < 3; ++ws)   // 0: loads, 1: store + load, 2: HBM loads
  for (int cold = 0; cold < (ws == 2 ? 1 : 2); ++cold) {
    for (const Mode& m : modes) {
      for (int rep = 0; rep < 3; ++rep) {
        static int launch = 0;
        ++launch;
        kern<<<m.grid, 64>>>(d, sink, out, m.spin_chaser, m.spin_other, cold || ws == 2, scratch, ws == 1, big,
                             ws == 2, launch * 4099);
        hipDeviceSynchronize();
        long long o[24];
        hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
        double ns = 0, ghz = 0;
        for (int w = 0; w < 8; ++w) {
          ns += o[w * 3] * 10.0 / kSteps / 8;
          ghz += (double)o[w * 3 + 1] / (o[w * 3] * 10.0) / 8;
        }
        printf("%s %s %-5s rep %d: %7.1f ns per dependent load, clock %.2f GHz\n", ws == 2 ? "hbm-load  " : ws ? "store+load" : "load      ",
               cold ? "no-warm" : "warm   ", m.name, rep, ns, ghz);
      }
    }
  }
  return 0;
}
