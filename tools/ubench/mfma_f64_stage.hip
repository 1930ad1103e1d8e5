// Microbenchmark (diagnostic, not product): does FP64 MFMA pay for the per-instance stage products of the lane
// Riccati kernel (cfg#3, one exo instance per lane)?  BASELINE config #3 names "MFMA on Jacobian-stack GEMM"; the
// products the exo stage forms are small and instance-private (P_xx A_k with 8x8 blocks, a distinct pair per lane),
// so an MFMA tile can only hold them block-diagonally.  Per wave (64 instances), each path forms the 64 products
// C_i = P_i A_i (8x8 * 8x8, 512 FMA each, 32,768 useful FMA per wave) and the wave's own s_memtime brackets it:
//   valu      : lane i multiplies its own P_i, A_i held in registers (the lane kernel's form)
//   mfma      : v_mfma_f64_16x16x4_f64 on block-diagonal pairs diag(P_2t, P_2t+1) * diag(A_2t, A_2t+1), operands
//               already in MFMA fragment layout in LDS (32 tiles x 4 k-steps = 128 MFMA, 25 % of the MACs useful)
//   mfma+relay: the same, plus the relayout the lane kernel would need (each lane writes its P_i, A_i to LDS and
//               reads the products back): what MFMA would actually cost inside sqp_lane_kernel
//   mfma_peak : 4 independent accumulator chains of dense 16x16x4 MFMAs (the unit's own rate)
// Every path's products are compared with a host fp64 reference (integer-valued data: exact).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int NB = 8;            // block size (exo x-rows: nx = 8)
constexpr int M2 = NB * NB;      // doubles per matrix
constexpr int REP = 16;          // repetitions inside the timed region (amortise s_memtime)

// zero-instruction register barrier on 16 doubles: the repetitions cannot be hoisted out of the timed loop
#define PIN16(x, o)                                                                                               \
  asm volatile("" : "+v"(x[o + 0]), "+v"(x[o + 1]), "+v"(x[o + 2]), "+v"(x[o + 3]), "+v"(x[o + 4]), "+v"(x[o + 5]), \
               "+v"(x[o + 6]), "+v"(x[o + 7]), "+v"(x[o + 8]), "+v"(x[o + 9]), "+v"(x[o + 10]), "+v"(x[o + 11]),   \
               "+v"(x[o + 12]), "+v"(x[o + 13]), "+v"(x[o + 14]), "+v"(x[o + 15]))
#define PIN64(x) do { PIN16(x, 0); PIN16(x, 16); PIN16(x, 32); PIN16(x, 48); } while (0)

__device__ __forceinline__ double pval(int inst, int i, int j) { return (double)(((inst * 7 + i * 3 + j * 5) % 9) - 4); }
__device__ __forceinline__ double aval(int inst, int i, int j) { return (double)(((inst * 5 + i * 11 + j * 2) % 7) - 3); }

// C_i = P_i A_i per lane: A_i in registers, P_i in LDS lane-interleaved [element][lane] (the lane kernel keeps P~
// in LDS the same way), C_i accumulated in registers
__global__ __launch_bounds__(64) void k_valu(double* out, long long* cyc) {
  extern __shared__ double lds[];
  const int l = threadIdx.x, inst = blockIdx.x * 64 + l;
  double A[M2], C[M2];
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      lds[(i * NB + j) * 64 + l] = pval(inst, i, j);
      A[i * NB + j] = aval(inst, i, j);
    }
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REP; ++r) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double p[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) p[k] = lds[(i * NB + k) * 64 + l];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NB; ++k) t = fma(p[k], A[k * NB + j], t);
        C[i * NB + j] = t;
      }
    }
    PIN64(A);
    PIN64(C);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  for (int e = 0; e < M2; ++e) out[(size_t)inst * M2 + e] = C[e];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// tile t of a wave: instances 2t, 2t+1 block-diagonally; 4 k-steps of 16x16x4.  A fragment (lane l): row l&15,
// k = 4s + (l>>4); B fragment: k = 4s + (l>>4), col l&15; C/D: col l&15, row (l>>4) + 4 reg.
__device__ __forceinline__ d4 tile_product(const double* sA, const double* sB, int t, int l) {
  d4 c = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const double a = sA[(t * 4 + s) * 64 + l];
    const double b = sB[(t * 4 + s) * 64 + l];
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  return c;
}

// fragment image of the block-diagonal operands of every tile: [tile][k-step][lane] (what an MFMA kernel would
// keep resident), built outside the timed region
__device__ void build_fragments(double* sA, double* sB, int wave) {
  const int l = threadIdx.x;
  for (int t = 0; t < 32; ++t)
    for (int s = 0; s < 4; ++s) {
      const int i = l & 15, k = 4 * s + (l >> 4), j = l & 15;
      const int ia = 2 * t + (i >> 3), ib = 2 * t + (j >> 3);
      const bool da = (i >> 3) == (k >> 3), db = (k >> 3) == (j >> 3);
      sA[(t * 4 + s) * 64 + l] = da ? pval(wave * 64 + ia, i & 7, k & 7) : 0.0;
      sB[(t * 4 + s) * 64 + l] = db ? aval(wave * 64 + ib, k & 7, j & 7) : 0.0;
    }
}

__global__ __launch_bounds__(64) void k_mfma(double* out, long long* cyc) {
  extern __shared__ double lds[];
  double* sA = lds;
  double* sB = lds + 32 * 4 * 64;
  const int l = threadIdx.x;
  build_fragments(sA, sB, blockIdx.x);
  __syncthreads();
  d4 acc[32];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REP; ++r) {
    asm volatile("" ::: "memory");  // operands re-read from LDS every repetition
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[t] = tile_product(sA, sB, t, l);
#pragma unroll
    for (int t = 0; t < 32; ++t) asm volatile("" : "+v"(acc[t]));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  // scatter the diagonal blocks back to [instance][8x8]
#pragma unroll
  for (int t = 0; t < 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = (l >> 4) + 4 * g, col = l & 15;
      if ((row >> 3) == (col >> 3)) {
        const int inst = blockIdx.x * 64 + 2 * t + (row >> 3);
        out[(size_t)inst * M2 + (row & 7) * NB + (col & 7)] = acc[t][g];
      }
    }
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// as k_mfma, with the relayout inside the timed region, starting from the lane kernel's layout (P_i lane-interleaved
// in LDS, A_i in lane i's registers): A_i -> LDS, block-diagonal fragments gathered from the two LDS images (an
// off-diagonal entry reads a zero slot), MFMA, the diagonal blocks scattered to LDS and read back by their lanes
__global__ __launch_bounds__(64) void k_mfma_relay(double* out, long long* cyc) {
  extern __shared__ double lds[];
  double* sP = lds;                 // [64 elements][64 lanes]
  double* sAm = lds + 64 * M2;      // [64][64]
  double* sC = sAm + 64 * M2;       // [64][64]
  double* sZ = sC + 64 * M2;        // one zero
  const int l = threadIdx.x, inst = blockIdx.x * 64 + l;
  double A[M2], C[M2];
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      sP[(i * NB + j) * 64 + l] = pval(inst, i, j);
      A[i * NB + j] = aval(inst, i, j);
    }
  if (l == 0) sZ[0] = 0.0;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REP; ++r) {
#pragma unroll
    for (int e = 0; e < M2; ++e) sAm[e * 64 + l] = A[e];
    __syncthreads();
    int lv = l;
    asm volatile("" : "+v"(lv));   // fragment addresses formed per repetition (not 256 hoisted VGPRs)
    const int i = lv & 15, kq = lv >> 4, j = lv & 15;
    const int zP = (int)(sZ - sP), zA = (int)(sZ - sAm), zC = (int)(sZ + 1 - sC);
    // per k-step / result register: base offset and tile stride (2 instances per tile; stride 0 = the zero or junk
    // slot for entries off the diagonal blocks) -- the block-diagonal pattern does not depend on the tile
    int ba[4], sa[4], bb[4], sb[4], bc[4], sc[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int k = 4 * s2 + kq;
      const bool da = (i >> 3) == (k >> 3), db = (k >> 3) == (j >> 3);
      ba[s2] = da ? ((i & 7) * NB + (k & 7)) * 64 + (i >> 3) : zP;
      sa[s2] = da ? 2 : 0;
      bb[s2] = db ? ((k & 7) * NB + (j & 7)) * 64 + (j >> 3) : zA;
      sb[s2] = db ? 2 : 0;
      const int row = kq + 4 * s2, col = j;
      const bool dc = (row >> 3) == (col >> 3);
      bc[s2] = dc ? ((row & 7) * NB + (col & 7)) * 64 + (row >> 3) : zC;
      sc[s2] = dc ? 2 : 0;
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) {
      d4 c = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(sP[ba[s2] + sa[s2] * t], sAm[bb[s2] + sb[s2] * t], c, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) sC[bc[g] + sc[g] * t] = c[g];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < M2; ++e) C[e] = sC[e * 64 + l];
    PIN64(A);
    PIN64(C);
    __syncthreads();
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  for (int e = 0; e < M2; ++e) out[(size_t)inst * M2 + e] = C[e];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// dense MFMA rate: 4 independent accumulator chains
__global__ __launch_bounds__(64) void k_mfma_peak(double* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

static double host_ref(int inst, int i, int j) {
  double t = 0.0;
  for (int k = 0; k < NB; ++k) {
    const double p = (double)(((inst * 7 + i * 3 + k * 5) % 9) - 4), a = (double)(((inst * 5 + k * 11 + j * 2) % 7) - 3);
    t += p * a;
  }
  return t;
}

static double mean(const std::vector<long long>& v) {
  double s = 0;
  for (auto x : v) s += (double)x;
  return s / v.size();
}

int main() {
  // 1024 waves = 1 per SIMD for the register-only kernels; the LDS kernels use 64 KB / 96 KB per wave, so fewer
  // are resident at once -- every rate below is per WAVE (its own s_memtime), not per device
  const int W = 1024;
  double* d_out;
  long long* d_cyc;
  (void)hipMalloc(&d_out, (size_t)W * 64 * M2 * sizeof(double));
  (void)hipMalloc(&d_cyc, W * sizeof(long long));
  std::vector<double> h((size_t)W * 64 * M2);
  std::vector<long long> cyc(W);
  auto check = [&](const char* name) {
    (void)hipMemcpy(h.data(), d_out, h.size() * sizeof(double), hipMemcpyDeviceToHost);
    long bad = 0;
    for (int inst = 0; inst < W * 64; inst += 97)
      for (int i = 0; i < NB; ++i)
        for (int j = 0; j < NB; ++j) bad += h[(size_t)inst * M2 + i * NB + j] != host_ref(inst, i, j);
    printf("  %s: products %s\n", name, bad ? "WRONG" : "exact");
    return bad == 0;
  };
  const double useful = 64.0 * NB * NB * NB * REP;   // useful FMA per wave in the timed region
  bool ok = true;
  const size_t lds0 = M2 * 64 * sizeof(double);
  hipLaunchKernelGGL(k_valu, dim3(W), dim3(64), lds0, 0, d_out, d_cyc);
  hipLaunchKernelGGL(k_valu, dim3(W), dim3(64), lds0, 0, d_out, d_cyc);
  hipDeviceSynchronize();
  (void)hipMemcpy(cyc.data(), d_cyc, W * 8, hipMemcpyDeviceToHost);
  const double cv = mean(cyc);
  printf("valu       : %8.0f cycles/wave for 64 products x %d -> %6.2f useful FMA/cycle/wave\n", cv, REP, useful / cv);
  ok &= check("valu");
  const size_t lds1 = 2 * 32 * 4 * 64 * sizeof(double);
  hipFuncSetAttribute((const void*)k_mfma, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
  hipLaunchKernelGGL(k_mfma, dim3(W), dim3(64), lds1, 0, d_out, d_cyc);
  hipLaunchKernelGGL(k_mfma, dim3(W), dim3(64), lds1, 0, d_out, d_cyc);
  hipDeviceSynchronize();
  (void)hipMemcpy(cyc.data(), d_cyc, W * 8, hipMemcpyDeviceToHost);
  const double cm = mean(cyc);
  printf("mfma       : %8.0f cycles/wave (128 MFMA x %d, operands resident) -> %6.2f useful FMA/cycle/wave "
         "(%.1f cycles per MFMA)\n", cm, REP, useful / cm, cm / (128.0 * REP));
  ok &= check("mfma");
  const size_t lds2 = (3 * 64 * M2 + 2) * sizeof(double);
  hipFuncSetAttribute((const void*)k_mfma_relay, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
  hipLaunchKernelGGL(k_mfma_relay, dim3(W), dim3(64), lds2, 0, d_out, d_cyc);
  hipLaunchKernelGGL(k_mfma_relay, dim3(W), dim3(64), lds2, 0, d_out, d_cyc);
  hipDeviceSynchronize();
  (void)hipMemcpy(cyc.data(), d_cyc, W * 8, hipMemcpyDeviceToHost);
  const double cr = mean(cyc);
  printf("mfma+relay : %8.0f cycles/wave (lane layout -> LDS -> MFMA -> lanes) -> %6.2f useful FMA/cycle/wave\n", cr,
         useful / cr);
  ok &= check("mfma+relay");
  const int it = 4096;
  hipLaunchKernelGGL(k_mfma_peak, dim3(W), dim3(64), 0, 0, d_out, d_cyc, it);
  hipLaunchKernelGGL(k_mfma_peak, dim3(W), dim3(64), 0, 0, d_out, d_cyc, it);
  hipDeviceSynchronize();
  (void)hipMemcpy(cyc.data(), d_cyc, W * 8, hipMemcpyDeviceToHost);
  const double cp = mean(cyc);
  printf("mfma_peak  : %.1f cycles per dense v_mfma_f64_16x16x4 (1 wave/SIMD) = %.1f FMA/cycle/wave\n",
         cp / (4.0 * it), 1024.0 * 4 * it / cp);
  return ok ? 0 : 1;
}
