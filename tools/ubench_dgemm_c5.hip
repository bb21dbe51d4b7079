// k_dgemm2 (product shape D2Prod, raw-buffer LDS-DMA pieces) at the two
// Stereo_SIMM NF0-sized products of config 5, against the same products with
// the M edge trimmed to whole 128-row tiles -- how much the ragged last
// m-tile (2049 = 16 x 128 + 1, 1092 = 8 x 128 + 68) costs.
//   SF0 = WF0 HF0             M = F = 2049,  N = 20000, K = NF0 = 1092
//   NPD = WF0^T [T0 | T1]     M = NF0 = 1092, N = 40000, K = F = 2049
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=true \
//        tools/ubench_dgemm_c5.hip -o tools/ubench_dgemm_c5
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../pyfasst_amd/csrc/fasst_dgemm2.h"

using namespace fasst;

template <class L>
static double time_it(L &&launch, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) launch();
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

static void fill(double *d, size_t n, unsigned long long seed) {
  std::vector<double> h(n);
  unsigned long long x = seed * 0x9E3779B97F4A7C15ULL + 88172645463325252ULL;
  for (auto &v : h) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    v = (double)(x >> 11) * (1.0 / 9007199254740992.0) + 0.1;
  }
  (void)hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
}

static double run(const char *tag, const double *A, int lda, const double *B, int ldb, double *C, int ldc,
                  int M, int N, int K, int reps = 20, int order = 0) {
  using CF = D2Prod;
  Dgemm2Args g{};
  g.A = A;
  g.B = B;
  g.C = C;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.mt = (M + CF::BM - 1) / CF::BM;
  g.nt = (N + CF::BN - 1) / CF::BN;
  (void)order;
  (void)hipFuncSetAttribute((const void *)k_dgemm2<CF, false, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)CF::smem);
  const double fl = 2.0 * M * (double)N * K;
  const double ms =
      time_it([&] { k_dgemm2<CF, false, false, true><<<g.mt * g.nt, CF::NT, CF::smem>>>(g); }, reps);
  printf("o%d %-10s M=%5d N=%5d K=%5d tiles %3d x %3d: %.3f ms  %.1f TFLOP/s\n", order, tag, M, N, K, g.mt, g.nt, ms,
         fl / ms / 1e9);
  return ms;
}

int main() {
  const int F = 2049, FP = 2064, NF0 = 1092, NF0P = 1104, N = 20000, N2 = 40000;
  double *WF0T, *HF0, *WF0K, *T0, *C;
  (void)hipMalloc(&WF0T, sizeof(double) * NF0 * FP);   // [NF0][FP]  (k-major A of SF0)
  (void)hipMalloc(&HF0, sizeof(double) * NF0 * N);     // [NF0][N]
  (void)hipMalloc(&WF0K, sizeof(double) * F * NF0P);   // [F][NF0P] (k-major A of NPD)
  (void)hipMalloc(&T0, sizeof(double) * F * N2);       // [F][2N]
  (void)hipMalloc(&C, sizeof(double) * F * N2);
  fill(WF0T, (size_t)NF0 * FP, 1);
  fill(HF0, (size_t)NF0 * N, 2);
  fill(WF0K, (size_t)F * NF0P, 3);
  fill(T0, (size_t)F * N2, 4);
  // clock warm-up
  for (int w = 0; w < 20; ++w) run("warm", WF0T, FP, HF0, N, C, N, F, N, NF0, 1);
  for (int r = 0; r < 2; ++r) {
    for (int o = 0; o < 4; ++o) {
      run("SF0", WF0T, FP, HF0, N, C, N, F, N, NF0, 20, o);
      run("NPD", WF0K, NF0P, T0, N2, C, N2, NF0, N2, F, 20, o);
    }
    run("SF0 M-1", WF0T, FP, HF0, N, C, N, F - 1, N, NF0);
    run("NPD M=1024", WF0K, NF0P, T0, N2, C, N2, 1024, N2, F);
  }
  return 0;
}
