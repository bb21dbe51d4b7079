// k_gemm44 (v_mfma_f64_4x4x4_4b) vs k_gemm (16x16x4) vs rocBLAS dgemm at the
// Stereo_SIMM sizes (config 5), with a max-relative check against rocBLAS.
//   SF0 = WF0 HF0      (F x NF0)(NF0 x N)   NN
//   NUM = WF0^T T0     (NF0 x F)(F x N)     TN
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_gemm44.hip -lrocblas -o /tmp/ubench_gemm44
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../pyfasst_amd/csrc/fasst_gemm.h"

using namespace fasst;

template <class L>
static double time_it(L &&launch, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i) launch();
  hipEventRecord(e0, nullptr);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

static double maxrel(const double *a, const double *b, size_t n) {
  std::vector<double> ha(n), hb(n);
  hipMemcpy(ha.data(), a, n * sizeof(double), hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), b, n * sizeof(double), hipMemcpyDeviceToHost);
  double mx = 0, ref = 0;
  for (size_t i = 0; i < n; ++i) {
    mx = std::fmax(mx, std::fabs(ha[i] - hb[i]));
    ref = std::fmax(ref, std::fabs(hb[i]));
  }
  return mx / ref;
}

template <bool TA, int NW, int WGM, int RM, int RN>
static void run44(const char *tag, const double *A, int lda, const double *B, double *C, int M, int N,
                  int K, const double *Cref, double fl) {
  GemmArgs g{};
  g.A = A;
  g.B[0] = B;
  g.C[0] = C;
  g.lda = lda;
  g.ldb = N;
  g.ldc = N;
  g.M = M;
  g.N = N;
  g.K = K;
  g.kchunk = (K + kGBK - 1) / kGBK * kGBK;
  g.slab = 0;
  constexpr int WGN = NW / WGM, BM = 16 * RM * WGM, BN = 4 * RN * WGN;
  constexpr size_t lds = gemm44_smem<TA, false, 1, NW, WGM, RM, RN>();
  auto kern = k_gemm44<TA, false, 1, NW, WGM, RM, RN>;
  hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, 1);
  hipMemset(C, 0, sizeof(double) * M * N);
  double ms = time_it([&] { kern<<<grid, 64 * NW, lds>>>(g); }, 10);
  printf("k_gemm44<%s NW=%d WGM=%d RM=%d RN=%d BM=%d BN=%d lds=%zu> %-4s: %.3f ms  %.1f TFLOP/s  maxrel %.2e\n",
         TA ? "T" : "N", NW, WGM, RM, RN, BM, BN, lds, tag, ms, fl / ms / 1e9,
         maxrel(C, Cref, (size_t)M * N));
}

int main() {
  const int F = 2049, NF0 = 1092, N = 20000;
  double *WF0, *HF0, *SF0, *T0, *NUM, *C;
  hipMalloc(&WF0, sizeof(double) * F * NF0);
  hipMalloc(&HF0, sizeof(double) * NF0 * N);
  hipMalloc(&SF0, sizeof(double) * F * N);
  hipMalloc(&T0, sizeof(double) * F * N);
  hipMalloc(&NUM, sizeof(double) * NF0 * N);
  hipMalloc(&C, sizeof(double) * F * N);
  {
    std::vector<double> h((size_t)F * N);
    unsigned long long x = 88172645463325252ULL;
    for (auto &v : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v = (double)(x >> 11) * (1.0 / 9007199254740992.0) + 0.1;
    }
    hipMemcpy(WF0, h.data(), sizeof(double) * F * NF0, hipMemcpyHostToDevice);
    hipMemcpy(HF0, h.data() + 7, sizeof(double) * NF0 * N, hipMemcpyHostToDevice);
    hipMemcpy(T0, h.data() + 13, sizeof(double) * F * N, hipMemcpyHostToDevice);
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  const double one = 1.0, zero = 0.0;
  const double fl = 2.0 * F * NF0 * (double)N;
  // clock warm-up (~0.5 s) before anything is timed
  for (int w = 0; w < 300; ++w)
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, N, F, NF0, &one, HF0, N, WF0,
                  NF0, &zero, SF0, N);
  hipDeviceSynchronize();
  double ms1 = time_it([&] { rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, N, F, NF0,
                                           &one, HF0, N, WF0, NF0, &zero, SF0, N); }, 10);
  double ms2 = time_it([&] { rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, N, NF0,
                                           F, &one, T0, N, WF0, NF0, &zero, NUM, N); }, 10);
  printf("rocblas dgemm NN SF0 = WF0 HF0 : %.3f ms  %.1f TFLOP/s\n", ms1, fl / ms1 / 1e9);
  printf("rocblas dgemm TN NUM = WF0^T T0: %.3f ms  %.1f TFLOP/s\n", ms2, fl / ms2 / 1e9);
  run44<false, 8, 2, 8, 8>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0, fl);
  run44<false, 4, 2, 4, 16>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0, fl);
  run44<false, 4, 2, 8, 8>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0, fl);
  run44<false, 4, 1, 8, 16>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0, fl);
  run44<false, 4, 4, 4, 8>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0, fl);
  run44<true, 8, 2, 8, 8>("TN", WF0, NF0, T0, C, NF0, N, F, NUM, fl);
  run44<true, 4, 2, 4, 16>("TN", WF0, NF0, T0, C, NF0, N, F, NUM, fl);
  run44<true, 4, 2, 8, 8>("TN", WF0, NF0, T0, C, NF0, N, F, NUM, fl);
  rocblas_destroy_handle(h);
  return 0;
}
