// k_dgemm (fasst_dgemm.h) vs rocBLAS dgemm at the Stereo_SIMM product shapes
// (config 5), with a max-relative check against rocBLAS:
//   SF0 = WF0 HF0             (F x NF0)(NF0 x N)    NN
//   [NUM|DEN] = WF0^T [T0|T1] (NF0 x F)(F x 2N)     TN
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=true \
//        tools/ubench_dgemm2.hip -lrocblas -o tools/ubench_dgemm2
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../pyfasst_amd/csrc/fasst_dgemm.h"

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

template <bool TA, int IG = 0, int SM = 0>
static void run(const char *tag, const double *A, int lda, const double *B, double *C, int M, int N,
                int K, const double *Cref, int order = 0) {
  DgemmArgs g{};
  g.A = A;
  g.B = B;
  g.C = C;
  g.lda = lda;
  g.ldb = N;
  g.ldc = N;
  g.M = M;
  g.N = N;
  g.K = K;
  g.mt = (M + kDBM - 1) / kDBM;
  g.nt = (N + kDBN - 1) / kDBN;
  g.order = order;
  constexpr size_t lds = dgemm_smem<TA>();
  hipFuncSetAttribute((const void *)k_dgemm<TA, IG, SM>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int nb = ((g.mt * g.nt + 7) / 8) * 8;
  hipMemset(C, 0, sizeof(double) * M * N);
  const double fl = 2.0 * M * (double)N * K;
  double ms = time_it([&] { k_dgemm<TA, IG, SM><<<nb, 256, lds>>>(g); }, 10);
  printf("k_dgemm<%s,ig%d,sm%d> %-3s order %d M=%d N=%d K=%d lds=%zu: %.3f ms  %.1f TFLOP/s  maxrel %.2e\n",
         TA ? "T" : "N", IG, SM, tag, order, M, N, K, lds, ms, fl / ms / 1e9, maxrel(C, Cref, (size_t)M * N));
}

int main() {
  const int F = 2049, NF0 = 1092, N = 20000, N2 = 40000;
  double *WF0, *HF0, *SF0, *T0, *NUM, *C;
  hipMalloc(&WF0, sizeof(double) * F * NF0);
  hipMalloc(&HF0, sizeof(double) * NF0 * N);
  hipMalloc(&SF0, sizeof(double) * F * N);
  hipMalloc(&T0, sizeof(double) * F * N2);
  hipMalloc(&NUM, sizeof(double) * NF0 * N2);
  hipMalloc(&C, sizeof(double) * F * N2);
  {
    std::vector<double> h((size_t)F * N2);
    unsigned long long x = 88172645463325252ULL;
    for (auto &v : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v = (double)(x >> 11) * (1.0 / 9007199254740992.0) + 0.1;
    }
    hipMemcpy(WF0, h.data(), sizeof(double) * F * NF0, hipMemcpyHostToDevice);
    hipMemcpy(HF0, h.data() + 7, sizeof(double) * NF0 * N, hipMemcpyHostToDevice);
    hipMemcpy(T0, h.data() + 13, sizeof(double) * F * N2, hipMemcpyHostToDevice);
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  const double one = 1.0, zero = 0.0;
  for (int w = 0; w < 300; ++w)   // clock warm-up (~0.5 s)
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, N, F, NF0, &one, HF0, N, WF0,
                  NF0, &zero, SF0, N);
  hipDeviceSynchronize();
  double ms1 = time_it([&] { rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, N, F, NF0,
                                           &one, HF0, N, WF0, NF0, &zero, SF0, N); }, 10);
  double ms2 = time_it([&] { rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, N2, NF0,
                                           F, &one, T0, N2, WF0, NF0, &zero, NUM, N2); }, 10);
  printf("rocblas NN SF0 = WF0 HF0       M=%d N=%d K=%d: %.3f ms  %.1f TFLOP/s\n", F, N, NF0, ms1,
         2.0 * F * NF0 * (double)N / ms1 / 1e9);
  printf("rocblas TN [NUM|DEN] = WF0^T T M=%d N=%d K=%d: %.3f ms  %.1f TFLOP/s\n", NF0, N2, F, ms2,
         2.0 * F * NF0 * (double)N2 / ms2 / 1e9);
  for (int r = 0; r < 2; ++r) {   // interleaved A/B: default, store mid-chunk
    run<false>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0);
    run<false, 0, 1>("NN", WF0, NF0, HF0, C, F, N, NF0, SF0);
    run<true>("TN", WF0, NF0, T0, C, NF0, N2, F, NUM);
    run<true, 0, 1>("TN", WF0, NF0, T0, C, NF0, N2, F, NUM);
  }
  rocblas_destroy_handle(h);
  return 0;
}
