// rocBLAS dgemm vs the engine's FP64 GEMM at the Stereo_SIMM sizes (config 5):
//   SF0 = WF0 HF0           (F x NF0) (NF0 x N)
//   num = WF0^T T0          (NF0 x F) (F x N)
// Row-major operands are passed to column-major rocBLAS as the transposed
// product C^T = B^T A^T.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_dgemm.hip -lrocblas -o /tmp/ubench_dgemm
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>

static double time_gemm(rocblas_handle h, rocblas_operation ta, rocblas_operation tb, int m, int n,
                        int k, const double *A, int lda, const double *B, int ldb, double *C,
                        int ldc, int reps) {
  const double one = 1.0, zero = 0.0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i) rocblas_dgemm(h, ta, tb, m, n, k, &one, A, lda, B, ldb, &zero, C, ldc);
  hipEventRecord(e0, nullptr);
  for (int i = 0; i < reps; ++i)
    rocblas_dgemm(h, ta, tb, m, n, k, &one, A, lda, B, ldb, &zero, C, ldc);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const int F = 2049, NF0 = 1092, N = 20000;
  double *WF0, *HF0, *SF0, *T0, *NUM;
  hipMalloc(&WF0, sizeof(double) * F * NF0);
  hipMalloc(&HF0, sizeof(double) * NF0 * N);
  hipMalloc(&SF0, sizeof(double) * F * N);
  hipMalloc(&T0, sizeof(double) * F * N);
  hipMalloc(&NUM, sizeof(double) * NF0 * N);
  // random positive operands (zero operands run at a higher clock: power)
  {
    std::vector<double> h((size_t)F * N);
    unsigned long long x = 88172645463325252ULL;
    for (auto &v : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v = (double)(x >> 11) * (1.0 / 9007199254740992.0) + 0.1;
    }
    hipMemcpy(WF0, h.data(), sizeof(double) * F * NF0, hipMemcpyHostToDevice);
    hipMemcpy(HF0, h.data(), sizeof(double) * NF0 * N, hipMemcpyHostToDevice);
    hipMemcpy(T0, h.data(), sizeof(double) * F * N, hipMemcpyHostToDevice);
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  // SF0 (row-major F x N) = WF0 (F x NF0) HF0 (NF0 x N)
  // column-major: SF0^T (N x F) = HF0^T (N x NF0) WF0^T (NF0 x F)
  double ms1 = time_gemm(h, rocblas_operation_none, rocblas_operation_none, N, F, NF0, HF0, N, WF0,
                         NF0, SF0, N, 10);
  // NUM (row-major NF0 x N) = WF0^T (NF0 x F) T0 (F x N)
  // column-major: NUM^T (N x NF0) = T0^T (N x F) WF0 (F x NF0)  [WF0 col-major is NF0 x F -> transpose]
  double ms2 = time_gemm(h, rocblas_operation_none, rocblas_operation_transpose, N, NF0, F, T0, N, WF0,
                         NF0, NUM, N, 10);
  const double fl = 2.0 * F * NF0 * (double)N;
  printf("rocblas dgemm SF0 = WF0 HF0     : %.3f ms  %.1f TFLOP/s\n", ms1, fl / ms1 / 1e9);
  printf("rocblas dgemm NUM = WF0^T T0    : %.3f ms  %.1f TFLOP/s\n", ms2, fl / ms2 / 1e9);
  rocblas_destroy_handle(h);
  return 0;
}
