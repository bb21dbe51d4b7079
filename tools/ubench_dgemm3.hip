// k_dgemm2 (fasst_dgemm2.h: global_load_lds stages, 4x4x4_4b MFMA) vs the
// round-2 k_dgemm and rocBLAS dgemm at the Stereo_SIMM product shapes
// (config 5), max-relative check against rocBLAS, random operands:
//   SF0 = WF0 HF0             (F x NF0)(NF0 x N)   A = WF0^T kept k-major
//   [NUM|DEN] = WF0^T [T0|T1] (NF0 x F)(F x 2N)    A = WF0 (k-major as stored)
// plus edge shapes (odd N, odd M, K not a multiple of 16).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=true \
//        tools/ubench_dgemm3.hip -lrocblas -o tools/ubench_dgemm3
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../pyfasst_amd/csrc/fasst_dgemm.h"
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

static double maxrel(const double *a, const double *b, int M, int N, int ldc) {
  std::vector<double> ha((size_t)M * ldc), hb((size_t)M * ldc);
  (void)hipMemcpy(ha.data(), a, ha.size() * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipMemcpy(hb.data(), b, hb.size() * sizeof(double), hipMemcpyDeviceToHost);
  double mx = 0, ref = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      const size_t i = (size_t)m * ldc + n;
      mx = std::fmax(mx, std::fabs(ha[i] - hb[i]));
      ref = std::fmax(ref, std::fabs(hb[i]));
    }
  return mx / ref;
}

// C = A^T B with A [K][lda], B [K][ldb], C [M][ldc] (row-major) on rocBLAS
static void blas_ta(rocblas_handle h, const double *A, int lda, const double *B, int ldb, double *C,
                    int ldc, int M, int N, int K) {
  const double one = 1.0, zero = 0.0;
  rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, N, M, K, &one, B, ldb, A, lda,
                &zero, C, ldc);
}

template <class CF, bool A4 = false, bool B4 = false>
static double run2(const char *tag, const double *A, int lda, const double *B, int ldb, double *C,
                   int ldc, int M, int N, int K, const double *Cref, int reps = 10) {
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
  (void)hipFuncSetAttribute((const void *)k_dgemm2<CF, A4, B4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)CF::smem);
  (void)hipMemset(C, 0, sizeof(double) * M * ldc);
  const double fl = 2.0 * M * (double)N * K;
  const double ms = time_it([&] { k_dgemm2<CF, A4, B4><<<g.mt * g.nt, CF::NT, CF::smem>>>(g); }, reps);
  printf("k_dgemm2<NS=%d,BK=%d,%dx%d,occ%d,mf%d,A4=%d,B4=%d> %-7s M=%d N=%d K=%d lda=%d ldb=%d: %.3f ms  %.1f TFLOP/s  maxrel %.2e\n",
         CF::NS, CF::BK, CF::WGM, CF::WGN, CF::OCC, CF::MF, A4, B4, tag, M, N, K, lda, ldb, ms, fl / ms / 1e9,
         maxrel(C, Cref, M, N, ldc));
  return ms;
}

// the shapes swept: (stages, k-rows per stage, wave grid, blocks per CU)
using C1 = D2Cfg<2, 16, 2, 2, 2>;      // 74 KB, 4x4x4_4b
using C2 = D2Cfg<2, 16, 2, 2, 2, 1>;   // 74 KB, 16x16x4
using C3 = D2Cfg<2, 32, 2, 2, 1, 1>;   // 147 KB, 16x16x4, one block per CU
using C4 = D2Cfg<4, 8, 4, 2, 1>;       // 256 x 128, 106 KB
using C5 = D2Cfg<4, 8, 4, 2, 1, 1>;    // 256 x 128, 106 KB, 16x16x4
using C6 = D2Cfg<3, 8, 2, 2, 2, 1>;    // 55 KB, 16x16x4
using C7 = D2Cfg<3, 8, 2, 2, 2>;       // 55 KB
template <class F>
static void sweep(F &&f) {
  f(C1{});
  f(C2{});
  f(C3{});
  f(C4{});
  f(C5{});
  f(C6{});
  f(C7{});
}

static void run1(const char *tag, const double *A, int lda, const double *B, double *C, int M, int N,
                 int K, const double *Cref) {
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
  g.order = 0;
  constexpr size_t lds = dgemm_smem<true>();
  (void)hipFuncSetAttribute((const void *)k_dgemm<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int nb = ((g.mt * g.nt + 7) / 8) * 8;
  const double fl = 2.0 * M * (double)N * K;
  const double ms = time_it([&] { k_dgemm<true><<<nb, 256, lds>>>(g); }, 10);
  printf("k_dgemm<T> (r2)   %-8s M=%d N=%d K=%d: %.3f ms  %.1f TFLOP/s  maxrel %.2e\n", tag, M, N, K,
         ms, fl / ms / 1e9, maxrel(C, Cref, M, N, N));
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

int main(int argc, char **argv) {
  const bool prof = argc > 1;   // profiling mode: the NPD product on rocBLAS and k_dgemm2 only
  const int F = 2049, NF0 = 1092, N = 20000, N2 = 40000, FP = 2064;
  double *WF0, *WF0T, *HF0, *T0, *C, *Cref;
  (void)hipMalloc(&WF0, sizeof(double) * F * NF0);        // [F][NF0]
  (void)hipMalloc(&WF0T, sizeof(double) * NF0 * FP);      // [NF0][FP]
  (void)hipMalloc(&HF0, sizeof(double) * NF0 * N);
  (void)hipMalloc(&T0, sizeof(double) * F * N2);
  (void)hipMalloc(&C, sizeof(double) * F * N2);
  (void)hipMalloc(&Cref, sizeof(double) * F * N2);
  fill(WF0, (size_t)F * NF0, 1);
  fill(HF0, (size_t)NF0 * N, 2);
  fill(T0, (size_t)F * N2, 3);
  {
    std::vector<double> w((size_t)F * NF0), wt((size_t)NF0 * FP, 0.0);
    (void)hipMemcpy(w.data(), WF0, w.size() * 8, hipMemcpyDeviceToHost);
    for (int f = 0; f < F; ++f)
      for (int k = 0; k < NF0; ++k) wt[(size_t)k * FP + f] = w[(size_t)f * NF0 + k];
    (void)hipMemcpy(WF0T, wt.data(), wt.size() * 8, hipMemcpyHostToDevice);
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  // clock warm-up (~0.5 s)
  for (int w = 0; w < 300; ++w) blas_ta(h, WF0T, FP, HF0, N, Cref, N, F, N, NF0);
  (void)hipDeviceSynchronize();
  if (prof) {
    for (int r = 0; r < 5; ++r) blas_ta(h, WF0, NF0, T0, N2, Cref, N2, NF0, N2, F);
    run2<C1>("NPD", WF0, NF0, T0, N2, C, N2, NF0, N2, F, Cref, 5);
    run2<C2>("NPD", WF0, NF0, T0, N2, C, N2, NF0, N2, F, Cref, 5);
    (void)hipDeviceSynchronize();
    return 0;
  }
  const double fl = 2.0 * F * NF0 * (double)N;
  double ms = time_it([&] { blas_ta(h, WF0T, FP, HF0, N, Cref, N, F, N, NF0); }, 10);
  printf("rocblas SF0 = WF0 HF0      M=%d N=%d K=%d: %.3f ms  %.1f TFLOP/s\n", F, N, NF0, ms, fl / ms / 1e9);
  sweep([&](auto cf) { run2<decltype(cf)>("SF0", WF0T, FP, HF0, N, C, N, F, N, NF0, Cref); });
  ms = time_it([&] { blas_ta(h, WF0, NF0, T0, N2, Cref, N2, NF0, N2, F); }, 10);
  printf("rocblas NPD = WF0^T T      M=%d N=%d K=%d: %.3f ms  %.1f TFLOP/s\n", NF0, N2, F, ms,
         2.0 * NF0 * (double)N2 * F / ms / 1e9);
  sweep([&](auto cf) { run2<decltype(cf)>("NPD", WF0, NF0, T0, N2, C, N2, NF0, N2, F, Cref); });
  run1("NPD", WF0, NF0, T0, C, NF0, N2, F, Cref);
  // edges: odd N (ldb even), odd M with even lda, K % 16 != 0, small
  struct E { int M, N, K, lda, ldb; } es[] = {{1091, 1999, 1000, 1092, 2000}, {130, 258, 37, 130, 258},
                                             {7, 5, 3, 8, 6}, {2049, 300, 1092, 2064, 300}};
  for (auto e : es) {
    blas_ta(h, WF0T, e.lda, HF0, e.ldb, Cref, e.N, e.M, e.N, e.K);
    run2<C1>("edge", WF0T, e.lda, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 2);
    run2<C2>("edge", WF0T, e.lda, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 2);
    run2<D2Prod, true, true>("edge4", WF0T, e.lda, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 2);
  }
  // odd leading dimensions (rows 8-byte aligned only): the 4-byte load variants
  struct E2 { int M, N, K, lda, ldb; } es2[] = {{1091, 1999, 1000, 1091, 1999}, {2049, 19999, 1092, 2049, 19999},
                                              {130, 257, 37, 131, 257}};
  for (auto e : es2) {
    blas_ta(h, WF0T, e.lda, HF0, e.ldb, Cref, e.N, e.M, e.N, e.K);
    run2<D2Prod, true, true>("odd-ld", WF0T, e.lda, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 3);
    run2<C4, true, true>("odd-ld", WF0T, e.lda, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 3);
    const int lda2 = e.lda + (e.lda & 1);
    blas_ta(h, WF0T, lda2, HF0, e.ldb, Cref, e.N, e.M, e.N, e.K);
    run2<D2Prod, false, true>("odd-ldb", WF0T, lda2, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 3);
    run2<C4, false, true>("odd-ldb", WF0T, lda2, HF0, e.ldb, C, e.N, e.M, e.N, e.K, Cref, 3);
  }
  rocblas_destroy_handle(h);
  return 0;
}
