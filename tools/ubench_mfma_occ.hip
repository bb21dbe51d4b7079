// v_mfma_f64_16x16x4f64 throughput vs waves per SIMD and operand reuse
// (after a clock warm-up).  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma_occ.hip -o tools/ubench_mfma_occ
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

// NA A operands x NB B operands, NA*NB accumulators (a GEMM-like register tile)
template <int NA, int NB>
__global__ __launch_bounds__(256) void k_tile(double *out, int iters, double a0) {
  d4 acc[NA][NB];
  double a[NA], b[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) a[i] = a0 + i * 1e-3 + threadIdx.x * 1e-9;
#pragma unroll
  for (int j = 0; j < NB; ++j) b[j] = a0 - j * 1e-3 - threadIdx.x * 1e-9;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < NA; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_4x4(double *out, int iters, double a0) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0;
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double *out;
  (void)hipMalloc(&out, 256 * 8192 * sizeof(double));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms;
  for (int w = 0; w < 60; ++w) k_tile<4, 2><<<2048, 256>>>(out, 2000, 1.0);
  (void)hipDeviceSynchronize();
#define RUN_T(NA, NB, BLOCKS, IT)                                                           \
  (void)hipEventRecord(e0);                                                                 \
  k_tile<NA, NB><<<BLOCKS, 256>>>(out, IT, 1.0);                                            \
  (void)hipEventRecord(e1);                                                                 \
  (void)hipEventSynchronize(e1);                                                            \
  (void)hipEventElapsedTime(&ms, e0, e1);                                                   \
  printf("16x16x4 tile %dx%d blocks=%d (%.2f waves/SIMD): %.2f TFLOP/s (%.1f cyc/MFMA/SIMD @2.4GHz)\n", \
         NA, NB, BLOCKS, BLOCKS * 4 / 1024.0,                                               \
         (double)BLOCKS * 4 * IT * NA * NB * 2048.0 / (ms * 1e-3) / 1e12,                   \
         (ms * 1e-3 * 2.4e9) / ((double)BLOCKS * 4 / 1024.0 * IT * NA * NB));
  RUN_T(1, 1, 256, 16000) RUN_T(4, 2, 256, 4000) RUN_T(8, 2, 256, 2000) RUN_T(4, 4, 256, 2000)
  RUN_T(4, 2, 512, 2000) RUN_T(8, 2, 512, 1000) RUN_T(4, 2, 1024, 1000) RUN_T(8, 2, 1024, 500)
  RUN_T(4, 2, 2048, 500) RUN_T(1, 1, 2048, 4000)
#define RUN_4(N, BLOCKS, IT)                                                                \
  (void)hipEventRecord(e0);                                                                 \
  k_4x4<N><<<BLOCKS, 256>>>(out, IT, 1.0);                                                  \
  (void)hipEventRecord(e1);                                                                 \
  (void)hipEventSynchronize(e1);                                                            \
  (void)hipEventElapsedTime(&ms, e0, e1);                                                   \
  printf("4x4x4_4b acc=%d blocks=%d: %.2f TFLOP/s\n", N, BLOCKS,                            \
         (double)BLOCKS * 4 * IT * N * 512.0 / (ms * 1e-3) / 1e12);
  RUN_4(16, 256, 8000) RUN_4(16, 2048, 1000)
  return 0;
}
