// FP64 peak calibration on MI355X: v_mfma_f64_16x16x4f64 and v_fma_f64 throughput.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_fp64.hip -o /tmp/ubench_fp64
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double *out, int iters, double a0) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NCH>
__global__ __launch_bounds__(256) void k_fma(double *out, int iters, double a0) {
  double x[NCH];
  for (int i = 0; i < NCH; ++i) x[i] = a0 + i + threadIdx.x * 1e-9;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < NCH; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA and VALU FMA chains interleaved in one wave: NA MFMA accumulators,
// NC VALU chains, R VALU rounds per MFMA round
template <int NA, int NC, int R>
__global__ __launch_bounds__(256) void k_mix(double *out, int iters, double a0) {
  d4 acc[NA];
  for (int i = 0; i < NA; ++i) acc[i] = d4{0, 0, 0, 0};
  double x[NC];
  for (int i = 0; i < NC; ++i) x[i] = a0 + i + threadIdx.x * 1e-9;
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NA; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < NC; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < NA; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < NC; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma4(double *out, int iters, double a0) {
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
  hipMalloc(&out, 256 * 8192 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 2000;
  float ms;
  // warm: ~0.5 s of MFMA work first, so every test runs at the settled clock
  // (the round-1 figures for 16x16x4 ran first, during the clock ramp)
  for (int w = 0; w < 40; ++w) k_mfma<8><<<blocks, 256>>>(out, iters, 1.0);
  hipDeviceSynchronize();
#define RUN_MFMA(N)                                                                         \
  hipEventRecord(e0);                                                                       \
  k_mfma<N><<<blocks, 256>>>(out, iters, 1.0);                                              \
  hipEventRecord(e1);                                                                       \
  hipEventSynchronize(e1);                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                         \
  printf("mfma_f64_16x16x4 acc=%d: %.2f TFLOP/s (%.1f cyc/MFMA/SIMD @2.4GHz)\n", N,        \
         (double)blocks * 4 * iters * N * 2048.0 / (ms * 1e-3) / 1e12,                      \
         (ms * 1e-3 * 2.4e9) / ((double)blocks * 4 / 1024.0 * iters * N));
  RUN_MFMA(1) RUN_MFMA(2) RUN_MFMA(4) RUN_MFMA(8)
#define RUN_FMA(N)                                                                          \
  hipEventRecord(e0);                                                                       \
  k_fma<N><<<blocks, 256>>>(out, iters, 1.0);                                               \
  hipEventRecord(e1);                                                                       \
  hipEventSynchronize(e1);                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                         \
  printf("v_fma_f64 chains=%d: %.2f TFLOP/s\n", N,                                          \
         (double)blocks * 256 * iters * N * 2.0 / (ms * 1e-3) / 1e12);
  RUN_FMA(1) RUN_FMA(4) RUN_FMA(8) RUN_FMA(16)
#define RUN_MIX(NA, NC, R)                                                                  \
  hipEventRecord(e0);                                                                       \
  k_mix<NA, NC, R><<<blocks, 256>>>(out, iters, 1.0);                                       \
  hipEventRecord(e1);                                                                       \
  hipEventSynchronize(e1);                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                         \
  printf("mix mfma acc=%d + fma chains=%d x%d: %.2f TFLOP/s (mfma %.2f + valu %.2f)\n", NA, NC, R, \
         ((double)blocks * 4 * iters * NA * 2048.0 + (double)blocks * 256 * iters * NC * R * 2.0) / \
             (ms * 1e-3) / 1e12,                                                            \
         (double)blocks * 4 * iters * NA * 2048.0 / (ms * 1e-3) / 1e12,                     \
         (double)blocks * 256 * iters * NC * R * 2.0 / (ms * 1e-3) / 1e12);
  RUN_MIX(4, 8, 1) RUN_MIX(4, 8, 2) RUN_MIX(4, 8, 4) RUN_MIX(8, 8, 2) RUN_MIX(8, 16, 2)
#define RUN_MFMA4(N)                                                                        \
  hipEventRecord(e0);                                                                       \
  k_mfma4<N><<<blocks, 256>>>(out, iters, 1.0);                                             \
  hipEventRecord(e1);                                                                       \
  hipEventSynchronize(e1);                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                         \
  printf("mfma_f64_4x4x4_4b acc=%d: %.2f TFLOP/s\n", N,                                     \
         (double)blocks * 4 * iters * N * 512.0 / (ms * 1e-3) / 1e12);
  RUN_MFMA4(4) RUN_MFMA4(8) RUN_MFMA4(16)
  // 16x16x4 again, last (after the longest-running tests)
  RUN_MFMA(4) RUN_MFMA(8)
  return 0;
}
