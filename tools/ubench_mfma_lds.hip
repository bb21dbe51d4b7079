// Compute-side ceiling of an FP64 GEMM inner loop on gfx950: operands read
// from LDS every k-step (ds_read_b64), no global traffic, random data.
//   k16 : v_mfma_f64_16x16x4f64, wave tile 64 x 64 = 4 x 4 accumulators (d4),
//         per k-step 4 A + 4 B reads, 16 MFMAs
//   k44 : v_mfma_f64_4x4x4f64 (4 blocks), the four blocks as 2 (m) x 2 (n)
//         sub-blocks, wave tile (8 RA) x (8 RB) = RA x RB one-double
//         accumulators, per k-step RA + RB reads, RA RB MFMAs
// WPS = waves per SIMD (blocks of 256 threads per CU).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma_lds.hip -o tools/ubench_mfma_lds
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int P = 144;   // LDS pitch (doubles)

__device__ void fill(double *s, int n, double seed) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    unsigned long long x = (unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ULL + (unsigned long long)(seed * 1e6);
    x ^= x >> 29;
    s[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0) + 0.5;
  }
  __syncthreads();
}

template <int WPS>
__global__ __launch_bounds__(256, WPS) void k16(double *out, int iters) {
  __shared__ double s[2 * 16 * P];
  fill(s, 2 * 16 * P, blockIdx.x);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, tq = lane >> 4, wm = wv >> 1, wn = wv & 1;
  d4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0, 0, 0, 0};
  const double *sA = s, *sB = s + 16 * P;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kr = 4 * kk + tq;
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = sA[kr * P + wm * 64 + i * 16 + fl];
        b[i] = sB[kr * P + wn * 64 + i * 16 + fl];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  double t = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int WPS, int RA, int RB>
__global__ __launch_bounds__(256, WPS) void k44(double *out, int iters) {
  __shared__ double s[2 * 16 * P];
  fill(s, 2 * 16 * P, blockIdx.x);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int X = lane >> 4, b = (lane >> 2) & 3, Y = lane & 3;
  const int bm = b >> 1, bn = b & 1, wm = wv >> 1, wn = wv & 1;
  double acc[RA][RB];
  for (int i = 0; i < RA; ++i)
    for (int j = 0; j < RB; ++j) acc[i][j] = 0.0;
  const double *sA = s + wm * 8 * RA + 4 * bm + Y, *sB = s + 16 * P + wn * 8 * RB + 4 * bn + Y;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kr = 4 * kk + X;
      double a[RA], bb[RB];
#pragma unroll
      for (int i = 0; i < RA; ++i) a[i] = sA[kr * P + 8 * i];
#pragma unroll
      for (int j = 0; j < RB; ++j) bb[j] = sB[kr * P + 8 * j];
#pragma unroll
      for (int i = 0; i < RA; ++i)
#pragma unroll
        for (int j = 0; j < RB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
  }
  double t = 0;
  for (int i = 0; i < RA; ++i)
    for (int j = 0; j < RB; ++j) t += acc[i][j];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <class L>
static float timeit(L launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 30; ++w) launch();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 20;
}

int main() {
  double *out;
  (void)hipMalloc(&out, 256 * 256 * 16 * sizeof(double));
  const int iters = 200;
  // warm the clock
  for (int w = 0; w < 400; ++w) k16<2><<<512, 256>>>(out, iters);
  (void)hipDeviceSynchronize();
  for (int wps : {1, 2}) {
    const int nb = 256 * wps * 2;   // two rounds
    float ms = wps == 1 ? timeit([&] { k16<1><<<nb, 256>>>(out, iters); })
                        : timeit([&] { k16<2><<<nb, 256>>>(out, iters); });
    const double fl = (double)nb * 4 * iters * 4 * 16 * 2048.0;
    printf("k16 16x16x4 tile 64x64 WPS=%d: %.3f ms %.1f TF\n", wps, ms, fl / ms / 1e9);
  }
  for (int wps : {1, 2}) {
    const int nb = 256 * wps * 2;
    float ms = wps == 1 ? timeit([&] { k44<1, 8, 8><<<nb, 256>>>(out, iters); })
                        : timeit([&] { k44<2, 8, 8><<<nb, 256>>>(out, iters); });
    const double fl = (double)nb * 4 * iters * 4 * 64 * 512.0;
    printf("k44 4x4x4_4b tile 64x64 (8x8) WPS=%d: %.3f ms %.1f TF\n", wps, ms, fl / ms / 1e9);
  }
  {
    const int nb = 256 * 2;
    float ms = timeit([&] { k44<1, 16, 8><<<nb, 256>>>(out, iters); });
    const double fl = (double)nb * 4 * iters * 4 * 128 * 512.0;
    printf("k44 4x4x4_4b tile 128x64 (16x8) WPS=1: %.3f ms %.1f TF\n", ms, fl / ms / 1e9);
  }
  {
    const int nb = 256 * 2;
    float ms = timeit([&] { k44<1, 8, 16><<<nb, 256>>>(out, iters); });
    const double fl = (double)nb * 4 * iters * 4 * 128 * 512.0;
    printf("k44 4x4x4_4b tile 64x128 (8x16) WPS=1: %.3f ms %.1f TF\n", ms, fl / ms / 1e9);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
