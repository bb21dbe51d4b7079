// Do FP64 MFMA and FP64 VALU instructions of two waves on one SIMD execute
// at the same time on gfx950?  512-thread blocks (two waves per SIMD): waves
// 0-3 run a chain-free FP64 MFMA loop, waves 4-7 a chain-free v_fma_f64 loop.
// mode 0: both roles, 1: MFMA waves only, 2: VALU waves only.  If the pipes
// are separate, t(both) ~ max(t1, t2); if they share issue or the DP unit,
// t(both) ~ t1 + t2.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_coexec.hip -o tools/ubench_coexec
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int SHAPE, int VK = 0>  // SHAPE 0: 4x4x4_4b, 1: 16x16x4; VK 0: v_fma_f64, 1: u64 adds, 2: v_fma_f32
__global__ __launch_bounds__(512) void k_coexec(double *out, int mode, int iters_m, int iters_v) {
  const int wv = threadIdx.x >> 6;
  const double x = 1.0 + threadIdx.x * 1e-9;
  double r = 0.0;
  if (wv < 4) {
    if (mode == 2) return;
    if (SHAPE == 0) {
      double acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.0;
      for (int it = 0; it < iters_m; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, x + i, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) r += acc[i];
    } else {
      d4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = d4{0, 0, 0, 0};
      for (int it = 0; it < iters_m; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x + i, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    }
  } else {
    if (mode == 1) return;
    if (VK == 0) {
      double a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = x + i;
      for (int it = 0; it < iters_v; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = fma(a[i], x, 1e-12);
#pragma unroll
      for (int i = 0; i < 16; ++i) r += a[i];
    } else if (VK == 1) {   // 64-bit address arithmetic (v_lshl_add_u64)
      unsigned long long a[16];
      const unsigned long long st = (unsigned long long)out + threadIdx.x;
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = st + i;
      for (int it = 0; it < iters_v; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          a[i] = (a[i] << 3) + st;
          asm volatile("" : "+v"(a[i]));
        }
#pragma unroll
      for (int i = 0; i < 16; ++i) r += (double)(a[i] & 1023);
    } else {
      float a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = (float)x + i;
      for (int it = 0; it < iters_v; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = fmaf(a[i], (float)x, 1e-7f);
#pragma unroll
      for (int i = 0; i < 16; ++i) r += a[i];
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <class L>
static float timeit(L launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 10; ++w) launch();
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
  const int nb = 256 * 2;
  (void)hipMalloc(&out, (size_t)nb * 512 * sizeof(double));
  for (int w = 0; w < 200; ++w) k_coexec<0><<<nb, 512>>>(out, 0, 400, 400);
  (void)hipDeviceSynchronize();
  // 4x4x4_4b: 16 MFMAs per iteration; VALU: 16 FMAs per iteration
  const char *vname[3] = {"v_fma_f64", "v_lshl_add_u64", "v_fma_f32"};
  for (int vk = 0; vk < 3; ++vk)
  for (int shape = 0; shape < 2; ++shape) {
    const int im = shape == 0 ? 2000 : 500, iv = 2000;
    float t[3];
    for (int mode = 0; mode < 3; ++mode) {
      auto go = [&](auto L) { t[mode] = timeit(L); };
      if (shape == 0 && vk == 0) go([&] { k_coexec<0, 0><<<nb, 512>>>(out, mode, im, iv); });
      if (shape == 1 && vk == 0) go([&] { k_coexec<1, 0><<<nb, 512>>>(out, mode, im, iv); });
      if (shape == 0 && vk == 1) go([&] { k_coexec<0, 1><<<nb, 512>>>(out, mode, im, iv); });
      if (shape == 1 && vk == 1) go([&] { k_coexec<1, 1><<<nb, 512>>>(out, mode, im, iv); });
      if (shape == 0 && vk == 2) go([&] { k_coexec<0, 2><<<nb, 512>>>(out, mode, im, iv); });
      if (shape == 1 && vk == 2) go([&] { k_coexec<1, 2><<<nb, 512>>>(out, mode, im, iv); });
    }
    const double mf = (double)nb * 4 * im * (shape == 0 ? 16 * 512.0 : 4 * 2048.0);
    const double vf = (double)nb * 4 * 64 * iv * 16 * 2.0;
    printf("%s + %s: both %.3f ms | MFMA only %.3f ms (%.1f TF) | VALU only %.3f ms (%.1f T op/s) | "
           "both/(sum) %.2f both/(max) %.2f\n",
           shape == 0 ? "f64 4x4x4_4b" : "f64 16x16x4", vname[vk], t[0], t[1],
           mf / t[1] / 1e9, t[2], vf / t[2] / 1e9, t[0] / (t[1] + t[2]),
           t[0] / (t[1] > t[2] ? t[1] : t[2]));
  }
  (void)hipDeviceSynchronize();
  return 0;
}
