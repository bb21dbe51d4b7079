// The FB contraction's rho stream (C3: F=2049, T=10000, J=4, K=32) in two
// layouts, with and without its MFMAs:
//   strip : rho [J][Tp][Fp] (the E-step's layout), a wave's 16-frame x 32-bin
//           tile is 16 rows x 256 B, 16.5 KB apart
//   tiled : rho [J][Fp/32][Tp][32], the same tile is 4 KB contiguous and a
//           wave's frame chunk one sequential run
// MFMA on: num[2][2] += rho tile x (FW.H)^T tile (the k_fb_contract loop);
// off: the loads are summed (the streaming floor of the pattern).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_fbread.hip -o tools/ubench_fbread
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

template <bool TILED, bool MF>
__global__ __launch_bounds__(64) void k_fb(const double *__restrict__ rho, const double *__restrict__ fwht,
                                          double *__restrict__ out, int Fp, int Tp, int KP, int tpc, int ntt) {
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int fg = blockIdx.x, j = blockIdx.y;
  const int tb = blockIdx.z * tpc, te = min(tb + tpc, ntt);
  d4 num[2][2];
  for (int p = 0; p < 2; ++p)
    for (int k = 0; k < 2; ++k) num[p][k] = d4{0, 0, 0, 0};
  double acc = 0.0;
  const double *rj = rho + (size_t)j * Tp * Fp;
  for (int tt = tb; tt < te; ++tt) {
    const int t0 = tt * 16;
    double fb[4][2];
    const double *fwh = fwht + ((size_t)j * Tp + t0 + tq) * KP + fl;
    if (MF)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) fb[i][kc] = fwh[(size_t)(4 * i) * KP + kc * 16];
    double r[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + tq + 4 * i;
      const size_t off = TILED ? ((size_t)fg * Tp + t) * 32 + 2 * fl : (size_t)t * Fp + fg * 32 + 2 * fl;
      const double2 v = *(const double2 *)(rj + off);
      r[0][i] = v.x;
      r[1][i] = v.y;
    }
    if (MF) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int kc = 0; kc < 2; ++kc)
            num[p][kc] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[p][i], fb[i][kc], num[p][kc], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc += r[0][i] + r[1][i];
    }
  }
  double s = acc;
  for (int p = 0; p < 2; ++p)
    for (int k = 0; k < 2; ++k) s += num[p][k][0] + num[p][k][1] + num[p][k][2] + num[p][k][3];
  out[(((size_t)blockIdx.z * gridDim.y + j) * gridDim.x + fg) * 64 + lane] = s;
}

int main() {
  const int F = 2049, T = 10000, J = 4, KP = 32, Fp = 2080, Tp = 10000, ntt = Tp / 16, nfg = Fp / 32;
  const size_t plane = (size_t)Fp * Tp;
  double *rho, *fwht, *out;
  CK(hipMalloc(&rho, J * plane * 8));
  CK(hipMalloc(&fwht, (size_t)J * Tp * KP * 8));
  CK(hipMalloc(&out, (size_t)64 * nfg * J * 64 * 8));
  std::vector<double> h(J * plane);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 + (i % 977) * 1e-3;
  CK(hipMemcpy(rho, h.data(), J * plane * 8, hipMemcpyHostToDevice));
  CK(hipMemset(fwht, 0, (size_t)J * Tp * KP * 8));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)F * T * J * 8;
  auto timeit = [&](const char *name, auto launch) {
    for (int w = 0; w < 40; ++w) launch();
    hipEventRecord(e0);
    const int n = 100;
    for (int r = 0; r < n; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= n;
    printf("%-28s %.4f ms  %.0f GB/s of rho\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int nch : {19, 38}) {
    const int tpc = (ntt + nch - 1) / nch;
    const dim3 g(nfg, J, nch);
    char nm[64];
    snprintf(nm, 64, "strip mfma  nchunk=%d", nch);
    timeit(nm, [&] { k_fb<false, true><<<g, 64>>>(rho, fwht, out, Fp, Tp, KP, tpc, ntt); });
    snprintf(nm, 64, "tiled mfma  nchunk=%d", nch);
    timeit(nm, [&] { k_fb<true, true><<<g, 64>>>(rho, fwht, out, Fp, Tp, KP, tpc, ntt); });
    snprintf(nm, 64, "strip read  nchunk=%d", nch);
    timeit(nm, [&] { k_fb<false, false><<<g, 64>>>(rho, fwht, out, Fp, Tp, KP, tpc, ntt); });
    snprintf(nm, 64, "tiled read  nchunk=%d", nch);
    timeit(nm, [&] { k_fb<true, false><<<g, 64>>>(rho, fwht, out, Fp, Tp, KP, tpc, ntt); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
