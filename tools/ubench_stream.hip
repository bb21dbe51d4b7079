// HBM streaming floor of the E-step's access pattern (C3: F=2049, T=10000).
// Reads 4 Cx planes, writes J=4 rho planes, nothing else, in three layouts:
//   strip : [Tp][Fp] planes, block = one 16-bin tile walking a frame chunk,
//           a wave reads 4 rows x 128 B per instruction (the round-2 E-step)
//   tiled : [Fp/16][Tp][16] planes, same block walk: the strip is contiguous
//   flat  : grid-stride 16-byte streaming over the whole planes (the ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o tools/ubench_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NT>
__global__ __launch_bounds__(256, 2) void k_strip(const double *__restrict__ c0, const double *__restrict__ c1,
                                                  const double *__restrict__ c2, const double *__restrict__ c3,
                                                  double *__restrict__ out, int Fp, int Tp, int tpc, int ntt,
                                                  int tiled) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, tq = lane >> 4;
  const int ft = blockIdx.x, f = ft * 16 + fl;
  const int tb = blockIdx.y * tpc, te = min(tb + tpc, ntt);
  for (int tt = tb + wv; tt < te; tt += 4) {
    double x[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = tt * 16 + tq + 4 * i;
      const size_t off = tiled ? ((size_t)ft * Tp + t) * 16 + fl : (size_t)t * Fp + f;
      x[0][i] = __builtin_nontemporal_load(c0 + off);
      x[1][i] = __builtin_nontemporal_load(c1 + off);
      x[2][i] = __builtin_nontemporal_load(c2 + off);
      x[3][i] = __builtin_nontemporal_load(c3 + off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = tt * 16 + tq + 4 * i;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const double r = x[0][i] * (j + 1) + x[1][i] - x[2][i] * x[3][i];
        const size_t off = tiled ? (((size_t)j * (Fp / 16) + ft) * Tp + t) * 16 + fl
                                 : ((size_t)j * Tp + t) * Fp + f;
        __builtin_nontemporal_store(r, out + off);
      }
    }
  }
}

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_flat(const dv2 *__restrict__ c0, const dv2 *__restrict__ c1,
                                              const dv2 *__restrict__ c2, const dv2 *__restrict__ c3,
                                              dv2 *__restrict__ out, size_t n2) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
    const dv2 a = __builtin_nontemporal_load(c0 + i), b = __builtin_nontemporal_load(c1 + i);
    const dv2 c = __builtin_nontemporal_load(c2 + i), d = __builtin_nontemporal_load(c3 + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dv2 r;
      r.x = a.x * (j + 1) + b.x - c.x * d.x;
      r.y = a.y * (j + 1) + b.y - c.y * d.y;
      __builtin_nontemporal_store(r, out + j * n2 + i);
    }
  }
}

int main() {
  const int F = 2049, T = 10000, Fp = 2064, Tp = 10000, ntt = Tp / 16, nft = Fp / 16;
  const size_t plane = (size_t)Fp * Tp;
  double *c[4], *out;
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&c[i], plane * 8));
    CK(hipMemset(c[i], 0, plane * 8));
  }
  CK(hipMalloc(&out, 4 * plane * 8));
  std::vector<double> h(plane);
  for (size_t i = 0; i < plane; ++i) h[i] = 1.0 + (i % 977) * 1e-3;
  for (int i = 0; i < 4; ++i) CK(hipMemcpy(c[i], h.data(), plane * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)F * T * (32 + 32);
  auto timeit = [&](const char *name, auto launch) {
    for (int w = 0; w < 40; ++w) launch();  // clock ramp
    hipEventRecord(e0);
    const int n = 50;
    for (int r = 0; r < n; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= n;
    printf("%-28s %.4f ms  %.0f GB/s (algorithmic %.2f GB)\n", name, ms, bytes / (ms * 1e-3) / 1e9, bytes / 1e9);
  };
  for (int nch : {8, 15, 30, 60}) {
    const int tpc = (ntt + nch - 1) / nch;
    char nm[64];
    snprintf(nm, 64, "strip nchunk=%d", nch);
    timeit(nm, [&] { k_strip<4><<<dim3(nft, nch), 256>>>(c[0], c[1], c[2], c[3], out, Fp, Tp, tpc, ntt, 0); });
    snprintf(nm, 64, "tiled nchunk=%d", nch);
    timeit(nm, [&] { k_strip<4><<<dim3(nft, nch), 256>>>(c[0], c[1], c[2], c[3], out, Fp, Tp, tpc, ntt, 1); });
  }
  timeit("flat", [&] { k_flat<<<2048, 256>>>((dv2 *)c[0], (dv2 *)c[1], (dv2 *)c[2], (dv2 *)c[3],
                                              (dv2 *)out, plane / 2); });
  CK(hipDeviceSynchronize());
  return 0;
}
