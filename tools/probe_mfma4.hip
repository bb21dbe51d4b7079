// Probe the lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950: one wave per
// (la, lb) pair with A = e_la, B = e_lb; prints the lanes where D != 0.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_probe(unsigned long long *out) {
  const int la = blockIdx.x / 64, lb = blockIdx.x % 64, l = threadIdx.x;
  double a = l == la ? 1.0 : 0.0, b = l == lb ? 1.0 : 0.0;
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  unsigned long long m = __ballot(d != 0.0);
  if (l == 0) out[blockIdx.x] = m;
}
int main() {
  unsigned long long *d, h[4096];
  (void)hipMalloc(&d, sizeof(h));
  k_probe<<<4096, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < 4096; ++i)
    if (h[i]) printf("%d %d %llx\n", i / 64, i % 64, h[i]);
  return 0;
}
