// Itakura-Saito NMF multiplicative updates on MI355X (gfx950), FP64.
//
// Restates tools/nmf.py NMF_decomposition (:24-61) / NMF_decomp_init
// (:63-159).  One iteration:
//   hat = W H                      (MFMA GEMM, F x N x K)
//   X = SX/max(hat^2, eps), Y = 1/max(hat, eps)
//   num^T = H X^T, den^T = H Y^T   (one GEMM launch, shared H operand)
//   W *= num/max(den, eps); s = colsum(W), s[s==0] = 1; W /= s; H *= s
//   hat = W H; X, Y as above
//   num = W^T X, den = W^T Y       (one GEMM launch, shared W operand)
//   H *= num/max(den, eps)
#include "fasst_gemm.h"

#include <algorithm>

#include "../../include/fasst_nmf.h"

namespace fasst {

constexpr double kNmfEps = 1e-10;  // tools/nmf.py:22

__global__ void k_nmf_xy(const double *__restrict__ hat, const double *__restrict__ SX,
                         double *__restrict__ X, double *__restrict__ Y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const double h = hat[i];
    X[i] = SX[i] / fmax(h * h, kNmfEps);
    Y[i] = 1.0 / fmax(h, kNmfEps);
  }
}

// one block per component k: W[:, k] update, column sum, renormalisation
__global__ __launch_bounds__(256) void k_nmf_w(double *__restrict__ W,
                                               const double *__restrict__ numT,
                                               const double *__restrict__ denT,
                                               double *__restrict__ s_out, int F, int K) {
  __shared__ double s_red[256];
  const int k = blockIdx.x;
  double part = 0.0;
  for (int f = threadIdx.x; f < F; f += 256) {
    const double w = W[(size_t)f * K + k] * (numT[(size_t)k * F + f] / fmax(denT[(size_t)k * F + f], kNmfEps));
    W[(size_t)f * K + k] = w;
    part += w;
  }
  s_red[threadIdx.x] = part;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
    __syncthreads();
  }
  double s = s_red[0];
  if (s == 0) s = 1.0;  // sumW[sumW==0] = 1. (nmf.py:46)
  for (int f = threadIdx.x; f < F; f += 256) W[(size_t)f * K + k] /= s;
  if (threadIdx.x == 0) s_out[k] = s;
}

__global__ void k_nmf_hscale(double *__restrict__ H, const double *__restrict__ s, int K,
                             int N) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)K * N;
       i += (size_t)gridDim.x * blockDim.x)
    H[i] *= s[i / N];
}

__global__ void k_nmf_h(double *__restrict__ H, const double *__restrict__ num,
                        const double *__restrict__ den, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    H[i] *= num[i] / fmax(den[i], kNmfEps);
}

}  // namespace fasst

using namespace fasst;

struct nmf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int F = 0, N = 0, K = 0;
  DBuf<double> SX, W, H, hat, X, Y, numT, denT, num, den, s, work;
};

namespace {

int egrid_n(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 8192); }

int model_xy(nmf_ctx *c) {
  const double *Bs[1] = {c->H.p};
  double *Cs[1] = {c->hat.p};
  int st = gemm<false, false, 1>(c->stream, c->W.p, c->K, Bs, c->N, Cs, c->N, c->F, c->N, c->K,
                                 c->work.p);
  if (st) return st;
  const size_t FN = (size_t)c->F * c->N;
  k_nmf_xy<<<egrid_n(FN), 256, 0, c->stream>>>(c->hat.p, c->SX.p, c->X.p, c->Y.p, FN);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int nmf_iteration(nmf_ctx *c, int update_w, int update_h) {
  int st;
  const int F = c->F, N = c->N, K = c->K;
  if (update_w) {
    if ((st = model_xy(c))) return st;
    const double *Bs[2] = {c->X.p, c->Y.p};
    double *Cs[2] = {c->numT.p, c->denT.p};
    if ((st = gemm<false, true, 2>(c->stream, c->H.p, N, Bs, N, Cs, F, K, F, N, c->work.p)))
      return st;
    k_nmf_w<<<K, 256, 0, c->stream>>>(c->W.p, c->numT.p, c->denT.p, c->s.p, F, K);
    k_nmf_hscale<<<egrid_n((size_t)K * N), 256, 0, c->stream>>>(c->H.p, c->s.p, K, N);
    FASST_LAUNCH_CHECK();
  }
  if (update_h) {
    if ((st = model_xy(c))) return st;
    const double *Bs[2] = {c->X.p, c->Y.p};
    double *Cs[2] = {c->num.p, c->den.p};
    if ((st = gemm<true, false, 2>(c->stream, c->W.p, K, Bs, N, Cs, N, K, N, F, c->work.p)))
      return st;
    k_nmf_h<<<egrid_n((size_t)K * N), 256, 0, c->stream>>>(c->H.p, c->num.p, c->den.p,
                                                           (size_t)K * N);
    FASST_LAUNCH_CHECK();
  }
  return FASST_OK;
}

}  // namespace

extern "C" {

int nmf_create(int device, int F, int N, int K, nmf_ctx **out) {
  if (!out || F < 1 || N < 1 || K < 1) {
    set_error("nmf_create: bad sizes F=%d N=%d K=%d", F, N, K);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  nmf_ctx *c = new nmf_ctx();
  c->device = device;
  c->F = F;
  c->N = N;
  c->K = K;
  const size_t FN = (size_t)F * N;
  int st = FASST_OK;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) st = FASST_ERR_DEVICE;
  size_t gw = std::max({gemm_workspace(F, N, K, 1), gemm_workspace(K, F, N, 2),
                        gemm_workspace(K, N, F, 2), (size_t)1});
  if (!st) st = c->SX.alloc(FN);
  if (!st) st = c->W.alloc((size_t)F * K);
  if (!st) st = c->H.alloc((size_t)K * N);
  if (!st) st = c->hat.alloc(FN);
  if (!st) st = c->X.alloc(FN);
  if (!st) st = c->Y.alloc(FN);
  if (!st) st = c->numT.alloc((size_t)K * F);
  if (!st) st = c->denT.alloc((size_t)K * F);
  if (!st) st = c->num.alloc((size_t)K * N);
  if (!st) st = c->den.alloc((size_t)K * N);
  if (!st) st = c->s.alloc(K);
  if (!st) st = c->work.alloc(gw);
  if (st) {
    nmf_destroy(c);
    return st;
  }
  *out = c;
  return FASST_OK;
}

int nmf_destroy(nmf_ctx *c) {
  if (!c) return FASST_OK;
  {
    DeviceGuard g(c->device);
    if (c->stream) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamDestroy(c->stream);
    }
  }
  delete c;
  return FASST_OK;
}

int nmf_set_data(nmf_ctx *c, const double *SX) {
  if (!c || !SX) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  FASST_HIP(hipMemcpyAsync(c->SX.p, SX, (size_t)c->F * c->N * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_set_params(nmf_ctx *c, const double *W, const double *H) {
  if (!c || !W || !H) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  FASST_HIP(hipMemcpyAsync(c->W.p, W, (size_t)c->F * c->K * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(c->H.p, H, (size_t)c->K * c->N * 8, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_run(nmf_ctx *c, int n_iter, int update_w, int update_h) {
  if (!c || n_iter < 0) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  for (int it = 0; it < n_iter; ++it) {
    int st = nmf_iteration(c, update_w, update_h);
    if (st) return st;
  }
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int nmf_get_params(nmf_ctx *c, double *W, double *H) {
  if (!c) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (W) FASST_HIP(hipMemcpyAsync(W, c->W.p, (size_t)c->F * c->K * 8, hipMemcpyDeviceToHost, c->stream));
  if (H) FASST_HIP(hipMemcpyAsync(H, c->H.p, (size_t)c->K * c->N * 8, hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

}  // extern "C"
