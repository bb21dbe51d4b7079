// Viterbi melody tracker on MI355X (gfx950): the reference's only native
// component, _tracking.pyx:11-93 (Cython), as max-plus matrix-vector steps.
//
// Frame n needs every state's cum[., n-1], so frames are sequential; the
// parallelism is over target states s (and over the source states s' of
// each reduction):
//   k_vt_frame4    one launch per frame (kernel boundaries are the frame
//                  barrier -- no in-launch grid synchronisation): 4 waves per
//                  target s, each over a quarter of s' with coalesced reads of
//                  the target-major transition row TT[s][.] (L2-resident
//                  across frames: S^2 doubles = 9.5 MB at S = 1092, 1.2 MB per
//                  XCD), 64-lane (value, index) butterflies, then the 4 wave
//                  results folded in source order.
//   k_vt_block     small S (the matrix fits in LDS): ONE workgroup runs every
//                  frame with TT and the two cum vectors in LDS, 16 waves over
//                  the targets, a workgroup barrier per frame.
//   k_vt_jump / k_vt_chain / k_vt_fill  numpy.argmax of the last column, then
//                  the antecedent chain by chunk jumps (~2 sqrt(N) dependent
//                  loads instead of N).
// Tie and NaN rules are the pyx's strict '>' scan from s' = 0 (lines 70-82):
// the first maximal s' wins, a NaN candidate never wins, and a NaN at s' = 0
// sticks.  cum[s', n-1] + T[s', s] and "+ logDensity" are the reference's
// own double additions, so cum and the path are bit-identical.
#include "fasst_common.h"
#include "../../include/fasst_viterbi.h"

#include <algorithm>
#include <climits>
#include <cmath>

namespace fasst {

constexpr size_t kVtLdsBudget = 150 * 1024;

// (v, i) beats (bv, bi) if larger, or equal with a smaller index; NaN never beats
__device__ __forceinline__ void vt_better(double &bv, int &bi, double v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

__device__ __forceinline__ void vt_wave_reduce(double &bv, int &bi) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    vt_better(bv, bi, ov, oi);
  }
}

// max_{s'} (cum[s'] + row[s']) with the pyx's rules, result in every lane.
// The candidates of a lane are loaded kVtBatch at a time before any compare,
// so a wave keeps kVtBatch L2 round trips in flight instead of one.
constexpr int kVtBatch = 16;
__device__ __forceinline__ void vt_argmax(const double *__restrict__ cum,
                                          const double *__restrict__ row, int S, int lane,
                                          double &bv, int &bi) {
  bv = -INFINITY;
  bi = INT_MAX;
  for (int base = 0; base < S; base += 64 * kVtBatch) {
    double v[kVtBatch];
#pragma unroll
    for (int u = 0; u < kVtBatch; ++u) {
      const int sp = base + u * 64 + lane;
      v[u] = sp < S ? cum[sp] + row[sp] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < kVtBatch; ++u) {
      const int sp = base + u * 64 + lane;
      if (sp < S) vt_better(bv, bi, v[u], sp);
    }
  }
  vt_wave_reduce(bv, bi);
  const double v0 = cum[0] + row[0];
  if (v0 != v0) {   // NaN at s' = 0: nothing compares greater (pyx :77)
    bv = v0;
    bi = 0;
  }
}

__global__ void k_vt_init(const double *__restrict__ prior, const double *__restrict__ logd0,
                          double *__restrict__ cum, int S) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < S) cum[s] = prior[s] + logd0[s];   // pyx :60-63
}

// One frame step (large S): a block of NW waves per target s; wave q reduces
// the source range [q*Q, (q+1)*Q) over coalesced reads of the target-major
// row TT[s][.] (L2-resident across frames), thread 0 folds the NW (value,
// index) results in source order, so ties still resolve to the first maximal
// source and a NaN at s' = 0 (wave 0's range) still sticks.  NW = 4 measured
// best at S = 1092 (125 ms per 20000 frames vs 188 ms with one wave per
// target; 2 / 8 / 16 waves: 140 / 171 / 303 ms).
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_vt_frame4(const double *__restrict__ TT, long ldt,
                                                   const double *__restrict__ cum_prev,
                                                   double *__restrict__ cum_next,
                                                   const double *__restrict__ logd_n,
                                                   int *__restrict__ ante_n, int S) {
  __shared__ double s_v[NW];
  __shared__ int s_i[NW];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int s = blockIdx.x;
  const int Q = (S + NW - 1) / NW;
  const int lo = q * Q, hi = min(S, lo + Q);
  const double *row = TT + (size_t)s * ldt;
  double bv = -INFINITY;
  int bi = INT_MAX;
  for (int base = lo; base < hi; base += 64 * kVtBatch) {
    double v[kVtBatch];
#pragma unroll
    for (int u = 0; u < kVtBatch; ++u) {
      const int sp = base + u * 64 + lane;
      v[u] = sp < hi ? cum_prev[sp] + row[sp] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < kVtBatch; ++u) {
      const int sp = base + u * 64 + lane;
      if (sp < hi) vt_better(bv, bi, v[u], sp);
    }
  }
  vt_wave_reduce(bv, bi);
  if (q == 0) {
    const double v0 = cum_prev[0] + row[0];
    if (v0 != v0) {  // NaN at s' = 0: nothing compares greater (pyx :77)
      bv = v0;
      bi = 0;
    }
  }
  if (lane == 0) {
    s_v[q] = bv;
    s_i[q] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = s_v[0];
    int i = s_i[0];
    for (int w = 1; w < NW; ++w) vt_better(v, i, s_v[w], s_i[w]);
    cum_next[s] = v + logd_n[s];   // pyx :83-85
    ante_n[s] = i;
  }
}

// all frames in one workgroup: TT [S][S] and cum [2][Sp] in LDS
__global__ __launch_bounds__(1024) void k_vt_block(const double *__restrict__ TT, long ldt,
                                                   const double *__restrict__ logdT, long ldd,
                                                   const double *__restrict__ prior, int S, int N,
                                                   int *__restrict__ ante, long lda,
                                                   double *__restrict__ cum_last) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int Sp = (S + 1) & ~1;
  double *tt = sm;                      // [S][S]
  double *cum = sm + (size_t)S * S;     // [2][Sp]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = threadIdx.x; i < S * S; i += blockDim.x) {
    const int r = i / S, c = i - r * S;
    tt[i] = TT[(size_t)r * ldt + c];
  }
  for (int s = threadIdx.x; s < S; s += blockDim.x) cum[s] = prior[s] + logdT[s];
  __syncthreads();
  for (int n = 1; n < N; ++n) {
    const double *cp = cum + ((n - 1) & 1) * Sp;
    double *cn = cum + (n & 1) * Sp;
    const double *ld = logdT + (size_t)n * ldd;
    for (int s = wv; s < S; s += nw) {
      double bv;
      int bi;
      vt_argmax(cp, tt + (size_t)s * S, S, lane, bv, bi);
      if (lane == 0) {
        cn[s] = bv + ld[s];
        ante[(size_t)n * lda + s] = bi;
      }
    }
    __syncthreads();
  }
  const double *cl = cum + ((N - 1) & 1) * Sp;
  for (int s = threadIdx.x; s < S; s += blockDim.x) cum_last[s] = cl[s];
}

// Backtracking (pyx :87-92) in three passes over chunks of kVtChunk frames
// instead of one chain of N dependent loads:
//   k_vt_jump   for every chunk c and every state s at its last frame hi_c,
//               the state at its first frame lo_c (ante composed over the chunk)
//   k_vt_chain  numpy.argmax of cum[:, N-1] (first maximum, the first NaN if
//               any), then one jump per chunk from the last chunk to the first
//   k_vt_fill   every chunk expands its own piece of the path
constexpr int kVtChunk = 128;

__global__ void k_vt_jump(const int *__restrict__ ante, long lda, int S, int N,
                          int *__restrict__ jump) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
  if (s >= S) return;
  const int lo = c * kVtChunk, hi = min(N, lo + kVtChunk) - 1;
  int idx = s;
  for (int n = hi; n > lo; --n) idx = ante[(size_t)n * lda + idx];
  jump[(size_t)c * S + s] = idx;
}

__global__ void k_vt_chain(const double *__restrict__ cum_last, const int *__restrict__ ante,
                           long lda, const int *__restrict__ jump, int S, int N,
                           int *__restrict__ hi_state) {
  if (threadIdx.x != 0) return;
  int idx = 0;
  double mx = cum_last[0];
  if (mx == mx) {
    for (int s = 1; s < S; ++s) {
      const double c = cum_last[s];
      if (c != c) {
        idx = s;
        break;
      }
      if (c > mx) {
        mx = c;
        idx = s;
      }
    }
  }
  const int nch = (N + kVtChunk - 1) / kVtChunk;
  for (int c = nch - 1; c >= 0; --c) {
    hi_state[c] = idx;                                  // state at frame hi_c
    const int lo_state = jump[(size_t)c * S + idx];     // state at frame lo_c
    if (c > 0) idx = ante[(size_t)(c * kVtChunk) * lda + lo_state];
  }
}

__global__ void k_vt_fill(const int *__restrict__ ante, long lda, const int *__restrict__ hi_state,
                          int N, long long *__restrict__ path) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= (N + kVtChunk - 1) / kVtChunk) return;
  const int lo = c * kVtChunk, hi = min(N, lo + kVtChunk) - 1;
  int idx = hi_state[c];
  path[hi] = idx;
  for (int n = hi; n > lo; --n) {
    idx = ante[(size_t)n * lda + idx];
    path[n - 1] = idx;
  }
}

// out[c][r] = in[r][c] for r < R, c < C (row pitches ldi, ldo)
__global__ __launch_bounds__(256) void k_vt_transpose(const double *__restrict__ in, long ldi,
                                                      double *__restrict__ out, long ldo, int R,
                                                      int C) {
  __shared__ double t[16][17];
  const int c0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  if (r0 + ty < R && c0 + tx < C) t[ty][tx] = in[(size_t)(r0 + ty) * ldi + c0 + tx];
  __syncthreads();
  if (c0 + ty < C && r0 + tx < R) out[(size_t)(c0 + ty) * ldo + r0 + tx] = t[tx][ty];
}

static float g_vt_ms = 0.f;
static int g_vt_kind = -1;

}  // namespace fasst

using namespace fasst;

extern "C" {

int viterbi_tracking(int device, int n_states, int n_frames, const double *log_density,
                     long ld_density, const double *log_prior, const double *log_transition,
                     long ld_transition, long long *path) {
  const int S = n_states, N = n_frames;
  if (S < 1 || N < 1 || !log_density || !log_prior || !log_transition || !path ||
      ld_density < N || ld_transition < S) {
    set_error("viterbi_tracking: bad shape (S %d, N %d, ld %ld / %ld)", S, N, ld_density,
              ld_transition);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  const long Sp = round_up(S, 16);
  int st;
  DBuf<double> dD, dDT, dT, dTT, dprior, cum, clast;
  DBuf<int> ante, jump, hi_state;
  const int nch = (N + kVtChunk - 1) / kVtChunk;
  DBuf<long long> dpath;
  if ((st = dD.alloc((size_t)S * N)) || (st = dDT.alloc((size_t)N * Sp)) ||
      (st = dT.alloc((size_t)S * S)) || (st = dTT.alloc((size_t)S * Sp)) ||
      (st = dprior.alloc(S)) || (st = cum.alloc(2 * Sp)) || (st = clast.alloc(Sp)) ||
      (st = ante.alloc((size_t)N * Sp)) || (st = dpath.alloc(N)) ||
      (st = jump.alloc((size_t)nch * S)) || (st = hi_state.alloc(nch)))
    return st;
  FASST_HIP(hipMemcpy2D(dD.p, (size_t)N * sizeof(double), log_density,
                        (size_t)ld_density * sizeof(double), (size_t)N * sizeof(double), S,
                        hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy2D(dT.p, (size_t)S * sizeof(double), log_transition,
                        (size_t)ld_transition * sizeof(double), (size_t)S * sizeof(double), S,
                        hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dprior.p, log_prior, S * sizeof(double), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  FASST_HIP(hipEventCreate(&e0));
  FASST_HIP(hipEventCreate(&e1));
  FASST_HIP(hipEventRecord(e0, 0));
  // frame-major densities [N][Sp], target-major transitions TT[s][s'] = T[s'][s]
  k_vt_transpose<<<dim3((N + 15) / 16, (S + 15) / 16), 256>>>(dD.p, N, dDT.p, Sp, S, N);
  FASST_LAUNCH_CHECK();
  k_vt_transpose<<<dim3((S + 15) / 16, (S + 15) / 16), 256>>>(dT.p, S, dTT.p, Sp, S, S);
  FASST_LAUNCH_CHECK();
  const size_t lds = ((size_t)S * S + 2 * (size_t)((S + 1) & ~1)) * sizeof(double);
  if (lds <= kVtLdsBudget) {
    g_vt_kind = 0;
    if (lds > 64 * 1024)
      FASST_HIP(hipFuncSetAttribute((const void *)k_vt_block,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_vt_block<<<1, 1024, lds>>>(dTT.p, Sp, dDT.p, Sp, dprior.p, S, N, ante.p, Sp, clast.p);
    FASST_LAUNCH_CHECK();
  } else {
    g_vt_kind = 1;
    k_vt_init<<<(S + 255) / 256, 256>>>(dprior.p, dDT.p, cum.p, S);
    FASST_LAUNCH_CHECK();
    for (int n = 1; n < N; ++n) {
      const double *cp = cum.p + ((n - 1) & 1) * Sp;
      double *cn = cum.p + (n & 1) * Sp;
      k_vt_frame4<4><<<S, 256>>>(dTT.p, Sp, cp, cn, dDT.p + (size_t)n * Sp,
                                 ante.p + (size_t)n * Sp, S);
    }
    FASST_LAUNCH_CHECK();
    FASST_HIP(hipMemcpyAsync(clast.p, cum.p + ((N - 1) & 1) * Sp, S * sizeof(double),
                             hipMemcpyDeviceToDevice, 0));
  }
  k_vt_jump<<<dim3((S + 255) / 256, nch), 256>>>(ante.p, Sp, S, N, jump.p);
  FASST_LAUNCH_CHECK();
  k_vt_chain<<<1, 64>>>(clast.p, ante.p, Sp, jump.p, S, N, hi_state.p);
  FASST_LAUNCH_CHECK();
  k_vt_fill<<<(nch + 63) / 64, 64>>>(ante.p, Sp, hi_state.p, N, dpath.p);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipEventRecord(e1, 0));
  FASST_HIP(hipEventSynchronize(e1));
  FASST_HIP(hipEventElapsedTime(&g_vt_ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  FASST_HIP(hipMemcpy(path, dpath.p, (size_t)N * sizeof(long long), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int viterbi_last_timing(double *device_ms, int *path_kind) {
  if (device_ms) *device_ms = g_vt_ms;
  if (path_kind) *path_kind = g_vt_kind;
  return FASST_OK;
}

}  // extern "C"
