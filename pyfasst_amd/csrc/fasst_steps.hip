// The FASST GEM step methods as device calls (the class surface a script uses
// to drive a GEM iteration piecewise or to inspect its intermediates):
//
//   retrieve_subsrc_params  (audioModel.py:514-578)  fasst_source_powers
//   compute_suff_stat       (:580-764)               fasst_suff_stat
//   update_mix_matrix       (:766-889)               fasst_mix_solve
//   update_spectral_components (:1469-1978)          fasst_spectral_update (fasst_em.hip)
//   compute_sigma_comp_2d   (:1327-1372)             fasst_sigma_comp
//   compute_inv_sigma_mix_2d (:1374-1394)            fasst_inv_sigma_mix
//   compute_Wiener_gain_2d  (:1396-1467)             fasst_wiener_gain
//
// These take and return the reference's own arrays (per-rank powers
// [R][F][T], hat_Rss [F][R][R], ...), so they materialise what the fused GEM
// iteration (fasst_run) never stores; they are for scripts, not for the EM
// loop.  compute_suff_stat runs on arbitrary per-rank powers with the same
// algebra as the fused E-step (S = Sigma_x^-1, N = S Cx S - S, P = Cx S; the
// R x R pair loop becomes per-bin t-reductions of V_r1 V_r2 N and V_r P).
#include "fasst_ctx.h"

#include <cmath>
#include <vector>

namespace fasst {

__device__ __forceinline__ double2 c_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 c_mul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 c_conj(double2 a) { return make_double2(a.x, -a.y); }

// V[j][f][t] = sum_k W[j][k][f] H[j][k][t] (W = FB.FW in Wkf, H in TW's rows;
// (m0, m1): the columns of spectral components to include, bit k of word
// k / 64 -- KP reaches 128)
__device__ __forceinline__ bool col_in(unsigned long long m0, unsigned long long m1, int k) {
  return ((k < 64 ? m0 >> k : m1 >> (k - 64)) & 1ull) != 0;
}
__global__ void k_source_powers(const double *__restrict__ Wkf, const double *__restrict__ TW,
                                double *__restrict__ V, int F, int T, int Fp, int Tp, int KP,
                                int j0, unsigned long long m0, unsigned long long m1) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y, jj = blockIdx.z, j = j0 + jj;
  if (t >= T) return;
  double s = 0.0;
  for (int k = 0; k < KP; ++k)
    if (col_in(m0, m1, k)) s += Wkf[((size_t)j * KP + k) * Fp + f] * TW[((size_t)j * KP + k) * Tp + t];
  V[((size_t)jj * F + f) * T + t] = s;
}

// compute_suff_stat, one block per bin f: tiles of 256 frames; each thread
// forms its point (Sigma_x, the guarded inverse, loglik term, P, N, hat_Ws),
// then the block reduces the tile into the per-bin statistics
//   pair  PS[p][c] = sum_t V_r1 V_r2 N_c   (p = (r1 <= r2), c: n00 n11 n01r n01i)
//   cross CS[r][c] = sum_t V_r P_c          (c: P00 P01 P10 P11, re / im)
//   sV[r] = sum_t V_r
// and hat_Rss / hat_Rxs follow per bin (see the header of fasst_em.hip).
constexpr int kSsTile = 256;
constexpr int kSsMaxOut = 4 * (kStepMaxR * (kStepMaxR + 1) / 2) + 8 * kStepMaxR + kStepMaxR;
struct SSArgs {
  const double *cx00, *cx11, *cxr, *cxi;  // [Tp][Fp]
  const double *V;                        // [R][F][T]
  const double2 *mix;                     // [R][2][F]
  const double *psd;                      // [F]
  double2 *rss, *rxs;                     // [F][R][R], [F][2][R]
  double2 *rxx;                           // [3][F]
  double *ws;                             // [R][F][T]
  double *llb;                            // [F]
  int F, T, Fp, R;
};

__global__ __launch_bounds__(kSsTile) void k_suff_stat(const SSArgs a) {
  const int f = blockIdx.x, tid = threadIdx.x, R = a.R;
  const int NPAIR = R * (R + 1) / 2, NOUT = 4 * NPAIR + 8 * R + R;
  __shared__ double2 s_a[kStepMaxR][2];
  __shared__ double s_c[kStepMaxR][4];
  __shared__ double s_v[kStepMaxR][kSsTile];
  __shared__ double s_np[12][kSsTile];   // N (4) then P (8)
  __shared__ double s_out[kSsMaxOut];
  __shared__ double s_red[kSsTile];
  __shared__ unsigned char s_p1[kSsMaxOut], s_p2[kSsMaxOut];
  __shared__ double2 s_m[kStepMaxR * kStepMaxR];
  if (tid < R) {
    const double2 a0 = a.mix[((size_t)tid * 2 + 0) * a.F + f], a1 = a.mix[((size_t)tid * 2 + 1) * a.F + f];
    s_a[tid][0] = a0;
    s_a[tid][1] = a1;
    s_c[tid][0] = a0.x * a0.x + a0.y * a0.y;
    s_c[tid][1] = a1.x * a1.x + a1.y * a1.y;
    s_c[tid][2] = a0.x * a1.x + a0.y * a1.y;   // Re a0 conj(a1)
    s_c[tid][3] = a0.y * a1.x - a0.x * a1.y;   // Im a0 conj(a1)
  }
  // output o -> the (rank, rank) pair or rank it reduces
  for (int o = tid; o < NOUT; o += kSsTile) {
    int r1 = 0, r2 = 0;
    if (o < 4 * NPAIR) {
      int p = o / 4;
      while (p >= R - r1) {
        p -= R - r1;
        ++r1;
      }
      r2 = r1 + p;
    } else if (o < 4 * NPAIR + 8 * R) {
      r1 = (o - 4 * NPAIR) / 8;
    } else {
      r1 = o - 4 * NPAIR - 8 * R;
    }
    s_p1[o] = (unsigned char)r1;
    s_p2[o] = (unsigned char)r2;
  }
  __syncthreads();
  const double psd = a.psd[f];
  double acc[(kSsMaxOut + kSsTile - 1) / kSsTile];
#pragma unroll
  for (int u = 0; u < (kSsMaxOut + kSsTile - 1) / kSsTile; ++u) acc[u] = 0.0;
  double ll = 0.0, x0s = 0.0, x1s = 0.0, xrs = 0.0, xis = 0.0;
  for (int t0 = 0; t0 < a.T; t0 += kSsTile) {
    const int t = t0 + tid, n = min(kSsTile, a.T - t0);
    if (t < a.T) {
      const size_t ci = (size_t)t * a.Fp + f;
      const double x00 = a.cx00[ci], x11 = a.cx11[ci], xr = a.cxr[ci], xi = a.cxi[ci];
      x0s += x00;
      x1s += x11;
      xrs += xr;
      xis += xi;
      double d0 = psd, d1 = psd, ore = 0.0, oim = 0.0;
      for (int r = 0; r < R; ++r) {
        const double v = a.V[((size_t)r * a.F + f) * a.T + t];
        s_v[r][tid] = v;
        d0 += s_c[r][0] * v;
        d1 += s_c[r][1] * v;
        ore += s_c[r][2] * v;
        oim += s_c[r][3] * v;
      }
      // inv_herm_mat_2d (tools/signalTools.py:177-194)
      double det = d0 * d1 - (ore * ore + oim * oim);
      const double dg = det + kEps;
      det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
      const double i0 = d1 / det, i1 = d0 / det, ior = -ore / det, ioi = -oim / det;
      ll += log(det * M_PI) + i0 * x00 + i1 * x11 + 2.0 * (ior * xr + ioi * xi);
      const double p00r = x00 * i0 + xr * ior + xi * ioi, p00i = xi * ior - xr * ioi;
      const double p01r = x00 * ior + xr * i1, p01i = x00 * ioi + xi * i1;
      const double p10r = xr * i0 + x11 * ior, p10i = -xi * i0 - x11 * ioi;
      const double p11r = xr * ior + xi * ioi + x11 * i1, p11i = xr * ioi - xi * ior;
      const double n00 = p00r * i0 + (p10r * ior - p10i * ioi) - i0;
      const double n11 = (p01r * ior + p01i * ioi) + p11r * i1 - i1;
      const double n01r = p00r * ior + p00i * ioi + p10r * i1 - ior;
      const double n01i = p00r * ioi - p00i * ior - p10i * i1 - ioi;
      s_np[0][tid] = n00;
      s_np[1][tid] = n11;
      s_np[2][tid] = n01r;
      s_np[3][tid] = n01i;
      s_np[4][tid] = p00r;
      s_np[5][tid] = p00i;
      s_np[6][tid] = p01r;
      s_np[7][tid] = p01i;
      s_np[8][tid] = p10r;
      s_np[9][tid] = p10i;
      s_np[10][tid] = p11r;
      s_np[11][tid] = p11i;
      // hat_Ws[r] = |Re(V_r^2 a_r^H N a_r + V_r)|   (:727-729)
      for (int r = 0; r < R; ++r) {
        const double v = s_v[r][tid];
        const double q = s_c[r][0] * n00 + s_c[r][1] * n11 + 2.0 * (s_c[r][2] * n01r + s_c[r][3] * n01i);
        a.ws[((size_t)r * a.F + f) * a.T + t] = fabs(v * v * q + v);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < (kSsMaxOut + kSsTile - 1) / kSsTile; ++u) {
      const int o = tid + u * kSsTile;
      if (o >= NOUT) break;
      const int r1 = s_p1[o], r2 = s_p2[o];
      double s = 0.0;
      if (o < 4 * NPAIR) {
        const double *n_ = s_np[o & 3];
        for (int q = 0; q < n; ++q) s += s_v[r1][q] * s_v[r2][q] * n_[q];
      } else if (o < 4 * NPAIR + 8 * R) {
        const double *p_ = s_np[4 + (o - 4 * NPAIR) % 8];
        for (int q = 0; q < n; ++q) s += s_v[r1][q] * p_[q];
      } else {
        for (int q = 0; q < n; ++q) s += s_v[r1][q];
      }
      acc[u] += s;
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < (kSsMaxOut + kSsTile - 1) / kSsTile; ++u) {
    const int o = tid + u * kSsTile;
    if (o < NOUT) s_out[o] = acc[u];
  }
  // block sums in index order: loglik, then the four Cx planes
  double *sums[5] = {&ll, &x0s, &x1s, &xrs, &xis};
  double tot[5];
  for (int q = 0; q < 5; ++q) {
    s_red[tid] = *sums[q];
    __syncthreads();
    for (int w = kSsTile / 2; w > 0; w >>= 1) {
      if (tid < w) s_red[tid] += s_red[tid + w];
      __syncthreads();
    }
    tot[q] = s_red[0];
    __syncthreads();
  }
  const double invT = 1.0 / (double)a.T;
  if (tid == 0) {
    a.llb[f] = tot[0];
    a.rxx[0 * (size_t)a.F + f] = make_double2(tot[1] * invT, 0.0);
    a.rxx[1 * (size_t)a.F + f] = make_double2(tot[3] * invT, tot[4] * invT);
    a.rxx[2 * (size_t)a.F + f] = make_double2(tot[2] * invT, 0.0);
  }
  // hat_Rss[f][r1][r2] = a_r1^H M a_r2 / T + d_r1r2 mean_t V_r1, hermitised
  for (int e = tid; e < R * R; e += kSsTile) {
    const int r1 = e / R, r2 = e % R;
    auto entry = [&](int u1, int u2) {
      const int lo = min(u1, u2), hi = max(u1, u2);
      const int p = lo * R - lo * (lo - 1) / 2 + (hi - lo);
      const double m00 = s_out[4 * p], m11 = s_out[4 * p + 1];
      const double2 m01 = make_double2(s_out[4 * p + 2], s_out[4 * p + 3]);
      const double2 a0 = s_a[u1][0], a1 = s_a[u1][1], b0 = s_a[u2][0], b1 = s_a[u2][1];
      // conj(a0) (m00 b0 + m01 b1) + conj(a1) (conj(m01) b0 + m11 b1)
      double2 r0 = c_add(make_double2(m00 * b0.x, m00 * b0.y), c_mul(m01, b1));
      double2 rr = c_add(c_mul(c_conj(m01), b0), make_double2(m11 * b1.x, m11 * b1.y));
      double2 v = c_add(c_mul(c_conj(a0), r0), c_mul(c_conj(a1), rr));
      v.x *= invT;
      v.y *= invT;
      if (u1 == u2) v.x += s_out[4 * NPAIR + 8 * R + u1] * invT;
      return v;
    };
    s_m[e] = entry(r1, r2);
  }
  __syncthreads();
  // (each entry formed once, then averaged with its transpose: exactly Hermitian)
  for (int e = tid; e < R * R; e += kSsTile) {
    const int r1 = e / R, r2 = e % R;
    const double2 x = s_m[e], y = s_m[r2 * R + r1];
    a.rss[((size_t)f * R + r1) * R + r2] = make_double2((x.x + y.x) / 2.0, (x.y - y.y) / 2.0);
  }
  // hat_Rxs[f][c][r] = sum_c' (sum_t V_r P)[c][c'] a_r[c'] / T
  for (int e = tid; e < 2 * R; e += kSsTile) {
    const int c = e / R, r = e % R;
    const double *q = s_out + 4 * NPAIR + 8 * r;
    const double2 pc0 = make_double2(q[4 * c + 0], q[4 * c + 1]);   // P[c][0]
    const double2 pc1 = make_double2(q[4 * c + 2], q[4 * c + 3]);   // P[c][1]
    double2 v = c_add(c_mul(pc0, s_a[r][0]), c_mul(pc1, s_a[r][1]));
    a.rxs[((size_t)f * 2 + c) * R + r] = make_double2(v.x * invT, v.y * invT);
  }
}

// loglik = -(sum_f llb[f]) / (F T), summed in bin order
__global__ void k_ss_loglik(const double *__restrict__ llb, int F, double inv_ft, double *out) {
  __shared__ double s[256];
  double x = 0.0;
  for (int f = threadIdx.x; f < F; f += 256) x += llb[f];
  s[threadIdx.x] = x;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = -s[0] * inv_ft;
}

// update_mix_matrix, 'inst' rows (:808-839): b[u][c] = mean_f Re(hat_Rxs[f][c][u]
// - sum_o mix[o][c][f] hat_Rss[f][o][u]), m[u1][u2] = mean_f Re hat_Rss[f][u1][u2],
// x = solve(m^T, b^T) (partial pivoting); mix[u][c][f] = x[u][c] for every f
__global__ void k_mix_solve_inst(const double2 *__restrict__ rss, const double2 *__restrict__ rxs,
                                 double2 *__restrict__ mix, int F, int R, const int *__restrict__ kind,
                                 int *singular) {
  __shared__ double s_b[kStepMaxR][2], s_m[kStepMaxR][kStepMaxR];
  __shared__ int s_u[kStepMaxR], s_o[kStepMaxR], s_nu, s_no, s_sing;
  __shared__ double s_x[kStepMaxR][2];
  const int tid = threadIdx.x;
  if (tid == 0) {
    int nu = 0, no = 0;
    for (int r = 0; r < R; ++r) {
      if (kind[r] == 1) s_u[nu++] = r;
      else s_o[no++] = r;
    }
    s_nu = nu;
    s_no = no;
    s_sing = 0;
  }
  __syncthreads();
  const int nu = s_nu, no = s_no;
  if (nu == 0) return;
  if (tid < 2 * nu + nu * nu) {
    double s = 0.0;
    if (tid < 2 * nu) {
      const int c = tid / nu, u = s_u[tid % nu];
      for (int f = 0; f < F; ++f) {
        double2 x = rxs[((size_t)f * 2 + c) * R + u];
        for (int i = 0; i < no; ++i) {
          const int o = s_o[i];
          const double2 t = c_mul(mix[((size_t)o * 2 + c) * F + f], rss[((size_t)f * R + o) * R + u]);
          x.x -= t.x;
          x.y -= t.y;
        }
        s += x.x;
      }
      s_b[tid % nu][c] = s / F;
    } else {
      const int e = tid - 2 * nu, u1 = e / nu, u2 = e % nu;
      for (int f = 0; f < F; ++f) s += rss[((size_t)f * R + s_u[u1]) * R + s_u[u2]].x;
      s_m[u1][u2] = s / F;
    }
  }
  __syncthreads();
  if (tid == 0) {
    double L[kStepMaxR][kStepMaxR], B[kStepMaxR][2];
    for (int i = 0; i < nu; ++i) {
      for (int k = 0; k < nu; ++k) L[i][k] = s_m[k][i];   // m^T
      B[i][0] = s_b[i][0];
      B[i][1] = s_b[i][1];
    }
    bool sing = false;
    for (int k = 0; k < nu && !sing; ++k) {
      int piv = k;
      for (int i = k + 1; i < nu; ++i)
        if (fabs(L[i][k]) > fabs(L[piv][k])) piv = i;
      if (L[piv][k] == 0.0) {
        sing = true;
        break;
      }
      if (piv != k) {
        for (int c = 0; c < nu; ++c) {
          const double t = L[k][c];
          L[k][c] = L[piv][c];
          L[piv][c] = t;
        }
        for (int c = 0; c < 2; ++c) {
          const double t = B[k][c];
          B[k][c] = B[piv][c];
          B[piv][c] = t;
        }
      }
      for (int i = k + 1; i < nu; ++i) {
        const double m = L[i][k] / L[k][k];
        for (int c = k; c < nu; ++c) L[i][c] -= m * L[k][c];
        for (int c = 0; c < 2; ++c) B[i][c] -= m * B[k][c];
      }
    }
    if (sing) {
      s_sing = 1;
      *singular = 1;
    } else {
      for (int k = nu - 1; k >= 0; --k)
        for (int c = 0; c < 2; ++c) {
          double s = B[k][c];
          for (int i = k + 1; i < nu; ++i) s -= L[k][i] * s_x[i][c];
          s_x[k][c] = s / L[k][k];
        }
    }
  }
  __syncthreads();
  if (s_sing) return;
  for (int e = tid; e < nu * 2 * F; e += blockDim.x) {
    const int u = e / (2 * F), c = (e / F) % 2, f = e % F;
    mix[((size_t)s_u[u] * 2 + c) * F + f] = make_double2(s_x[u][c], 0.0);
  }
}

// update_mix_matrix, 'conv' rows (:844-863), every component free 'conv':
// mix[:, :, f] = solve(hat_Rss[f]^T, hat_Rxs[f]^T), LU with partial
// pivoting on |re| + |im| (LAPACK zgesv's izamax), one thread per bin
__global__ void k_mix_solve_conv(const double2 *__restrict__ rss, const double2 *__restrict__ rxs,
                                 double2 *__restrict__ mix, int F, int R, int *singular) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  double2 L[kStepMaxR][kStepMaxR], B[kStepMaxR][2];
  for (int i = 0; i < R; ++i) {
    for (int k = 0; k < R; ++k) L[i][k] = rss[((size_t)f * R + k) * R + i];   // hat_Rss[f]^T
    for (int c = 0; c < 2; ++c) B[i][c] = rxs[((size_t)f * 2 + c) * R + i];  // hat_Rxs[f]^T
  }
  auto cabs1 = [](double2 z) { return fabs(z.x) + fabs(z.y); };
  for (int k = 0; k < R; ++k) {
    int piv = k;
    for (int i = k + 1; i < R; ++i)
      if (cabs1(L[i][k]) > cabs1(L[piv][k])) piv = i;
    if (L[piv][k].x == 0.0 && L[piv][k].y == 0.0) {
      atomicOr(singular, 1);
      return;
    }
    if (piv != k) {
      for (int c = 0; c < R; ++c) {
        const double2 t = L[k][c];
        L[k][c] = L[piv][c];
        L[piv][c] = t;
      }
      for (int c = 0; c < 2; ++c) {
        const double2 t = B[k][c];
        B[k][c] = B[piv][c];
        B[piv][c] = t;
      }
    }
    const double2 d = L[k][k];
    const double dn = d.x * d.x + d.y * d.y;
    const double2 rinv = make_double2(d.x / dn, -d.y / dn);
    for (int i = k + 1; i < R; ++i) {
      const double2 m = c_mul(L[i][k], rinv);
      for (int c = k + 1; c < R; ++c) {
        const double2 t = c_mul(m, L[k][c]);
        L[i][c].x -= t.x;
        L[i][c].y -= t.y;
      }
      for (int c = 0; c < 2; ++c) {
        const double2 t = c_mul(m, B[k][c]);
        B[i][c].x -= t.x;
        B[i][c].y -= t.y;
      }
    }
  }
  for (int k = R - 1; k >= 0; --k) {
    const double2 d = L[k][k];
    const double dn = d.x * d.x + d.y * d.y;
    for (int c = 0; c < 2; ++c) {
      double2 s = B[k][c];
      for (int i = k + 1; i < R; ++i) {
        const double2 t = c_mul(L[k][i], B[i][c]);
        s.x -= t.x;
        s.y -= t.y;
      }
      B[k][c] = make_double2((s.x * d.x + s.y * d.y) / dn, (s.y * d.x - s.x * d.y) / dn);
    }
  }
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < 2; ++c) mix[((size_t)r * 2 + c) * F + f] = B[r][c];
}

// compute_sigma_comp_2d: diag[c][f][t] = R_cc(f) V, off[f][t] = R_01(f) V with
// R = sum_rank a a^H of spatial component j (mixing rows roff[j]..)
__global__ void k_sigma_comp(const double *__restrict__ Wkf, const double *__restrict__ TW,
                             const double2 *__restrict__ A, double *__restrict__ diag,
                             double2 *__restrict__ off, int F, int T, int Fp, int Tp, int KP, int j,
                             int r0, int r1, unsigned long long m0, unsigned long long m1) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y;
  if (t >= T) return;
  double v = 0.0;
  for (int k = 0; k < KP; ++k)
    if (col_in(m0, m1, k)) v += Wkf[((size_t)j * KP + k) * Fp + f] * TW[((size_t)j * KP + k) * Tp + t];
  double c0 = 0.0, c1 = 0.0;
  double2 co = make_double2(0.0, 0.0);
  for (int r = r0; r < r1; ++r) {
    const double2 a0 = A[(size_t)(2 * r) * Fp + f], a1 = A[(size_t)(2 * r + 1) * Fp + f];
    c0 += a0.x * a0.x + a0.y * a0.y;
    c1 += a1.x * a1.x + a1.y * a1.y;
    co = c_add(co, c_mul(a0, c_conj(a1)));
  }
  const size_t i = (size_t)f * T + t;
  diag[i] = c0 * v;
  diag[(size_t)F * T + i] = c1 * v;
  off[i] = make_double2(co.x * v, co.y * v);
}

// compute_inv_sigma_mix_2d: Sigma_x = sum_n Sigma_n + PSD I, inverted with
// inv_herm_mat_2d's guard
__global__ void k_inv_sigma_mix(const double *__restrict__ diag, const double2 *__restrict__ off,
                                const double *__restrict__ psd, double *__restrict__ idiag,
                                double2 *__restrict__ ioff, int n, int F, int T) {
  const size_t FT = (size_t)F * T;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < FT; i += (size_t)gridDim.x * blockDim.x) {
    double d0 = 0.0, d1 = 0.0;
    double2 o = make_double2(0.0, 0.0);
    for (int c = 0; c < n; ++c) {
      d0 += diag[((size_t)c * 2 + 0) * FT + i];
      d1 += diag[((size_t)c * 2 + 1) * FT + i];
      o = c_add(o, off[(size_t)c * FT + i]);
    }
    const double p = psd[i / T];
    d0 += p;
    d1 += p;
    double det = d0 * d1 - (o.x * o.x + o.y * o.y);
    const double dg = det + kEps;
    det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
    idiag[i] = d1 / det;
    idiag[FT + i] = d0 / det;
    ioff[i] = make_double2(-o.x / det, -o.y / det);
  }
}

// compute_Wiener_gain_2d (:1447-1465)
__global__ void k_wiener_gain(const double *__restrict__ sd, const double2 *__restrict__ so,
                              const double *__restrict__ isd, const double2 *__restrict__ iso,
                              double2 *__restrict__ WG, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double s0 = sd[i], s1 = sd[n + i], i0 = isd[i], i1 = isd[n + i];
    const double2 o = so[i], io = iso[i];
    const double2 w00 = c_mul(o, c_conj(io));
    WG[i] = make_double2(w00.x + s0 * i0, w00.y);
    WG[3 * n + i] = make_double2(w00.x + s1 * i1, -w00.y);
    const double2 w01 = c_add(make_double2(s0 * io.x, s0 * io.y), make_double2(o.x * i1, o.y * i1));
    WG[n + i] = w01;
    const double2 ic = c_conj(io);
    const double2 w10 = c_add(make_double2(o.x * i0, -o.y * i0), make_double2(s1 * ic.x, s1 * ic.y));
    WG[2 * n + i] = w10;
  }
}

static int grid_of(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 16384); }

}  // namespace fasst

using namespace fasst;

extern "C" {

int fasst_source_powers(fasst_ctx *c, int j0, int nj, const unsigned long long *colmask, double *V) {
  if (!c || !c->configured || !V || j0 < 0 || nj < 1 || j0 + nj > c->J) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  int st = launch_w_old(c);
  if (st) return st;
  DBuf<double> dV;
  if ((st = dV.alloc_uninit((size_t)c->F * c->T))) return st;
  for (int jj = 0; jj < nj; ++jj) {
    const unsigned long long m0 = colmask ? colmask[2 * jj] : ~0ull;
    const unsigned long long m1 = colmask ? colmask[2 * jj + 1] : ~0ull;
    k_source_powers<<<dim3((c->T + 255) / 256, c->F, 1), 256, 0, c->stream>>>(
        c->Wkf.p, c->TW.p, dV.p, c->F, c->T, c->Fp, c->Tp, c->KP, j0 + jj, m0, m1);
    FASST_LAUNCH_CHECK();
    FASST_HIP(hipMemcpyAsync(V + (size_t)jj * c->F * c->T, dV.p, (size_t)c->F * c->T * sizeof(double),
                             hipMemcpyDeviceToHost, c->stream));
  }
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_suff_stat(fasst_ctx *c, int R, const double *V, const double *mix, const double *psd,
                    double *rxx, double *rxs, double *rss, double *ws, double *loglik) {
  if (!c || R < 1 || !V || !mix || !psd || !rxx || !rxs || !rss || !ws || !loglik) {
    set_error("fasst_suff_stat: bad arguments (R %d <= %d)", R, kStepMaxR);
    return FASST_ERR_SHAPE;
  }
  if (R > kStepMaxR) {
    set_error("fasst_suff_stat: total rank %d above the step call's %d", R, kStepMaxR);
    return FASST_ERR_UNSUPPORTED;
  }
  if (!c->cx_ready || !c->cx.p || c->F < 1 || c->T < 1) {
    set_error("fasst_suff_stat: no observation resident (upload Cx first)");
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(c->device);
  const size_t FT = (size_t)c->F * c->T;
  DBuf<double> dV, dws, dpsd, dllb, dll;
  DBuf<double2> dmix, drss, drxs, drxx;
  int st;
  if ((st = dV.alloc_uninit((size_t)R * FT)) || (st = dws.alloc_uninit((size_t)R * FT)) ||
      (st = dpsd.alloc_uninit(c->F)) || (st = dllb.alloc_uninit(c->F)) || (st = dll.alloc_uninit(1)) ||
      (st = dmix.alloc_uninit((size_t)R * 2 * c->F)) || (st = drss.alloc_uninit((size_t)c->F * R * R)) ||
      (st = drxs.alloc_uninit((size_t)c->F * 2 * R)) || (st = drxx.alloc_uninit((size_t)3 * c->F)))
    return st;
  FASST_HIP(hipMemcpyAsync(dV.p, V, (size_t)R * FT * sizeof(double), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpyAsync(dmix.p, mix, (size_t)R * 2 * c->F * sizeof(double2), hipMemcpyHostToDevice,
                           c->stream));
  FASST_HIP(hipMemcpyAsync(dpsd.p, psd, c->F * sizeof(double), hipMemcpyHostToDevice, c->stream));
  SSArgs a;
  a.cx00 = c->cx.p;
  a.cx11 = c->cx.p + (size_t)c->Tp * c->Fp;
  a.cxr = c->cx.p + 2 * (size_t)c->Tp * c->Fp;
  a.cxi = c->cx.p + 3 * (size_t)c->Tp * c->Fp;
  a.V = dV.p;
  a.mix = dmix.p;
  a.psd = dpsd.p;
  a.rss = drss.p;
  a.rxs = drxs.p;
  a.rxx = drxx.p;
  a.ws = dws.p;
  a.llb = dllb.p;
  a.F = c->F;
  a.T = c->T;
  a.Fp = c->Fp;
  a.R = R;
  k_suff_stat<<<c->F, kSsTile, 0, c->stream>>>(a);
  FASST_LAUNCH_CHECK();
  k_ss_loglik<<<1, 256, 0, c->stream>>>(dllb.p, c->F, 1.0 / ((double)c->F * (double)c->T), dll.p);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(rxx, drxx.p, 3 * c->F * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipMemcpyAsync(rxs, drxs.p, (size_t)c->F * 2 * R * sizeof(double2), hipMemcpyDeviceToHost,
                           c->stream));
  FASST_HIP(hipMemcpyAsync(rss, drss.p, (size_t)c->F * R * R * sizeof(double2), hipMemcpyDeviceToHost,
                           c->stream));
  FASST_HIP(hipMemcpyAsync(ws, dws.p, (size_t)R * FT * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipMemcpyAsync(loglik, dll.p, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_mix_solve(int device, int F, int R, const double *rss, const double *rxs, double *mix,
                    const int *kind) {
  if (F < 1 || R < 1 || !rss || !rxs || !mix || !kind) {
    set_error("fasst_mix_solve: bad arguments (R %d <= %d)", R, kStepMaxR);
    return FASST_ERR_SHAPE;
  }
  if (R > kStepMaxR) {
    set_error("fasst_mix_solve: total rank %d above the step call's %d", R, kStepMaxR);
    return FASST_ERR_UNSUPPORTED;
  }
  int nconv = 0;
  for (int r = 0; r < R; ++r) nconv += kind[r] == 2;
  if (nconv && nconv != R) {
    // np.linalg.solve(hat_Rss[f].T, hat_Rxs_bis[f].T) with fewer right-hand
    // side rows than hat_Rss rows (:856-857): numpy raises ValueError
    set_error("update_mix_matrix: a free 'conv' component next to other components: "
              "solve(%d x %d, %d x 2)", R, R, nconv);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(device);
  DBuf<double2> drss, drxs, dmix;
  DBuf<int> dkind, dsing;
  int st;
  if ((st = drss.alloc_uninit((size_t)F * R * R)) || (st = drxs.alloc_uninit((size_t)F * 2 * R)) ||
      (st = dmix.alloc_uninit((size_t)R * 2 * F)) || (st = dkind.alloc_uninit(R)) || (st = dsing.alloc(1)))
    return st;
  FASST_HIP(hipMemcpy(drss.p, rss, (size_t)F * R * R * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(drxs.p, rxs, (size_t)F * 2 * R * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dmix.p, mix, (size_t)R * 2 * F * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dkind.p, kind, R * sizeof(int), hipMemcpyHostToDevice));
  k_mix_solve_inst<<<1, 1024, 0, nullptr>>>(drss.p, drxs.p, dmix.p, F, R, dkind.p, dsing.p);
  FASST_LAUNCH_CHECK();
  if (nconv) {
    k_mix_solve_conv<<<(F + 63) / 64, 64, 0, nullptr>>>(drss.p, drxs.p, dmix.p, F, R, dsing.p);
    FASST_LAUNCH_CHECK();
  }
  int sing = 0;
  FASST_HIP(hipMemcpy(&sing, dsing.p, sizeof(int), hipMemcpyDeviceToHost));
  if (sing) {
    set_error("Singular Matrix");
    return FASST_ERR_SINGULAR;
  }
  FASST_HIP(hipMemcpy(mix, dmix.p, (size_t)R * 2 * F * sizeof(double2), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int fasst_sigma_comp(fasst_ctx *c, int j, const unsigned long long *colmask, double *diag,
                     double *off) {
  if (!c || !c->configured || j < 0 || j >= c->J || !colmask || !diag || !off) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  int st;
  if ((st = launch_w_old(c)) || (st = build_inst_A(c))) return st;
  const size_t FT = (size_t)c->F * c->T;
  DBuf<double> dd;
  DBuf<double2> doff;
  if ((st = dd.alloc_uninit(2 * FT)) || (st = doff.alloc_uninit(FT))) return st;
  k_sigma_comp<<<dim3((c->T + 255) / 256, c->F), 256, 0, c->stream>>>(
      c->Wkf.p, c->TW.p, c->A.p, dd.p, doff.p, c->F, c->T, c->Fp, c->Tp, c->KP, j, c->roff[j],
      c->roff[j + 1], colmask[0], colmask[1]);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpyAsync(diag, dd.p, 2 * FT * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipMemcpyAsync(off, doff.p, FT * sizeof(double2), hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_inv_sigma_mix(int device, int n, int F, int T, const double *diag, const double *off,
                        const double *psd, double *idiag, double *ioff) {
  if (n < 1 || F < 1 || T < 1 || !diag || !off || !psd || !idiag || !ioff) return FASST_ERR_SHAPE;
  DeviceGuard g(device);
  const size_t FT = (size_t)F * T;
  DBuf<double> dd, dpsd, did;
  DBuf<double2> doff, dio;
  int st;
  if ((st = dd.alloc_uninit((size_t)n * 2 * FT)) || (st = doff.alloc_uninit((size_t)n * FT)) ||
      (st = dpsd.alloc_uninit(F)) || (st = did.alloc_uninit(2 * FT)) || (st = dio.alloc_uninit(FT)))
    return st;
  FASST_HIP(hipMemcpy(dd.p, diag, (size_t)n * 2 * FT * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(doff.p, off, (size_t)n * FT * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dpsd.p, psd, F * sizeof(double), hipMemcpyHostToDevice));
  k_inv_sigma_mix<<<grid_of(FT), 256>>>(dd.p, doff.p, dpsd.p, did.p, dio.p, n, F, T);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpy(idiag, did.p, 2 * FT * sizeof(double), hipMemcpyDeviceToHost));
  FASST_HIP(hipMemcpy(ioff, dio.p, FT * sizeof(double2), hipMemcpyDeviceToHost));
  return FASST_OK;
}

int fasst_wiener_gain(int device, long n, const double *sdiag, const double *soff,
                      const double *idiag, const double *ioff, double *WG) {
  if (n < 1 || !sdiag || !soff || !idiag || !ioff || !WG) return FASST_ERR_SHAPE;
  DeviceGuard g(device);
  DBuf<double> dsd, did;
  DBuf<double2> dso, dio, dwg;
  int st;
  if ((st = dsd.alloc_uninit(2 * (size_t)n)) || (st = did.alloc_uninit(2 * (size_t)n)) ||
      (st = dso.alloc_uninit(n)) || (st = dio.alloc_uninit(n)) || (st = dwg.alloc_uninit(4 * (size_t)n)))
    return st;
  FASST_HIP(hipMemcpy(dsd.p, sdiag, 2 * (size_t)n * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(did.p, idiag, 2 * (size_t)n * sizeof(double), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dso.p, soff, (size_t)n * sizeof(double2), hipMemcpyHostToDevice));
  FASST_HIP(hipMemcpy(dio.p, ioff, (size_t)n * sizeof(double2), hipMemcpyHostToDevice));
  k_wiener_gain<<<grid_of(n), 256>>>(dsd.p, dso.p, did.p, dio.p, dwg.p, (size_t)n);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipMemcpy(WG, dwg.p, 4 * (size_t)n * sizeof(double2), hipMemcpyDeviceToHost));
  return FASST_OK;
}

}  // extern "C"
