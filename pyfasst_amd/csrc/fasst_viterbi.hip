// Viterbi melody tracker on MI355X (gfx950): the reference's only native
// component, _tracking.pyx:11-93 (Cython), as max-plus matrix-vector steps.
//
// Frame n needs every state's cum[., n-1], so frames are sequential; the
// parallelism is over target states s (and over the source states s' of
// each reduction):
//   k_vt_persist   (default for 137 < S <= 2048) ONE cooperative launch runs
//                  the whole track: ~96 resident workgroups each own ~S/96
//                  targets with their transition rows in registers (and LDS),
//                  and exchange cum[., n] every frame through data-tagged
//                  16-byte granules (write-through stores, L1-bypassing
//                  polls; no grid barrier, no fence).  S = 1092, N = 20000:
//                  ~39 ms (1.9 us per frame: ~1 us exchange, ~0.8 us argmax)
//                  vs 125 ms for one launch per frame.
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
#include <atomic>
#include "fasst_common.h"
#include "../../include/fasst_viterbi.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <utility>

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

// ------------------------------------------------------------ persistent path
// ONE launch runs every frame.  Workgroup g owns the target states
// [g*spw, g*spw + spw) and keeps their transition rows TT[s][.] in LDS for the
// whole track; the frame-to-frame exchange of cum[., n-1] goes through
// data-tagged granules instead of a grid barrier (cdna_hip_programming.md
// Guideline 16, R2): the double cum[s, n] is published as two 8-byte words
// {tag = n + 1, low / high 32 bits}, each one agent-scope (write-through)
// store, into slot n & 1; every workgroup re-reads the whole slot with
// agent-scope loads until every tag it sees is n, so a word is never taken
// from a stale line and no fence is needed.  Two slots suffice: a workgroup
// can only publish frame n + 1 after EVERY workgroup published frame n, which
// each did only after reading all of frame n - 1.  Spins are bounded: a
// workgroup that waits too long (a grid that is not fully resident) raises the
// abort word, every other spin sees it and leaves, and the host reruns the
// track on the launch-per-frame path.
typedef unsigned long long vt_u64;
typedef __attribute__((address_space(1))) int vt_gint;
constexpr unsigned kVtSpinMax = 1u << 21;
constexpr int kVtPersistThreads = 1024;

typedef unsigned vt_u4 __attribute__((ext_vector_type(4)));
constexpr int kVtSc1 = 16;   // buffer cache-policy bit sc1 (agent scope: write-through / L1 bypass)

// {low 32 bits, tag, high 32 bits, tag}: two self-tagged 8-byte granules in
// one 16-byte write-through store (each half is untorn on its own)
__device__ __forceinline__ void vt_publish(__amdgpu_buffer_rsrc_t g, int slot_off, int s,
                                           unsigned tag, double v) {
  const vt_u64 b = (vt_u64)__double_as_longlong(v);
  vt_u4 x;
  x.x = (unsigned)b;
  x.y = tag;
  x.z = (unsigned)(b >> 32);
  x.w = tag;
  __builtin_amdgcn_raw_buffer_store_b128(x, g, slot_off + 16 * s, 0, kVtSc1);
}

// Branch-free argmax of one wave over its candidates (two passes): M = max of
// the non-NaN candidates (v_max_f64 ignores a quiet NaN, as the pyx's '>'
// never takes one), then the smallest source index whose candidate equals M
// (the pyx's first maximum).  Both passes are reduced over the wave with DPP
// row pairings and four readlanes.  Returns (index, or INT_MAX if the wave
// has only NaN candidates); the caller re-forms the value from the index.
__device__ __forceinline__ double vt_wave_max(double m) {
#define VT_MAX_STEP(CTRL)                                                                 \
  {                                                                                       \
    const long long b = __double_as_longlong(m);                                          \
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);         \
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false); \
    m = fmax(m, __longlong_as_double(((long long)hi << 32) | (unsigned)lo));              \
  }
  VT_MAX_STEP(0xB1) VT_MAX_STEP(0x4E) VT_MAX_STEP(0x141) VT_MAX_STEP(0x140)
#undef VT_MAX_STEP
  const long long b = __double_as_longlong(m);
  double r = -INFINITY;
#pragma unroll
  for (int l = 0; l < 64; l += 16)
    r = fmax(r, __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(b >> 32), l) << 32) |
                                     (unsigned)__builtin_amdgcn_readlane((int)b, l)));
  return r;
}

__device__ __forceinline__ int vt_wave_min_i(int x) {
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));
  return min(min(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
             min(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}

// Layout: the sources of a target are cut into wpt parts of NU*64 (NU even,
// the last ones padded), a part per wave, so a lane's NU candidates are
// sources lo + 128 v + 2 lane + {0, 1} with no range test: the LDS rows of TT and the cum vector
// have pitch P = wpt*NU*64 and hold -inf beyond S, and a -inf candidate at a
// padded source can never be the first maximum (a real source with the same
// value has a smaller index).
// LDS position of logical source s: lane l of part h owns the NU consecutive
// sources h*NU*64 + l*NU + u, stored where the lane reads them with 16-byte
// loads, pairs (u, u + 1) at h*NU*64 + (u / 2)*128 + 2 l + (u & 1)
template <int NU>
__device__ __forceinline__ int vt_pos(int s) {
  const int h = s / (NU * 64), r = s - h * (NU * 64);
  const int l = r / NU, u = r - l * NU;
  return h * (NU * 64) + (u >> 1) * 128 + 2 * l + (u & 1);
}

template <int NU>
__global__ __launch_bounds__(kVtPersistThreads) void k_vt_persist(
    const double *__restrict__ TT, long ldt, const double *__restrict__ logdT, long ldd,
    const double *__restrict__ prior, int S, int N, int spw, int wpt, int *__restrict__ ante,
    long lda, double *__restrict__ cum_last, vt_u64 *gran, int *abort_word,
    long long *__restrict__ probe, int sleep0, int sleepr) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ int s_i[kVtPersistThreads / 64];
  __shared__ double s_v[kVtPersistThreads / 64];
  __shared__ int s_fail;
  const int P = wpt * NU * 64;
  double *s_tt = sm;                       // [spw][P]
  double *s_cum = sm + (size_t)spw * P;    // [P]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int s0 = blockIdx.x * spw, ns = min(spw, S - s0);
  const int lt = w / wpt, h = w - lt * wpt;   // local target, its source part
  const int lo = h * NU * 64;
  const __amdgpu_buffer_rsrc_t g = __builtin_amdgcn_make_buffer_rsrc(gran, 0, 32 * S, 0x00020000);
  if (tid == 0) s_fail = 0;
  for (int i = tid; i < spw * P; i += blockDim.x) {
    const int r = i / P, c = i - r * P;
    s_tt[r * P + vt_pos<NU>(c)] = r < ns && c < S ? TT[(size_t)(s0 + r) * ldt + c] : -INFINITY;
  }
  for (int c = S + tid; c < P; c += blockDim.x) s_cum[vt_pos<NU>(c)] = -INFINITY;
  if (tid < ns) {   // frame 0 (pyx :60-63)
    const double c0 = prior[s0 + tid] + logdT[s0 + tid];
    vt_publish(g, 0, s0 + tid, 1u, c0);
    if (N == 1) cum_last[s0 + tid] = c0;
  }
  // a lane polls states tid and tid + blockDim.x (S <= 2 blockDim.x)
  const int sA = tid < S ? tid : 0, sB = tid + (int)blockDim.x < S ? tid + blockDim.x : 0;
  const int pA = vt_pos<NU>(sA), pB = vt_pos<NU>(sB);
  if (probe && blockIdx.x == 0 && tid == 0) {
    probe[0] = wall_clock64();
    probe[1] = clock64();
  }
  const double *row = s_tt + (size_t)min(lt, spw - 1) * P + lo;
  const double *cumw = s_cum + lo;
  __syncthreads();
  // the wave's transition values stay in registers for the whole track (the
  // LDS copy serves only the re-forming of one winning candidate per frame)
  double ttr[NU];
#pragma unroll
  for (int v = 0; v < NU / 2; ++v) {
    const double2 b = *(const double2 *)(row + v * 128 + 2 * lane);
    ttr[2 * v] = b.x;
    ttr[2 * v + 1] = b.y;
  }
  for (int n = 1; n < N; ++n) {
    // this frame's densities of the own targets, loaded before the wait
    const double ld_n = tid < ns ? logdT[(size_t)n * ldd + s0 + tid] : 0.0;
    const int src = ((n - 1) & 1) * 16 * S;
    const bool prb = probe && blockIdx.x == 0 && tid == 0 && n < 4096;
    if (prb && n == 4000) {
      probe[2] = wall_clock64();
      probe[3] = clock64();
    }
    if (prb) probe[8 * n] = wall_clock64();
    // gather cum[., n - 1] (tag n) from slot (n - 1) & 1 into LDS, re-polling
    // only the states not seen yet
    unsigned spins = 0;
    bool failed = false;
    bool needA = tid < S, needB = tid + (int)blockDim.x < S;
    for (int z = 0; z < sleep0; ++z) __builtin_amdgcn_s_sleep(1);
    for (;;) {
      vt_u4 pa, pb;
      if (needA) pa = __builtin_amdgcn_raw_buffer_load_b128(g, src + 16 * sA, 0, kVtSc1);
      if (needB) pb = __builtin_amdgcn_raw_buffer_load_b128(g, src + 16 * sB, 0, kVtSc1);
      if (needA && pa.y == (unsigned)n && pa.w == (unsigned)n) {
        s_cum[pA] = __longlong_as_double((long long)(((vt_u64)pa.z << 32) | pa.x));
        needA = false;
      }
      if (needB && pb.y == (unsigned)n && pb.w == (unsigned)n) {
        s_cum[pB] = __longlong_as_double((long long)(((vt_u64)pb.z << 32) | pb.x));
        needB = false;
      }
      if (__all(!needA && !needB)) break;
      ++spins;
      if (spins > kVtSpinMax ||
          ((spins & 255) == 0 &&
           __hip_atomic_load((vt_gint *)abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        failed = true;
        break;
      }
      for (int z = 0; z < sleepr; ++z) __builtin_amdgcn_s_sleep(1);
    }
    if (failed && lane == 0) {
      s_fail = 1;
      __hip_atomic_store((vt_gint *)abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (prb) probe[8 * n + 1] = wall_clock64();
    if (s_fail) break;   // uniform over the workgroup
    if (lt < ns) {
      // pass 1: the lane's NU sources (cum by 16-byte LDS reads), their max over
      // the wave.  v_max_f64 ignores a quiet NaN, as the pyx's '>' never
      // takes one.
      double m = -INFINITY;
#pragma unroll
      for (int v = 0; v < NU / 2; ++v) {
        const double2 a = *(const double2 *)(cumw + v * 128 + 2 * lane);
        m = fmax(m, fmax(a.x + ttr[2 * v], a.y + ttr[2 * v + 1]));
      }
      const double ml = m;
      if (prb) probe[8 * n + 2] = wall_clock64() + (m > 1e300 ? 1 : 0);
      m = vt_wave_max(m);
      // the first maximum: the first lane whose max is m (lanes own
      // consecutive sources), then in that lane the first u with candidate
      // m, found by NU lanes re-forming one candidate each.  If every
      // candidate is NaN, m = -inf matches lane 0's max and no candidate:
      // the part reports (INT_MAX, -inf) and never wins the fold.
      const int lw = __ffsll((unsigned long long)__ballot(ml == m)) - 1;
      const int pu = ((lane >> 1) * 128) + 2 * lw + (lane & 1);
      const double x = lane < NU ? cumw[pu] + row[pu] : -INFINITY;
      const unsigned long long bu = __ballot(lane < NU && x == m);
      int idx = INT_MAX;
      double vw = -INFINITY;
      if (bu) {
        const int uw = __ffsll(bu) - 1;
        idx = lo + lw * NU + uw;
        const long long xb = __double_as_longlong(x);
        vw = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(xb >> 32), uw) << 32) |
                                  (unsigned)__builtin_amdgcn_readlane((int)xb, uw));
      }
      if (prb) probe[8 * n + 3] = wall_clock64() + (idx == 12345 ? 1 : 0);
      if (h == 0) {
        const double v0 = s_cum[0] + row[0];   // source 0 sits at position 0
        if (v0 != v0) {   // NaN at s' = 0: nothing compares greater (pyx :77)
          idx = 0;
          vw = v0;
        }
      }
      if (lane == 0) {
        s_i[w] = idx;
        s_v[w] = vw;
      }
    }
    __syncthreads();
    if (prb) probe[8 * n + 4] = wall_clock64();
    if (tid < ns) {   // fold the parts in source order, publish (pyx :83-85)
      // part 0 always has an index (a value or NaN at 0); a part with only
      // NaN candidates (INT_MAX, -inf) never wins
      int i = s_i[tid * wpt];
      double v = s_v[tid * wpt];
      for (int q = 1; q < wpt; ++q) vt_better(v, i, s_v[tid * wpt + q], s_i[tid * wpt + q]);
      const int s = s0 + tid;
      v += ld_n;
      ante[(size_t)n * lda + s] = i;
      vt_publish(g, (n & 1) * 16 * S, s, (unsigned)n + 1u, v);
      if (n == N - 1) cum_last[s] = v;
    }
    if (prb) probe[8 * n + 5] = wall_clock64();
  }
}

typedef void (*vt_persist_fn)(const double *, long, const double *, long, const double *, int,
                              int, int, int, int *, long, double *, vt_u64 *, int *, long long *,
                              int, int);
template <int... I>
struct VtPersistTable {
  static constexpr vt_persist_fn fn[sizeof...(I)] = {k_vt_persist<2 * (I + 1)>...};
};
constexpr int kVtMaxNU = 20;
template <int... I>
static const vt_persist_fn *vt_table(std::integer_sequence<int, I...>) {
  return VtPersistTable<I...>::fn;
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
// persistent launches that aborted and were rerun on the per-frame path
// (about 3x slower): counted for viterbi_fallback_count and reported once
static std::atomic<int> g_vt_aborts{0};

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
  }
  bool done = lds <= kVtLdsBudget;
  // persistent path: G <= 240 workgroups of 1024 threads (one per CU), spw
  // targets each with their TT rows and the cum vector in LDS, wpt waves per target
  const char *force = getenv("FASST_VT_PATH");   // "frame": launch-per-frame (tests / A/B)
  // states per workgroup: about 96 workgroups when that fits (fewer pollers
  // of the exchange; measured best at S = 1092: 91 workgroups of 12 targets),
  // else the largest count with <= 20 candidates per lane in the LDS budget
  int spw = 0, wpt = 1, nu = 0;
  {
    const int lo_spw = (S + 239) / 240;
    const int want = std::max(lo_spw, (S + 95) / 96);
    for (int c = std::min(want, kVtPersistThreads / 64); c >= lo_spw && c >= 1; --c) {
      const int cw = std::max(1, (kVtPersistThreads / 64) / c);
      const int cn = (((S + cw - 1) / cw + 127) / 128) * 2;
      if (cn <= kVtMaxNU && (size_t)(c + 1) * cw * cn * 64 * sizeof(double) <= kVtLdsBudget) {
        spw = c;
        wpt = cw;
        nu = cn;
        break;
      }
    }
  }
  const size_t plds = (size_t)(spw + 1) * wpt * nu * 64 * sizeof(double);
  if (!done && spw > 0 && S <= 2 * kVtPersistThreads && !(force && std::string(force) == "frame")) {
    DBuf<vt_u64> gran;
    DBuf<int> abort_word;
    DBuf<long long> probe;
    const bool want_probe = getenv("FASST_VT_PROBE") != nullptr;   // diagnostics only
    if ((st = gran.alloc((size_t)4 * S)) || (st = abort_word.alloc(1))) return st;
    if (want_probe && (st = probe.alloc(8 * 4096))) return st;
    const void *kfn =
        (const void *)vt_table(std::make_integer_sequence<int, kVtMaxNU / 2>())[nu / 2 - 1];
    FASST_HIP(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds));
    const int G = (S + spw - 1) / spw;
    const double *pTT = dTT.p, *pDT = dDT.p, *ppr = dprior.p;
    long ldt = Sp, ldd = Sp, lda = Sp;
    int nS = S, nN = N, nspw = spw, nwpt = wpt;
    int *pante = ante.p, *pab = abort_word.p;
    double *pcl = clast.p;
    vt_u64 *pg = gran.p;
    long long *pprobe = probe.p;
    // the first poll of a frame waits ~0.35 us (13 x 64 clocks) after the own
    // publish: polling at once only loads the exchange while the other
    // workgroups store (S = 1092: 43.5 ms per track without the wait, 38.5
    // with it, 39-44 ms with 10 / 16 / 19 / 22)
    int sleep0 = 13, sleepr = 1;   // in s_sleep(1) units of 64 clocks
    void *args[] = {&pTT, &ldt, &pDT, &ldd, &ppr, &nS, &nN, &nspw, &nwpt,
                    &pante, &lda, &pcl, &pg, &pab, &pprobe, &sleep0, &sleepr};
    // the cooperative launch checks that the whole grid is co-resident
    const hipError_t e = hipLaunchCooperativeKernel(kfn, dim3(G),
                                                    dim3(kVtPersistThreads), args, plds, 0);
    if (e == hipSuccess) {
      int aborted = 1;
      FASST_HIP(hipMemcpy(&aborted, abort_word.p, sizeof(int), hipMemcpyDeviceToHost));
      if (!aborted) {
        g_vt_kind = 2;
        done = true;
      } else if (g_vt_aborts.fetch_add(1) == 0) {
        fprintf(stderr, "viterbi_tracking: the persistent launch aborted (its grid was not "
                "co-resident, e.g. another process shares the GPU); rerunning on the "
                "per-frame path (~3x slower). Further aborts are only counted "
                "(viterbi_fallback_count).\n");
      }
      if (want_probe) {   // per-phase means of workgroup 0 over frames 2..4095, us
        std::vector<long long> h(8 * 4096);
        FASST_HIP(hipMemcpy(h.data(), probe.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
        const int nf = std::min(N, 4096);
        double a[6] = {0, 0, 0, 0, 0, 0};
        for (int n = 2; n < nf; ++n) {
          for (int k = 0; k < 5; ++k) a[k] += h[8 * n + k + 1] - h[8 * n + k];
          a[5] += h[8 * n] - h[8 * (n - 1) + 5];
        }
        for (double &x : a) x = x * 0.01 / std::max(1, nf - 2);   // 100 MHz ticks
        const double mhz = N > 4000 ? (double)(h[3] - h[1]) / ((h[2] - h[0]) * 0.01) : 0.0;
        fprintf(stderr, "vt_probe G=%d spw=%d wpt=%d nu=%d: wait %.3f cand %.3f reduce %.3f "
                "bar %.3f publish %.3f gap %.3f us; core clock %.0f MHz\n",
                G, spw, wpt, nu, a[0], a[1], a[2], a[3], a[4], a[5], mhz);
      }
    } else {
      (void)hipGetLastError();   // too large for co-residency: per-frame launches
    }
  }
  if (!done) {
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

int viterbi_fallback_count(int *aborts) {
  if (!aborts) return FASST_ERR_SHAPE;
  *aborts = g_vt_aborts.load();
  return FASST_OK;
}

int viterbi_last_timing(double *device_ms, int *path_kind) {
  if (device_ms) *device_ms = g_vt_ms;
  if (path_kind) *path_kind = g_vt_kind;
  return FASST_OK;
}

}  // extern "C"
