// FASST generalized-EM iteration on MI355X (gfx950), FP64 throughout.
//
// One GEM iteration (audioModel.py:384-428) is a fixed sequence of launches
// on the context's stream:
//   k_w_from_fb   W = FB.FW                       (comp_spat_comp_power :485)
//   k_fwh_t       (FW.TW)^T                       (update_spectral_components :1541)
//   k_inst_A      per-bin mixing from 'inst' params (retrieve_subsrc_params :570-574)
//   k_estep<J>    fused E-step: V^T tiles on FP64 MFMA, Sigma_x, 2x2 inverse,
//                 loglik, posterior powers hat_W, per-bin sufficient
//                 statistics (compute_suff_stat :580-764)
//   k_loglik      loglik = -mean(...)             (:660-664)
//   k_mix_conv / k_mix_stats + k_mix_inst          (update_mix_matrix :766-889)
//   k_fb_contract FB numerator/denominator over t (MFMA, :1521-1575)
//   k_fb_update   FB *= (num/den)^omega, W_new = FB.FW
//   k_tw_contract TW numerator/denominator over f (MFMA) + TW update (:1634-1727)
//   k_renorm      renormalize_parameters          (:1980-2040)
//
// E-step restructuring (exact algebra, verified to 1e-15 against the
// reference): with S = Sigma_x^-1, N = S Cx S - S and P = Cx S (2x2 per
// (f,t)), the reference's R x R pair loop (:698-731) is
//   hat_Rss[f][r1,r2] = a_r1^H (sum_t V_j1 V_j2 N) a_r2 / T + d_r1r2 mean_t V_r1
//   hat_Rxs[f][c,r]   = sum_c' (sum_t V_j P)[c,c'] A_r,c' / T
//   hat_Ws[r](f,t)    = | V_j^2 a_r^H N a_r + V_j |
// because the mixing a_r is constant over t.  The t-reductions shrink from
// R^2 complex products per (f,t) to J(J+1)/2 x 4 + 9J real FMAs.
#include "fasst_ctx.h"

#include <cmath>
#include <cstring>
#include <mutex>

namespace fasst {

static thread_local std::string g_err;
void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

// Device-side halt: once an iteration raises a flag (singular mixing solve,
// dead TW) every later kernel of the batch returns at entry, so a batch of
// iterations is enqueued without host round trips and the state stays the
// one the flagged iteration left (flags layout in fasst_ctx.h).
#define HALT_GUARD(h)                                   \
  do {                                                  \
    if ((h) && *(volatile const int *)(h)) return;      \
  } while (0)

// XCD-aware logical block: workgroups b, b + 8, ... of a launch share an XCD
// (dispatch is round-robin over the 8 XCDs, for speed only, never
// correctness); the bijective remap of cdna_hip_programming.md gives each XCD
// a contiguous run of the logical (x fastest, z slowest) sequence, so the
// blocks that re-read one operand slice (the E-step's TW chunk, the
// contractions' W / (FW H)^T slices) meet in one 4 MB L2.  At C3 it takes
// 9-14 % off the HBM fetch of the E-step and both contractions (rocprofv3
// FETCH_SIZE, profiles/r4_bench.txt vs the row-major order) at equal time.
__device__ __forceinline__ dim3 xcd_block() {
  const int nx = gridDim.x, ny = gridDim.y, n = nx * ny * gridDim.z;
  const int b = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int q = n / 8, r = n % 8, x = b % 8;
  const int L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  return dim3(L % nx, (L / nx) % ny, L / (nx * ny));
}

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// max(x, y) as ONE v_max_f64: fmax() lowers to llvm.maxnum, whose operands
// the backend first canonicalises (a second v_max_f64 each) unless it can
// prove them canonical, which it cannot for MFMA results.  For the finite
// operands it is used on the two forms agree.
__device__ __forceinline__ double vmax_f64(double x, double y) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

// 1/x for finite normal x (the E-step's guarded det and max(V, eps)):
// v_rcp_f64 + two Newton steps (<= 1 ulp) instead of the ~10-instruction
// IEEE division sequence.
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}

// ---------------------------------------------------------------- prep
// W[j] = FB[j] . FW[j], written [KP][Fp] (f contiguous).
// one block per (16-bin tile, source): FB tile and FW staged in LDS; the
// outputs are written bin-fastest (coalesced Wkf rows)
template <bool FWG>   // FWG: FW read from L2 (KP > 64), else staged in LDS
__global__ __launch_bounds__(256) void k_w_from_fb(const double *__restrict__ FB,
                                                   const double *__restrict__ FW,
                                                   double *__restrict__ Wkf,
                                                   double *__restrict__ Wfk, int J, int Fp,
                                                   int KP, const int *halt) {
  HALT_GUARD(halt);
  extern __shared__ __attribute__((aligned(16))) double s_m[];
  double *s_fb = s_m;             // [16][KP + 1]
  double *s_fw = s_m + 16 * (KP + 1);  // [KP][KP] (KP <= 64; else FW is read from L2)
  constexpr bool fwg = FWG;
  const int j = blockIdx.y, f0 = blockIdx.x * 16;
  const double *fw = fwg ? FW + (size_t)j * KP * KP : s_fw;
  for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
    const int fl = idx / KP, q = idx % KP;
    s_fb[fl * (KP + 1) + q] = FB[((size_t)j * Fp + f0 + fl) * KP + q];
  }
  if constexpr (fwg) {
    // KP = 128 on the matrix cores: D[k][f] = sum_q FW[q][k] FB[f][q] per
    // 16 x 16 tile (16x16x4: A = FW^T rows from L2, B = the FB tile in LDS),
    // wave w forming the k tiles w, w + 4, ...; lane (fl, tq) then holds
    // W[k = 16 kc + tq + 4 i][f0 + fl] (128-byte Wkf row pieces)
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, fl = lane & 15, tq = lane >> 4;
    for (int kc = wv; kc < KP / 16; kc += 4) {
      d4 d = d4{0.0, 0.0, 0.0, 0.0};
      for (int q0 = 0; q0 < KP; q0 += 4)
        d = __builtin_amdgcn_mfma_f64_16x16x4f64(fw[(size_t)(q0 + tq) * KP + 16 * kc + fl],
                                                 s_fb[fl * (KP + 1) + q0 + tq], d, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 16 * kc + tq + 4 * i;
        Wkf[((size_t)j * KP + k) * Fp + f0 + fl] = d[i];
        if (Wfk) Wfk[((size_t)j * Fp + f0 + fl) * KP + k] = d[i];
      }
    }
    return;
  }
  if (!fwg)
    for (int idx = threadIdx.x; idx < KP * KP; idx += blockDim.x)
      s_fw[idx] = FW[(size_t)j * KP * KP + idx];
  __syncthreads();
  for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
    const int k = idx / 16, fl = idx % 16;
    double s = 0.0;
    for (int q = 0; q < KP; ++q) s += s_fb[fl * (KP + 1) + q] * fw[q * KP + k];
    Wkf[((size_t)j * KP + k) * Fp + f0 + fl] = s;
    if (Wfk) Wfk[((size_t)j * Fp + f0 + fl) * KP + k] = s;
  }
}

// FWHt[j][t][k] = sum_q FW[j][k][q] TW[j][q][t]; one block per (64-frame
// tile, source): FW and the TW tile staged in LDS, coalesced [t][k] writes.
template <bool FWG>
__global__ __launch_bounds__(256) void k_fwh_t(const double *__restrict__ FW,
                                               const double *__restrict__ TW,
                                               double *__restrict__ FWHt, double *__restrict__ TWt,
                                               int J, int Tp, int KP, const int *halt) {
  HALT_GUARD(halt);
  extern __shared__ __attribute__((aligned(16))) double s_f[];
  // FWG (KP = 128): FW's [KP][KP] copy and the TW tile do not fit LDS
  // together, so FW goes through it in two halves of its rows q (the
  // contraction index), each thread keeping its outputs in registers (FW
  // read straight from L2 was a 1 KB-stride gather per lane: 1.36 ms at
  // J = 8, K = 128)
  constexpr bool fwg = FWG;
  double *s_fw = s_f;                                  // [QH][KP] (q-major, transposed)
  double *s_tw = s_f + (fwg ? 16 * KP : KP * KP);      // [KP][64]
  const int j = blockIdx.y, t0 = blockIdx.x * 64;
  const int tn = min(64, Tp - t0);
  for (int idx = threadIdx.x; idx < KP * 64; idx += blockDim.x) {
    const int q = idx >> 6, tl = idx & 63;
    s_tw[idx] = tl < tn ? TW[((size_t)j * KP + q) * Tp + t0 + tl] : 0.0;
  }
  if constexpr (fwg) {
    // KP = 128 on the matrix cores: wave w forms frames 16 w .. 16 w + 15,
    // D[k][t] = sum_q FW[k][q] TW[q][t] per 16 x 16 tile (16x16x4: A = FW
    // through LDS transposed, QB rows q at a time; B = the TW tile); lane
    // (fl, tq) then holds FWHt[t0 + 16 w + fl][16 kc + tq + 4 i]
    constexpr int KPG = 128, QB = 16;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, fl = lane & 15, tq = lane >> 4;
    d4 d[KPG / 16];
#pragma unroll
    for (int kc = 0; kc < KPG / 16; ++kc) d[kc] = d4{0.0, 0.0, 0.0, 0.0};
    for (int qb = 0; qb < KPG; qb += QB) {
      __syncthreads();   // (qb > 0: the previous chunk's reads are done)
      for (int idx = threadIdx.x; idx < QB * KPG; idx += blockDim.x) {
        const int k = idx / QB, q = idx % QB;   // (coalesced over q in FW's rows)
        s_fw[q * KPG + k] = FW[((size_t)j * KPG + k) * KPG + qb + q];
      }
      __syncthreads();
#pragma unroll
      for (int kc = 0; kc < KPG / 16; ++kc)
#pragma unroll
        for (int q0 = 0; q0 < QB; q0 += 4)
          d[kc] = __builtin_amdgcn_mfma_f64_16x16x4f64(s_fw[(q0 + tq) * KPG + 16 * kc + fl],
                                                       s_tw[(qb + q0 + tq) * 64 + 16 * wv + fl], d[kc], 0, 0,
                                                       0);
    }
    const int tl = 16 * wv + fl;
    if (tl < tn)
#pragma unroll
      for (int kc = 0; kc < KPG / 16; ++kc)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 16 * kc + tq + 4 * i;
          FWHt[((size_t)j * Tp + t0 + tl) * KPG + k] = d[kc][i];
          if (TWt) TWt[((size_t)j * Tp + t0 + tl) * KPG + k] = s_tw[k * 64 + tl];
        }
    return;
  }
  for (int idx = threadIdx.x; idx < KP * KP; idx += blockDim.x) {
    const int k = idx / KP, q = idx % KP;  // stored transposed: s_fw[q][k]
    s_fw[q * KP + k] = FW[(size_t)j * KP * KP + idx];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < tn * KP; idx += blockDim.x) {
    const int tl = idx / KP, k = idx % KP;
    double s = 0.0;
    for (int q = 0; q < KP; ++q) s += s_fw[q * KP + k] * s_tw[q * 64 + tl];
    FWHt[((size_t)j * Tp + t0 + tl) * KP + k] = s;
    if (TWt) TWt[((size_t)j * Tp + t0 + tl) * KP + k] = s_tw[k * 64 + tl];  // H^T (FW update)
  }
}

// 'inst' mixing replicated over bins: A[r][c][f] = params[c][r], for the
// rows of rowm ('inst' sources; a mixed model's 'conv' rows hold their own
// per-bin filters)
__global__ void k_inst_A(const double2 *__restrict__ Pinst, double2 *__restrict__ A, int R,
                         int F, int Fp, unsigned rowm, const int *halt) {
  HALT_GUARD(halt);
  const int n = R * 2 * Fp;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
    const int f = idx % Fp;
    const int rc = idx / Fp;
    if (rowm >> (rc >> 1) & 1u) A[idx] = f < F ? Pinst[rc] : make_double2(0.0, 0.0);
  }
}

// ---------------------------------------------------------------- E-step
struct EArgs {
  const double *cx00, *cx11, *cxr, *cxi;  // [Tp][Fp]
  const double *TW;                       // [J][KP][Tp]
  const double *Wkf;                      // [J][KP][Fp]
  const double2 *A;                       // [R][2][Fp]
  const double *psd;                      // [Fp]
  double *hatW;                           // [J][Tp][Fp]: rho = hat_W / max(V, eps)
  double *part;                           // [nchunk][Fp][NACC]
  double *llpart;                         // [nchunk][nft]
  int F, T, Fp, Tp, KP, R, ntt, tpc, nft;
  int ybase, tbase;  // this launch's chunks start at partial ybase, frame tile tbase (ntt = end)
  int roff[kMaxJ + 1];
  const int *halt;
};

// Single-pass E-step with the per-bin t-reductions on the matrix cores.
//
// Every statistic of the E-step is a per-bin dot product over frames:
//   cross  Q_j[c]      = sum_t V_j P_c        (P = Cx S, 8 real components)
//   pairs  M_p[c]      = sum_t V_j1 V_j2 N_c  (N = S Cx S - S, 4 components)
// For one bin these are tiny GEMMs, (J x T).(T x 8) and (NP x T).(T x 4).
// v_mfma_f64_4x4x4_4b runs four independent 4x4x4 products per instruction,
// one per block of 16 lanes (lane = 16 X + 4 b + Y: A[m=Y][k=X],
// B[k=X][n=Y], D[m=X][n=Y] of block b; tools/probe_mfma4.hip), so with
// block = bin and k = frame, ONE instruction contracts 4 frames of 4 bins
// for a 4 x 4 block of statistics.  After each frame group, every lane drops
// its point's operands (V, P, N and the pair products V_j1 V_j2) into a
// per-wave LDS slab in the MFMA operand layout, and the wave issues
// 4 bin groups x (2 + ceil(NP/4)) MFMAs.  The accumulators shrink from
// 4 J(J+1)/2 + 8J doubles per lane (72 at J = 4, what forced the round-1
// E-step into two launches) to 4 (2 + ceil(NP/4)) (20 at J = 4), so ONE pass
// streams Cx once, forms V, Sigma_x and its inverse once per point, and keeps
// two waves per SIMD; the 72 FMAs per point leave the VALU for the matrix
// pipe (4x4x4_4b runs at 74.7 TF on this chip, profiles/r1_ubench_fp64.txt).
__device__ __forceinline__ double mfma44(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// Reader-formed pair operands (RP, J >= 4): the slab holds V, P and N only,
// and the reader forms the pair operands V_j1 V_j2 itself.  With the sources
// padded to Q = 4 (J = 4) or 8 (J > 4), lane m of a 4-pair group reads the Q
// rotated values W_e = V_{(m + e) mod Q} of its point, and the pairs are the
// groups (base, d): pair m of a group is (base + m, base + m + d mod Q), its
// operand W_base W_{(base + d) mod Q} -- static register indices.  Q = 8: the
// 36 pairs are {0, 4} x {0..3} plus (0, 4); Q = 4: the 10 pairs are
// (0, 0), (0, 1) and (0, 2) (rows m = 2, 3 of the last repeat rows 0, 1).
// The writer's J (J + 1) / 2 products and their slab stores go (J = 8: 56 ->
// 20 stores per point, J = 4: 26 -> 16), the reader's loads stay or drop
// (J = 8: 14 -> 11 per bin group), and the slab shrinks.  Same-box A/B at
// C3 (J = 4): E-step 0.373 vs 0.390 ms, iteration 1.040 vs 1.068 ms; J = 6 /
// 8 (K = 32): 0.813 / 1.002 ms against 1.083 / 1.663 ms with writer-formed
// pairs.
// VR (J > 4): also the per-source pipelined V tile, one wave per SIMD (the
// register file, not the LDS, bounds it: at two waves the kernel spills
// 500+ bytes per lane to scratch) and the epilogue one bin group at a time.
template <int J>
struct MXShape {
  static constexpr bool VR = J > 4;
  static constexpr bool RP = J >= 4;
  static constexpr int Q = J > 4 ? 8 : 4;       // RP: sources padded to Q
  static constexpr int NP = J * (J + 1) / 2;
  static constexpr int NPG = RP ? (Q == 8 ? 9 : 3) : (NP + 3) / 4;   // pair groups of 4
  static constexpr int NVG = (J + 3) / 4;       // source groups of 4
  static constexpr int SP = NVG, SN = NVG + 2, SV2 = NVG + 3;  // set offsets: P lo/hi, N, VV
  static constexpr int NSET = NVG + 3 + (RP ? 0 : NPG);  // V groups | P lo | P hi | N | VV groups
  static constexpr int GS = NSET * 64 + 1;      // doubles per bin group (+1: bank skew)
  // VST (J > 4): the V sets of all four point rounds are written once per
  // tile, right after the V tile ([round][bin group][NVG sets], VGS each),
  // then P / N per round ([bin group][3 sets], PGS each)
  static constexpr bool VST = VR;
  static constexpr int VGS = NVG * 64 + 1, PGS = 3 * 64 + 1;
  static constexpr int SLAB = VST ? 16 * VGS + 4 * PGS : 4 * GS;   // doubles per wave
};
// RP pair group h: (base, d)
template <int Q>
__host__ __device__ constexpr int rp_base(int h) { return Q == 4 || h == 8 ? 0 : 4 * (h & 1); }
template <int Q>
__host__ __device__ constexpr int rp_d(int h) { return Q == 4 ? h : (h == 8 ? 4 : h >> 1); }
// canonical index (j1 <= j2, j1 major) of the pair lane m of group h
// accumulates, or -1 (a padded source or a repeated pair)
template <int J>
__host__ __device__ constexpr int rp_pair(int h, int m) {
  constexpr int Q = MXShape<J>::Q;
  if (!MXShape<J>::RP) return 4 * h + m < MXShape<J>::NP ? 4 * h + m : -1;
  const int j1 = rp_base<Q>(h) + m, j2 = (rp_base<Q>(h) + m + rp_d<Q>(h)) & (Q - 1);
  if (j1 >= J || j2 >= J || (Q == 4 && rp_d<Q>(h) == 2 && m >= 2)) return -1;
  const int lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
  return lo * J - lo * (lo - 1) / 2 + (hi - lo);
}
// does RP pair group h hold a live pair
template <int J>
__host__ __device__ constexpr bool rp_live(int h) {
  for (int m = 0; m < 4; ++m)
    if (rp_pair<J>(h, m) >= 0) return true;
  return false;
}

// the W tile sits in LDS unless it would push the block past 160 KB (J = 8,
// K = 128); then the V tiles read their W operand from L2
template <int J, int NKS>
__host__ __device__ constexpr bool mx_w_in_lds() {
  return (size_t)(4 + J * 4 * NKS * 16 + 4 * MXShape<J>::SLAB + J * 4 * 16) * sizeof(double) <=
         160 * 1024;
}
template <int J, int NKS>
static constexpr size_t estep_mx_smem() {
  return (size_t)(4 + (mx_w_in_lds<J, NKS>() ? J * 4 * NKS * 16 : 0) + 4 * MXShape<J>::SLAB) *
         sizeof(double);
}

// (the LDS slabs allow two blocks per CU, so the register budget is that of
// two waves per SIMD: amdgpu_waves_per_eu tells the scheduler, which would
// otherwise serialise the operand loads to fit three)
// (more than 4 sources: one block per CU -- the slabs alone pass 80 KB -- so
// one wave per SIMD and the full 512-register file)
// (no-load-store-opt: the compiler otherwise pairs the slab / W-tile reads
// into ds_read2_b64 / ds_read2st64_b64, which take 8 LDS cycles for the 4 of
// two ds_read_b64 -- MI355X_MICROARCH.md §LDS -- and the LDS is this kernel's
// busiest unit)
// raw-buffer forms of the E-step's streaming accesses: wave-uniform
// resource (SGPRs, formed on the scalar unit) + 32-bit per-lane offset, so
// no 64-bit VALU address arithmetic per access (aux 2 = non-temporal)
typedef unsigned es_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t es_rsrc(const double *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), 0, 0x7fffffff, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ double es_ld(__amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  const es_u2 x = __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, (int)so, AUX);
  return __builtin_bit_cast(double, x);
}
template <int AUX>
__device__ __forceinline__ void es_st(double v, __amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(es_u2, v), r, (int)vo, (int)so, AUX);
}

// (J = 4 at K = 128: the 64 KB W tile leaves one block per CU, so one wave
// per SIMD and the full register file for the pipelined V tile)
template <int J, int NKS, int RKU>
__global__ __launch_bounds__(256, (J > 4 || (J == 4 && NKS == 32)) ? 1 : 2)
__attribute__((amdgpu_waves_per_eu(1, (J > 4 || (J == 4 && NKS == 32)) ? 1 : 2))) FASST_NO_LDS_PAIRING
void k_estep_mx(const EArgs a) {
  HALT_GUARD(a.halt);
  using S = MXShape<J>;
  constexpr bool VR = S::VR, RP = S::RP;
  constexpr int Q = S::Q;
  constexpr int NP = S::NP, NPG = S::NPG, NVG = S::NVG;
  constexpr int NACC = 4 * NP + 8 * J;
  constexpr int KP = 4 * NKS;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // per-source Sigma_x coefficients in a static array: the compiler can see
  // that the slab stores never touch them and reuse each read within a tile
  __shared__ double s_cj[J * 4 * 16];      // [J][4][16]
  constexpr bool WL = mx_w_in_lds<J, NKS>();
  double *s_ll = smem;                     // [4]
  double *s_w = s_ll + 4;                  // [J][KP][16] W tile (if WL)
  double *s_slab = s_w + (WL ? J * KP * 16 : 0);  // [4 waves][SLAB] operand slabs
  double *s_red = s_w;                     // [4][NACC][16 | 4] (epilogue, aliases W + slabs)

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fl = lane & 15, tq = lane >> 4;
  const dim3 bi = xcd_block();   // x: 16-bin tile, y: frame chunk
  const int f0 = bi.x * 16;
  const int f = f0 + fl;
  double *slab = s_slab + wv * S::SLAB;

  if (WL)
    for (int idx = tid; idx < J * KP * 16; idx += 256) {
      const int ff = idx & 15, jk = idx >> 4;
      s_w[idx] = a.Wkf[(size_t)jk * a.Fp + f0 + ff];
    }
  // operand slots no point writes (sources >= J, pairs >= NP) stay zero
  for (int idx = tid; idx < 4 * S::SLAB; idx += 256) s_slab[idx] = 0.0;
  if (tid < 16) {
    const int ff = f0 + tid;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      double al = 0, be = 0, gr = 0, gi = 0;
      for (int r = a.roff[j]; r < a.roff[j + 1]; ++r) {
        const double2 a0 = a.A[(size_t)(2 * r) * a.Fp + ff];
        const double2 a1 = a.A[(size_t)(2 * r + 1) * a.Fp + ff];
        al += a0.x * a0.x + a0.y * a0.y;
        be += a1.x * a1.x + a1.y * a1.y;
        gr += a0.x * a1.x + a0.y * a1.y;  // Re a0 conj(a1)
        gi += a0.y * a1.x - a0.x * a1.y;  // Im a0 conj(a1)
      }
      s_cj[(j * 4 + 0) * 16 + tid] = al;
      s_cj[(j * 4 + 1) * 16 + tid] = be;
      s_cj[(j * 4 + 2) * 16 + tid] = gr;
      s_cj[(j * 4 + 3) * 16 + tid] = gi;
    }
  }
  __syncthreads();

  // CJR (J >= 4): the lane's Sigma_x coefficients in registers for the
  // whole kernel (J = 8: 474 -> 240 LDS reads and 243 -> 84 waits per tile,
  // E-step 1.00 -> 0.98 ms; J = 4: 0.372 -> 0.364 ms, same-box A/B)
  constexpr bool CJR = J >= 4;
  constexpr bool NF = J >= 4;
  double cjr[CJR ? J : 1][4];
  if constexpr (CJR)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) cjr[j][c] = s_cj[(j * 4 + c) * 16 + fl];
  double inv_rk[J];
#pragma unroll
  for (int j = 0; j < J; ++j)
    inv_rk[j] = RKU ? 1.0 / (double)RKU : 1.0 / (double)(a.roff[j + 1] - a.roff[j]);
  const double psd = a.psd[f];
  const bool fvalid = f < a.F;
  // writer side: this lane's point goes to bin group g = fl / 4, block b = fl % 4, X = tq
  double *wr = slab + (fl >> 2) * S::GS + 16 * tq + 4 * (fl & 3);
  // reader side: operands of lane (X, b, Y) sit at [group][set][lane]
  const double *rd = slab + lane;
  auto slab_fence0 = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // RP: W_e = V_{(m + e) mod Q} of the lane's point (m = Y) sits in set
  // ((m + e) mod Q) / 4 at Y' = (m + e) mod 4 of the same (X, b)
  const double *rdq = slab + (lane & ~3);
  constexpr bool VST = S::VST;
  // VST: this lane's V of round i at wrv + i 4 VGS (+ (j >> 2) 64 + (j & 3)),
  // its P / N at wpn; the reader's V of round i, bin group g at
  // rdq + (4 i + g) VGS, P / N at rpn + g PGS
  double *wrv = slab + (fl >> 2) * S::VGS + 16 * tq + 4 * (fl & 3);
  double *wpn = slab + 16 * S::VGS + (fl >> 2) * S::PGS + 16 * tq + 4 * (fl & 3);
  const double *rpn = slab + 16 * S::VGS + lane;
  int vro[Q];
#pragma unroll
  for (int e = 0; e < Q; ++e) {
    const int j = ((lane & 3) + e) & (Q - 1);
    vro[e] = (j >> 2) * 64 + (j & 3);
  }

  double xacc[4][NVG][2], pacc[4][NPG];  // D operands (4x4 blocks per bin group)
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int vg = 0; vg < NVG; ++vg) xacc[g][vg][0] = xacc[g][vg][1] = 0.0;
#pragma unroll
    for (int h = 0; h < NPG; ++h) pacc[g][h] = 0.0;
  }
  double ll = 0.0, lm = 1.0, lev = 0.0, xmin = 1.0;

  const int tb = a.tbase + bi.y * a.tpc;
  const int te = min(tb + a.tpc, a.ntt);
  // SA: wave-uniform buffer resources (SGPRs, formed on the scalar unit) +
  // 32-bit per-lane byte offsets instead of one 64-bit VALU address
  // computation per access
  constexpr bool SA = true;
  int wvu = wv;
  if constexpr (SA) wvu = __builtin_amdgcn_readfirstlane(wv);
  const unsigned vo_tw = (unsigned)(tq * a.Tp + fl) * 8u;   // TW[j][k = tq + 4s][t0 + fl]
  const unsigned vo_cx = (unsigned)(tq * a.Fp + f) * 8u;    // plane[t0 + tq + 4i][f]
  // Cx of frame tile tt (raw-buffer form; the flat form without SA)
  auto load_cx = [&](int tt, double (&c)[4][4]) {
    const int t0 = tt * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (SA) {
        const size_t ro = (size_t)t0 * a.Fp;
        const unsigned so = (unsigned)(4 * i * a.Fp) * 8u;
        c[0][i] = es_ld<2>(es_rsrc(a.cx00 + ro), vo_cx, so);
        c[1][i] = es_ld<2>(es_rsrc(a.cx11 + ro), vo_cx, so);
        c[2][i] = es_ld<2>(es_rsrc(a.cxr + ro), vo_cx, so);
        c[3][i] = es_ld<2>(es_rsrc(a.cxi + ro), vo_cx, so);
      } else {
        const size_t off = (size_t)(t0 + tq + 4 * i) * a.Fp + f;
        c[0][i] = __builtin_nontemporal_load(a.cx00 + off);
        c[1][i] = __builtin_nontemporal_load(a.cx11 + off);
        c[2][i] = __builtin_nontemporal_load(a.cxr + off);
        c[3][i] = __builtin_nontemporal_load(a.cxi + off);
      }
    }
  };
  // CXE (J > 4): the next tile's Cx loads are issued right after this
  // tile's last point consumed its Cx (in the pipelined point loop), so they
  // land during the last point's MFMAs and the next tile's V tile (J = 6 /
  // 8: 0.790 / 0.961 -> 0.749 / 0.944 ms; at J = 4, two waves per SIMD,
  // 0.361 -> 0.368 ms: not used there)
  constexpr bool CXE = J > 4;
  double cxv[4][4];
  if (CXE && tb + wvu < te) load_cx(tb + wvu, cxv);
  for (int tt = tb + wvu; tt < te; tt += 4) {
    const int t0 = tt * 16;
    int lofs = 0;  // launder: re-read the loop-invariant LDS data per tile
    asm volatile("" : "+v"(lofs));
    // all TW operands in flight before the first MFMA (the scheduler would
    // otherwise pair each load with its MFMA and wait on every one); with more
    // than 32 operands (J > 4 or K > 32 at J = 4) the sources beyond the first
    // 32 operands load next to their own MFMAs
    // (VR: none up front -- the V loop below pipelines them source by source)
    // CP: more operands than that (J <= 4 at K >= 64): the V tiles as one
    // pipeline of 8-MFMA chunks over (source, k), each chunk's TW operands
    // issued two chunks ahead -- the per-source inline loads left each
    // source's load latency exposed (J = 4, K = 128: 2.70 ms).  (The same
    // pipeline for the VR loop with W from L2, J > 4 at K = 128, crashes
    // ROCm 7.2's compiler at distance 2 and spills 0.4-1.8 KB per lane at 1.)
    constexpr bool CP = !VR && J * NKS > 32;
    constexpr int JA = (VR || CP) ? 1 : (J * NKS <= 32) ? J : (32 / NKS > 0 ? 32 / NKS : 1);
    double twv[JA][NKS];
#pragma unroll
    for (int j = 0; j < (CP ? 0 : JA); ++j) {
      const double *tw = a.TW + ((size_t)j * KP + tq) * a.Tp + t0 + fl;
#pragma unroll
      for (int s = 0; s < NKS; ++s)
        twv[j][s] = SA ? es_ld<0>(es_rsrc(a.TW + t0), vo_tw, (unsigned)((j * KP + 4 * s) * a.Tp) * 8u)
                       : tw[(size_t)(4 * s) * a.Tp];
    }
    if constexpr (!CXE) load_cx(tt, cxv);  // this tile's Cx (in flight with the TW operands)
    __builtin_amdgcn_sched_barrier(0);
    d4 v[J];
    if constexpr (CP) {
      constexpr int CH = 8, CPS = NKS / CH, NCH = J * CPS, PD = 2;   // chunks, prefetch distance
      static_assert(NKS % CH == 0, "k chunks of 8");
      double ta[PD + 1][CH], wa[PD + 1][WL ? 1 : CH];
      auto ld = [&](int u, int sl) {
        const int j = u / CPS, s0 = (u % CPS) * CH;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const int s = s0 + c;
          ta[sl][c] = es_ld<0>(es_rsrc(a.TW + t0), vo_tw, (unsigned)((j * KP + 4 * s) * a.Tp) * 8u);
          if constexpr (!WL)
            wa[sl][c] = a.Wkf[lofs + ((size_t)j * KP + tq + 4 * s) * a.Fp + f];
        }
      };
#pragma unroll
      for (int u = 0; u < PD; ++u) ld(u, u);
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        if (u + PD < NCH) ld(u + PD, (u + PD) % (PD + 1));
        __builtin_amdgcn_sched_barrier(0);
        const int j = u / CPS, s0 = (u % CPS) * CH, sl = u % (PD + 1);
        if (s0 == 0) v[j] = d4{0.0, 0.0, 0.0, 0.0};
        const double *sw = s_w + lofs + (j * KP + tq) * 16 + fl;
#pragma unroll
        for (int c = 0; c < CH; ++c)
          v[j] = mfma4(ta[sl][c], WL ? sw[4 * (s0 + c) * 16] : wa[sl][WL ? 0 : c], v[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (VR && !(WL || NKS <= 16)) {
      // J > 4 at K = 128 (W from L2): a runtime loop over the sources, each
      // source's V tile a 4-chunk pipeline of 8 MFMAs with the next chunk's TW
      // and W operands in flight (the last chunk prefetches source j + 1's
      // first), written to the VST slab as soon as it is formed -- the fully
      // unrolled form crashes or spills (CP above); the inline loads left one
      // L2 round trip per source exposed (J = 8, K = 128: 6.85 ms)
      slab_fence0();   // the previous tile's last reads before these writes
      constexpr int CH = 8, CPS = NKS / CH;
      double ta[2][CH], wa[2][CH];
      auto ld = [&](int j, int s0, int sl) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          ta[sl][c] = es_ld<0>(es_rsrc(a.TW + t0), vo_tw, (unsigned)((j * KP + 4 * (s0 + c)) * a.Tp) * 8u);
          wa[sl][c] = a.Wkf[lofs + ((size_t)j * KP + tq + 4 * (s0 + c)) * a.Fp + f];
        }
      };
      ld(0, 0, 0);
#pragma unroll 1
      for (int j = 0; j < J; ++j) {
        d4 vj = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < CPS; ++c) {
          const int sl = c & 1;
          if (c + 1 < CPS)
            ld(j, (c + 1) * CH, sl ^ 1);
          else if (j + 1 < J)
            ld(j + 1, 0, sl ^ 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int cc = 0; cc < CH; ++cc) vj = mfma4(ta[sl][cc], wa[sl][cc], vj);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) wrv[i * 4 * S::VGS + (j >> 2) * 64 + (j & 3)] = vj[i];
      }
    } else if constexpr (VR) {
      // source j + 1's TW operands in flight while source j's MFMAs run; the
      // barriers keep the scheduler from hoisting every source's loads (at
      // K = 64 / 128 they alone would fill the register file)
      // (W from L2 at K = 128, J = 8: no prefetch, or the operands alone spill)
      constexpr bool PFS = WL || NKS <= 16;
      double tn[NKS];
#pragma unroll
      for (int s = 0; s < NKS; ++s) tn[s] = twv[0][s];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        double tc[NKS];
#pragma unroll
        for (int s = 0; s < NKS; ++s)
          tc[s] = PFS || j == 0 ? tn[s]
                               : es_ld<0>(es_rsrc(a.TW + t0), vo_tw, (unsigned)((j * KP + 4 * s) * a.Tp) * 8u);
        if (PFS && j + 1 < J) {
#pragma unroll
          for (int s = 0; s < NKS; ++s)
            tn[s] = es_ld<0>(es_rsrc(a.TW + t0), vo_tw, (unsigned)(((j + 1) * KP + 4 * s) * a.Tp) * 8u);
        }
        __builtin_amdgcn_sched_barrier(0);
        v[j] = d4{0.0, 0.0, 0.0, 0.0};
        const double *sw = s_w + lofs + (j * KP + tq) * 16 + fl;
        const double *gw = a.Wkf + lofs + ((size_t)j * KP + tq) * a.Fp + f;
#pragma unroll
        for (int s = 0; s < NKS; ++s)
          v[j] = mfma4(tc[s], WL ? sw[4 * s * 16] : gw[(size_t)(4 * s) * a.Fp], v[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int j = 0; j < ((VR || CP) ? 0 : J); ++j) {
      v[j] = d4{0.0, 0.0, 0.0, 0.0};
      const double *sw = s_w + lofs + (j * KP + tq) * 16 + fl;
      const double *gw = a.Wkf + lofs + ((size_t)j * KP + tq) * a.Fp + f;
      const double *tw = a.TW + ((size_t)j * KP + tq) * a.Tp + t0 + fl;
#pragma unroll
      for (int s = 0; s < NKS; ++s)
        v[j] = mfma4(j < JA ? twv[j < JA ? j : 0][s] : tw[(size_t)(4 * s) * a.Tp],
                     WL ? sw[4 * s * 16] : gw[(size_t)(4 * s) * a.Fp], v[j]);
    }
    if constexpr (VST && (WL || NKS <= 16)) {   // (else written by the loop above)
      slab_fence0();   // the previous tile's last reads before these writes
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) wrv[i * 4 * S::VGS + (j >> 2) * 64 + (j & 3)] = v[j][i];
    }
    const double *cj = s_cj + lofs + fl;
    // the lane's Sigma_x coefficients: LDS (re-read per tile) or, with
    // CJR, the registers loaded once per kernel
    auto cjv = [&](int j, int c) { return CJR ? cjr[j][c] : cj[(j * 4 + c) * 16]; };
    // point i of the lane's four (frame t0 + tq + 4 i): Sigma_x, its guarded
    // inverse, loglik, P = Cx S, N = S Cx S - S, and rho stored; no LDS
    auto pt_valu = [&](int i, double (&P)[8], double (&N)[4]) {
      const int t = t0 + tq + 4 * i;
      const double x00 = cxv[0][i], x11 = cxv[1][i], xr = cxv[2][i], xi = cxv[3][i];
      double V[J];
#pragma unroll
      for (int j = 0; j < J; ++j) V[j] = VST ? wrv[i * 4 * S::VGS + (j >> 2) * 64 + (j & 3)] : v[j][i];
      // Sigma_x = sum_r V_r a_r a_r^H + PSD I   (compute_suff_stat :613-652)
      double d0 = psd, d1 = psd, ore = 0.0, oim = 0.0;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        d0 += cjv(j, 0) * V[j];
        d1 += cjv(j, 1) * V[j];
        ore += cjv(j, 2) * V[j];
        oim += cjv(j, 3) * V[j];
      }
      // inv_herm_mat_2d (signalTools.py:177-194)
      double det = d0 * d1 - (ore * ore + oim * oim);
      const double dg = det + kEps;
      const double sg = dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0);
      det = sg * fmax(fabs(det), kEps);
      const double rdet = rcp_nr(det);
      const double i0 = d1 * rdet, i1 = d0 * rdet, ior = -ore * rdet, ioi = -oim * rdet;
      if (fvalid && t < a.T) {
        // log(det pi) as mantissa product x 2^exponent (v_frexp_*: 0, inf and
        // NaN pass through the mantissa, so log(lm) gives -inf / inf / NaN as
        // log() would; a negative det, which the guard only lets through for
        // a Sigma_x that is not positive semi-definite, is flagged in xmin)
        const double x = det * M_PI;
        lev += (double)__builtin_amdgcn_frexp_exp(x);
        lm *= __builtin_amdgcn_frexp_mant(x);
        xmin = fmin(xmin, x);
        ll += i0 * x00 + i1 * x11 + 2.0 * (ior * xr + ioi * xi);
      }
      // P = Cx S, N = S Cx S - S = P^H S - S
      P[0] = x00 * i0 + xr * ior + xi * ioi;   // p00r
      P[1] = xi * ior - xr * ioi;              // p00i
      P[2] = x00 * ior + xr * i1;              // p01r
      P[3] = x00 * ioi + xi * i1;              // p01i
      P[4] = xr * i0 + x11 * ior;              // p10r
      P[5] = -xi * i0 - x11 * ioi;             // p10i
      P[6] = xr * ior + xi * ioi + x11 * i1;   // p11r
      P[7] = xr * ioi - xi * ior;              // p11i
      N[0] = P[0] * i0 + (P[4] * ior - P[5] * ioi) - i0;          // n00
      N[1] = (P[2] * ior + P[3] * ioi) + P[6] * i1 - i1;          // n11
      N[2] = P[0] * ior + P[1] * ioi + P[4] * i1 - ior;           // n01r
      N[3] = P[0] * ioi - P[1] * ior - P[5] * i1 - ioi;           // n01i
      // hat_W[j] = mean over the ranks of j of |V^2 a_r^H N a_r + V| (:727-729,
      // :413-414) in the rank-merged form |V^2 (sum_r a_r^H N a_r) / rk + V|
      // (each rank's term is a posterior second moment, >= 0: the two forms
      // differ by rounding), with sum_r a_r^H N a_r = tr(N sum_r a_r a_r^H) from
      // the Sigma_x coefficients; stored as rho = (hat_W / vm^2) vm,
      // vm = max(V, eps): the FB ratio of update_spectral_components
      // (:1521-1575, N1), formed where V is at hand
      // Since V >= 0, rho = |V^2 q + V| / max(V, eps) = |V q + 1| min(V / eps, 1)
      // (q = a^H N a / rk): no reciprocal (the two forms differ by rounding)
      // NF: the factors 2 (the off-diagonal pair) and 1 / rk (a uniform rank)
      // folded into N once per point instead of once per source
      double Nf[4];
      {
        const double ir = RKU ? 1.0 / (double)RKU : 1.0;
        Nf[0] = N[0] * ir;
        Nf[1] = N[1] * ir;
        Nf[2] = N[2] * (2.0 * ir);
        Nf[3] = N[3] * (2.0 * ir);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const double Vj = V[j];
        double q;
        if constexpr (NF) {
          q = cjv(j, 0) * Nf[0] + cjv(j, 1) * Nf[1] + cjv(j, 2) * Nf[2] + cjv(j, 3) * Nf[3];
          if constexpr (RKU == 0) q *= inv_rk[j];
        } else {
          const double qa = (cjv(j, 0) * N[0] + cjv(j, 1) * N[1]) +
                            2.0 * (cjv(j, 2) * N[2] + cjv(j, 3) * N[3]);
          q = RKU == 1 ? qa : qa * inv_rk[j];
        }
        const double val = fabs(fma(Vj, q, 1.0)) * fmin(Vj * (1.0 / kEps), 1.0);
        if constexpr (SA)
          es_st<2>(val, es_rsrc(a.hatW + ((size_t)j * a.Tp + t0) * a.Fp), vo_cx,
                               (unsigned)(4 * i * a.Fp) * 8u);
        else
          __builtin_nontemporal_store(val, a.hatW + ((size_t)j * a.Tp + t) * a.Fp + f);
      }
    };
    // point i's MFMA operands -> the wave's slab (reader layout)
    auto pt_write = [&](int i, const double (&P)[8], const double (&N)[4]) {
      if constexpr (VST) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          wpn[0 * 64 + c] = P[c];
          wpn[1 * 64 + c] = P[4 + c];
          wpn[2 * 64 + c] = N[c];
        }
        return;
      }
      double V[J];
#pragma unroll
      for (int j = 0; j < J; ++j) V[j] = v[j][i];
#pragma unroll
      for (int j = 0; j < J; ++j) wr[(j >> 2) * 64 + (j & 3)] = V[j];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        wr[(S::SP + 0) * 64 + c] = P[c];
        wr[(S::SP + 1) * 64 + c] = P[4 + c];
        wr[S::SN * 64 + c] = N[c];
      }
      if constexpr (!RP) {
        int p = 0;
#pragma unroll
        for (int j1 = 0; j1 < J; ++j1)
#pragma unroll
          for (int j2 = j1; j2 < J; ++j2, ++p)
            wr[(S::SV2 + (p >> 2)) * 64 + (p & 3)] = V[j1] * V[j2];
      }
    };
    // SWP (J >= 4): the next point's VALU work sits between this point's slab
    // reads and its MFMAs (J = 4 with the reader-formed pairs: 0.370 -> 0.367
    // ms alone, 0.373 -> 0.3625 with CJR; with the writer-formed pairs it was
    // neutral; at J > 4 the unpipelined form also tripped ROCm 7.2's
    // AGPR-copy rewrite pass)
    constexpr bool SWP = J >= 4;

    auto slab_fence = [&]() {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // the slab's operands of the 4 bin groups in flight at once, then the
    // MFMAs (read -> wait -> MFMA one at a time left the LDS latency exposed);
    // with SWP the next point's VALU work sits between the reads and the
    // MFMAs (its slab writes after them)
    auto mfma_pass = [&](int i, auto between) {
      if constexpr (VST) {
        // the bin groups in two halves (half the operands live)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          double w[2][Q], pn[2][3];
#pragma unroll
          for (int g2 = 0; g2 < 2; ++g2) {
            const int g = 2 * hh + g2;
#pragma unroll
            for (int e = 0; e < Q; ++e) w[g2][e] = rdq[(4 * i + g) * S::VGS + vro[e]];
#pragma unroll
            for (int q = 0; q < 3; ++q) pn[g2][q] = rpn[g * S::PGS + q * 64];
          }
          __builtin_amdgcn_sched_barrier(0);
          if (hh == 0) {
            between();
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int g2 = 0; g2 < 2; ++g2) {
            const int g = 2 * hh + g2;
#pragma unroll
            for (int vg = 0; vg < NVG; ++vg) {
              xacc[g][vg][0] = mfma44(w[g2][4 * vg], pn[g2][0], xacc[g][vg][0]);
              xacc[g][vg][1] = mfma44(w[g2][4 * vg], pn[g2][1], xacc[g][vg][1]);
            }
#pragma unroll
            for (int h = 0; h < NPG; ++h)
              if (rp_live<J>(h))
                pacc[g][h] = mfma44(w[g2][rp_base<Q>(h)] * w[g2][(rp_base<Q>(h) + rp_d<Q>(h)) & (Q - 1)],
                                    pn[g2][2], pacc[g][h]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        return;
      }
      if constexpr (RP) {
        // rotated sources W_e, then P lo / hi and N, of the 4 bin groups
        double w[4][Q], pn[4][3];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int e = 0; e < Q; ++e) w[g][e] = rdq[g * S::GS + vro[e]];
#pragma unroll
          for (int q = 0; q < 3; ++q) pn[g][q] = rd[g * S::GS + (S::SP + q) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SWP) {
          between();
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int vg = 0; vg < NVG; ++vg) {
            xacc[g][vg][0] = mfma44(w[g][4 * vg], pn[g][0], xacc[g][vg][0]);
            xacc[g][vg][1] = mfma44(w[g][4 * vg], pn[g][1], xacc[g][vg][1]);
          }
#pragma unroll
          for (int h = 0; h < NPG; ++h)
            if (rp_live<J>(h))
              pacc[g][h] = mfma44(w[g][rp_base<Q>(h)] * w[g][(rp_base<Q>(h) + rp_d<Q>(h)) & (Q - 1)],
                                  pn[g][2], pacc[g][h]);
        }
        return;
      }
      double opd[4][S::NSET];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int q = 0; q < S::NSET; ++q) opd[g][q] = rd[g * S::GS + q * 64];
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (SWP) {
        between();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int vg = 0; vg < NVG; ++vg) {
          xacc[g][vg][0] = mfma44(opd[g][vg], opd[g][S::SP], xacc[g][vg][0]);
          xacc[g][vg][1] = mfma44(opd[g][vg], opd[g][S::SP + 1], xacc[g][vg][1]);
        }
#pragma unroll
        for (int h = 0; h < NPG; ++h)
          pacc[g][h] = mfma44(opd[g][S::SV2 + h], opd[g][S::SN], pacc[g][h]);
      }
    };
    if constexpr (SWP) {
      double Pc[8], Nc[4];
      pt_valu(0, Pc, Nc);
      pt_write(0, Pc, Nc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        slab_fence();   // point i's slab writes land before the cross-lane reads
        double Pn[8], Nn[4];
        mfma_pass(i, [&]() {
          if (i < 3) pt_valu(i + 1, Pn, Nn);
          if (CXE && i == 2 && tt + 4 < te) load_cx(tt + 4, cxv);
        });
        slab_fence();   // point i + 1's writes must not overtake point i's reads
        if (i < 3) pt_write(i + 1, Pn, Nn);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double P[8], N[4];
        pt_valu(i, P, N);
        pt_write(i, P, N);
        slab_fence();   // the slab writes land before the cross-lane reads
        mfma_pass(i, []() {});
        slab_fence();   // the next point's writes must not overtake these reads
      }
    }
    // keep lm in [0.5, 1): at most 4 factors >= 0.5 were multiplied in
    lev += (double)__builtin_amdgcn_frexp_exp(lm);
    lm = __builtin_amdgcn_frexp_mant(lm);
  }
  ll += (log(lm) + lev * M_LN2) + (xmin < 0.0 ? NAN : 0.0);

  // epilogue: lane (X = m, b, Y = n) holds, per bin group g, the 4x4 blocks
  // D[m][n] of bin f0 + 4g + b: cross (j = m, c = 4h + n), pairs (p = 4h + m, c = n)
  // (VR: pair m of group (base, d); the four waves' sums go through LDS one
  // bin group at a time, [4][NACC][4], to fit the smaller slab allocation)
#pragma unroll
  for (int mm = 1; mm < 64; mm <<= 1) ll += __shfl_xor(ll, mm, 64);
  if constexpr (VR) {
    static_assert(4 * NACC * 4 <= 4 * S::SLAB, "VR epilogue fits the slabs");
    const int m = lane >> 4, bb = (lane >> 2) & 3, n = lane & 3;
    double *red = s_slab;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __syncthreads();  // (g = 0: the slabs' last reads; else the previous group's sums)
#pragma unroll
      for (int vg = 0; vg < NVG; ++vg) {
        const int j = 4 * vg + m;
        if (j < J) {
          red[((wv * NACC) + 4 * NP + 8 * j + n) * 4 + bb] = xacc[g][vg][0];
          red[((wv * NACC) + 4 * NP + 8 * j + 4 + n) * 4 + bb] = xacc[g][vg][1];
        }
      }
#pragma unroll
      for (int h = 0; h < NPG; ++h) {
        const int p = rp_pair<J>(h, m);
        if (p >= 0) red[((wv * NACC) + 4 * p + n) * 4 + bb] = pacc[g][h];
      }
      __syncthreads();
      for (int idx = tid; idx < NACC * 4; idx += 256) {
        const int u = idx >> 2, ff = idx & 3;
        const double x = red[(0 * NACC + u) * 4 + ff] + red[(1 * NACC + u) * 4 + ff] +
                         red[(2 * NACC + u) * 4 + ff] + red[(3 * NACC + u) * 4 + ff];
        a.part[((size_t)(a.ybase + bi.y) * a.Fp + f0 + 4 * g + ff) * NACC + u] = x;
      }
    }
    if (lane == 0) s_ll[wv] = ll;
    __syncthreads();
    if (tid == 0)
      a.llpart[(a.ybase + bi.y) * a.nft + bi.x] = ((s_ll[0] + s_ll[1]) + s_ll[2]) + s_ll[3];
    return;
  }
  __syncthreads();  // s_red aliases the W tile and the slabs
  double *red = s_red + wv * NACC * 16;
  {
    const int m = lane >> 4, bb = (lane >> 2) & 3, n = lane & 3;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int bin = 4 * g + bb;
#pragma unroll
      for (int vg = 0; vg < NVG; ++vg) {
        const int j = 4 * vg + m;
        if (j < J) {
          red[(4 * NP + 8 * j + n) * 16 + bin] = xacc[g][vg][0];
          red[(4 * NP + 8 * j + 4 + n) * 16 + bin] = xacc[g][vg][1];
        }
      }
#pragma unroll
      for (int h = 0; h < NPG; ++h) {
        const int p = rp_pair<J>(h, m);
        if (p >= 0) red[(4 * p + n) * 16 + bin] = pacc[g][h];
      }
    }
  }
  if (lane == 0) s_ll[wv] = ll;
  __syncthreads();
  for (int idx = tid; idx < NACC * 16; idx += 256) {
    const int u = idx >> 4, ff = idx & 15;
    const double x = s_red[(0 * NACC + u) * 16 + ff] + s_red[(1 * NACC + u) * 16 + ff] +
                     s_red[(2 * NACC + u) * 16 + ff] + s_red[(3 * NACC + u) * 16 + ff];
    a.part[((size_t)(a.ybase + bi.y) * a.Fp + f0 + ff) * NACC + u] = x;
  }
  if (tid == 0)
    a.llpart[(a.ybase + bi.y) * a.nft + bi.x] = ((s_ll[0] + s_ll[1]) + s_ll[2]) + s_ll[3];
}

// ---------------------------------------------------------------- E-step, J > 8
// More than 8 sources (up to kMaxJ): the statistics no longer fit the
// single-pass kernel's registers (J (J + 1) / 2 pair and 8 J cross sums per
// bin), so the E-step runs in two passes over a scratch copy of its point
// quantities.  k_egen_point: one wave per 16 x 16 (bin, frame) tile, V_j on
// 16x16x4 MFMA (the k_estep_mx / k_wiener tile), then per point Sigma_x, its
// guarded inverse, the loglik term, P = Cx S, N = S Cx S - S and rho, with V_j,
// N and P written to frame-major scratch planes.  k_egen_stats: one block per
// (16-bin tile, frame chunk) sums the pair statistics V_j1 V_j2 N_c and the
// cross statistics V_j P_c over its frames (tiles staged in LDS) into the
// k_estep_mx partial layout, so k_mix reads it unchanged.
struct GArgs {
  double *V;     // [J][Tp][Fp]
  double *NP;    // [12][Tp][Fp]: N0..N3, P0..P7
  double *lw;    // [ntt][nft] per-wave loglik partials
  int J;
};

// V_j of the tile: per source, its NKS TW / W operand pairs in chunks of CH,
// every chunk's loads issued one chunk ahead of its MFMAs (two static register
// buffers; the unrolled (source, chunk) sequence fixes which), so a wave waits
// one memory round trip per chunk instead of one per MFMA.  The loads are
// unconditional (a chunk past source J - 1 re-reads its last), so every path
// reaches each wait with the same loads outstanding.
template <int NKS>
__global__ __launch_bounds__(64) void k_egen_point(const EArgs a, const GArgs g) {
  HALT_GUARD(a.halt);
  constexpr int CH = NKS < 8 ? NKS : 8, NCH = NKS / CH, NST = kMaxJ * NCH;
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int tt = blockIdx.x, ft = blockIdx.y, t0 = tt * 16, f0 = ft * 16, f = f0 + fl;
  const int J = g.J;
  __shared__ double s_c[kMaxJ][4][16];   // Sigma_x coefficients of the tile's bins
  __shared__ double s_irk[kMaxJ];
  double ta[2][CH], wa[2][CH];
  auto load = [&](int buf, int st) {
    const int j = min(st / NCH, J - 1), s0 = (st % NCH) * CH;
    const double *tw = a.TW + ((size_t)j * a.KP + tq + 4 * s0) * a.Tp + t0 + fl;
    const double *wk = a.Wkf + ((size_t)j * a.KP + tq + 4 * s0) * a.Fp + f;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      ta[buf][u] = tw[(size_t)(4 * u) * a.Tp];
      wa[buf][u] = wk[(size_t)(4 * u) * a.Fp];
    }
  };
  load(0, 0);
  // lane (fl, tq): the coefficients of sources tq, tq + 4, ... of bin fl
  for (int j = tq; j < J; j += 4) {
    double al = 0, be = 0, gr = 0, gi = 0;
    for (int r = a.roff[j]; r < a.roff[j + 1]; ++r) {
      const double2 a0 = a.A[(size_t)(2 * r) * a.Fp + f];
      const double2 a1 = a.A[(size_t)(2 * r + 1) * a.Fp + f];
      al += a0.x * a0.x + a0.y * a0.y;
      be += a1.x * a1.x + a1.y * a1.y;
      gr += a0.x * a1.x + a0.y * a1.y;
      gi += a0.y * a1.x - a0.x * a1.y;
    }
    s_c[j][0][fl] = al;
    s_c[j][1][fl] = be;
    s_c[j][2][fl] = gr;
    s_c[j][3][fl] = gi;
  }
  if (lane < J) s_irk[lane] = 1.0 / (double)(a.roff[lane + 1] - a.roff[lane]);
  d4 v[kMaxJ];
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) v[j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    const int j = st / NCH, cur = st & 1;
    if (j >= J) break;   // (wave-uniform)
    if (st + 1 < NST) load(cur ^ 1, st + 1);
    asm volatile("" ::: "memory");   // (keeps the prefetch here, not sunk past the next break)
#pragma unroll
    for (int u = 0; u < CH; ++u) v[j] = mfma4(ta[cur][u], wa[cur][u], v[j]);
  }
  __syncthreads();
  const size_t plane = (size_t)a.Tp * a.Fp;
  const double psd = a.psd[f];
  double ll = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + tq + 4 * i;
    const size_t o = (size_t)t * a.Fp + f;
    const double x00 = a.cx00[o], x11 = a.cx11[o], xr = a.cxr[o], xi = a.cxi[o];
    double d0 = psd, d1 = psd, ore = 0.0, oim = 0.0;
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j)
      if (j < J) {
        d0 += s_c[j][0][fl] * v[j][i];
        d1 += s_c[j][1][fl] * v[j][i];
        ore += s_c[j][2][fl] * v[j][i];
        oim += s_c[j][3][fl] * v[j][i];
      }
    // inv_herm_mat_2d (signalTools.py:177-194)
    double det = d0 * d1 - (ore * ore + oim * oim);
    const double dg = det + kEps;
    det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
    const double rdet = rcp_nr(det);
    const double i0 = d1 * rdet, i1 = d0 * rdet, ior = -ore * rdet, ioi = -oim * rdet;
    if (f < a.F && t < a.T) ll += log(det * M_PI) + (i0 * x00 + i1 * x11 + 2.0 * (ior * xr + ioi * xi));
    double P[8], N[4];
    P[0] = x00 * i0 + xr * ior + xi * ioi;
    P[1] = xi * ior - xr * ioi;
    P[2] = x00 * ior + xr * i1;
    P[3] = x00 * ioi + xi * i1;
    P[4] = xr * i0 + x11 * ior;
    P[5] = -xi * i0 - x11 * ioi;
    P[6] = xr * ior + xi * ioi + x11 * i1;
    P[7] = xr * ioi - xi * ior;
    N[0] = P[0] * i0 + (P[4] * ior - P[5] * ioi) - i0;
    N[1] = (P[2] * ior + P[3] * ioi) + P[6] * i1 - i1;
    N[2] = P[0] * ior + P[1] * ioi + P[4] * i1 - ior;
    N[3] = P[0] * ioi - P[1] * ior - P[5] * i1 - ioi;
#pragma unroll
    for (int c = 0; c < 4; ++c) g.NP[c * plane + o] = N[c];
#pragma unroll
    for (int c = 0; c < 8; ++c) g.NP[(4 + c) * plane + o] = P[c];
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j)
      if (j < J) {
        const double Vj = v[j][i];
        g.V[j * plane + o] = Vj;
        // rho = |V^2 q + V| / max(V, eps) = |V q + 1| min(V / eps, 1), q the
        // rank-merged quadratic form (as k_estep_mx)
        const double q = ((s_c[j][0][fl] * N[0] + s_c[j][1][fl] * N[1]) +
                          2.0 * (s_c[j][2][fl] * N[2] + s_c[j][3][fl] * N[3])) * s_irk[j];
        a.hatW[j * plane + o] = fabs(fma(Vj, q, 1.0)) * fmin(Vj * (1.0 / kEps), 1.0);
      }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) ll += __shfl_xor(ll, m, 64);
  if (lane == 0) g.lw[(size_t)tt * a.nft + ft] = ll;
}

// The statistics as 16x16x4 FP64 MFMAs per bin, frames as the k dimension:
// with A[m = j1][k = t] = V_j1(t) and B[k = t][n = j2] = V_j2(t) N_c(t),
// D[j1][j2] accumulates the pair sums of component c for all (j1, j2) at
// once (the j1 > j2 half is discarded), and B[k = t][n = c] = P_c(t) gives
// the cross sums D[j][c].  Lane (fl, tq) supplies the A and B operands of
// row/column fl and frame tq from one LDS read of V_fl(t).  Block = 8 waves
// on one (16-bin tile, frame chunk); wave wv owns bins 2 wv, 2 wv + 1 (five
// 16x16 accumulators each).  A frame tile's J + 12 planes are staged point-
// major in LDS ([16 frames][16 bins][RS], RS = (J + 12) | 1 so the 16 rows a
// wave reads land on distinct banks), the next tile's values already in
// flight in registers while the current one is summed.  (Was VALU pair FMAs
// over the same staged tile at 5.48 ms for J = 16 at C3's size;
// profiles/r6_struct_J16K32_sum.txt.)
constexpr int kEgsThreads = 512;
constexpr int kEgsRows = (kMaxJ + 12) | 1;
__global__ __launch_bounds__(kEgsThreads) void k_egen_stats(const EArgs a, const GArgs g) {
  HALT_GUARD(a.halt);
  const int J = g.J, NP = J * (J + 1) / 2, NACC = 4 * NP + 8 * J;
  const int tid = threadIdx.x, lane = tid & 63, fl = lane & 15, tq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ft = blockIdx.x, f0 = ft * 16, y = blockIdx.y;
  const int nr = J + 12, RS = nr | 1;
  extern __shared__ __attribute__((aligned(16))) double s_t[];   // [16 frames][16 bins][RS]
  d4 acc[2][5];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int c = 0; c < 5; ++c) acc[bi][c] = d4{0.0, 0.0, 0.0, 0.0};
  const size_t plane = (size_t)a.Tp * a.Fp;
  const int tb = a.tbase + y * a.tpc, te = min(tb + a.tpc, a.ntt);
  // staging: thread tid carries point e = tid & 255 of rows r = 2 k + (tid >> 8)
  // (wave-uniform: each row's plane is a scalar base, the point a 32-bit offset)
  const int e = tid & 255, rh = __builtin_amdgcn_readfirstlane(tid >> 8), etl = e >> 4, efl = e & 15;
  constexpr int kPre = (kMaxJ + 12 + 1) / 2;
  double pre[2][kPre];   // two tiles in flight
  // Loads and stores unconditional (rows past nr repeat the last; a tile
  // past the chunk re-reads its last and is never staged), so every path
  // reaches the loop head with the same two batches outstanding and the
  // older one is waited for alone.
  auto load = [&](double(&p)[kPre], int tt) {
    const unsigned o = (unsigned)((min(tt, te - 1) * 16 + etl) * a.Fp + f0 + efl);
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int r = min(2 * k + rh, nr - 1);
      const double *base = r < J ? g.V + r * plane : g.NP + (r - J) * plane;
      p[k] = __builtin_nontemporal_load(base + o);
    }
  };
  auto stage = [&](const double(&p)[kPre]) {
    __syncthreads();   // (the previous tile's reads)
#pragma unroll
    for (int k = 0; k < kPre; ++k) s_t[e * RS + min(2 * k + rh, nr - 1)] = p[k];
    __syncthreads();
  };
  // MFMA operands: lane (fl, tq) reads V_fl (fl < J), N_0..3 and P_fl (fl <
  // 8) of its point; out-of-range lanes read a valid slot and select zero
  const int vcol = min(fl, J - 1), xcol = J + 4 + (fl & 7);
  const bool vok = fl < J, xok = fl < 8;
  auto sum_tile = [&]() {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const int b = 2 * wv + bi;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double *pt = s_t + ((4 * q + tq) * 16 + b) * RS;   // point (frame 4 q + tq, bin b)
        const double vr = pt[vcol], pr = pt[xcol];
        const double n0 = pt[J], n1 = pt[J + 1], n2 = pt[J + 2], n3 = pt[J + 3];
        const double v = vok ? vr : 0.0, px = xok ? pr : 0.0;
        acc[bi][0] = mfma4(v, v * n0, acc[bi][0]);
        acc[bi][1] = mfma4(v, v * n1, acc[bi][1]);
        acc[bi][2] = mfma4(v, v * n2, acc[bi][2]);
        acc[bi][3] = mfma4(v, v * n3, acc[bi][3]);
        acc[bi][4] = mfma4(v, px, acc[bi][4]);
      }
    }
  };
  if (tb < te) {
    load(pre[0], tb);
    load(pre[1], tb + 1);
    for (int tt = tb; tt < te; tt += 2) {
      stage(pre[0]);
      load(pre[0], tt + 2);
      sum_tile();
      if (tt + 1 < te) {   // (block-uniform)
        stage(pre[1]);
        sum_tile();
      }
      load(pre[1], tt + 3);
    }
  }
  // lane (fl, tq), register i: D[tq + 4 i][fl]
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    double *out = a.part + ((size_t)(a.ybase + y) * a.Fp + f0 + 2 * wv + bi) * NACC;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j1 = tq + 4 * i, j2 = fl;
      if (j1 <= j2 && j2 < J) {
        const int p = j1 * J - j1 * (j1 - 1) / 2 + j2 - j1;   // canonical index of (j1, j2)
#pragma unroll
        for (int c = 0; c < 4; ++c) out[4 * p + c] = acc[bi][c][i];
      }
      if (j1 < J && fl < 8) out[4 * NP + 8 * j1 + fl] = acc[bi][4][i];
    }
  }
  if (tid == 0) {   // the chunk's loglik, its tiles in order
    double l = 0.0;
    for (int tt = tb; tt < te; ++tt) l += g.lw[(size_t)tt * a.nft + ft];
    a.llpart[(a.ybase + y) * a.nft + ft] = l;
  }
}

// Fused many-source E-step (J > 8, KP <= 32): k_egen_point's point pass and
// k_egen_stats' statistics in one block per (16-bin tile, frame chunk), V, N
// and P never leaving the LDS slab (the two-pass form writes and re-reads
// 28 planes, 4.6 GB at J = 16 and C3's size, and its point pass is bound by
// those writes; profiles/r6_ab_egen_point.txt).  Per frame tile, three phases
// between barriers:
//   V      wave wv forms V of sources 2 wv, 2 wv + 1 on 16x16x4 MFMA (its W
//          operands held in registers for the chunk, the next tile's TW
//          operands loaded while the current tile is summed) into the slab;
//   point  thread pair (2 e, 2 e + 1) owns point e: Sigma_x summed over the
//          even / odd sources and combined across the pair, then both form
//          the guarded inverse, P and N (the pair's halves write N and P to
//          the slab) and rho of their own sources to global;
//   stats  as k_egen_stats, from the slab.
template <int NKS>
__global__ __launch_bounds__(kEgsThreads) void k_egen_fused(const EArgs a, const GArgs g) {
  HALT_GUARD(a.halt);
  const int J = g.J, NP = J * (J + 1) / 2, NACC = 4 * NP + 8 * J;
  const int tid = threadIdx.x, lane = tid & 63, fl = lane & 15, tq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ft = blockIdx.x, f0 = ft * 16, y = blockIdx.y;
  const int nr = J + 12, RS = nr | 1;
  const int tb = a.tbase + y * a.tpc, te = min(tb + a.tpc, a.ntt);
  const size_t plane = (size_t)a.Tp * a.Fp;
  extern __shared__ __attribute__((aligned(16))) double s_t[];   // [256 points][RS], then W
  double *s_w = s_t + 256 * RS;           // [J][KP][16 bins]: the tile's W operands
  // Sigma_x coefficients per (source, component, bin), the source stride 80
  // doubles (= 16 mod 32 banks) so a half-wave's 16 bins x even / odd
  // sources fall on 32 distinct banks
  __shared__ double s_cfb[kMaxJ][80];
  auto cf = [&](int b, int j, int c) -> double & { return s_cfb[j][16 * c + b]; };
  __shared__ double s_irk[kMaxJ];
  __shared__ double s_ll[kEgsThreads / 64];
  if (tid < 16 * J) {
    const int j = tid >> 4, b = tid & 15, f = f0 + b;
    double al = 0, be = 0, gr = 0, gi = 0;
    for (int r = a.roff[j]; r < a.roff[j + 1]; ++r) {
      const double2 a0 = a.A[(size_t)(2 * r) * a.Fp + f];
      const double2 a1 = a.A[(size_t)(2 * r + 1) * a.Fp + f];
      al += a0.x * a0.x + a0.y * a0.y;
      be += a1.x * a1.x + a1.y * a1.y;
      gr += a0.x * a1.x + a0.y * a1.y;
      gi += a0.y * a1.x - a0.x * a1.y;
    }
    cf(b, j, 0) = al;
    cf(b, j, 1) = be;
    cf(b, j, 2) = gr;
    cf(b, j, 3) = gi;
  }
  if (tid < J) s_irk[tid] = 1.0 / (double)(a.roff[tid + 1] - a.roff[tid]);
  constexpr int KP = 4 * NKS;
  for (int idx = tid; idx < J * KP * 16; idx += kEgsThreads)
    s_w[idx] = a.Wkf[(size_t)(idx >> 4) * a.Fp + f0 + (idx & 15)];
  // V phase: sources ja, ja + 1 of this wave (clamped operands past J - 1)
  const int ja = 2 * wv, jA = min(ja, J - 1), jB = min(ja + 1, J - 1);
  const double *wA = s_w + (jA * KP + tq) * 16 + fl, *wB = s_w + (jB * KP + tq) * 16 + fl;
  double tr[2][NKS];
  auto load_tw = [&](int tt) {
    const int t = min(tt, te - 1) * 16 + fl;
    const double *tA = a.TW + ((size_t)jA * a.KP + tq) * a.Tp + t;
    const double *tB = a.TW + ((size_t)jB * a.KP + tq) * a.Tp + t;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      tr[0][s] = tA[(size_t)(4 * s) * a.Tp];
      tr[1][s] = tB[(size_t)(4 * s) * a.Tp];
    }
  };
  // point phase: point e = (frame tl, bin b), half h (even / odd sources)
  const int e = tid >> 1, h = tid & 1, tl = e >> 4, b = e & 15, f = f0 + b;
  const double psd = a.psd[f];
  double cx[4];
  auto load_cx = [&](int tt) {
    const size_t o = (size_t)(min(tt, te - 1) * 16 + tl) * a.Fp + f;
    cx[0] = a.cx00[o];
    cx[1] = a.cx11[o];
    cx[2] = a.cxr[o];
    cx[3] = a.cxi[o];
  };
  // statistics phase: v_mfma_f64_4x4x4_4b with block = bin (lane = 16 X +
  // 4 b + Y: A[m=Y][k=X], B[k=X][n=Y], D[m=X][n=Y] of block b), k = frame.
  // Wave wv owns bin quad bq = wv / 2 (bins 4 bq + b) and half hf = wv % 2:
  // the pair blocks (j1 block jb1 <= j2 block jb2, 4 sources each) of
  // components 2 hf, 2 hf + 1 and the cross blocks of sources 8 hf .. 8 hf + 7
  // -- 24 one-double accumulators, upper-triangle blocks only (40% fewer
  // matrix cycles than all 16 x 16 pairs on 16x16x4)
  const int X = lane >> 4, Yl = lane & 3, bq = wv >> 1, hf = wv & 1;
  const int sbin = 4 * bq + ((lane >> 2) & 3);
  double accp[10][2], accx[2][2];
#pragma unroll
  for (int pb = 0; pb < 10; ++pb) accp[pb][0] = accp[pb][1] = 0.0;
#pragma unroll
  for (int u = 0; u < 2; ++u) accx[u][0] = accx[u][1] = 0.0;
  double ll = 0.0;
  if (tb < te) {
    load_tw(tb);
    load_cx(tb);
  }
  for (int tt = tb; tt < te; ++tt) {
    __syncthreads();   // (the slab's previous readers; at the first tile, s_cf)
    {
      d4 vA = d4{0.0, 0.0, 0.0, 0.0}, vB = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        vA = mfma4(tr[0][s], wA[64 * s], vA);
        vB = mfma4(tr[1][s], wB[64 * s], vB);
      }
      load_tw(tt + 1);
      if (ja < J)   // (wave-uniform)
#pragma unroll
        for (int i = 0; i < 4; ++i) s_t[((tq + 4 * i) * 16 + fl) * RS + ja] = vA[i];
      if (ja + 1 < J)
#pragma unroll
        for (int i = 0; i < 4; ++i) s_t[((tq + 4 * i) * 16 + fl) * RS + ja + 1] = vB[i];
    }
    __syncthreads();
    {
      double *pt = s_t + e * RS;
      double d0 = 0.0, d1 = 0.0, ore = 0.0, oim = 0.0, vk[kMaxJ / 2];
#pragma unroll
      for (int m = 0; m < kMaxJ / 2; ++m) {
        const int j = 2 * m + h, jc = min(j, J - 1);
        vk[m] = pt[jc];   // (kept for rho below)
        const double vj = j < J ? vk[m] : 0.0;
        d0 = fma(cf(b, jc, 0), vj, d0);
        d1 = fma(cf(b, jc, 1), vj, d1);
        ore = fma(cf(b, jc, 2), vj, ore);
        oim = fma(cf(b, jc, 3), vj, oim);
      }
      d0 = psd + (d0 + __shfl_xor(d0, 1, 64));
      d1 = psd + (d1 + __shfl_xor(d1, 1, 64));
      ore += __shfl_xor(ore, 1, 64);
      oim += __shfl_xor(oim, 1, 64);
      const double x00 = cx[0], x11 = cx[1], xr = cx[2], xi = cx[3];
      load_cx(tt + 1);
      // inv_herm_mat_2d (signalTools.py:177-194)
      double det = d0 * d1 - (ore * ore + oim * oim);
      const double dg = det + kEps;
      det = (dg > 0.0 ? 1.0 : (dg < 0.0 ? -1.0 : 0.0)) * fmax(fabs(det), kEps);
      const double rdet = rcp_nr(det);
      const double i0 = d1 * rdet, i1 = d0 * rdet, ior = -ore * rdet, ioi = -oim * rdet;
      const int t = tt * 16 + tl;
      if (h == 0 && f < a.F && t < a.T)
        ll += log(det * M_PI) + (i0 * x00 + i1 * x11 + 2.0 * (ior * xr + ioi * xi));
      double P[8], N[4];
      P[0] = x00 * i0 + xr * ior + xi * ioi;
      P[1] = xi * ior - xr * ioi;
      P[2] = x00 * ior + xr * i1;
      P[3] = x00 * ioi + xi * i1;
      P[4] = xr * i0 + x11 * ior;
      P[5] = -xi * i0 - x11 * ioi;
      P[6] = xr * ior + xi * ioi + x11 * i1;
      P[7] = xr * ioi - xi * ior;
      N[0] = P[0] * i0 + (P[4] * ior - P[5] * ioi) - i0;
      N[1] = (P[2] * ior + P[3] * ioi) + P[6] * i1 - i1;
      N[2] = P[0] * ior + P[1] * ioi + P[4] * i1 - ior;
      N[3] = P[0] * ioi - P[1] * ior - P[5] * i1 - ioi;
      if (h == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) pt[J + c] = N[c];
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) pt[J + 4 + c] = P[c];
      }
      const size_t o = (size_t)t * a.Fp + f;
      // (sources past J - 1 clamp to J - 1 and store the very value its
      // owner stores -- both halves hold bit-identical N -- so the stores
      // need no lane-divergent branch)
#pragma unroll
      for (int m = 0; m < kMaxJ / 2; ++m) {
        const int j = min(2 * m + h, J - 1);
        // rho = |V q + 1| min(V / eps, 1), q the rank-merged quadratic form
        const double q = ((cf(b, j, 0) * N[0] + cf(b, j, 1) * N[1]) +
                          2.0 * (cf(b, j, 2) * N[2] + cf(b, j, 3) * N[3])) * s_irk[j];
        const double vj = vk[m];   // (= pt[j]: the same clamped source)
        __builtin_nontemporal_store(fabs(fma(vj, q, 1.0)) * fmin(vj * (1.0 / kEps), 1.0),
                                    a.hatW + j * plane + o);
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {
      const double *pt = s_t + ((4 * g + X) * 16 + sbin) * RS;   // point (frame 4 g + X, bin sbin)
      double va[4], bn[4][2], px[2];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int jj = 4 * jb + Yl;
        const double v = pt[min(jj, J - 1)];
        va[jb] = jj < J ? v : 0.0;
      }
      const double nc0 = pt[J + 2 * hf], nc1 = pt[J + 2 * hf + 1];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        bn[jb][0] = va[jb] * nc0;
        bn[jb][1] = va[jb] * nc1;
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) px[cb] = pt[J + 4 + 4 * cb + Yl];
      // (the ten blocks spelled out: constant register indices)
#define EGF_PB(pb, j1b, j2b)                                              \
  if (4 * (j2b) < J) {   /* (wave-uniform) */                             \
    accp[pb][0] = mfma44(va[j1b], bn[j2b][0], accp[pb][0]);              \
    accp[pb][1] = mfma44(va[j1b], bn[j2b][1], accp[pb][1]);              \
  }
      EGF_PB(0, 0, 0) EGF_PB(1, 0, 1) EGF_PB(2, 0, 2) EGF_PB(3, 0, 3) EGF_PB(4, 1, 1)
      EGF_PB(5, 1, 2) EGF_PB(6, 1, 3) EGF_PB(7, 2, 2) EGF_PB(8, 2, 3) EGF_PB(9, 3, 3)
#undef EGF_PB
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (4 * (2 * hf + u) >= J) continue;   // (wave-uniform)
        // (its own LDS read: selecting va[2 hf + u] became a scratch access)
        const int jj = 4 * (2 * hf + u) + Yl;
        const double vr = pt[min(jj, J - 1)], vs = jj < J ? vr : 0.0;
        accx[u][0] = mfma44(vs, px[0], accx[u][0]);
        accx[u][1] = mfma44(vs, px[1], accx[u][1]);
      }
    }
  }
  // lane (X, b, Y) holds D[X][Y] of its bin: pair (4 jb1 + X, 4 jb2 + Y),
  // cross (source 4 jb + X, component 4 cb + Y)
  {
    double *out = a.part + ((size_t)(a.ybase + y) * a.Fp + f0 + sbin) * NACC;
#pragma unroll
    for (int pb = 0; pb < 10; ++pb) {
      const int jb1 = pb < 4 ? 0 : pb < 7 ? 1 : pb < 9 ? 2 : 3;
      const int jb2 = pb < 4 ? pb : pb < 7 ? pb - 3 : pb < 9 ? pb - 5 : 3;
      const int j1 = 4 * jb1 + X, j2 = 4 * jb2 + Yl;
      if (j1 <= j2 && j2 < J) {
        const int p = j1 * J - j1 * (j1 - 1) / 2 + j2 - j1;   // canonical index of (j1, j2)
        out[4 * p + 2 * hf] = accp[pb][0];
        out[4 * p + 2 * hf + 1] = accp[pb][1];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 4 * (2 * hf + u) + X;
      if (j < J) {
        out[4 * NP + 8 * j + Yl] = accx[u][0];
        out[4 * NP + 8 * j + 4 + Yl] = accx[u][1];
      }
    }
  }
  // the chunk's loglik: lanes in order within a wave, then waves in order
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) ll += __shfl_xor(ll, m, 64);
  if (lane == 0) s_ll[wv] = ll;
  __syncthreads();
  if (tid == 0) {
    double l = 0.0;
    for (int w = 0; w < kEgsThreads / 64; ++w) l += s_ll[w];
    a.llpart[(a.ybase + y) * a.nft + ft] = l;
  }
}

// sum_t TW[j][k][t] (for mean_t V_j = W_j . sum_t H_j, the hat_Rss diagonal term)
__global__ void k_tw_rowsum(const double *__restrict__ TW, double *__restrict__ hsum, int T,
                            int Tp, const int *halt) {
  HALT_GUARD(halt);
  __shared__ double s[256];
  const double *row = TW + (size_t)blockIdx.x * Tp;
  double x = 0.0;
  for (int t = threadIdx.x; t < T; t += 256) x += row[t];
  s[threadIdx.x] = x;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) hsum[blockIdx.x] = s[0];
}

__global__ void k_loglik(const double *__restrict__ llpart, int n, double *__restrict__ out,
                         double inv_FT, const int *halt) {
  HALT_GUARD(halt);
  __shared__ double s[256];
  double x = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) x += llpart[i];
  s[threadIdx.x] = x;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = -(s[0] * inv_FT);
}

// sum_{c < n} p[c * stride] in index order (bit-identical to the plain loop)
// with 8 loads in flight: the chunk reductions below were load-latency bound
__device__ __forceinline__ double chunk_sum(const double *__restrict__ p, size_t stride, int n) {
  double x = 0.0;
  int c = 0;
  for (; c + 8 <= n; c += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(c + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) x += v[u];
  }
  for (; c < n; ++c) x += p[(size_t)c * stride];
  return x;
}

// ---------------------------------------------------------------- mixing
struct MArgs {
  const double *part;  // [nchunk][Fp][NACC]
  const double *Wkf;   // [J][KP][Fp]   (W before the spectral update)
  const double *hsum;  // [J][KP]       sum_t TW
  double2 *A;          // [R][2][Fp]
  double2 *rss, *rxs;  // inst: [Fp][R][R], [Fp][2][R]
  int *flags;
  int F, Fp, J, R, nchunk, nacc, conv_update, KP;
  double invT;
  int jr[kMaxR];
  const int *halt;
};

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 cadd(double2 a, double2 b) {
  return make_double2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ double2 csub(double2 a, double2 b) {
  return make_double2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ double2 cscale(double2 a, double s) {
  return make_double2(a.x * s, a.y * s);
}
__device__ __forceinline__ double2 cdiv(double2 a, double2 b) {
  // Smith's algorithm (as the C99 / numpy complex division)
  if (fabs(b.x) >= fabs(b.y)) {
    const double r = b.y / b.x, d = b.x + b.y * r;
    return make_double2((a.x + a.y * r) / d, (a.y - a.x * r) / d);
  }
  const double r = b.x / b.y, d = b.x * r + b.y;
  return make_double2((a.x * r + a.y) / d, (a.y * r - a.x) / d);
}

// One wave per bin f: sufficient statistics -> hat_Rss, hat_Rxs (:698-755),
// hermitised (:734-740); for 'conv' the per-bin solve hat_Rss^T X = hat_Rxs^T
// (:854-863) by LU with partial pivoting on |re|+|im| (LAPACK zgesv), the
// matrix entries spread over the lanes; for 'inst' the per-bin statistics are
// stored for k_mix_inst.
// QM: statistics per lane, ceil(NACC / 64) (2 at J = 4; the J > 8 models
// take the kMaxJ ceiling, the others stay at their own register count)
// RQ: hat_Rss entries per lane, ceil(R^2 / 64) (4 up to R = 16)
template <int QM, int RQ = 4>
__global__ __launch_bounds__(64) void k_mix(const MArgs a) {
  HALT_GUARD(a.halt);
  // LDS sized by this model's J, R, KP (mix_smem): with the kMaxJ / kMaxR /
  // kMaxKP ceilings a block took 19 KB, so only 8 blocks fit a CU and the
  // 2049 bins of C3 ran as two rounds of the whole latency chain
  extern __shared__ __attribute__((aligned(16))) double s_mix[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int J = a.J, R = a.R, NACC = a.nacc;
  const int W = R + 2;
  double2 *s_A = (double2 *)s_mix;           // [R][2]
  double2 *s_L = s_A + 2 * R;                // [R][R + 2]: [M^T | hat_Rxs^T]
  double2 *s_H = s_L + R * W;                // [R][R]
  double2 *s_mult = s_H + R * R;             // [R]
  double *s_acc = (double *)(s_mult + R);    // [NACC]
  double *s_sv = s_acc + NACC;               // [J]
  double *s_wh0 = s_sv + J;                  // [J * KP] W_j(f, k)
  double *s_wh1 = s_wh0 + J * a.KP;          // [J * KP] sum_t TW_j(k, t)
  const int NP = J * (J + 1) / 2;
  {  // NACC = 72 > 64 lanes for J = 4: a lane sums up to 4 statistics, the
     // loads of all of them for 8 chunks in flight together (chunk order kept)
    constexpr int kQ = QM;
    double x[kQ] = {};
    const size_t cs = (size_t)a.Fp * NACC;
    const double *p0 = a.part + (size_t)f * NACC + lane;
    for (int c = 0; c < a.nchunk; c += 8) {
      double v[kQ][8];
#pragma unroll
      for (int q = 0; q < kQ; ++q)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[q][u] = (lane + 64 * q < NACC && c + u < a.nchunk) ? p0[(size_t)(c + u) * cs + 64 * q] : 0.0;
#pragma unroll
      for (int q = 0; q < kQ; ++q)
#pragma unroll
        for (int u = 0; u < 8; ++u) x[q] += v[q][u];
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q)
      if (lane + 64 * q < NACC) s_acc[lane + 64 * q] = x[q];
  }
  if (lane < 2 * R) s_A[(lane >> 1) * 2 + (lane & 1)] = a.A[(size_t)lane * a.Fp + f];
  // sum_t V_j(f, t) = sum_k W_j(f, k) sum_t TW_j(k, t): the operands are
  // loaded by all lanes at once (a per-source loop over k was a chain of
  // global-latency round trips), then summed in k order
  for (int i = lane; i < J * a.KP; i += 64) {
    s_wh0[i] = a.Wkf[(size_t)i * a.Fp + f];
    s_wh1[i] = a.hsum[i];
  }
  __syncthreads();
  if (lane < J) {
    double sv = 0.0;
    for (int k = 0; k < a.KP; ++k) sv += s_wh0[lane * a.KP + k] * s_wh1[lane * a.KP + k];
    s_sv[lane] = sv;
  }
  __syncthreads();
  // hat_Rss entries (r1, r2), R^2 <= 256: four per lane at most
  for (int e = lane; e < R * R; e += 64) {
    const int r1 = e / R, r2 = e % R;
    const int j1 = a.jr[r1], j2 = a.jr[r2];
    const int lo = min(j1, j2), hi = max(j1, j2);
    const int p = lo * J - lo * (lo - 1) / 2 + (hi - lo);
    const double n00 = s_acc[4 * p], n11 = s_acc[4 * p + 1];
    const double2 n01 = make_double2(s_acc[4 * p + 2], s_acc[4 * p + 3]);
    const double2 c10 = cconj(s_A[(r1) * 2 + (0)]), c11 = cconj(s_A[(r1) * 2 + (1)]);
    double2 v = cscale(cmul(c10, s_A[(r2) * 2 + (0)]), n00);               // a_r1^H Nsum a_r2
    v = cadd(v, cmul(cmul(c10, n01), s_A[(r2) * 2 + (1)]));
    v = cadd(v, cmul(cmul(c11, cconj(n01)), s_A[(r2) * 2 + (0)]));
    v = cadd(v, cscale(cmul(c11, s_A[(r2) * 2 + (1)]), n11));
    v = cscale(v, a.invT);
    if (r1 == r2) v.x += s_sv[j1] * a.invT;
    s_H[(r1) * R + (r2)] = v;
  }
  __syncthreads();
  double2 hv[RQ];  // hermitised entries of this lane (e = lane + 64 q)
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int e = lane + 64 * q;
    hv[q] = make_double2(0.0, 0.0);
    if (e < R * R) {
      const int r1 = e / R, r2 = e % R;
      const double2 x = s_H[(r1) * R + (r2)], y = s_H[(r2) * R + (r1)];
      hv[q] = cscale(cadd(x, cconj(y)), 0.5);
    }
  }
  if (lane < 2 * R) {  // hat_Rxs[f][c][r] = sum_c' Q_j[c][c'] A_r,c' / T
    const int r = lane >> 1, c = lane & 1;
    const double *qq = s_acc + 4 * NP + 8 * a.jr[r];
    const double2 q0 = make_double2(qq[4 * c + 0], qq[4 * c + 1]);
    const double2 q1 = make_double2(qq[4 * c + 2], qq[4 * c + 3]);
    s_L[(r) * W + (R + c)] = cscale(cadd(cmul(q0, s_A[(r) * 2 + (0)]), cmul(q1, s_A[(r) * 2 + (1)])), a.invT);
  }
  if (!a.conv_update) {
    __syncthreads();
    if (a.rss) {
#pragma unroll
      for (int q = 0; q < RQ; ++q) {
        const int e = lane + 64 * q;
        if (e < R * R) a.rss[((size_t)f * R + e / R) * R + e % R] = hv[q];
      }
      if (lane < 2 * R) {
        const int r = lane >> 1, c = lane & 1;
        a.rxs[((size_t)f * 2 + c) * R + r] = s_L[(r) * W + (R + c)];
      }
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < RQ; ++q) {  // L = hermitised(hat_Rss)^T
    const int e = lane + 64 * q;
    if (e < R * R) s_L[(e % R) * W + (e / R)] = hv[q];
  }
  __syncthreads();
  for (int k = 0; k < R; ++k) {
    // pivot: first row i >= k maximising |re|+|im| of L[i][k]
    double m = -1.0;
    int mi = R;
    if (lane >= k && lane < R) {
      m = fabs(s_L[(lane) * W + (k)].x) + fabs(s_L[(lane) * W + (k)].y);
      mi = lane;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double om = __shfl_xor(m, off, 64);
      const int oi = __shfl_xor(mi, off, 64);
      if (om > m || (om == m && oi < mi)) {
        m = om;
        mi = oi;
      }
    }
    if (m == 0.0) {
      if (lane == 0) {
        atomicOr(a.flags, 1);
        atomicOr(a.flags + kFlagHalt, 1);
      }
      return;
    }
    if (mi != k && lane < W) {
      const double2 t = s_L[(k) * W + (lane)];
      s_L[(k) * W + (lane)] = s_L[(mi) * W + (lane)];
      s_L[(mi) * W + (lane)] = t;
    }
    __syncthreads();
    if (lane > k && lane < R) s_mult[lane] = cmul(s_L[(lane) * W + (k)], cdiv(make_double2(1.0, 0.0), s_L[(k) * W + (k)]));
    __syncthreads();
    const int nr = R - k - 1, nc = W - k - 1;
    for (int e = lane; e < nr * nc; e += 64) {
      const int i = k + 1 + e / nc, c = k + 1 + e % nc;
      s_L[(i) * W + (c)] = csub(s_L[(i) * W + (c)], cmul(s_mult[i], s_L[(k) * W + (c)]));
    }
    __syncthreads();
  }
  for (int i = R - 1; i >= 0; --i) {
    if (lane < 2) {
      double2 x = s_L[(i) * W + (R + lane)];
      for (int q = i + 1; q < R; ++q) x = csub(x, cmul(s_L[(i) * W + (q)], s_L[(q) * W + (R + lane)]));
      s_L[(i) * W + (R + lane)] = cdiv(x, s_L[(i) * W + (i)]);
    }
    __syncthreads();
  }
  if (lane < 2 * R) a.A[(size_t)lane * a.Fp + f] = s_L[(lane >> 1) * W + (R + (lane & 1))];
}

static size_t mix_smem(int J, int R, int KP, int nacc) {
  return (size_t)(2 * R + R * (R + 2) + R * R + R) * sizeof(double2) +
         (size_t)(nacc + J + 2 * J * KP) * sizeof(double);
}

// 'inst' update (:808-839): f-means of the statistics, real R_u x R_u solve.
struct IArgs {
  const double2 *rss, *rxs, *A;
  double2 *Pinst;
  int *flags;
  int F, Fp, R, nu, no;
  int upd[kMaxR], oth[kMaxR];
  const int *halt;
};
__global__ void k_mix_inst(const IArgs a) {
  HALT_GUARD(a.halt);
  __shared__ double s_b[kMaxR][2];
  __shared__ double s_m[kMaxR][kMaxR];
  const int nu = a.nu, R = a.R;
  const int tid = threadIdx.x;
  const int nb = 2 * nu, nm = nu * nu;
  // (2 nu + nu^2 reaches 288 at nu = 16: more entries than threads)
  for (int idx = tid; idx < nb + nm; idx += blockDim.x) {
    double s = 0.0;
    if (idx < nb) {
      const int c = idx / nu, u = idx % nu, ru = a.upd[u];
      for (int f = 0; f < a.F; ++f) {
        double2 x = a.rxs[((size_t)f * 2 + c) * R + ru];
        for (int o = 0; o < a.no; ++o) {
          const int ro = a.oth[o];
          x = csub(x, cmul(a.A[(size_t)(2 * ro + c) * a.Fp + f], a.rss[((size_t)f * R + ro) * R + ru]));
        }
        s += x.x;
      }
      s_b[u][c] = s / a.F;
    } else {
      const int e = idx - nb, u1 = e / nu, u2 = e % nu;
      for (int f = 0; f < a.F; ++f) s += a.rss[((size_t)f * R + a.upd[u1]) * R + a.upd[u2]].x;
      s_m[u1][u2] = s / a.F;
    }
  }
  __syncthreads();
  if (tid != 0) return;
  // (the serial solve on LDS copies: up to 32 x 32 would not fit registers)
  __shared__ double Lm[kMaxR][kMaxR], B[kMaxR][2];
  for (int i = 0; i < nu; ++i) {
    for (int k = 0; k < nu; ++k) Lm[i][k] = s_m[k][i];  // rm^T
    B[i][0] = s_b[i][0];
    B[i][1] = s_b[i][1];
  }
  for (int k = 0; k < nu; ++k) {
    int piv = k;
    double best = fabs(Lm[k][k]);
    for (int i = k + 1; i < nu; ++i)
      if (fabs(Lm[i][k]) > best) {
        best = fabs(Lm[i][k]);
        piv = i;
      }
    if (best == 0.0) {
      atomicOr(a.flags, 1);
      atomicOr(a.flags + kFlagHalt, 1);
      return;
    }
    if (piv != k) {
      for (int c = 0; c < nu; ++c) {
        const double t = Lm[k][c];
        Lm[k][c] = Lm[piv][c];
        Lm[piv][c] = t;
      }
      for (int c = 0; c < 2; ++c) {
        const double t = B[k][c];
        B[k][c] = B[piv][c];
        B[piv][c] = t;
      }
    }
    const double rinv = 1.0 / Lm[k][k];
    for (int i = k + 1; i < nu; ++i) {
      const double l = Lm[i][k] * rinv;
      for (int c = k + 1; c < nu; ++c) Lm[i][c] -= l * Lm[k][c];
      for (int c = 0; c < 2; ++c) B[i][c] -= l * B[k][c];
    }
  }
  for (int i = nu - 1; i >= 0; --i)
    for (int c = 0; c < 2; ++c) {
      double x = B[i][c];
      for (int q = i + 1; q < nu; ++q) x -= Lm[i][q] * B[q][c];
      B[i][c] = x / Lm[i][i];
    }
  for (int u = 0; u < nu; ++u)
    for (int c = 0; c < 2; ++c) a.Pinst[a.upd[u] * 2 + c] = make_double2(B[u][c], 0.0);
}

// ---------------------------------------------------------------- FB update
struct BArgs {
  const double *TW, *Wkf, *FWHt, *hatW;
  const double *hatW2;  // DEN: the denominator ratio plane (multi-block update)
  double *bnum;  // [nchunk][J][Fp][KP]
  double *bden;  // DEN: [nchunk][J][Fp][KP]
  int F, T, Fp, Tp, KP, J, ntt, nft, tpc;
  int zbase, tbase;  // this launch's chunks start at partial zbase, frame tile tbase (ntt = end)
  int fb_free[kMaxJ];
  const int *halt;
};

// FB numerator over t (:1521-1575), one wave per (FPW bin tiles, source,
// frame chunk):  num[f][k] = sum_t rho[f][t] (FW.H)^T[t][k] with
// rho = hat_W / V^2 * V formed by the E-step (N1: other_fact_power ==
// spat_comp_power == V).  The denominator sum_t (V * (1/V)) (FW.H)^T[t][k] is
// the f-independent sum_t (FW.H)^T[t][k] = (FW . rowsum(TW))[k] (to one
// rounding of V*(1/V)); k_fb_update forms it from hsum, and only the
// numerator is contracted here: a plain (F x T).(T x K) product whose rho
// tiles arrive bins-on-lanes, i.e. already in the A-operand layout, and whose
// (FW.H)^T B operand is shared by the FPW bin tiles.
// DEN (several spectral components on source j, audioModel.py:1525-1571):
// the numerator plane is (hat_W_j / V_j^2) other and a second plane
// other / V_j is contracted into the denominator the same way.
// Without DEN and FPW even the tiles are interleaved (bin f in tile f mod
// FPW), so each lane's rho values arrive as 16-byte loads (C3: 0.166 ->
// 0.155 ms at FPW = 2, same-box A/B).
template <int NKC, int FPW, bool DEN = false>
__global__ __launch_bounds__(64) void k_fb_contract(const BArgs a) {
  HALT_GUARD(a.halt);
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const dim3 bi = xcd_block();   // x: bin-tile group, y: source, z: frame chunk
  const int ft0 = bi.x * FPW, j = bi.y;
  if (!a.fb_free[j]) return;
  d4 num[FPW][NKC], den[DEN ? FPW : 1][NKC];
#pragma unroll
  for (int p = 0; p < FPW; ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) num[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < (DEN ? FPW : 1); ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) den[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
  const int tb = a.tbase + bi.z * a.tpc, te = min(tb + a.tpc, a.ntt);
  const double *rhoj = a.hatW + (size_t)j * a.Tp * a.Fp;
  const double *rdj = DEN ? a.hatW2 + (size_t)j * a.Tp * a.Fp : nullptr;
  for (int tt = tb; tt < te; ++tt) {
    const int t0 = tt * 16;
    double fb[4][NKC];
    const double *fwh = a.FWHt + ((size_t)j * a.Tp + t0 + tq) * a.KP + fl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) fb[i][kc] = fwh[(size_t)(4 * i) * a.KP + kc * 16];
    if constexpr (FPW % 2 == 0 && !DEN) {
      // the wave's FPW bin tiles interleaved: lane fl loads bins
      // FPW fl .. FPW fl + FPW - 1 of the 16 FPW-bin group with 16-byte loads
      // (tile p = the bins == p mod FPW): 4 rows x 16 FPW contiguous doubles
      // per load instruction instead of 4 x 16
      const int fp = ft0 * 16 + FPW * fl;
      double r[FPW][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = t0 + tq + 4 * i < a.T && fp < a.Fp;
        const double *src = rhoj + (size_t)(t0 + tq + 4 * i) * a.Fp + fp;
#pragma unroll
        for (int h = 0; h < FPW; h += 2) {
          const double2 v = ok ? *(const double2 *)(src + h) : make_double2(0.0, 0.0);
          r[h][i] = v.x;
          r[h + 1][i] = v.y;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int p = 0; p < FPW; ++p)
#pragma unroll
          for (int kc = 0; kc < NKC; ++kc) num[p][kc] = mfma4(r[p][i], fb[i][kc], num[p][kc]);
      continue;
    }
#pragma unroll
    for (int p = 0; p < FPW; ++p) {
      if (ft0 + p >= a.nft) break;  // wave-uniform: no bin tile left
      const int f = (ft0 + p) * 16 + fl;
      double r1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        r1[i] = t0 + tq + 4 * i < a.T ? rhoj[(size_t)(t0 + tq + 4 * i) * a.Fp + f] : 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) num[p][kc] = mfma4(r1[i], fb[i][kc], num[p][kc]);
      if constexpr (DEN) {
        double r2[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          r2[i] = t0 + tq + 4 * i < a.T ? rdj[(size_t)(t0 + tq + 4 * i) * a.Fp + f] : 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kc = 0; kc < NKC; ++kc) den[p][kc] = mfma4(r2[i], fb[i][kc], den[p][kc]);
      }
    }
  }
  const size_t base = ((size_t)(a.zbase + bi.z) * a.J + j) * a.Fp;
  if constexpr (FPW % 2 == 0 && !DEN) {   // interleaved tiles: tile p holds bins p mod FPW
#pragma unroll
    for (int p = 0; p < FPW; ++p)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int f = ft0 * 16 + FPW * (tq + 4 * m) + p;
          if (f < a.Fp) a.bnum[(base + f) * a.KP + kc * 16 + fl] = num[p][kc][m];
        }
    return;
  }
#pragma unroll
  for (int p = 0; p < FPW; ++p) {
    if (ft0 + p >= a.nft) break;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const size_t o = (base + (ft0 + p) * 16 + tq + 4 * m) * a.KP + kc * 16 + fl;
        a.bnum[o] = num[p][kc][m];
        if constexpr (DEN) a.bden[o] = den[DEN ? p : 0][kc][m];
      }
  }
}

struct UArgs {
  double *FB;
  const double *FW, *bnum, *hsum;
  const double *bden;  // null: den = FW . rowsum(TW); else contracted per (f, k)
  double *Wkf_new, *Wfk_new;
  int F, Fp, KP, J, nchunk;
  double omega;
  int kb0[kMaxJ], kb1[kMaxJ], fb_free[kMaxJ];  // columns [kb0, kb1) are updated
  // fused tail (pmax non-null): the renormalisation's stage-1 statistics of
  // this block's 16 bins, the FB column maxima [J][nft][KP] (the mixing
  // filters' energy is k_renorm_scales', read after the mixing update)
  double *pmax;
  const int *halt;
};
__device__ double block_sum(double x, double *s);
// FB *= (num / max(den, eps))^omega with den = FW . rowsum(TW) (see
// k_fb_contract) or, for one of several spectral components, the contracted
// denominator; then W_new = FB . FW in both layouts.
template <bool FWG>
__global__ __launch_bounds__(256) void k_fb_update(const UArgs a) {
  HALT_GUARD(a.halt);
  // LDS: FW [KP][KP] | FB rows [16][PB] | den [KP] | W_new rows [16][KP + 1]
  extern __shared__ __attribute__((aligned(16))) double s_fw[];
  const int f0 = blockIdx.x * 16, j = blockIdx.y;
  const int KP = a.KP;
  constexpr bool fwg = FWG;   // FW read from L2 (its [KP][KP] copy would not fit)
  const int PB = fwg ? KP + 1 : KP;   // (odd pitch: the MFMA B reads of 16 rows)
  const double *fw = fwg ? a.FW + (size_t)j * KP * KP : s_fw;
  double *s_fb = s_fw + (fwg ? 0 : KP * KP);
  double *s_den = s_fb + 16 * PB;
  double *s_wn = s_den + KP;
  if (!fwg)
    for (int idx = threadIdx.x; idx < KP * KP; idx += blockDim.x)
      s_fw[idx] = a.FW[(size_t)j * KP * KP + idx];
  for (int k = threadIdx.x; k < KP; k += blockDim.x) s_den[k] = a.hsum[(size_t)j * KP + k];
  __syncthreads();
  double dk = 0.0;
  if (threadIdx.x < KP)
    for (int q = 0; q < KP; ++q) dk += fw[threadIdx.x * KP + q] * s_den[q];
  __syncthreads();
  if (threadIdx.x < KP) s_den[threadIdx.x] = dk;
  __syncthreads();
  for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
    const int fl = idx / KP, k = idx % KP, f = f0 + fl;
    const size_t o = ((size_t)j * a.Fp + f) * KP + k;
    double fb = a.FB[o];
    if (a.fb_free[j] && f < a.F && k >= a.kb0[j] && k < a.kb1[j]) {
      double num = 0.0;
      num = chunk_sum(a.bnum + ((size_t)j * a.Fp + f) * KP + k, (size_t)a.J * a.Fp * KP, a.nchunk);
      const double den =
          a.bden ? chunk_sum(a.bden + ((size_t)j * a.Fp + f) * KP + k, (size_t)a.J * a.Fp * KP,
                             a.nchunk)
                 : s_den[k];
      const double ratio = num / fmax(den, kEps);
      fb *= a.omega == 1.0 ? ratio : pow(ratio, a.omega);
      a.FB[o] = fb;
    }
    s_fb[fl * PB + k] = fb;
  }
  __syncthreads();
  // W_new = FB . FW: [f][k] rows written coalesced over k here, the [k][f]
  // layout from the LDS copy below (coalesced over the 16 bins)
  if constexpr (fwg) {
    // KP = 128 on the matrix cores (as k_w_from_fb): D[k][f] = sum_q FW[q][k]
    // FB[f][q] per 16 x 16 tile, wave w forming the k tiles w, w + 4, ...
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, fl = lane & 15, tq = lane >> 4;
    for (int kc = wv; kc < KP / 16; kc += 4) {
      d4 d = d4{0.0, 0.0, 0.0, 0.0};
      for (int q0 = 0; q0 < KP; q0 += 4)
        d = mfma4(fw[(size_t)(q0 + tq) * KP + 16 * kc + fl], s_fb[fl * PB + q0 + tq], d);
#pragma unroll
      for (int i = 0; i < 4; ++i) s_wn[fl * (KP + 1) + 16 * kc + tq + 4 * i] = d[i];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
      const int fl = idx / KP, k = idx % KP;
      a.Wfk_new[((size_t)j * a.Fp + f0 + fl) * KP + k] = s_wn[fl * (KP + 1) + k];
    }
  } else {
    for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
      const int fl = idx / KP, k = idx % KP, f = f0 + fl;
      double s = 0.0;
      for (int q = 0; q < KP; ++q) s += s_fb[fl * KP + q] * fw[q * KP + k];
      a.Wfk_new[((size_t)j * a.Fp + f) * KP + k] = s;
      s_wn[fl * (KP + 1) + k] = s;
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 16 * KP; idx += blockDim.x) {
    const int k = idx / 16, fl = idx % 16;
    a.Wkf_new[((size_t)j * KP + k) * a.Fp + f0 + fl] = s_wn[fl * (KP + 1) + k];
  }
  if (!a.pmax) return;
  // renormalize_parameters' statistics of the updated FB rows (k_renorm_stats
  // per 16-bin block; max_f is exact in any order)
  const int nb = min(16, a.F - f0);
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    double m = -INFINITY;
    for (int fl = 0; fl < nb; ++fl) m = fmax(m, s_fb[fl * PB + k]);
    a.pmax[((size_t)j * gridDim.x + blockIdx.x) * KP + k] = m;
  }
}

// ---------------------------------------------------------------- FW update
// update_spectral_components, FW branch (audioModel.py:1578-1631), for the
// sources whose FW_frdm_prior is 'free'.  With one NMF factor other =
// max(V_old, eps) (N1) and the spatial power of the FW step is
// vm = max(V_mid, eps), V_mid = (FB_new FW_old) H (comp_spat_comp_power after
// the FB update, :1582-1588), so
//   num[k1][k2] = sum_f FB_new[f][k1] sum_t (hat_W / vm^2) other H[k2][t]
//   den[k1][k2] = sum_f FB_new[f][k1] sum_t (other / vm) H[k2][t]
// k_fw_contract forms the two ratio tiles (V_old and V_mid on the MFMA pipe,
// hat_W = rho * other from the E-step) and contracts them over t with H^T
// (G[f][k] per frame chunk, the k_fb_contract operand layout); k_fw_reduce
// contracts G with FB_new over bins (partials per bin chunk); k_fw_final
// applies FW *= (num / max(den, eps))^omega.
struct FWArgs {
  const double *TW, *TWt, *Wkf_old, *Wkf_mid, *hatW, *FB;
  double *gnum, *gden;  // [nchunk][J][Fp][KP]
  double *pnum, *pden;  // [nfc][J][KP][KP]
  double *FW;
  int F, T, Fp, Tp, KP, J, ntt, tpc, nchunk, nfc, fpc;
  int K[kMaxJ], fw_free[kMaxJ];
  int kb0[kMaxJ], kb1[kMaxJ];  // the FW block [kb0, kb1)^2 updated (BLK: the V tiles too)
  const double *cp, *pw;       // LAM: corrPen / powers planes of k_multi_prep
  double omega;
  const int *halt;
};

// BLK (one of several spectral components on source j): V_old / V_mid are the
// component's own powers (comp_spat_comp_power(..., spec_comp_ind=[k]),
// :1582-1588) and rho is the plane hat_W_j / max(V_c_old, eps).
template <int NKC, bool BLK = false, bool LAM = false>
__global__ __launch_bounds__(64) void k_fw_contract(const FWArgs a) {
  HALT_GUARD(a.halt);
  constexpr int NKS = 4 * NKC;
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int j = blockIdx.y;
  if (!a.fw_free[j]) return;
  const int f0 = blockIdx.x * 16, f = f0 + fl;
  const int KP = a.KP;
  double wo[NKS], wmid[NKS];  // B operands of the V tiles: W[k = tq + 4 s][f]
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    wo[s] = a.Wkf_old[((size_t)j * KP + tq + 4 * s) * a.Fp + f];
    wmid[s] = a.Wkf_mid[((size_t)j * KP + tq + 4 * s) * a.Fp + f];
    if constexpr (BLK) {
      const int k = tq + 4 * s;
      if (k < a.kb0[j] || k >= a.kb1[j]) wo[s] = wmid[s] = 0.0;
    }
  }
  d4 gn[NKC], gd[NKC];
#pragma unroll
  for (int kc = 0; kc < NKC; ++kc) gn[kc] = gd[kc] = d4{0.0, 0.0, 0.0, 0.0};
  const double *rhoj = a.hatW + (size_t)j * a.Tp * a.Fp;
  const int tb = blockIdx.z * a.tpc, te = min(tb + a.tpc, a.ntt);
  for (int tt = tb; tt < te; ++tt) {
    const int t0 = tt * 16;
    const double *tw = a.TW + ((size_t)j * KP + tq) * a.Tp + t0 + fl;
    d4 vo = d4{0.0, 0.0, 0.0, 0.0}, vm = vo;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const double h = tw[(size_t)(4 * s) * a.Tp];
      vo = mfma4(h, wo[s], vo);
      vm = mfma4(h, wmid[s], vm);
    }
    double rn[4], rd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + tq + 4 * i;
      const bool ok = t < a.T && f < a.F;
      const double rho = ok ? rhoj[(size_t)t * a.Fp + f] : 0.0;
      const double other = fmax(vo[i], kEps);
      const double rv = 1.0 / fmax(vm[i], kEps);
      if constexpr (LAM) {   // corrPen terms (audioModel.py:1596-1628)
        const size_t o = (size_t)j * a.Tp * a.Fp + (size_t)t * a.Fp + f;
        const double cp = ok ? a.cp[o] : 0.0, pw = ok ? a.pw[o] : 1.0;
        const double vmm = fmax(vm[i], kEps);
        rn[i] = ok ? ((rho * other) * (rv * rv) + cp * (2.0 * (vmm / pw))) * other : 0.0;
        rd[i] = ok ? other * (rv + cp) : 0.0;
      } else {
        rn[i] = ok ? ((rho * other) * (rv * rv)) * other : 0.0;  // (hat_W / vm^2) other
        rd[i] = ok ? other * rv : 0.0;                           // other (1 / vm)
      }
    }
    const double *ht = a.TWt + ((size_t)j * a.Tp + t0 + tq) * KP + fl;  // H^T[t][k]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        const double h = ht[(size_t)(4 * i) * KP + kc * 16];
        gn[kc] = mfma4(rn[i], h, gn[kc]);
        gd[kc] = mfma4(rd[i], h, gd[kc]);
      }
  }
  const size_t base = ((size_t)blockIdx.z * a.J + j) * a.Fp;
#pragma unroll
  for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const size_t o = (base + f0 + tq + 4 * m) * KP + kc * 16 + fl;
      a.gnum[o] = gn[kc][m];
      a.gden[o] = gd[kc][m];
    }
}

// partial FB_new^T G over the bins of chunk blockIdx.x (G summed over the
// frame chunks first, in chunk order)
__global__ __launch_bounds__(256) void k_fw_reduce(const FWArgs a) {
  HALT_GUARD(a.halt);
  const int j = blockIdx.y, fc = blockIdx.x;
  if (!a.fw_free[j]) return;
  const int KP = a.KP, K = a.K[j];
  extern __shared__ __attribute__((aligned(16))) double s_g[];  // [fpc][KP] x 3
  double *s_n = s_g, *s_d = s_g + a.fpc * KP, *s_b = s_g + 2 * a.fpc * KP;
  const int fb = fc * a.fpc, fe = min(fb + a.fpc, a.F), nf = fe - fb;
  for (int idx = threadIdx.x; idx < nf * KP; idx += blockDim.x) {
    const int fl = idx / KP, k = idx % KP, f = fb + fl;
    double n = 0.0, d = 0.0;
    for (int c = 0; c < a.nchunk; ++c) {
      const size_t o = (((size_t)c * a.J + j) * a.Fp + f) * KP + k;
      n += a.gnum[o];
      d += a.gden[o];
    }
    s_n[idx] = n;
    s_d[idx] = d;
    s_b[idx] = a.FB[((size_t)j * a.Fp + f) * KP + k];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) {
    const int k1 = idx / K, k2 = idx % K;
    double n = 0.0, d = 0.0;
    for (int fl = 0; fl < nf; ++fl) {
      const double b = s_b[fl * KP + k1];
      n += b * s_n[fl * KP + k2];
      d += b * s_d[fl * KP + k2];
    }
    const size_t o = (((size_t)fc * a.J + j) * KP + k1) * KP + k2;
    a.pnum[o] = n;
    a.pden[o] = d;
  }
}

__global__ __launch_bounds__(256) void k_fw_final(const FWArgs a) {
  HALT_GUARD(a.halt);
  const int j = blockIdx.x;
  if (!a.fw_free[j]) return;
  const int KP = a.KP, K = a.K[j];
  double *FW = a.FW + (size_t)j * KP * KP;
  for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) {
    const int k1 = idx / K, k2 = idx % K;
    double n = 0.0, d = 0.0;
    for (int fc = 0; fc < a.nfc; ++fc) {
      const size_t o = (((size_t)fc * a.J + j) * KP + k1) * KP + k2;
      n += a.pnum[o];
      d += a.pden[o];
    }
    if (k1 < a.kb0[j] || k1 >= a.kb1[j] || k2 < a.kb0[j] || k2 >= a.kb1[j]) continue;
    const double ratio = n / fmax(d, kEps);
    FW[k1 * KP + k2] *= a.omega == 1.0 ? ratio : pow(ratio, a.omega);
  }
}

// ---------------------------------------------------------------- TW update
struct TArgs {
  const double *TW, *Wkf_old, *Wkf_new, *Wfk_new, *hatW;
  double *tnum, *tden;  // [nsplit][J][Tp][KP]
  int F, T, Fp, Tp, KP, J, nft, ntt, fpc;
  int tw_free[kMaxJ];
  int kb0[kMaxJ], kb1[kMaxJ];  // BLK: the V tiles sum the columns [kb0, kb1) only
  const double *cp, *pw;       // LAM: corrPen / powers planes of k_multi_prep
  const double *oth;           // TBQ: max(V_c, eps) plane of k_multi_prep
  double omega;
  const int *halt;
};

// TW numerator / denominator over f (:1694-1726), one wave per (TPW frame
// tiles, source, bin chunk):
//   num[k][t] = sum_f W_new[f][k] * V_old * hat_W / V_new^2,
//   den[k][t] = sum_f W_new[f][k] * V_old / V_new
// V_old = W_old . TW, V_new = W_new . TW recomputed in registers, hat_W =
// rho * max(V_old, eps) from the E-step's rho; the W operands (A of the V
// tiles, B of the contraction) are shared by the TPW frame tiles.  Partial
// sums per bin chunk go to tnum / tden.
// BLK (one of several spectral components on source j): V_old / V_new are the
// component's own powers W_c H_c (the reference's spec_comp_ind=[k],
// audioModel.py:1639-1645), and rho is the plane hat_W_j / max(V_c_old, eps).
// TBQ (the TB step of a component with time blobs, :1931-1978): H has moved
// since the step's start, so other = max(V_c_old, eps) comes from a plane,
// hatW is hat_W_j itself, and num's ratio is hat_W / max(V_new^2, eps).
template <int NKC, int TPW, bool BLK = false, bool LAM = false, bool TBQ = false>
__global__ __launch_bounds__(64) void k_tw_contract(const TArgs a) {
  HALT_GUARD(a.halt);
  constexpr int NKS = 4 * NKC;
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const dim3 bi = xcd_block();   // x: frame-tile group, y: source, z: bin chunk
  const int tt0 = bi.x * TPW, j = bi.y;
  if (!a.tw_free[j]) return;
  double bt[TPW][NKS];
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    const bool tin = tt0 + p < a.ntt;
    const double *tw = a.TW + ((size_t)j * a.KP + tq) * a.Tp + (tt0 + p) * 16 + fl;
#pragma unroll
    for (int s = 0; s < NKS; ++s) bt[p][s] = tin ? tw[(size_t)(4 * s) * a.Tp] : 0.0;
  }
  d4 num[TPW][NKC], den[TPW][NKC];
#pragma unroll
  for (int p = 0; p < TPW; ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) num[p][kc] = den[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
  const int fb = bi.z * a.fpc, fe = min(fb + a.fpc, a.nft);
  // the V tiles' bin rows are permuted (lane fl's A row is bin
  // 4 (fl & 3) + (fl >> 2)) so that a lane's four D values are the four
  // consecutive bins 4 tq .. 4 tq + 3: its rho values arrive as two 16-byte
  // loads (C3: 0.401 -> 0.381 ms, same-box A/B); the contraction's B rows
  // (W_new) follow the same order
  const int fpl = 4 * (fl & 3) + (fl >> 2);
  const int bq = 4 * tq, bs = 1;   // D value i is bin f0 + bq + bs i
  const double *wo = a.Wkf_old + ((size_t)j * a.KP + tq) * a.Fp + fpl;
  const double *wn = a.Wkf_new + ((size_t)j * a.KP + tq) * a.Fp + fpl;
  const double *wfk = a.Wfk_new + ((size_t)j * a.Fp + bq) * a.KP + fl;
  const double *hwj = a.hatW + (size_t)j * a.Tp * a.Fp;
  for (int ft = fb; ft < fe; ++ft) {
    const int f0 = ft * 16;
    double ao[NKS], an[NKS], bw[4][NKC];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      ao[s] = TBQ ? 0.0 : wo[(size_t)(4 * s) * a.Fp + f0];
      an[s] = wn[(size_t)(4 * s) * a.Fp + f0];
      if constexpr (BLK) {
        const int k = tq + 4 * s;
        if (k < a.kb0[j] || k >= a.kb1[j]) ao[s] = an[s] = 0.0;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) bw[i][kc] = wfk[(size_t)(f0 + bs * i) * a.KP + kc * 16];
#pragma unroll
    for (int p = 0; p < TPW; ++p) {
      if (tt0 + p >= a.ntt) break;  // wave-uniform: no frame tile left
      const int t = (tt0 + p) * 16 + fl;
      double h[4];
      {  // (last use of rho: non-temporal)
        typedef double dv2 __attribute__((ext_vector_type(2)));
        const dv2 *hp = (const dv2 *)(hwj + (size_t)t * a.Fp + f0 + bq);
        const dv2 h01 = __builtin_nontemporal_load(hp), h23 = __builtin_nontemporal_load(hp + 1);
        h[0] = h01.x;
        h[1] = h01.y;
        h[2] = h23.x;
        h[3] = h23.y;
      }
      d4 vo = d4{0.0, 0.0, 0.0, 0.0}, vn = vo;
      d4 vo2 = vo, vn2 = vo;
#pragma unroll
      for (int s = 0; s < NKS; s += 2) {
        if constexpr (!TBQ) {
          vo = mfma4(ao[s], bt[p][s], vo);
          vo2 = mfma4(ao[s + 1], bt[p][s + 1], vo2);
        }
        vn = mfma4(an[s], bt[p][s], vn);
        vn2 = mfma4(an[s + 1], bt[p][s + 1], vn2);
      }
      vo += vo2;
      vn += vn2;
      {
        const bool tok = t < a.T;
        double r3[4], r4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double vm = fmax(vn[i], kEps);
          const double rv = rcp_nr(vm);
          const bool ok = tok && f0 + bq + bs * i < a.F;
          const size_t o = (size_t)j * a.Tp * a.Fp + (size_t)t * a.Fp + f0 + bq + bs * i;
          double other, q;
          if constexpr (TBQ) {
            other = ok ? a.oth[o] : 0.0;
            q = h[i] / fmax(vm * vm, kEps);   // hat_W / max(V^2, eps) (:1971-1973)
          } else {
            other = fmax(vo[i], kEps);
            q = (h[i] * other) * (rv * rv);   // hat_W from the E-step's rho
          }
          if constexpr (LAM) {   // corrPen terms (audioModel.py:1650-1719)
            const double cp = ok ? a.cp[o] : 0.0, pw = ok ? a.pw[o] : 1.0;
            r3[i] = ok ? other * (q + cp * (2.0 * (vm / pw))) : 0.0;
            r4[i] = ok ? other * (rv + cp) : 0.0;
          } else {
            r3[i] = ok ? other * q : 0.0;
            r4[i] = ok ? other * rv : 0.0;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kc = 0; kc < NKC; ++kc) {
            num[p][kc] = mfma4(r3[i], bw[i][kc], num[p][kc]);
            den[p][kc] = mfma4(r4[i], bw[i][kc], den[p][kc]);
          }
      }
    }
  }
  const size_t base = ((size_t)bi.z * a.J + j) * a.Tp;
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    if (tt0 + p >= a.ntt) break;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const size_t o = (base + (tt0 + p) * 16 + tq + 4 * m) * a.KP + kc * 16 + fl;
        a.tnum[o] = num[p][kc][m];
        a.tden[o] = den[p][kc][m];
      }
  }
}

// k_tw_contract's plain form (one spectral component per source, no
// lambdaCorr / time blobs, KP <= 64) with its per-bin-step operands staged in
// LDS by LDS-DMA (raw-buffer loads ... lds: no VGPR cost, NS stages in
// flight): a block of NW waves shares one source and bin chunk, wave w owns
// TPW frame tiles.  Stage c (bin tile fb + c) holds
//   Wo [KP][16]  W_old rows      (Wkf_old: KP / 8 pieces of 8 rows x 128 B;
//                not with SO)
//   Wn [KP][16]  W_new rows      (Wkf_new)
//   Wf [16][KP]  W_new, [f][k]   (Wfk_new, 16 KP contiguous doubles; a row r
//                with bit 2 set has its 128-B halves swapped, so the rows 4
//                apart that one ds_read_b64 lane group reads hit disjoint
//                bank halves; the DMA source applies the same involution)
//   rho [NW][TPW][8 granules][16 frames] x 16 B: the wave's own rho tiles,
//                granule-major so a lane's four consecutive bins are two
//                conflict-free ds_read_b128
// One s_barrier per bin step: wait (counted vmcnt) for the wave's own stage c
// pieces -> barrier -> issue stage c + NS - 1 into the buffer stage c - 1
// left -> compute stage c.  The arithmetic is k_tw_contract's, term for term.
template <int NKC, int NW, int TPW, int NS>
struct TwlCfg {
  static constexpr int NKC_ = NKC, NW_ = NW, TPW_ = TPW, NS_ = NS, NT = 64 * NW;
  static constexpr int KP = 16 * NKC;
  static constexpr int NWO = KP / 8;                // W pieces: Wo, Wn, Wf
  static constexpr int WPI = 3 * NWO;               // 1 KB W pieces per stage
  static constexpr int WD = 128 * WPI;              // W doubles per stage
  static constexpr int WN0 = 16 * KP, WF0 = 32 * KP;   // Wn / Wf offsets
  static constexpr int RD = 256;                    // rho doubles per frame tile
  static constexpr int SS = WD + NW * TPW * RD;     // doubles per stage
  static constexpr size_t smem = (size_t)NS * SS * sizeof(double);
  static constexpr int WPW = (WPI + NW - 1) / NW;   // W pieces per wave (upper bound)
  static constexpr int LPC = WPI / NW + 2 * TPW;    // loads per wave per stage (lower bound)
};

typedef __attribute__((address_space(3))) void lds_void_t;

// (the body is a device function: the host pass of a kernel template
// analyses its body, and the AMDGPU buffer-resource builtins do not exist there)
template <class CF>
__device__ __forceinline__ void tw_contract_lds_body(const TArgs &a);
template <class CF>
__global__ __launch_bounds__(CF::NT) FASST_NO_LDS_PAIRING
void k_tw_contract_lds(const TArgs a) {
  tw_contract_lds_body<CF>(a);
}
template <class CF>
__device__ __forceinline__ void tw_contract_lds_body(const TArgs &a) {
  HALT_GUARD(a.halt);
  constexpr int NKC = CF::NKC_, NW = CF::NW_, TPW = CF::TPW_, NS = CF::NS_;
  constexpr int KP = CF::KP, NKS = 4 * NKC, SS = CF::SS, WPI = CF::WPI, NWO = CF::NWO;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // (wv through readfirstlane: the compiler then knows it is wave-uniform, so
  // the piece / tile branches below are scalar, not exec-masked waterfalls)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fl = lane & 15, tq = lane >> 4;
  const dim3 bi = xcd_block();   // x: frame-tile group, y: source, z: bin chunk
  const int j = bi.y;
  if (!a.tw_free[j]) return;
  const int tt0 = (bi.x * NW + wv) * TPW;   // this wave's first frame tile
  const int fb = bi.z * a.fpc, fe = min(fb + a.fpc, a.nft), nst = fe - fb;
  // TW operands of the V tiles (resident for the whole bin loop)
  double bt[TPW][NKS];
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    const bool tin = tt0 + p < a.ntt;
    const double *tw = a.TW + ((size_t)j * a.KP + tq) * a.Tp + (tt0 + p) * 16 + fl;
#pragma unroll
    for (int s = 0; s < NKS; ++s) bt[p][s] = tin ? tw[(size_t)(4 * s) * a.Tp] : 0.0;
  }
  // (retire them before the first DMA: a use of an ordinary load while LDS-DMA
  // is in flight would drain the DMA ring)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // buffer resources: W rows of source j, its rho plane
  const unsigned wbytes = (unsigned)((size_t)KP * a.Fp * sizeof(double));
  const unsigned pbytes = (unsigned)((size_t)a.Tp * a.Fp * sizeof(double));
  const __amdgpu_buffer_rsrc_t rWo = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.Wkf_old + (size_t)j * KP * a.Fp), 0, wbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rWn = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.Wkf_new + (size_t)j * KP * a.Fp), 0, wbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rWf = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.Wfk_new + (size_t)j * a.Fp * KP), 0, wbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.hatW + (size_t)j * a.Tp * a.Fp), 0, pbytes, 0x00020000);
  // per-lane byte offsets of this wave's pieces (loop-invariant; the bin
  // step's offset rides in the SGPR soffset)
  constexpr int WPW = CF::WPW;
  static_assert(WPW <= 8, "W pieces per wave");
  unsigned wvo[8];
#pragma unroll
  for (int r = 0; r < WPW; ++r) {
    const int p = wv + NW * r;
    unsigned o = 0;
    if (p < NWO + KP / 8) {          // Wo / Wn: row 8 p' + lane / 8, granule lane % 8
      const int pp = p < NWO ? p : p - NWO, k = 8 * pp + (lane >> 3);
      o = (unsigned)(((size_t)k * a.Fp + 2 * (lane & 7)) * sizeof(double));
    } else if (p < WPI) {            // Wf: LDS position P -> element P ^ swz
      const int P = (p - NWO - KP / 8) * 128 + 2 * lane;
      const int e = P ^ ((((P / KP) >> 2) & 1) << 4);
      o = (unsigned)(e * sizeof(double));
    }
    wvo[r] = o;
  }
  unsigned rvo[TPW][2];
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    // frame tiles past the last one re-read the last (never used)
    const int tt = min(tt0 + p, a.ntt - 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int g = 4 * q + (lane >> 4);
      rvo[p][q] = (unsigned)(((size_t)(tt * 16 + fl) * a.Fp + 2 * g) * sizeof(double));
    }
  }
  auto issue = [&](int c) {   // stage c (bin tile fb + c) into buffer c % NS
    double *st = smem + (c % NS) * SS;
    const int f0 = (fb + c) * 16;
#pragma unroll
    for (int r = 0; r < WPW; ++r) {
      const int p = wv + NW * r;
      // (wave-uniform branches: one resource per call, never a runtime
      // select of a 128-bit resource)
      lds_void_t *d = (lds_void_t *)(st + 128 * p);
      if (p < NWO)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rWo, d, 16, wvo[r], f0 * 8, 0, 0);
      else if (p < NWO + KP / 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rWn, d, 16, wvo[r], f0 * 8, 0, 0);
      else if (p < WPI)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rWf, d, 16, wvo[r], f0 * KP * 8, 0, 0);
    }
    double *sr = st + CF::WD + wv * TPW * CF::RD;
#pragma unroll
    for (int p = 0; p < TPW; ++p)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rR, (lds_void_t *)(sr + p * CF::RD + 128 * q), 16,
                                                 rvo[p][q], f0 * 8, 0, 0);
  };
  d4 num[TPW][NKC], den[TPW][NKC];
#pragma unroll
  for (int p = 0; p < TPW; ++p)
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) num[p][kc] = den[p][kc] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < NS - 1; ++c)
    if (c < nst) issue(c);
  // lane's LDS read offsets (doubles) inside a stage
  const int fpl = 4 * (fl & 3) + (fl >> 2);   // V-tile bin row permutation (k_tw_contract)
  const int ow = tq * 16 + fpl;   // Wo / Wn: row tq + 4 s at + 64 s
  // Wf element (4 tq + i, 16 kc + fl) sits at (4 tq + i) KP + 16 kc + fl
  // with bit 4 flipped for odd tq: + 16 where the flipped bit was 0 (even kc,
  // or even i at KP = 16, where bit 4 is the row's low bit), - 16 otherwise
  const int s1 = (tq & 1) << 4;
  const int ofp = CF::WF0 + 4 * tq * KP + fl + s1, ofm = ofp - 2 * s1;
  const int orr = CF::WD + wv * TPW * CF::RD + (2 * tq * 16 + fl) * 2;   // granules 2 tq, 2 tq + 1
  for (int c = 0; c < nst; ++c) {
    // this wave's stage c pieces have landed (younger stages may still fly)
    const int ahead = min(NS - 2, nst - 1 - c);
    if (NS >= 3 && ahead >= 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CF::LPC < 63 ? CF::LPC : 63) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's stage c is in; stage c - 1 is read
    if (c + NS - 1 < nst) issue(c + NS - 1);
    const double *st = smem + (c % NS) * SS;
#pragma unroll
    for (int p = 0; p < TPW; ++p) {
      if (tt0 + p >= a.ntt) break;  // wave-uniform: no frame tile left
      typedef double dv2 __attribute__((ext_vector_type(2)));
      const dv2 h01 = *(const dv2 *)(st + orr + p * CF::RD);
      const dv2 h23 = *(const dv2 *)(st + orr + p * CF::RD + 32);
      const double h[4] = {h01.x, h01.y, h23.x, h23.y};
      // (this kernel is bound by MFMA + VALU issue, which do not overlap on
      // gfx950: one accumulation chain per V tile, one Newton step on
      // v_rcp_f64, no padding masks -- a bin past F meets W_new's zero rows
      // in the contraction, a frame past T lands in num / den columns
      // k_tw_update never reads, and every padded operand is finite)
      d4 vo = d4{0.0, 0.0, 0.0, 0.0}, vn = vo;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        vo = mfma4(st[ow + 64 * s], bt[p][s], vo);
        vn = mfma4(st[CF::WN0 + ow + 64 * s], bt[p][s], vn);
      }
      double r3[4], r4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double vm = vmax_f64(vn[i], kEps);
        double rv = __builtin_amdgcn_rcp(vm);
        rv = fma(fma(-vm, rv, 1.0), rv, rv);
        const double other = vmax_f64(vo[i], kEps);
        r4[i] = other * rv;                // other / V_new
        r3[i] = (h[i] * r4[i]) * r4[i];    // other hat_W / V_new^2, hat_W = rho other
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
          const bool ev = ((KP == 16 ? i : kc) & 1) == 0;
          const double bw = st[(ev ? ofp : ofm) + i * KP + kc * 16];
          num[p][kc] = mfma4(r3[i], bw, num[p][kc]);
          den[p][kc] = mfma4(r4[i], bw, den[p][kc]);
        }
    }
  }
  const size_t base = ((size_t)bi.z * a.J + j) * a.Tp;
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    if (tt0 + p >= a.ntt) break;
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const size_t o = (base + (tt0 + p) * 16 + tq + 4 * m) * a.KP + kc * 16 + fl;
        a.tnum[o] = num[p][kc][m];
        a.tden[o] = den[p][kc][m];
      }
  }
}

struct TUArgs {
  double *TW;
  const double *tnum, *tden;
  int T, Tp, KP, J, nsplit;
  double omega;
  int kb0[kMaxJ], kb1[kMaxJ], tw_free[kMaxJ];  // rows [kb0, kb1) are updated
  // fused tail (scal non-null): the renormalisation's TW column scale w2
  // (k_renorm_scales) applied after the update to the K[j] live rows, and the
  // restart test's partial sums per block into tpart [slot][ntb]
  const double *scal;
  double *tpart;
  int ntb, K[kMaxJ], soff[kMaxJ];
  // and (FWHt non-null) the next iteration's spectral-update
  // operands from the final TW of its 64 frames: FWHt = (FW TW)^T with the
  // renormalised FW (k_fwh_t's sum), and per-block TW row sums hpart
  // [J][KP][ntb] (k_tw_rowsum's; reduced in k_renorm_tail)
  const double *FW;
  double *FWHt, *hpart;
  const int *halt;
};
// TW *= (sum_chunks num / max(sum_chunks den, eps))^omega   (:1718-1726)
__global__ __launch_bounds__(256) void k_tw_update(const TUArgs a) {
  HALT_GUARD(a.halt);
  __shared__ double s_r[64][65];
  // (prep: the block's final TW rows [KP][64], padding rows / frames 0)
  extern __shared__ __attribute__((aligned(16))) double s_y[];
  const int j = blockIdx.y, t0 = blockIdx.x * 64;
  if (a.scal) {
    // y = fl(fl(TW r) w2): the two roundings of k_tw_update then k_renorm_apply
    const bool fr = a.tw_free[j];
    const double *w2 = a.scal + (size_t)j * (2 + 2 * a.KP) + 2 + a.KP;
    const bool prep = a.FWHt != nullptr;
    if (prep)
      for (int idx = threadIdx.x; idx < a.KP * 64; idx += blockDim.x) s_y[idx] = 0.0;
    // the prep's FW values (4 per thread: all of them at KP = 32) in flight
    // from the start; the source's FW block is in range for every idx < KP^2
    double fwv[4];
    if (prep)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = min((int)threadIdx.x + 256 * e, a.KP * a.KP - 1), k = idx / a.KP, q = idx % a.KP;
        fwv[e] = a.FW[(size_t)j * a.KP * a.KP + (size_t)k * a.KP + q];
      }
    double tsum = 0.0;
    for (int kb = 0; kb < a.K[j]; kb += 64) {
      const int kn = min(64, a.K[j] - kb);
      // the block's TW values in flight before the ratio loads (their two
      // latency chains overlap); raw-buffer loads on the source's plane, an
      // offset past it (elements past kn, frames past Tp) reads 0
      const __amdgpu_buffer_rsrc_t rtw = __builtin_amdgcn_make_buffer_rsrc(
          a.TW + (size_t)j * a.KP * a.Tp, 0, (int)((size_t)a.KP * a.Tp * 8), 0x00020000);
      // (8 per thread: all of them at K <= 32; the rest load in place)
      double xv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int idx = threadIdx.x + 256 * e, kl = idx / 64, tl = idx % 64;
        const unsigned vo = idx < 64 * kn ? (unsigned)(((kb + kl) * a.Tp + t0 + tl) * 8) : 0x7ffffff0u;
        xv[e] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rtw, (int)vo, 0, 0));
      }
      if (fr)
        for (int idx = threadIdx.x; idx < 64 * kn; idx += blockDim.x) {
          const int tl = idx / kn, kl = idx % kn, t = t0 + tl;
          double r = 1.0;
          if (t < a.T) {
            double num = 0.0, den = 0.0;
            for (int c = 0; c < a.nsplit; ++c) {
              const size_t o = (((size_t)c * a.J + j) * a.Tp + t) * a.KP + kb + kl;
              num += a.tnum[o];
              den += a.tden[o];
            }
            const double ratio = num / fmax(den, kEps);
            r = a.omega == 1.0 ? ratio : pow(ratio, a.omega);
          }
          s_r[kl][tl] = r;
        }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int idx = threadIdx.x + 256 * e;
        const int kl = idx / 64, tl = idx % 64, t = t0 + tl, k = kb + kl;
        if (idx < 64 * kn && t < a.T) {
          double *p = a.TW + ((size_t)j * a.KP + k) * a.Tp + t;
          double x = e < 8 ? xv[e < 8 ? e : 0] : *p;
          if (fr && k >= a.kb0[j] && k < a.kb1[j]) x *= s_r[kl][tl];
          const double y = x * w2[k];
          *p = y;
          tsum += y;
          if (prep) s_y[k * 64 + tl] = y;
        }
      }
      __syncthreads();
    }
    tsum = block_sum(tsum, &s_r[0][0]);
    if (threadIdx.x == 0) a.tpart[(size_t)a.soff[j] * a.ntb + blockIdx.x] = tsum;
    if (!prep) return;
    // FW (renormalised by k_renorm_rows, which this launch waits for)
    // transposed into s_r, s_fw[q][k] = FW[k][q], QB rows q at a time (all of
    // them at KP <= 64, the only sizes spectral_update asks this for)
    const int KP = a.KP;
    double *s_fw = &s_r[0][0];
    const double *gfw = a.FW + (size_t)j * KP * KP;
    const int QB = KP <= 64 ? KP : 32;
    // FWHt^T tiles on the matrix cores: wave w forms frames 16 w .. 16 w + 15,
    // D[k][t] = sum_q FW[k][q] y[q][t] (16x16x4 per 16 k x 4 q); lane (fl,
    // tq) then holds FWHt[16 w + fl][16 kc + tq + 4 i]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, fl = lane & 15, tq = lane >> 4;
    const int tn = min(64, a.Tp - t0);
    d4 d[kMaxKP / 16];
#pragma unroll
    for (int kc = 0; kc < kMaxKP / 16; ++kc) d[kc] = d4{0.0, 0.0, 0.0, 0.0};
    for (int qb = 0; qb < KP; qb += QB) {
      if (QB == KP) {   // (qb = 0: the values loaded at entry, then the rest)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int idx = threadIdx.x + 256 * e;
          if (idx < KP * KP) s_fw[(idx % KP) * KP + idx / KP] = fwv[e];
        }
      }
      for (int idx = threadIdx.x + (QB == KP ? 1024 : 0); idx < QB * KP; idx += blockDim.x) {
        const int k = idx / QB, q = idx % QB;   // (coalesced over q in FW's rows)
        s_fw[q * KP + k] = gfw[(size_t)k * KP + qb + q];
      }
      __syncthreads();
#pragma unroll
      for (int kc = 0; kc < kMaxKP / 16; ++kc)
        if (16 * kc < KP)
          for (int q0 = 0; q0 < QB; q0 += 4)
            d[kc] = mfma4(s_fw[(q0 + tq) * KP + 16 * kc + fl], s_y[(qb + q0 + tq) * 64 + 16 * wv + fl],
                          d[kc]);
      __syncthreads();
    }
    if (16 * wv + fl < tn)
#pragma unroll
      for (int kc = 0; kc < kMaxKP / 16; ++kc)
        if (16 * kc < KP)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            a.FWHt[((size_t)j * a.Tp + t0 + 16 * wv + fl) * KP + 16 * kc + tq + 4 * i] = d[kc][i];
    // row sums over the block's frames (t < T: the padding frames hold 0):
    // one wave per row, lane = frame, the wave's tree
    for (int q = wv; q < KP; q += 4) {
      double h = s_y[q * 64 + lane];
#pragma unroll
      for (int mm = 32; mm > 0; mm >>= 1) h += __shfl_xor(h, mm, 64);
      if (lane == 0) a.hpart[((size_t)j * KP + q) * a.ntb + blockIdx.x] = h;
    }
    return;
  }
  if (!a.tw_free[j]) return;
  // ratios for 64 frames x KP components (coalesced over k), then a
  // transposed, coalesced-over-t read-modify-write of TW
  for (int kb = 0; kb < a.KP; kb += 64) {
    const int kn = min(64, a.KP - kb);
    for (int idx = threadIdx.x; idx < 64 * kn; idx += blockDim.x) {
      const int tl = idx / kn, kl = idx % kn, t = t0 + tl;
      double r = 1.0;
      if (t < a.T) {
        double num = 0.0, den = 0.0;
        for (int c = 0; c < a.nsplit; ++c) {
          const size_t o = (((size_t)c * a.J + j) * a.Tp + t) * a.KP + kb + kl;
          num += a.tnum[o];
          den += a.tden[o];
        }
        const double ratio = num / fmax(den, kEps);
        r = a.omega == 1.0 ? ratio : pow(ratio, a.omega);
      }
      s_r[kl][tl] = r;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 64 * kn; idx += blockDim.x) {
      const int kl = idx / 64, tl = idx % 64, t = t0 + tl, k = kb + kl;
      if (t < a.T && k >= a.kb0[j] && k < a.kb1[j])
        a.TW[((size_t)j * a.KP + k) * a.Tp + t] *= s_r[kl][tl];
    }
    __syncthreads();
  }
}

// ------------------------------------------------- several spectral components
// update_spectral_components (audioModel.py:1479-1727) when source j holds
// several spectral components: they are updated one after the other in the
// reference's key order (block b of every source at step b), each seeing the
// components updated before it.  For block c of source j, with
// V_j = sum of all its components' powers (current parameters), V_c the
// block's own power and hat_W_j the E-step's posterior power:
//   FB: num = ((hat_W_j / max(V_j)^2) max(V_c)) (FW H)^T, den = (max(V_c) /
//       max(V_j)) (FW H)^T (:1513-1575, other = max(V_c): N1)
//   TW: k_tw_contract<BLK> with V_old / V_new of the block and the plane
//       rho_c = hat_W_j / max(V_c_old) (:1634-1727, spec_comp_ind=[k])
// k_multi_prep forms the three planes (rnum, rden, rho_c) of step b from the
// current W (Wkf, all blocks) and TW; at step 0 it also turns the E-step's
// rho_j = hat_W_j / max(V_j) back into hat_W_j in place (the later steps need
// hat_W_j itself, V_j having moved).
struct MPArgs {
  const double *TW, *Wkf;
  double *hatW, *rnum, *rden, *rtw;   // planes [J][Tp][Fp]
  double *rcp, *rpow;                 // LAM: corrPen and max(sum_j V_j, eps) planes
  double *roth;                       // time blobs: max(V_c, eps) at the step's start
  double lambda;
  int F, T, Fp, Tp, KP, J, ntt, tpc, first;
  int on[kMaxJ], kb0[kMaxJ], kb1[kMaxJ];
  const int *halt;
};

// LAM (lambdaCorr > 0, audioModel.py:1484-1507, :1544-1569): the planes
// carry the inter-source correlation penalty of the component's FB step,
//   powers = max(sum_j' V_j', eps) (comp_spat_cmps_powers, summed in source
//   order), minus = max(powers - max(V_j, eps), eps) (the reference's
//   `np.all(minus >= 0)` branch always holds: a sum of non-negative powers is
//   never below one of its terms), cp = lambda minus / max(powers^2, eps)
//   rden = other (1/max(V_j) + cp), rnum = (hat_W/max(V_j)^2 + cp 2 (max(V_j)/powers)) other
// and cp / powers go to two more planes for the FW / TW steps, which use the
// same cp with the component's own power (:1596-1620, :1650-1719).
template <int NKC, bool LAM = false>
__global__ __launch_bounds__(64) void k_multi_prep(const MPArgs a) {
  HALT_GUARD(a.halt);
  constexpr int NKS = 4 * NKC;
  const int lane = threadIdx.x, fl = lane & 15, tq = lane >> 4;
  const int j = blockIdx.y;
  if (!a.on[j]) return;
  const int f0 = blockIdx.x * 16, f = f0 + fl;
  double wj[NKS], wc[NKS];   // B operands of the V tiles: W[k = tq + 4 s][f]
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int k = tq + 4 * s;
    const double w = a.Wkf[((size_t)j * a.KP + k) * a.Fp + f];
    wj[s] = w;
    wc[s] = k >= a.kb0[j] && k < a.kb1[j] ? w : 0.0;
  }
  const size_t pj = (size_t)j * a.Tp * a.Fp;
  const int tb = blockIdx.z * a.tpc, te = min(tb + a.tpc, a.ntt);
  for (int tt = tb; tt < te; ++tt) {
    const int t0 = tt * 16;
    const double *tw = a.TW + ((size_t)j * a.KP + tq) * a.Tp + t0 + fl;
    d4 vj = d4{0.0, 0.0, 0.0, 0.0}, vc = vj, vall = vj;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const double h = tw[(size_t)(4 * s) * a.Tp];
      vj = mfma4(h, wj[s], vj);
      vc = mfma4(h, wc[s], vc);
    }
    if constexpr (LAM) {
      for (int jj = 0; jj < a.J; ++jj) {   // sum_j' V_j' in source order
        d4 v = d4{0.0, 0.0, 0.0, 0.0};
        if (jj == j) {
          v = vj;
        } else {
          const double *twj = a.TW + ((size_t)jj * a.KP + tq) * a.Tp + t0 + fl;
          const double *wk = a.Wkf + ((size_t)jj * a.KP + tq) * a.Fp + f;
          for (int s = 0; s < NKS; ++s)
            v = mfma4(twj[(size_t)(4 * s) * a.Tp], wk[(size_t)(4 * s) * a.Fp], v);
        }
        vall += v;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + tq + 4 * i;
      const size_t o = pj + (size_t)t * a.Fp + f;
      if (t >= a.T || f >= a.F) {
        a.rnum[o] = a.rden[o] = a.rtw[o] = 0.0;
        if constexpr (LAM) a.rcp[o] = a.rpow[o] = 0.0;
        if (a.roth) a.roth[o] = 0.0;
        continue;
      }
      const double sj = fmax(vj[i], kEps), sc = fmax(vc[i], kEps);
      double hw;
      if (a.first) {
        hw = a.hatW[o] * sj;   // rho_j max(V_j) (the E-step stored rho_j)
        a.hatW[o] = hw;
      } else {
        hw = a.hatW[o];
      }
      if constexpr (LAM) {
        const double pw = fmax(vall[i], kEps);
        const double minus = fmax(pw - sj, kEps);
        const double cp = a.lambda * minus / fmax(pw * pw, kEps);
        a.rden[o] = sc * (1.0 / sj + cp);
        a.rnum[o] = (hw / (sj * sj) + cp * (2.0 * (sj / pw))) * sc;
        a.rcp[o] = cp;
        a.rpow[o] = pw;
      } else {
        a.rnum[o] = (hw / (sj * sj)) * sc;
        a.rden[o] = sc * (1.0 / sj);
      }
      a.rtw[o] = hw / sc;
      if (a.roth) a.roth[o] = sc;
    }
  }
}

// ---------------------------------------------------------------- renormalize
struct RArgs {
  double2 *A, *Pinst;
  double *FB, *FW, *TW;
  double *scal;   // [J][2 + 2*KP]: e_j, -, w_j[KP], w2_j[KP] (stage 2 -> 3)
  double *pmax;   // [J][nchunk][KP] column maxima of FB per bin chunk
  double *pe;     // [J][nchunk] partial mixing-filter energy (conv)
  double *tpart;  // [nslot][nchunk] partial sums of the rescaled TW, per block
  int *flags;
  // fused tail (k_renorm_scales / _rows / _tail): k_fb_update's column
  // maxima [J][nstat][KP], k_tw_update's restart sums [nslot][ntb], the
  // E-step's loglik partials
  const double *pmax2, *tpart2, *llpart;
  double *ll_out;
  // k_tw_update's TW row-sum partials [J][KP][ntb] -> hsum [J][KP] (null: the
  // next iteration's k_tw_rowsum forms hsum)
  const double *hpart;
  double *hsum;
  int J;
  double inv_FT;
  int nstat, ntb, nll;
  int F, T, Fp, Tp, KP, nchunk, tpc, fpc, nslot;
  unsigned convm;    // bit j: spatial component j is 'conv' (per-bin filters in A)
  int K[kMaxJ], roff[kMaxJ + 1];
  // spectral components of source j (column blocks of FB / FW / TW) and the
  // slot of block 0
  int nblk[kMaxJ], kb[kMaxJ][kMaxBlk + 1], soff[kMaxJ + 1];
  unsigned tbmask;   // slots with time blobs: their restart test is k_tb_renorm's
  const int *halt;
};

__device__ double block_sum(double x, double *s) {
  s[threadIdx.x] = x;
  __syncthreads();
  for (int w = blockDim.x >> 1; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  const double r = s[0];
  __syncthreads();
  return r;
}

// renormalize_parameters (audioModel.py:1991-2037) in two passes over
// (source, chunk) blocks.  Stage 1: per bin chunk, the column maxima of FB
// and (conv) the partial energy of the mixing filters.  Since x -> fl(x e) is
// monotone for e >= 0, max_f fl(FB e) = fl(e max_f FB): the maxima are taken
// on the raw FB and scaled in stage 2.
__global__ __launch_bounds__(256) void k_renorm_stats(const RArgs a) {
  HALT_GUARD(a.halt);
  __shared__ double s_red[256];
  const int j = blockIdx.y, c = blockIdx.x, KP = a.KP;
  const int fb = c * a.fpc, fe = min(fb + a.fpc, a.F);
  const int groups = blockDim.x / KP, k = threadIdx.x % KP, g = threadIdx.x / KP;
  double m = -INFINITY;
  if (g < groups)
    for (int f = fb + g; f < fe; f += groups) m = fmax(m, a.FB[((size_t)j * a.Fp + f) * KP + k]);
  s_red[threadIdx.x] = m;
  __syncthreads();
  if (threadIdx.x < KP) {
    double x = s_red[threadIdx.x];
    for (int q = 1; q < groups; ++q) x = fmax(x, s_red[q * KP + threadIdx.x]);
    a.pmax[((size_t)j * a.nchunk + c) * KP + threadIdx.x] = x;
  }
  __syncthreads();
  if (a.convm >> j & 1u) {
    const int r0 = a.roff[j], nr = a.roff[j + 1] - r0, w = fe - fb;
    double e = 0.0;
    for (int idx = threadIdx.x; idx < nr * 2 * w; idx += blockDim.x) {
      const int f = fb + idx % w, rc = idx / w;
      const double2 x = a.A[(size_t)(2 * r0 + rc) * a.Fp + f];
      e += x.x * x.x + x.y * x.y;
    }
    e = block_sum(e, s_red);
    if (threadIdx.x == 0) a.pe[(size_t)j * a.nchunk + c] = e;
  }
}

// Stage 2: every block recombines the (tiny) stage-1 partials into e_j,
// w_j[k] = max_f FB[:,k] e_j (0 -> 1) and w2_j[c] = mean_r FW[r,c] w_j[r]
// (0 -> 1), then scales its chunk: FB rows (FB e / w), TW columns (TW w2,
// with partial sums for the restart test), the mixing filters / sqrt(e).
// FW and the 'inst' parameters are read by every block here, so they are
// rewritten in stage 3 from the scales chunk 0 records.
template <bool BIG>
__global__ __launch_bounds__(256) void k_renorm_apply(const RArgs a) {
  HALT_GUARD(a.halt);
  __shared__ double s_red[256];
  __shared__ double s_w[kMaxKP], s_w2[kMaxKP];
  __shared__ double s_e;
  __shared__ double s_big[64 * 64];   // chunk maxima, then FW_j (KP <= 64; else from L2)
  const int j = blockIdx.y, c = blockIdx.x;
  const int K = a.K[j], KP = a.KP;
  const int r0 = a.roff[j], nr = a.roff[j + 1] - r0;
  // the cross-chunk statistics are loaded by all threads at once and folded
  // in LDS (a per-thread loop over the chunks was a chain of dependent
  // global-latency round trips), in the same order as before
  const bool cj = a.convm >> j & 1u;
  const int ne = cj ? a.nchunk : nr * 2;
  for (int q = threadIdx.x; q < ne; q += blockDim.x) {
    if (cj) {
      s_red[q] = a.pe[(size_t)j * a.nchunk + q];
    } else {
      const double2 x = a.Pinst[2 * r0 + q];
      s_red[q] = x.x * x.x + x.y * x.y;
    }
  }
  constexpr bool big = BIG;   // chunk maxima / FW too large for s_big: read from L2
  const double *pmx = big ? a.pmax + (size_t)j * a.nchunk * KP : s_big;
  const double *fwb = big ? a.FW + (size_t)j * KP * KP : s_big;
  if (!big)
    for (int i = threadIdx.x; i < a.nchunk * KP; i += blockDim.x)
      s_big[i] = a.pmax[(size_t)j * a.nchunk * KP + i];
  __syncthreads();
  if (threadIdx.x == 0) {
    double e = 0.0;
    for (int q = 0; q < ne; ++q) e += s_red[q];
    s_e = e / (double)(cj ? nr * 2 * a.F : nr * 2);
  }
  __syncthreads();
  const double e = s_e;
  if (threadIdx.x < KP) {
    double m = -INFINITY;
    for (int q = 0; q < a.nchunk; ++q) m = fmax(m, pmx[q * KP + threadIdx.x]);
    const double w = m * e;
    s_w[threadIdx.x] = w == 0.0 ? 1.0 : w;
  }
  __syncthreads();
  if (!big)
    for (int i = threadIdx.x; i < KP * KP; i += blockDim.x) s_big[i] = a.FW[(size_t)j * KP * KP + i];
  __syncthreads();
  if (threadIdx.x < K) {
    // FW.mean(axis=0) of the column's own spectral component (block)
    const int cc = threadIdx.x;
    int b = 0;
    while (b + 1 < a.nblk[j] && cc >= a.kb[j][b + 1]) ++b;
    const int r0b = a.kb[j][b], r1b = a.kb[j][b + 1];
    double s = 0.0;
    for (int r = r0b; r < r1b; ++r) s += fwb[r * KP + cc] * s_w[r];
    s /= (double)(r1b - r0b);
    s_w2[cc] = s == 0.0 ? 1.0 : s;
  }
  __syncthreads();
  // FB rows of this chunk (only the K live columns carry data)
  // (element loops below load a batch of kRnB values before storing any, so
  // a thread keeps kRnB memory round trips in flight)
  constexpr int kRnB = 8;
  const int fb = c * a.fpc, fe = min(fb + a.fpc, a.F);
  {
    const int n = (fe - fb) * KP;
    for (int base = threadIdx.x; base < n; base += kRnB * blockDim.x) {
      double x[kRnB];
#pragma unroll
      for (int u = 0; u < kRnB; ++u) {
        const int idx = base + u * blockDim.x;
        x[u] = idx < n ? a.FB[((size_t)j * a.Fp + fb + idx / KP) * KP + idx % KP] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kRnB; ++u) {
        const int idx = base + u * blockDim.x, k = idx % KP;
        if (idx < n && k < K)
          a.FB[((size_t)j * a.Fp + fb + idx / KP) * KP + k] = (x[u] * e) / s_w[k];
      }
    }
  }
  const double se = sqrt(e);
  if (cj) {
    const int w = fe - fb;
    for (int idx = threadIdx.x; idx < nr * 2 * w; idx += blockDim.x) {
      const int f = fb + idx % w, rc = idx / w;
      double2 *p = a.A + (size_t)(2 * r0 + rc) * a.Fp + f;
      *p = make_double2(p->x / se, p->y / se);
    }
  }
  if (c == 0) {  // FW and 'inst' parameters are rewritten in stage 3 (read above)
    double *sc = a.scal + (size_t)j * (2 + 2 * KP);
    if (threadIdx.x == 0) sc[0] = e;
    if (threadIdx.x < KP) {
      sc[2 + threadIdx.x] = s_w[threadIdx.x];
      sc[2 + KP + threadIdx.x] = s_w2[threadIdx.x];
    }
  }
  double *TW = a.TW + (size_t)j * KP * a.Tp;
  const int t0 = c * a.tpc, t1 = min(t0 + a.tpc, a.T);
  const int w = t1 - t0;
  for (int b = 0; b < a.nblk[j]; ++b) {   // one restart sum per spectral component
    const int rb = a.kb[j][b], nrow = a.kb[j][b + 1] - rb;
    double tsum = 0.0;
    if (w > 0)
      for (int base = threadIdx.x; base < nrow * w; base += kRnB * blockDim.x) {
        double x[kRnB];
#pragma unroll
        for (int u = 0; u < kRnB; ++u) {
          const int idx = base + u * blockDim.x;
          x[u] = idx < nrow * w ? TW[(size_t)(rb + idx / w) * a.Tp + t0 + idx % w] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kRnB; ++u) {
          const int idx = base + u * blockDim.x;
          if (idx < nrow * w) {
            const double y = x[u] * s_w2[rb + idx / w];
            TW[(size_t)(rb + idx / w) * a.Tp + t0 + idx % w] = y;
            tsum += y;
          }
        }
      }
    tsum = block_sum(tsum, s_red);
    if (threadIdx.x == 0) a.tpart[(size_t)(a.soff[j] + b) * a.nchunk + c] = tsum;
  }
}

// Stage 3 (one block): FW = FW w / w2, 'inst' parameters / sqrt(e), and the
// restart test sum(TW_j) < eps -> host-side random restart (audioModel.py:2023)
__global__ void k_renorm_final(const RArgs a, int J, int iter) {
  HALT_GUARD(a.halt);
  for (int j = 0; j < J; ++j) {
    const int K = a.K[j], KP = a.KP;
    const double *sc = a.scal + (size_t)j * (2 + 2 * KP);
    double *FW = a.FW + (size_t)j * KP * KP;
    for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) {
      const int r = idx / K, cc = idx % K;
      FW[r * KP + cc] = (FW[r * KP + cc] * sc[2 + r]) / sc[2 + KP + cc];
    }
    const int r0 = a.roff[j], nr = a.roff[j + 1] - r0;
    if (!(a.convm >> j & 1u) && threadIdx.x < nr * 2) {
      const double se = sqrt(sc[0]);
      double2 *p = a.Pinst + 2 * r0 + threadIdx.x;
      *p = make_double2(p->x / se, p->y / se);
    }
  }
  __shared__ double s_t[kMaxSlot * 64];   // the per-chunk TW sums, loaded at once
  for (int i = threadIdx.x; i < a.nslot * a.nchunk; i += blockDim.x) s_t[i] = a.tpart[i];
  __syncthreads();
  const int sl = threadIdx.x;   // one TW restart test per spectral component
  if (sl >= a.nslot || (a.tbmask >> sl & 1u)) return;
  double s = 0.0;
  for (int c = 0; c < a.nchunk; ++c) s += s_t[sl * a.nchunk + c];
  const int dead = s < kEps ? 1 : 0;
  a.flags[1 + sl] = dead;
  if (dead) {
    a.flags[kFlagHalt] = 1;
    a.flags[kFlagIter] = iter;
  }
}

// Fused tail of gem_iteration (one spectral component per source, no time
// blobs, fixed FW): the same renormalize_parameters (audioModel.py:1991-2037)
// with the FB column maxima taken by k_fb_update, the scales formed once per
// source (k_renorm_scales) after the mixing update, and the FB / mixing / FW
// rescale (k_renorm_rows) on the side stream while the TW contraction runs;
// TW's rescale and restart sums ride in k_tw_update, and k_renorm_tail closes
// the iteration with the restart test and the loglik sum.
//
// k_renorm_scales, one block per source: e_j = mean |params|^2 (the 'conv'
// filters read from A itself, 'inst' from Pinst), w_j[k] = e_j max_f FB[f][k]
// (0 -> 1), w2_j[c] = mean_r FW[r][c] w_j[r] over the K live rows (0 -> 1).
// Every thread issues its loads in batches before using any: the round-5
// form walked the 129 maxima, the energy partials and the K x K FW as chains
// of dependent loads (105 us beside the TW contraction, profiles/r5_bench.txt)
__global__ __launch_bounds__(1024) void k_renorm_scales(const RArgs a) {
  HALT_GUARD(a.halt);
  constexpr int NT = 1024, B = 16;   // threads; loads in flight per thread and batch
  __shared__ double s_red[NT];
  __shared__ double s_w[kMaxKP];
  const int t = threadIdx.x, j = blockIdx.x, K = a.K[j], KP = a.KP, ns = a.nstat;
  const int r0 = a.roff[j], nr = a.roff[j + 1] - r0;
  const bool cj = a.convm >> j & 1u;
  // e_j: the 'conv' filters A[r][c][f] of the source's nr ranks (one batch
  // of loads per thread up to 8 ranks at C3's F)
  const int ne = cj ? nr * 2 * a.F : nr * 2;
  double e = 0.0;
  for (int base = t; base < ne; base += B * NT) {
    double2 x[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int idx = base + u * NT;
      x[u] = idx >= ne ? make_double2(0.0, 0.0)
                       : (cj ? a.A[(size_t)(2 * r0 + idx / a.F) * a.Fp + idx % a.F] : a.Pinst[2 * r0 + idx]);
    }
#pragma unroll
    for (int u = 0; u < B; ++u) e += x[u].x * x[u].x + x[u].y * x[u].y;
  }
  // column maxima over k_fb_update's blocks: thread (g, k) takes blocks
  // q = g mod G (max is exact in any order; 5 per thread at C3)
  const int G = NT / KP;
  double m = -INFINITY;
  for (int q0 = t / KP; q0 < ns; q0 += B * G) {
    double x[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int q = q0 + u * G;
      x[u] = q < ns ? a.pmax2[((size_t)j * ns + q) * KP + t % KP] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < B; ++u) m = fmax(m, x[u]);
  }
  // FW[r][c] of thread (g, c): rows r = g, g + G, ... (all of them in one
  // batch up to K = 64 at KP = 64, K = 32 at KP = 32: one row per thread)
  const int cc = t % KP;
  const double *fw = a.FW + (size_t)j * KP * KP;
  constexpr int RB = 8;
  double fr[RB];
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int r = t / KP + u * G;
    fr[u] = r < K && cc < K ? fw[r * KP + cc] : 0.0;
  }
  e = block_sum(e, s_red) / (double)ne;
  s_red[t] = m;
  __syncthreads();
  for (int k = t; k < KP; k += NT) {
    double x = -INFINITY;
    for (int g = 0; g < G; ++g) x = fmax(x, s_red[g * KP + k]);
    const double w = x * e;
    s_w[k] = w == 0.0 ? 1.0 : w;
  }
  __syncthreads();
  // FW.mean(axis=0) of the column's spectral component: the thread's rows,
  // then the groups in order (one row per group: the sequential row order)
  double sp = 0.0;
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int r = t / KP + u * G;
    if (r < K) sp += fr[u] * s_w[r];
  }
  for (int r = t / KP + RB * G; r < K; r += G) sp += fw[r * KP + cc] * s_w[r];   // (K > RB G only)
  s_red[t] = sp;
  __syncthreads();
  double *sc = a.scal + (size_t)j * (2 + 2 * KP);
  if (t < KP) {
    double s = 1.0;
    if (t < K) {
      s = 0.0;
      for (int g = 0; g < G; ++g) s += s_red[g * KP + t];
      s /= (double)K;
      if (s == 0.0) s = 1.0;
    }
    sc[2 + t] = s_w[t];
    sc[2 + KP + t] = s;
  }
  if (t == 0) sc[0] = e;
}

// FB rows of 16 bins (FB e / w), the 'conv' filters / sqrt(e); block x = 0
// also rescales FW (FW w / w2) and the 'inst' parameters of its source
__global__ __launch_bounds__(256) void k_renorm_rows(const RArgs a) {
  HALT_GUARD(a.halt);
  const int j = blockIdx.y, f0 = blockIdx.x * 16, K = a.K[j], KP = a.KP;
  const int nb = min(16, a.F - f0);
  const double *sc = a.scal + (size_t)j * (2 + 2 * KP);
  const double e = sc[0], se = sqrt(e);
  for (int idx = threadIdx.x; idx < nb * KP; idx += blockDim.x) {
    const int k = idx % KP;
    double *p = a.FB + ((size_t)j * a.Fp + f0 + idx / KP) * KP + k;
    if (k < K) *p = (*p * e) / sc[2 + k];
  }
  const int r0 = a.roff[j], nr = a.roff[j + 1] - r0;
  if (a.convm >> j & 1u) {
    for (int idx = threadIdx.x; idx < nr * 2 * nb; idx += blockDim.x) {
      double2 *p = a.A + (size_t)(2 * r0 + idx / nb) * a.Fp + f0 + idx % nb;
      *p = make_double2(p->x / se, p->y / se);
    }
  } else if (blockIdx.x == 0 && threadIdx.x < nr * 2) {
    double2 *p = a.Pinst + 2 * r0 + threadIdx.x;
    *p = make_double2(p->x / se, p->y / se);
  }
  if (blockIdx.x == 0) {
    double *FW = a.FW + (size_t)j * KP * KP;
    for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) {
      const int r = idx / K, cc = idx % K;
      FW[r * KP + cc] = (FW[r * KP + cc] * sc[2 + r]) / sc[2 + KP + cc];
    }
  }
}

// one block: the iteration's loglik (k_loglik's sum) and the TW restart test
// from k_tw_update's partial sums (audioModel.py:2023)
__global__ __launch_bounds__(256) void k_renorm_tail(const RArgs a, int iter) {
  HALT_GUARD(a.halt);
  if (blockIdx.x > 0) {
    // blocks 1..: hsum[r] = sum_t TW row r from k_tw_update's per-block
    // partials, one wave per row (lane-strided, then the wave's tree: a
    // fixed order)
    const int r = (blockIdx.x - 1) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= a.J * a.KP) return;
    double h = 0.0;
    for (int b = lane; b < a.ntb; b += 64) h += a.hpart[(size_t)r * a.ntb + b];
#pragma unroll
    for (int mm = 32; mm > 0; mm >>= 1) h += __shfl_xor(h, mm, 64);
    if (lane == 0) a.hsum[r] = h;
    return;
  }
  __shared__ double s[256];
  double x = 0.0;
  for (int i = threadIdx.x; i < a.nll; i += 256) x += a.llpart[i];
  s[threadIdx.x] = x;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.ll_out[0] = -(s[0] * a.inv_FT);
  __syncthreads();
  for (int sl = 0; sl < a.nslot; ++sl) {
    double t = 0.0;
    for (int c = threadIdx.x; c < a.ntb; c += 256) t += a.tpart2[(size_t)sl * a.ntb + c];
    t = block_sum(t, s);
    if (threadIdx.x == 0) {
      const int dead = t < kEps ? 1 : 0;
      a.flags[1 + sl] = dead;
      if (dead) {
        a.flags[kFlagHalt] = 1;
        a.flags[kFlagIter] = iter;
      }
    }
  }
}

// ---------------------------------------------------------------- time blobs
// A spectral component with time blobs (TB, audioModel.py:430-498) has
// H = TW TB.  Its factor TW ("TWs", block rows x L) and TB (L x T) live in the
// slot buffer tb[j][b] (tb_layout) and the block's rows of the model TW hold
// H, so every other kernel (E-step, FB / FW / TW contractions, Wiener) reads
// H unchanged.  Both updates reuse the block's TW contraction, which leaves
// G = W^T R over f per frame in tnum / tden (W = FB FW of the block):
//   TW step (:1665-1691): num = G TB^T, den likewise        (k_tb_tw_red)
//   TB step (:1931-1978): num = TWs^T G, with R's ratio hat_W / max(V^2, eps)
//                         (k_tw_contract<TBQ>, then k_tb_tb_upd)
// the reference's (W TWs)^T R reassociated; H is rebuilt after each (k_tb_h).
struct TBLayout {
  size_t tws, tb, num, den, n;   // offsets (doubles) in the slot buffer, total
};
__host__ __device__ inline TBLayout tb_layout(int kbw, int L, int Tp) {
  TBLayout o;
  o.tws = 0;
  o.tb = (size_t)kbw * L;
  o.num = o.tb + (size_t)L * Tp;
  o.den = o.num + (size_t)kbw * L;
  o.n = o.den + (size_t)kbw * L;
  return o;
}

struct TBArgs {
  double *tb[kMaxJ];   // the step's slot buffer per source (null: no time blobs)
  int L[kMaxJ], kb0[kMaxJ], kbw[kMaxJ];
  double *TW;
  const double *tnum, *tden;   // [nsplit][J][Tp][KP] of k_tw_contract
  int T, Tp, KP, J, nsplit;
  double omega;
  // iter >= 0 (renormalisation): a halt raised in this same iteration does not
  // stop the kernel (the host reads a consistent TWs / TB), an earlier one does
  const int *flags;
  int iter;
  const int *halt;
};

__device__ inline bool tb_halted(const int *halt, const int *flags, int iter) {
  if (!halt || !*(volatile const int *)halt) return false;
  return iter < 0 || *(volatile const int *)(flags + kFlagIter) < iter;
}

// TW step: num[k][l] = sum_t G_num[t][k] TB[l][t] (chunks summed first), one
// block per (blob, 16 rows, source)
__global__ __launch_bounds__(256) void k_tb_tw_red(const TBArgs a) {
  if (tb_halted(a.halt, a.flags, a.iter)) return;
  __shared__ double s_red[256];
  const int l = blockIdx.x, k0 = blockIdx.y * 16, j = blockIdx.z;
  if (!a.tb[j] || l >= a.L[j] || k0 >= a.kbw[j]) return;
  const int L = a.L[j], kbw = a.kbw[j], nk = min(16, kbw - k0);
  const TBLayout o = tb_layout(kbw, L, a.Tp);
  const double *TB = a.tb[j] + o.tb + (size_t)l * a.Tp;
  double num[16], den[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) num[i] = den[i] = 0.0;
  for (int t = threadIdx.x; t < a.T; t += blockDim.x) {
    const double bl = TB[t];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < nk) {
        double sn = 0.0, sd = 0.0;
        for (int c = 0; c < a.nsplit; ++c) {
          const size_t q = (((size_t)c * a.J + j) * a.Tp + t) * a.KP + a.kb0[j] + k0 + i;
          sn += a.tnum[q];
          sd += a.tden[q];
        }
        num[i] += sn * bl;
        den[i] += sd * bl;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < nk) {
      const double rn = block_sum(num[i], s_red), rd = block_sum(den[i], s_red);
      if (threadIdx.x == 0) {
        a.tb[j][o.num + (size_t)(k0 + i) * L + l] = rn;
        a.tb[j][o.den + (size_t)(k0 + i) * L + l] = rd;
      }
    }
  }
}

// TWs *= (num / max(den, eps))^omega   (:1718-1726)
__global__ __launch_bounds__(256) void k_tb_tw_apply(const TBArgs a) {
  if (tb_halted(a.halt, a.flags, a.iter)) return;
  const int j = blockIdx.x;
  if (!a.tb[j]) return;
  const TBLayout o = tb_layout(a.kbw[j], a.L[j], a.Tp);
  double *p = a.tb[j];
  for (int i = threadIdx.x; i < a.kbw[j] * a.L[j]; i += blockDim.x) {
    const double r = p[o.num + i] / fmax(p[o.den + i], kEps);
    p[o.tws + i] *= a.omega == 1.0 ? r : pow(r, a.omega);
  }
}

// TB step: num[l][t] = sum_k TWs[k][l] G_num[t][k], TB *= (num / max(den,
// eps))^omega (:1974-1977); 64 frames per block, accumulators in LDS
__global__ __launch_bounds__(64) void k_tb_tb_upd(const TBArgs a) {
  if (tb_halted(a.halt, a.flags, a.iter)) return;
  extern __shared__ double s_tb[];
  const int j = blockIdx.y;
  if (!a.tb[j]) return;
  const int L = a.L[j], kbw = a.kbw[j], tid = threadIdx.x;
  const TBLayout o = tb_layout(kbw, L, a.Tp);
  double *s_tw = s_tb, *s_num = s_tb + kbw * L, *s_den = s_num + 64 * L;
  for (int i = tid; i < kbw * L; i += 64) s_tw[i] = a.tb[j][o.tws + i];
  for (int l = 0; l < L; ++l) s_num[l * 64 + tid] = s_den[l * 64 + tid] = 0.0;
  __syncthreads();
  const int t = blockIdx.x * 64 + tid;
  if (t >= a.T) return;
  for (int k = 0; k < kbw; ++k) {
    double sn = 0.0, sd = 0.0;
    for (int c = 0; c < a.nsplit; ++c) {
      const size_t q = (((size_t)c * a.J + j) * a.Tp + t) * a.KP + a.kb0[j] + k;
      sn += a.tnum[q];
      sd += a.tden[q];
    }
    for (int l = 0; l < L; ++l) {
      const double w = s_tw[k * L + l];
      s_num[l * 64 + tid] += w * sn;
      s_den[l * 64 + tid] += w * sd;
    }
  }
  double *TB = a.tb[j] + o.tb;
  for (int l = 0; l < L; ++l) {
    const double r = s_num[l * 64 + tid] / fmax(s_den[l * 64 + tid], kEps);
    TB[(size_t)l * a.Tp + t] *= a.omega == 1.0 ? r : pow(r, a.omega);
  }
}

// H = TWs TB into the block's rows of TW (padding frames stay zero)
__global__ __launch_bounds__(256) void k_tb_h(const TBArgs a) {
  if (tb_halted(a.halt, a.flags, a.iter)) return;
  extern __shared__ double s_tw[];
  const int j = blockIdx.y;
  if (!a.tb[j]) return;
  const int L = a.L[j], kbw = a.kbw[j];
  const TBLayout o = tb_layout(kbw, L, a.Tp);
  for (int i = threadIdx.x; i < kbw * L; i += blockDim.x) s_tw[i] = a.tb[j][o.tws + i];
  __syncthreads();
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.Tp) return;
  const double *TB = a.tb[j] + o.tb;
  for (int k = 0; k < kbw; ++k) {
    double h = 0.0;
    for (int l = 0; l < L; ++l) h += s_tw[k * L + l] * TB[(size_t)l * a.Tp + t];
    a.TW[((size_t)j * a.KP + a.kb0[j] + k) * a.Tp + t] = t < a.T ? h : 0.0;
  }
}

// renormalize_parameters for a component with time blobs (:2019-2033), after
// k_renorm_final: TWs *= w (the FW column means, as the block's H rows got in
// k_renorm_apply), the restart test on sum(TWs), then TB /= m, TWs *= m with
// m = TB.mean(axis=1).  A dead component is left to the host (redraw, then
// the TB step of the renormalisation), one block per (component, source).
struct TBRArgs {
  double *tb[kMaxJ][kMaxBlk];
  int L[kMaxJ][kMaxBlk], kb0[kMaxJ][kMaxBlk], kbw[kMaxJ][kMaxBlk], slot[kMaxJ][kMaxBlk];
  const double *scal;   // RArgs::scal: w2 = FW column means at [j][2 + KP + k]
  int *flags;
  const int *halt;
  int T, Tp, KP, iter;
};
__global__ __launch_bounds__(256) void k_tb_renorm(const TBRArgs a) {
  if (tb_halted(a.halt, a.flags, a.iter)) return;
  __shared__ double s_red[256];
  __shared__ double s_m[kMaxTB];
  const int b = blockIdx.x, j = blockIdx.y;
  double *p = a.tb[j][b];
  if (!p) return;
  const int L = a.L[j][b], kbw = a.kbw[j][b], n = kbw * L;
  const TBLayout o = tb_layout(kbw, L, a.Tp);
  const double *w2 = a.scal + (size_t)j * (2 + 2 * a.KP) + 2 + a.KP + a.kb0[j][b];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double y = p[o.tws + i] * w2[i / L];
    p[o.tws + i] = y;
    s += y;
  }
  s = block_sum(s, s_red);
  const int dead = s < kEps ? 1 : 0;
  if (threadIdx.x == 0) {
    a.flags[1 + a.slot[j][b]] = dead;
    if (dead) {
      a.flags[kFlagHalt] = 1;
      a.flags[kFlagIter] = a.iter;
    }
  }
  if (dead) return;
  double *TB = p + o.tb;
  for (int l = 0; l < L; ++l) {
    double m = 0.0;
    for (int t = threadIdx.x; t < a.T; t += blockDim.x) m += TB[(size_t)l * a.Tp + t];
    m = block_sum(m, s_red) / (double)a.T;
    if (m == 0.0) m = 1.0;
    for (int t = threadIdx.x; t < a.T; t += blockDim.x) TB[(size_t)l * a.Tp + t] /= m;
    if (threadIdx.x == 0) s_m[l] = m;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) p[o.tws + i] *= s_m[i % L];
}

// ---------------------------------------------------------------- host side
enum KernelId {
  KW = 0, KFWH, KINSTA, KESTEP, KLL, KMIX, KMIXI, KFBC, KFBU, KTWC, KREN, KTWU, KFWU, KROWS, KRTAIL
};
static const char *kKernelNames[fasst_ctx::kNK] = {
    "k_w_from_fb", "k_fwh_t", "k_inst_A", "k_estep", "k_loglik", "k_mix",
    "k_mix_inst", "k_fb_contract", "k_fb_update", "k_tw_contract", "k_renorm", "k_tw_update",
    "k_fw_update", "k_tw_rowsum", "k_renorm_tail"};

// per-kernel timing: an event pair around the launch on the stream it runs on
// (s = nullptr: the main stream), slot = the iteration's place in the ring
static inline void prof_begin(fasst_ctx *c, int id, hipStream_t s = nullptr) {
  if (c->prof) {
    (void)hipEventRecord(c->ev0[id][c->pslot], s ? s : c->stream);
    c->used[id][c->pslot] = 1;
  }
}
static inline void prof_end(fasst_ctx *c, int id, hipStream_t s = nullptr) {
  if (c->prof) (void)hipEventRecord(c->ev1[id][c->pslot], s ? s : c->stream);
}
// after a device sync: fold the recorded event pairs into the averages
static void prof_collect(fasst_ctx *c) {
  if (!c->prof) return;
  for (int i = 0; i < fasst_ctx::kNK; ++i)
    for (int q = 0; q < fasst_ctx::kProfRing; ++q) {
      if (!c->used[i][q]) continue;
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, c->ev0[i][q], c->ev1[i][q]) == hipSuccess) {
        c->prof_ms[i] += ms;
        c->prof_cnt[i] += 1;
      }
      c->used[i][q] = 0;
    }
}

static int launch_grid(size_t n, int block = 256) {
  size_t g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  return (int)(g ? g : 1);
}

static int estep_occupancy(const fasst_ctx *c);
static int contract_occupancy(const fasst_ctx *c);
static int twl_occupancy(const fasst_ctx *c, int *units);
static int tpw_of(const fasst_ctx *c);
// bins per block of the FW update's f-contraction (k_fw_reduce holds three
// [fpc][KP] tiles in LDS: 96 KB at KP = 128 with 32 bins)
static int fw_fpc(const fasst_ctx *c) { return c->KP > 64 ? 32 : kFwFpc; }
// dynamic LDS of the kernels that stage FW ([KP][KP] when KP <= 64) next to
// `rest` doubles
static size_t fw_lds(const fasst_ctx *c, int rest) {
  return (size_t)((c->KP > 64 ? 0 : c->KP * c->KP) + rest) * sizeof(double);
}

// Split count c in [1, max_split] for a launch of unit * c equal blocks on
// `cap` resident slots: maximises the filled fraction of the last round
// (unit c / (cap ceil(unit c / cap))), preferring fewer splits within 1.5%.
static int best_split(long unit, long cap, int max_split) {
  max_split = std::max(1, max_split);
  auto eff = [&](int k) {
    const long blocks = unit * k;
    const long rounds = (blocks + cap - 1) / cap;
    return (double)blocks / (double)(rounds * cap);
  };
  double best = 0.0;
  for (int k = 1; k <= max_split; ++k) best = std::max(best, eff(k));
  for (int k = 1; k <= max_split; ++k)
    if (eff(k) >= best - 0.015) return k;
  return 1;
}

// Dynamic-LDS ceilings of the kernels whose launches may pass the 64 KB
// default, raised once per model configuration to the most any structure asks
// of them (not per iteration: the sizes depend only on the model shape, and
// a ceiling above a launch's own size costs nothing)
static int set_lds_limits() {
  struct L {
    const void *f;
    size_t bytes;
  };
  const L lim[] = {
      {(const void *)k_fw_reduce, (size_t)3 * 32 * kMaxKP * sizeof(double)},
      {(const void *)k_fwh_t<true>, (size_t)(16 + 64) * kMaxKP * sizeof(double)},
      {(const void *)k_egen_stats, (size_t)kEgsRows * 256 * sizeof(double)},
      {(const void *)k_egen_fused<4>, (size_t)(kEgsRows * 256 + kMaxJ * 16 * 16) * sizeof(double)},
      {(const void *)k_egen_fused<8>, (size_t)(kEgsRows * 256 + kMaxJ * 32 * 16) * sizeof(double)},
      {(const void *)k_mix<(4 * (kMaxJ * (kMaxJ + 1) / 2) + 8 * kMaxJ + 63) / 64, (kMaxR * kMaxR + 63) / 64>,
       mix_smem(kMaxJ, kMaxR, kMaxKP, 4 * (kMaxJ * (kMaxJ + 1) / 2) + 8 * kMaxJ)},
  };
  for (const L &l : lim)
    if (hipFuncSetAttribute(l.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l.bytes) != hipSuccess) {
      set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize, %zu) failed", l.bytes);
      return FASST_ERR_DEVICE;
    }
  return FASST_OK;
}

int configure_model(fasst_ctx *c, int J, const int *rank, const int *K, const int *convj) {
  if (J < 1 || J > kMaxJ) {
    set_error("J=%d outside the HIP path (1..%d sources)", J, kMaxJ);
    return FASST_ERR_UNSUPPORTED;
  }
  int R = 0, kmax = 0;
  for (int j = 0; j < J; ++j) {
    if (rank[j] < 1 || K[j] < 1) {
      set_error("bad rank/K for source %d", j);
      return FASST_ERR_SHAPE;
    }
    R += rank[j];
    kmax = std::max(kmax, K[j]);
  }
  if (R > kMaxR || kmax > kMaxKP) {
    set_error("total rank %d (max %d) / K %d (max %d) outside the HIP path", R, kMaxR, kmax,
              kMaxKP);
    return FASST_ERR_UNSUPPORTED;
  }
  if (int st = set_lds_limits()) return st;
  c->J = J;
  c->R = R;
  c->convm = 0;
  for (int j = 0; j < J; ++j)
    if (convj[j]) c->convm |= 1u << j;
  // conv: every source 'conv' (per-bin mixing update); otherwise the 'inst'
  // update runs over the free 'inst' sources with the rest held fixed
  const int conv = c->convm == (1u << J) - 1u ? 1 : 0;
  c->conv = conv;
  // the E-step addresses TW through a raw buffer resource with 32-bit byte
  // offsets (j KP + 4 s) Tp 8 (k_estep_mx's SA form)
  {
    const int KPc = kmax <= 16 ? 16 : (kmax <= 32 ? 32 : (kmax <= 64 ? 64 : 128));
    if ((size_t)J * KPc * c->Tp * sizeof(double) >= (1ull << 31)) {
      set_error("J %d x K %d x T %d: the TW plane passes the E-step's 2 GB buffer offsets", J,
                KPc, c->T);
      return FASST_ERR_UNSUPPORTED;
    }
  }
  c->KP = kmax <= 16 ? 16 : (kmax <= 32 ? 32 : (kmax <= 64 ? 64 : 128));
  c->roff[0] = 0;
  for (int j = 0; j < J; ++j) {
    c->rank[j] = rank[j];
    c->K[j] = K[j];
    c->roff[j + 1] = c->roff[j] + rank[j];
    c->spat_free[j] = c->fb_free[j] = c->tw_free[j] = 1;
    c->fw_free[j] = 0;
    c->nblk[j] = 1;   // one spectral component per source until fasst_set_blocks
    c->kb[j][0] = 0;
    c->kb[j][1] = K[j];
    c->bfb[j][0] = c->btw[j][0] = 1;
    c->bfw[j][0] = 0;
    c->soff[j] = j;
  }
  c->soff[J] = c->nslot = J;
  c->maxblk = 1;
  c->multi = 0;
  for (int j = 0; j < kMaxJ; ++j)
    for (int b = 0; b < kMaxBlk; ++b) {
      c->tb[j][b].release();
      c->tbl[j][b] = c->btb[j][b] = 0;
    }
  c->anytb = 0;
  c->nsrc = 0;
  c->lambda = 0.0;
  c->nseq = 0;
  const int Fp = c->Fp, Tp = c->Tp, KP = c->KP;
  // Launch shapes sized to whole rounds of resident blocks (a partial last
  // round idles most of the chip): E-step blocks = f tiles x frame chunks,
  // FB waves = bin-tile pairs x sources x frame chunks, TW waves = frame-tile
  // pairs x sources x bin chunks.
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const long cap_e = (long)estep_occupancy(c) * ncu;
  // (measured at C3: chunks of >= ~40 frame tiles keep the E-step's per-block
  // prologue/epilogue small; the contractions tolerate finer splits)
  c->nchunk_e = best_split(c->nft, cap_e, c->ntt / 40);
  if (const char *v = getenv("FASST_NCHUNK_E")) c->nchunk_e = std::max(1, std::min(atoi(v), c->ntt));
  c->tpc_e = (c->ntt + c->nchunk_e - 1) / c->nchunk_e;
  c->nchunk_e = (c->ntt + c->tpc_e - 1) / c->tpc_e;
  const long cap_b = (long)contract_occupancy(c) * ncu;
  c->nchunk_b = best_split((long)((c->nft + kFPW - 1) / kFPW) * J, cap_b, c->ntt / 32);
  if (const char *v = getenv("FASST_NCHUNK_B")) c->nchunk_b = std::max(1, std::min(atoi(v), c->ntt));
  c->tpc_b = (c->ntt + c->nchunk_b - 1) / c->nchunk_b;
  c->nchunk_b = (c->ntt + c->tpc_b - 1) / c->tpc_b;
  // (the bin split also multiplies k_tw_update's reduction: a fixed, small
  // split measured best at C3)
  c->nsplit_t = std::max(1, std::min(4, c->nft / 32));
  int tw_units = 0;
  const long cap_t = (long)twl_occupancy(c, &tw_units) * ncu;
  if ((long)tw_units * J * c->nsplit_t < cap_t)
    c->nsplit_t = best_split((long)tw_units * J, cap_t, c->nft / 16);
  if (const char *v = getenv("FASST_NSPLIT_T")) c->nsplit_t = std::max(1, std::min(atoi(v), c->nft));
  c->fpc_t = (c->nft + c->nsplit_t - 1) / c->nsplit_t;
  c->nsplit_t = (c->nft + c->fpc_t - 1) / c->fpc_t;
  if (getenv("FASST_VERBOSE"))
    fprintf(stderr,
            "fasst: %d CUs; estep %d chunks (cap %ld blocks); fb %d chunks (cap %ld); tw %d "
            "splits (cap %ld)\n",
            ncu, c->nchunk_e, cap_e, c->nchunk_b, cap_b, c->nsplit_t, cap_t);
  const int NP = J * (J + 1) / 2;
  c->nacc = 4 * NP + 8 * J;
  int st;
#define ALLOC(buf, n) \
  if ((st = c->buf.alloc(n)) != FASST_OK) return st
  ALLOC(FB, (size_t)J * Fp * KP);
  ALLOC(FW, (size_t)J * KP * KP);
  ALLOC(TW, (size_t)J * KP * Tp);
  ALLOC(Wkf, (size_t)J * KP * Fp);
  ALLOC(Wkf_new, (size_t)J * KP * Fp);
  ALLOC(Wfk_new, (size_t)J * Fp * KP);
  ALLOC(FWHt, (size_t)J * Tp * KP);
  ALLOC(hatW, (size_t)J * Tp * Fp);
  ALLOC(A, (size_t)R * 2 * Fp);
  ALLOC(Pinst, (size_t)R * 2);
  // (+8 chunks: the interleaved E-step / FB ranges round their chunks up)
  ALLOC(epart, (size_t)(c->nchunk_e + 8) * Fp * c->nacc);
  ALLOC(llpart, (size_t)(c->nchunk_e + 8) * c->nft);
  ALLOC(bnum, (size_t)(c->nchunk_b + 8) * J * Fp * KP);
  // FW update (free FW only, allocated with the model so set_spectral may switch it on)
  ALLOC(gden, (size_t)c->nchunk_b * J * Fp * KP);
  ALLOC(TWt, (size_t)J * Tp * KP);
  ALLOC(pnum, (size_t)((c->F + fw_fpc(c) - 1) / fw_fpc(c)) * J * KP * KP);
  ALLOC(pden, (size_t)((c->F + fw_fpc(c) - 1) / fw_fpc(c)) * J * KP * KP);
  ALLOC(tnum, (size_t)c->nsplit_t * J * Tp * KP);
  ALLOC(tden, (size_t)c->nsplit_t * J * Tp * KP);
  ALLOC(rss, conv ? 0 : (size_t)Fp * R * R);
  ALLOC(rxs, conv ? 0 : (size_t)Fp * 2 * R);
  ALLOC(flags, kNFlags);
  ALLOC(hsum, (size_t)J * KP);
  // renormalisation chunks (every stage-2 block re-reduces all stage-1
  // partials, so more chunks measured slower at C3)
  c->nchunk_r = std::max(1, std::min(64, std::min((c->T + 255) / 256, (c->F + 15) / 16)));
  ALLOC(rscal, (size_t)J * (2 + 2 * KP));
  ALLOC(rpmax, (size_t)J * c->nchunk_r * KP);
  ALLOC(rpe, (size_t)J * c->nchunk_r);
  ALLOC(rtpart, (size_t)kMaxSlot * c->nchunk_r);
  c->ntb = (Tp + 63) / 64;
  ALLOC(rpmax2, (size_t)J * c->nft * KP);
  ALLOC(rtpart2, (size_t)kMaxSlot * c->ntb);
  ALLOC(Wkf_next, (size_t)J * KP * Fp);
  ALLOC(hpart, (size_t)J * KP * c->ntb);
  if (J > 8 && KP > 32) {   // the two-pass E-step's scratch: V_j, N, P planes and per-tile logliks
    ALLOC(vgen, (size_t)J * Tp * Fp);
    ALLOC(npgen, (size_t)12 * Tp * Fp);
    ALLOC(lgen, (size_t)c->ntt * c->nft);
  } else {
    c->vgen.release();
    c->npgen.release();
    c->lgen.release();
  }
  c->w_ready = c->prep_ready = 0;
#undef ALLOC
  c->configured = 1;
  return FASST_OK;
}

int build_inst_A(fasst_ctx *c) {
  if (c->conv) return FASST_OK;
  unsigned rowm = 0;
  for (int j = 0; j < c->J; ++j)
    if (!(c->convm >> j & 1u))
      for (int r = c->roff[j]; r < c->roff[j + 1]; ++r) rowm |= 1u << r;
  prof_begin(c, KINSTA);
  k_inst_A<<<launch_grid((size_t)c->R * 2 * c->Fp), 256, 0, c->stream>>>(c->Pinst.p, c->A.p, c->R,
                                                                        c->F, c->Fp, rowm, c->halt);
  prof_end(c, KINSTA);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

int launch_w_old(fasst_ctx *c) {
  prof_begin(c, KW);
  (c->KP > 64 ? k_w_from_fb<true> : k_w_from_fb<false>)<<<dim3(c->nft, c->J), 256, fw_lds(c, 16 * (c->KP + 1)),
                c->stream>>>(c->FB.p, c->FW.p, c->Wkf.p, nullptr, c->J, c->Fp, c->KP, c->halt);
  prof_end(c, KW);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

static void update_multi(fasst_ctx *c) {
  c->anytb = 0;
  for (int j = 0; j < c->J; ++j)
    for (int b = 0; b < c->nblk[j]; ++b) c->anytb |= c->tbl[j][b] > 0;
  c->multi = c->maxblk > 1 || c->lambda > 0.0 || c->anytb;
}

// Time-blob arguments of step b (only_j as multi_step); which = 0: every
// block with time blobs, 1: those whose TW is free, 2: those whose TB is free
static TBArgs tb_args(const fasst_ctx *c, int b, int only_j, int which, double omega) {
  TBArgs a{};
  for (int j = 0; j < kMaxJ; ++j) {
    bool on = j < c->J && b < c->nblk[j] && c->tbl[j][b] > 0 && (only_j < 0 || j == only_j);
    if (on && which == 1) on = c->btw[j][b] != 0;
    if (on && which == 2) on = c->btb[j][b] != 0;
    a.tb[j] = on ? c->tb[j][b].p : nullptr;
    a.L[j] = on ? c->tbl[j][b] : 0;
    a.kb0[j] = on ? c->kb[j][b] : 0;
    a.kbw[j] = on ? c->kb[j][b + 1] - c->kb[j][b] : 0;
  }
  a.TW = c->TW.p;
  a.tnum = c->tnum.p;
  a.tden = c->tden.p;
  a.T = c->T;
  a.Tp = c->Tp;
  a.KP = c->KP;
  a.J = c->J;
  a.nsplit = c->nsplit_t;
  a.omega = omega;
  a.flags = nullptr;
  a.iter = -1;
  a.halt = c->halt;
  return a;
}

static bool tb_any(const TBArgs &a, int *lmax, int *kwmax) {
  bool any = false;
  *lmax = *kwmax = 0;
  for (int j = 0; j < kMaxJ; ++j)
    if (a.tb[j]) {
      any = true;
      *lmax = std::max(*lmax, a.L[j]);
      *kwmax = std::max(*kwmax, a.kbw[j]);
    }
  return any;
}

static int launch_tb_h(fasst_ctx *c, const TBArgs &a) {
  int lmax, kwmax;
  if (!tb_any(a, &lmax, &kwmax)) return FASST_OK;
  k_tb_h<<<dim3((c->Tp + 255) / 256, c->J), 256, (size_t)kwmax * lmax * sizeof(double),
           c->stream>>>(a);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

static RArgs renorm_args(fasst_ctx *c) {
  RArgs r{};
  r.A = c->A.p;
  r.Pinst = c->Pinst.p;
  r.FB = c->FB.p;
  r.FW = c->FW.p;
  r.TW = c->TW.p;
  r.scal = c->rscal.p;
  r.pmax = c->rpmax.p;
  r.pe = c->rpe.p;
  r.tpart = c->rtpart.p;
  r.flags = c->flags.p;
  r.halt = c->halt;
  r.F = c->F;
  r.T = c->T;
  r.Fp = c->Fp;
  r.Tp = c->Tp;
  r.KP = c->KP;
  r.convm = c->convm;
  r.nchunk = c->nchunk_r;
  r.tpc = (c->T + c->nchunk_r - 1) / c->nchunk_r;
  r.fpc = (c->F + c->nchunk_r - 1) / c->nchunk_r;
  r.nslot = c->nslot;
  r.tbmask = 0;
  for (int j = 0; j < c->J; ++j)
    for (int b = 0; b < c->nblk[j]; ++b)
      if (c->tbl[j][b] > 0) r.tbmask |= 1u << (c->soff[j] + b);
  for (int j = 0; j < kMaxJ; ++j) {
    r.K[j] = j < c->J ? c->K[j] : 0;
    r.nblk[j] = j < c->J ? c->nblk[j] : 0;
    for (int b = 0; b <= kMaxBlk; ++b) r.kb[j][b] = j < c->J ? c->kb[j][b] : 0;
  }
  for (int j = 0; j <= kMaxJ; ++j) {
    r.roff[j] = j <= c->J ? c->roff[j] : c->R;
    r.soff[j] = j <= c->J ? c->soff[j] : c->nslot;
  }
  r.pmax2 = c->rpmax2.p;
  r.tpart2 = c->rtpart2.p;
  r.llpart = c->llpart.p;
  r.ll_out = nullptr;
  r.inv_FT = 1.0 / ((double)c->F * (double)c->T);
  r.nstat = c->nft;
  r.ntb = c->ntb;
  r.nll = c->nchunk_e * c->nft;
  return r;
}

static int launch_renorm(fasst_ctx *c, int iter) {
  RArgs r = renorm_args(c);
  prof_begin(c, KREN);
  k_renorm_stats<<<dim3(c->nchunk_r, c->J), 256, 0, c->stream>>>(r);
  if (c->nchunk_r * c->KP > 64 * 64 || c->KP > 64)
    k_renorm_apply<true><<<dim3(c->nchunk_r, c->J), 256, 0, c->stream>>>(r);
  else
    k_renorm_apply<false><<<dim3(c->nchunk_r, c->J), 256, 0, c->stream>>>(r);
  k_renorm_final<<<1, 256, 0, c->stream>>>(r, c->J, iter);
  FASST_LAUNCH_CHECK();
  if (c->anytb) {
    TBRArgs tr{};
    tr.scal = c->rscal.p;
    tr.flags = c->flags.p;
    tr.halt = c->halt;
    tr.T = c->T;
    tr.Tp = c->Tp;
    tr.KP = c->KP;
    tr.iter = iter;
    for (int j = 0; j < kMaxJ; ++j)
      for (int b = 0; b < kMaxBlk; ++b) {
        const bool on = j < c->J && b < c->nblk[j] && c->tbl[j][b] > 0;
        tr.tb[j][b] = on ? c->tb[j][b].p : nullptr;
        tr.L[j][b] = on ? c->tbl[j][b] : 0;
        tr.kb0[j][b] = on ? c->kb[j][b] : 0;
        tr.kbw[j][b] = on ? c->kb[j][b + 1] - c->kb[j][b] : 0;
        tr.slot[j][b] = on ? c->soff[j] + b : 0;
      }
    k_tb_renorm<<<dim3(kMaxBlk, c->J), 256, 0, c->stream>>>(tr);
    FASST_LAUNCH_CHECK();
    for (int b = 0; b < c->maxblk; ++b) {
      TBArgs ta = tb_args(c, b, -1, 0, 1.0);
      ta.flags = c->flags.p;
      ta.iter = iter;
      if (int st = launch_tb_h(c, ta)) return st;
    }
  }
  prof_end(c, KREN);
  return FASST_OK;
}

// gem_iteration's fused renormalisation tail (§3.3a of DESIGN.md; see
// k_renorm_scales), the default for the structures it covers: one spectral
// component per source (!multi), no time blobs (!anytb), no free FW.  The
// context's ftail (FASST_FAST_TAIL, read at creation) selects the form:
//   0  the unfused k_renorm_stats / _apply / _final (the A/B reference);
//   1  the fused tail: k_fb_update's stage-1 statistics, k_renorm_scales /
//      _rows and the next W on the side stream beside the TW contraction,
//      the TW rescale inside k_tw_update, k_renorm_tail;
//   2  (default) as 1, and at KP <= 64 k_tw_update also forms the next
//      iteration's (FW.TW)^T and TW row-sum partials (reduced into hsum by
//      k_renorm_tail), so the next iteration of the batch skips
//      launch_spectral_prep.
// Every form is tested against the others and the oracle, halted batches
// included (tests/test_gpu_fast_tail.py).
static bool fast_tail(const fasst_ctx *c) {
  if (!c->ftail || c->multi || c->anytb) return false;
  for (int j = 0; j < c->J; ++j)
    if (c->fw_free[j]) return false;
  return true;
}

// update_mix_matrix (audioModel.py:766-889) on stream s: k_mix (per-bin
// statistics, hat_Rss / hat_Rxs, the 'conv' solves) and k_mix_inst (the
// 'inst' f-mean solve), when some spatial component is free
static int launch_mix(fasst_ctx *c, hipStream_t s) {
  const int J = c->J;
  bool any_free = false;
  for (int j = 0; j < J; ++j) any_free |= c->spat_free[j] != 0;
  if (any_free) {
    MArgs m{};
    m.part = c->epart.p;
    m.Wkf = c->Wkf.p;
    m.hsum = c->hsum.p;
    m.KP = c->KP;
    m.A = c->A.p;
    m.rss = c->rss.p;
    m.rxs = c->rxs.p;
    m.flags = c->flags.p;
    m.halt = c->halt;
    m.F = c->F;
    m.Fp = c->Fp;
    m.J = J;
    m.R = c->R;
    m.nchunk = c->nchunk_e;
    m.nacc = c->nacc;
    m.conv_update = c->conv ? 1 : 0;
    m.invT = 1.0 / (double)c->T;
    for (int j = 0; j < J; ++j)
      for (int r = c->roff[j]; r < c->roff[j + 1]; ++r) m.jr[r] = j;
    prof_begin(c, KMIX, s);
    {
      const size_t ms = mix_smem(J, c->R, c->KP, c->nacc);
      const int q = (c->nacc + 63) / 64;
      constexpr int QX = (4 * (kMaxJ * (kMaxJ + 1) / 2) + 8 * kMaxJ + 63) / 64;
      if (c->R > 16) {   // (R^2 > 256 hat_Rss entries: 16 per lane; up to ~73 KB of LDS)
        k_mix<QX, (kMaxR * kMaxR + 63) / 64><<<c->F, 64, ms, s>>>(m);
      }
      else if (q <= 2)
        k_mix<2><<<c->F, 64, ms, s>>>(m);
      else if (q <= 4)   // (J <= 8: 4 J (J + 1) / 2 + 8 J <= 208)
        k_mix<4><<<c->F, 64, ms, s>>>(m);
      else
        k_mix<QX><<<c->F, 64, ms, s>>>(m);
    }
    prof_end(c, KMIX, s);
    FASST_LAUNCH_CHECK();
    if (!c->conv) {
      IArgs ia{};
      ia.rss = c->rss.p;
      ia.rxs = c->rxs.p;
      ia.A = c->A.p;
      ia.Pinst = c->Pinst.p;
      ia.flags = c->flags.p;
      ia.halt = c->halt;
      ia.F = c->F;
      ia.Fp = c->Fp;
      ia.R = c->R;
      ia.nu = ia.no = 0;
      for (int j = 0; j < J; ++j)
        for (int r = c->roff[j]; r < c->roff[j + 1]; ++r) {
          if (c->spat_free[j])
            ia.upd[ia.nu++] = r;
          else
            ia.oth[ia.no++] = r;
        }
      prof_begin(c, KMIXI, s);
      k_mix_inst<<<1, 256, 0, s>>>(ia);
      prof_end(c, KMIXI, s);
      FASST_LAUNCH_CHECK();
    }
  }
  return FASST_OK;
}

// the scales and the FB / mixing / FW rescale, after k_fb_update: on the side
// stream beside the TW contraction; ev_scales gates k_tw_update, ev_rows the
// iteration's end
static int launch_tail_side(fasst_ctx *c) {
  const RArgs r = renorm_args(c);
  hipStream_t side = c->aux;
  FASST_HIP(hipEventRecord(c->ev_tail, c->stream));
  FASST_HIP(hipStreamWaitEvent(c->aux, c->ev_tail, 0));
  prof_begin(c, KREN, side);
  k_renorm_scales<<<c->J, 1024, 0, side>>>(r);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipEventRecord(c->ev_scales, c->aux));
  k_renorm_rows<<<dim3(c->nft, c->J), 256, 0, side>>>(r);
  FASST_LAUNCH_CHECK();
  prof_end(c, KREN, side);
  // the next iteration's W (the TW contraction still reads Wkf)
  prof_begin(c, KW, side);
  (c->KP > 64 ? k_w_from_fb<true> : k_w_from_fb<false>)<<<dim3(c->nft, c->J), 256,
                fw_lds(c, 16 * (c->KP + 1)), side>>>(c->FB.p, c->FW.p, c->Wkf_next.p, nullptr,
                                                     c->J, c->Fp, c->KP, c->halt);
  prof_end(c, KW, side);
  FASST_LAUNCH_CHECK();
  FASST_HIP(hipEventRecord(c->ev_rows, c->aux));
  return FASST_OK;
}

// E-step instantiation chosen from the model structure; `f` receives an
// ETag carrying the template parameters (used for launches and occupancy).
template <int J_, int NKS_, int RKU_>
struct ETag {
  static constexpr int J = J_, NKS = NKS_, RKU = RKU_;
};

template <int J, int NKS, class F>
static void estep_dispatch_r(const fasst_ctx *c, F &&f) {
  bool all1 = true, all2 = true;
  for (int j = 0; j < J; ++j) {
    all1 &= c->rank[j] == 1;
    all2 &= c->rank[j] == 2;
  }
  if (all1)
    f(ETag<J, NKS, 1>{});
  else if (all2)
    f(ETag<J, NKS, 2>{});
  else
    f(ETag<J, NKS, 0>{});
}

template <int J, class F>
static void estep_dispatch_j(const fasst_ctx *c, F &&f) {
  switch (c->KP) {
    case 16: estep_dispatch_r<J, 4>(c, f); break;
    case 32: estep_dispatch_r<J, 8>(c, f); break;
    case 64: estep_dispatch_r<J, 16>(c, f); break;
    default: f(ETag<J, 32, 0>{}); break;   // K up to 128: general ranks only
  }
}

template <class F>
static void estep_dispatch(const fasst_ctx *c, F &&f) {
  switch (c->J) {
    case 1: estep_dispatch_j<1>(c, f); break;
    case 2: estep_dispatch_j<2>(c, f); break;
    case 3: estep_dispatch_j<3>(c, f); break;
    case 4: estep_dispatch_j<4>(c, f); break;
    case 5: estep_dispatch_j<5>(c, f); break;
    case 6: estep_dispatch_j<6>(c, f); break;
    case 7: estep_dispatch_j<7>(c, f); break;
    default: estep_dispatch_j<8>(c, f); break;
  }
}

static void launch_estep(fasst_ctx *c, const EArgs &e, int ny) {
  estep_dispatch(c, [&](auto tag) {
    using T = decltype(tag);
    prof_begin(c, KESTEP);
    k_estep_mx<T::J, T::NKS, T::RKU>
        <<<dim3(c->nft, ny), 256, estep_mx_smem<T::J, T::NKS>(), c->stream>>>(e);
    prof_end(c, KESTEP);
  });
}

// resident E-step blocks per CU
static int estep_occupancy(const fasst_ctx *c) {
  int occ = 1;
  estep_dispatch(c, [&](auto tag) {
    using T = decltype(tag);
    constexpr size_t smem = estep_mx_smem<T::J, T::NKS>();
    (void)hipFuncSetAttribute((const void *)k_estep_mx<T::J, T::NKS, T::RKU>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_estep_mx<T::J, T::NKS, T::RKU>, 256,
                                                     smem) != hipSuccess)
      n = 1;
    occ = std::max(1, n);
  });
  return occ;
}

// frame tiles per wave of the TW contraction: KP = 128 keeps one (its
// numerator / denominator tiles alone fill 128 VGPRs)
template <int NKC>
constexpr int tpw_for() { return NKC > 4 ? 1 : kTPW; }
static int tpw_of(const fasst_ctx *c) { return c->KP > 64 ? 1 : kTPW; }

static void launch_fw_reduce(fasst_ctx *c, const FWArgs &w) {
  const size_t lds = (size_t)3 * w.fpc * c->KP * sizeof(double);   // (ceiling: set_lds_limits)
  k_fw_reduce<<<dim3(w.nfc, c->J), 256, lds, c->stream>>>(w);
}

// k_tw_contract_lds's shape: 8 waves per block, one frame tile per wave, two
// LDS stages (C3 same-box A/B, k_tw_contract 0.395 ms: NW x TPW x NS = 8 x 1 x
// 2 0.378, 4 x 2 x 2 0.379, 4 x 1 x 3 0.396, 4 x 2 x 3 0.437 ms; the other
// shapes and the register-operand k_tw_contract of rounds 1-4 were deleted
// after the A/B)
template <int NKC>
using TwlShape = TwlCfg<NKC, 8, 1, 2>;

template <int NKC>
static void launch_contract(fasst_ctx *c, const BArgs &b, const TArgs &t, bool fb, int nz = 0) {
  if (fb) {
    prof_begin(c, KFBC);
    k_fb_contract<NKC, kFPW><<<dim3((c->nft + kFPW - 1) / kFPW, c->J, nz ? nz : c->nchunk_b), 64,
                               0, c->stream>>>(b);
    prof_end(c, KFBC);
    return;
  }
  using CF = TwlShape<NKC>;
  prof_begin(c, KTWC);
  const int g = (c->ntt + CF::NW_ * CF::TPW_ - 1) / (CF::NW_ * CF::TPW_);
  k_tw_contract_lds<CF><<<dim3(g, c->J, c->nsplit_t), CF::NT, CF::smem, c->stream>>>(t);
  prof_end(c, KTWC);
}

// resident k_tw_contract_lds blocks per CU, and its frame-tile groups (units)
template <int NKC>
static int twl_occ_of(const fasst_ctx *c, int *units) {
  using CF = TwlShape<NKC>;
  (void)hipFuncSetAttribute((const void *)k_tw_contract_lds<CF>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)CF::smem);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_tw_contract_lds<CF>, CF::NT, CF::smem) !=
      hipSuccess)
    n = 1;
  *units = (c->ntt + CF::NW_ * CF::TPW_ - 1) / (CF::NW_ * CF::TPW_);
  return std::max(1, n);
}
static int twl_occupancy(const fasst_ctx *c, int *units) {
  switch (c->KP) {
    case 16: return twl_occ_of<1>(c, units);
    case 32: return twl_occ_of<2>(c, units);
    case 64: return twl_occ_of<4>(c, units);
    default: return twl_occ_of<8>(c, units);
  }
}

// resident k_fb_contract waves per CU
static int contract_occupancy(const fasst_ctx *c) {
  int n = 1;
  hipError_t e = hipSuccess;
  switch (c->KP / 16) {
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fb_contract<1, kFPW>, 64, 0); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fb_contract<2, kFPW>, 64, 0); break;
    case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fb_contract<4, kFPW>, 64, 0); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fb_contract<8, kFPW>, 64, 0); break;
  }
  return e == hipSuccess ? std::max(1, n) : 1;
}

// Spectral update of a model with several spectral components on some source
// (see k_multi_prep): step b updates block b of every source that has one
// (FB, then TW), all launches on c->stream; W = FB FW of the step's result
// becomes the next step's current W.
// one step: block b of every source that has one (only_j < 0), or of source
// only_j alone (lambdaCorr > 0: the penalty couples the sources, so the
// components go one at a time in the reference's key order)
// The fused-tail pointers of k_fb_update / k_tw_update are null or the
// context's own buffers; anything else is refused here, on the host, before a
// kernel could dereference it (an uninitialised argument struct on the
// multi-block path once sent garbage pointers to the device)
static int check_tail_args(const fasst_ctx *c, const UArgs &u, const TUArgs &tu) {
  const bool ok_u = !u.pmax || u.pmax == c->rpmax2.p;
  const bool ok_t = !tu.scal || (tu.scal == c->rscal.p && tu.tpart == c->rtpart2.p &&
                                 (!tu.FWHt || (tu.FWHt == c->FWHt.p && tu.hpart == c->hpart.p &&
                                               tu.FW == c->FW.p)));
  if (ok_u && ok_t) return FASST_OK;
  set_error("internal: fused renormalisation arguments do not point at the context's buffers");
  return FASST_ERR_SHAPE;
}

static int multi_step(fasst_ctx *c, double omega, int b, int only_j) {
  const int J = c->J, nkc = c->KP / 16;
  const size_t plane = (size_t)J * c->Tp * c->Fp;
  const bool lam = c->lambda > 0.0;
  {
    MPArgs mp{};
    mp.TW = c->TW.p;
    mp.Wkf = c->Wkf.p;
    mp.hatW = c->hatW.p;
    mp.rnum = c->mplanes.p;
    mp.rden = c->mplanes.p + plane;
    mp.rtw = c->mplanes.p + 2 * plane;
    mp.rcp = c->mplanes.p + 3 * plane;
    mp.rpow = c->mplanes.p + 4 * plane;
    mp.roth = nullptr;
    mp.lambda = c->lambda;
    mp.F = c->F;
    mp.T = c->T;
    mp.Fp = c->Fp;
    mp.Tp = c->Tp;
    mp.KP = c->KP;
    mp.J = J;
    mp.ntt = c->ntt;
    mp.tpc = c->tpc_b;
    mp.first = b == 0;
    mp.halt = c->halt;
    BArgs bb{};
    bb.TW = c->TW.p;
    bb.Wkf = c->Wkf.p;
    bb.FWHt = c->FWHt.p;
    bb.hatW = mp.rnum;
    bb.hatW2 = mp.rden;
    bb.bnum = c->bnum.p;
    bb.bden = c->bden.p;
    bb.halt = c->halt;
    bb.F = c->F;
    bb.T = c->T;
    bb.Fp = c->Fp;
    bb.Tp = c->Tp;
    bb.KP = c->KP;
    bb.J = J;
    bb.ntt = c->ntt;
    bb.nft = c->nft;
    bb.tpc = c->tpc_b;
    bb.zbase = bb.tbase = 0;
    UArgs u{};   // (pmax null: no fused-tail statistics on this path)
    u.FB = c->FB.p;
    u.FW = c->FW.p;
    u.bnum = c->bnum.p;
    u.bden = c->bden.p;
    u.hsum = c->hsum.p;
    u.Wkf_new = c->Wkf_new.p;
    u.Wfk_new = c->Wfk_new.p;
    u.halt = c->halt;
    u.F = c->F;
    u.Fp = c->Fp;
    u.KP = c->KP;
    u.J = J;
    u.nchunk = c->nchunk_b;
    u.omega = omega;
    TArgs t{};
    t.TW = c->TW.p;
    t.Wkf_old = c->Wkf.p;
    t.Wkf_new = c->Wkf_new.p;
    t.Wfk_new = c->Wfk_new.p;
    t.hatW = mp.rtw;
    t.tnum = c->tnum.p;
    t.tden = c->tden.p;
    t.halt = c->halt;
    t.F = c->F;
    t.T = c->T;
    t.Fp = c->Fp;
    t.Tp = c->Tp;
    t.KP = c->KP;
    t.J = J;
    t.nft = c->nft;
    t.ntt = c->ntt;
    t.fpc = c->fpc_t;
    TUArgs tu{};   // (scal null: the plain TW update)
    tu.TW = c->TW.p;
    tu.tnum = c->tnum.p;
    tu.tden = c->tden.p;
    tu.halt = c->halt;
    tu.T = c->T;
    tu.Tp = c->Tp;
    tu.KP = c->KP;
    tu.J = J;
    tu.nsplit = c->nsplit_t;
    tu.omega = omega;
    t.cp = mp.rcp;
    t.pw = mp.rpow;
    t.oth = nullptr;
    t.omega = omega;
    const TBArgs tbw = tb_args(c, b, only_j, 1, omega), tbb = tb_args(c, b, only_j, 2, omega);
    int lmax, kwmax;
    const bool any_tbb = tb_any(tbb, &lmax, &kwmax);
    if (any_tbb) mp.roth = c->mplanes.p + 5 * plane;
    for (int j = 0; j < kMaxJ; ++j) {
      const bool has = j < J && b < c->nblk[j] && (only_j < 0 || j == only_j);
      mp.on[j] = has;
      const int k0 = has ? c->kb[j][b] : 0, k1 = has ? c->kb[j][b + 1] : 0;
      mp.kb0[j] = u.kb0[j] = t.kb0[j] = tu.kb0[j] = k0;
      mp.kb1[j] = u.kb1[j] = t.kb1[j] = tu.kb1[j] = k1;
      bb.fb_free[j] = u.fb_free[j] = has && c->bfb[j][b];
      t.tw_free[j] = has && c->btw[j][b];
      tu.tw_free[j] = t.tw_free[j] && !tbw.tb[j];   // time blobs: k_tb_tw_red / apply
    }
    const dim3 gp(c->nft, J, c->nchunk_b);
    const dim3 gb((c->nft + kFPW - 1) / kFPW, J, c->nchunk_b);
    const dim3 gt((c->ntt + tpw_of(c) - 1) / tpw_of(c), J, c->nsplit_t);
    switch (nkc) {
      case 1:
        if (lam) k_multi_prep<1, true><<<gp, 64, 0, c->stream>>>(mp);
        else k_multi_prep<1><<<gp, 64, 0, c->stream>>>(mp);
        k_fb_contract<1, kFPW, true><<<gb, 64, 0, c->stream>>>(bb);
        break;
      case 2:
        if (lam) k_multi_prep<2, true><<<gp, 64, 0, c->stream>>>(mp);
        else k_multi_prep<2><<<gp, 64, 0, c->stream>>>(mp);
        k_fb_contract<2, kFPW, true><<<gb, 64, 0, c->stream>>>(bb);
        break;
      case 4:
        if (lam) k_multi_prep<4, true><<<gp, 64, 0, c->stream>>>(mp);
        else k_multi_prep<4><<<gp, 64, 0, c->stream>>>(mp);
        k_fb_contract<4, kFPW, true><<<gb, 64, 0, c->stream>>>(bb);
        break;
      default:   // KP = 128
        if (lam) k_multi_prep<8, true><<<gp, 64, 0, c->stream>>>(mp);
        else k_multi_prep<8><<<gp, 64, 0, c->stream>>>(mp);
        k_fb_contract<8, kFPW, true><<<gb, 64, 0, c->stream>>>(bb);
        break;
    }
    FASST_LAUNCH_CHECK();
    if (int st = check_tail_args(c, u, tu)) return st;
    (c->KP > 64 ? k_fb_update<true> : k_fb_update<false>)<<<dim3(c->nft, J), 256,
                  fw_lds(c, 16 * (c->KP + 1) + c->KP + 16 * (c->KP + 1)),
                  c->stream>>>(u);
    FASST_LAUNCH_CHECK();
    bool any_fw = false;
    for (int j = 0; j < J; ++j) any_fw |= b < c->nblk[j] && c->bfw[j][b] && (only_j < 0 || j == only_j);
    if (any_fw) {
      // FW update of the step's components (:1578-1631): V_mid = (FB_new FW) H
      // of the component, then W_new rebuilt with FW_new
      FWArgs w{};
      w.TW = c->TW.p;
      w.TWt = c->TWt.p;
      w.Wkf_old = c->Wkf.p;
      w.Wkf_mid = c->Wkf_new.p;
      w.hatW = mp.rtw;
      w.FB = c->FB.p;
      w.gnum = c->bnum.p;
      w.gden = c->gden.p;
      w.pnum = c->pnum.p;
      w.pden = c->pden.p;
      w.FW = c->FW.p;
      w.F = c->F;
      w.T = c->T;
      w.Fp = c->Fp;
      w.Tp = c->Tp;
      w.KP = c->KP;
      w.J = J;
      w.ntt = c->ntt;
      w.tpc = c->tpc_b;
      w.nchunk = c->nchunk_b;
      w.fpc = fw_fpc(c);
      w.nfc = (c->F + w.fpc - 1) / w.fpc;
      w.omega = omega;
      w.halt = c->halt;
      w.cp = mp.rcp;
      w.pw = mp.rpow;
      for (int j = 0; j < kMaxJ; ++j) {
        const bool has = j < J && b < c->nblk[j] && (only_j < 0 || j == only_j);
        w.K[j] = j < J ? c->K[j] : 0;
        w.fw_free[j] = has && c->bfw[j][b];
        w.kb0[j] = has ? c->kb[j][b] : 0;
        w.kb1[j] = has ? c->kb[j][b + 1] : 0;
      }
      const dim3 gc(c->nft, J, c->nchunk_b);
      switch (nkc) {
        case 1:
          if (lam) k_fw_contract<1, true, true><<<gc, 64, 0, c->stream>>>(w);
          else k_fw_contract<1, true><<<gc, 64, 0, c->stream>>>(w);
          break;
        case 2:
          if (lam) k_fw_contract<2, true, true><<<gc, 64, 0, c->stream>>>(w);
          else k_fw_contract<2, true><<<gc, 64, 0, c->stream>>>(w);
          break;
        case 4:
          if (lam) k_fw_contract<4, true, true><<<gc, 64, 0, c->stream>>>(w);
          else k_fw_contract<4, true><<<gc, 64, 0, c->stream>>>(w);
          break;
        default:
          if (lam) k_fw_contract<8, true, true><<<gc, 64, 0, c->stream>>>(w);
          else k_fw_contract<8, true><<<gc, 64, 0, c->stream>>>(w);
          break;
      }
      launch_fw_reduce(c, w);
      k_fw_final<<<J, 256, 0, c->stream>>>(w);
      (c->KP > 64 ? k_w_from_fb<true> : k_w_from_fb<false>)<<<dim3(c->nft, J), 256, fw_lds(c, 16 * (c->KP + 1)),
                    c->stream>>>(c->FB.p, c->FW.p, c->Wkf_new.p, c->Wfk_new.p, J, c->Fp, c->KP,
                                 c->halt);
      FASST_LAUNCH_CHECK();
    }
    switch (nkc) {
      case 1:
        if (lam) k_tw_contract<1, kTPW, true, true><<<gt, 64, 0, c->stream>>>(t);
        else k_tw_contract<1, kTPW, true><<<gt, 64, 0, c->stream>>>(t);
        break;
      case 2:
        if (lam) k_tw_contract<2, kTPW, true, true><<<gt, 64, 0, c->stream>>>(t);
        else k_tw_contract<2, kTPW, true><<<gt, 64, 0, c->stream>>>(t);
        break;
      case 4:
        if (lam) k_tw_contract<4, kTPW, true, true><<<gt, 64, 0, c->stream>>>(t);
        else k_tw_contract<4, kTPW, true><<<gt, 64, 0, c->stream>>>(t);
        break;
      default:   // (one frame tile per wave at KP = 128)
        if (lam) k_tw_contract<8, 1, true, true><<<gt, 64, 0, c->stream>>>(t);
        else k_tw_contract<8, 1, true><<<gt, 64, 0, c->stream>>>(t);
        break;
    }
    FASST_LAUNCH_CHECK();
    k_tw_update<<<dim3((c->Tp + 63) / 64, J), 256, 0, c->stream>>>(tu);
    FASST_LAUNCH_CHECK();
    if (tb_any(tbw, &lmax, &kwmax)) {   // TW with time blobs (:1665-1691)
      k_tb_tw_red<<<dim3(lmax, (kwmax + 15) / 16, J), 256, 0, c->stream>>>(tbw);
      k_tb_tw_apply<<<J, 256, 0, c->stream>>>(tbw);
      FASST_LAUNCH_CHECK();
      if (int st = launch_tb_h(c, tbw)) return st;
    }
    if (tb_any(tbb, &lmax, &kwmax)) {   // TB (:1931-1978) with the updated H
      TArgs t2 = t;
      t2.hatW = c->hatW.p;
      t2.oth = mp.roth;
      for (int j = 0; j < kMaxJ; ++j) t2.tw_free[j] = tbb.tb[j] != nullptr;
      switch (nkc) {
        case 1:
          if (lam) k_tw_contract<1, kTPW, true, true, true><<<gt, 64, 0, c->stream>>>(t2);
          else k_tw_contract<1, kTPW, true, false, true><<<gt, 64, 0, c->stream>>>(t2);
          break;
        case 2:
          if (lam) k_tw_contract<2, kTPW, true, true, true><<<gt, 64, 0, c->stream>>>(t2);
          else k_tw_contract<2, kTPW, true, false, true><<<gt, 64, 0, c->stream>>>(t2);
          break;
        case 4:
          if (lam) k_tw_contract<4, kTPW, true, true, true><<<gt, 64, 0, c->stream>>>(t2);
          else k_tw_contract<4, kTPW, true, false, true><<<gt, 64, 0, c->stream>>>(t2);
          break;
        default:
          if (lam) k_tw_contract<8, 1, true, true, true><<<gt, 64, 0, c->stream>>>(t2);
          else k_tw_contract<8, 1, true, false, true><<<gt, 64, 0, c->stream>>>(t2);
          break;
      }
      k_tb_tb_upd<<<dim3((c->T + 63) / 64, J), 64,
                    (size_t)(kwmax * lmax + 2 * 64 * lmax) * sizeof(double), c->stream>>>(tbb);
      FASST_LAUNCH_CHECK();
      if (int st = launch_tb_h(c, tbb)) return st;
    }
    // the step's W = FB FW is the current W of the next step
    FASST_HIP(hipMemcpyAsync(c->Wkf.p, c->Wkf_new.p, (size_t)J * c->KP * c->Fp * sizeof(double),
                             hipMemcpyDeviceToDevice, c->stream));
  }
  return FASST_OK;
}

static int multi_spectral(fasst_ctx *c, double omega) {
  int st;
  if (c->lambda > 0.0) {
    for (int q = 0; q < c->nseq; ++q)
      if ((st = multi_step(c, omega, c->seq_b[q], c->seq_j[q]))) return st;
    return FASST_OK;
  }
  for (int b = 0; b < c->maxblk; ++b)
    if ((st = multi_step(c, omega, b, -1))) return st;
  return FASST_OK;
}

// (FW.TW)^T and the TW row sums of the previous parameters, the operands of
// the spectral update; fork: on the side stream (joined by the caller
// through ev_join before their first consumer)
static int launch_spectral_prep(fasst_ctx *c, bool fork) {
  const int J = c->J;
  hipStream_t side = fork ? c->aux : c->stream;
  if (fork) {
    FASST_HIP(hipEventRecord(c->ev_fork, c->stream));
    FASST_HIP(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
  }
  prof_begin(c, KFWH, side);
  bool any_fw = false;
  for (int j = 0; j < J; ++j) any_fw |= c->fw_free[j] != 0;
  // (KP > 64: 16-row FW chunk + TW tile, 80 KB of LDS, two blocks per CU;
  // ceiling set by set_lds_limits)
  (c->KP > 64 ? k_fwh_t<true> : k_fwh_t<false>)<<<dim3((c->Tp + 63) / 64, J), 256,
            c->KP > 64 ? (16 + 64) * c->KP * sizeof(double) : fw_lds(c, c->KP * 64),
            side>>>(c->FW.p, c->TW.p, c->FWHt.p, any_fw ? c->TWt.p : nullptr, J, c->Tp, c->KP,
                    c->halt);
  prof_end(c, KFWH, side);
  FASST_LAUNCH_CHECK();
  prof_begin(c, KROWS, side);
  k_tw_rowsum<<<J * c->KP, 256, 0, side>>>(c->TW.p, c->hsum.p, c->T, c->Tp, c->halt);
  prof_end(c, KROWS, side);
  FASST_LAUNCH_CHECK();
  if (fork) FASST_HIP(hipEventRecord(c->ev_join, c->aux));
  return FASST_OK;
}

// update_spectral_components (audioModel.py:1469-1978) from the rho planes in
// c->hatW (rho_j = hat_W_j / max(V_j, eps), V from the parameters before the
// update), after launch_spectral_prep and launch_w_old.  tail (fast_tail
// models inside gem_iteration): the fused renormalisation tail, its scales /
// rescale forked onto the side stream beside the TW contraction
static int spectral_update(fasst_ctx *c, double omega, bool tail = false) {
  const int J = c->J;
  const int nkc = c->KP / 16;
  bool any_fw = false;
  for (int j = 0; j < J; ++j) any_fw |= c->fw_free[j] != 0;
  if (c->multi) return multi_spectral(c, omega);
  BArgs b{};
  b.TW = c->TW.p;
  b.Wkf = c->Wkf.p;
  b.FWHt = c->FWHt.p;
  b.hatW = c->hatW.p;
  b.hatW2 = nullptr;
  b.bnum = c->bnum.p;
  b.bden = nullptr;
  b.halt = c->halt;
  b.F = c->F;
  b.T = c->T;
  b.Fp = c->Fp;
  b.Tp = c->Tp;
  b.KP = c->KP;
  b.J = J;
  b.ntt = c->ntt;
  b.nft = c->nft;
  b.tpc = c->tpc_b;
  b.zbase = b.tbase = 0;
  for (int j = 0; j < kMaxJ; ++j) b.fb_free[j] = j < J ? c->fb_free[j] : 0;
  // spectral update: FB then TW (one NMF factor per source)
  TArgs t{};
  t.TW = c->TW.p;
  t.Wkf_old = c->Wkf.p;
  t.Wkf_new = c->Wkf_new.p;
  t.Wfk_new = c->Wfk_new.p;
  t.hatW = c->hatW.p;
  t.tnum = c->tnum.p;
  t.halt = c->halt;
  t.tden = c->tden.p;
  t.F = c->F;
  t.T = c->T;
  t.Fp = c->Fp;
  t.Tp = c->Tp;
  t.KP = c->KP;
  t.J = J;
  t.nft = c->nft;
  t.ntt = c->ntt;
  t.fpc = c->fpc_t;
  t.cp = t.pw = t.oth = nullptr;
  t.omega = omega;
  TUArgs tu{};
  tu.TW = c->TW.p;
  tu.tnum = c->tnum.p;
  tu.halt = c->halt;
  tu.tden = c->tden.p;
  tu.T = c->T;
  tu.Tp = c->Tp;
  tu.KP = c->KP;
  tu.J = J;
  tu.nsplit = c->nsplit_t;
  tu.omega = omega;
  UArgs u{};
  u.FB = c->FB.p;
  u.FW = c->FW.p;
  u.bnum = c->bnum.p;
  u.halt = c->halt;
  u.hsum = c->hsum.p;
  u.Wkf_new = c->Wkf_new.p;
  u.Wfk_new = c->Wfk_new.p;
  u.F = c->F;
  u.Fp = c->Fp;
  u.KP = c->KP;
  u.J = J;
  u.nchunk = c->nchunk_b;
  u.omega = omega;
  u.bden = nullptr;
  u.pmax = tail ? c->rpmax2.p : nullptr;
  tu.scal = tail ? c->rscal.p : nullptr;
  tu.tpart = c->rtpart2.p;
  tu.ntb = c->ntb;
  // the next iteration's FWHt / TW row sums formed here too (KP <= 64)
  // (not at KP = 128: its 64 KB TW tile leaves k_tw_update one block per CU,
  // 0.12 -> 0.38 ms at J = 4, more than the 0.23 ms it takes off the E-step)
  const bool prep = tail && c->ftail >= 2 && c->KP <= 64;
  tu.FW = c->FW.p;
  tu.FWHt = prep ? c->FWHt.p : nullptr;
  tu.hpart = c->hpart.p;
  for (int j = 0; j < kMaxJ; ++j) {
    tu.K[j] = j < J ? c->K[j] : 0;
    tu.soff[j] = j < J ? c->soff[j] : 0;
  }
  for (int j = 0; j < kMaxJ; ++j) {
    const bool in = j < J;
    tu.kb0[j] = u.kb0[j] = t.kb0[j] = 0;
    tu.kb1[j] = u.kb1[j] = t.kb1[j] = in ? c->K[j] : 0;
    t.tw_free[j] = tu.tw_free[j] = in ? c->tw_free[j] : 0;
    u.fb_free[j] = in ? c->fb_free[j] : 0;
  }
  switch (nkc) {
    case 1: launch_contract<1>(c, b, t, true); break;
    case 2: launch_contract<2>(c, b, t, true); break;
    case 4: launch_contract<4>(c, b, t, true); break;
    default: launch_contract<8>(c, b, t, true); break;
  }
  FASST_LAUNCH_CHECK();
  if (int st = check_tail_args(c, u, tu)) return st;
  prof_begin(c, KFBU);
  (c->KP > 64 ? k_fb_update<true> : k_fb_update<false>)<<<dim3(c->nft, J), 256,
                fw_lds(c, 16 * (c->KP + 1) + c->KP + 16 * (c->KP + 1)),
                c->stream>>>(u);
  prof_end(c, KFBU);
  FASST_LAUNCH_CHECK();
  if (tail)
    if (int st = launch_tail_side(c)) return st;
  if (any_fw) {
    // FW update (:1578-1631) between the FB and TW updates; W_new = FB_new FW_old
    // from k_fb_update is the V_mid operand, then W_new is rebuilt with FW_new
    FWArgs w{};
    w.TW = c->TW.p;
    w.TWt = c->TWt.p;
    w.Wkf_old = c->Wkf.p;
    w.Wkf_mid = c->Wkf_new.p;
    w.hatW = c->hatW.p;
    w.FB = c->FB.p;
    w.gnum = c->bnum.p;
    w.gden = c->gden.p;
    w.pnum = c->pnum.p;
    w.pden = c->pden.p;
    w.FW = c->FW.p;
    w.F = c->F;
    w.T = c->T;
    w.Fp = c->Fp;
    w.Tp = c->Tp;
    w.KP = c->KP;
    w.J = J;
    w.ntt = c->ntt;
    w.tpc = c->tpc_b;
    w.nchunk = c->nchunk_b;
    w.fpc = fw_fpc(c);
    w.nfc = (c->F + w.fpc - 1) / w.fpc;
    w.omega = omega;
    w.halt = c->halt;
    for (int j = 0; j < kMaxJ; ++j) {
      w.K[j] = j < J ? c->K[j] : 0;
      w.fw_free[j] = j < J ? c->fw_free[j] : 0;
      w.kb0[j] = 0;
      w.kb1[j] = w.K[j];
    }
    prof_begin(c, KFWU);
    const dim3 gc(c->nft, J, c->nchunk_b);
    switch (nkc) {
      case 1: k_fw_contract<1><<<gc, 64, 0, c->stream>>>(w); break;
      case 2: k_fw_contract<2><<<gc, 64, 0, c->stream>>>(w); break;
      case 4: k_fw_contract<4><<<gc, 64, 0, c->stream>>>(w); break;
      default: k_fw_contract<8><<<gc, 64, 0, c->stream>>>(w); break;
    }
    launch_fw_reduce(c, w);
    k_fw_final<<<J, 256, 0, c->stream>>>(w);
    (c->KP > 64 ? k_w_from_fb<true> : k_w_from_fb<false>)<<<dim3(c->nft, J), 256, fw_lds(c, 16 * (c->KP + 1)),
                  c->stream>>>(c->FB.p, c->FW.p, c->Wkf_new.p, c->Wfk_new.p, J, c->Fp, c->KP,
                               c->halt);
    prof_end(c, KFWU);
    FASST_LAUNCH_CHECK();
  }
  switch (nkc) {
    case 1: launch_contract<1>(c, b, t, false); break;
    case 2: launch_contract<2>(c, b, t, false); break;
    case 4: launch_contract<4>(c, b, t, false); break;
    default: launch_contract<8>(c, b, t, false); break;
  }
  FASST_LAUNCH_CHECK();
  // (prep reads the renormalised FW: wait for k_renorm_rows, else the scales)
  if (tail) FASST_HIP(hipStreamWaitEvent(c->stream, prep ? c->ev_rows : c->ev_scales, 0));
  prof_begin(c, KTWU);
  k_tw_update<<<dim3(c->ntb, J), 256, prep ? (size_t)c->KP * 64 * sizeof(double) : 0, c->stream>>>(tu);
  prof_end(c, KTWU);
  FASST_LAUNCH_CHECK();
  return FASST_OK;
}

// rho_j = hat_W_j / max(V_j, eps) into the [J][Tp][Fp] plane the spectral
// update reads, from a caller's hat_W [J][F][T] (update_spectral_components
// called on its own); V_j from the current parameters (Wkf = FB.FW)
__global__ void k_rho_from_hatw(const double *__restrict__ hw, const double *__restrict__ Wkf,
                                const double *__restrict__ TW, double *__restrict__ rho, int F,
                                int T, int Fp, int Tp, int KP) {
  const int f = blockIdx.x * 64 + (threadIdx.x & 63), t = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int j = blockIdx.z;
  if (f >= F || t >= T) return;
  double v = 0.0;
  for (int k = 0; k < KP; ++k) v += Wkf[((size_t)j * KP + k) * Fp + f] * TW[((size_t)j * KP + k) * Tp + t];
  rho[((size_t)j * Tp + t) * Fp + f] = hw[((size_t)j * F + f) * T + t] / fmax(v, kEps);
}

// One GEM iteration, all launches asynchronous on c->stream.
static int gem_iteration(fasst_ctx *c, const double *psd_dev, double *ll_dev, double omega,
                         int iter) {
  const int J = c->J;
  if (!c->conv) {
    // a free 'conv' component next to other components: the reference's conv
    // solve (audioModel.py:856-857) passes the full hat_Rss[f].T against the
    // free components' right-hand side only, and np.linalg.solve raises
    for (int j = 0; j < J; ++j)
      if ((c->convm >> j & 1u) && c->spat_free[j]) {
        set_error("spatial component %d is 'conv' and free next to other components: the "
                  "reference's mixing solve (audioModel.py:856-857) raises for this structure",
                  j);
        return FASST_ERR_UNSUPPORTED;
      }
  }
  // (FW.TW)^T and the TW row sums depend only on the previous iteration's
  // parameters: forked onto the side stream beside the E-step (unless the
  // previous iteration's fused tail in the same batch formed them)
  const bool prep_ready = c->prep_ready;
  c->prep_ready = 0;
  int st = prep_ready ? FASST_OK : launch_spectral_prep(c, true);
  if (st) return st;
  const bool w_ready = c->w_ready;   // (the previous iteration's fused tail formed W)
  c->w_ready = 0;
  if (!w_ready && (st = launch_w_old(c))) return st;
  st = build_inst_A(c);
  if (st) return st;
  EArgs e{};
  e.cx00 = c->cx.p;
  e.cx11 = c->cx.p + (size_t)c->Tp * c->Fp;
  e.cxr = c->cx.p + 2 * (size_t)c->Tp * c->Fp;
  e.cxi = c->cx.p + 3 * (size_t)c->Tp * c->Fp;
  e.TW = c->TW.p;
  e.Wkf = c->Wkf.p;
  e.A = c->A.p;
  e.psd = psd_dev;
  e.hatW = c->hatW.p;
  e.halt = c->halt;
  e.part = c->epart.p;
  e.llpart = c->llpart.p;
  e.F = c->F;
  e.T = c->T;
  e.Fp = c->Fp;
  e.Tp = c->Tp;
  e.KP = c->KP;
  e.R = c->R;
  e.ntt = c->ntt;
  e.tpc = c->tpc_e;
  e.nft = c->nft;
  for (int j = 0; j <= kMaxJ; ++j) e.roff[j] = j <= J ? c->roff[j] : c->R;
  e.ybase = e.tbase = 0;
  if (J > 8 && c->KP <= 32) {   // the fused many-source E-step
    GArgs gg{};
    gg.J = J;
    const size_t lds = (size_t)(((J + 12) | 1) * 256 + J * c->KP * 16) * sizeof(double);   // (ceiling: set_lds_limits)
    prof_begin(c, KESTEP);
    if (c->KP == 16)
      k_egen_fused<4><<<dim3(c->nft, c->nchunk_e), kEgsThreads, lds, c->stream>>>(e, gg);
    else
      k_egen_fused<8><<<dim3(c->nft, c->nchunk_e), kEgsThreads, lds, c->stream>>>(e, gg);
    prof_end(c, KESTEP);
  } else if (J > 8) {   // the two-pass E-step (k_egen_point / k_egen_stats)
    GArgs gg{};
    gg.V = c->vgen.p;
    gg.NP = c->npgen.p;
    gg.lw = c->lgen.p;
    gg.J = J;
    prof_begin(c, KESTEP);
    switch (c->KP) {
      case 16: k_egen_point<4><<<dim3(c->ntt, c->nft), 64, 0, c->stream>>>(e, gg); break;
      case 32: k_egen_point<8><<<dim3(c->ntt, c->nft), 64, 0, c->stream>>>(e, gg); break;
      case 64: k_egen_point<16><<<dim3(c->ntt, c->nft), 64, 0, c->stream>>>(e, gg); break;
      default: k_egen_point<32><<<dim3(c->ntt, c->nft), 64, 0, c->stream>>>(e, gg); break;
    }
    const size_t lds = (size_t)((J + 12) | 1) * 256 * sizeof(double);   // (ceiling: set_lds_limits)
    k_egen_stats<<<dim3(c->nft, c->nchunk_e), kEgsThreads, lds, c->stream>>>(e, gg);
    prof_end(c, KESTEP);
  } else {
    launch_estep(c, e, c->nchunk_e);
  }
  FASST_LAUNCH_CHECK();
  if (!prep_ready) FASST_HIP(hipStreamWaitEvent(c->stream, c->ev_join, 0));  // hsum, FWHt below
  const bool ft = fast_tail(c);
  if (!ft) {   // (fused tail: summed by k_renorm_tail)
    prof_begin(c, KLL);
    k_loglik<<<1, 256, 0, c->stream>>>(c->llpart.p, c->nchunk_e * c->nft, ll_dev,
                                       1.0 / ((double)c->F * (double)c->T), c->halt);
    prof_end(c, KLL);
    FASST_LAUNCH_CHECK();
  }
  // mixing update (update_mix_matrix, :766-889).  (On the side stream beside
  // the TW contraction instead, after the FB update: k_mix stretched to 0.18
  // ms and took 23 us from the TW contraction and 14 us from the FB
  // contraction for the 30 us it left the critical path; profiles/r6_ab_mix_side.txt)
  if ((st = launch_mix(c, c->stream))) return st;
  if ((st = spectral_update(c, omega, ft))) return st;
  if (!ft) return launch_renorm(c, iter);
  FASST_HIP(hipStreamWaitEvent(c->stream, c->ev_rows, 0));
  RArgs r = renorm_args(c);
  r.ll_out = ll_dev;
  const bool prep = c->ftail >= 2 && c->KP <= 64;   // (spectral_update's k_tw_update formed FWHt)
  r.hpart = prep ? c->hpart.p : nullptr;
  r.hsum = c->hsum.p;
  r.J = J;
  prof_begin(c, KRTAIL);
  k_renorm_tail<<<1 + (prep ? (J * c->KP + 3) / 4 : 0), 256, 0, c->stream>>>(r, iter);
  prof_end(c, KRTAIL);
  FASST_LAUNCH_CHECK();
  std::swap(c->Wkf.p, c->Wkf_next.p);
  c->w_ready = 1;
  c->prep_ready = prep;
  return FASST_OK;
}

}  // namespace fasst

using namespace fasst;

// ============================================================================ C ABI
extern "C" {

const char *fasst_last_error(void) { return fasst::g_err.c_str(); }

int fasst_abi_version(void) { return FASST_ABI_VERSION; }

int fasst_device_count(int *n) {
  FASST_HIP(hipGetDeviceCount(n));
  return FASST_OK;
}

int fasst_create(int device, int F, int T, fasst_ctx **out) {
  if (!out || F < 1 || T < 1) {
    set_error("fasst_create: bad arguments F=%d T=%d", F, T);
    return FASST_ERR_SHAPE;
  }
  int ndev = 0;
  FASST_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("fasst_create: device %d not present (%d visible)", device, ndev);
    return FASST_ERR_DEVICE;
  }
  DeviceGuard g(device);
  fasst_ctx *c = new fasst_ctx();
  c->device = device;
  c->F = F;
  c->T = T;
  c->Fp = round_up(F, kTile);
  c->Tp = round_up(T, kTile);
  c->nft = c->Fp / kTile;
  c->ntt = c->Tp / kTile;
  if (const char *v = getenv("FASST_FAST_TAIL")) c->ftail = atoi(v);
  int st = FASST_OK;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_tail, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_scales, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_rows, hipEventDisableTiming) != hipSuccess) {
    set_error("hipStreamCreate / hipEventCreate failed");
    st = FASST_ERR_DEVICE;
  }
  if (!st) st = c->cx.alloc((size_t)4 * c->Tp * c->Fp);
  if (!st && hipHostMalloc((void **)&c->h_flags, kNFlags * sizeof(int)) != hipSuccess)
    st = FASST_ERR_OOM;
  if (!st && hipHostMalloc((void **)&c->h_ll, 64 * sizeof(double)) != hipSuccess) st = FASST_ERR_OOM;
  if (st) {
    fasst_destroy(c);
    return st;
  }
  *out = c;
  return FASST_OK;
}

int fasst_configure_types(fasst_ctx *c, int J, const int *rank, const int *K,
                          const int *mix_conv) {
  if (!c || !rank || !K || !mix_conv) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  return configure_model(c, J, rank, K, mix_conv);
}

int fasst_configure(fasst_ctx *c, int J, const int *rank, const int *K, int mix_conv) {
  if (!c || !rank || !K) return FASST_ERR_SHAPE;
  if (J < 1 || J > kMaxJ) return configure_model(c, J, rank, K, nullptr);
  int types[kMaxJ];
  for (int j = 0; j < J; ++j) types[j] = mix_conv ? 1 : 0;
  DeviceGuard g(c->device);
  return configure_model(c, J, rank, K, types);
}

int fasst_destroy(fasst_ctx *c) {
  if (!c) return FASST_OK;
  {
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    if (c->h_ll) (void)hipHostFree(c->h_ll);
    c->cx.release();
    c->X.release();
    c->FB.release();
    c->FW.release();
    c->TW.release();
    c->Wkf.release();
    c->Wkf_new.release();
    c->Wfk_new.release();
    c->FWHt.release();
    c->hatW.release();
    c->A.release();
    c->Pinst.release();
    c->epart.release();
    c->llpart.release();
    c->bnum.release();
    c->tnum.release();
    c->tden.release();
    c->psd.release();
    c->ll.release();
    c->rss.release();
    c->rxs.release();
    c->flags.release();
    c->hsum.release();
    c->rscal.release();
    c->rpmax.release();
    c->rpe.release();
    c->rtpart.release();
    c->rpmax2.release();
    c->rtpart2.release();
    c->hpart.release();
    c->vgen.release();
    c->npgen.release();
    c->lgen.release();
    c->Wkf_next.release();
    c->mplanes.release();
    c->bden.release();
    for (int i = 0; i < fasst_ctx::kNK; ++i) {
      for (int q = 0; q < fasst_ctx::kProfRing; ++q) {
        if (c->ev0[i][q]) (void)hipEventDestroy(c->ev0[i][q]);
        if (c->ev1[i][q]) (void)hipEventDestroy(c->ev1[i][q]);
      }
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_tail) (void)hipEventDestroy(c->ev_tail);
    if (c->ev_scales) (void)hipEventDestroy(c->ev_scales);
    if (c->ev_rows) (void)hipEventDestroy(c->ev_rows);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;
  return FASST_OK;
}

static int need_model(fasst_ctx *c, int j) {
  if (!c || !c->configured) {
    set_error("context not configured");
    return FASST_ERR_SHAPE;
  }
  if (j < 0 || j >= c->J) {
    set_error("component %d out of range (J=%d)", j, c->J);
    return FASST_ERR_SHAPE;
  }
  return FASST_OK;
}

int fasst_set_spatial(fasst_ctx *c, int j, const double *params, int free_) {
  int st = need_model(c, j);
  if (st) return st;
  DeviceGuard g(c->device);
  c->spat_free[j] = free_ ? 1 : 0;
  const int r0 = c->roff[j], nr = c->rank[j];
  const double2 *p = reinterpret_cast<const double2 *>(params);
  if (c->convm >> j & 1u) {
    // params [r][C][F] -> A[r][c][f] (row pitch Fp)
    FASST_HIP(hipMemcpy2DAsync(c->A.p + (size_t)2 * r0 * c->Fp, c->Fp * sizeof(double2), p,
                               c->F * sizeof(double2), c->F * sizeof(double2), (size_t)nr * 2,
                               hipMemcpyHostToDevice, c->stream));
  } else {
    // params [C][r] -> Pinst[r][c]
    std::vector<double2> tmp((size_t)nr * 2);
    for (int r = 0; r < nr; ++r)
      for (int ch = 0; ch < 2; ++ch) tmp[(size_t)r * 2 + ch] = p[(size_t)ch * nr + r];
    FASST_HIP(hipMemcpyAsync(c->Pinst.p + 2 * r0, tmp.data(), tmp.size() * sizeof(double2),
                             hipMemcpyHostToDevice, c->stream));
    FASST_HIP(hipStreamSynchronize(c->stream));
  }
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_get_spatial(fasst_ctx *c, int j, double *params) {
  int st = need_model(c, j);
  if (st) return st;
  DeviceGuard g(c->device);
  const int r0 = c->roff[j], nr = c->rank[j];
  double2 *p = reinterpret_cast<double2 *>(params);
  if (c->convm >> j & 1u) {
    FASST_HIP(hipMemcpy2DAsync(p, c->F * sizeof(double2), c->A.p + (size_t)2 * r0 * c->Fp,
                               c->Fp * sizeof(double2), c->F * sizeof(double2), (size_t)nr * 2,
                               hipMemcpyDeviceToHost, c->stream));
    FASST_HIP(hipStreamSynchronize(c->stream));
  } else {
    std::vector<double2> tmp((size_t)nr * 2);
    FASST_HIP(hipMemcpyAsync(tmp.data(), c->Pinst.p + 2 * r0, tmp.size() * sizeof(double2),
                             hipMemcpyDeviceToHost, c->stream));
    FASST_HIP(hipStreamSynchronize(c->stream));
    for (int r = 0; r < nr; ++r)
      for (int ch = 0; ch < 2; ++ch) p[(size_t)ch * nr + r] = tmp[(size_t)r * 2 + ch];
  }
  return FASST_OK;
}

int fasst_set_fw_prior(fasst_ctx *c, int j, int fw_free) {
  int st = need_model(c, j);
  if (st) return st;

  c->fw_free[j] = fw_free ? 1 : 0;
  if (c->nblk[j] == 1) c->bfw[j][0] = c->fw_free[j];
  return FASST_OK;
}

int fasst_set_blocks(fasst_ctx *c, int j, int nblk, const int *kb, const int *fb_free,
                     const int *fw_free, const int *tw_free) {
  int st = need_model(c, j);
  if (st) return st;
  if (nblk < 1 || nblk > kMaxBlk || !kb || !fb_free || !fw_free || !tw_free) {
    set_error("source %d: %d spectral components (1..%d on the HIP path)", j, nblk, kMaxBlk);
    return nblk > kMaxBlk ? FASST_ERR_UNSUPPORTED : FASST_ERR_SHAPE;
  }
  if (kb[0] != 0 || kb[nblk] != c->K[j]) {
    set_error("source %d: component blocks must cover its %d columns", j, c->K[j]);
    return FASST_ERR_SHAPE;
  }
  for (int b = 0; b < nblk; ++b)
    if (kb[b + 1] <= kb[b]) {
      set_error("source %d: empty or unordered component block %d", j, b);
      return FASST_ERR_SHAPE;
    }
  int nslot = 0, maxblk = 0;
  for (int i = 0; i < c->J; ++i) {
    const int n = i == j ? nblk : c->nblk[i];
    nslot += n;
    maxblk = std::max(maxblk, n);
  }
  if (nslot > kMaxSlot) {
    set_error("%d spectral components in all (max %d on the HIP path)", nslot, kMaxSlot);
    return FASST_ERR_UNSUPPORTED;
  }
  DeviceGuard g(c->device);
  if (maxblk > 1) {
    const size_t plane = (size_t)c->J * c->Tp * c->Fp;
    if (c->mplanes.n < 5 * plane && (st = c->mplanes.alloc(5 * plane))) return st;
    const size_t nb = (size_t)c->nchunk_b * c->J * c->Fp * c->KP;
    if (c->bden.n < nb && (st = c->bden.alloc(nb))) return st;
  }
  bool same = c->nblk[j] == nblk;
  for (int b = 0; same && b <= nblk; ++b) same = c->kb[j][b] == kb[b];
  c->nblk[j] = nblk;
  for (int b = 0; b <= nblk; ++b) c->kb[j][b] = kb[b];
  bool fbf = false, twf = false, fwf = false;
  for (int b = 0; b < nblk; ++b) {
    c->bfb[j][b] = fb_free[b] ? 1 : 0;
    c->bfw[j][b] = fw_free[b] ? 1 : 0;
    c->btw[j][b] = tw_free[b] ? 1 : 0;
    fbf |= c->bfb[j][b] != 0;
    fwf |= c->bfw[j][b] != 0;
    twf |= c->btw[j][b] != 0;
  }
  c->fb_free[j] = fbf;
  c->fw_free[j] = fwf;
  c->tw_free[j] = twf;
  c->soff[0] = 0;
  for (int i = 0; i < c->J; ++i) c->soff[i + 1] = c->soff[i] + c->nblk[i];
  c->nslot = nslot;
  c->maxblk = maxblk;
  if (!same)   // the blocks moved: their time blobs go (an unchanged layout,
               // e.g. the per-iteration re-upload, keeps them and their buffers)
    for (int b = 0; b < kMaxBlk; ++b) {
      c->tb[j][b].release();
      c->tbl[j][b] = c->btb[j][b] = 0;
    }
  update_multi(c);
  return FASST_OK;
}

int fasst_set_corr(fasst_ctx *c, double lambda, int nseq, const int *seq_j, const int *seq_b) {
  int st = need_model(c, 0);
  if (st) return st;
  if (!(lambda >= 0.0) || (lambda > 0.0 && (nseq < 1 || nseq > kMaxSlot || !seq_j || !seq_b))) {
    set_error("fasst_set_corr: lambda %g with %d components", lambda, nseq);
    return FASST_ERR_SHAPE;
  }
  if (lambda > 0.0) {
    int seen[kMaxJ][kMaxBlk] = {{0}};
    for (int q = 0; q < nseq; ++q) {
      const int j = seq_j[q], b = seq_b[q];
      if (j < 0 || j >= c->J || b < 0 || b >= c->nblk[j] || seen[j][b]++) {
        set_error("fasst_set_corr: bad component (%d, %d) at position %d", j, b, q);
        return FASST_ERR_SHAPE;
      }
      c->seq_j[q] = j;
      c->seq_b[q] = b;
    }
    if (nseq != c->nslot) {
      set_error("fasst_set_corr: %d components given, the model has %d", nseq, c->nslot);
      return FASST_ERR_SHAPE;
    }
    DeviceGuard g(c->device);
    const size_t plane = (size_t)c->J * c->Tp * c->Fp;
    if (c->mplanes.n < 5 * plane && (st = c->mplanes.alloc(5 * plane))) return st;
    const size_t nb = (size_t)c->nchunk_b * c->J * c->Fp * c->KP;
    if (c->bden.n < nb && (st = c->bden.alloc(nb))) return st;
  }
  c->lambda = lambda;
  c->nseq = lambda > 0.0 ? nseq : 0;
  update_multi(c);
  return FASST_OK;
}

int fasst_set_tb(fasst_ctx *c, int j, int b, int L, const double *TW, const double *TB,
                 int tb_free) {
  int st = need_model(c, j);
  if (st) return st;
  if (b < 0 || b >= c->nblk[j] || L < 0 || L > kMaxTB || (L > 0 && (!TW || !TB))) {
    set_error("fasst_set_tb: source %d component %d with %d time blobs (1..%d)", j, b, L, kMaxTB);
    return L > kMaxTB ? FASST_ERR_UNSUPPORTED : FASST_ERR_SHAPE;
  }
  DeviceGuard g(c->device);
  if (L == 0) {
    c->tb[j][b].release();
    c->tbl[j][b] = c->btb[j][b] = 0;
    update_multi(c);
    return FASST_OK;
  }
  const int kbw = c->kb[j][b + 1] - c->kb[j][b];
  const TBLayout o = tb_layout(kbw, L, c->Tp);
  const size_t plane = (size_t)c->J * c->Tp * c->Fp;
  if (c->mplanes.n < 6 * plane && (st = c->mplanes.alloc(6 * plane))) return st;
  const size_t nb = (size_t)c->nchunk_b * c->J * c->Fp * c->KP;
  if (c->bden.n < nb && (st = c->bden.alloc(nb))) return st;
  // a buffer large enough is reused (no hipMalloc / device-wide sync on the
  // per-iteration re-upload); either way it is zero-filled: TB's padding
  // frames stay 0
  if (c->tb[j][b].n < o.n) {
    if ((st = c->tb[j][b].alloc(o.n))) return st;
  } else {
    FASST_HIP(hipMemsetAsync(c->tb[j][b].p, 0, o.n * sizeof(double), c->stream));
  }
  FASST_HIP(hipMemcpyAsync(c->tb[j][b].p + o.tws, TW, (size_t)kbw * L * sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemcpy2DAsync(c->tb[j][b].p + o.tb, c->Tp * sizeof(double), TB,
                             c->T * sizeof(double), c->T * sizeof(double), L,
                             hipMemcpyHostToDevice, c->stream));
  c->tbl[j][b] = L;
  c->btb[j][b] = tb_free ? 1 : 0;
  update_multi(c);
  c->halt = nullptr;
  TBArgs a = tb_args(c, b, j, 0, 1.0);   // H = TW TB into the block's rows
  if ((st = launch_tb_h(c, a))) return st;
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_get_tb(fasst_ctx *c, int j, int b, double *TW, double *TB) {
  int st = need_model(c, j);
  if (st) return st;
  if (b < 0 || b >= c->nblk[j] || c->tbl[j][b] == 0) {
    set_error("fasst_get_tb: source %d component %d has no time blobs", j, b);
    return FASST_ERR_SHAPE;
  }
  DeviceGuard g(c->device);
  const int kbw = c->kb[j][b + 1] - c->kb[j][b], L = c->tbl[j][b];
  const TBLayout o = tb_layout(kbw, L, c->Tp);
  if (TW)
    FASST_HIP(hipMemcpyAsync(TW, c->tb[j][b].p + o.tws, (size_t)kbw * L * sizeof(double),
                             hipMemcpyDeviceToHost, c->stream));
  if (TB)
    FASST_HIP(hipMemcpy2DAsync(TB, c->T * sizeof(double), c->tb[j][b].p + o.tb,
                               c->Tp * sizeof(double), c->T * sizeof(double), L,
                               hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_set_spectral(fasst_ctx *c, int j, const double *FB, const double *FW, const double *TW,
                       int fb_free, int tw_free) {
  int st = need_model(c, j);
  if (st) return st;
  DeviceGuard g(c->device);
  const int K = c->K[j], KP = c->KP;
  c->fb_free[j] = fb_free ? 1 : 0;
  c->tw_free[j] = tw_free ? 1 : 0;
  if (c->nblk[j] == 1) {
    c->bfb[j][0] = c->fb_free[j];
    c->btw[j][0] = c->tw_free[j];
  }
  FASST_HIP(hipMemsetAsync(c->FW.p + (size_t)j * KP * KP, 0, (size_t)KP * KP * sizeof(double),
                           c->stream));
  FASST_HIP(hipMemcpy2DAsync(c->FB.p + (size_t)j * c->Fp * KP, KP * sizeof(double), FB,
                             K * sizeof(double), K * sizeof(double), c->F, hipMemcpyHostToDevice,
                             c->stream));
  FASST_HIP(hipMemcpy2DAsync(c->FW.p + (size_t)j * KP * KP, KP * sizeof(double), FW,
                             K * sizeof(double), K * sizeof(double), K, hipMemcpyHostToDevice,
                             c->stream));
  FASST_HIP(hipMemcpy2DAsync(c->TW.p + (size_t)j * KP * c->Tp, c->Tp * sizeof(double), TW,
                             c->T * sizeof(double), c->T * sizeof(double), K,
                             hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_get_spectral(fasst_ctx *c, int j, double *FB, double *FW, double *TW) {
  int st = need_model(c, j);
  if (st) return st;
  DeviceGuard g(c->device);
  const int K = c->K[j], KP = c->KP;
  if (FB)
    FASST_HIP(hipMemcpy2DAsync(FB, K * sizeof(double), c->FB.p + (size_t)j * c->Fp * KP,
                               KP * sizeof(double), K * sizeof(double), c->F,
                               hipMemcpyDeviceToHost, c->stream));
  if (FW)
    FASST_HIP(hipMemcpy2DAsync(FW, K * sizeof(double), c->FW.p + (size_t)j * KP * KP,
                               KP * sizeof(double), K * sizeof(double), K, hipMemcpyDeviceToHost,
                               c->stream));
  if (TW)
    FASST_HIP(hipMemcpy2DAsync(TW, c->T * sizeof(double), c->TW.p + (size_t)j * KP * c->Tp,
                               c->Tp * sizeof(double), c->T * sizeof(double), K,
                               hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_spectral_update(fasst_ctx *c, const double *hat_W, double omega) {
  int st = need_model(c, 0);
  if (st) return st;
  if (!hat_W) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  const size_t n = (size_t)c->J * c->F * c->T;
  DBuf<double> dh;
  if ((st = dh.alloc_uninit(n))) return st;
  FASST_HIP(hipMemcpyAsync(dh.p, hat_W, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemsetAsync(c->flags.p, 0, kNFlags * sizeof(int), c->stream));
  c->halt = nullptr;
  if ((st = launch_spectral_prep(c, false)) || (st = launch_w_old(c))) return st;
  FASST_HIP(hipMemsetAsync(c->hatW.p, 0, (size_t)c->J * c->Tp * c->Fp * sizeof(double), c->stream));
  k_rho_from_hatw<<<dim3((c->F + 63) / 64, (c->T + 3) / 4, c->J), 256, 0, c->stream>>>(
      dh.p, c->Wkf.p, c->TW.p, c->hatW.p, c->F, c->T, c->Fp, c->Tp, c->KP);
  FASST_LAUNCH_CHECK();
  if ((st = spectral_update(c, omega))) return st;
  FASST_HIP(hipStreamSynchronize(c->stream));
  return FASST_OK;
}

int fasst_renormalize(fasst_ctx *c, int *restart_mask) {
  int st = need_model(c, 0);
  if (st) return st;
  DeviceGuard g(c->device);
  FASST_HIP(hipMemsetAsync(c->flags.p, 0, kNFlags * sizeof(int), c->stream));
  c->halt = nullptr;
  st = launch_renorm(c, 0);
  if (st) return st;
  FASST_HIP(hipMemcpyAsync(c->h_flags, c->flags.p, kNFlags * sizeof(int),
                           hipMemcpyDeviceToHost, c->stream));
  FASST_HIP(hipStreamSynchronize(c->stream));
  int mask = 0;
  for (int sl = 0; sl < c->nslot; ++sl)
    if (c->h_flags[1 + sl]) mask |= 1 << sl;
  if (restart_mask) *restart_mask = mask;
  return FASST_OK;
}

int fasst_run(fasst_ctx *c, int n_iter, const double *psd, double omega, double *logliks,
              int *restart_mask, int *iters_done) {
  int st = need_model(c, 0);
  if (st) return st;
  if (n_iter < 0 || (n_iter > 0 && (!psd || !logliks))) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (iters_done) *iters_done = 0;
  if (restart_mask) *restart_mask = 0;
  if (n_iter == 0) return FASST_OK;
  if (c->psd_cap < n_iter) {
    if ((st = c->psd.alloc((size_t)n_iter * c->Fp))) return st;
    c->psd_cap = n_iter;
  }
  if (c->ll_cap < n_iter) {
    if ((st = c->ll.alloc(n_iter))) return st;
    c->ll_cap = n_iter;
  }
  FASST_HIP(hipMemsetAsync(c->psd.p, 0, (size_t)n_iter * c->Fp * sizeof(double), c->stream));
  FASST_HIP(hipMemcpy2DAsync(c->psd.p, c->Fp * sizeof(double), psd, c->F * sizeof(double),
                             c->F * sizeof(double), n_iter, hipMemcpyHostToDevice, c->stream));
  FASST_HIP(hipMemsetAsync(c->flags.p, 0, kNFlags * sizeof(int), c->stream));
  // Without profiling the whole batch is enqueued at once: a flag raised in
  // iteration i halts every later kernel on the device (HALT_GUARD), and the
  // host reads the flags once at the end.  Profiling keeps one sync per
  // iteration so the per-kernel events can be folded.
  c->halt = c->flags.p + kFlagHalt;
  c->w_ready = c->prep_ready = 0;
  const int sync_every = c->prof ? fasst_ctx::kProfRing : n_iter;
  int done = 0;
  for (int it = 0; it < n_iter; ++it) {
    c->pslot = it % fasst_ctx::kProfRing;
    st = gem_iteration(c, c->psd.p + (size_t)it * c->Fp, c->ll.p + it, omega, it);
    if (st) {
      c->halt = nullptr;
      return st;
    }
    if ((it + 1) % sync_every && it + 1 < n_iter) continue;
    FASST_HIP(hipMemcpyAsync(c->h_flags, c->flags.p, kNFlags * sizeof(int),
                             hipMemcpyDeviceToHost, c->stream));
    FASST_HIP(hipStreamSynchronize(c->stream));
    prof_collect(c);
    done = it + 1;
    if (c->h_flags[kFlagHalt] || c->h_flags[0]) break;
  }
  c->halt = nullptr;
  // a halted batch skipped its later iterations' kernels while the host still
  // swapped the fused tail's W buffers: rebuild W = FB.FW from the parameters
  if (c->w_ready && (c->h_flags[kFlagHalt] || c->h_flags[0])) {
    if ((st = launch_w_old(c))) return st;
    FASST_HIP(hipStreamSynchronize(c->stream));
  }
  c->w_ready = c->prep_ready = 0;
  if (c->h_flags[0]) {
    set_error("Singular Matrix");
    return FASST_ERR_SINGULAR;
  }
  int mask = 0;
  for (int sl = 0; sl < c->nslot; ++sl)
    if (c->h_flags[1 + sl]) mask |= 1 << sl;
  if (mask) done = c->h_flags[kFlagIter] + 1;
  if (iters_done) *iters_done = done;
  FASST_HIP(hipMemcpy(logliks, c->ll.p, (size_t)done * sizeof(double), hipMemcpyDeviceToHost));
  if (mask) {
    if (restart_mask) *restart_mask = mask;
    return FASST_TW_RESTART;
  }
  return FASST_OK;
}

}  // extern "C"

extern "C" {

int fasst_set_profiling(fasst_ctx *c, int on) {
  if (!c) return FASST_ERR_SHAPE;
  DeviceGuard g(c->device);
  if (on && !c->ev0[0][0])
    for (int i = 0; i < fasst_ctx::kNK; ++i)
      for (int q = 0; q < fasst_ctx::kProfRing; ++q) {
        FASST_HIP(hipEventCreate(&c->ev0[i][q]));
        FASST_HIP(hipEventCreate(&c->ev1[i][q]));
      }
  c->prof = on ? 1 : 0;
  c->pslot = 0;
  for (int i = 0; i < fasst_ctx::kNK; ++i) {
    c->prof_ms[i] = 0.0;
    c->prof_cnt[i] = 0;
    for (int q = 0; q < fasst_ctx::kProfRing; ++q) c->used[i][q] = 0;
  }
  return FASST_OK;
}

int fasst_kernel_times(fasst_ctx *c, double *avg_ms, long *counts, int nk) {
  if (!c || !avg_ms) return FASST_ERR_SHAPE;
  for (int i = 0; i < nk && i < fasst_ctx::kNK; ++i) {
    avg_ms[i] = c->prof_cnt[i] ? c->prof_ms[i] / (double)c->prof_cnt[i] : 0.0;
    if (counts) counts[i] = c->prof_cnt[i];
  }
  return fasst_ctx::kNK;
}

const char *fasst_kernel_name(int i) {
  return (i >= 0 && i < fasst_ctx::kNK) ? kKernelNames[i] : "";
}

}  // extern "C"
