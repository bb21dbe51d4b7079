// Device-resident state of one FASST model (one GPU, one stream).
//
// HBM layout (all float64; Fp = F rounded up to 16, Tp = T rounded up to 16,
// KP = max K rounded up to 16; padding is zero and masked where it matters):
//   cx      4 planes [Tp][Fp]   Cx00, Cx11, Re Cx01, Im Cx01  (frame-major,
//                               bins contiguous: the E-step's V^T tiles read
//                               16 consecutive bins per 128-B segment)
//   X       [2][Tp][Fp] double2 resident channel STFTs (optional)
//   FB      [J][Fp][KP]         frequency bases           (canonical)
//   FW      [J][KP][KP]         frequency weights         (canonical)
//   TW      [J][KP][Tp]         time weights              (canonical)
//   Pinst   [R][2] double2      'inst' mixing params       (canonical)
//   A       [R][2][Fp] double2  per-bin mixing matrix ('conv' canonical)
//   Wkf     [J][KP][Fp]         W = FB.FW   (MFMA operand layout)
//   Wkf_new / Wfk_new           W after the FB update, both operand layouts
//   FWHt    [J][Tp][KP]         (FW.TW)^T  (B operand of the FB contraction)
//   hatW    [J][Tp][Fp]         posterior source power hat_W
#pragma once
#include "fasst_common.h"

struct fasst_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // side stream: the small per-iteration prep kernels ((FW.TW)^T, TW row sums)
  // run there, forked at the iteration start and joined before their first
  // consumer, so they overlap the E-step instead of serialising before it
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // the renormalisation's scales and FB / FW / mixing rescale run on the side
  // stream beside the TW contraction (gem_iteration's fused tail)
  hipEvent_t ev_tail = nullptr, ev_scales = nullptr, ev_rows = nullptr;
  // observation
  int F = 0, T = 0, Fp = 0, Tp = 0, nft = 0, ntt = 0;
  fasst::DBuf<double> cx;        // 4*Tp*Fp
  fasst::DBuf<double> vgen, npgen, lgen;   // J > 8: the two-pass E-step's scratch planes
  bool cx_ready = false;          // an observation was written (set_cx / set_stft / set_audio)
  fasst::DBuf<double2> X;        // 2*Tp*Fp (resident STFT, optional)
  bool have_X = false;
  // model
  int J = 0, R = 0, KP = 0, conv = 0, configured = 0;
  unsigned convm = 0;  // bit j: source j is 'conv' (conv == every source 'conv')
  int rank[fasst::kMaxJ] = {0}, roff[fasst::kMaxJ + 1] = {0}, K[fasst::kMaxJ] = {0};
  int spat_free[fasst::kMaxJ] = {0}, fb_free[fasst::kMaxJ] = {0}, tw_free[fasst::kMaxJ] = {0};
  int fw_free[fasst::kMaxJ] = {0};
  // spectral components of source j: column blocks [kb[j][b], kb[j][b + 1]) of
  // its FB / FW (block diagonal) / TW, in the reference's spec_comps key
  // order; slot soff[j] + b carries block b's TW restart flag.  multi != 0
  // when some source has several blocks (the sequential multi-block update)
  int nblk[fasst::kMaxJ] = {0}, kb[fasst::kMaxJ][fasst::kMaxBlk + 1] = {{0}};
  int soff[fasst::kMaxJ + 1] = {0}, nslot = 0, maxblk = 0, multi = 0;
  int bfb[fasst::kMaxJ][fasst::kMaxBlk] = {{0}}, btw[fasst::kMaxJ][fasst::kMaxBlk] = {{0}};
  int bfw[fasst::kMaxJ][fasst::kMaxBlk] = {{0}};
  // time blobs (fasst_set_tb): block b of source j with tbl[j][b] = L > 0 has
  // H = TW.TB; its factor TW (block rows x L) and TB (L x Tp) live in
  // tb[j][b] (layout tb_layout in fasst_em.hip) and the block's rows of TW
  // hold H; btb[j][b]: TB free.  Any time blob routes through the multi path
  fasst::DBuf<double> tb[fasst::kMaxJ][fasst::kMaxBlk];
  int tbl[fasst::kMaxJ][fasst::kMaxBlk] = {{0}}, btb[fasst::kMaxJ][fasst::kMaxBlk] = {{0}};
  int anytb = 0;
  fasst::DBuf<double> FB, FW, TW, Wkf, Wkf_new, Wfk_new, FWHt, hatW;
  // multi-block update: ratio planes [6][J][Tp][Fp] (rnum, rden, rho_c, corrPen,
  // powers, and with time blobs max(V_c, eps)), FB den
  fasst::DBuf<double> mplanes, bden;
  // lambdaCorr > 0 (fasst_set_corr): the components go one at a time in the
  // reference's key order (seq_j[q], seq_b[q]) through the multi-block path
  double lambda = 0.0;
  int nseq = 0, seq_j[fasst::kMaxSlot] = {0}, seq_b[fasst::kMaxSlot] = {0};
  // separation sources (fasst_set_sources; nsrc == 0: one per spatial
  // component): source n sums the terms [toff[n], toff[n + 1]), term i = the
  // columns tmask[i] (bit k = column k) of spatial component tj[i]
  int nsrc = 0, toff[fasst::kMaxSlot + 1] = {0}, tj[fasst::kMaxSlot] = {0};
  unsigned long long tmask[fasst::kMaxSlot][2] = {{0}};   // 128-bit column sets
  fasst::DBuf<double2> A, Pinst;
  // work space
  int nchunk_e = 1, tpc_e = 1, nchunk_b = 1, tpc_b = 1, nacc = 0;
  int nsplit_t = 1, fpc_t = 1;  // TW contraction bin chunks
  fasst::DBuf<double> epart, llpart, bnum, tnum, tden, psd, ll, hsum, rscal, rpmax, rpe, rtpart;
  fasst::DBuf<double> gden, TWt, pnum, pden;  // FW update (free FW)
  int nchunk_r = 1;
  // fused tail: FB column maxima / mixing energy per k_fb_update block, TW
  // restart sums per k_tw_update block
  fasst::DBuf<double> rpmax2, rpe2, rtpart2;
  int ntb = 1;
  // W = FB.FW of the renormalised parameters, formed on the side stream by
  // the fused tail and swapped into Wkf at the iteration's end; w_ready: the
  // next iteration of the same fasst_run batch skips launch_w_old
  fasst::DBuf<double> Wkf_next;
  int w_ready = 0;
  // FWHt and hsum of the final TW formed by the fused k_tw_update / tail
  // (hpart: its per-block row sums): the next iteration of the batch skips
  // launch_spectral_prep (no side-stream work beside its E-step)
  fasst::DBuf<double> hpart;
  int prep_ready = 0;
  // the fused tail is taken for the structures it covers (fast_tail in
  // fasst_em.hip) unless FASST_FAST_TAIL=0 was set when this context was
  // created; 2 (default): it also forms the next iteration's FWHt / hsum
  int ftail = 2;
  fasst::DBuf<double2> rss, rxs;
  fasst::DBuf<int> flags;        // [0] singular, [1..nslot] TW restart, [kFlagHalt] halt,
                                 // [kFlagIter] iteration that raised a restart
  int *h_flags = nullptr;        // pinned host mirror
  const int *halt = nullptr;     // flags + kFlagHalt while fasst_run enqueues a batch
  double *h_ll = nullptr;        // pinned host mirror (one value)
  int psd_cap = 0, ll_cap = 0;
  // per-kernel HIP-event timing (fasst_set_profiling / fasst_kernel_times)
  // (events on the stream each kernel runs on, the side-stream fork kept, a
  // ring of kProfRing iterations between host syncs: the timed schedule)
  static constexpr int kNK = 15, kProfRing = 32;
  int prof = 0, pslot = 0;
  hipEvent_t ev0[kNK][kProfRing] = {}, ev1[kNK][kProfRing] = {};
  int used[kNK][kProfRing] = {{0}};
  double prof_ms[kNK] = {0};
  long prof_cnt[kNK] = {0};
};

namespace fasst {
int configure_model(fasst_ctx *c, int J, const int *rank, const int *K, const int *convj);
int build_inst_A(fasst_ctx *c);
int launch_w_old(fasst_ctx *c);  // Wkf = FB.FW
}  // namespace fasst
