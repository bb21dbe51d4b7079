// Shared definitions of the MI355X FASST engine (gfx950, HIP).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdarg>
#include <string>
#include <vector>

#include "../../include/fasst_hip.h"

namespace fasst {

// Kernel attribute: keep adjacent LDS reads / writes as separate ds_read_b64 /
// ds_write_b64 instead of ds_read2_b64 / ds_read2st64_b64 pairs, which take
// 8 LDS cycles for the 2 + 2 of two single reads (MI355X_MICROARCH.md §LDS).
// A device-code target feature: the host pass of the same source does not
// know it, so it is spelled only for the device pass.
#if defined(__HIP_DEVICE_COMPILE__)
#define FASST_NO_LDS_PAIRING __attribute__((target("no-load-store-opt")))
#else
#define FASST_NO_LDS_PAIRING
#endif

constexpr double kEps = 1e-10;  // audioModel.py:61, tools/signalTools.py:11
constexpr int kMaxJ = 16;       // sources (spatial components; > 8: the two-pass E-step)
constexpr int kMaxR = 32;       // total spatial rank (the GEM path; the step calls: kStepMaxR)
constexpr int kStepMaxR = 16;   // total spatial rank of fasst_suff_stat / fasst_mix_solve
constexpr int kMaxKP = 128;     // padded NMF components (K > 64: one spectral
                                // component per source, fixed FW, no lambdaCorr / TB)
constexpr int kFwFpc = 64;      // bins per block of the FW update's f-contraction
constexpr int kTile = 16;       // MFMA f64 16x16x4 tile edge
// several spectral components per spatial component: source j's NMF columns
// are cut into <= kMaxBlk blocks (one per spectral component); the blocks of
// all sources (the "slots") carry the TW restart flags
constexpr int kMaxBlk = 8, kMaxSlot = 16;
constexpr int kMaxTB = 64;  // time blobs per spectral component
constexpr int kFlagHalt = 1 + kMaxSlot, kFlagIter = 2 + kMaxSlot, kNFlags = 3 + kMaxSlot;
#ifndef FASST_FPW
#define FASST_FPW 2
#endif
#ifndef FASST_TPW
#define FASST_TPW 2
#endif
constexpr int kFPW = FASST_FPW;  // bin tiles per wave, FB contraction
constexpr int kTPW = FASST_TPW;  // frame tiles per wave, TW contraction

typedef double d4 __attribute__((ext_vector_type(4)));

void set_error(const char *fmt, ...);

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

#define FASST_HIP(call)                                                      \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::fasst::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,          \
                         hipGetErrorString(e_));                             \
      return e_ == hipErrorOutOfMemory ? FASST_ERR_OOM : FASST_ERR_DEVICE;   \
    }                                                                        \
  } while (0)

#define FASST_LAUNCH_CHECK()                                                 \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ::fasst::set_error("%s:%d kernel launch: %s", __FILE__, __LINE__,      \
                         hipGetErrorString(e_));                             \
      return FASST_ERR_DEVICE;                                               \
    }                                                                        \
  } while (0)

// Scoped device selection (restores the caller's device).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Device buffer owned by a context; freed in the destructor.
template <typename T>
struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  int alloc(size_t count) {
    release();
    if (count == 0) return FASST_OK;
    FASST_HIP(hipMalloc(&p, count * sizeof(T)));
    n = count;
    // zero-fill and wait: the context stream is non-blocking, so a pending
    // null-stream memset could otherwise land after later stream work
    FASST_HIP(hipMemset(p, 0, count * sizeof(T)));
    FASST_HIP(hipDeviceSynchronize());
    return FASST_OK;
  }
  // scratch that every reader writes before it reads: no zero-fill, no sync
  int alloc_uninit(size_t count) {
    release();
    if (count == 0) return FASST_OK;
    FASST_HIP(hipMalloc(&p, count * sizeof(T)));
    n = count;
    return FASST_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DBuf() { release(); }
};

}  // namespace fasst
