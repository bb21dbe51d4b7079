/*
 * fasst_viterbi.h -- C ABI of the Viterbi melody tracker (libfasst_hip.so).
 *
 * Replaces the reference's only native component, the Cython tracker
 *   viterbiTracking(int numberOfStates, int numberOfFrames, logDensity,
 *                   logPriorDensities, logTransitionMatrix)
 *   (SeparateLeadStereo/tracking/_tracking.pyx:11-93; called by
 *   SeparateLeadProcess.runViterbi, SeparateLeadStereoTF.py:1220-1222)
 * and its pure-Python twin tracking.viterbiTrackingArray (tracking.py:87-151).
 *
 *   cum[s, 0]  = log_prior[s] + log_density[s, 0]
 *   cum[s, n]  = max_{s'} (cum[s', n-1] + log_transition[s', s]) + log_density[s, n]
 *   ante[s, n] = the first s' reaching the max (the pyx's strict '>' scan)
 *   path[N-1]  = argmax_s cum[s, N-1] (numpy.argmax), path[n] = ante[path[n+1], n+1]
 *
 * Only the first n_states rows / columns of the inputs are read (the
 * pipeline passes NF0 states with NF0 + 1 rows).  The additions are the
 * reference's own double additions, so the path is bit-identical.
 * Conventions: fasst_hip.h.  log_density: row s at log_density + s*ld_density
 * (frames contiguous); log_transition: row s' at log_transition +
 * s'*ld_transition; path: int64 (numpy's default int).
 */
#ifndef FASST_VITERBI_H
#define FASST_VITERBI_H

#include "fasst_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int viterbi_tracking(int device, int n_states, int n_frames, const double *log_density,
                     long ld_density, const double *log_prior, const double *log_transition,
                     long ld_transition, long long *path);

/* Device time (HIP events) of the last viterbi_tracking call, without the
 * host<->device copies; and which kernel path it used (0: one workgroup
 * holding the whole transition matrix in LDS, 1: one launch per frame,
 * 2: one persistent cooperative launch).                                   */
int viterbi_last_timing(double *device_ms, int *path_kind);

/* Number of persistent launches in this process that aborted (grid not
 * co-resident) and were rerun on the per-frame path (about 3x slower); the
 * first one is also reported on stderr.                                    */
int viterbi_fallback_count(int *aborts);

#ifdef __cplusplus
}
#endif

#endif /* FASST_VITERBI_H */
