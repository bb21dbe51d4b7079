#!/bin/bash
# EM parity tests (incl. the mixed-type golden case), then rocprofv3 passes:
# the C3 bench (trace + FETCH / WRITE) and the C5 Stereo_SIMM aux bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_parity.py || exit $?
PROF_TAG=prof_c3 STEPS=50 bash tools/gpu_prof.sh || exit $?
python3 tools/summarize_prof.py gpurun_out/prof_c3 gpurun_out/prof_c3/summary && head -30 gpurun_out/prof_c3/summary.txt
PROF_TAG=prof_simm bash tools/gpu_prof_simm.sh || exit $?
