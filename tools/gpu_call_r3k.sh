#!/bin/bash
# FB contraction raw-buffer rho loads: EM parity subset, then same-box C3 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/em_tests.log 2>&1; rc=$?; tail -3 gpurun_out/em_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_only.sh build/ab/fbold.so build/ab/fbraw.so
