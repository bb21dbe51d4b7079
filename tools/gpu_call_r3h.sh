#!/bin/bash
# NMF fused-kernel rework: NMF parity tests, then same-box A/B of the spread / fold knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nmf.py tests/test_gpu_nmfinit.py > gpurun_out/nmf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/nmf_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=100 bash tools/gpu_ab_aux.sh build/ab/pair.so build/ab/stage.so || exit $?
bash tools/gpu_prof_nmf.sh
