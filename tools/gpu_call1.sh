#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_mfma_lds > gpurun_out/ubench_mfma_lds.txt 2>&1
rc=$?; cat gpurun_out/ubench_mfma_lds.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tests.sh tests/test_gpu_c4.py tests/test_gpu_fullsize.py
