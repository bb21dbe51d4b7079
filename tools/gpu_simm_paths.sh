#!/bin/bash
# SIMM parity on every GEMM path (rocBLAS / k_dgemm / k_gemm) incl. C5 full size.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sp
timeout -k 10 600 python -u -m pytest tests/test_gpu_simm.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sp/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/sp/pytest.log; exit $rc
