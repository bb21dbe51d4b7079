#!/bin/bash
# GPU test suite (optionally a subset: tools/gpu_tests.sh tests/test_gpu_c4.py ...)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|drift|passed|failed" gpurun_out/pytest_gpu.log | tail -60
exit $rc
