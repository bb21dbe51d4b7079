#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not config5" > gpurun_out/pytest_em.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_em.log; [ $rc -eq 0 ] || exit $rc
AB_AUX="" bash tools/gpu_lib_ab.sh build/ab/r2head.so pyfasst_amd/libfasst_hip.so || exit $?
cd /tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1; echo "list rc=$?"
