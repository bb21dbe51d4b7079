#!/bin/bash
# EM parity tests on the current library, then a same-box A/B against a saved
# build (pyfasst_amd/libfasst_hip_base.so) on the C3 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/ab_tests.log)"; [ $rc -eq 0 ] || exit $rc
AB_AUX="" bash tools/gpu_lib_ab.sh pyfasst_amd/libfasst_hip_base.so pyfasst_amd/libfasst_hip.so
