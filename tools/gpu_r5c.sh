#!/bin/bash
# k_tw_update batched element loops (occupancy-3 form): parity + same-box A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
FASST_TWU_BATCH=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fast_tail.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fast_tail or end_to_end or restart" -p no:cacheprovider > gpurun_out/t5.log 2>&1
rc=$?; tail -1 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash tools/gpu_ab.sh "twu0:FASST_TWU_BATCH=0" "twu1:FASST_TWU_BATCH=1"
