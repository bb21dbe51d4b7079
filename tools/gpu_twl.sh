#!/bin/bash
# k_tw_contract_lds shapes: the EM parity subset under each FASST_TWL, then a
# same-box A/B of the bench (0 = the register-operand k_tw_contract)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SUB="tests/test_gpu_parity.py tests/test_gpu_fast_tail.py tests/test_gpu_fullsize.py"
for v in ${TWLS:-1 2 3 4}; do
  FASST_TWL=$v timeout -k 10 600 python -u -m pytest $SUB -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "stft_domain or end_to_end or restart or fast_tail or fullsize or c3 or multi or lambda" -p no:cacheprovider \
    > gpurun_out/twl_tests_$v.log 2>&1
  rc=$?; echo "TWL=$v pytest rc=$rc: $(tail -1 gpurun_out/twl_tests_$v.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/twl_tests_$v.log | head -20; exit $rc; }
done
ROUNDS=${ROUNDS:-2} bash tools/gpu_ab.sh $(for v in ${ABS:-0 1 2 3 4 5}; do echo "twl$v:FASST_TWL=$v"; done)
