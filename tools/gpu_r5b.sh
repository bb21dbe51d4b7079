#!/bin/bash
# round-5 batch: step-method / nnls tests, the FB rho-stream ubench, SIMM
# A/B (k_dgemm2 tile order) and per-kernel traces of the HMT chunk widths
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_steps.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?; tail -1 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/ubench_fbread > gpurun_out/fbread.txt 2>&1 || exit 1
cat gpurun_out/fbread.txt
FASST_D2_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_simm.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "simm or config5" -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?; tail -1 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash tools/gpu_simm_ab.sh "ord0:FASST_D2_ORDER=0" "ord1:FASST_D2_ORDER=1" || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 32 16; do
  FASST_HMT_KC=$v FASST_D2_ORDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kc$v" -o run --output-format csv \
    -- python3 "$R/tools/bench_aux.py" --workload simm --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/kc$v.log" 2>&1 || exit 1
  echo "KC=$v"; find "$R/gpurun_out/kc$v" -name "*kernel_stats.csv" -exec grep -E "k_simm|k_dgemm2" {} \;
done
cd "$R"
FASST_TWU_BATCH=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fast_tail.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fast_tail or end_to_end or restart" -p no:cacheprovider > gpurun_out/t4.log 2>&1
rc=$?; tail -1 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash tools/gpu_ab.sh "twu0:FASST_TWU_BATCH=0" "twu1:FASST_TWU_BATCH=1"
