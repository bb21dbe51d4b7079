#!/bin/bash
# Viterbi tests + bench + rocprofv3 kernel stats (gpurun).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-viterbi}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/bench_aux.py" --workload viterbi --steps 2 --warmup 1 > "$OUT/viterbi.json" 2> "$OUT/viterbi.err" || exit $?
cat "$OUT/viterbi.json"
# rocprofv3 has been seen to crash at process exit after the cooperative
# launch with its stats already written: accept that, nothing else
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" --workload viterbi --steps 1 --warmup 0 > "$OUT/prof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 139 -a -s "$OUT/trace/run_kernel_stats.csv" ] || exit $rc
cut -c1-150 "$OUT/trace/run_kernel_stats.csv"
