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
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" --workload viterbi --steps 1 --warmup 0 > "$OUT/prof.log" 2>&1 || exit $?
cut -c1-150 "$OUT/trace/run_kernel_stats.csv"
