#!/bin/bash
# SIMM / NMF secondary benchmarks + rocprofv3 kernel stats (gpurun).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-aux}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/bench_aux.py" --workload nmf --steps 50 --warmup 5 > "$OUT/nmf.json" 2> "$OUT/nmf.err" || exit $?
cat "$OUT/nmf.json"
timeout -k 10 400 python3 "$R/tools/bench_aux.py" --workload simm --steps 5 --warmup 1 > "$OUT/simm.json" 2> "$OUT/simm.err" || exit $?
cat "$OUT/simm.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/simm_trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" --workload simm --steps 3 --warmup 0 > "$OUT/prof_simm.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/nmf_trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" --workload nmf --steps 20 --warmup 0 > "$OUT/prof_nmf.log" 2>&1 || exit $?
find "$OUT" -name "*kernel_stats.csv"
