#!/bin/bash
# CQT front-end bench + rocprofv3 kernel stats (gpurun).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-cqt}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/bench_aux.py" --workload cqt --steps 3 --warmup 1 > "$OUT/cqt.json" 2> "$OUT/cqt.err" || exit $?
cat "$OUT/cqt.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/cqt_trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" --workload cqt --steps 2 --warmup 0 > "$OUT/prof_cqt.log" 2>&1 || exit $?
find "$OUT" -name "*kernel_stats.csv" | xargs -I{} sh -c 'cut -c1-160 {}'
