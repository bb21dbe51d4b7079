#!/bin/bash
# rocprofv3 kernel-trace summary of the C2 IS-NMF aux bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/nmfprof
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/nmfprof -o nmf --output-format csv -- \
  python3 tools/bench_aux.py --workload nmf --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/nmfprof/bench.log 2>&1 || exit $?
f=$(find gpurun_out/nmfprof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-60s %5s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
