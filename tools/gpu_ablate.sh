#!/bin/bash
# E-step ablation timings (FASST_ABLATE bit builds: 1 no log, 2 no hat_W, 4 no
# sufficient-statistic accumulation): rocprofv3 kernel stats per ablation.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/ablate"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ab in ${1:-0 1 2 4 7}; do
  FASST_ABLATE=$ab timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/a$ab" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/a$ab.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "ablate $ab rc=$rc"; exit $rc; }
  python3 - "$OUT/a$ab/run_kernel_stats.csv" $ab <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_estep" in r["Name"]:
        print("ablate", sys.argv[2], r["Name"][:40], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
