#!/bin/bash
# NMF fused-kernel geometry sweep (timing only): per-kernel averages per (build, FASST_NMF_WAVES)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for cfg in pair:1024 abl5:1024; do
  lib=${cfg%%:*}; wv=${cfg##*:}; d=gpurun_out/sweep_${lib}_$wv
  mkdir -p $d
  FASST_NMF_WAVES=$wv FASST_HIP_LIB=$PWD/build/ab/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
    python3 tools/bench_aux.py --workload nmf --steps 30 --warmup 5 --no-cpu-baseline > $d/bench.log 2>&1 || exit $?
  python3 - $cfg $d/run_kernel_stats.csv <<'PY'
import csv, sys
print(sys.argv[1], "  ".join("%s %.1f" % (r["Name"].split("(")[0].split("::")[-1][:14], float(r["AverageNs"])/1e3) for r in csv.DictReader(open(sys.argv[2])) if "num" in r["Name"]))
PY
done
