#!/bin/bash
# IS-NMF launch-geometry sweep (C2 size) + one rocprofv3 kernel summary
set -o pipefail
mkdir -p gpurun_out
for pw in 1 2; do
  for w in 512 1024 2048; do
    r=$(FASST_NMF_PW=$pw FASST_NMF_WAVES=$w timeout -k 10 120 python -u tools/bench_aux.py --workload nmf --steps 50 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "pw=$pw waves=$w $r"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nmf -o nmf -- python3 $GRAFT_REPO_ROOT/tools/bench_aux.py --workload nmf --steps 20 --warmup 2 > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/prof_nmf -name "*kernel_stats.csv" -exec head -8 {} \;
