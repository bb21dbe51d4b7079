#!/bin/bash
# rocprofv3 kernel stats of the IS-NMF secondary bench (config 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && cd gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d prof_nmf -o nmf --output-format csv -- python3 ../tools/bench_aux.py --workload nmf --steps 100 --warmup 10 > prof_nmf.log 2>&1; r=$?
tail -2 prof_nmf.log; [ $r = 0 ] || exit $r
f=$(find prof_nmf -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -20
