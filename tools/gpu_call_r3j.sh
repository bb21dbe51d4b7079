#!/bin/bash
# Round-3 final: full GPU suite + smoke + default bench, then the C2 IS-NMF
# aux line (with its CPU baseline) and its rocprofv3 kernel summary
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check_all.sh || exit $?
timeout -k 10 300 python tools/bench_aux.py --workload nmf --steps 200 --warmup 20 > gpurun_out/nmf_aux.json 2> gpurun_out/nmf_aux.err || exit $?
tail -1 gpurun_out/nmf_aux.json
bash tools/gpu_prof_nmf.sh
