#!/bin/bash
# streaming-floor probe + a short bench (kernel times)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_stream > gpurun_out/ubench_stream.txt 2>&1
rc=$?; cat gpurun_out/ubench_stream.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 30 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/bench.log; exit $rc
