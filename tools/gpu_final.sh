#!/bin/bash
# Round-end measurement: the default bench line (200 iterations + the CPU
# baseline), the C3 rocprofv3 passes and the SIMM / NMF aux benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_line.json 2> gpurun_out/bench_line.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_line.json; [ $rc -eq 0 ] || exit $rc
PROF_TAG=${TAG:-r2c}_prof bash tools/gpu_prof.sh || exit $?
PROF_TAG=${TAG:-r2c}_aux bash tools/gpu_aux.sh || exit $?
