#!/bin/bash
# same-box A/B of library builds on one tools/bench_aux.py workload (2 rounds)
# Usage: WORKLOAD=nmf tools/gpu_ab_aux.sh build/ab/a.so build/ab/b.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "$@"; do
    FASST_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_aux.py --workload ${WORKLOAD:-nmf} \
      --steps ${AB_STEPS:-50} --warmup 5 --no-cpu-baseline > gpurun_out/ab_aux.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/ab_aux.log; exit $rc; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_aux.log").read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step", d["ms_per_step"], d.get("kernels_ms", ""), flush=True)
PY
  done
done
