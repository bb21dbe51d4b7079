#!/bin/bash
# A/B of environment settings on the Stereo_SIMM secondary bench (config 5).
# Usage: tools/gpu_ab_simm.sh "FASST_X=0" "FASST_HIP_LIB=/path/variant.so" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 300 python3 tools/bench_aux.py --workload simm --steps 10 --warmup 2 > gpurun_out/ab_simm.log 2>&1 || { tail -5 gpurun_out/ab_simm.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_simm.log').read().strip().splitlines()[-1]);print('$v',d['ms_per_step'])"
done
