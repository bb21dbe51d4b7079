#!/bin/bash
# C5 bench under environment settings (A/B of launch geometry knobs).
# Usage: tools/gpu_ab_simm_env.sh "FASST_HMT_NZ=15" "FASST_WMT_NZ=8" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python tools/bench_aux.py --workload simm --steps 20 --warmup 3 > gpurun_out/ab_simm.log 2>&1 || { tail -3 gpurun_out/ab_simm.log; exit 1; }
  echo "$v $(python -c "import json;print(json.loads(open('gpurun_out/ab_simm.log').read().strip().splitlines()[-1])['ms_per_step'])")"
done
