#!/bin/bash
# C5 Stereo_SIMM: same-box A/B of env variants (tools/bench_aux.py --workload simm)
# Usage: tools/gpu_simm_ab.sh "name:ENV=1" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-2}"); do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    env $envs timeout -k 10 300 python tools/bench_aux.py --workload simm --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
      > gpurun_out/sab_$name.json 2> gpurun_out/sab_$name.err || { echo "FAILED $name"; tail -5 gpurun_out/sab_$name.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/sab_$name.json').read().strip().splitlines()[-1])
print('%-10s %.4f ms/it %.2f it/s' % ('$name', d['ms_per_step'], d['value']), flush=True)"
  done
done
