#!/bin/bash
# A/B of environment switches on the bench (kernel times from HIP events).
# Usage: tools/gpu_ab.sh "FASST_MFMA16=1" "FASST_MFMA16=0"   (AB_STEPS / AB_WARMUP override 10 / 2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-2} --no-cpu-baseline > gpurun_out/ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab.log; exit $rc; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step", d["ms_per_step"], d["kernels_ms"])
PY
done
