#!/bin/bash
# E-step ablation timings (FASST_ABLATE bit builds: 1 no log, 2 no hat_W, 4 no
# sufficient-statistic accumulation); each a short bench, k_estep ms reported.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for ab in ${ABLATIONS:-0 1 2 4 7}; do
  FASST_ABLATE=$ab timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ablate_$ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "ablate $ab rc=$rc"; exit $rc; }
  python - $ab <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ablate_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
print("ablate", sys.argv[1], "ms/step", d["ms_per_step"], d["kernels_ms"])
PY
done
