#!/bin/bash
# structure variants of the C3 bench (J = 6, 8 at K = 32; K = 64 at J = 4),
# the headline bench, and the C5 SIMM aux bench with its full-size CPU baseline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/var
for v in "--J 6" "--J 8" "--K 64" "--J 8 --K 64"; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline $v > gpurun_out/var/b.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/var/b.log; exit $rc; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/var/b.log").read().strip().splitlines()[-1])
print(sys.argv[1], json.dumps({"ms_per_step": d["ms_per_step"], "value": d["value"], "kernels_ms": d["kernels_ms"], "config": d["config"]}), flush=True)
PY
  cp gpurun_out/var/b.log "gpurun_out/var/bench_$(echo $v | tr -d ' -').json"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/var/head.json 2>&1 || exit $?
tail -c 600 gpurun_out/var/head.json
timeout -k 10 600 python tools/bench_aux.py --workload simm --steps 20 --warmup 3 > gpurun_out/var/simm.json 2>&1 || exit $?
tail -c 1500 gpurun_out/var/simm.json
