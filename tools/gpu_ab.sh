#!/bin/bash
# Same-box A/B of bench.py variants, alternated ROUNDS times.
# Usage: tools/gpu_ab.sh "name:ENV=1 ENV2=0" "name2:ENV=0" ...
# (BENCH_ARGS overrides the bench arguments; ROUNDS the repetitions.)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A="${BENCH_ARGS:---steps 200 --warmup 10 --no-cpu-baseline}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    env $envs timeout -k 10 300 python bench.py $A > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err \
      || { echo "FAILED $name"; tail -5 gpurun_out/ab_$name.err; exit 1; }
    python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print("%-12s %8.4f ms %8.2f it/s | %s" % (sys.argv[1], d["ms_per_step"], d["value"],
      " ".join("%s=%.4f" % (n, v) for n, v in sorted(k.items()))), flush=True)
PY
  done
done
