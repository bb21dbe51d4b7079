#!/bin/bash
# bench.py on the structure variants (J sources x K NMF components, C3 F x T)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for jk in ${STRUCTS:-4x64 4x128 8x32 8x128}; do
  J=${jk%x*}; K=${jk#*x}
  timeout -k 10 300 python bench.py --J $J --K $K --steps ${STEPS:-20} --warmup 3 --warm-s 0.5 --no-cpu-baseline \
    > gpurun_out/st_$jk.json 2> gpurun_out/st_$jk.err || { echo "FAILED $jk"; tail -5 gpurun_out/st_$jk.err; exit 1; }
  python - $jk <<'PY'
import json, sys
d = json.loads(open("gpurun_out/st_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print("%-6s %8.4f ms | %s" % (sys.argv[1], d["ms_per_step"], " ".join("%s=%.4f" % (n, v) for n, v in sorted(k.items()))), flush=True)
PY
done
