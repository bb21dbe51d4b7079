#!/bin/bash
# full GPU suite + smoke, A/B of the FW-staging fix, bench with / without the
# torch.distributed (RCCL) process group on one rank
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
AB_AUX=none AB_STEPS=100 bash tools/gpu_lib_ab.sh build/ab/prefix.so build/ab/cur.so || exit $?
for mode in plain dist plain dist; do
  if [ $mode = dist ]; then
    FASST_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 100 --warmup 5 \
      --no-cpu-baseline > gpurun_out/b_$mode.json 2> gpurun_out/b_$mode.err || exit 1
  else
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/b_$mode.json 2> gpurun_out/b_$mode.err || exit 1
  fi
  python - $mode <<'PY'
import json, sys
d = json.loads(open("gpurun_out/b_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d["value"], d["kernels_ms"]["k_estep"], d["kernels_ms"]["k_tw_contract"], flush=True)
PY
done
