#!/bin/bash
# where does the one-rank torch.distributed run lose ~3%: torchrun's
# environment, the gloo process group, or the RCCL one?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name, env..., -- cmd
  local name=$1; shift
  env "$@" > gpurun_out/d_$name.json 2> gpurun_out/d_$name.err || { tail -5 gpurun_out/d_$name.err; exit 1; }
  python - $name <<'PY'
import json, sys
d = json.loads(open("gpurun_out/d_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d["value"], d["kernels_ms"]["k_estep"], d["kernels_ms"]["k_tw_contract"], flush=True)
PY
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513"
B="bench.py --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  run plain timeout -k 10 300 python $B
  run trun timeout -k 10 300 $TR $B
  run gloo FASST_BENCH_DIST=1 FASST_BENCH_BACKEND=gloo timeout -k 10 300 $TR $B
  run nccl FASST_BENCH_DIST=1 timeout -k 10 300 $TR $B
done
