#!/bin/bash
# One-rank bench.py (C3, 100 steps) with and without an RCCL process group:
# plain python; the round-3 order (lazy communicator created by the barrier
# right before the timed loop, gpurun_tmp/bench_r3.py); this round's order
# (eager communicator + barrier before the engine exists); the same with more
# hardware queues.  Then the self-launched two-rank bench (--gpus 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name, env..., -- cmd
  local name=$1; shift
  env "$@" > gpurun_out/d_$name.json 2> gpurun_out/d_$name.err || { tail -5 gpurun_out/d_$name.err; exit 1; }
  python - $name <<'PY'
import json, sys
d = json.loads(open("gpurun_out/d_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d["value"], d["kernels_ms"]["k_estep"], d["kernels_ms"]["k_tw_contract"], d.get("control_plane"), flush=True)
PY
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513"
A="--gpus 1 --steps 100 --warmup 5 --no-cpu-baseline"
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpus', os.cpu_count())"
for r in 1 2; do
  run plain timeout -k 10 300 python bench.py $A
  run nccl_lazy FASST_BENCH_DIST=1 FASST_BENCH_BACKEND=nccl timeout -k 10 300 $TR gpurun_tmp/bench_r3.py $A
  run nccl_eager FASST_BENCH_DIST=1 timeout -k 10 300 $TR bench.py $A
  run nccl_eager_q8 GPU_MAX_HW_QUEUES=8 FASST_BENCH_DIST=1 timeout -k 10 300 $TR bench.py $A
done
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/d_gpus2.json 2> gpurun_out/d_gpus2.err || { tail -5 gpurun_out/d_gpus2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/d_gpus2.json').read().strip().splitlines()[-1])
print('gpus2', d['n_gpus'], d['value'], d['control_plane'], d['clips'])"
