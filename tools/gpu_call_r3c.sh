#!/bin/bash
# K > 64 / mixed-type parity, IS-NMF K-split A/B, and the RCCL (nccl) path of
# bench.py on one rank (process group initialised on the real GPU)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_nmf.py || exit $?
WORKLOAD=nmf AB_STEPS=100 bash tools/gpu_ab_aux.sh build/ab/cur.so build/ab/nmfks.so || exit $?
FASST_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/bench_nccl1.json 2> gpurun_out/bench_nccl1.err || { tail -20 gpurun_out/bench_nccl1.err; exit 1; }
tail -c 400 gpurun_out/bench_nccl1.json
