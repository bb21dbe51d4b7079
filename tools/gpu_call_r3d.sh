#!/bin/bash
# round-3 batch: parity (EM incl. K > 64 / mixed types, IS-NMF, pipeline incl.
# initHF00='nnls'), IS-NMF K-split A/B, the RCCL path on one rank, the NNLS
# aux bench, and the E-step trim / FB last-chunk-first A/Bs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: tests ran in the previous call
WORKLOAD=nmf AB_STEPS=100 bash tools/gpu_ab_aux.sh build/ab/cur.so build/ab/nmfks.so || exit $?
FASST_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/bench_nccl1.json 2> gpurun_out/bench_nccl1.err || { tail -20 gpurun_out/bench_nccl1.err; exit 1; }
tail -c 300 gpurun_out/bench_nccl1.json; echo
timeout -k 10 300 python tools/bench_aux.py --workload nnls --steps 3 --warmup 1 > gpurun_out/nnls_bench.json 2>&1 || { tail -20 gpurun_out/nnls_bench.json; exit 1; }
tail -c 800 gpurun_out/nnls_bench.json; echo
AB_AUX=none AB_STEPS=100 bash tools/gpu_lib_ab.sh build/ab/cur.so build/ab/trim.so build/ab/fbrev.so
