#!/bin/bash
# IS-NMF (config 2) parity tests, then A/B of environment settings on the NMF bench.
# Usage: tools/gpu_ab_nmf.sh "FASST_NMF_PW=2" "FASST_NMF_PW=1 FASST_NMF_WAVES=2048" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && \
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nmf.py tests/test_gpu_nmfinit.py tests/test_gpu_mono_wiener.py > gpurun_out/nmf_t.log 2>&1; r=$?; tail -2 gpurun_out/nmf_t.log; [ $r = 0 ] || exit $r
for v in "$@"; do
  env $v timeout -k 10 200 python3 tools/bench_aux.py --workload nmf --steps 300 --warmup 30 > gpurun_out/ab_nmf.log 2>&1 || { tail -5 gpurun_out/ab_nmf.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_nmf.log').read().strip().splitlines()[-1]);print('$v',d['ms_per_step'], d.get('roofline',{}).get('achieved'))"
done
