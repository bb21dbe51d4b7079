#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_dgemm3 > gpurun_out/ubench_dgemm3.txt 2>&1
rc=$?; grep -E "rocblas|_da|NS=2,BK=16,2x2,occ2,mf0,A4=0,B4=0|4x2,occ1,mf0,A4=1|4x2,occ1,mf0,A4=0,B4=1" gpurun_out/ubench_dgemm3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_simm.py tests/test_gpu_lead.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "simm or SIMM or lead or pipeline or config5" > gpurun_out/pytest_simm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_simm.log; [ $rc -eq 0 ] || exit $rc
for lib in build/ab/r2head.so pyfasst_amd/libfasst_hip.so; do
  FASST_HIP_LIB=$PWD/$lib timeout -k 10 300 python tools/bench_aux.py --workload simm --steps 20 --warmup 3 > gpurun_out/ab_aux.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/ab_aux.log; exit $rc; }
  python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_aux.log").read().strip().splitlines()[-1])
print(sys.argv[1], "simm ms/step", d["ms_per_step"], flush=True)
PY
done
