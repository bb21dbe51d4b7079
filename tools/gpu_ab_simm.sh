#!/bin/bash
# SIMM parity tests on the current library, then the C5 bench against a saved
# build (pyfasst_amd/libfasst_hip_base.so), same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest -x -q -p no:cacheprovider tests/test_gpu_simm.py tests/test_gpu_lead.py tests/test_gpu_pipeline.py "tests/test_gpu_fullsize.py::test_config5_full_size_vs_oracle" > gpurun_out/ab_simm_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/ab_simm_tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for lib in pyfasst_amd/libfasst_hip_base.so pyfasst_amd/libfasst_hip.so; do
  FASST_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_aux.py --workload simm --steps 20 --warmup 3 > gpurun_out/ab_simm.log 2>&1 || exit $?
  echo "$lib $(python -c "import json;print(json.loads(open('gpurun_out/ab_simm.log').read().strip().splitlines()[-1])['ms_per_step'])")"
done
done
