cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 tests/test_gpu_simm.py tests/test_gpu_lead.py tests/test_gpu_pipeline.py "tests/test_gpu_fullsize.py::test_config5_full_size_vs_oracle" > gpurun_out/simm_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/simm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_aux.py --workload simm --steps 20 --warmup 3 > gpurun_out/simm_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/simm_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/simm_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_aux.py --workload simm --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/simm_prof.log 2>&1
echo "prof rc=$?"
