#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_dgemm3 > gpurun_out/ubench_dgemm3.txt 2>&1
rc=$?; cat gpurun_out/ubench_dgemm3.txt; exit $rc
