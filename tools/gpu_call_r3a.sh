#!/bin/bash
# FP64 MFMA / VALU co-execution probe, then a same-box A/B of E-step variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_coexec > gpurun_out/ubench_coexec.txt 2>&1
rc=$?; cat gpurun_out/ubench_coexec.txt; [ $rc -eq 0 ] || exit $rc
AB_AUX=none AB_STEPS=100 bash tools/gpu_lib_ab.sh "$@"
