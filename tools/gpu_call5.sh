#!/bin/bash
# SQ counters: k_dgemm2 vs rocBLAS (NPD product), then the IS-NMF contractions
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
PROF_TAG=sq_dgemm bash tools/gpu_pmc_sq.sh "k_dgemm2|Cijk" "$R/tools/ubench_dgemm3" prof || exit $?
PROF_TAG=sq_nmf bash tools/gpu_pmc_sq.sh "k_nmf" python3 "$R/tools/bench_aux.py" --workload nmf --steps 5 --warmup 1 || exit $?
