#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB_AUX=none bash tools/gpu_lib_ab.sh build/ab/head.so build/ab/estep_pf.so || exit $?
PROF_TAG=prof_simm bash tools/gpu_prof_simm.sh || exit $?
