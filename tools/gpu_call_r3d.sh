#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_call_r3c.sh || exit $?
AB_AUX=none AB_STEPS=100 bash tools/gpu_lib_ab.sh build/ab/e.so build/ab/trim.so
