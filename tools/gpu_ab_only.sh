#!/bin/bash
# same-box A/B of library builds on the C3 bench only (100 iterations x 2 rounds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_AUX=${AB_AUX:-none} AB_STEPS=${AB_STEPS:-100} bash tools/gpu_lib_ab.sh "$@"
