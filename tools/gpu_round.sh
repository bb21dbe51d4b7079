#!/bin/bash
# Round-end evidence in one call: GPU tests + smoke + short bench, the C3
# rocprofv3 passes (trace, FETCH_SIZE, WRITE_SIZE) and the SIMM / NMF aux benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_check.sh || exit $?
PROF_TAG=${TAG:-r2b}_prof bash tools/gpu_prof.sh || exit $?
PROF_TAG=${TAG:-r2b}_aux bash tools/gpu_aux.sh || exit $?
