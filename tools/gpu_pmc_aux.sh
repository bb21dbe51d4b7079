#!/bin/bash
# PMC passes over a tools/bench_aux.py workload (one counter group per rocprofv3 run).
# Usage: WORKLOAD=nmf tools/gpu_pmc_aux.sh "SQ_WAVE_CYCLES,SQ_WAIT_ANY:SQ_INSTS_VALU"
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-pmc_aux}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=':' read -ra PGRP <<< "${1:-SQ_WAVE_CYCLES,SQ_BUSY_CYCLES}"
i=0
for g in "${PGRP[@]}"; do
  timeout -k 10 200 rocprofv3 --pmc ${g//,/ } -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$R/tools/bench_aux.py" --workload ${WORKLOAD:-nmf} --steps 10 --warmup 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
