#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench run.
# Usage: tools/gpu_pmc.sh "SQ_WAVE_CYCLES,SQ_WAIT_ANY:SQ_INSTS_VALU,SQ_INSTS_MFMA"
#        (":" separates passes, "," separates the counters of one pass)
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=':' read -ra PGRP <<< "${1:-SQ_WAVE_CYCLES,SQ_BUSY_CYCLES}"
i=0
for g in "${PGRP[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc ${g//,/ } -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
