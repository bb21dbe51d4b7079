#!/bin/bash
# SQ pipe-utilisation passes (one rocprofv3 --pmc run per group, kernel-filtered)
# over a short run.  Usage: tools/gpu_pmc_sq.sh [KERNEL_REGEX [COMMAND...]]
# (default command: a 3-step C3 bench run)
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-sq}"
RX="${1:-k_estep|k_tw_contract|k_fb_contract}"
shift
CMD=("$@")
[ ${#CMD[@]} -gt 0 ] || CMD=(python3 "$R/bench.py" --steps 3 --warmup 1 --warm-s 0 --no-cpu-baseline)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAVES"
)
i=0
for g in "${GROUPS_[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "$RX" -d "$OUT/p$i" -o run --output-format csv \
    -- "${CMD[@]}" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
  i=$((i+1))
done
python3 "$R/tools/summarize_sq.py" "$OUT" | tee "$OUT/summary.txt"
