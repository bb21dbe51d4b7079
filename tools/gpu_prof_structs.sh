#!/bin/bash
# rocprofv3 trace + FETCH / WRITE passes of the structure variants (J x K at C3 F x T)
R="${GRAFT_REPO_ROOT:-/root/repo}"
for jk in ${STRUCTS:-4x128 8x32 8x128 12x32}; do
  J=${jk%x*}; K=${jk#*x}
  PROF_TAG=st_J${J}K${K} STEPS=10 BENCH_ARGS="--J $J --K $K --warm-s 0.5" bash "$R/tools/gpu_prof.sh" > "$R/gpurun_out/st_prof_$jk.log" 2>&1 || { tail -5 "$R/gpurun_out/st_prof_$jk.log"; exit 1; }
  python3 "$R/tools/summarize_prof.py" "$R/gpurun_out/st_J${J}K${K}" "$R/gpurun_out/st_J${J}K${K}_sum" > /dev/null && head -8 "$R/gpurun_out/st_J${J}K${K}_sum.txt"
done
