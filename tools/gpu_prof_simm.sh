#!/bin/bash
# rocprofv3 over the C5 Stereo_SIMM aux bench: kernel trace + stats, then the
# FETCH_SIZE and WRITE_SIZE passes (separate runs), summarised per kernel
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-prof_simm}"
W=${WORKLOAD:-simm}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--workload $W --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" $ARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 "$OUT/trace.log"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" $ARGS > "$OUT/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 "$R/tools/bench_aux.py" $ARGS > "$OUT/write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/summarize_prof.py" "$OUT" "$OUT/summary" && cat "$OUT/summary.txt"
