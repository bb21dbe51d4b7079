#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${PROF_TAG:-prof}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# (warmup 20: the first ~15 iterations run while the GPU clock ramps up)
ARGS="--steps ${STEPS:-50} --warmup 20 --no-cpu-baseline $BENCH_ARGS"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" $ARGS > "$OUT/bench_trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 "$OUT/bench_trace.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_write.log" 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
