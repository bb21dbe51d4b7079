#!/bin/bash
# round-3 aux benches (every other §8 row, with CPU baselines), the counter
# list of the box's rocprofv3 (is there an infinity-cache / DRAM split?)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/aux
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/aux/rocprof_counters.txt 2>&1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
grep -i -E "MALL|DRAM|EA0_RD|EA_RD|infinity" gpurun_out/aux/rocprof_counters.txt | head -20
for w in simm nmf separate cqt viterbi wf0 nnls; do
  st=20; [ $w = nnls ] && st=3; [ $w = simm ] && st=20
  timeout -k 10 400 python tools/bench_aux.py --workload $w --steps $st --warmup 3 > gpurun_out/aux/$w.json 2>&1 || { echo "$w failed"; tail -5 gpurun_out/aux/$w.json; exit 1; }
  tail -n 1 gpurun_out/aux/$w.json | head -c 600; echo
done
