#!/bin/bash
# every tools/bench_aux.py workload once (with its CPU baseline), one JSON
# line each, into gpurun_out/aux_bench.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/aux_bench.jsonl
for w in simm nmf cqt viterbi wf0 separate nnls; do
  timeout -k 10 400 python tools/bench_aux.py --workload $w > gpurun_out/aux_$w.json 2> gpurun_out/aux_$w.err || { echo "$w failed"; tail -3 gpurun_out/aux_$w.err; exit 1; }
  tail -1 gpurun_out/aux_$w.json >> gpurun_out/aux_bench.jsonl
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d.get('value'), d.get('unit'), d.get('ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/aux_$w.json $w
done
