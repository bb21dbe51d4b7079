#!/bin/bash
# Viterbi persistent-kernel grid: states per workgroup x initial poll delay x
# retry delay (s_sleep(1) units of 64 clocks) (gpurun).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/vt_ab2"
mkdir -p "$OUT"
cd "$R"
for spw in ${VT_SPWS:-10 12}; do for z in ${VT_SLEEPS:-8 12 16 20}; do for r in ${VT_SLEEPRS:-1}; do
  FASST_VT_SLEEPR=$r FASST_VT_SLEEP0=$z FASST_VT_SPW=$spw timeout -k 10 120 python3 tools/bench_aux.py --workload viterbi --steps 3 --warmup 1 > "$OUT/r.json" 2> "$OUT/r.err" || exit $?
  echo "spw=$spw sleep0=$z sleepr=$r $(python3 -c "import json; d=json.load(open('$OUT/r.json')); print(d['device_ms'], d['us_per_frame'])")"
done; done; done
