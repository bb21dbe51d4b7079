#!/bin/bash
# Viterbi A/B over the persistent kernel's states-per-workgroup knob (gpurun).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/vt_ab"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 200 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for spw in ${VT_SPWS:-5 8 12 16}; do
  FASST_VT_SPW=$spw timeout -k 10 120 python3 tools/bench_aux.py --workload viterbi --steps 3 --warmup 1 > "$OUT/spw$spw.json" 2> "$OUT/spw$spw.err" || exit $?
  grep -m1 vt_probe "$OUT/spw$spw.err"; echo "spw=$spw $(python3 -c "import json,sys; d=json.load(open('$OUT/spw$spw.json')); print(d['device_ms'], d['us_per_frame'])")"
done
FASST_VT_PATH=frame timeout -k 10 120 python3 tools/bench_aux.py --workload viterbi --steps 2 --warmup 1 > "$OUT/frame.json" 2>&1 || exit $?
echo "frame $(python3 -c "import json; d=json.load(open('$OUT/frame.json')); print(d['device_ms'], d['us_per_frame'])")"
