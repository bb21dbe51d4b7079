#!/bin/bash
# Same-box A/B of two builds of the library (FASST_HIP_LIB): the C3 bench
# (200 iterations after 30 warm-up), then the SIMM / IS-NMF aux benches.
# Usage: tools/gpu_lib_ab.sh pyfasst_amd/libfasst_hip.so pyfasst_amd/libfasst_hip_vf.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "$@"; do
    FASST_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${AB_STEPS:-200} --warmup 30 \
      --no-cpu-baseline > gpurun_out/ab.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/ab.log; exit $rc; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
print(sys.argv[1], "C3 ms/step", d["ms_per_step"], d["kernels_ms"], flush=True)
PY
  done
done
for w in ${AB_AUX:-simm nmf}; do
  [ "$w" = none ] && continue
  for lib in "$@"; do
    FASST_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_aux.py --workload $w --steps 20 \
      --warmup 3 --no-cpu-baseline > gpurun_out/ab_aux.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$lib $w rc=$rc"; tail -5 gpurun_out/ab_aux.log; exit $rc; }
    python - "$lib" "$w" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_aux.log").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "ms/step", d["ms_per_step"], flush=True)
PY
  done
done
