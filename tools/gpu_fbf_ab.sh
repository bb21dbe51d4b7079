cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAILED $name"; tail -5 gpurun_out/ab_$name.err; exit 1; }
python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print("%-8s %8.4f ms %8.2f it/s | %s" % (sys.argv[1], d["ms_per_step"], d["value"], " ".join("%s=%.4f" % (n, v) for n, v in sorted(k.items()) if v > 0.02)), flush=True)
PY
}
for r in 1 2; do
run base0 FASST_FBF=0
run full FASST_FBF=1
run bar FASST_HIP_LIB=$PWD/pyfasst_amd/libfasst_hip_dbg1.so
run noMF FASST_HIP_LIB=$PWD/pyfasst_amd/libfasst_hip_dbg2.so
run wronly FASST_HIP_LIB=$PWD/pyfasst_amd/libfasst_hip_dbg3.so
done
