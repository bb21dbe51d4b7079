cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/bench_default_$i.json 2> gpurun_out/bench_default_$i.err || exit $?
done
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_200.json 2> gpurun_out/bench_200.err || exit $?
for f in gpurun_out/bench_default_1.json gpurun_out/bench_default_2.json gpurun_out/bench_200.json; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['iteration']['traffic_ratio'], d.get('cpu_baseline',{}).get('value'))" $f
done
