cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('$v',d['ms_per_step'])"
done
