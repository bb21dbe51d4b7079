#!/bin/bash
# Full GPU check: the -m gpu suite, smoke(), and the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -c 3000 gpurun_out/bench.json
