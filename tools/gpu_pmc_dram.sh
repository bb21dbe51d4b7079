#!/bin/bash
# memory-side read requests: all (TCC_EA0_RDREQ) vs those the TCC sends to
# DRAM (TCC_EA0_RDREQ_DRAM), per kernel of the C3 bench, for the given builds
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/dram"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  FASST_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum \
    -d "$R/gpurun_out/dram/$tag" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/dram/$tag.log" 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
