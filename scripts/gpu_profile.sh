#!/bin/bash
# gpu_profile.sh TAG [BENCH_ARGS...] -- run on the GPU box (via gpurun) from the repo root.
# 1. rocprofv3 --kernel-trace --stats of the bench command          -> gpurun_out/TAG_kt/
# 2. rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes,
#    a 1-frame bench so counters see uncontended launches)            -> gpurun_out/TAG_pmc_{fetch,write}/
# Every GPU step is time-limited; the first failure ends the script.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/${TAG}_kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/${TAG}_pmc_fetch" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 1 --warmup 1 --batch 1 --threads 1 > "$OUT/${TAG}_pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/${TAG}_pmc_write" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 1 --warmup 1 --batch 1 --threads 1 > "$OUT/${TAG}_pmc_write.log" 2>&1
echo "profile $TAG done"
