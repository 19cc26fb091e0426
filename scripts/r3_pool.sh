#!/bin/bash
# r3_pool.sh TAG -- serving step with more stream-coder waves in flight
# (two launches of 768 / 1024 frames), ring vs double-buffered level 0.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --pool 768 > "$OUT/${TAG}_p768.log" 2> "$OUT/${TAG}_p768.err"
RIC_FQZ_ASYNC=0 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --pool 768 > "$OUT/${TAG}_p768a0.log" 2> "$OUT/${TAG}_p768a0.err"
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --pool 1024 > "$OUT/${TAG}_p1024.log" 2> "$OUT/${TAG}_p1024.err"
echo "pool $TAG done"
