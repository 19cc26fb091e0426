#!/bin/bash
# r3_pool2.sh TAG -- serving step at 1792 / 1920 stream-coder waves in flight,
# double-buffered level 0 (RIC_FQZ_ASYNC=0).  A step that fails (out of
# memory) ends the script.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
RIC_FQZ_ASYNC=0 timeout -k 10 450 python3 -u bench.py --no-cpu-baseline --pool 896 > "$OUT/${TAG}_p896a0.log" 2> "$OUT/${TAG}_p896a0.err"
RIC_FQZ_ASYNC=0 timeout -k 10 450 python3 -u bench.py --no-cpu-baseline --pool 960 > "$OUT/${TAG}_p960a0.log" 2> "$OUT/${TAG}_p960a0.err"
echo "pool2 $TAG done"
