#!/bin/bash
# r3_dig.sh TAG -- batch tests (digests) and the default bench.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 900 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "dig $TAG done"
