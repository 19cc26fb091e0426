#!/bin/bash
# r3_ring.sh TAG -- GPU coder + batch tests, then the default bench.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coder.py tests/test_gpu_batch.py -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 900 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "ring $TAG done"
