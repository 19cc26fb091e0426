#!/bin/bash
# r3_split.sh TAG -- the split-encoder and batch GPU tests, then the default bench.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_batch.py tests/test_gpu_coder.py -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 700 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "split $TAG done"
