#!/bin/bash
# r5_tests.sh TAG [pytest -k expr] -- GPU tests on the box (run via gpurun):
# the selected tests with output (-s), then the whole GPU suite.
set -e -o pipefail
TAG=$1
K=${2:-}
OUT=gpurun_out
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread -k "$K" > "$OUT/${TAG}_sel.log" 2>&1
fi
if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/${TAG}_all.log" 2>&1
fi
echo "tests $TAG done"
