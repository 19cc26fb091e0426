#!/bin/bash
# r6_tests.sh TAG [pytest -k expr] -- GPU tests on the box (run via gpurun):
# the selected tests with output (-s), then the whole GPU suite (SKIP_ALL=1:
# not).  AB_ENV="VAR=x": the selected tests first run once more with that
# environment, where a test failure (pytest status 1) is an expected outcome.
set -e -o pipefail
TAG=$1
K=${2:-}
OUT=gpurun_out
mkdir -p "$OUT"
sel() {
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread -k "$K"
}
if [ -n "$K" ] && [ -n "$AB_ENV" ]; then
  rc=0
  env $AB_ENV timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread \
      -k "$K" > "$OUT/${TAG}_ab.log" 2>&1 || rc=$?
  echo "A/B run ($AB_ENV): pytest status $rc"
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$K" ]; then
  sel > "$OUT/${TAG}_sel.log" 2>&1
fi
if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/${TAG}_all.log" 2>&1
fi
echo "tests $TAG done"
