#!/bin/bash
# r2_check.sh TAG [tests|bench|all] -- GPU parity tests then a short bench,
# each step under its own time limit; stops at the first step that ends in a
# fault, abort, segfault or time limit (anything but 0 or a test failure).
TAG=${1:-r2}
WHAT=${2:-all}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
step() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "$OUT/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  step tnew 400 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_golden.py tests/test_gpu_api.py -m gpu -q \
       --timeout 240 --timeout-method thread
  step tall 500 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  step bench 400 python3 -u bench.py --steps ${STEPS:-3} --warmup 1
fi
echo "r2_check $TAG done"
