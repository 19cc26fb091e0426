#!/bin/bash
# r3_cmp.sh TAG -- band sums check, the API / batch / coder GPU tests, then the default bench.
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 120 python3 -u scripts/dbg/band_sums_check.py > "$OUT/${1}_sums.log" 2>&1
echo "sums rc=$?"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_api.py tests/test_gpu_batch.py tests/test_gpu_coder.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/${1}_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python3 -u bench.py > "$OUT/${1}_bench.log" 2> "$OUT/${1}_bench.err"
echo "done $1"
