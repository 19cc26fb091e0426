#!/bin/bash
# r3_video.sh TAG -- video parity tests (all, no -x), then the intra/coder
# tests and the default bench line.  Each GPU step has its own time limit.
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -v --timeout 120 --timeout-method thread > "$OUT/${1}_video.log" 2>&1
rc=$?
echo "video tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/${1}_coder.log" 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > "$OUT/${1}_bench.log" 2> "$OUT/${1}_bench.err"
echo "done $1"
