#!/bin/bash
# r3_full.sh TAG -- video parity tests, then the whole GPU suite (both without
# -x, so one call reports every failure), then the default bench line.  A
# timeout / crash (rc > 1) ends the script.
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -v --timeout 120 --timeout-method thread > "$OUT/${1}_video.log" 2>&1
rc=$?; echo "video rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --deselect tests/test_gpu_video.py --timeout 200 --timeout-method thread > "$OUT/${1}_all.log" 2>&1
rc=$?; echo "suite rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python3 -u bench.py > "$OUT/${1}_bench.log" 2> "$OUT/${1}_bench.err"
echo "done $1"
