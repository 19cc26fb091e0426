#!/bin/bash
# r3_full2.sh TAG -- video tests, the whole GPU suite, the video bench, then
# the default bench.  A timeout / crash (rc > 1) ends the script.
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -v --timeout 120 --timeout-method thread > "$OUT/${1}_video.log" 2>&1
rc=$?; echo "video rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --deselect tests/test_gpu_video.py --timeout 300 --timeout-method thread > "$OUT/${1}_all.log" 2>&1
rc=$?; echo "suite rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u scripts/video_bench.py --w 1920 --h 1080 --frames 30 > "$OUT/${1}_vbench.log" 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > "$OUT/${1}_bench.log" 2> "$OUT/${1}_bench.err"
echo "done $1"
