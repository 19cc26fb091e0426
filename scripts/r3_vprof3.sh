#!/bin/bash
# r3_vprof3.sh TAG -- video parity tests, then the video bench, its kernel
# trace and the FETCH_SIZE / WRITE_SIZE passes (1080p, 30 frames).
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/${TAG}_video.log" 2>&1
bash "$R/scripts/r3_vprof.sh" "$TAG" 1920 1080 30
