#!/bin/bash
# r3_vprof2.sh TAG W H FRAMES -- video parity tests, the video bench (with the
# reference's CPU time), then its rocprofv3 kernel trace.
set -e -o pipefail
TAG=$1; W=${2:-1920}; H=${3:-1080}; F=${4:-30}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_video.log" 2>&1
timeout -k 10 300 python3 -u "$R/scripts/video_bench.py" --w $W --h $H --frames $F > "$OUT/${TAG}_vbench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/scripts/video_bench.py" --w $W --h $H --frames $F --cpu-frames 0 > "$OUT/${TAG}_kt.log" 2>&1
echo "vprof2 $TAG done"
