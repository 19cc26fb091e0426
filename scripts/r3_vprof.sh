#!/bin/bash
# r3_vprof.sh TAG W H FRAMES -- the video bench, its rocprofv3 kernel trace
# (--stats), then one --pmc pass each for FETCH_SIZE and WRITE_SIZE.
set -e -o pipefail
TAG=$1; W=${2:-1920}; H=${3:-1080}; F=${4:-30}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 300 python3 -u "$R/scripts/video_bench.py" --w $W --h $H --frames $F > "$OUT/${TAG}_vbench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/scripts/video_bench.py" --w $W --h $H --frames $F --cpu-frames 0 > "$OUT/${TAG}_kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/${TAG}_pmc_fetch" -o run -- \
    python3 "$R/scripts/video_bench.py" --w $W --h $H --frames $F --cpu-frames 0 > "$OUT/${TAG}_pf.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/${TAG}_pmc_write" -o run -- \
    python3 "$R/scripts/video_bench.py" --w $W --h $H --frames $F --cpu-frames 0 > "$OUT/${TAG}_pw.log" 2>&1
echo "vprof $TAG done"
