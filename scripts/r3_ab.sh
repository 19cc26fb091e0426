#!/bin/bash
# r3_ab.sh TAG -- serving-step A/B of the batched level-0 hand-off (ring vs
# double buffer, RIC_FQZ_ASYNC), then the stream coder's SQ / GRBM counters at
# 1024 streams in flight (1080p) for its scalar-issue fraction.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > "$OUT/${TAG}_async1.log" 2> "$OUT/${TAG}_async1.err"
RIC_FQZ_ASYNC=0 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > "$OUT/${TAG}_async0.log" 2> "$OUT/${TAG}_async0.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    -f csv -d "$OUT/${TAG}_sq" -o run -- python3 "$R/scripts/gc_probe.py" --w 1920 --h 1080 --n 1024 --reps 1 --check 1 > "$OUT/${TAG}_sq.log" 2>&1
echo "ab $TAG done"
