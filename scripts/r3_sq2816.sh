#!/bin/bash
# r3_sq2816.sh TAG -- the stream coder's SQ / GRBM counters at 2816 streams in
# flight (1080p), the serving step's count.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    -f csv -d "$OUT/${TAG}_sq" -o run -- python3 "$R/scripts/gc_probe.py" --w 1920 --h 1080 --n 2816 --reps 1 --check 1 > "$OUT/${TAG}_sq.log" 2>&1
echo "sq $TAG done"
