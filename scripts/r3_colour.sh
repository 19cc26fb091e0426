#!/bin/bash
# r3_colour.sh TAG -- the GPU coder tests (gray + colour) and the hybrid
# tests, then the stream coder's SQ counters at 1920 streams in flight.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coder.py tests/test_gpu_batch.py -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    -f csv -d "$OUT/${TAG}_sq" -o run -- python3 "$R/scripts/gc_probe.py" --w 1920 --h 1080 --n 1920 --reps 1 --check 1 > "$OUT/${TAG}_sq.log" 2>&1
echo "colour $TAG done"
