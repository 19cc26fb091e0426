#!/bin/bash
# r3_pcs.sh TAG -- host-trap PC sampling of the GPU stream coder (1080p, 256
# streams): where the encoder's and decoder's waves spend their time.
set -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 500 -f csv -d "$OUT/${TAG}_pcs" -o run -- \
    python3 "$R/scripts/gc_probe.py" --w 1920 --h 1080 --n 256 --reps 1 --check 1 > "$OUT/${TAG}_pcs.log" 2>&1
echo "pcs rc=$?"
